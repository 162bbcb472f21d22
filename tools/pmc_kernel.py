"""Per-launch averages of every counter a rocprofv3 --pmc pass collected for the kernels whose name
matches a regex, plus the kernel-trace average duration.

    python tools/pmc_kernel.py gpurun_out/corrpmc2 corr_mfma
"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    root, pat = sys.argv[1], re.compile(sys.argv[2])
    for f in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
        acc = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if pat.search(r["Kernel_Name"]):
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in sorted(acc.items()):
            print(f"{os.path.basename(os.path.dirname(f)):8s} {k:28s} {sum(v) / len(v):16.1f}  ({len(v)} launches)")
    for f in glob.glob(os.path.join(root, "*", "run_kernel_stats.csv")):
        for r in csv.DictReader(open(f)):
            if pat.search(r["Name"]):
                print(f"trace    {r['Name'][:90]}  calls {r['Calls']}  avg {float(r['AverageNs']) / 1e3:.1f} us")


if __name__ == "__main__":
    main()
