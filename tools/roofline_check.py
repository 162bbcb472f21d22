"""Check bench.py's live (HIP-event) kernel-instance timings against a rocprofv3
--kernel-trace --stats summary of the same command.

    python tools/roofline_check.py profiles/r01_v2_bench.json profiles/r01_v2_kernel_stats.csv [steps+warmup]

For every kernel instance bench.py reports, prints launches/step and average launch duration
from both sources (rocprof counts warmup steps too, so its per-step counts are divided by
steps + warmup). The dominant instance (bench roofline.kernel) must agree within a few %.
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kname  # noqa: E402


def main():
    bench = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    # bench.py runs warmup + an unprofiled and a profiled pass of `steps` each
    nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 2 * bench["steps"] + bench["warmup"]
    rp = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(sys.argv[2])):
        inst = kname.instance(r["Name"])
        if inst:
            rp[inst][0] += int(r["Calls"])
            rp[inst][1] += float(r["TotalDurationNs"])
    dom = (bench.get("roofline") or {}).get("kernel")
    print(f"{'instance':44s} {'bench l/step':>12s} {'rocprof l/step':>14s} {'bench avg us':>12s} {'rocprof avg us':>14s}  ratio")
    for inst, v in bench.get("kernel_instances", {}).items():
        if inst not in rp:
            continue
        c, ns = rp[inst]
        b_avg = v["ms_per_step"] / v["launches_per_step"] * 1e3
        r_avg = ns / c / 1e3
        mark = "  <- roofline.kernel" if inst == dom else ""
        print(f"{inst:44s} {v['launches_per_step']:12.1f} {c / nsteps:14.1f} {b_avg:12.1f} {r_avg:14.1f}  {b_avg / r_avg:5.3f}{mark}")


if __name__ == "__main__":
    main()
