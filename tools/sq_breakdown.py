"""Per-kernel SQ counter breakdown from rocprofv3 --pmc runs (counter_collection.csv dirs):
wave-cycle shares (WAIT_ANY / WAIT_INST_ANY / ACTIVE), MFMA busy vs the 2.4 GHz peak and vs the
GRBM-active clock, instruction mix.   python tools/sq_breakdown.py DIR [DIR ...]"""
import collections
import csv
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kname  # noqa: E402


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    ns = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
            seen = set()
            for r in csv.DictReader(open(f)):
                k = kname.short(r["Kernel_Name"]) if hasattr(kname, "short") else r["Kernel_Name"][:60]
                agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
                key = (f, r["Dispatch_Id"])
                if key not in seen:
                    seen.add(key)
                    ns[(k, d)] += float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                    cnt[(k, d)] += 1
    for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0)):
        w = c.get("SQ_WAVE_CYCLES", 0)
        line = f"{k[:58]:58s}"
        if w:
            line += (f" wait {c['SQ_WAIT_ANY'] / w:5.1%} instwait {c['SQ_WAIT_INST_ANY'] / w:5.1%}"
                     f" active {c['SQ_ACTIVE_INST_ANY'] / w:5.1%} valu {c['SQ_ACTIVE_INST_VALU'] / w:5.1%}"
                     f" ldsw {c['SQ_WAIT_INST_LDS'] / w:5.1%}")
        d1 = sys.argv[1]
        if (k, d1) in ns and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            t = ns[(k, d1)] * 1e-9
            line += f" mfma@2.4 {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (t * 2.4e9 * 1024):5.1%}"
        if "GRBM_GUI_ACTIVE" in c and "SQ_INSTS_MFMA" in c:
            line += f" | valu/mfma {c['SQ_INSTS_VALU'] / max(c['SQ_INSTS_MFMA'], 1):5.1f} lds/mfma {c['SQ_INSTS_LDS'] / max(c['SQ_INSTS_MFMA'], 1):4.2f}"
        if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
            line += f" ldsconf {c['SQ_LDS_BANK_CONFLICT'] / c['SQ_LDS_IDX_ACTIVE']:5.1%}"
        print(line)


if __name__ == "__main__":
    main()
