"""Summarise rocprofv3 --pmc runs (one directory per pass, counter_collection.csv) per kernel
instance (tools/kname.py), with the gfx950 corrections of MI355X_MICROARCH.md (HBM section):

  * FETCH_SIZE / WRITE_SIZE are KiB per dispatch; FETCH_SIZE counts half the bytes of a wide
    (16 B/lane) coalesced read on gfx950 -> HBM read bytes = 2 * 1024 * FETCH_SIZE;
  * SQ_VALU_MFMA_BUSY_CYCLES counts SIMD cycles with the matrix core busy, summed over the chip
    (16 per v_mfma_f32_16x16x32_bf16 = 16384 flop, i.e. 1024 flop per busy cycle at the bf16
    dense rate; calibrated on the dense GEMMs, where busy * 1024 / duration equals the algorithmic
    flop rate to 1%): MFMA utilisation = busy / (duration * 2.4 GHz * 1024 SIMDs). Padded MFMAs
    (head_dim 48 -> 64, short sequences) count as busy: counter util >= algorithmic util.

    python tools/pmc_summary.py --out profiles/r01_pmc.json gpurun_out/pmc_mfma gpurun_out/pmc_fetch gpurun_out/pmc_write
"""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import kname  # noqa: E402

SIMDS = 256 * 4
CLK_GHZ = 2.4


def load_dir(d):
    """-> {dispatch_id: {"name", "ns", counters...}}"""
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    disp = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            did = (f, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            e = disp.setdefault(did, {"name": r["Kernel_Name"]})
            if r.get("Start_Timestamp") and r.get("End_Timestamp"):
                e["ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    # durations from the kernel trace of the same pass when the counter rows lack timestamps
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if tr and not any("ns" in e for e in disp.values()):
        dur = {}
        for f in tr:
            for r in csv.DictReader(open(f)):
                dur[r.get("Dispatch_Id") or r.get("Correlation_Id")] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        for (f, did), e in disp.items():
            if did in dur:
                e["ns"] = dur[did]
    return disp


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--config", default="{}", help="JSON of the profiled bench.py config (batch, frames, image, tracks)")
    args = ap.parse_args()
    agg = defaultdict(lambda: defaultdict(float))
    for d in args.dirs:
        for e in load_dir(d).values():
            inst = kname.instance(e["name"])
            if inst is None:
                continue
            a = agg[inst]
            a[f"dispatches@{os.path.basename(d.rstrip('/'))}"] += 1
            for k, v in e.items():
                if k != "name":
                    a[k] += v
                    a[f"n_{k}"] += 1
    res = {}
    for inst, a in agg.items():
        r = {}
        for k in list(a):
            if k.startswith("n_") or k.startswith("dispatches@"):
                continue
            r[k + "_per_dispatch"] = a[k] / a["n_" + k]
        ns = r.get("ns_per_dispatch")
        if "FETCH_SIZE_per_dispatch" in r:
            r["hbm_read_bytes_per_dispatch"] = 2 * 1024 * r["FETCH_SIZE_per_dispatch"]
        if "WRITE_SIZE_per_dispatch" in r:
            r["hbm_write_bytes_per_dispatch"] = 1024 * r["WRITE_SIZE_per_dispatch"]
        if "hbm_read_bytes_per_dispatch" in r and "hbm_write_bytes_per_dispatch" in r:
            r["hbm_bytes_per_dispatch"] = r["hbm_read_bytes_per_dispatch"] + r["hbm_write_bytes_per_dispatch"]
        if "SQ_VALU_MFMA_BUSY_CYCLES_per_dispatch" in r and ns:
            clk = CLK_GHZ
            if "GRBM_GUI_ACTIVE_per_dispatch" in r:
                # GRBM_GUI_ACTIVE is summed over the 8 XCDs' GRBMs (measured: ~19.2 cycles/ns)
                r["grbm_clock_ghz"] = r["GRBM_GUI_ACTIVE_per_dispatch"] / ns / 8
            busy = r["SQ_VALU_MFMA_BUSY_CYCLES_per_dispatch"]
            r["mfma_util"] = busy / (ns * clk * SIMDS)
            r["mfma_equiv_tflops"] = busy * 1024 / ns / 1e3
        res[inst] = r
    order = sorted(res, key=lambda k: -(res[k].get("ns_per_dispatch", 0) * max(
        [v for kk, v in agg[k].items() if kk.startswith("dispatches@")] or [1])))
    for inst in order[:args.top]:
        r = res[inst]
        line = f"{inst:44s}"
        if "ns_per_dispatch" in r:
            line += f" {r['ns_per_dispatch'] / 1e3:9.1f} us"
        if "mfma_util" in r:
            line += f"  mfma {100 * r['mfma_util']:5.1f}%"
        if "hbm_bytes_per_dispatch" in r:
            ns = r.get("ns_per_dispatch") or 1
            line += f"  hbm {r['hbm_bytes_per_dispatch'] / 1e6:9.2f} MB ({r['hbm_bytes_per_dispatch'] / ns:7.0f} GB/s)"
        print(line)
    if args.out:
        with open(args.out, "w") as f:
            json.dump({"source": [os.path.basename(d.rstrip("/")) for d in args.dirs], "config": json.loads(args.config),
                       "notes": __doc__.strip().splitlines()[0], "instances": res}, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
