"""A/B of the persistent GEMMs on the step's forward Linear shapes: the overlapped-epilogue
256 x 128 kernel (gemm_pp2.hip, plan kind 5) against the round-3 w4 kernel (COMET_GEMM_NO_PP2=1),
interleaved rounds in one process, random data, plus the max difference of the two outputs.

    python tools/pp2_bench.py [--resid] > gpurun_out/pp2_bench.txt
"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402

SHAPES = [  # (M, N, K, act, out dtype, resid): the step's instances (profiles/r03_v3/gemm_shapes.txt)
    (65536, 1536, 384, 1, torch.bfloat16, False),
    (74368, 3072, 768, 1, torch.bfloat16, False),
    (74368, 2304, 768, 0, torch.bfloat16, False),
    (65536, 1152, 384, 0, torch.bfloat16, False),
    (65536, 768, 384, 0, torch.bfloat16, False),
    (65536, 384, 384, 0, torch.bfloat16, False),
    (65536, 1536, 768, 0, torch.bfloat16, False),
    (73856, 3072, 768, 1, torch.bfloat16, False),
    (74368, 768, 3072, 0, torch.float32, True),
    (74368, 768, 768, 0, torch.float32, True),
    (73856, 768, 3072, 0, torch.float32, True),
]


def timed(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    resid_too = "--resid" in sys.argv
    if resid_too:
        os.environ["COMET_PP2_RESID"] = "1"
    dev = "cuda"
    print(f"{'M':>6} {'N':>5} {'K':>5} act out   res | pp2 ms  TF/s (plan) | w4 ms  TF/s | w4/pp2 | max|pp2-w4|", flush=True)
    for M, N, K, act, odt, res in SHAPES:
        if res and not resid_too:
            continue
        g = torch.Generator(device=dev).manual_seed(0)
        x = (torch.rand(M, K, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev, generator=g) * 2 - 1) * 0.05).to(torch.bfloat16)
        b = torch.rand(N, device=dev, generator=g)
        r = torch.rand(M, N, device=dev, generator=g, dtype=torch.float32) if res else None
        outs = {}
        for arm in ("pp2", "w4"):
            outs[arm] = torch.empty(M, N, device=dev, dtype=odt)

        def run(arm):
            if arm == "w4":
                os.environ["COMET_GEMM_NO_PP2"] = "1"
            else:
                os.environ.pop("COMET_GEMM_NO_PP2", None)
            ops.linear(x, w, bias=b, act=act, resid=r, out=outs[arm], out_dtype=odt)
            return int(ops._PLAN[0])

        plans = {arm: run(arm) for arm in ("pp2", "w4")}
        torch.cuda.synchronize()
        ts = {"pp2": [], "w4": []}
        for _ in range(5):  # interleaved rounds
            for arm in ("pp2", "w4"):
                run(arm)
                torch.cuda.synchronize()
                ts[arm].append(timed(lambda: run(arm), 10))
        os.environ.pop("COMET_GEMM_NO_PP2", None)
        fl = 2.0 * M * N * K
        t2, t4 = statistics.median(ts["pp2"]), statistics.median(ts["w4"])
        d = (outs["pp2"].float() - outs["w4"].float()).abs().max().item()
        print(f"{M:6d} {N:5d} {K:5d} {act:3d} {str(odt)[6:]:8s} {int(res)} | {t2:.4f} {fl / t2 / 1e9:7.1f} ({plans['pp2']}) | "
              f"{t4:.4f} {fl / t4 / 1e9:7.1f} | {t4 / t2:5.3f} | {d:.3e}", flush=True)


if __name__ == "__main__":
    main()
