"""Per-shape GEMM/attention time of one bench train step (B=8, T=16, 512^2, bf16) on the GPU.

    python tools/gemm_shapes.py [--batch 8] > gpurun_out/gemm_shapes.txt
"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))

import bench  # noqa: E402
from comet_amd import functional as F  # noqa: E402
from comet_amd.config import instantiate, load_config  # noqa: E402
from comet_amd.profiler import PROF  # noqa: E402
from comet_amd.train import build_optimizer, train_step  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    cfg = load_config()
    torch.manual_seed(0)
    model = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg).to(dev)
    opt, sched = build_optimizer(cfg, model, 1000)
    img, tracks, cams = bench.synthetic(args.batch, 16, 512, 512, dev, seed=1)
    for it in range(2):
        if it == 1:
            PROF.enabled = True
            PROF.detail = True
            PROF.reset()
        with F.precision(torch.bfloat16):
            train_step(model, img, cams, tracks, opt, sched, cfg)
        torch.cuda.synchronize()
    s = PROF.summary()
    tot = sum(v["ms"] for v in s.values())
    print(f"total profiled ms {tot:.2f}")
    for k, v in sorted(s.items(), key=lambda kv: -kv[1]["ms"]):
        tf = v["flops"] / (v["ms"] * 1e-3) / 1e12 if v["ms"] > 0 else 0
        print(f"{v['ms']:9.3f} ms {v['launches']:5d}x {tf:8.1f} TF/s  {k}")


if __name__ == "__main__":
    main()
