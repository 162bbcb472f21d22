"""Attribute the torch (non-libcomet) kernels of one bench train step to model source lines.

    python tools/glue_profile.py > gpurun_out/glue.txt
"""
import collections
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))

import bench  # noqa: E402
from comet_amd import functional as F  # noqa: E402
from comet_amd.config import instantiate, load_config  # noqa: E402
from comet_amd.train import build_optimizer, train_step  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    cfg = load_config()
    torch.manual_seed(0)
    model = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg).to(dev)
    opt, sched = build_optimizer(cfg, model, 1000)
    img, tracks, cams = bench.synthetic(8, 16, 512, 512, dev, seed=1)
    with F.precision(torch.bfloat16):
        train_step(model, img, cams, tracks, opt, sched, cfg)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=True) as prof:
        with F.precision(torch.bfloat16):
            train_step(model, img, cams, tracks, opt, sched, cfg)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_stack_n=6).table(sort_by="self_device_time_total", row_limit=25,
                                                       max_name_column_width=40))
    agg = collections.defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.device_time_total <= 0:
            continue
        site = "?"
        for fr in (ev.stack or []):
            if "comet_amd" in fr and "functional.py" not in fr and "ops.py" not in fr:
                site = fr.split("comet-pose-estimation_amd/")[-1]
                break
        key = (ev.name, site)
        agg[key][0] += 1
        agg[key][1] += ev.device_time_total / 1e3
    # backward ops run on the autograd engine's thread (no Python stack): name the autograd node
    # (parent "autograd::engine::evaluate_function: XBackward") and the op's input shapes instead
    byshape = collections.defaultdict(lambda: [0, 0.0])
    for ev in prof.events():
        if not ev.name.startswith("aten::") or ev.device_time_total <= 0:
            continue
        node, p = "fwd", ev.cpu_parent
        while p is not None:
            if p.name.startswith("autograd::engine::evaluate_function"):
                node = p.name.split(":")[-1].strip()
                break
            if p.cpu_parent is None:
                node = "fwd:" + p.name
            p = p.cpu_parent
        if ev.cpu_parent is not None and ev.cpu_parent.name.startswith("aten::"):
            continue  # count each kernel once, at its outermost aten op
        key = (ev.name, node, str(ev.input_shapes)[:90])
        byshape[key][0] += 1
        byshape[key][1] += ev.device_time_total / 1e3
    print("by autograd node / input shapes:")
    for (name, node, shp), (n, ms) in sorted(byshape.items(), key=lambda kv: -kv[1][1])[:40]:
        print(f"{ms:8.3f} ms {n:5d}x  {name:22s} {node:34s} {shp}")
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    tot = sum(v[1] for _, v in rows)
    print(f"torch aten kernels: {tot:.2f} ms")
    for (name, site), (n, ms) in rows[:40]:
        print(f"{ms:8.3f} ms {n:5d}x  {name:32s} {site}")


if __name__ == "__main__":
    main()
