"""Data-path throughput: one training sequence = T=16 frames 640 x 480 cropped to a
square box and LANCZOS-resized to 512 x 512 + ImageNet normalisation. Reference path: PIL crop +
resize per frame + float normalisation on the CPU (kubric_movif_SFM_dataset_YT.py:236-260); build:
upload the uint8 frames + comet_lanczos_crop_resize. Decoding is excluded from both (same PIL
decoder). Prints sequences/s for each.

    python tools/data_bench.py
"""
import os
import sys
import time

import numpy as np
import torch
from PIL import Image

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd.data import crop_resize_normalize  # noqa: E402

T, H, W, OUT, BOX = 16, 480, 640, (512, 512), (150, 60, 510, 420)
MEAN = torch.tensor([0.485, 0.456, 0.406])[None, :, None, None]
STD = torch.tensor([0.229, 0.224, 0.225])[None, :, None, None]


def cpu_path(frames):
    rgbs = [np.asarray(Image.fromarray(f).crop(BOX).resize(OUT, Image.Resampling.LANCZOS)) for f in frames]
    video = torch.from_numpy(np.stack(rgbs, 0)).permute(0, 3, 1, 2).float() / 255.0
    return (video - MEAN) / STD


def main():
    torch.set_num_threads(1)
    frames = np.random.default_rng(0).integers(0, 256, size=(T, H, W, 3), dtype=np.uint8)
    cpu_path(frames)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < 3.0:
        cpu_path(frames)
        n += 1
    cpu = n / (time.perf_counter() - t0)
    host = torch.from_numpy(frames).pin_memory()
    dev = host.cuda()
    for _ in range(3):
        crop_resize_normalize(dev, BOX, OUT)
    torch.cuda.synchronize()
    iters = 200
    t0 = time.perf_counter()
    for _ in range(iters):
        crop_resize_normalize(dev, BOX, OUT)
    torch.cuda.synchronize()
    gpu = iters / (time.perf_counter() - t0)
    t0 = time.perf_counter()
    for _ in range(iters):
        crop_resize_normalize(host.cuda(non_blocking=True), BOX, OUT)
    torch.cuda.synchronize()
    gpu_up = iters / (time.perf_counter() - t0)
    print(f"T={T} {W}x{H} -> {OUT[0]}x{OUT[1]}: PIL CPU path (1 thread) {cpu:.1f} seq/s | HIP path, frames in HBM "
          f"{gpu:.0f} seq/s | incl. pinned H2D upload {gpu_up:.0f} seq/s")


if __name__ == "__main__":
    main()
