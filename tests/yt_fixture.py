"""Synthetic on-disk sequences in YTDataset's format (kubric_movif_SFM_dataset_YT.py:113-172) for
the data-path tests and tools/gen_golden.py --data: PNG frames (lossless, so every decoder sees the
same pixels), PNG masks of a moving box, 4x4 GT poses (random rotations, z in [4, 12]) as text."""
import os

import numpy as np
from PIL import Image


def make_dataset(root, n_models=1, n_seqs=2, frames=12, size=(160, 120), seed=0):
    """root/model{i}/seq_{j}/{frames,GroundTruth,Mask}; size = (width, height)."""
    rng = np.random.default_rng(seed)
    W, H = size
    for m in range(n_models):
        for q in range(n_seqs):
            d = os.path.join(root, f"model{m}", f"seq_{q}")
            for sub in ("frames", "GroundTruth", "Mask"):
                os.makedirs(os.path.join(d, sub), exist_ok=True)
            # box of the object: drifts across the frame, partly leaves it in sequence 1
            bw, bh = int(W * 0.35), int(H * 0.4)
            x, y = rng.integers(0, W - bw), rng.integers(0, H - bh)
            vx, vy = rng.integers(-6, 7), rng.integers(-5, 6)
            for f in range(frames):
                img = rng.integers(0, 256, size=(H, W, 3), dtype=np.uint8)
                img[::7] //= 3  # some structure for the filters
                Image.fromarray(img).save(os.path.join(d, "frames", f"frame_{f:04d}.png"))
                mask = np.zeros((H, W), np.uint8)
                x0, y0 = int(np.clip(x + vx * f, -bw // 2, W - 1)), int(np.clip(y + vy * f, -bh // 2, H - 1))
                mask[max(y0, 0):max(y0 + bh, 0), max(x0, 0):max(x0 + bw, 0)] = 255
                if q == 1 and f == 3:
                    mask[:] = 0  # an empty mask: the whole frame is its box
                Image.fromarray(mask).save(os.path.join(d, "Mask", f"mask_{f:04d}.png"))
                a = rng.normal(size=4)
                a /= np.linalg.norm(a)
                w_, x_, y_, z_ = a
                R = np.array([[1 - 2 * (y_ * y_ + z_ * z_), 2 * (x_ * y_ - z_ * w_), 2 * (x_ * z_ + y_ * w_)],
                              [2 * (x_ * y_ + z_ * w_), 1 - 2 * (x_ * x_ + z_ * z_), 2 * (y_ * z_ - x_ * w_)],
                              [2 * (x_ * z_ - y_ * w_), 2 * (y_ * z_ + x_ * w_), 1 - 2 * (x_ * x_ + y_ * y_)]])
                M = np.eye(4)
                M[:3, :3] = R
                M[:3, 3] = [rng.normal() * 0.5, rng.normal() * 0.5, 4 + 8 * rng.random()]
                np.savetxt(os.path.join(d, "GroundTruth", f"obj_w2c_{f:04d}.txt"), M)
    return root
