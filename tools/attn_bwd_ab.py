"""A/B of the flash attention backward kernels on the camera head's shapes: the default against
the variant an environment switch selects (e.g. COMET_ATTN_BWD_SEQ=1), interleaved rounds in one
process, random data, with the max difference of the two gradient sets.

    python tools/attn_bwd_ab.py COMET_ATTN_BWD_SEQ > gpurun_out/attn_bwd_ab.txt
"""
import os
import statistics
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import ops  # noqa: E402

SHAPES = [  # (name, B, H, Lq, Lk, D)
    ("head self", 128, 8, 577, 577, 96),
    ("head cross", 8, 8, 8655, 577, 96),
    ("dino-like self D64", 128, 12, 581, 581, 64),
    ("tracker D48", 128, 8, 512, 64, 48),
]


def main():
    var = sys.argv[1] if len(sys.argv) > 1 else "COMET_ATTN_BWD_SEQ"
    dev = "cuda"
    print(f"variant switch: {var}=1 (B arm)")
    print(f"{'shape':22s} | A ms  TF/s | B ms  TF/s | B/A time | max|dA-dB|", flush=True)
    for name, B, H, Lq, Lk, D in SHAPES:
        C = H * D
        g = torch.Generator(device=dev).manual_seed(0)
        q = torch.randn(B, Lq, C, device=dev, generator=g).to(torch.bfloat16)
        k = torch.randn(B, Lk, C, device=dev, generator=g).to(torch.bfloat16)
        v = torch.randn(B, Lk, C, device=dev, generator=g).to(torch.bfloat16)
        scale = D ** -0.5
        o, lse = ops.attention(q, k, v, H, scale=scale, lse=True)
        do = torch.randn(B, Lq, C, device=dev, generator=g).to(torch.bfloat16)
        grads = {}

        def run(arm):
            if arm == "B":
                os.environ[var] = "1"
            else:
                os.environ.pop(var, None)
            dq, dk, dv = torch.empty_like(q), torch.empty_like(k), torch.empty_like(v)
            ops.attention_bwd(q, k, v, o, lse, do, H, scale, dq, dk, dv)
            grads[arm] = (dq, dk, dv)

        ts = {"A": [], "B": []}
        for arm in ("A", "B"):
            run(arm)
        torch.cuda.synchronize()
        for _ in range(5):
            for arm in ("A", "B"):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(5):
                    run(arm)
                e1.record()
                torch.cuda.synchronize()
                ts[arm].append(e0.elapsed_time(e1) / 5)
        os.environ.pop(var, None)
        fl = 10.0 * B * H * Lq * Lk * D
        a, b = statistics.median(ts["A"]), statistics.median(ts["B"])
        d = max((x.float() - y.float()).abs().max().item() for x, y in zip(grads["A"], grads["B"]))
        print(f"{name:22s} | {a:.4f} {fl / a / 1e9:6.1f} | {b:.4f} {fl / b / 1e9:6.1f} | {b / a:.3f} | {d:.3e}", flush=True)


if __name__ == "__main__":
    main()
