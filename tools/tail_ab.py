"""Memory-bound tail kernels on the step's largest shapes, each timed with HIP events in alternation
with and without one measurement environment setting (read per launch).

    python tools/tail_ab.py VAR=VALUE [VAR=VALUE ...]
e.g. COMET_LN_WGS=4096 (a LayerNorm-forward grid-size switch measured in round 6 and not kept), COMET_COLSUM_WGS=1024
(act_bwd_colsum workgroup target).
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tools"), os.path.join(ROOT, "comet-pose-estimation_amd")]
from comet_amd import _lib as L  # noqa: E402
from comet_amd import ops  # noqa: E402
from tile_bench import timed  # noqa: E402


def main():
    arms = [a.split("=", 1) for a in sys.argv[1:]]
    torch.manual_seed(0)
    x = torch.randn(74368, 768, device="cuda")
    w, b = torch.randn(768, device="cuda"), torch.randn(768, device="cuda")
    g = torch.randn(73856, 768, device="cuda")
    gb = torch.randn(73856, 2304, device="cuda").to(torch.bfloat16)
    db = torch.empty(2304, device="cuda")
    x32 = torch.randn(65536, 32, device="cuda")
    x128 = torch.randn(65536, 128, device="cuda")
    w32, w128 = torch.randn(32, device="cuda"), torch.randn(128, device="cuda")
    fpyr = [torch.randn(65536, n, n, 32, device="cuda").to(torch.bfloat16) for n in (31, 15, 7)]
    ffeat = torch.randn(65536, 32, device="cuda")
    fco = torch.rand(65536, 2, device="cuda") * 31
    fout = torch.empty(65536, 147, device="cuda")
    B, N, S, lat, corrdim = 1, 4096, 16, 128, 405
    tdim = 2 * (lat // 2) + 2 + corrdim + lat + 1  # 664, the coarse tracker
    tco = torch.rand(B * N * S, 2, device="cuda") * 60
    tfe = torch.randn(B * N * S, lat, device="cuda")
    tcorr = torch.randn(B * N * S, corrdim, device="cuda")
    tpos = torch.randn(B * N, tdim, device="cuda")
    tx = torch.empty(B * N * S, (tdim + 63) // 64 * 64, device="cuda", dtype=torch.bfloat16)
    cases = {
        "tracker_tokens coarse (65536 rows, 664 -> 704 bf16)": (
            lambda: ops.tracker_tokens(tco, tfe, lat, tcorr, corrdim, tpos, tdim, tx, B * N * S, S),
            65536 * (704 * 2 + corrdim * 4 + lat * 4)),
        "corr_sample fine (65536 rows, C 32, r 3, 3 levels)": (
            lambda: ops.corr_sample(fpyr, 3, ffeat, fco, fout, 0, 4096, 1, 16), 65536 * (147 * 4 + 32 * 4 + 8 + 3 * 100 * 64)),
        "layernorm f32 65536 x 32 (tracker GroupNorm(1, 32))": (
            lambda: ops.layernorm(x32, w32, w32, eps=1e-5, out_dtype=torch.float32), 65536 * 32 * 8),
        "layernorm f32 65536 x 128 (tracker GroupNorm(1, 128))": (
            lambda: ops.layernorm(x128, w128, w128, eps=1e-5, out_dtype=torch.float32), 65536 * 128 * 8),
        "layernorm f32 -> bf16 74368 x 768 (DINOv2 norm1/2)": (
            lambda: ops.layernorm(x, w, b, eps=1e-6, out_dtype=torch.bfloat16), 74368 * 768 * 6),
        "act_bwd_colsum f32 -> bf16 + colsum 73856 x 768": (
            lambda: ops.act_bwd_colsum(L.ACT_NONE, None, g, out_dtype=torch.bfloat16, dbias=db[:768]), 73856 * 768 * 6),
        "act_bwd_colsum bf16 colsum 73856 x 2304": (
            lambda: ops.act_bwd_colsum(L.ACT_NONE, None, gb, dbias=db, want_out=False), 73856 * 2304 * 2),
    }
    for name, (fn, nbytes) in cases.items():
        res = {"default": []}
        for k, v in arms:
            res[f"{k}={v}"] = []
        for _ in range(3):
            res["default"].append(timed(fn))
            for k, v in arms:
                os.environ[k] = v
                res[f"{k}={v}"].append(timed(fn))
                del os.environ[k]
        print(name + ": " + "  ".join(f"{a} {min(t):7.1f} us ({nbytes / min(t) / 1e6:.2f} TB/s)" for a, t in res.items()),
              flush=True)


if __name__ == "__main__":
    main()
