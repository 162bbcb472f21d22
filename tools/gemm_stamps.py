"""Per-tile phase timing of the persistent GEMM from the diagnostic build's clock stamps.

    COMET_HIP_LIB=comet-pose-estimation_amd/libcomet_hip_stamp.so \
        python tools/gemm_stamps.py M N K [act] [f32|bf16] [resid]

(make -C comet-pose-estimation_amd STAMPS=1 builds the library.) Wave 0 of each workgroup stamps
the shader clock at each tile's k-loop start (0), before (1) and after (2) its epilogue; waves 0 and 4
(one SIMD's pair) stamp k-tile 3 of each tile: its start, k-step 0 issued, past the waits, past the
barrier, k-step 1 issued. Prints, over the workgroups, the k-loop and epilogue cycles per tile, the
gap between tiles and the k-tile-3 segments per wave. Only 256 x 256 instances keep their counted
vmcnt waits exact with the stamp stores in the loop (the A-ring instances leave pieces in flight).
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
from comet_amd import _lib as L, ops  # noqa: E402

WG, TILES = 256, 64


def main():
    M, N, K = (int(v) for v in sys.argv[1:4])
    ln_mode = sys.argv[4][3:] if len(sys.argv) > 4 and sys.argv[4].startswith("ln_") else None  # ln_norm2 / ln_dual / ln_dual_ctx
    act = int(sys.argv[4]) if len(sys.argv) > 4 and ln_mode is None else 0
    odt = torch.float32 if len(sys.argv) > 5 and sys.argv[5] == "f32" else torch.bfloat16
    res = len(sys.argv) > 6 and sys.argv[6] == "1"
    lib = L.load()
    if not hasattr(lib, "comet_gemm_stamps"):
        raise SystemExit(f"{L.LIB_PATH} is not the STAMPS=1 build")
    lib.comet_gemm_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int]
    x = (torch.rand(M, K, device="cuda") * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device="cuda") * 2 - 1) * 0.05).to(torch.bfloat16)
    b = torch.rand(N, device="cuda")
    r = torch.rand(M, N, device="cuda", dtype=odt) if res else None
    out = torch.empty(M, N, device="cuda", dtype=odt)
    if ln_mode is not None:  # row-LN GEMM (comet_gemm_rowln): f32 residual stream + LayerNorm epilogue
        r = torch.rand(M, N, device="cuda")
        z = (torch.rand(N, device="cuda"), torch.rand(N, device="cuda"), 1e-5) if ln_mode == "dual_ctx" else None
        odt = torch.float32
        call = lambda: ops.linear_rowln(x, w, b, r, raw=ln_mode == "norm2", y16_eps=1e-6, z=z)  # noqa: E731
    else:
        call = lambda: ops.linear(x, w, bias=b, act=act, resid=r, out=out, out_dtype=odt)  # noqa: E731
    for _ in range(20):  # warm (clock settles under load)
        call()
    torch.cuda.synchronize()
    lib.comet_gemm_stamps(None, 0, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    call()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3
    buf = np.zeros(WG * TILES * 8, dtype=np.uint64)
    lib.comet_gemm_stamps(buf.ctypes.data, buf.size, 0)
    st = buf.reshape(WG, TILES, 8).astype(np.int64)
    used = st[:, 0, 0] != 0
    st = st[used]
    kl, ep, gap, ntile = [], [], [], []
    # intra-k-tile stamps of k-tile 3 (waves 0 and 4: tile slots t and t + 32): 3 k-tile start,
    # 4 k-step 0 issued, 5 past the waits, 6 past the barrier, 7 k-step 1 issued
    seg = {w: {"k-step 0 issue": [], "waits": [], "barrier": [], "k-step 1 issue": [], "k-tile": []} for w in (0, 4)}
    for w_ in st:
        n = min(int(np.count_nonzero(w_[:32, 0])), 32)
        ntile.append(n)
        for t in range(n):
            kl.append(w_[t, 1] - w_[t, 0])
            ep.append(w_[t, 2] - w_[t, 1])
            if t + 1 < n:
                gap.append(w_[t + 1, 0] - w_[t, 2])
            for w, row in ((0, w_[t]), (4, w_[t + 32])):
                if all(row[i] for i in (3, 4, 5, 6, 7)):
                    d = seg[w]
                    d["k-step 0 issue"].append(row[4] - row[3])
                    d["waits"].append(row[5] - row[4])
                    d["barrier"].append(row[6] - row[5])
                    d["k-step 1 issue"].append(row[7] - row[6])
                    d["k-tile"].append(row[7] - row[3])
    f = lambda a: f"mean {np.mean(a):8.0f}  p10 {np.percentile(a, 10):8.0f}  p90 {np.percentile(a, 90):8.0f}"  # noqa: E731
    nk = K // 64  # (s_memtime counters are per XCD: only differences within a workgroup are used)
    print(f"M{M} N{N} K{K} {('rowln ' + ln_mode) if ln_mode else f'act{act}'} {odt} res{int(res)}: {us:.1f} us, {2 * M * N * K / us / 1e6:.0f} TF/s; "
          f"{len(st)} workgroups, tiles per workgroup (first 32) {min(ntile)}-{max(ntile)}, {nk} k-tiles per tile")
    print(f"  k-loop per tile   (cycles) {f(kl)}   per k-tile {np.mean(kl) / nk:.0f}")
    for w in (0, 4):
        for k, v in seg[w].items():
            if v:
                print(f"  k-tile 3, wave {w}: {k:15s} {f(v)}")
    print(f"  epilogue per tile (cycles) {f(ep)}")
    print(f"  gap to next tile  (cycles) {f(gap) if gap else '-'}")
    print(f"  share: k-loop {np.sum(kl) / (np.sum(kl) + np.sum(ep) + np.sum(gap)):.3f}  "
          f"epilogue {np.sum(ep) / (np.sum(kl) + np.sum(ep) + np.sum(gap)):.3f}")


if __name__ == "__main__":
    main()
