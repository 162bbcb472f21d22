"""One op, many times, bit-compared with its first result: run two at once (tools/gpu/steps.sh
pair:...) to see whether the op's result depends on another process sharing the GPU.

    python tools/op_repeat.py <case> [reps]
cases:
  rowln_split   comet_gemm_rowln, M 8192 K 1536 -> N 384 (+ bias, residual, bf16 LN copy): the
                split-K partials (256-row kernel) + LN reduce path (the tracker's fc2 at B = 1)
  rowln_pp      comet_gemm_rowln, M 65536 K 384 -> N 384: the persistent row-LN kernel
  split_gemm    comet_gemm with split_k = 2 on the same operands (128 x 128 kernel partials + the
                generic split reduce), f32 out
  tile128       comet_gemm on the 128 x 128 kernel without split (M 2048, K 1536 -> N 384)
  conv          comet_conv2d_nhwc 3x3 64 -> 64 on 8 x 64 x 64
  torch_mm      torch bf16 512^3 matmul (hipBLASLt)
  big_gemm      comet_gemm, M 8192 K 1536 -> N 384 f32 + bias + residual without split
  pp_gelu       comet_gemm persistent, M 8192 K 384 -> N 1536 GELU bf16
  ln            comet_layernorm (dual f32 + bf16 copy), M 65536 x 384: wave reductions, no LDS-DMA
  attn          flash attention forward, 512 x 8 heads x 16 tokens x 48 (LDS, no LDS-DMA)
  pp_ping       comet_gemm persistent ping-pong (asm LDS-DMA), M 74368 K 768 -> N 2304 bf16
  shfl0..6      comet_shfl_probe mode 0 (ds_bpermute), 1 (DPP + permlane), 2 (own LDS words),
                3 (two sums as packed v_pk_add_f32), 4 (the same two sums, scalar adds), 5 (one
                v_pk_add_f32 with op_sel cross-half reads), 6 (plain v_pk_add_f32), 7-11 (single VOP3P
                op_sel forms), 12 (an MFMA stream, as a load): the count of wrong lane results,
                which must stay 0
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "comet-pose-estimation_amd")]


def where(a, b):
    d = a != b
    n = int(d.sum())
    if n == 0:
        return None
    d2 = d.reshape(-1, a.shape[-1])
    rows = d2.any(1).nonzero().flatten()
    cols = d2.any(0).nonzero().flatten()
    return (f"{n} differ, max |diff| {(a.float() - b.float()).abs().max().item():.3e}; rows {rows[:8].tolist()}.. "
            f"({rows.numel()}), cols {cols.min().item()}..{cols.max().item()} ({cols.numel()})")


def fit_ln(c, y, yref):
    """For the first row whose bf16 LN copy differs: the row statistics of c (f64), and the (mean,
    1/std) that best explain the differing lane group's y16 values (least squares on y = (c - m) r)."""
    d = (y != yref).any(1).nonzero().flatten()
    r = int(d[0])
    cr = c[r].double().cpu()
    mu, var = cr.mean().item(), cr.var(unbiased=False).item()
    cols = (y[r] != yref[r]).nonzero().flatten().cpu()
    lo = int(cols.min()) // 64 * 64
    sl = slice(lo, lo + 64)
    for name, t in (("got", y), ("ref", yref)):
        yy = t[r, sl].double().cpu()
        A = torch.stack([cr[sl], torch.ones(64, dtype=torch.float64)], 1)
        sol = torch.linalg.lstsq(A, yy.unsqueeze(1)).solution.flatten()
        rr, b = sol[0].item(), sol[1].item()
        print(f"    row {r} cols {lo}..{lo + 63} {name}: fitted 1/std {rr:.6f} mean {-b / rr:.6f}  "
              f"(row: 1/std {1 / (var + 1e-5) ** 0.5:.6f} mean {mu:.6f})", flush=True)
    print(f"    c row: first 8 of the group {cr[sl][:8].tolist()}", flush=True)
    out = os.environ.get("OP_REPEAT_DUMP")
    if out and not os.path.exists(out):
        import numpy as np
        np.savez(out, row=r, c=c[r].float().cpu().numpy(), y=y[r].float().cpu().numpy(),
                 yref=yref[r].float().cpu().numpy())


def main():
    from comet_amd import ops
    case = sys.argv[1]
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    g = torch.Generator(device="cuda").manual_seed(1)
    if case in ("rowln_split", "split_gemm", "big_gemm"):
        M, K, N = 8192, 1536, 384
    elif case in ("rowln_pp", "ln"):
        M, K, N = 65536, 384, 384
    elif case == "pp_ping":
        M, K, N = 74368, 768, 2304
    else:
        M, K, N = 8192, 384, 1536
    x = torch.randn(M, K, device="cuda", generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda", generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device="cuda", generator=g)
    r = torch.randn(M, N, device="cuda", generator=g)

    xc = torch.randn(8, 64, 64, 64, device="cuda", generator=g).to(torch.bfloat16)
    wc = (torch.randn(64, 9 * 64, device="cuda", generator=g) * 0.05).to(torch.bfloat16)
    xs = torch.randn(512, 512, device="cuda", generator=g).to(torch.bfloat16)
    ws_ = torch.randn(512, 512, device="cuda", generator=g).to(torch.bfloat16)

    def run():
        if case.startswith("shfl"):
            import ctypes
            from comet_amd import _lib as L
            bad = torch.zeros(1, device="cuda", dtype=torch.int32)
            L.check(L.load().comet_shfl_probe(2048, 64, int(case[4:]), ctypes.c_void_p(bad.data_ptr()), ops.stream()),
                    "comet_shfl_probe")
            return [bad]
        if case.startswith("rowln"):
            c, y, _ = ops.linear_rowln(x, w, b, r, raw=True, y16_eps=1e-5)
            return [c, y]
        if case == "split_gemm":
            c = torch.empty(M, N, device="cuda")
            ops.gemm_raw(x, w, c, m=M, n=N, k=K, layout_a=0, lda=K, layout_b=0, ldb=K, ldc=N, split_k=2)
            return [c]
        if case == "ln":
            c, y = ops.layernorm(r, eps=1e-5, out_dtype=torch.float32, dual=True)
            return [c, y]
        if case == "attn":
            q = x[:, :384].reshape(512, 16, 384)
            return [ops.attention(q, q, q, 8, 384 ** -0.5)] if hasattr(ops, "attention") else []
        if case == "pp_ping":
            return [ops.linear(x, w, out_dtype=torch.bfloat16)]
        if case == "tile128":  # the 128 x 128 kernel without split (M < 4096: no 256-row plan)
            c = torch.empty(2048, N, device="cuda")
            ops.gemm_raw(x[:2048], w, c, m=2048, n=N, k=K, layout_a=0, lda=K, layout_b=0, ldb=K, ldc=N)
            return [c]
        if case == "conv":  # 3x3 64 -> 64 NHWC convolution (the BasicEncoder's)
            return [ops.conv2d_nhwc(xc, wc, 3, 3, 1, 1)]
        if case == "torch_mm":  # hipBLASLt, small enough for several workgroups per CU
            return [xs @ ws_]
        if case == "big_gemm":
            return [ops.linear(x, w, bias=b, resid=r, out_dtype=torch.float32)]
        return [ops.linear(x, w, bias=b, act=1, out_dtype=torch.bfloat16)]

    ref = [t.clone() for t in run()]
    torch.cuda.synchronize()
    ref_h = [t.cpu() for t in ref]
    print(f"{case}: plan {tuple(ops._PLAN)}", flush=True)
    if case.startswith("shfl"):
        print(f"{case}: first run counts {ref_h[0].item()} wrong lane results", flush=True)
    bad = 0
    t0 = time.time()
    for i in range(reps):
        outs = run()
        for k, (o, rr) in enumerate(zip(outs, ref)):
            wh = where(o, rr)
            if wh is not None:
                bad += 1
                if bad <= 5:
                    # read again: a second device comparison, and the host copy (DMA engine, not the
                    # compute units' caches) -- which tells a wrong value in memory from a stale read
                    torch.cuda.synchronize()
                    again = where(o, rr)
                    host = where(o.cpu(), ref_h[k])
                    print(f"rep {i} output {k}: {wh}\n    device re-read: {again}\n    host copy: {host}", flush=True)
                    if case.startswith("rowln") and k == 1:
                        fit_ln(outs[0], o, rr)
        if time.time() - t0 > 60:
            print(f"stopping at rep {i} (time)", flush=True)
            break
    torch.cuda.synchronize()
    print(f"{case}: {bad} differing outputs over {i + 1} repetitions", flush=True)
    if case.startswith("shfl"):
        print(f"{case}: last run counts {outs[0].item()} wrong lane results", flush=True)


if __name__ == "__main__":
    main()
