"""Tensor-level wrappers over the C-ABI (raw kernels, no autograd).

Every function enqueues on torch's current HIP stream and returns device tensors. No op here
has a CPU/PyTorch fallback: a missing library or an unsupported shape raises.
"""
import ctypes

import torch

from . import _lib as L
from .profiler import PROF

_DT = {torch.float32: L.F32, torch.bfloat16: L.BF16}


def dt(t):
    try:
        return _DT[t.dtype]
    except KeyError:
        raise L.CometHipError(f"unsupported dtype {t.dtype}") from None


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return None if t is None else t.data_ptr()


def _req_cuda(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise L.CometHipError("comet ops need device tensors (no CPU fallback)")


# ------------------------------------------------------------------------------------------
# GEMM
# ------------------------------------------------------------------------------------------
def gemm_raw(a, b, c, *, m, n, k, layout_a, lda, layout_b, ldb, ldc, batch=(1, 1),
             stride_a=(0, 0), stride_b=(0, 0), stride_c=(0, 0), bias=None, bias_mode=0,
             stride_bias=(0, 0), resid=None, ldr=0, stride_r=(0, 0), beta=1.0, aux=None,
             ldaux=0, stride_aux=(0, 0), alpha=1.0, act=L.ACT_NONE, split_k=0, compute=None):
    _req_cuda(a, b, c, bias, resid, aux)
    conv_a = conv_b = 0
    cdt = compute or (a.dtype if a.dtype == b.dtype else torch.bfloat16)
    if cdt == torch.bfloat16:
        # f32 operands of a bf16 GEMM are rounded to bf16 on load when their rows allow 16-B
        # vectors (convert_b: layout_b 1 only), otherwise by a cast pass here
        if a.dtype == torch.float32:
            if _cvt_ok(a, lda, stride_a, k if layout_a == 0 else m):
                conv_a = 1
            else:
                a = _dense_bf16(a)
        if b.dtype == torch.float32:
            if layout_b == 1 and _cvt_ok(b, ldb, stride_b, n):
                conv_b = 1
            else:
                b = _dense_bf16(b)
    elif a.dtype != torch.float32 or b.dtype != torch.float32:
        raise L.CometHipError("gemm: an f32 GEMM needs f32 operands")
    if bias is not None and bias.dtype != torch.float32:
        raise L.CometHipError("gemm: bias must be f32")
    for t in (resid, aux):
        if t is not None and t.dtype != c.dtype:
            raise L.CometHipError("gemm: resid/aux must have the output dtype")
    g = L.GemmArgs()
    g.dtype_ab = _DT[cdt]
    g.dtype_c, g.layout_a, g.layout_b = dt(c), layout_a, layout_b
    g.convert_a, g.convert_b = conv_a, conv_b
    g.m, g.n, g.k = m, n, k
    g.batch[0], g.batch[1] = batch
    g.a, g.lda = _p(a), lda
    g.stride_a[0], g.stride_a[1] = stride_a
    g.b, g.ldb = _p(b), ldb
    g.stride_b[0], g.stride_b[1] = stride_b
    g.c, g.ldc = _p(c), ldc
    g.stride_c[0], g.stride_c[1] = stride_c
    g.bias, g.bias_mode = _p(bias), (bias_mode if bias is not None else 0)
    g.stride_bias[0], g.stride_bias[1] = stride_bias
    g.resid, g.ldr = _p(resid), ldr
    g.stride_r[0], g.stride_r[1] = stride_r
    g.aux, g.ldaux = _p(aux), ldaux
    g.stride_aux[0], g.stride_aux[1] = stride_aux
    g.alpha, g.beta, g.act = alpha, beta, act
    g.split_k = split_k
    lib = L.load()
    ws_bytes = ctypes.c_int64(0)
    L.check(lib.comet_gemm_plan(ctypes.byref(g), ctypes.byref(ws_bytes), _PLAN), "comet_gemm_plan")
    ws = None
    if ws_bytes.value > 0:  # split-K partials (torch caching allocator: no device sync)
        ws = torch.empty((ws_bytes.value + 3) // 4, device=c.device, dtype=torch.float32)
        g.workspace, g.workspace_bytes = ws.data_ptr(), ws_bytes.value
    e0 = PROF.start()
    L.check(lib.comet_gemm(ctypes.byref(g), stream()), "comet_gemm")
    if e0 is not None:
        name = "comet_gemm|" + _plan_name(layout_a, layout_b, cdt, c.dtype, ws_bytes.value > 0 and _PLAN[0] != 3)
        if PROF.detail:
            name = (f"gemm L{layout_a}{layout_b} {a.dtype}->{c.dtype} M{m} N{n} K{k} b{batch[0]}x{batch[1]}"
                    f" act{act}{' bias' if bias is not None else ''}{' res' if resid is not None else ''}")
        nb = batch[0] * batch[1]
        io = (a.element_size() * m * k + b.element_size() * k * n +
              c.element_size() * m * n * (1 + (resid is not None) + (aux is not None)))
        PROF.stop(e0, name, 2.0 * m * n * k * nb, float(io * nb))
    return c


_PLAN = (ctypes.c_int32 * 3)()


def _plan_name(la, lb, cdt, odt, split):
    """Kernel instance of the last comet_gemm_plan (matches the rocprof kernel names:
    big::gemm_big_kernel<TC, BN, LA, LB, SPLIT>, bf::gemm_bf16_kernel<...>, gemm_skinny_kernel)."""
    kind, bn = _PLAN[0], _PLAN[1]
    out = "split" if split else ("bf16" if odt == torch.bfloat16 else "f32")
    if kind == 0:
        return f"skinny.{out}"
    if kind == 1:
        return f"big{bn}.L{la}{lb}.{out}"
    if kind == 3:  # persistent tile kernel: _PLAN[2] = tile rows
        return f"pp{_PLAN[2]}x{bn}.L{la}{lb}.{out}"
    return f"tile128.L{la}{lb}.{'bf16' if cdt == torch.bfloat16 else 'f32'}.{out}"


def _cvt_ok(t, ld, st, contig):
    return t.data_ptr() % 16 == 0 and ld % 8 == 0 and st[0] % 8 == 0 and st[1] % 8 == 0 and contig % 8 == 0


def _dense_bf16(t):
    """bf16 copy of an f32 GEMM operand that cannot be converted on load (same strides)."""
    if t.is_contiguous():
        return cast(t, torch.bfloat16)
    out = torch.empty_strided(t.shape, t.stride(), device=t.device, dtype=torch.bfloat16)
    out.copy_(t)  # rare misaligned view; keeps the caller's ld / strides valid
    return out


def linear(x, w, bias=None, act=L.ACT_NONE, resid=None, out=None, out_dtype=None, aux=None,
           beta=1.0, alpha=1.0):
    """y[..., N] = act(x[..., K] @ w[N, K]^T + bias) + beta*resid. x rows may be strided."""
    K = x.shape[-1]
    N = w.shape[0]
    if w.shape[1] != K:
        raise L.CometHipError(f"linear: x has K={K}, weight {tuple(w.shape)}")
    x2 = x.reshape(-1, K) if x.dim() != 2 else x
    if x2.stride(-1) != 1:
        x2 = x2.contiguous()
    M = x2.shape[0]
    if out is None:
        out = torch.empty(*x.shape[:-1], N, device=x.device, dtype=out_dtype or x.dtype)
    o2 = out.reshape(-1, N) if out.dim() != 2 else out
    if o2.stride(-1) != 1:
        raise L.CometHipError("linear: output must be row-contiguous")
    r2 = None
    if resid is not None:
        r2 = resid.reshape(-1, N) if resid.dim() != 2 else resid
    a2 = None
    if aux is not None:
        a2 = aux.reshape(-1, N) if aux.dim() != 2 else aux
    wc = w if w.stride(-1) == 1 else w.contiguous()
    gemm_raw(x2, wc, o2, m=M, n=N, k=K, layout_a=0, lda=x2.stride(0), layout_b=0,
             ldb=wc.stride(0), ldc=o2.stride(0), bias=bias, bias_mode=1, resid=r2,
             ldr=(r2.stride(0) if r2 is not None else 0), beta=beta, aux=a2,
             ldaux=(a2.stride(0) if a2 is not None else 0), alpha=alpha, act=act)
    return out


def _rowln_args(x2, wc, o2, bias, r2):
    M, K = x2.shape
    N = wc.shape[0]
    g = L.GemmArgs()
    g.dtype_ab, g.dtype_c, g.layout_a, g.layout_b = L.BF16, L.F32, 0, 0
    g.m, g.n, g.k = M, N, K
    g.batch[0] = g.batch[1] = 1
    g.a, g.lda = x2.data_ptr(), x2.stride(0)
    g.b, g.ldb = wc.data_ptr(), wc.stride(0)
    g.c, g.ldc = o2.data_ptr(), o2.stride(0)
    g.bias, g.bias_mode = _p(bias), (1 if bias is not None else 0)
    g.resid, g.ldr = r2.data_ptr(), r2.stride(0)
    g.alpha, g.beta, g.act = 1.0, 1.0, L.ACT_NONE
    return g


def linear_rowln_ok(x, w, resid, bias=None, z=None):
    """True when comet_gemm_rowln takes this Linear (bf16 operands, f32 residual output, N in
    {256, 384}, K % 64 == 0, M >= 4096, 16-B aligned bias / affine LN vectors; see
    include/comet_hip.h)."""
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or resid is None or resid.dtype != torch.float32:
        return False
    K, N = x.shape[-1], w.shape[0]
    if N not in (256, 384) or resid.shape[-1] != N or x.stride(-1) != 1 or w.stride(-1) != 1:
        return False
    # the kernel reads bias and the affine LN weight / shift four columns (16 B) at a time
    for t in (bias, *(z[:2] if z is not None else ())):
        if t is not None and (t.data_ptr() % 16 != 0 or t.dtype != torch.float32 or not t.is_contiguous()):
            return False
    x2 = x.reshape(-1, K)
    r2 = resid.reshape(-1, N)
    g = _rowln_args(x2, w, r2, bias, r2)
    return bool(L.load().comet_gemm_rowln_ok(ctypes.byref(g)))


def _dact_args(dy2, wc, out):
    M, N2 = dy2.shape
    K2 = wc.shape[1]
    g = L.GemmArgs()
    g.dtype_ab, g.dtype_c, g.layout_a, g.layout_b = L.BF16, L.BF16, 0, 1
    g.m, g.n, g.k = M, K2, N2
    g.batch[0] = g.batch[1] = 1
    g.a, g.lda = dy2.data_ptr(), dy2.stride(0)
    g.b, g.ldb = wc.data_ptr(), wc.stride(0)
    g.c, g.ldc = out.data_ptr(), out.stride(0)
    g.alpha, g.beta, g.act = 1.0, 1.0, L.ACT_NONE
    return g


def linear_dact_ok(dy2, wc, pre, act):
    """True when comet_gemm_dact takes the input gradient of y = Linear(h) fused with the backward
    of h = act(pre) (bf16 dY [M, N2] and weight [N2, K2], pre bf16 [M, K2]; include/comet_hip.h)."""
    if dy2.dtype != torch.bfloat16 or wc.dtype != torch.bfloat16 or pre is None or pre.dtype != torch.bfloat16:
        return False
    if dy2.dim() != 2 or pre.dim() != 2 or dy2.stride(-1) != 1 or wc.stride(-1) != 1 or pre.stride(-1) != 1:
        return False
    if pre.shape != (dy2.shape[0], wc.shape[1]) or dy2.shape[1] != wc.shape[0]:
        return False
    g = _dact_args(dy2, wc, pre)  # alignment of the output is that of a fresh tensor
    return bool(L.load().comet_gemm_dact_ok(ctypes.byref(g), act, pre.data_ptr(), pre.stride(0)))


def linear_dact(dy2, wc, pre, act, dbias=None):
    """dPre = act'(pre) * (dY @ W) in bf16 and dbias = its column sums, in one kernel
    (comet_gemm_dact): the hidden gradient of an MLP, fc2's dX fused with fc1's activation
    backward. dY [M, N2] bf16, W [N2, K2] (fc2.weight in the compute dtype), pre [M, K2] bf16."""
    _req_cuda(dy2, wc, pre, dbias)
    M, K2 = dy2.shape[0], wc.shape[1]
    out = torch.empty(M, K2, device=dy2.device, dtype=torch.bfloat16)
    g = _dact_args(dy2, wc, out)
    e0 = PROF.start()
    L.check(L.load().comet_gemm_dact(ctypes.byref(g), act, pre.data_ptr(), pre.stride(0), _p(dbias), stream()),
            "comet_gemm_dact")
    if e0 is not None:
        N2 = dy2.shape[1]
        name = f"gemm_dact M{M} N{K2} K{N2}" if PROF.detail else "comet_gemm_dact"
        PROF.stop(e0, name, 2.0 * M * K2 * N2, float(2 * M * N2 + 2 * N2 * K2 + 2 * M * K2 * 2))
    return out


def linear_rowln(x, w, bias, resid, *, raw=True, y16_eps=None, z=None):
    """v = x @ w^T + bias + resid (f32) with the row LayerNorms its consumers need written by the
    same kernel (comet_gemm_rowln). Returns (c, y16, z16):
      c   = v (raw) or LN(v; y16_eps) in f32 (raw=False: the dual copy of AttnBlock norm1),
      y16 = LN(v; y16_eps) in bf16 when y16_eps is not None,
      z16 = LN(v; z_eps) * z_w + z_b in bf16 when z = (z_w, z_b, z_eps)."""
    _req_cuda(x, w, bias, resid)
    K, N = x.shape[-1], w.shape[0]
    x2 = x.reshape(-1, K)
    r2 = resid.reshape(-1, N)
    M = x2.shape[0]
    c = torch.empty(*x.shape[:-1], N, device=x.device, dtype=torch.float32)
    o2 = c.view(-1, N)
    g = _rowln_args(x2, w, o2, bias, r2)
    a = L.RowLNArgs()
    a.raw_c = 1 if raw else 0
    y16 = z16 = None
    if y16_eps is not None or not raw:
        if y16_eps is None:
            raise L.CometHipError("linear_rowln: raw=False needs y16_eps")
        a.eps_y = float(y16_eps)
        y16 = torch.empty(*x.shape[:-1], N, device=x.device, dtype=torch.bfloat16)
        a.y16, a.ldy = y16.data_ptr(), N
    if z is not None:
        zw, zb, zeps = z
        z16 = torch.empty(*x.shape[:-1], N, device=x.device, dtype=torch.bfloat16)
        a.z16, a.ldz, a.zw, a.zb, a.eps_z = z16.data_ptr(), N, zw.data_ptr(), zb.data_ptr(), float(zeps)
    lib = L.load()
    ws_bytes = ctypes.c_int64(0)
    L.check(lib.comet_gemm_rowln_workspace(ctypes.byref(g), ctypes.byref(ws_bytes)), "comet_gemm_rowln_workspace")
    ws = None
    if ws_bytes.value > 0:  # split-K partials of the few-row path (torch caching allocator)
        ws = torch.empty((ws_bytes.value + 3) // 4, device=x.device, dtype=torch.float32)
        g.workspace, g.workspace_bytes = ws.data_ptr(), ws_bytes.value
    e0 = PROF.start()
    L.check(lib.comet_gemm_rowln(ctypes.byref(g), ctypes.byref(a), stream()), "comet_gemm_rowln")
    if e0 is not None:
        name = "comet_gemm_rowln"
        if PROF.detail:
            name = f"gemm_rowln M{M} N{N} K{K} raw{int(raw)} y16{int(y16 is not None)} z16{int(z16 is not None)}"
        io = 2 * M * K + 2 * K * N + 4 * M * N * 2 + 2 * M * N * ((y16 is not None) + (z16 is not None))
        PROF.stop(e0, name, 2.0 * M * N * K, float(io))
    return c, y16, z16


def _ln_args(c_shape, dev, raw, y16_eps, z):
    a = L.RowLNArgs()
    a.raw_c = 1 if raw else 0
    y16 = z16 = None
    N = c_shape[-1]
    if y16_eps is not None or not raw:
        if y16_eps is None:
            raise L.CometHipError("raw=False needs y16_eps")
        a.eps_y = float(y16_eps)
        y16 = torch.empty(*c_shape, device=dev, dtype=torch.bfloat16)
        a.y16, a.ldy = y16.data_ptr(), N
    if z is not None:
        zw, zb, zeps = z
        z16 = torch.empty(*c_shape, device=dev, dtype=torch.bfloat16)
        a.z16, a.ldz, a.zw, a.zb, a.eps_z = z16.data_ptr(), N, zw.data_ptr(), zb.data_ptr(), float(zeps)
    return a, y16, z16


# ------------------------------------------------------------------------------------------
# LayerNorm
# ------------------------------------------------------------------------------------------
def _rows2d(x):
    """(rows, row stride) of a tensor whose last dim is unit-stride and whose leading dims
    collapse to a single uniform row stride; None if they do not."""
    if x.stride(-1) != 1:
        return None
    C = x.shape[-1]
    rows = x.numel() // C
    if x.dim() == 1:
        return rows, C
    lead = [(s, st) for s, st in zip(x.shape[:-1], x.stride()[:-1]) if s != 1]
    if not lead:
        return rows, C
    ld = lead[-1][1]
    expect = ld
    for s, st in reversed(lead):
        if st != expect:
            return None
        expect = st * s
    return rows, ld


def layernorm(x, weight=None, bias=None, eps=1e-5, out_dtype=None, stats=False, out=None, relu=False,
              dual=False):
    """Row LayerNorm. dual=True also returns a bf16 copy of the output (written by the same
    kernel): (y, y_bf16[, mean, rstd])."""
    _req_cuda(x)
    C = x.shape[-1]
    r = _rows2d(x)
    xc = x
    if r is None:
        xc = x.contiguous()
        r = _rows2d(xc)
    rows, ldx = r
    y = out if out is not None else torch.empty(x.shape, device=x.device, dtype=out_dtype or x.dtype)
    ry = _rows2d(y)
    if ry is None:
        raise L.CometHipError("layernorm: output rows must be uniformly strided")
    y2 = torch.empty(x.shape, device=x.device, dtype=torch.bfloat16) if dual else None
    mean = rstd = None
    if stats:
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    L.check(L.load().comet_layernorm_fwd(dt(xc), dt(y), _p(xc), _p(weight), _p(bias), _p(y), _p(y2), _p(mean),
                                         _p(rstd), rows, C, ldx, ry[1], C, float(eps), int(relu), stream()),
            "layernorm")
    outs = (y, y2) if dual else (y,)
    if stats:
        outs = outs + (mean, rstd)
    return outs if len(outs) > 1 else y


def layernorm_bwd(x, dy, mean, rstd, weight=None, dweight=None, dbias=None, dx=None, accumulate=False, dy2=None,
                  dx_dtype=torch.float32):
    """dx = LN backward of dy (+ dy2, bf16); dweight/dbias accumulated."""
    C = x.shape[-1]
    rows = x.numel() // C
    xc = x.contiguous()
    dyc = dy.contiguous()
    dy2c = dy2.contiguous() if dy2 is not None else None
    if dx is None:
        dx = torch.empty(x.shape, device=x.device, dtype=dx_dtype)
        accumulate = False
    L.check(L.load().comet_layernorm_bwd(dt(xc), dt(dyc), _p(xc), _p(dyc), _p(dy2c), _p(mean), _p(rstd),
                                         _p(weight), dt(dx), _p(dx), _p(dweight), _p(dbias), rows, C,
                                         int(accumulate), stream()), "layernorm_bwd")
    return dx


def layernorm_bwd_res(x, dy, dres, mean, rstd, weight=None, dweight=None, dbias=None):
    """dx (f32) = dres + LN backward of dy (x + f(LN(x)) without a separate gradient add)."""
    C = x.shape[-1]
    rows = x.numel() // C
    xc, dyc, drc = x.contiguous(), dy.contiguous(), dres.contiguous().float()
    dx = torch.empty(x.shape, device=x.device, dtype=torch.float32)
    L.check(L.load().comet_layernorm_bwd_res(dt(xc), dt(dyc), _p(xc), _p(dyc), _p(drc), _p(mean), _p(rstd),
                                             _p(weight), _p(dx), _p(dweight), _p(dbias), rows, C, stream()),
            "layernorm_bwd_res")
    return dx


# ------------------------------------------------------------------------------------------
# Attention
# ------------------------------------------------------------------------------------------
def attention(q, k, v, heads, scale=None, out=None, lse=False):
    """Multi-head attention on token-major views: q [B, Lq, H*D], k/v [B, Lk, H*D] (last dim
    unit-stride; rows may be strided, e.g. slices of a packed qkv projection). 4-D views
    [B, L, T, H*D] attend over L for every (b, t) (inner batch, no permute)."""
    _req_cuda(q, k, v)
    inner = q.dim() == 4
    if inner:
        B, Lq, T, C = q.shape
    else:
        B, Lq, C = q.shape
        T = 1
    Lk = k.shape[1]
    D = C // heads
    if q.stride(-1) != 1 or k.stride(-1) != 1 or v.stride(-1) != 1:
        raise L.CometHipError("attention: head dim must be unit-stride")
    if scale is None:
        scale = D ** -0.5
    if out is None:
        out = torch.empty(q.shape, device=q.device, dtype=q.dtype)
    lse_t = torch.empty(B * T, heads, Lq, device=q.device, dtype=torch.float32) if lse else None
    a = L.AttnArgs()
    a.dtype, a.head_dim = dt(q), D
    a.batch, a.heads, a.lq, a.lk = B * T, heads, Lq, Lk
    a.q, a.sq_b, a.sq_h, a.sq_l = _p(q), q.stride(0), D, q.stride(1)
    a.k, a.sk_b, a.sk_h, a.sk_l = _p(k), k.stride(0), D, k.stride(1)
    a.v, a.sv_b, a.sv_h, a.sv_l = _p(v), v.stride(0), D, v.stride(1)
    a.o, a.so_b, a.so_h, a.so_l = _p(out), out.stride(0), D, out.stride(1)
    if inner:
        a.batch_inner = T
        a.sq_i, a.sk_i, a.sv_i, a.so_i = q.stride(2), k.stride(2), v.stride(2), out.stride(2)
    a.lse, a.scale = _p(lse_t), float(scale)
    e0 = PROF.start()
    L.check(L.load().comet_attention_fwd(ctypes.byref(a), stream()), "attention")
    if e0 is not None:
        short = q.dtype == torch.bfloat16 and Lq <= 16 and Lk <= 16
        name = (f"attn fwd B{B} T{T} H{heads} Lq{Lq} Lk{Lk} D{D}" if PROF.detail else
                f"comet_attention_fwd|{'small' if short else 'tile'}.{'bf16' if q.dtype == torch.bfloat16 else 'f32'}.D{D}")
        PROF.stop(e0, name, 4.0 * B * T * heads * Lq * Lk * D)
    return (out, lse_t) if lse else out


def attention_bwd(q, k, v, o, lse, do, heads, scale, dq, dk, dv):
    """Fused bf16 attention backward (comet_attention_bwd). All tensors are token-major views
    [B, L, H*D] with unit-stride last dim; dq/dk/dv may be strided slices of packed buffers."""
    _req_cuda(q, k, v, o, do, dq, dk, dv, lse)
    B, Lq, C = q.shape
    Lk = k.shape[1]
    D = C // heads
    delta = torch.empty(B, heads, Lq, device=q.device, dtype=torch.float32)
    a = L.AttnBwdArgs()
    a.dtype, a.head_dim = dt(q), D
    a.batch, a.heads, a.lq, a.lk = B, heads, Lq, Lk
    for name, t in (("q", q), ("k", k), ("v", v), ("o", o), ("d", do), ("dq", dq), ("dk", dk), ("dv", dv)):
        if t.stride(2) != 1:
            raise L.CometHipError("attention_bwd: head dim must be unit-stride")
        field = "dout" if name == "d" else name
        setattr(a, field, _p(t))
        setattr(a, f"s{name}_b", t.stride(0))
        setattr(a, f"s{name}_h", D)
        setattr(a, f"s{name}_l", t.stride(1))
    a.lse, a.delta, a.scale = _p(lse), _p(delta), float(scale)
    e0 = PROF.start()
    L.check(L.load().comet_attention_bwd(ctypes.byref(a), stream()), "attention_bwd")
    if e0 is not None:
        name = f"attn bwd B{B} H{heads} Lq{Lq} Lk{Lk} D{D}" if PROF.detail else f"comet_attention_bwd|D{D}"
        PROF.stop(e0, name, 10.0 * B * heads * Lq * Lk * D)


def attention_bwd_ok(q, k, v, o, do, heads):
    D = q.shape[-1] // heads
    ts = (q, k, v, o, do)
    return (q.dtype == torch.bfloat16 and D in (32, 48, 64, 96) and all(t.dtype == torch.bfloat16 for t in ts)
            and all(t.stride(2) == 1 and t.stride(0) % 8 == 0 and t.stride(1) % 8 == 0 and t.data_ptr() % 16 == 0
                    for t in ts))


# ------------------------------------------------------------------------------------------
# Misc elementwise
# ------------------------------------------------------------------------------------------
def cast(x, dtype, out=None):
    xc = x.contiguous()
    out = out if out is not None else torch.empty(x.shape, device=x.device, dtype=dtype)
    L.check(L.load().comet_cast(dt(xc), dt(out), _p(xc), _p(out), xc.numel(), stream()), "cast")
    return out


def act_bwd(act, pre, dy, out_dtype=None):
    dyc = dy.contiguous()
    dx = torch.empty(pre.shape, device=pre.device, dtype=out_dtype or pre.dtype)
    L.check(L.load().comet_act_bwd(act, dt(pre), dt(dyc), _p(pre), _p(dyc), _p(dx), dt(dx), pre.numel(),
                                   stream()), "act_bwd")
    return dx


def act_bwd_colsum(act, pre, dy, out_dtype=None, dbias=None, accumulate=False, want_out=True):
    """One pass: g = dy * act'(pre) -> out (out_dtype) and dbias (+)= column sums of g.
    dy [rows, cols] contiguous; pre same shape (ignored for ACT_NONE)."""
    rows, cols = dy.shape
    out = torch.empty(rows, cols, device=dy.device, dtype=out_dtype or dy.dtype) if want_out else None
    pre_p = _p(pre) if act != L.ACT_NONE else None
    L.check(L.load().comet_act_bwd_colsum(act, dt(pre) if pre is not None else 0, pre_p, dt(dy), _p(dy),
                                          dt(out) if out is not None else 0, _p(out), _p(dbias), rows, cols,
                                          int(accumulate), stream()), "act_bwd_colsum")
    return out


def colsum(x2d, out=None, accumulate=False):
    rows, cols = x2d.shape
    if out is None:
        out = torch.empty(cols, device=x2d.device, dtype=torch.float32)
        accumulate = False
    L.check(L.load().comet_colsum(dt(x2d), _p(x2d), _p(out), rows, cols, x2d.stride(0), int(accumulate),
                                  stream()), "colsum")
    return out


def conv2d_nhwc(x, w, kh, kw, stride, pad, bias=None, act=L.ACT_NONE, resid=None, beta=1.0, out=None,
                out_dtype=None):
    """Implicit-GEMM conv (comet_conv2d_nhwc). x [n,h,w,c] bf16 (c % 8 == 0), w [cout, ldw] bf16 with
    columns (ky, kx, ci). Returns y [n, oh, ow, cout]."""
    _req_cuda(x, w, bias, resid)
    n, h, wd, c = x.shape
    cout = w.shape[0]
    oh = (h + 2 * pad - kh) // stride + 1
    ow = (wd + 2 * pad - kw) // stride + 1
    if not x.is_contiguous():
        x = x.contiguous()
    if out is None:
        out = torch.empty(n, oh, ow, cout, device=x.device, dtype=out_dtype or x.dtype)
    a = L.ConvArgs()
    a.dtype, a.dtype_y = dt(x), dt(out)
    a.x, a.n, a.h, a.w, a.c = _p(x), n, h, wd, c
    a.weight, a.cout, a.ldw = _p(w), cout, w.stride(0)
    a.kh, a.kw, a.stride, a.pad = kh, kw, stride, pad
    a.bias = _p(bias)
    a.y, a.ldy = _p(out), cout
    a.resid, a.ldr, a.beta = _p(resid), (cout if resid is not None else 0), beta
    a.act = act
    e0 = PROF.start()
    L.check(L.load().comet_conv2d_nhwc(ctypes.byref(a), stream()), "comet_conv2d_nhwc")
    if e0 is not None:
        name = f"conv {kh}x{kw}s{stride} c{c}->{cout} {h}x{wd} n{n}" if PROF.detail else "comet_conv2d_nhwc"
        PROF.stop(e0, name, 2.0 * n * oh * ow * cout * kh * kw * c)
    return out


def im2col_nhwc(x, kh, kw, stride, pad, out_dtype=None, ldc=None):
    n, h, w, c = x.shape
    oh = (h + 2 * pad - kh) // stride + 1
    ow = (w + 2 * pad - kw) // stride + 1
    kk = kh * kw * c
    ldc = ldc or kk
    cols = torch.empty(n * oh * ow, ldc, device=x.device, dtype=out_dtype or x.dtype)
    L.check(L.load().comet_im2col_nhwc(dt(x), dt(cols), _p(x), _p(cols), n, h, w, c, kh, kw, stride, pad,
                                       oh, ow, ldc, stream()), "im2col")
    return cols, oh, ow


def instnorm_nhwc(x, res=None, relu=False, eps=1e-5, out=None, relu_inner=False):
    n, h, w, c = x.shape
    out = out if out is not None else torch.empty_like(x)
    lib = L.load()
    nb = ctypes.c_int64(0)
    L.check(lib.comet_instnorm_workspace(n, h * w, c, ctypes.byref(nb)), "instnorm_workspace")
    ws = torch.empty((nb.value + 3) // 4, device=x.device, dtype=torch.float32) if nb.value else None
    L.check(lib.comet_instnorm_nhwc(dt(x), _p(x), _p(res), _p(out), n, h * w, c, float(eps),
                                    int(relu), int(relu_inner), _p(ws), nb.value, stream()), "instnorm")
    return out


def resize_bilinear(x, oh, ow, nhwc, out=None, add=False, out_dtype=None):
    if nhwc:
        n, h, w, c = x.shape
        shape = (n, oh, ow, c)
    else:
        n, c, h, w = x.shape
        shape = (n, c, oh, ow)
    xc = x.contiguous()
    if out is None:
        out = torch.empty(shape, device=x.device, dtype=out_dtype or x.dtype)
        add = False
    L.check(L.load().comet_resize_bilinear(dt(xc), dt(out), int(nhwc), _p(xc), _p(out), n, c, h, w, oh, ow,
                                           int(add), stream()), "resize_bilinear")
    return out


def cast_multi_f32_bf16(srcs, dsts):
    """dst[i].copy_(src[i]) f32 -> bf16 (contiguous, equal numel) in few launches."""
    n = len(srcs)
    S = (ctypes.c_void_p * n)(*[t.data_ptr() for t in srcs])
    D = (ctypes.c_void_p * n)(*[t.data_ptr() for t in dsts])
    Z = (ctypes.c_int64 * n)(*[t.numel() for t in srcs])
    L.check(L.load().comet_cast_multi_f32_bf16(S, D, Z, n, stream()), "cast_multi")


def resize_bilinear_pool(x, oh, ow):
    """NHWC x [n, h, w, c] -> (y [n, oh, ow, c] bilinear, align_corners=True; its 2 x 2 average
    pool [n, oh // 2, ow // 2, c]) in one kernel: resize_bilinear + avgpool2_nhwc bit for bit."""
    n, h, w, c = x.shape
    xc = x.contiguous()
    y = torch.empty(n, oh, ow, c, device=x.device, dtype=x.dtype)
    p = torch.empty(n, oh // 2, ow // 2, c, device=x.device, dtype=x.dtype)
    L.check(L.load().comet_resize_bilinear_pool_nhwc(dt(xc), dt(y), _p(xc), _p(y), _p(p), n, c, h, w, oh, ow,
                                                     stream()), "resize_bilinear_pool")
    return y, p


def conv1x1_resize_pool(x, w, b, oh, ow, up1=None, up2=None, pool2=False):
    """NHWC bf16 x [n, h, w, c]: x2 = (x + up(up1)) + up(up2) (optional, each rounded to bf16 as
    resize_bilinear(..., out=x, add=True)), t = x2 + x2 W^T + b (W [c, c] bf16, b f32), y = resize(t)
    to [n, oh, ow, c], pool = avgpool2(y) (and with pool2: avgpool2(pool)), in one kernel -- the
    unfused calls bit for bit, without x2 or t in HBM (the fine ShallowEncoder's tail, blocks.py:97-110,
    and the fine correlation pyramid's levels 1-2)."""
    n, h, ww, c = x.shape
    y = torch.empty(n, oh, ow, c, device=x.device, dtype=x.dtype)
    p = torch.empty(n, oh // 2, ow // 2, c, device=x.device, dtype=x.dtype)
    q = torch.empty(n, oh // 4, ow // 4, c, device=x.device, dtype=x.dtype) if pool2 else None
    h1, w1 = (up1.shape[1], up1.shape[2]) if up1 is not None else (0, 0)
    h2, w2 = (up2.shape[1], up2.shape[2]) if up2 is not None else (0, 0)
    L.check(L.load().comet_conv1x1_resize_pool_nhwc(_p(x), _p(up1), h1, w1, _p(up2), h2, w2, _p(w), _p(b), _p(y),
                                                    _p(p), _p(q), n, c, h, ww, oh, ow, stream()), "conv1x1_resize_pool")
    return (y, p, q) if pool2 else (y, p)


def conv1x1_resize_pool_ok(x, w, b, *ups):
    n, h, ww, c = x.shape
    ok = (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and c in (32, 64) and x.is_contiguous()
          and w.is_contiguous() and tuple(w.shape) == (c, c) and (h * ww) % 16 == 0 and 4 * h * ww * c <= 49152
          and x.data_ptr() % 16 == 0 and w.data_ptr() % 16 == 0
          and (b is None or (b.dtype == torch.float32 and b.is_contiguous())))
    for u in ups:
        ok = ok and (u.dtype == torch.bfloat16 and u.is_contiguous() and u.shape[0] == n and u.shape[3] == c
                     and u.data_ptr() % 16 == 0)
    return ok


def resize_pool_ok(x):
    """comet_resize_bilinear_pool_nhwc's conditions (c % 8, 16-B alignment, input image <= 32 KiB)."""
    n, h, w, c = x.shape
    return (x.is_contiguous() and c in (8, 16, 32, 64, 128, 256) and x.data_ptr() % 16 == 0
            and h * w * c * x.element_size() <= 32768)


def resize_bilinear_into(x, out, add=False):
    """NHWC x [n, h, w, c] resized into out [n, oh, ow, c], a channel slice of a wider NHWC tensor
    (out.stride() == (oh*ow*ld, ow*ld, ld, 1))."""
    n, h, w, c = x.shape
    on, oh, ow, oc = out.shape
    ld = out.stride(2)
    assert on == n and oc == c and out.stride(3) == 1 and out.stride(1) == ow * ld and out.stride(0) == oh * ow * ld
    xc = x.contiguous()
    L.check(L.load().comet_resize_bilinear_nhwc_into(dt(xc), dt(out), _p(xc), _p(out), n, c, h, w, oh, ow, ld,
                                                     int(add), stream()), "resize_bilinear_into")
    return out


# ------------------------------------------------------------------------------------------
# camera head helpers
# ------------------------------------------------------------------------------------------
def _chk(rc, what):
    L.check(rc, what)


def act_fwd(act, x, out_dtype=None):
    xc = x.contiguous()
    y = torch.empty(x.shape, device=x.device, dtype=out_dtype or x.dtype)
    _chk(L.load().comet_act_fwd(act, dt(xc), dt(y), _p(xc), _p(y), xc.numel(), stream()), "act_fwd")
    return y


def binary(op, a, b, out=None):
    a = a.contiguous()
    b = b.contiguous()
    out = out if out is not None else torch.empty_like(a)
    _chk(L.load().comet_binary(op, dt(a), _p(a), _p(b), _p(out), a.numel(), stream()), "binary")
    return out


def add_relu(a, b):
    return binary(1, a, b)


def add(a, b, out=None):
    return binary(0, a, b, out)


def add_rows(x, table, period, out_dtype=None, out=None):
    """x [..., C] (+ table[(row % period), :]); table f32 [period, C]."""
    C = x.shape[-1]
    r = _rows2d(x)
    xc = x
    if r is None:
        xc = x.contiguous()
        r = _rows2d(xc)
    rows, ldx = r
    y = out if out is not None else torch.empty(x.shape, device=x.device, dtype=out_dtype or x.dtype)
    ry = _rows2d(y)
    _chk(L.load().comet_add_rows(dt(xc), dt(y), _p(xc), _p(table), _p(y), rows, C, period, ldx, ry[1], stream()),
         "add_rows")
    return y


def rowscale(x, w):
    xc = x.contiguous()
    C = x.shape[-1]
    y = torch.empty_like(xc)
    _chk(L.load().comet_rowscale_fwd(dt(xc), _p(xc), _p(w), _p(y), xc.numel() // C, C, stream()), "rowscale")
    return y


def rowscale_bwd(x, w, dy, need_dx=True, need_dw=True):
    xc = x.contiguous()
    C = x.shape[-1]
    rows = xc.numel() // C
    dyc = dy.contiguous().float() if dy.dtype != torch.float32 else dy.contiguous()
    dx = torch.empty(x.shape, device=x.device, dtype=torch.float32) if need_dx else None
    dw = torch.empty(w.shape, device=x.device, dtype=torch.float32) if need_dw else None
    _chk(L.load().comet_rowscale_bwd(dt(xc), _p(xc), _p(w), _p(dyc), _p(dx), _p(dw), rows, C, stream()),
         "rowscale_bwd")
    return dx, dw


def sincos_table(pos, dim, out=None, col0=0):
    """get_1d_sincos_pos_embed_from_grid(dim, pos) on device -> [len(pos), dim] f32."""
    pos = pos.contiguous().float()
    m = pos.numel()
    if out is None:
        out = torch.empty(m, dim, device=pos.device, dtype=torch.float32)
    _chk(L.load().comet_sincos_table(_p(pos), _p(out), m, dim, out.stride(0), col0, stream()), "sincos")
    return out


def sincos_2d(embed_dim, gh, gw, device):
    """get_2d_sincos_pos_embed(embed_dim, (gh, gw)) as a [gh*gw, embed_dim] row table (row =
    y*gw + x; first half encodes x (column), second half y (row): utils.py:724-804)."""
    xs = torch.arange(gw, device=device, dtype=torch.float32).repeat(gh)
    ys = torch.arange(gh, device=device, dtype=torch.float32).repeat_interleave(gw)
    out = torch.empty(gh * gw, embed_dim, device=device, dtype=torch.float32)
    sincos_table(xs, embed_dim // 2, out=out, col0=0)
    sincos_table(ys, embed_dim // 2, out=out, col0=embed_dim // 2)
    return out


def _ratio_args(ratio):
    """(host value, device pointer or None): a ratio already in HBM (float64 tensor) is read by the
    kernel, a host float / CPU tensor (the DataLoader's collated float64) is passed by value --
    neither path synchronises the device."""
    if torch.is_tensor(ratio):
        if ratio.is_cuda:
            r = ratio.reshape(-1)[:1].to(torch.float64).contiguous()
            return 0.0, r, _p(r)
        return float(ratio.reshape(-1)[0]), None, None
    return float(ratio), None, None


def pose_encode(R, T_uvz, focal, ratio, B, S):
    enc = torch.empty(B * S, 8, device=R.device, dtype=torch.float32)
    rh, keep, rd = _ratio_args(ratio)
    _chk(L.load().comet_pose_encode(_p(R.contiguous()), _p(T_uvz.contiguous()), _p(focal.contiguous()),
                                    rh, rd, _p(enc), B, S, stream()), "pose_encode")
    return enc


def pose_decode(enc, R_gt, T_gt, ratio, intr, B, S):
    Rout = torch.empty(B * S, 4, device=enc.device, dtype=torch.float32)
    Tout = torch.empty(B * S, 3, device=enc.device, dtype=torch.float64)
    fx, fy, cx, cy = intr
    rh, keep, rd = _ratio_args(ratio)
    _chk(L.load().comet_pose_decode(_p(enc.contiguous()), _p(R_gt.contiguous()), _p(T_gt.contiguous()), rh, rd,
                                    fx, fy, cx, cy, _p(Rout), _p(Tout), B, S, stream()), "pose_decode")
    return Rout, Tout


def pose_encode3(R, T, B, S):
    """camera_to_pose_encoding3 per sequence -> [B*S, 8] (column 7 zero padding)."""
    enc = torch.empty(B * S, 8, device=R.device, dtype=torch.float32)
    _chk(L.load().comet_pose_encode3(_p(R.contiguous()), _p(T.contiguous()), _p(enc), B, S, stream()), "pose_encode3")
    return enc


def pose_decode3(enc, R_gt, T_gt, B, S):
    """pose_encoding_to_camera3 per sequence -> (R [B*S, 4], T [B*S, 3]) f32."""
    Rout = torch.empty(B * S, 4, device=enc.device, dtype=torch.float32)
    Tout = torch.empty(B * S, 3, device=enc.device, dtype=torch.float32)
    _chk(L.load().comet_pose_decode3(_p(enc.contiguous()), _p(R_gt.contiguous()), _p(T_gt.contiguous()), _p(Rout),
                                     _p(Tout), B, S, stream()), "pose_decode3")
    return Rout, Tout


# ------------------------------------------------------------------------------------------
# tracker
# ------------------------------------------------------------------------------------------
def sample_bilinear(fmap_nhwc, coords, border=True, out=None):
    """fmap [B, H, W, C], coords [B, R, 2] (pixel x, y) -> [B, R, C] f32."""
    B, H, W, C = fmap_nhwc.shape
    R = coords.shape[1]
    cc = coords.contiguous().float()
    if out is None:
        out = torch.empty(B, R, C, device=coords.device, dtype=torch.float32)
    _chk(L.load().comet_sample_bilinear(dt(fmap_nhwc), _p(fmap_nhwc), fmap_nhwc.stride(0), H, W, C, _p(cc),
                                        cc.stride(0), cc.stride(1), _p(out), out.stride(0), out.stride(1), B, R,
                                        int(border), stream()), "sample_bilinear")
    return out


def corr_sample(pyramid, radius, feats, coords, out, col0, B, N, S):
    C = pyramid[0].shape[-1]
    levels = len(pyramid)
    ptrs = (ctypes.c_void_p * levels)(*[p.data_ptr() for p in pyramid])
    hs = (ctypes.c_int * levels)(*[p.shape[1] for p in pyramid])
    ws = (ctypes.c_int * levels)(*[p.shape[2] for p in pyramid])
    _chk(L.load().comet_corr_sample(dt(pyramid[0]), dt(feats), ptrs, hs, ws, levels, radius, C, _p(feats), _p(coords),
                                    _p(out), out.stride(0), col0, B, N, S, stream()), "corr_sample")


def tracker_tokens(coords, feats, latent, corr, corrdim, pos, tdim, x, rows, S):
    """x [rows, ldx] (ldx = x.stride(0) >= tdim): the update former's input tokens; columns tdim.. are
    zero padding (the input GEMM's K rounded up to its k-tile)."""
    _chk(L.load().comet_tracker_tokens(dt(x), _p(coords), _p(feats), latent, _p(corr), corr.stride(0), corrdim,
                                       _p(pos), tdim, _p(x), x.stride(0), rows, S, stream()), "tracker_tokens")


def coords_update(coords, delta, preds, scale, B, N, S):
    _chk(L.load().comet_coords_update(dt(delta), _p(coords), _p(delta), delta.stride(0), _p(preds), float(scale),
                                      B, N, S, stream()), "coords_update")


def avgpool2_nhwc(x):
    n, H, W, C = x.shape
    y = torch.empty(n, H // 2, W // 2, C, device=x.device, dtype=x.dtype)
    _chk(L.load().comet_avgpool2_nhwc(dt(x), _p(x), _p(y), n, H, W, C, stream()), "avgpool2")
    return y


def patch_gather(images, coarse, pradius, out_dtype, cpad=3):
    B, S, _, H, W = images.shape
    N = coarse.shape[2]
    P = 2 * pradius + 1
    patches = torch.empty(B * S * N, P, P, cpad, device=images.device, dtype=out_dtype)
    topleft = torch.empty(B, S, N, 2, device=images.device, dtype=torch.int32)
    query = torch.empty(B * N, 2, device=images.device, dtype=torch.float32)
    _chk(L.load().comet_patch_gather(dt(patches), _p(images.contiguous()), _p(coarse.contiguous()), _p(patches),
                                     _p(topleft), _p(query), B, S, N, H, W, pradius, cpad, stream()), "patch_gather")
    return patches, topleft, query


def images_nhwc(images, oh, ow, out_dtype, cpad=3):
    """[n, 3, H, W] f32 -> [n, oh, ow, cpad] (align_corners resize when the size changes)."""
    n, _, H, W = images.shape
    out = torch.empty(n, oh, ow, cpad, device=images.device, dtype=out_dtype)
    _chk(L.load().comet_images_nhwc(dt(out), _p(images.contiguous()), _p(out), n, H, W, oh, ow, cpad, stream()),
         "images_nhwc")
    return out


def refine_combine(fine, topleft, coarse, B, S, N):
    refined = torch.empty(B, S, N, 2, device=fine.device, dtype=torch.float32)
    _chk(L.load().comet_refine_combine(_p(fine), _p(topleft), _p(coarse.contiguous()), _p(refined), B, S, N, stream()),
         "refine_combine")
    return refined


def track_score(qfeat, pfeat, fine, B, S, N, sradius=2):
    P, C = pfeat.shape[-2], pfeat.shape[-1]
    score = torch.empty(B, S, N, device=qfeat.device, dtype=torch.float32)
    inv = torch.empty(B, S, N, device=qfeat.device, dtype=torch.float32)
    _chk(L.load().comet_track_score(dt(pfeat), _p(qfeat.contiguous()), _p(pfeat), _p(fine.contiguous()), _p(score),
                                    _p(inv), B, S, N, P, C, sradius, stream()), "track_score")
    return score, inv


def dino_prep(images_flat, R, patch, ldc, mean3, std3, out_dtype):
    BS, _, H, W = images_flat.shape
    g = R // patch
    cols = torch.empty(BS * g * g, ldc, device=images_flat.device, dtype=out_dtype)
    _chk(L.load().comet_dino_prep(dt(cols), _p(images_flat.contiguous()), _p(cols), BS, H, W, R, patch, ldc,
                                  _p(mean3), _p(std3), stream()), "dino_prep")
    return cols


def harmonic_fwd(x, freqs, append_input, diag_cov=None):
    dim = x.shape[-1]
    n = freqs.numel()
    rows = x.numel() // dim
    xc = x.contiguous().float()
    cov = diag_cov.contiguous().float() if diag_cov is not None else None
    y = torch.empty(*x.shape[:-1], dim * (2 * n + int(append_input)), device=x.device, dtype=torch.float32)
    _chk(L.load().comet_harmonic_fwd(_p(xc), _p(cov), _p(freqs), _p(y), rows, dim, n, int(append_input), stream()),
         "harmonic_fwd")
    return y


def harmonic_bwd(x, freqs, append_input, dy, diag_cov=None):
    dim = x.shape[-1]
    n = freqs.numel()
    rows = x.numel() // dim
    xc = x.contiguous().float()
    cov = diag_cov.contiguous().float() if diag_cov is not None else None
    dyc = dy.contiguous().float()
    dx = torch.empty(x.shape, device=x.device, dtype=torch.float32)
    dcov = torch.empty(x.shape, device=x.device, dtype=torch.float32) if cov is not None else None
    _chk(L.load().comet_harmonic_bwd(_p(xc), _p(cov), _p(freqs), _p(dyc), _p(dx), _p(dcov), rows, dim, n,
                                     int(append_input), stream()), "harmonic_bwd")
    return dx, dcov


# ------------------------------------------------------------------------------------------
# Live timing of the memory-bound ops (bench.py's profiled pass, PROF.enabled): every op below is
# bracketed with HIP events on the launching stream and keyed "comet_<op>" with its ALGORITHMIC
# bytes -- every tensor argument read or written once plus every tensor it returns (an output
# passed in and returned counts once; the gather ops count the taps they read, _gather_bytes) --
# so the bench line carries a TB/s figure per memory-bound
# op. With PROF.detail (tools/gemm_shapes.py) the key is the op, its tensor shapes and the calling
# model line instead. Ops called from inside another bracketed op are not bracketed again.
# ------------------------------------------------------------------------------------------
_TIMED_DEPTH = [0]


def _tensor_bytes(objs, seen):
    n = 0
    for a in objs:
        if isinstance(a, torch.Tensor):
            if id(a) not in seen:
                seen.add(id(a))
                n += a.numel() * a.element_size()
        elif isinstance(a, (list, tuple)):
            n += _tensor_bytes(a, seen)
    return n


def _gather_bytes(name, args, out):
    """Algorithmic bytes of the gather ops, which read a small part of a large map (the generic
    rule would count the whole map): the taps actually read + the indices + the output."""
    nb = lambda t: t.numel() * t.element_size()  # noqa: E731
    if name == "sample_bilinear":   # 4 bilinear corners per output value
        fmap, coords = args[0], args[1]
        return 4 * out.numel() * fmap.element_size() + nb(coords) + nb(out)
    if name == "track_score":       # (2r+1)^2 window of each track's patch feature map
        qfeat, pfeat, fine = args[0], args[1], args[2]
        r = args[6] if len(args) > 6 else 2
        C = pfeat.shape[-1]
        tracks = out[0].numel()
        return nb(qfeat) + tracks * (2 * r + 1) ** 2 * C * pfeat.element_size() + nb(fine) + nb(out[0]) + nb(out[1])
    if name == "corr_sample":       # each track's (2r+4)^2 pixel grid per level, at most every pixel once
        pyramid, radius, feats, coords, o = args[0], args[1], args[2], args[3], args[4]
        gs = 2 * radius + 4
        tracks = coords.shape[0]
        n = nb(feats) + nb(coords) + o.shape[0] * len(pyramid) * (2 * radius + 1) ** 2 * o.element_size()
        for lv in pyramid:
            fr, H, W, C = lv.shape
            n += min(tracks * min(gs, H) * min(gs, W), fr * H * W) * C * lv.element_size()
        return n
    if name == "patch_gather":      # the gathered patches are read once and written once
        patches = out[0]
        return 2 * nb(patches) + nb(args[1]) + nb(out[1]) + nb(out[2])
    return None


def _timed(fn):
    import functools
    import os
    import sys

    @functools.wraps(fn)
    def wrap(*args, **kwargs):
        if not PROF.enabled or _TIMED_DEPTH[0] > 0:
            return fn(*args, **kwargs)
        if PROF.detail:
            f = sys._getframe(1)
            while f is not None and f.f_code.co_filename.endswith("ops.py"):
                f = f.f_back
            sites = []
            while f is not None and len(sites) < 2:
                sites.append(f"{os.path.basename(f.f_code.co_filename)}:{f.f_lineno}")
                f = f.f_back
            site = "<".join(sites) or "?"
            shapes = ",".join("x".join(map(str, a.shape)) + str(a.dtype)[6:] for a in args if isinstance(a, torch.Tensor))
            name = f"{fn.__name__} [{shapes}] @{site}"
        else:
            name = "comet_" + fn.__name__
        e0 = PROF.start()
        _TIMED_DEPTH[0] += 1
        try:
            out = fn(*args, **kwargs)
        finally:
            _TIMED_DEPTH[0] -= 1
        nb = _gather_bytes(fn.__name__, args, out)
        if nb is None:
            seen = set()
            nb = _tensor_bytes(args, seen) + _tensor_bytes(kwargs.values(), seen)
            nb += _tensor_bytes(out if isinstance(out, (list, tuple)) else (out,), seen)
        PROF.stop(e0, name, 0.0, float(nb))
        return out
    return wrap


for _name in ("layernorm", "layernorm_bwd", "layernorm_bwd_res", "cast", "cast_multi_f32_bf16", "act_bwd", "colsum",
              "act_bwd_colsum", "instnorm_nhwc", "resize_bilinear", "resize_bilinear_into", "resize_bilinear_pool", "conv1x1_resize_pool", "im2col_nhwc", "act_fwd",
              "binary", "add_rows", "rowscale", "rowscale_bwd", "sample_bilinear", "corr_sample", "tracker_tokens",
              "coords_update", "avgpool2_nhwc", "patch_gather", "refine_combine", "track_score", "dino_prep",
              "pose_encode", "pose_decode", "pose_encode3", "pose_decode3", "images_nhwc", "harmonic_fwd",
              "harmonic_bwd", "sincos_table"):
    globals()[_name] = _timed(globals()[_name])
