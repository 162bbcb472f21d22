"""Tensor-level wrappers over the C-ABI (raw kernels, no autograd).

Every function enqueues on torch's current HIP stream and returns device tensors. No op here
has a CPU/PyTorch fallback: a missing library or an unsupported shape raises.
"""
import ctypes

import torch

from . import _lib as L

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
             ldaux=0, stride_aux=(0, 0), alpha=1.0, act=L.ACT_NONE):
    _req_cuda(a, b, c, bias, resid, aux)
    if a.dtype != b.dtype:
        raise L.CometHipError("gemm: A and B must share a dtype")
    if bias is not None and bias.dtype != torch.float32:
        raise L.CometHipError("gemm: bias must be f32")
    for t in (resid, aux):
        if t is not None and t.dtype != c.dtype:
            raise L.CometHipError("gemm: resid/aux must have the output dtype")
    g = L.GemmArgs()
    g.dtype_ab, g.dtype_c, g.layout_a, g.layout_b = dt(a), dt(c), layout_a, layout_b
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
    L.check(L.load().comet_gemm(ctypes.byref(g), stream()), "comet_gemm")
    return c


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


# ------------------------------------------------------------------------------------------
# LayerNorm
# ------------------------------------------------------------------------------------------
def layernorm(x, weight=None, bias=None, eps=1e-5, out_dtype=None, stats=False, out=None):
    _req_cuda(x)
    C = x.shape[-1]
    xc = x if x.is_contiguous() else x.contiguous()
    rows = xc.numel() // C
    y = out if out is not None else torch.empty(x.shape, device=x.device, dtype=out_dtype or x.dtype)
    mean = rstd = None
    if stats:
        mean = torch.empty(rows, device=x.device, dtype=torch.float32)
        rstd = torch.empty(rows, device=x.device, dtype=torch.float32)
    L.check(L.load().comet_layernorm_fwd(dt(xc), dt(y), _p(xc), _p(weight), _p(bias), _p(y), _p(mean),
                                         _p(rstd), rows, C, float(eps), stream()), "layernorm")
    if stats:
        return y, mean, rstd
    return y


def layernorm_bwd(x, dy, mean, rstd, weight=None, dweight=None, dbias=None, dx=None, accumulate=False):
    C = x.shape[-1]
    rows = x.numel() // C
    xc = x.contiguous()
    dyc = dy.contiguous()
    if dx is None:
        dx = torch.empty(x.shape, device=x.device, dtype=torch.float32)
        accumulate = False
    L.check(L.load().comet_layernorm_bwd(dt(xc), dt(dyc), _p(xc), _p(dyc), _p(mean), _p(rstd), _p(weight),
                                         _p(dx), _p(dweight), _p(dbias), rows, C, int(accumulate),
                                         stream()), "layernorm_bwd")
    return dx


# ------------------------------------------------------------------------------------------
# Attention
# ------------------------------------------------------------------------------------------
def attention(q, k, v, heads, scale=None, out=None, lse=False):
    """Multi-head attention on token-major views: q [B, Lq, H*D], k/v [B, Lk, H*D] (last dim
    unit-stride; rows may be strided, e.g. slices of a packed qkv projection)."""
    _req_cuda(q, k, v)
    B, Lq, C = q.shape
    Lk = k.shape[1]
    D = C // heads
    if q.stride(2) != 1 or k.stride(2) != 1 or v.stride(2) != 1:
        raise L.CometHipError("attention: head dim must be unit-stride")
    if scale is None:
        scale = D ** -0.5
    if out is None:
        out = torch.empty(B, Lq, C, device=q.device, dtype=q.dtype)
    lse_t = torch.empty(B, heads, Lq, device=q.device, dtype=torch.float32) if lse else None
    a = L.AttnArgs()
    a.dtype, a.head_dim = dt(q), D
    a.batch, a.heads, a.lq, a.lk = B, heads, Lq, Lk
    a.q, a.sq_b, a.sq_h, a.sq_l = _p(q), q.stride(0), D, q.stride(1)
    a.k, a.sk_b, a.sk_h, a.sk_l = _p(k), k.stride(0), D, k.stride(1)
    a.v, a.sv_b, a.sv_h, a.sv_l = _p(v), v.stride(0), D, v.stride(1)
    a.o, a.so_b, a.so_h, a.so_l = _p(out), out.stride(0), D, out.stride(1)
    a.lse, a.scale = _p(lse_t), float(scale)
    L.check(L.load().comet_attention_fwd(ctypes.byref(a), stream()), "attention")
    return (out, lse_t) if lse else out


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


def colsum(x2d, out=None, accumulate=False):
    rows, cols = x2d.shape
    if out is None:
        out = torch.empty(cols, device=x2d.device, dtype=torch.float32)
        accumulate = False
    L.check(L.load().comet_colsum(dt(x2d), _p(x2d), _p(out), rows, cols, x2d.stride(0), int(accumulate),
                                  stream()), "colsum")
    return out


def im2col_nhwc(x, kh, kw, stride, pad, out_dtype=None, ldc=None):
    n, h, w, c = x.shape
    oh = (h + 2 * pad - kh) // stride + 1
    ow = (w + 2 * pad - kw) // stride + 1
    kk = kh * kw * c
    ldc = ldc or kk
    cols = torch.empty(n * oh * ow, ldc, device=x.device, dtype=out_dtype or x.dtype)
    if ldc != kk:
        cols[:, kk:].zero_()
    L.check(L.load().comet_im2col_nhwc(dt(x), dt(cols), _p(x), _p(cols), n, h, w, c, kh, kw, stride, pad,
                                       oh, ow, ldc, stream()), "im2col")
    return cols, oh, ow


def instnorm_nhwc(x, res=None, relu=False, eps=1e-5, out=None):
    n, h, w, c = x.shape
    out = out if out is not None else torch.empty_like(x)
    L.check(L.load().comet_instnorm_nhwc(dt(x), _p(x), _p(res), _p(out), n, h * w, c, float(eps),
                                         int(relu), 0, stream()), "instnorm")
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
