"""Kernel-level parity: every libcomet_hip.so op against a plain PyTorch fp32/fp64 CPU
reference of the same op (seeded random inputs, shapes covering tails and all layouts)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _ops():
    from comet_amd import ops
    return ops


def _rand(*shape, dtype=torch.float32, scale=1.0, seed=0):
    g = torch.Generator().manual_seed(seed)
    return (torch.randn(*shape, generator=g) * scale).to(dtype)


def _close(got, ref, rtol, atol, what=""):
    got = got.detach().float().cpu()
    ref = ref.detach().float().cpu()
    err = (got - ref).abs()
    tol = atol + rtol * ref.abs()
    bad = (err > tol)
    assert not bad.any(), f"{what}: max err {err.max().item():.3e} (ref max {ref.abs().max().item():.3e}), {bad.sum().item()} bad"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("mnk", [(128, 128, 64), (200, 130, 664), (1, 4, 768), (77, 3, 2), (300, 520, 96)])
def test_gemm_layouts(dtype, la, lb, mnk):
    ops = _ops()
    M, N, K = mnk
    A = _rand(M, K, dtype=dtype, seed=1)
    B = _rand(N, K, dtype=dtype, seed=2)
    ref = A.double() @ B.double().t()
    Ad = (A if la == 0 else A.t().contiguous()).to(DEV)
    Bd = (B if lb == 0 else B.t().contiguous()).to(DEV)
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    ops.gemm_raw(Ad, Bd, C, m=M, n=N, k=K, layout_a=la, lda=(K if la == 0 else M),
                 layout_b=lb, ldb=(K if lb == 0 else N), ldc=N)
    tol = 2e-5 if dtype == torch.float32 else 1e-3
    _close(C, ref, tol, tol * math.sqrt(K), f"gemm {dtype} la={la} lb={lb} {mnk}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("mnk,split", [((128, 128, 8192), 0), ((200, 136, 5000), 0), ((130, 77, 4099), 0),
                                       ((96, 40, 3001), 7), ((256, 384, 2048), 3)])
def test_gemm_splitk(dtype, la, lb, mnk, split):
    """Split-K path (weight-gradient shapes: few output tiles, long K), auto and forced splits,
    vectorised and scalar (misaligned) loaders; partial sums reduced in a fixed order."""
    ops = _ops()
    M, N, K = mnk
    A = _rand(M, K, dtype=dtype, seed=11)
    B = _rand(N, K, dtype=dtype, seed=12)
    ref = A.double() @ B.double().t()
    Ad = (A if la == 0 else A.t().contiguous()).to(DEV)
    Bd = (B if lb == 0 else B.t().contiguous()).to(DEV)
    outs = []
    for _ in range(2):
        C = torch.empty(M, N, device=DEV, dtype=torch.float32)
        ops.gemm_raw(Ad, Bd, C, m=M, n=N, k=K, layout_a=la, lda=(K if la == 0 else M),
                     layout_b=lb, ldb=(K if lb == 0 else N), ldc=N, split_k=split)
        outs.append(C)
    tol = 2e-5 if dtype == torch.float32 else 1e-3
    _close(outs[0], ref, tol, tol * math.sqrt(K), f"splitk gemm {dtype} la={la} lb={lb} {mnk} split={split}")
    assert torch.equal(outs[0], outs[1]), "split-K result not deterministic"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_splitk_epilogue_batched(dtype):
    ops = _ops()
    nb0, nb1, M, N, K = 2, 3, 72, 136, 1536
    A = _rand(nb0, nb1, K, M, dtype=dtype, seed=13)           # layout 1 (dW-like: A[k*lda + m])
    B = _rand(nb0, nb1, K, N, dtype=dtype, seed=14)           # layout 1
    bias = _rand(nb0, nb1, M, seed=15)                        # per-row bias
    r = _rand(nb0, nb1, M, N, seed=16)
    pre = torch.einsum("abkm,abkn->abmn", A.double(), B.double()) * 0.5 + bias.double()[..., None]
    ref = F.relu(pre) + 2.0 * r.double()
    out = torch.empty(nb0, nb1, M, N, device=DEV, dtype=torch.float32)
    aux = torch.empty_like(out)
    Ad, Bd = A.to(DEV), B.to(DEV)
    ops.gemm_raw(Ad, Bd, out, m=M, n=N, k=K, layout_a=1, lda=M, layout_b=1, ldb=N, ldc=N, batch=(nb0, nb1),
                 stride_a=(nb1 * K * M, K * M), stride_b=(nb1 * K * N, K * N), stride_c=(nb1 * M * N, M * N),
                 bias=bias.to(DEV), bias_mode=2, stride_bias=(nb1 * M, M), resid=r.to(DEV), ldr=N,
                 stride_r=(nb1 * M * N, M * N), beta=2.0, aux=aux, ldaux=N, stride_aux=(nb1 * M * N, M * N),
                 alpha=0.5, act=2, split_k=4)
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    _close(out, ref, tol, 1e-3 * math.sqrt(K) / 10, "split epilogue out")
    _close(aux, pre, tol, 1e-3 * math.sqrt(K) / 10, "split epilogue aux")


@pytest.mark.parametrize("geo", [(3, 17, 13, 16, 40, 3, 1, 1), (2, 33, 30, 64, 96, 3, 2, 1), (2, 16, 16, 32, 32, 1, 2, 0),
                                 (1, 12, 12, 416, 256, 3, 1, 1), (2, 20, 18, 8, 64, 7, 2, 3), (65, 9, 9, 32, 32, 3, 2, 1),
                                 # narrow-output path (M >= 16384, cout <= 64)
                                 (200, 16, 16, 32, 32, 3, 1, 1), (100, 31, 31, 8, 32, 3, 2, 1), (64, 20, 20, 16, 64, 3, 1, 1),
                                 (300, 16, 16, 32, 32, 1, 2, 0), (70, 30, 30, 8, 48, 3, 1, 1),
                                 # 128 x 64 (N <= 64) tile: the BasicEncoder's 64 -> 64 convolutions
                                 (4, 40, 40, 64, 64, 3, 1, 1), (3, 21, 19, 64, 56, 3, 1, 1),
                                 # rows-in-LDS 3x3 kernel (c = cout = 64, w % 32 == 0, n*h >= 256): row
                                 # ranges of 2 rows cross image boundaries; w = 128 (the encoder's)
                                 (3, 100, 96, 64, 64, 3, 1, 1), (2, 130, 128, 64, 64, 3, 1, 1),
                                 (1, 300, 32, 64, 64, 3, 1, 1)])
@pytest.mark.parametrize("epi", ["bias", "bias_relu_resid"])
def test_conv2d_nhwc_implicit_gemm(geo, epi):
    """comet_conv2d_nhwc (implicit GEMM, bf16) vs torch conv2d in f64 on the same bf16 inputs."""
    ops = _ops()
    n, h, w, c, cout, k, s, p = geo
    x = _rand(n, c, h, w, seed=20).to(torch.bfloat16)
    wt = _rand(cout, c, k, k, seed=21, scale=1.0 / math.sqrt(c * k * k)).to(torch.bfloat16)
    b = _rand(cout, seed=22)
    ref = F.conv2d(x.double(), wt.double(), b.double(), stride=s, padding=p).permute(0, 2, 3, 1)
    K = c * k * k
    Kp = (K + 7) // 8 * 8
    wm = torch.zeros(cout, Kp, dtype=torch.bfloat16)
    wm[:, :K] = wt.permute(0, 2, 3, 1).reshape(cout, K)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    kw = dict(bias=b.to(DEV), out_dtype=torch.float32)
    if epi == "bias_relu_resid":
        r = _rand(*ref.shape, seed=23)
        ref = F.relu(ref) + 0.5 * r.double()
        kw.update(act=2, resid=r.to(DEV), beta=0.5)
    y = ops.conv2d_nhwc(xd, wm.to(DEV), k, k, s, p, **kw)
    _close(y, ref, 1e-3, 1e-3, f"conv {geo} {epi}")


@pytest.mark.parametrize("resid", [False, True])
def test_conv3_rows_bf16_out_matches_generic_path(resid, monkeypatch):
    """bf16 output of the rows-in-LDS 3x3 kernel (BasicEncoder 64 -> 64 at 128 x 128) vs f64 and
    vs the implicit-GEMM path (COMET_CONV_NO_ROWS=1) on the same inputs: both round the same f32
    sums to bf16, so they differ by at most one bf16 ulp where the summation order flips it."""
    ops = _ops()
    n, h, w, c = 2, 128, 128, 64
    x = _rand(n, c, h, w, seed=24).to(torch.bfloat16)
    wt = _rand(c, c, 3, 3, seed=25, scale=1.0 / math.sqrt(c * 9)).to(torch.bfloat16)
    b = _rand(c, seed=26)
    ref = F.conv2d(x.double(), wt.double(), b.double(), padding=1).permute(0, 2, 3, 1)
    wm = wt.permute(0, 2, 3, 1).reshape(c, 9 * c).contiguous().to(DEV)
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    kw = dict(bias=b.to(DEV), out_dtype=torch.bfloat16)
    if resid:
        r = _rand(*ref.shape, seed=27).to(torch.bfloat16)
        ref = F.relu(ref) + 0.5 * r.double()
        kw.update(act=2, resid=r.to(DEV), beta=0.5)
    y = ops.conv2d_nhwc(xd, wm, 3, 3, 1, 1, **kw)
    _close(y, ref, 1e-2, 1e-2, f"conv rows bf16 resid={resid}")
    monkeypatch.setenv("COMET_CONV_NO_ROWS", "1")
    y2 = ops.conv2d_nhwc(xd, wm, 3, 3, 1, 1, **kw)
    d = (y.float() - y2.float()).abs()
    assert (d <= 2 ** -7 * y2.float().abs() + 1e-6).all(), f"rows vs generic: max diff {d.max().item():.3e}"


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_gemm_epilogue_bias_gelu_resid_aux(dtype):
    ops = _ops()
    M, N, K = 257, 384, 192
    x = _rand(M, K, dtype=dtype, seed=3)
    w = _rand(N, K, dtype=dtype, seed=4, scale=0.1)
    b = _rand(N, seed=5)
    r = _rand(M, N, seed=6)
    pre = x.double() @ w.double().t() + b.double()
    ref = F.gelu(pre) + 0.5 * r.double()
    out = torch.empty(M, N, device=DEV, dtype=torch.float32)
    aux = torch.empty(M, N, device=DEV, dtype=torch.float32)
    ops.linear(x.to(DEV), w.to(DEV), bias=b.to(DEV), act=1, resid=r.to(DEV), beta=0.5, out=out, aux=aux)
    tol = 1e-5 if dtype == torch.float32 else 2e-3
    _close(out, ref, tol, 1e-3, "epilogue out")
    _close(aux, pre, tol, 1e-3, "epilogue aux")


@pytest.mark.parametrize("mnk", [(257, 384, 64), (4096, 1536, 384)])
def test_gemm_gelu_epilogue_precision(mnk):
    """The epilogue GELU (csrc/common.hpp gelu_erf, exp2-polynomial form; tools/gelu_fit.py) against the f64
    erf GELU of the kernel's own f32 pre-activation (aux): pre-activations over [-12, 12] via the bias,
    |err| <= 3e-7 + one f32 rounding of the output (the fit's bound is 2.8e-7)."""
    ops = _ops()
    M, N, K = mnk
    x = _rand(M, K, dtype=torch.bfloat16, seed=7)
    w = _rand(N, K, dtype=torch.bfloat16, seed=8, scale=0.02)
    b = torch.linspace(-12, 12, N)
    out = torch.empty(M, N, device=DEV, dtype=torch.float32)
    aux = torch.empty(M, N, device=DEV, dtype=torch.float32)
    ops.linear(x.to(DEV), w.to(DEV), bias=b.to(DEV), act=1, out=out, aux=aux)
    pre = aux.double()
    assert pre.min().item() < -11 and pre.max().item() > 11
    ref = F.gelu(pre)
    err = (out.double() - ref).abs()
    bound = 3e-7 + 2 ** -24 * ref.abs()
    assert (err <= bound).all(), f"GELU epilogue: max err {err.max().item():.3e} at pre {pre.flatten()[err.argmax()].item():.4f}"
    assert torch.isfinite(out).all()


@pytest.mark.parametrize("mnk,dtype", [((257, 384, 64), torch.float32), ((8192, 1536, 384), torch.bfloat16)])
def test_gelu_non_finite_propagates(mnk, dtype):
    """NaN / +inf / -inf pre-activations give NaN through the GELU GEMM epilogue (the persistent
    kernel's bf16 pairs for the second shape) and comet_act_fwd, as torch's f32 GELU does
    (F.gelu(inf) = F.gelu(-inf) = nan on the CPU); finite columns are untouched."""
    ops = _ops()
    M, N, K = mnk
    x = _rand(M, K, dtype=dtype, seed=7)
    w = _rand(N, K, dtype=dtype, seed=8, scale=0.02)
    b = torch.linspace(-3, 3, N)
    bad_cols = {5: float("nan"), 6: float("inf"), 7: float("-inf"), N - 2: float("nan"), N - 1: float("-inf")}
    for c, v in bad_cols.items():
        b[c] = v
    out = torch.empty(M, N, device=DEV, dtype=dtype)
    ops.linear(x.to(DEV), w.to(DEV), bias=b.to(DEV), act=1, out=out)
    o = out.float().cpu()
    cols = torch.tensor(sorted(bad_cols))
    assert torch.isnan(o[:, cols]).all(), "GELU epilogue hid a non-finite pre-activation"
    keep = torch.ones(N, dtype=torch.bool)
    keep[cols] = False
    assert torch.isfinite(o[:, keep]).all()
    v = torch.tensor([float("nan"), float("inf"), float("-inf"), -50.0, 0.0, 2.0] * 64)
    for dt_ in (torch.float32, torch.bfloat16):
        y = ops.act_fwd(1, v.to(DEV, dt_)).float().cpu()
        ref = F.gelu(v.to(dt_).float())
        assert torch.isnan(y[:: 6]).all() and torch.isnan(y[1:: 6]).all() and torch.isnan(y[2:: 6]).all()
        fin = torch.isfinite(ref)
        assert torch.allclose(y[fin], ref[fin], atol=1e-2 if dt_ == torch.bfloat16 else 1e-6)


def test_gemm_batched_strided():
    ops = _ops()
    # per (b, h): C = Q_bh K_bh^T with q/k packed [B, L, 3, H, D]
    B, L, H, D = 3, 70, 4, 32
    qkv = _rand(B, L, 3, H, D, seed=7).to(DEV)
    q = qkv[:, :, 0]
    k = qkv[:, :, 1]
    S = torch.empty(B, H, L, L, device=DEV)
    ops.gemm_raw(q, k, S, m=L, n=L, k=D, layout_a=0, lda=3 * H * D, layout_b=0, ldb=3 * H * D, ldc=L,
                 batch=(B, H), stride_a=(L * 3 * H * D, D), stride_b=(L * 3 * H * D, D),
                 stride_c=(H * L * L, L * L))
    ref = torch.einsum("blhd,bmhd->bhlm", q.double().cpu(), k.double().cpu())
    _close(S, ref, 2e-5, 1e-4, "batched gemm")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("affine,eps,cols", [(False, 1e-6, 768), (True, 1e-5, 768), (True, 1e-5, 256), (True, 1e-5, 130)])
def test_layernorm_fwd_bwd(dtype, affine, eps, cols):
    ops = _ops()
    rows = 333
    x = _rand(rows, cols, seed=8, scale=3.0) + 1.5
    w = _rand(cols, seed=9) if affine else None
    b = _rand(cols, seed=10) if affine else None
    xd = x.to(dtype)
    xr = xd.double().requires_grad_(True)
    wr = w.double().requires_grad_(True) if affine else None
    br = b.double().requires_grad_(True) if affine else None
    yr = F.layer_norm(xr, (cols,), wr, br, eps)
    dy = _rand(rows, cols, seed=11)
    yr.backward(dy.double())
    y, mean, rstd = ops.layernorm(xd.to(DEV), w.to(DEV) if affine else None, b.to(DEV) if affine else None,
                                  eps=eps, out_dtype=torch.float32, stats=True)
    _close(y, yr.detach(), 1e-5, 1e-5, "ln fwd")
    dw = torch.zeros(cols, device=DEV) if affine else None
    db = torch.zeros(cols, device=DEV) if affine else None
    dx = ops.layernorm_bwd(xd.to(DEV), dy.to(DEV), mean, rstd, w.to(DEV) if affine else None, dw, db)
    _close(dx, xr.grad, 1e-4, 1e-4, "ln dx")
    if affine:
        _close(dw, wr.grad, 1e-4, 1e-3, "ln dw")
        _close(db, br.grad, 1e-4, 1e-3, "ln db")


def _attn_ref(q, k, v, heads, scale):
    B, Lq, C = q.shape
    D = C // heads
    qh = q.double().reshape(B, Lq, heads, D).transpose(1, 2)
    kh = k.double().reshape(B, -1, heads, D).transpose(1, 2)
    vh = v.double().reshape(B, -1, heads, D).transpose(1, 2)
    s = qh @ kh.transpose(-1, -2) * scale
    lse = torch.logsumexp(s, -1)
    o = torch.softmax(s, -1) @ vh
    return o.transpose(1, 2).reshape(B, Lq, C), lse


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("D", [32, 48, 64, 96])
@pytest.mark.parametrize("lq,lk", [(16, 16), (577, 577), (1, 512), (130, 77), (64, 200), (300, 128), (129, 64)])
def test_attention_fwd(dtype, D, lq, lk):
    ops = _ops()
    B, H = 2, 3
    q = _rand(B, lq, H * D, dtype=dtype, seed=12)
    k = _rand(B, lk, H * D, dtype=dtype, seed=13)
    v = _rand(B, lk, H * D, dtype=dtype, seed=14)
    scale = D ** -0.5
    ref, lse_ref = _attn_ref(q, k, v, H, scale)
    out, lse = ops.attention(q.to(DEV), k.to(DEV), v.to(DEV), H, scale, lse=True)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    _close(out, ref, tol, tol, f"attn {dtype} D={D} {lq}x{lk}")
    _close(lse, lse_ref, 1e-4, 1e-4 if dtype == torch.float32 else 1e-2, "lse")


def test_attention_strided_packed_qkv():
    ops = _ops()
    B, L, H, D = 2, 100, 8, 96
    C = H * D
    qkv = _rand(B, L, 3 * C, seed=15).to(DEV)
    q, k, v = qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:]
    out = ops.attention(q, k, v, H)
    ref, _ = _attn_ref(q.cpu(), k.cpu(), v.cpu(), H, D ** -0.5)
    _close(out, ref, 2e-5, 2e-5, "packed qkv attention")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_attention_large_logits_rescale(dtype):
    """Force the online-softmax rescale path: a spike key in a late tile (bf16: the lazy rescale
    that skips O *= alpha while no lane's running max moves)."""
    ops = _ops()
    B, H, D, L = 1, 2, 64, 300
    q = _rand(B, L, H * D, seed=16)
    k = _rand(B, L, H * D, seed=17)
    k[0, 250] = q[0].mean(0) * 40
    k[0, 299] = q[0].mean(0) * 60  # spike in the ragged last tile
    v = _rand(B, L, H * D, seed=18)
    q, k, v = q.to(dtype), k.to(dtype), v.to(dtype)
    ref, lse_ref = _attn_ref(q, k, v, H, D ** -0.5)
    out, lse = ops.attention(q.to(DEV), k.to(DEV), v.to(DEV), H, lse=True)
    tol = 2e-5 if dtype == torch.float32 else 2e-2
    _close(out, ref, tol, tol, f"rescale {dtype}")
    _close(lse, lse_ref, 1e-4, 1e-4 if dtype == torch.float32 else 2e-2, "rescale lse")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_conv_via_im2col(dtype):
    ops = _ops()
    N, Cin, H, W, Cout = 2, 5, 17, 19, 24
    for (k, s, p) in [(7, 2, 3), (3, 1, 1), (1, 1, 0), (3, 2, 1), (14, 14, 0)]:
        Hs, Ws = (28, 42) if k == 14 else (H, W)
        x = _rand(N, Cin, Hs, Ws, dtype=dtype, seed=19)
        w = _rand(Cout, Cin, k, k, dtype=dtype, seed=20, scale=0.2)
        b = _rand(Cout, seed=21)
        ref = F.conv2d(x.double(), w.double(), b.double(), stride=s, padding=p)
        xn = x.permute(0, 2, 3, 1).contiguous().to(DEV)
        cols, oh, ow = ops.im2col_nhwc(xn, k, k, s, p)
        wm = w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous().to(DEV)
        y = ops.linear(cols, wm, bias=b.to(DEV), out_dtype=torch.float32)
        y = y.reshape(N, oh, ow, Cout).permute(0, 3, 1, 2)
        tol = 1e-5 if dtype == torch.float32 else 2e-3
        _close(y, ref, tol, tol * 10, f"conv k={k} s={s}")


def test_instnorm_and_resize():
    ops = _ops()
    x = _rand(3, 40, 23, 21, seed=22) * 2 + 1
    res = _rand(3, 40, 23, 21, seed=23)
    ref = F.relu(F.instance_norm(x.double()) + res.double())
    y = ops.instnorm_nhwc(x.permute(0, 2, 3, 1).contiguous().to(DEV), res.permute(0, 2, 3, 1).contiguous().to(DEV), relu=True)
    _close(y.permute(0, 3, 1, 2), ref, 1e-5, 1e-5, "instnorm")
    for (oh, ow) in [(11, 10), (64, 64), (31, 31), (1, 1)]:
        r = F.interpolate(x, (oh, ow), mode="bilinear", align_corners=True)
        y1 = ops.resize_bilinear(x.to(DEV), oh, ow, nhwc=False)
        _close(y1, r, 1e-5, 1e-5, f"resize nchw {oh}x{ow}")
        y2 = ops.resize_bilinear(x.permute(0, 2, 3, 1).contiguous().to(DEV), oh, ow, nhwc=True)
        _close(y2.permute(0, 3, 1, 2), r, 1e-5, 1e-5, f"resize nhwc {oh}x{ow}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,c,h,w", [(2, 96, 128, 128), (700, 32, 16, 16), (3, 12, 9, 7), (5, 256, 33, 17), (1, 64, 8, 8),
                                     (999, 32, 4, 4), (333, 16, 8, 8), (17, 8, 5, 7), (9, 64, 12, 11)])
@pytest.mark.parametrize("mode", ["plain", "inner_res_relu"])
def test_instnorm_shapes(dtype, n, c, h, w, mode):
    """Chunked (partials + apply), fused (one block per image), one-wave-per-image (small bf16
    images, incl. a partial last workgroup and partial pixel slots) and generic (c % 8 != 0) paths;
    inputs with a large common offset exercise the shifted-moment variance."""
    ops = _ops()
    x = (_rand(n, c, h, w, seed=30) * 0.5 + 40.0).to(dtype)
    res = _rand(n, c, h, w, seed=31).to(dtype) if mode != "plain" else None
    ref = F.instance_norm(x.double(), eps=1e-5)
    if mode != "plain":
        ref = F.relu(F.relu(ref) + res.double())
    y = ops.instnorm_nhwc(x.permute(0, 2, 3, 1).contiguous().to(DEV),
                          res.permute(0, 2, 3, 1).contiguous().to(DEV) if res is not None else None,
                          relu=mode != "plain", relu_inner=mode != "plain")
    tol = 2e-4 if dtype == torch.float32 else 1.6e-2
    _close(y.permute(0, 3, 1, 2), ref, tol, tol, f"instnorm {dtype} {(n, c, h, w)} {mode}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_resize_nhwc_vector_add(dtype):
    ops = _ops()
    x = _rand(4, 64, 37, 29, seed=32).to(dtype)
    base = _rand(4, 64, 64, 64, seed=33).to(dtype)
    ref = F.interpolate(x.double(), (64, 64), mode="bilinear", align_corners=True) + base.double()
    out = base.permute(0, 2, 3, 1).contiguous().to(DEV)
    ops.resize_bilinear(x.permute(0, 2, 3, 1).contiguous().to(DEV), 64, 64, nhwc=True, out=out, add=True)
    # f32 coordinates as ATen (align_corners lambdas in f32) vs an f64 reference
    tol = 5e-5 if dtype == torch.float32 else 1.6e-2
    _close(out.permute(0, 3, 1, 2), ref, tol, tol, f"resize nhwc add {dtype}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,c,h,w,oh,ow", [(300, 32, 16, 16, 31, 31), (3, 416, 16, 16, 64, 64), (7, 8, 5, 3, 1, 1),
                                           (2, 128, 64, 64, 32, 32)])
def test_resize_nhwc_row_blocked(dtype, n, c, h, w, oh, ow):
    """Row-blocked NHWC resize: several output rows per block (ow * c/8 < 256), one row looped over
    (> 256 items), 1 x 1 output; vs ATen align_corners in f64."""
    ops = _ops()
    x = _rand(n, c, h, w, seed=34).to(dtype)
    ref = F.interpolate(x.double(), (oh, ow), mode="bilinear", align_corners=True)
    y = ops.resize_bilinear(x.permute(0, 2, 3, 1).contiguous().to(DEV), oh, ow, nhwc=True)
    tol = 5e-5 if dtype == torch.float32 else 1.6e-2
    _close(y.permute(0, 3, 1, 2), ref, tol, tol, f"resize rows {dtype} {(n, c, h, w, oh, ow)}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,c,h,w", [(300, 32, 31, 31), (4, 128, 64, 64), (2, 128, 5, 7), (3, 12, 8, 8)])
def test_avgpool2_nhwc(dtype, n, c, h, w):
    """2x2 average pool (CorrBlock pyramid, blocks.py:351-429: F.avg_pool2d(k=2, s=2), odd sizes
    floor): row-blocked 8-channel path and the scalar path (c % 8 != 0)."""
    ops = _ops()
    x = _rand(n, c, h, w, seed=35).to(dtype)
    ref = F.avg_pool2d(x.double(), 2, stride=2)
    y = ops.avgpool2_nhwc(x.permute(0, 2, 3, 1).contiguous().to(DEV))
    tol = 1e-6 if dtype == torch.float32 else 8e-3
    _close(y.permute(0, 3, 1, 2), ref, tol, tol, f"avgpool2 {dtype} {(n, c, h, w)}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,S,N", [(2, 5, 37), (1, 16, 64)])
def test_track_score_parallel_matches_serial(dtype, B, S, N, monkeypatch):
    """compute_score_fn (refine_track.py:174-278): the one-thread-per-window kernel equals the
    per-track loop (whose parity with the reference is pinned end to end by the model goldens),
    incl. windows clamped at the patch border."""
    ops = _ops()
    P, C = 31, 32
    q = _rand(B * N, C, seed=36).to(DEV)
    pf = _rand(B * N, S, P, P, C, seed=37).to(dtype).to(DEV)
    fine = (torch.rand(B * N, S, 2, generator=torch.Generator().manual_seed(38)) * 34 - 2).to(DEV)
    s1, i1 = ops.track_score(q, pf, fine, B, S, N)
    monkeypatch.setenv("COMET_SCORE_SERIAL", "1")
    s2, i2 = ops.track_score(q, pf, fine, B, S, N)
    _close(s1, s2.double(), 1e-5, 1e-5, "score")
    _close(i1, i2.double(), 1e-5, 1e-5, "inv score")


@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("which", ["a", "b", "ab"])
@pytest.mark.parametrize("mnk", [(200, 136, 264), (96, 64, 6000)])
def test_gemm_f32_operands_converted_on_load(la, lb, which, mnk):
    """bf16 GEMM with f32 operands rounded to bf16 on load (convert_a / convert_b) equals the GEMM of
    the pre-rounded operands exactly up to f32 accumulation order."""
    ops = _ops()
    M, N, K = mnk
    A = _rand(M, K, seed=40)
    B = _rand(N, K, seed=41)
    ref = A.to(torch.bfloat16).double() @ B.to(torch.bfloat16).double().t()
    Ad = (A if la == 0 else A.t().contiguous()).to(DEV)
    Bd = (B if lb == 0 else B.t().contiguous()).to(DEV)
    if "a" not in which:
        Ad = Ad.to(torch.bfloat16)
    if "b" not in which:
        Bd = Bd.to(torch.bfloat16)
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    ops.gemm_raw(Ad, Bd, C, m=M, n=N, k=K, layout_a=la, lda=(K if la == 0 else M), layout_b=lb,
                 ldb=(K if lb == 0 else N), ldc=N, compute=torch.bfloat16)
    _close(C, ref, 1e-4, 1e-4 * math.sqrt(K), f"cvt gemm la={la} lb={lb} {which} {mnk}")


@pytest.mark.parametrize("act", [0, 1, 2, 3])
@pytest.mark.parametrize("dtypes", [(torch.float32, torch.bfloat16), (torch.bfloat16, torch.bfloat16), (torch.float32, torch.float32)])
def test_act_bwd_colsum(act, dtypes):
    ops = _ops()
    dy_dt, out_dt = dtypes
    rows, cols = 3001, 392
    pre = _rand(rows, cols, seed=42).to(torch.bfloat16)
    dy = _rand(rows, cols, seed=43).to(dy_dt)
    p = pre.double()
    g = {0: torch.ones_like(p), 1: None, 2: (p > 0).double(), 3: torch.sigmoid(p) * (1 - torch.sigmoid(p))}[act]
    if act == 1:
        cdf = 0.5 * (1 + torch.erf(p / math.sqrt(2)))
        g = cdf + p * torch.exp(-0.5 * p * p) / math.sqrt(2 * math.pi)
    ref = dy.double() * g
    db = torch.full((cols,), 5.0, device=DEV)
    out = ops.act_bwd_colsum(act, pre.to(DEV), dy.to(DEV), out_dtype=out_dt, dbias=db, accumulate=True)
    tol = 1e-5 if out_dt == torch.float32 else 8e-3
    _close(out, ref, tol, tol, f"act_bwd_colsum out act={act}")
    # bf16 out: db sums the rounded values; a rounding-boundary flip moves one term by 1 bf16 ulp
    _close(db, ref.to(out_dt).double().sum(0) + 5.0, 1e-4, 1e-3 if out_dt == torch.float32 else 8e-3,
           f"act_bwd_colsum db act={act}")


@pytest.mark.parametrize("rows,cols", [(0, 768), (1, 4), (5, 100), (128, 768), (128, 3072), (577, 768),
                                       (4096, 392), (4097, 392), (20000, 130)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_colsum(rows, cols, dtype):
    """comet_colsum (the f32 path's bias gradients) vs f64 sums, on a strided (ld > cols) view, both
    without and with accumulate: the few-rows kernel (rows <= 4096, round 5) and the atomic one."""
    ops = _ops()
    g = torch.Generator().manual_seed(rows + cols)
    big = torch.randn(rows, cols + 24, generator=g).to(dtype).to(DEV)
    x = big[:, 8:8 + cols]
    ref = x.double().sum(0)
    out = ops.colsum(x)
    _close(out, ref, 1e-5, 1e-5 * max(1.0, math.sqrt(rows)), f"colsum {rows}x{cols} {dtype}")
    acc = torch.full((cols,), 2.5, device=DEV)
    ops.colsum(x, out=acc, accumulate=True)
    _close(acc, ref + 2.5, 1e-5, 1e-5 * max(1.0, math.sqrt(rows)), f"colsum accumulate {rows}x{cols} {dtype}")


@pytest.mark.parametrize("D", [32, 48, 64, 96])
@pytest.mark.parametrize("lq,lk", [(577, 577), (130, 1000), (16, 16), (200, 70)])
def test_flash_attention_bwd(D, lq, lk):
    """comet_attention_bwd (bf16) vs f64 autograd of softmax(q k^T s) v on the same bf16 inputs,
    with packed-projection strides like the model's (q/k/v slices of one [B, L, 3C] buffer)."""
    ops = _ops()
    B, H = 2, 3
    C = H * D
    g = torch.Generator().manual_seed(50)
    q = torch.randn(B, lq, C, generator=g).to(torch.bfloat16)
    kv = torch.randn(B, lk, 2 * C, generator=g).to(torch.bfloat16)
    do = torch.randn(B, lq, C, generator=g).to(torch.bfloat16)
    scale = D ** -0.5
    qd, kvd = q.to(DEV), kv.to(DEV)
    k, v = kvd[..., :C], kvd[..., C:]
    o, lse = ops.attention(qd, k, v, H, scale, lse=True)
    dq = torch.empty_like(qd)
    dkv = torch.empty_like(kvd)
    ops.attention_bwd(qd, k, v, o, lse, do.to(DEV), H, scale, dq, dkv[..., :C], dkv[..., C:])
    # reference
    qr = q.double().view(B, lq, H, D).transpose(1, 2).requires_grad_(True)
    kr = kv[..., :C].double().reshape(B, lk, H, D).transpose(1, 2).requires_grad_(True)
    vr = kv[..., C:].double().reshape(B, lk, H, D).transpose(1, 2).requires_grad_(True)
    p = torch.softmax(qr @ kr.transpose(-1, -2) * scale, -1)
    out = (p @ vr)
    out.backward(o.detach().cpu().double().view(B, lq, H, D).transpose(1, 2) * 0 + do.double().view(B, lq, H, D).transpose(1, 2))
    ref_dq = qr.grad.transpose(1, 2).reshape(B, lq, C)
    ref_dk = kr.grad.transpose(1, 2).reshape(B, lk, C)
    ref_dv = vr.grad.transpose(1, 2).reshape(B, lk, C)
    for name, got, ref in (("dq", dq, ref_dq), ("dk", dkv[..., :C], ref_dk), ("dv", dkv[..., C:], ref_dv)):
        m = ref.abs().max().item()
        _close(got, ref, 2e-2, 2e-2 * m, f"flash bwd {name} D={D} lq={lq} lk={lk}")


@pytest.mark.parametrize("cols", [384, 768, 1024, 130])
def test_layernorm_dual_output_and_two_grads(cols):
    """Vectorised LN: f32 output + bf16 copy in one kernel; backward of dy (f32) + dy2 (bf16)
    with dx in bf16 (cols=130 exercises the scalar fallback with one output / f32 dx)."""
    ops = _ops()
    rows = 517
    x = _rand(rows, cols, seed=60, scale=2.0) + 0.7
    dy = _rand(rows, cols, seed=61)
    dy2 = _rand(rows, cols, seed=62).to(torch.bfloat16)
    xr = x.double().requires_grad_(True)
    yr = F.layer_norm(xr, (cols,), eps=1e-6)
    vec = cols % 8 == 0
    if vec:
        y, y16, mean, rstd = ops.layernorm(x.to(DEV), eps=1e-6, out_dtype=torch.float32, stats=True, dual=True)
        _close(y16, yr.detach(), 8e-3, 8e-3, "ln dual bf16 copy")
        yr.backward(dy.double() + dy2.double())
        dx = ops.layernorm_bwd(x.to(DEV), dy.to(DEV), mean, rstd, dy2=dy2.to(DEV), dx_dtype=torch.bfloat16)
        _close(dx, xr.grad, 1e-2, 1e-2, "ln dx (dy + dy2, bf16 out)")
    else:
        y, mean, rstd = ops.layernorm(x.to(DEV), eps=1e-6, out_dtype=torch.float32, stats=True)
        yr.backward(dy.double())
        dx = ops.layernorm_bwd(x.to(DEV), dy.to(DEV), mean, rstd)
        _close(dx, xr.grad, 1e-4, 1e-4, "ln dx scalar path")
    _close(y, yr.detach(), 1e-5, 1e-5, "ln y f32")


@pytest.mark.parametrize("D", [32, 48, 64, 96])
@pytest.mark.parametrize("lq,lk", [(16, 16), (5, 11), (16, 3), (1, 16), (9, 1)])
def test_attention_short_sequences(D, lq, lk):
    """Short-sequence path (one wave per (batch, head), Lq, Lk <= 16) incl. batch*heads not a
    multiple of 4 and packed strides."""
    ops = _ops()
    B, H = 7, 3
    C = H * D
    qkv = _rand(B, 16, 3 * C, seed=70).to(torch.bfloat16)
    q, k, v = qkv[:, :lq, :C], qkv[:, :lk, C:2 * C], qkv[:, :lk, 2 * C:]
    ref, lse_ref = _attn_ref(q, k, v, H, D ** -0.5)
    qd = qkv.to(DEV)
    out, lse = ops.attention(qd[:, :lq, :C], qd[:, :lk, C:2 * C], qd[:, :lk, 2 * C:], H, D ** -0.5, lse=True)
    _close(out, ref, 2e-2, 2e-2, f"short attn D={D} {lq}x{lk}")
    _close(lse, lse_ref, 1e-2, 1e-2, "short attn lse")


@pytest.mark.parametrize("n,k", [(32, 32), (16, 96), (64, 256), (48, 40)])
@pytest.mark.parametrize("out_dtype", [torch.bfloat16, torch.float32])
def test_gemm_skinny_narrow_outputs(n, k, out_dtype):
    """Narrow-N path (M >= 16384, N <= 64): bias + ReLU + residual epilogue vs f64."""
    ops = _ops()
    M = 20001
    x = _rand(M, k, seed=80).to(torch.bfloat16)
    w = _rand(n, k, seed=81, scale=0.2).to(torch.bfloat16)
    b = _rand(n, seed=82)
    r = _rand(M, n, seed=83).to(out_dtype)
    ref = F.relu(x.double() @ w.double().t() + b.double()) + 0.5 * r.double()
    out = ops.linear(x.to(DEV), w.to(DEV), bias=b.to(DEV), act=2, resid=r.to(DEV), beta=0.5, out_dtype=out_dtype)
    tol = 1e-4 if out_dtype == torch.float32 else 1e-2
    _close(out, ref, tol, tol, f"skinny gemm n={n} k={k} {out_dtype}")


@pytest.mark.parametrize("mnk", [(5000, 1100, 128), (4096, 512, 64), (8191, 768, 384), (4100, 1000, 192), (4500, 256, 320),
                                 (4097, 640, 128)])
@pytest.mark.parametrize("epi", ["plain_f32", "gelu_aux_bf16", "bias_resid_f32"])
def test_gemm_256_tile_path(mnk, epi):
    """256 x 256 glds kernel (forward Linear shapes: k-contiguous bf16, K % 64 == 0, M >= 4096,
    N >= 256) with M / N tails and every epilogue, vs f64."""
    ops = _ops()
    M, N, K = mnk
    x = _rand(M, K, seed=90).to(torch.bfloat16)
    w = _rand(N, K, seed=91, scale=0.1).to(torch.bfloat16)
    b = _rand(N, seed=92)
    pre = x.double() @ w.double().t()
    if epi == "plain_f32":
        out = ops.linear(x.to(DEV), w.to(DEV), out_dtype=torch.float32)
        _close(out, pre, 1e-4, 1e-4 * math.sqrt(K), f"256 plain {mnk}")
    elif epi == "gelu_bf16":
        # interior tiles store 16 B per lane (permlane16 pairs), edge tiles 8 B: both against f64,
        # and the wide stores bit-identical to the 8-B ones (COMET_GEMM_NO_WIDE=1)
        out = ops.linear(xd, wd, bias=bd, act=1, out_dtype=torch.bfloat16)
        _close(out, F.gelu(pre + b.double()), 1e-2, 1e-2, f"pp gelu {mnk}")
        monkeypatch.setenv("COMET_GEMM_NO_WIDE", "1")
        out8 = ops.linear(xd, wd, bias=bd, act=1, out_dtype=torch.bfloat16)
        assert torch.equal(out, out8), f"wide vs 8-B stores differ at {mnk}"
    elif epi == "gelu_aux_bf16":
        aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        out = ops.linear(x.to(DEV), w.to(DEV), bias=b.to(DEV), act=1, aux=aux, out_dtype=torch.bfloat16)
        _close(aux, pre + b.double(), 1e-2, 1e-2, f"256 aux {mnk}")
        _close(out, F.gelu(pre + b.double()), 1e-2, 1e-2, f"256 gelu {mnk}")
    else:
        r = _rand(M, N, seed=93)
        out = ops.linear(x.to(DEV), w.to(DEV), bias=b.to(DEV), resid=r.to(DEV), beta=0.5, out_dtype=torch.float32)
        _close(out, pre + b.double() + 0.5 * r.double(), 1e-4, 1e-4 * math.sqrt(K), f"256 resid {mnk}")


@pytest.mark.parametrize("mnk", [(20000, 3072, 192), (70001, 768, 64), (33000, 1152, 256), (4100, 1024, 1536),
                                 (20001, 384, 1536), (8200, 384, 384), (65536, 384, 64),
                                 (8192, 1536, 384), (6000, 768, 192), (8200, 1152, 320)])
@pytest.mark.parametrize("epi", ["plain_f32", "gelu_aux_bf16", "gelu_bf16", "bias_resid_f32", "inplace_resid_f32"])
def test_gemm_persistent_path(mnk, epi, monkeypatch):
    """Persistent kernel (256 x 256 tiles; 128 x 384 for N = 384): several tiles per workgroup
    (k-tile prefetch across tile boundaries), M / N tails, direct (bf16) and parked (f32) epilogues
    incl. an in-place residual (out is resid), vs f64."""
    ops = _ops()
    M, N, K = mnk
    x = _rand(M, K, seed=94).to(torch.bfloat16)
    w = _rand(N, K, seed=95, scale=0.1).to(torch.bfloat16)
    b = _rand(N, seed=96)
    pre = x.double() @ w.double().t()
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    if epi == "plain_f32":
        out = ops.linear(xd, wd, out_dtype=torch.float32)
        _close(out, pre, 1e-4, 1e-4 * math.sqrt(K), f"pp plain {mnk}")
    elif epi == "gelu_aux_bf16":
        aux = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
        out = ops.linear(xd, wd, bias=bd, act=1, aux=aux, out_dtype=torch.bfloat16)
        _close(aux, pre + b.double(), 1e-2, 1e-2, f"pp aux {mnk}")
        _close(out, F.gelu(pre + b.double()), 1e-2, 1e-2, f"pp gelu {mnk}")
    else:
        r = _rand(M, N, seed=97)
        rd = r.to(DEV)
        if epi == "inplace_resid_f32":
            out = ops.linear(xd, wd, bias=bd, resid=rd, beta=0.5, out=rd, out_dtype=torch.float32)
        else:
            out = ops.linear(xd, wd, bias=bd, resid=rd, beta=0.5, out_dtype=torch.float32)
        _close(out, pre + b.double() + 0.5 * r.double(), 1e-4, 1e-4 * math.sqrt(K), f"pp resid {mnk}")


@pytest.mark.parametrize("tile", ["256x256", "128x256", "128x384", "64x384"])
@pytest.mark.parametrize("mnk", [(5000, 1000, 192), (9000, 1536, 384)])
def test_gemm_persistent_tiles(tile, mnk, monkeypatch):
    """Every tile instance of the persistent kernel (COMET_PP_TILE override) on M / N tails (N = 1000
    leaves a partial 384- and 256-column tile), GELU bf16 and residual f32 epilogues, vs f64."""
    ops = _ops()
    monkeypatch.setenv("COMET_PP_TILE", tile)
    M, N, K = mnk
    x = _rand(M, K, seed=98).to(torch.bfloat16)
    w = _rand(N, K, seed=99, scale=0.1).to(torch.bfloat16)
    b = _rand(N, seed=100)
    r = _rand(M, N, seed=101)
    pre = x.double() @ w.double().t() + b.double()
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    out = ops.linear(xd, wd, bias=bd, act=1, out_dtype=torch.bfloat16)
    _close(out, F.gelu(pre), 1e-2, 1e-2, f"pp {tile} gelu {mnk}")
    out = ops.linear(xd, wd, bias=bd, resid=r.to(DEV), out_dtype=torch.float32)
    _close(out, pre + r.double(), 1e-4, 1e-4 * math.sqrt(K), f"pp {tile} resid {mnk}")


@pytest.mark.parametrize("la,lb", [(0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("mnk", [(4096, 512, 128), (768, 3072, 20480), (1000, 1000, 640), (384, 1152, 8192)])
def test_gemm_256_tile_transposed_and_split(la, lb, mnk):
    """256-row tile kernel with row-contiguous operands (dX = dY.W, dW = dY^T.X shapes), incl. the
    split-K partial path for long K, vs f64."""
    ops = _ops()
    M, N, K = mnk
    A = _rand(M, K, seed=100).to(torch.bfloat16)
    B = _rand(N, K, seed=101).to(torch.bfloat16)
    ref = A.double() @ B.double().t()
    Ad = (A if la == 0 else A.t().contiguous()).to(DEV)
    Bd = (B if lb == 0 else B.t().contiguous()).to(DEV)
    C = torch.empty(M, N, device=DEV, dtype=torch.float32)
    ops.gemm_raw(Ad, Bd, C, m=M, n=N, k=K, layout_a=la, lda=(K if la == 0 else M), layout_b=lb,
                 ldb=(K if lb == 0 else N), ldc=N)
    _close(C, ref, 1e-3, 1e-3 * math.sqrt(K), f"256 la={la} lb={lb} {mnk}")


@pytest.mark.parametrize("D", [32, 48, 64])
def test_attention_inner_batch_4d(D):
    """[B, L, T, H*D] views: attention over L for every (b, t) (space blocks without permute)."""
    ops = _ops()
    B, L, T, H = 2, 70, 5, 3
    C = H * D
    x = _rand(B, L, T, 3 * C, seed=110).to(torch.bfloat16)
    q, k, v = x[..., :C], x[..., C:2 * C], x[..., 2 * C:]
    ref = torch.empty(B, L, T, C, dtype=torch.float64)
    for t in range(T):
        ref[:, :, t], _ = _attn_ref(q[:, :, t], k[:, :, t], v[:, :, t], H, D ** -0.5)
    xd = x.to(DEV)
    out = ops.attention(xd[..., :C], xd[..., C:2 * C], xd[..., 2 * C:], H)
    _close(out, ref, 2e-2, 2e-2, f"inner-batch attention D={D}")


@pytest.mark.parametrize("cols,xdt,ydt", [(768, torch.float32, torch.bfloat16), (384, torch.float32, torch.float32),
                                          (768, torch.bfloat16, torch.bfloat16), (1024, torch.float32, torch.bfloat16)])
def test_layernorm_persistent_rows(cols, xdt, ydt, monkeypatch):
    """Persistent-row LayerNorm forward (each wave walks several rows with the next row
    prefetched): 20011 rows > 2048 x 4 waves, vs f64 and bit-exact vs the one-row-per-wave kernel."""
    ops = _ops()
    rows = 20011
    x = (_rand(rows, cols, seed=120, scale=2.0) + 0.3).to(xdt)
    w, b = _rand(cols, seed=121), _rand(cols, seed=122)
    ref = F.layer_norm(x.double(), (cols,), w.double(), b.double(), 1e-5)
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    y, mean, rstd = ops.layernorm(xd, wd, bd, eps=1e-5, out_dtype=ydt, stats=True)
    tol = 1e-5 if ydt == torch.float32 else 8e-3
    _close(y, ref, tol, tol, f"ln rows {cols} {xdt}->{ydt}")
    monkeypatch.setenv("COMET_LN_FLAT", "1")
    y1, mean1, rstd1 = ops.layernorm(xd, wd, bd, eps=1e-5, out_dtype=ydt, stats=True)
    assert torch.equal(mean, mean1) and torch.equal(rstd, rstd1)
    tol1 = 1e-6 if ydt == torch.float32 else 8e-3  # one bf16 ulp if an fma contracts differently
    _close(y, y1.double(), tol1, tol1, "ln rows vs one-row-per-wave")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_tracker_tokens_row_blocked(dtype, monkeypatch):
    """comet_tracker_tokens (base_track_predictor.py:186-222 token assembly): the wave-per-row
    4-column kernel (default, round 5) and the row-blocked kernel (COMET_TOKENS_ROWS=1) bit-identical
    to the flat element-wise kernel, incl. the zero pad columns."""
    ops = _ops()
    B, N, S, lat, corrdim = 2, 37, 5, 128, 324
    tdim = 2 * (lat // 2) + 2 + corrdim + lat + 6
    rows = B * N * S
    coords = (_rand(rows, 2, seed=130) * 20).to(DEV)
    feats = _rand(rows, lat, seed=131).to(DEV)
    corr = _rand(rows, corrdim + 4, seed=132).to(DEV)[:, :corrdim]
    pos = _rand(B * N, tdim, seed=133).to(DEV)
    x1 = torch.empty(rows, tdim, device=DEV, dtype=dtype)
    x2 = torch.empty(rows, tdim, device=DEV, dtype=dtype)
    x3 = torch.empty(rows, tdim, device=DEV, dtype=dtype)
    ops.tracker_tokens(coords, feats, lat, corr, corrdim, pos, tdim, x1, rows, S)
    monkeypatch.setenv("COMET_TOKENS_ROWS", "1")
    ops.tracker_tokens(coords, feats, lat, corr, corrdim, pos, tdim, x3, rows, S)
    monkeypatch.setenv("COMET_TOKENS_FLAT", "1")
    ops.tracker_tokens(coords, feats, lat, corr, corrdim, pos, tdim, x2, rows, S)
    assert torch.equal(x1, x2) and torch.equal(x3, x2)
    # spot check against the definition: frame-0 rows have zero flow -> emb = sin(0)/cos(0)
    E = lat // 2
    r0 = x1[0].float().cpu() - pos[0].cpu()
    tol = 1e-6 if dtype == torch.float32 else 5e-2
    assert (r0[0:2 * E:2].abs() <= tol).all() and ((r0[1:2 * E:2] - 1).abs() <= tol).all()
    # rows padded to a 64-column multiple (the bf16 update former's input, round 6): the same tdim
    # columns, zeros after them
    tdp = (tdim + 63) // 64 * 64
    xp = torch.full((rows, tdp), 7.0, device=DEV, dtype=dtype)
    monkeypatch.delenv("COMET_TOKENS_ROWS")
    monkeypatch.delenv("COMET_TOKENS_FLAT")
    ops.tracker_tokens(coords, feats, lat, corr, corrdim, pos, tdim, xp, rows, S)
    assert torch.equal(xp[:, :tdim], x2) and (xp[:, tdim:] == 0).all()


def test_update_former_input_gemm_padded_k():
    """The update former's input Linear on zero-padded bf16 tokens (K 664 -> 704, 216 -> 256, with
    the weight's columns padded alike, functional.wcast_kpad) equals the unpadded GEMM within f32
    summation order and takes the persistent kernel (blocks.py:157, modules.py:119-154)."""
    from comet_amd import functional as Fn
    ops = _ops()
    for M, N, K in [(65536, 384, 664), (65536, 256, 216)]:
        Kp = (K + 63) // 64 * 64
        g = torch.Generator(device=DEV).manual_seed(K)
        x = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
        xp = torch.zeros(M, Kp, device=DEV, dtype=torch.bfloat16)
        xp[:, :K] = x
        w = torch.nn.Parameter(torch.randn(N, K, device=DEV, generator=g) * K ** -0.5)
        b = torch.randn(N, device=DEV, generator=g)
        with torch.no_grad(), Fn.precision(torch.bfloat16):
            y = Fn.linear(x, w, b, out_dtype=torch.float32)
            yp = Fn.linear(xp, Fn.wcast_kpad(w, Kp), b, out_dtype=torch.float32)
        assert tuple(ops._PLAN)[0] == 3, f"padded K {Kp}: expected the persistent plan, got {tuple(ops._PLAN)}"
        ref = x.double() @ w.detach().to(torch.bfloat16).double().t() + b.double()
        for out in (y, yp):
            assert ((out.double() - ref).abs() <= 1e-5 * ref.abs() + 2e-5 * K ** 0.5).all()
        Fn.invalidate_weight_cache([w])


def _corr_ref(pyr, radius, feats, coords, B, N, S):
    """CorrBlock.corr + CorrBlock.sample (blocks.py:351-429) in f64: per level, the correlation map
    f . fmap / sqrt(C) sampled bilinearly (zeros padding, align_corners=True pixel coordinates) at
    (x/2^l + i - r, y/2^l + j - r), window index i on x."""
    C = pyr[0].shape[-1]
    win = 2 * radius + 1
    out = torch.zeros(B * N * S, len(pyr) * win * win, dtype=torch.float64)
    d = torch.arange(-radius, radius + 1, dtype=torch.float64)
    for l, fm in enumerate(pyr):
        fm = fm.double().cpu()
        H, W = fm.shape[1], fm.shape[2]
        for t in range(B * N * S):
            s = t % S
            b = t // S // N
            cmap = fm[b * S + s] @ feats[t].double().cpu() / math.sqrt(C)  # [H, W]
            xl = coords[t, 0].item() / 2 ** l
            yl = coords[t, 1].item() / 2 ** l
            X = (xl + d).view(win, 1).expand(win, win)   # i on x
            Y = (yl + d).view(1, win).expand(win, win)   # j on y
            x0, y0 = torch.floor(X), torch.floor(Y)
            v = torch.zeros(win, win, dtype=torch.float64)
            for dx in (0, 1):
                for dy in (0, 1):
                    xi, yi = x0 + dx, y0 + dy
                    wgt = (1 - (X - xi).abs()) * (1 - (Y - yi).abs())
                    ok = (xi >= 0) & (xi < W) & (yi >= 0) & (yi < H)
                    g = cmap[yi.clamp(0, H - 1).long(), xi.clamp(0, W - 1).long()]
                    v += torch.where(ok, g * wgt, torch.zeros_like(g))
            out[t, l * win * win:(l + 1) * win * win] = v.reshape(-1)
    return out


@pytest.mark.parametrize("C,radius,dtype", [(128, 4, torch.bfloat16), (128, 3, torch.float32), (32, 3, torch.bfloat16),
                                            (128, 6, torch.bfloat16), (32, 6, torch.float32), (128, 1, torch.bfloat16)])
def test_corr_sample_vs_f64(C, radius, dtype):
    """comet_corr_sample (fused CorrBlock corr + window sampling) vs an f64 restatement (tracks
    near and beyond the map border)."""
    ops = _ops()
    B, N, S, levels = 2, 3, 2, 3
    H0 = 20
    pyr = [_rand(B * S, H0 >> l, H0 >> l, C, seed=140 + l).to(dtype).to(DEV) for l in range(levels)]
    rows = B * N * S
    feats = _rand(rows, C, seed=150)
    coords = torch.rand(rows, 2, generator=torch.Generator().manual_seed(151)) * (H0 + 8) - 4
    win = 2 * radius + 1
    out = torch.full((rows, levels * win * win + 5), 7.0, device=DEV)
    ops.corr_sample(pyr, radius, feats.to(DEV), coords.to(DEV), out, 2, B, N, S)
    ref = _corr_ref(pyr, radius, feats, coords, B, N, S)
    _close(out[:, 2:2 + levels * win * win], ref, 1e-4, 1e-4, f"corr C={C} r={radius}")
    assert (out[:, :2] == 7.0).all() and (out[:, 2 + levels * win * win:] == 7.0).all()


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_corr_sample_wave_per_row_bit_identical(dtype, monkeypatch):
    """The fine tracker's correlation (C = 32, radius 3, 3 levels on 31 x 31 patch maps and their
    pools): the one-wave-per-row kernel (default) equals the one-workgroup-per-row kernel
    (COMET_CORR_BLOCK=1) bit for bit, for a row count that does not fill the last workgroup, tracks
    near and beyond the border and a NaN track; and both match the f64 restatement."""
    ops = _ops()
    B, N, S, levels, radius, C = 1, 37, 3, 3, 3, 32
    sizes = [31, 15, 7]
    pyr = [_rand(B * S, sizes[l], sizes[l], C, seed=340 + l).to(dtype).to(DEV) for l in range(levels)]
    rows = B * N * S
    feats = _rand(rows, C, seed=350)
    coords = torch.rand(rows, 2, generator=torch.Generator().manual_seed(351)) * 39 - 4
    coords[7] = float("nan")
    win = 2 * radius + 1
    outs = []
    for block in (False, True):
        if block:
            monkeypatch.setenv("COMET_CORR_BLOCK", "1")
        o = torch.full((rows, levels * win * win + 2), 7.0, device=DEV)
        ops.corr_sample(pyr, radius, feats.to(DEV), coords.to(DEV), o, 1, B, N, S)
        outs.append(o)
    assert torch.equal(torch.nan_to_num(outs[0], nan=123.0), torch.nan_to_num(outs[1], nan=123.0))
    ok = torch.ones(rows, dtype=torch.bool)
    ok[7] = False
    cref = coords.clone()
    cref[7] = 0.0  # (the f64 restatement indexes with the coordinates; the NaN row is not compared)
    ref = _corr_ref(pyr, radius, feats, cref, B, N, S)
    _close(outs[0][ok.to(DEV), 1:1 + levels * win * win], ref[ok], 1e-4, 1e-4, "corr wave C=32")
    assert (outs[0][:, :1] == 7.0).all() and (outs[0][:, 1 + levels * win * win:] == 7.0).all()


@pytest.mark.parametrize("layout", ["uniform", "clustered", "outside"])
def test_corr_sample_mfma_vs_f64(layout):
    """The matrix-core CorrBlock path (bf16 maps, C = 128, >= 16 tracks per frame: the coarse
    tracker's case) vs the f64 restatement: N = 200 tracks per frame (not a multiple of the 16-track
    wave groups or the 64-track workgroups), 4 levels; tracks spread over the map, all in one spot
    (every wave's box the same), or partly far outside the map."""
    ops = _ops()
    B, N, S, levels, radius, C, H0 = 1, 200, 2, 4, 4, 128, 40
    pyr = [_rand(B * S, H0 >> l, H0 >> l, C, seed=240 + l).to(torch.bfloat16).to(DEV) for l in range(levels)]
    rows = B * N * S
    feats = _rand(rows, C, seed=250)
    g = torch.Generator().manual_seed(251)
    if layout == "uniform":
        coords = torch.rand(rows, 2, generator=g) * (H0 + 8) - 4
    elif layout == "clustered":
        coords = 17.3 + torch.rand(rows, 2, generator=g) * 0.5
    else:
        coords = torch.rand(rows, 2, generator=g) * (H0 + 8) - 4
        coords[::3] = coords[::3] * 40 - 800
    win = 2 * radius + 1
    out = torch.full((rows, levels * win * win + 3), 7.0, device=DEV)
    ops.corr_sample(pyr, radius, feats.to(DEV), coords.to(DEV), out, 1, B, N, S)
    ref = _corr_ref(pyr, radius, feats, coords, B, N, S)
    _close(out[:, 1:1 + levels * win * win], ref, 1e-4, 1e-4, f"corr mfma {layout}")
    assert (out[:, :1] == 7.0).all() and (out[:, 1 + levels * win * win:] == 7.0).all()


def test_corr_sample_mfma_matches_valu_headline(monkeypatch):
    """At the coarse tracker's headline shape per frame (N = 512 tracks, 64 x 64 x 128 bf16 maps,
    4 levels, radius 4), the matrix-core path equals the VALU kernel (COMET_CORR_VALU=1) up to f32
    summation order; tracks with NaN coordinates leave the other tracks' rows untouched."""
    ops = _ops()
    B, N, S, levels, radius, C, H0 = 2, 512, 3, 4, 4, 128, 64
    pyr = [(_rand(B * S, H0 >> l, H0 >> l, C, seed=260 + l) * 2).to(torch.bfloat16).to(DEV) for l in range(levels)]
    rows = B * N * S
    feats = _rand(rows, C, seed=270).to(DEV)
    coords = (torch.rand(rows, 2, generator=torch.Generator().manual_seed(271)) * 70 - 3).to(DEV)
    coords[5] = float("nan")
    win = 2 * radius + 1
    outs = []
    for valu in (False, True):
        if valu:
            monkeypatch.setenv("COMET_CORR_VALU", "1")
        o = torch.empty(rows, levels * win * win, device=DEV)
        ops.corr_sample(pyr, radius, feats, coords, o, 0, B, N, S)
        outs.append(o)
    ok = torch.ones(rows, dtype=torch.bool, device=DEV)
    ok[5] = False
    a, v = outs[0][ok], outs[1][ok]
    assert torch.isfinite(a).all()
    # both sum 128 exact products in f32, in different orders: the difference is f32 rounding of
    # sums whose terms reach ~|v|max, so it is bounded against the output scale, not per element:
    # at most ~128 roundings of 2^-24 (7.6e-6); observed 1.5-2.3e-6 (the VALU kernel's add order
    # moved when the library stopped SLP-packing its f32 adds, round 6)
    err = ((a - v).abs().max() / v.abs().max()).item()
    assert err < 8e-6, err


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_resize_into_channel_slices(dtype):
    """BasicEncoder concat (blocks.py:102-107): four maps resized straight into their channel
    slices of one NHWC tensor equal torch.cat of the separate resizes."""
    ops = _ops()
    n, oh, ow = 3, 24, 24
    parts = [_rand(n, 48, 48, 64, seed=160), _rand(n, 24, 24, 96, seed=161), _rand(n, 12, 12, 128, seed=162),
             _rand(n, 6, 6, 128, seed=163)]
    parts = [p.to(dtype).to(DEV) for p in parts]
    x = torch.full((n, oh, ow, 416), 3.0, device=DEV, dtype=dtype)
    c0 = 0
    for p in parts:
        ops.resize_bilinear_into(p, x[..., c0:c0 + p.shape[-1]])
        c0 += p.shape[-1]
    ref = torch.cat([ops.resize_bilinear(p, oh, ow, nhwc=True) for p in parts], dim=-1)
    # the small parts take the whole-image kernel in resize_bilinear: equal up to fma contraction
    tol = 1e-5 if dtype == torch.float32 else 8e-3
    _close(x, ref.double(), tol, tol, "resize into slices vs cat")


@pytest.mark.parametrize("la,lb", [(1, 1), (0, 1), (1, 0)])
@pytest.mark.parametrize("mnk", [(256, 512, 5000), (512, 768, 1100), (768, 256, 4161)])
@pytest.mark.parametrize("out", [torch.float32, torch.bfloat16])
def test_gemm_256_tile_ragged_k(la, lb, mnk, out, monkeypatch):
    """dW-shaped GEMMs with K % 64 != 0 (token counts like 8 x 15 x 577): the 64-multiple part as
    256-row split-K partials plus the remainder as one more partial, one reduce with the bias
    epilogue; vs f64 and vs the generic 128 x 128 path."""
    ops = _ops()
    M, N, K = mnk
    A = _rand(M, K, seed=170).to(torch.bfloat16)
    B = _rand(N, K, seed=171).to(torch.bfloat16)
    bias = _rand(N, seed=172)
    ref = A.double() @ B.double().t() + bias.double()
    Ad = (A if la == 0 else A.t().contiguous()).to(DEV)
    Bd = (B if lb == 0 else B.t().contiguous()).to(DEV)
    res = []
    for env in (None, "1"):
        if env:
            monkeypatch.setenv("COMET_GEMM_NO_RAGGED", env)
        C = torch.empty(M, N, device=DEV, dtype=out)
        ops.gemm_raw(Ad, Bd, C, m=M, n=N, k=K, layout_a=la, lda=(K if la == 0 else M), layout_b=lb,
                     ldb=(K if lb == 0 else N), ldc=N, bias=bias.to(DEV), bias_mode=1)
        res.append(C)
    tol = 1e-3 if out == torch.float32 else 8e-3
    _close(res[0], ref, tol, 1e-3 * math.sqrt(K), f"ragged-K la={la} lb={lb} {mnk}")
    _close(res[0], res[1].double(), tol, 1e-3 * math.sqrt(K), "ragged-K vs generic path")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("n,c,h,w,oh,ow,add", [(500, 32, 16, 16, 31, 31, False), (300, 32, 8, 8, 16, 16, True),
                                               (70, 32, 4, 4, 16, 16, True), (9, 64, 11, 7, 5, 9, False)])
def test_resize_nhwc_whole_image(dtype, n, c, h, w, oh, ow, add, monkeypatch):
    """One-workgroup-per-image NHWC resize (input staged in LDS; ShallowEncoder patch maps,
    blocks.py:179-202) vs ATen align_corners in f64, and equal to the row kernel."""
    ops = _ops()
    x = _rand(n, c, h, w, seed=180).to(dtype)
    base = _rand(n, c, oh, ow, seed=181).to(dtype)
    ref = F.interpolate(x.double(), (oh, ow), mode="bilinear", align_corners=True)
    if add:
        ref = ref + base.double()
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    outs = []
    for env in (None, "1"):
        if env:
            monkeypatch.setenv("COMET_RESIZE_ROWS", env)
        out = base.permute(0, 2, 3, 1).contiguous().to(DEV)
        y = ops.resize_bilinear(xd, oh, ow, nhwc=True, out=out if add else None, add=add)
        outs.append(y)
    tol = 5e-5 if dtype == torch.float32 else 1.6e-2
    _close(outs[0].permute(0, 3, 1, 2), ref, tol, tol, f"resize img {dtype} {(n, c, h, w, oh, ow, add)}")
    tol1 = 1e-5 if dtype == torch.float32 else 8e-3  # fma contraction may differ between the kernels
    _close(outs[0], outs[1].double(), tol1, tol1, "whole-image vs row kernel")


def test_sq_norm_multi_vectorised_and_ragged():
    """comet_sq_norm_multi (clip_grad_norm_'s total norm, train_util.py:311-332): 16-B loads with
    scalar heads / tails for unaligned views and ragged sizes, > 24 tensors (several launches)."""
    import ctypes
    from comet_amd import _lib as L
    from comet_amd import ops
    base = _rand(3_000_000, seed=190).to(DEV)
    views = [base[1:1 + 1_000_003], base[8:8 + 17], base[1_100_001:1_100_001 + 5], base[2_000_000:2_900_000]]
    views += [base[100 + 37 * i: 100 + 37 * i + 3 + i] for i in range(30)]
    out = torch.zeros(1, device=DEV)
    part = torch.empty(L.SQ_NORM_PARTIALS, device=DEV)
    arr = (ctypes.c_void_p * len(views))(*[v.data_ptr() for v in views])
    sz = (ctypes.c_int64 * len(views))(*[v.numel() for v in views])
    L.check(L.load().comet_sq_norm_multi(arr, sz, len(views), out.data_ptr(), part.data_ptr(), ops.stream()), "sq_norm")
    ref = sum((v.double().cpu() ** 2).sum() for v in views)
    _close(out, ref.reshape(1), 1e-5, 0, "sq_norm_multi")


def test_sq_norm_multi_bit_identical_across_launches():
    """The clip coefficient of every data-parallel replica comes from this sum: it is a fixed-order
    two-pass reduction (per-workgroup partials, folded in index order), so repeated launches -- and
    launches with another stream's kernels on the GPU -- return the same bits (round 5: one f32
    atomicAdd per workgroup, arrival order). Sizes of the camera predictor's
    gradient set (train_eval_func_new_cp5.py:797-801)."""
    import ctypes
    from comet_amd import _lib as L
    from comet_amd import ops
    torch.manual_seed(5)
    ts = [torch.randn(n, device=DEV) * (1 + i % 7) for i, n in enumerate(
        [768 * 768 * 3, 768 * 3, 768 * 768, 768, 3072 * 768, 3072, 768 * 3072, 768, 1] * 4 + [5, 17, 1_000_003])]
    arr = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
    sz = (ctypes.c_int64 * len(ts))(*[t.numel() for t in ts])
    lib = L.load()
    side = torch.cuda.Stream()
    big = torch.randn(4096, 4096, device=DEV, dtype=torch.bfloat16)
    outs = []
    for it in range(20):
        with torch.cuda.stream(side):  # unrelated work competing for the CUs
            big @ big
        out = torch.zeros(1, device=DEV)
        part = torch.empty(L.SQ_NORM_PARTIALS, device=DEV)
        L.check(lib.comet_sq_norm_multi(arr, sz, len(ts), out.data_ptr(), part.data_ptr(), ops.stream()), "sq_norm")
        outs.append(out)
    torch.cuda.synchronize()
    vals = torch.cat(outs).cpu()
    ref = sum((t.double() ** 2).sum().item() for t in ts)
    assert abs(vals[0].item() - ref) <= 1e-5 * ref
    assert torch.equal(vals, vals[:1].expand_as(vals)), f"sq_norm varies between launches: {vals.unique().tolist()}"


def test_persistent_gemm_leaves_no_lds_writes_in_flight():
    """A GEMM workgroup must not end with LDS-DMA pieces in flight: the CU hands its LDS to the next
    workgroup at once, and when that belongs to another stream's (or another process's) kernel the
    late k-tile bytes overwrite it. comet_lds_probe workgroups own a whole CU's LDS and count words
    that change under them, on a second stream beside persistent GEMMs whose epilogue issues no load
    (no bias, bf16 out: the lock-step loop's trailing re-loads are drained only by the exit wait).
    Measured 0 with and without that wait (tools/lds_race.py, profiles/r06_race/r06a): the wait is
    kept as the guarantee, this test as its guard."""
    import sys
    import os
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import lds_race
    got = lds_race.run(iters=20)
    print(got)
    assert all(n == 0 for n in got.values()), f"probe LDS words overwritten: {got}"


def test_kernels_exact_beside_a_concurrent_mfma_stream():
    """gfx950 returns wrong values from a packed-FP32 instruction whose low result reads the high
    dword of its second / third source while another wave on the same SIMD issues MFMAs (round 6:
    two ranks sharing the GPU saw 1e-3 run-to-run gradient variation; the first differing op was the
    row-LN reduce's centring, tools/op_record.py, profiles/r06_race). The library is built without
    those forms (Makefile -fno-slp-vectorize, tools/isa_hazard.py). Here the kernels that carried
    them -- the row-LN split reduce (gemm.hip), the LayerNorm backward (norm.hip) -- run on one stream
    while a second stream keeps the SIMDs busy with an MFMA stream (comet_shfl_probe mode 12), and
    must repeat their isolated result bit for bit. Positive control: the hazard's own form (probe
    mode 7) beside the same load must fail, or the two streams never shared a SIMD and the test
    proves nothing (then it skips)."""
    import ctypes
    from comet_amd import _lib as L
    from comet_amd import ops
    lib = L.load()
    g = torch.Generator(device=DEV).manual_seed(11)
    M, K, N = 8192, 1536, 384
    x = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV, generator=g)
    r = torch.randn(M, N, device=DEV, generator=g)
    xl = torch.randn(65536, 384, device=DEV, generator=g)
    dy = torch.randn(65536, 384, device=DEV, generator=g).to(torch.bfloat16)
    lw = torch.randn(384, device=DEV, generator=g)
    _, mean, rstd = ops.layernorm(xl, lw, eps=1e-5, stats=True)

    def victims():
        c, y, _ = ops.linear_rowln(x, w, b, r, raw=True, y16_eps=1e-5)
        dw = torch.zeros(384, device=DEV)
        dx = ops.layernorm_bwd(xl, dy, mean, rstd, lw, dweight=dw)
        return [c, y, dx]

    ref = [t.clone() for t in victims()]
    side = torch.cuda.Stream()
    ctl = torch.zeros(1, device=DEV, dtype=torch.int32)
    load = torch.zeros(1, device=DEV, dtype=torch.int32)
    torch.cuda.synchronize()
    bad = []
    for it in range(40):
        with torch.cuda.stream(side):
            L.check(lib.comet_shfl_probe(4096, 64, 12, ctypes.c_void_p(load.data_ptr()), ops.stream()), "probe")
        outs = victims()
        with torch.cuda.stream(side):
            L.check(lib.comet_shfl_probe(4096, 64, 12, ctypes.c_void_p(load.data_ptr()), ops.stream()), "probe")
        L.check(lib.comet_shfl_probe(1024, 16, 7, ctypes.c_void_p(ctl.data_ptr()), ops.stream()), "probe")
        bad += [(it, k) for k, (o, rr) in enumerate(zip(outs, ref)) if not torch.equal(o, rr)]
    torch.cuda.synchronize()
    print(f"hazard control: {ctl.item()} wrong lane results; product kernels differing: {bad[:10]}")
    assert not bad, f"outputs differ beside the MFMA stream: {bad[:10]}"
    if ctl.item() == 0:
        pytest.skip("the two streams never shared a SIMD (control clean): nothing was tested")


# 256 x 256 tiles with the ping-pong k-loop: by default bf16 outputs without activation / residual
# at K >= 768 and any output at K >= 2048 (gemm.hip launch_pp); (M, N) give >= 256 tiles (full-height
# tiles), M / N tails and workgroups with 2-3 tiles each
_PING_SHAPES = [(20000, 1000, 768), (33000, 1000, 768), (8200, 2304, 1536), (16500, 1000, 3072), (70001, 768, 2048)]


@pytest.mark.parametrize("ping", ["default", "1", "0"])
@pytest.mark.parametrize("mnk", _PING_SHAPES)
@pytest.mark.parametrize("epi", ["plain_bf16", "bias_bf16", "resid_f32", "inplace_resid_f32"])
def test_gemm_ping_pong_path(mnk, epi, ping, monkeypatch):
    """The ping-pong k-loop (gemm.hip PING instances: two wave groups one barrier apart over a 4-slot
    ring, asm LDS-DMA with counted waits) against f64, on the shapes that select it by default and
    forced on / off (COMET_GEMM_PING) over the same shapes: bf16 park epilogue with and without bias,
    f32 residual epilogue in place and not (modules.py:119-154 Linear)."""
    ops = _ops()
    M, N, K = mnk
    if epi.endswith("_f32") and K < 2048 and ping == "default":
        pytest.skip("f32 outputs take the ping-pong loop at K >= 2048 only (covered by the forced runs)")
    if ping != "default":
        monkeypatch.setenv("COMET_GEMM_PING", ping)
    g = torch.Generator(device=DEV).manual_seed(K + N)
    xd = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    wd = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).to(torch.bfloat16)
    bd = torch.randn(N, device=DEV, generator=g)
    pre = xd.double() @ wd.double().t()
    if epi == "plain_bf16":
        out = ops.linear(xd, wd, out_dtype=torch.bfloat16)
        ref = pre
    elif epi == "bias_bf16":
        out = ops.linear(xd, wd, bias=bd, out_dtype=torch.bfloat16)
        ref = pre + bd.double()
    else:
        rd = torch.randn(M, N, device=DEV, generator=g)
        ref = pre + bd.double() + 0.5 * rd.double()
        out = ops.linear(xd, wd, bias=bd, resid=rd, beta=0.5, out=rd if epi == "inplace_resid_f32" else None,
                         out_dtype=torch.float32)
    plan = tuple(ops._PLAN)
    assert plan[0] == 3 and plan[1] == 256 and plan[2] == 256, f"expected the 256 x 256 persistent plan, got {plan}"
    err = (out.double() - ref).abs()
    tol = (8e-3 * ref.abs() + 8e-3) if out.dtype == torch.bfloat16 else (1e-4 * ref.abs() + 2e-5 * math.sqrt(K))
    bad = int((err > tol).sum())
    assert bad == 0, f"{epi} {mnk} ping={ping}: max err {err.max().item():.3e}, {bad} bad"


@pytest.mark.parametrize("mnk", [(74368 + 40, 2304 + 16, 768), (20000, 1000, 768), (65536, 1152, 384),
                                 (9000, 768, 1024), (33000, 768, 3072)])
@pytest.mark.parametrize("odt", ["bf16_gelu", "f32_resid"])
def test_gemm_tile_order(mnk, odt, monkeypatch):
    """The persistent kernel's two tile orders (gemm.hip: XCD-banded waves, the default, and per-XCD
    contiguous tile ranges, COMET_GEMM_RASTER=1, a measurement switch) compute every tile the same
    way: bit-identical outputs, within the f64 bound, on tiled shapes with M / N tails and tile counts
    that do not divide by the 8 XCDs (modules.py:119-154 Linear)."""
    ops = _ops()
    M, N, K = mnk
    g = torch.Generator(device=DEV).manual_seed(M + K)
    xd = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    wd = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).to(torch.bfloat16)
    bd = torch.randn(N, device=DEV, generator=g)
    rd = torch.randn(M, N, device=DEV, generator=g) if odt == "f32_resid" else None
    outs = {}
    for mode in ("0", "1"):
        monkeypatch.setenv("COMET_GEMM_RASTER", mode)
        if rd is None:
            outs[mode] = ops.linear(xd, wd, bias=bd, act=1, out_dtype=torch.bfloat16)
        else:
            outs[mode] = ops.linear(xd, wd, bias=bd, resid=rd, out_dtype=torch.float32)
        assert ops._PLAN[0] == 3, f"expected the persistent plan, got {tuple(ops._PLAN)}"
    assert torch.equal(outs["0"], outs["1"]), f"{mnk} {odt}: the tile order changed the result"
    pre = xd.double() @ wd.double().t() + bd.double()
    if rd is None:
        ref = torch.nn.functional.gelu(pre)
        tol = 1e-2 * ref.abs() + 1e-2
    else:
        ref = pre + rd.double()
        tol = 1e-4 * ref.abs() + 2e-5 * math.sqrt(K)
    err = (outs["1"].double() - ref).abs()
    bad = int((err > tol).sum())
    assert bad == 0, f"{mnk} {odt}: max err {err.max().item():.3e}, {bad} bad"


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("geo", [(512, 16, 16, 32, 31, 31), (64, 16, 16, 32, 30, 30), (33, 9, 13, 16, 17, 24),
                                 (8, 4, 4, 64, 3, 2)])
def test_resize_bilinear_pool_fused(dtype, geo):
    """comet_resize_bilinear_pool_nhwc (the fine ShallowEncoder's last up-sampling with the fine
    pyramid's 2 x 2 average pool, blocks.py:371 / refine_track.py) equals comet_resize_bilinear
    followed by comet_avgpool2_nhwc bit for bit, odd and even output sizes; and both match torch's
    F.interpolate(align_corners=True) + F.avg_pool2d."""
    ops = _ops()
    n, h, w, c, oh, ow = geo
    g = torch.Generator(device=DEV).manual_seed(n + oh)
    x = torch.randn(n, h, w, c, device=DEV, generator=g).to(dtype)
    y, p = ops.resize_bilinear_pool(x, oh, ow)
    y_ref = ops.resize_bilinear(x, oh, ow, nhwc=True)
    p_ref = ops.avgpool2_nhwc(y_ref)
    assert torch.equal(y, y_ref) and torch.equal(p, p_ref)
    yt = torch.nn.functional.interpolate(x.permute(0, 3, 1, 2).float(), size=(oh, ow), mode="bilinear",
                                         align_corners=True)
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert (y.permute(0, 3, 1, 2).float() - yt).abs().max().item() <= tol * (1 + yt.abs().max().item())
    pt = torch.nn.functional.avg_pool2d(y.permute(0, 3, 1, 2).float(), 2, stride=2)
    assert (p.permute(0, 3, 1, 2).float() - pt).abs().max().item() <= tol * (1 + pt.abs().max().item())


@pytest.mark.parametrize("ups", [0, 2])
@pytest.mark.parametrize("c,n,hw,o", [(32, 128, 16, 31), (32, 64, 16, 30), (64, 256, 8, 15)])
def test_conv1x1_resize_pool_fused(c, n, hw, o, ups):
    """comet_conv1x1_resize_pool_nhwc (the fine ShallowEncoder's tail, blocks.py:97-110: the two
    resize-and-adds of layer1 / layer2's outputs, conv2 + residual, the final up-sampling and the
    fine pyramid's levels 1 and 2) equals the unfused calls bit for bit -- resize_bilinear(out=x, add=True)
    twice, the narrow GEMM (linear with resid, M >= 16384 rows: the skinny kernel), resize_bilinear
    and avgpool2_nhwc -- and t matches an f64 reference."""
    ops = _ops()
    g = torch.Generator(device=DEV).manual_seed(c + n + o + ups)
    x = torch.randn(n, hw, hw, c, device=DEV, generator=g).to(torch.bfloat16)
    u1 = torch.randn(n, hw // 2, hw // 2, c, device=DEV, generator=g).to(torch.bfloat16) if ups else None
    u2 = torch.randn(n, hw // 4, hw // 4, c, device=DEV, generator=g).to(torch.bfloat16) if ups else None
    w = (torch.randn(c, c, device=DEV, generator=g) * c ** -0.5).to(torch.bfloat16)
    b = torch.randn(c, device=DEV, generator=g)
    y, p, q = ops.conv1x1_resize_pool(x, w, b, o, o, up1=u1, up2=u2, pool2=True)
    y2, p2 = ops.conv1x1_resize_pool(x, w, b, o, o, up1=u1, up2=u2)
    assert torch.equal(y, y2) and torch.equal(p, p2)
    x2 = x.clone()
    if ups:
        ops.resize_bilinear(u1, hw, hw, nhwc=True, out=x2, add=True)
        ops.resize_bilinear(u2, hw, hw, nhwc=True, out=x2, add=True)
    t = ops.linear(x2.reshape(-1, c), w, bias=b, resid=x2.reshape(-1, c), out_dtype=torch.bfloat16)
    assert tuple(ops._PLAN)[0] == 0, f"expected the skinny GEMM plan, got {tuple(ops._PLAN)}"
    tref = (x2.reshape(-1, c).double() @ w.double().t() + b.double() + x2.reshape(-1, c).double())
    assert ((t.double() - tref).abs() <= 1e-2 * tref.abs() + 1e-2).all()
    y_ref = ops.resize_bilinear(t.reshape(n, hw, hw, c), o, o, nhwc=True)
    p_ref = ops.avgpool2_nhwc(y_ref)
    assert torch.equal(y, y_ref), f"y: max diff {(y.float() - y_ref.float()).abs().max().item():.3e}"
    assert torch.equal(p, p_ref), f"pool: max diff {(p.float() - p_ref.float()).abs().max().item():.3e}"
    assert torch.equal(q, ops.avgpool2_nhwc(p_ref)), "second pyramid level differs"


@pytest.mark.parametrize("cols", [8, 32, 64])
@pytest.mark.parametrize("dts", [(torch.float32, torch.float32), (torch.float32, torch.bfloat16),
                                 (torch.bfloat16, torch.bfloat16)])
def test_layernorm_narrow_rows_bit_identical(cols, dts, monkeypatch):
    """The several-rows-per-wave LayerNorm for narrow rows (the tracker's GroupNorm(1, 32),
    base_track_predictor.py:81,238; bf16 rows up to 64 columns) equals the one-row-per-wave kernel
    (COMET_LN_NO_NARROW=1) bit for bit -- outputs, the bf16 copy, mean and rstd -- with affine
    weights, relu, and a row count that does not fill the last wave; and matches torch's f32 LN."""
    ops = _ops()
    tx, ty = dts
    g = torch.Generator(device=DEV).manual_seed(cols)
    rows = 1001
    x = (torch.randn(rows, cols, device=DEV, generator=g) * 3 + 1).to(tx)
    w = torch.randn(cols, device=DEV, generator=g)
    b = torch.randn(cols, device=DEV, generator=g)
    outs = []
    for narrow in (True, False):
        if not narrow:
            monkeypatch.setenv("COMET_LN_NO_NARROW", "1")
        outs.append(ops.layernorm(x, w, b, eps=1e-5, out_dtype=ty, stats=True, dual=True, relu=True))
    for a, r in zip(outs[0], outs[1]):
        assert torch.equal(a, r)
    ref = torch.relu(torch.nn.functional.layer_norm(x.float(), (cols,), w, b, eps=1e-5))
    tol = 1e-5 if ty == torch.float32 else 1e-2
    assert (outs[0][0].float() - ref).abs().max().item() <= tol * (1 + ref.abs().max().item())


def test_cast_multi_and_weight_cache_refresh():
    """comet_cast_multi_f32_bf16 equals torch's RNE .to(bfloat16) bit for bit (aligned and
    unaligned views, > 48 tensors); refresh_weight_cache re-casts cached copies in place after
    the parameters change."""
    from comet_amd import functional as Fn
    from comet_amd import ops
    base = _rand(200_000, seed=200).to(DEV)
    srcs = [base[1:1 + 999], base[1024:1024 + 4096], base[9000:9000 + 7]] + [base[10000 + 64 * i:10000 + 64 * i + 33 + i] for i in range(60)]
    dsts = [torch.empty(s.numel(), device=DEV, dtype=torch.bfloat16) for s in srcs]
    ops.cast_multi_f32_bf16(srcs, dsts)
    for s, d in zip(srcs, dsts):
        assert torch.equal(d, s.to(torch.bfloat16))
    w = torch.nn.Parameter(_rand(384, 96, seed=201).to(DEV))
    c_full, c_top = Fn.wcast(w), Fn.wcast(w[:128])
    with torch.no_grad():
        w.mul_(1.5).add_(0.25)
    Fn.refresh_weight_cache([w])
    assert Fn.wcast(w) is c_full and torch.equal(c_full, w.detach().to(torch.bfloat16))
    assert torch.equal(Fn.wcast(w[:128]), w.detach()[:128].to(torch.bfloat16))
    Fn.invalidate_weight_cache([w])


@pytest.mark.parametrize("mnk", [(65536, 384, 384), (8192, 384, 1536), (8192 + 40, 384, 384), (65536, 256, 256),
                                 (8192, 256, 1024), (4096 + 100, 256, 256)])
@pytest.mark.parametrize("mode", ["raw_y16", "dual", "dual_ctx", "raw_only"])
def test_gemm_rowln(mnk, mode):
    """comet_gemm_rowln: residual GEMM with the consumers' row LayerNorms in the epilogue (tracker
    update former, modules.py:248-344) vs f64: one tile spans the row (N = 384: 128 x 384 / 64 x 384
    tiles; N = 256: 256 x 256 / 128 x 256), M tails take the edge copy of the epilogue."""
    ops = _ops()
    M, N, K = mnk
    x = _rand(M, K, seed=101).to(torch.bfloat16)
    w = _rand(N, K, seed=102, scale=K ** -0.5).to(torch.bfloat16)
    b = _rand(N, seed=103, scale=0.1)
    r = _rand(M, N, seed=104) + 0.5  # nonzero row means: the LN must remove them
    zw, zb = _rand(N, seed=105), _rand(N, seed=106)
    v = x.double() @ w.double().t() + b.double() + r.double()
    mu = v.mean(-1, keepdim=True)
    var = v.var(-1, unbiased=False, keepdim=True)
    ln6 = (v - mu) / torch.sqrt(var + 1e-6)
    ln5 = (v - mu) / torch.sqrt(var + 1e-5) * zw.double() + zb.double()
    xd, wd, bd, rd = x.to(DEV), w.to(DEV), b.to(DEV), r.to(DEV)
    assert ops.linear_rowln_ok(xd, wd, rd)
    raw = mode in ("raw_y16", "raw_only")
    c, y16, z16 = ops.linear_rowln(xd, wd, bd, rd, raw=raw, y16_eps=None if mode == "raw_only" else 1e-6,
                                   z=(zw.to(DEV), zb.to(DEV), 1e-5) if mode == "dual_ctx" else None)
    tol = 2e-5 * math.sqrt(K)
    _close(c, v if raw else ln6, 1e-4, tol, f"rowln c {mnk} {mode}")
    if mode == "raw_only":
        assert y16 is None and z16 is None
    else:
        _close(y16, ln6, 8e-3, 8e-3, f"rowln y16 {mnk} {mode}")
    if mode == "dual_ctx":
        _close(z16, ln5, 8e-3, 3e-2, f"rowln z16 {mnk} {mode}")
    torch.cuda.synchronize()


def test_gemm_rowln_matches_separate_kernels():
    """The fused epilogue equals the GEMM + LayerNorm kernels it replaces (bf16 outputs bit-equal
    up to one rounding step, f32 within summation-order noise)."""
    ops = _ops()
    M, N, K = 16384, 384, 1536
    x = _rand(M, K, seed=111).to(torch.bfloat16).to(DEV)
    w = _rand(N, K, seed=112, scale=K ** -0.5).to(torch.bfloat16).to(DEV)
    b = _rand(N, seed=113, scale=0.1).to(DEV)
    r = _rand(M, N, seed=114).to(DEV)
    c, y16, _ = ops.linear_rowln(x, w, b, r, raw=False, y16_eps=1e-6)
    ref = ops.linear(x, w, bias=b, resid=r, out_dtype=torch.float32)
    y32r, y16r = ops.layernorm(ref, eps=1e-6, out_dtype=torch.float32, dual=True)
    _close(c, y32r, 1e-5, 1e-5, "rowln dual f32 vs separate")
    d = (y16.float() - y16r.float()).abs() / y16r.float().abs().clamp_min(1e-3)
    assert d.max().item() <= 2 ** -7, d.max().item()


@pytest.mark.parametrize("mnk", [(8192, 1536, 384), (4096 + 72, 3072, 768), (65536, 1024, 256)])
@pytest.mark.parametrize("act", [1, 2])
def test_gemm_persistent_preact_bf16(mnk, act):
    """Persistent kernel, bf16 output with an activation and no aux: bias + activation applied to
    the accumulators before the parked whole-line stores (PREACT), M tails; vs f64."""
    ops = _ops()
    M, N, K = mnk
    x = _rand(M, K, seed=131).to(torch.bfloat16)
    w = _rand(N, K, seed=132, scale=K ** -0.5).to(torch.bfloat16)
    b = _rand(N, seed=133)
    pre = x.double() @ w.double().t() + b.double()
    ref = F.gelu(pre) if act == 1 else torch.relu(pre)
    out = ops.linear(x.to(DEV), w.to(DEV), bias=b.to(DEV), act=act, out_dtype=torch.bfloat16)
    _close(out, ref, 1e-2, 1e-2, f"pp preact {mnk} act{act}")




@pytest.mark.parametrize("la,lb", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("mnk", [(16, 768, 768), (16, 768, 2304), (128, 2304, 768), (128, 768, 3072), (48, 96, 640)])
@pytest.mark.parametrize("out", [torch.float32, torch.bfloat16])
def test_gemm_small_split_matches_unsplit(la, lb, mnk, out, monkeypatch):
    """Few-tile short-K bf16 GEMMs (the camera trunk's M = 16-128 token GEMMs) split K over
    workgroups (choose_splits); the split result equals the unsplit one to f32 summation order and
    both are within bf16-operand tolerance of f64."""
    ops = _ops()
    M, N, K = mnk
    A = _rand(M, K, dtype=torch.bfloat16, seed=21)
    B = _rand(N, K, dtype=torch.bfloat16, seed=22)
    bias = _rand(N, seed=23).to(DEV)
    ref = A.double() @ B.double().t() + bias.double().cpu()
    Ad = (A if la == 0 else A.t().contiguous()).to(DEV)
    Bd = (B if lb == 0 else B.t().contiguous()).to(DEV)
    res = {}
    for mode in ("split", "nosplit"):
        if mode == "nosplit":
            monkeypatch.setenv("COMET_GEMM_NO_SMALLSPLIT", "1")
        C = torch.full((M, N), float("nan"), device=DEV, dtype=out)
        ops.gemm_raw(Ad, Bd, C, m=M, n=N, k=K, layout_a=la, lda=(K if la == 0 else M),
                     layout_b=lb, ldb=(K if lb == 0 else N), ldc=N, bias=bias, bias_mode=1)
        res[mode] = C.double().cpu()
    monkeypatch.delenv("COMET_GEMM_NO_SMALLSPLIT", raising=False)
    q = 2.0 ** -8 if out == torch.bfloat16 else 0.0
    for mode, C in res.items():
        _close(C, ref, q + 1e-5, 1e-4 * math.sqrt(K), f"{mode} {mnk} la={la} lb={lb} {out}")
    d = (res["split"] - res["nosplit"]).abs().max().item()
    assert d <= (2 * q + 1e-5) * ref.abs().max().item(), f"split vs unsplit differ by {d:.3e}"


# ---- round 4 paths, the defaults since round 5: the fused Mlp node, the 32-row row-LN tiles; last in the file ----
@pytest.mark.parametrize("M,N2,K2", [(4133, 256, 1024), (8192, 768, 3072)])
def test_gemm_dact_vs_torch(M, N2, K2):
    """comet_gemm_dact: dPre = GELU'(pre) * (dY @ W) in bf16 and dbias = column sums of the stored
    values, against torch in f32 (the erf GELU derivative) on the same bf16 operands; the bias
    gradient against the column sums of our own bf16 output (what the next GEMMs consume)."""
    ops = _ops()
    from comet_amd import _lib as L
    g = torch.Generator().manual_seed(M + N2)
    dy = (torch.randn(M, N2, generator=g) * 0.1).to(torch.bfloat16).to(DEV)
    w = (torch.randn(N2, K2, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    pre = (torch.randn(M, K2, generator=g) * 2).to(torch.bfloat16).to(DEV)
    assert ops.linear_dact_ok(dy, w, pre, L.ACT_GELU)
    db = torch.full((K2,), 5.0, device=DEV)
    out = ops.linear_dact(dy, w, pre, L.ACT_GELU, dbias=db)
    x = pre.double()
    gelu_d = 0.5 * (1 + torch.erf(x / math.sqrt(2))) + x * torch.exp(-0.5 * x * x) / math.sqrt(2 * math.pi)
    ref = (dy.double() @ w.double()) * gelu_d
    _close(out, ref, 8e-3, 1e-4 * ref.abs().max().item(), f"dact {M}x{N2}x{K2}")
    cs = out.double().sum(0)
    _close(db, cs, 1e-5, 1e-5 * cs.abs().max().item(), "dact dbias")
    # not eligible: a pre-activation of another shape, or few output tiles over a short K (the
    # 256-row kernel would not take the GEMM; the Mlp node then runs GEMM + comet_act_bwd_colsum)
    assert not ops.linear_dact_ok(dy, w, pre[:, :K2 - 8], L.ACT_GELU)
    assert not ops.linear_dact_ok(dy[:300], w, pre[:300], L.ACT_GELU)


@pytest.mark.parametrize("rows", [8 * 577, 128])
def test_mlp_fused_backward_matches_unfused(monkeypatch, rows):
    """The camera head's Mlp as one autograd node (the default; fc2's input gradient fused with
    fc1's GELU backward, comet_gemm_dact) against the two-Linear path (GEMM + comet_act_bwd_colsum) at a
    T_P-like shape in bf16: the forward is the same kernels (bit-identical); the gradients differ
    by one bf16 rounding of the hidden gradient (the fused path rounds once). 128 rows (the camera
    trunk's token count) take the node's unfused fallback."""
    _ops()
    from comet_amd import functional as F
    from comet_amd.models.modules import Mlp
    torch.manual_seed(0)
    mlp = Mlp(768, 3072).to(DEV)
    x0 = torch.randn(rows, 768, device=DEV)
    r0 = torch.randn(rows, 768, device=DEV)
    outs = {}
    for fused in (True, False):
        monkeypatch.setattr(F, "_MLP_UNFUSED", not fused)
        mlp.zero_grad(set_to_none=True)
        x = x0.clone().requires_grad_(True)
        r = r0.clone().requires_grad_(True)
        with F.precision(torch.bfloat16):
            y = mlp(x, resid=r)
        (y * torch.linspace(-1, 1, 768, device=DEV)).sum().backward()
        outs[fused] = (y.detach(), x.grad, r.grad, mlp.fc1.weight.grad, mlp.fc1.bias.grad, mlp.fc2.weight.grad,
                       mlp.fc2.bias.grad)
    names = ("y", "dx", "dresid", "dw1", "db1", "dw2", "db2")
    for n, a, b in zip(names, outs[True], outs[False]):
        if n in ("y", "dresid", "dw2"):
            assert torch.equal(a, b), n
        elif n == "db2":  # column sums by float atomics: summation order only
            assert ((a - b).abs().max() <= 1e-5 * b.abs().max()).item(), n
        else:
            rel = ((a.float() - b.float()).norm() / b.float().norm()).item()
            assert rel < 1e-2, (n, rel)


@pytest.mark.parametrize("M,K", [(8192, 384), (8192, 1536), (8192 - 40, 1536), (4096 + 8, 384)])
def test_gemm_rowln_32row_tiles(M, K, monkeypatch):
    """32 x 384 row-LN tiles (the default since round 5 where the 64-row grid fills at most half
    the CUs; four A pieces per k-tile, waves 4-7 load the same pieces as waves 0-3) equal the 64 x 384
    tiles (COMET_ROWLN_NO32=1): f32 dual copy within summation-order noise (the same k order per
    element: bit-equal expected), both bf16 LayerNorms; M tails."""
    ops = _ops()
    N = 384
    x = _rand(M, K, seed=121).to(torch.bfloat16).to(DEV)
    w = _rand(N, K, seed=122, scale=K ** -0.5).to(torch.bfloat16).to(DEV)
    b = _rand(N, seed=123, scale=0.1).to(DEV)
    r = _rand(M, N, seed=124).to(DEV)
    zw, zb = (1 + _rand(N, seed=125, scale=0.1)).to(DEV), _rand(N, seed=126, scale=0.1).to(DEV)
    monkeypatch.setenv("COMET_ROWLN_NOSPLIT", "1")  # the persistent kernel's tiles, not the split-K path
    outs = []
    for v32 in (False, True):
        if v32:
            monkeypatch.delenv("COMET_ROWLN_NO32", raising=False)
        else:
            monkeypatch.setenv("COMET_ROWLN_NO32", "1")
        outs.append(ops.linear_rowln(x, w, b, r, raw=False, y16_eps=1e-6, z=(zw, zb, 1e-5)))
    for a, c, what in zip(outs[1], outs[0], ("c", "y16", "z16")):
        _close(a, c.double(), 1e-5 if what == "c" else 8e-3, 1e-5 if what == "c" else 8e-3, f"rowln 32 vs 64 {what} M{M} K{K}")
    v = x.double() @ w.double().t() + b.double() + r.double()
    ln = (v - v.mean(1, keepdim=True)) / torch.sqrt(v.var(1, unbiased=False, keepdim=True) + 1e-6)
    _close(outs[1][0], ln, 1e-4, 1e-4, "rowln 32 vs f64")


def test_mlp_narrow_output_takes_two_linear_path():
    """The GAPR quaternion head's Mlp(768 -> 1536 -> 4) (camera_predictor10.py:385-413): a 4-wide
    output is not a multiple of 8 (the fused node's column-sum kernels), so mlp() keeps the two
    Linear nodes; forward and backward run (round 4's COMET_MLP_FUSE=1 raised here in the bench
    step) and equal the explicit two-Linear path bit for bit."""
    _ops()
    from comet_amd import functional as F
    from comet_amd.models.modules import Mlp
    torch.manual_seed(1)
    mlp = Mlp(768, 1536, out_features=4).to(DEV)
    x0 = torch.randn(128, 768, device=DEV)
    res = {}
    for unfused in (False, True):
        F._MLP_UNFUSED, old = unfused, F._MLP_UNFUSED
        try:
            mlp.zero_grad(set_to_none=True)
            x = x0.clone().requires_grad_(True)
            with F.precision(torch.bfloat16):
                y = mlp(x)
            y.square().sum().backward()
        finally:
            F._MLP_UNFUSED = old
        res[unfused] = (y.detach(), x.grad, mlp.fc1.weight.grad, mlp.fc2.weight.grad, mlp.fc2.bias.grad)
    for a, b in zip(res[False], res[True]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("M,N,K,raw,zed", [(8192, 384, 1536, False, True), (8192, 384, 1536, False, False),
                                           (8192 - 40, 384, 1536, True, False), (4096 + 8, 256, 1024, False, True),
                                           (8192, 384, 768, True, True)])
def test_gemm_rowln_split_reduce(M, N, K, raw, zed, monkeypatch):
    """Few-row row-LN GEMMs with a long K (round 5: split-K partials of the 256-row kernel + one LN
    reduce, comet_gemm_rowln_workspace > 0) equal the single-kernel persistent path
    (COMET_ROWLN_NOSPLIT=1) within f32 summation order, and the f64 LayerNorm; row tails, N = 256."""
    ops = _ops()
    from comet_amd import _lib as L
    import ctypes
    x = _rand(M, K, seed=131).to(torch.bfloat16).to(DEV)
    w = _rand(N, K, seed=132, scale=K ** -0.5).to(torch.bfloat16).to(DEV)
    b = _rand(N, seed=133, scale=0.1).to(DEV)
    r = _rand(M, N, seed=134).to(DEV)
    z = ((1 + _rand(N, seed=135, scale=0.1)).to(DEV), _rand(N, seed=136, scale=0.1).to(DEV), 1e-5) if zed else None
    g = ops._rowln_args(x, w, r, b, r)
    nb = ctypes.c_int64(0)
    L.check(L.load().comet_gemm_rowln_workspace(ctypes.byref(g), ctypes.byref(nb)), "ws")
    assert nb.value > 0, "the split path must be taken at this shape"
    outs = []
    for nosplit in (False, True):
        if nosplit:
            monkeypatch.setenv("COMET_ROWLN_NOSPLIT", "1")
        outs.append(ops.linear_rowln(x, w, b, r, raw=raw, y16_eps=1e-6, z=z))
    monkeypatch.delenv("COMET_ROWLN_NOSPLIT")
    for a, c, what in zip(outs[0], outs[1], ("c", "y16", "z16")):
        if c is None:
            assert a is None
            continue
        tol = 2e-5 if what == "c" else 8e-3
        _close(a, c.double(), tol, tol, f"rowln split vs single {what} M{M} N{N} K{K}")
    v = x.double() @ w.double().t() + b.double() + r.double()
    ln = (v - v.mean(1, keepdim=True)) / torch.sqrt(v.var(1, unbiased=False, keepdim=True) + 1e-6)
    _close(outs[0][0], v if raw else ln, 1e-4, 1e-4, "rowln split vs f64")


@pytest.mark.parametrize("dt_in,dt_out", [(torch.float32, torch.bfloat16), (torch.float32, torch.float32),
                                          (torch.bfloat16, torch.float32)])
@pytest.mark.parametrize("rows,cols", [(4096 * 16, 384), (3, 4), (5, 6)])
def test_add_rows_elementwise(dt_in, dt_out, rows, cols):
    """comet_add_rows with period == rows (the update formers' tokens + init before the flow head,
    round 5: the 4-wide elementwise path when aligned, the generic path otherwise) equals torch's f32
    sum rounded once to the output dtype."""
    ops = _ops()
    g = torch.Generator().manual_seed(rows + cols)
    x = torch.randn(rows, cols, generator=g).to(dt_in).to(DEV)
    t = torch.randn(rows, cols, generator=g).to(DEV)
    y = ops.add_rows(x, t, period=rows, out_dtype=dt_out)
    ref = (x.float() + t).to(dt_out)
    assert y.dtype == dt_out and torch.equal(y, ref)
