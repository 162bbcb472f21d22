"""Transformer / CNN building blocks of the COMET hot path (mirror of comet/models/modules.py).

Parameter names and shapes match the reference exactly (state_dict drop-in); forward and
backward run through comet_amd.functional (libcomet_hip.so). Residual streams are f32.

  Mlp            modules.py:119-154   fc1 -> GELU(erf) -> fc2
  AttnBlock      modules.py:248-295   x = LN(x); x = x + MHA(x); x = x + Mlp(LN(x))
  CrossAttnBlock modules.py:298-344   same with ctx = LN_affine(ctx, eps 1e-5)
  ResidualBlock  modules.py:39-116    conv3x3-IN-ReLU x2 (+ 1x1 s2 downsample), NHWC
"""

import torch
import torch.nn as nn

from .. import _lib as L
from .. import functional as F
from .. import ops


class Mlp(nn.Module):
    def __init__(self, in_features, hidden_features=None, out_features=None, act_layer=nn.GELU,
                 norm_layer=None, bias=True, drop=0.0, use_conv=False):
        super().__init__()
        out_features = out_features or in_features
        hidden_features = hidden_features or in_features
        self.fc1 = nn.Linear(in_features, hidden_features, bias=bias)
        self.act = act_layer()
        self.drop1 = nn.Dropout(drop)
        self.fc2 = nn.Linear(hidden_features, out_features, bias=bias)
        self.drop2 = nn.Dropout(drop)

    def forward(self, x, resid=None, out_dtype=torch.float32):
        return F.mlp(x, self.fc1.weight, self.fc1.bias, self.fc2.weight, self.fc2.bias, resid=resid, out_dtype=out_dtype)


def _mha_holder(C, heads):
    """nn.MultiheadAttention used only as the parameter container (in_proj_weight [3C, C],
    in_proj_bias, out_proj.{weight,bias}) so checkpoints load unchanged."""
    return nn.MultiheadAttention(embed_dim=C, num_heads=heads, batch_first=True)


class AttnBlock(nn.Module):
    def __init__(self, hidden_size, num_heads, attn_class=nn.MultiheadAttention, mlp_ratio=4.0, **kw):
        super().__init__()
        self.norm1 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.norm2 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.attn = _mha_holder(hidden_size, num_heads)
        self.mlp = Mlp(in_features=hidden_size, hidden_features=int(hidden_size * mlp_ratio), drop=0)
        self.heads = num_heads

    def forward(self, x, mask=None):
        C = x.shape[-1]
        a = self.attn
        x, xc = F.layer_norm_dual(x, eps=1e-6)  # residual is the normed x (modules.py:290)
        qkv = F.linear(xc, a.in_proj_weight, a.in_proj_bias)
        o = F.attention(qkv, None, self.heads, C)
        x = F.linear(o, a.out_proj.weight, a.out_proj.bias, resid=x, out_dtype=torch.float32)
        xr, xn = F.res_layer_norm(x, eps=1e-6)
        return self.mlp(xn, resid=xr)


def _res_ln(x, w, b, resid, raw=True, y16_eps=None, z=None):
    """No-grad residual Linear whose consumers are LayerNorms: (c, y16, z16) as ops.linear_rowln
    (one kernel with the LayerNorms in its epilogue when eligible; otherwise the GEMM and the
    LayerNorm kernels separately, same outputs). y16 / z16 are in the compute dtype."""
    wc = F.wcast(w)
    xc = x if x.dtype == wc.dtype else ops.cast(x, wc.dtype)
    if ops.linear_rowln_ok(xc, wc, resid, bias=b, z=z):
        return ops.linear_rowln(xc, wc, b, resid, raw=raw, y16_eps=y16_eps, z=z)
    cdt = F.compute_dtype()
    c = ops.linear(xc, wc, bias=b, resid=resid, out_dtype=torch.float32)
    y16 = z16 = None
    if z is not None:
        z16 = ops.layernorm(c, z[0], z[1], eps=z[2], out_dtype=cdt)
    if not raw:
        if cdt == torch.bfloat16:
            c, y16 = ops.layernorm(c, eps=y16_eps, out_dtype=torch.float32, dual=True)
        else:
            c = y16 = ops.layernorm(c, eps=y16_eps, out_dtype=torch.float32)
    elif y16_eps is not None:
        y16 = ops.layernorm(c, eps=y16_eps, out_dtype=cdt)
    return c, y16, z16


def norm1_dual(x):
    """(f32, compute dtype) copies of the non-affine LN (eps 1e-6) that opens AttnBlock /
    CrossAttnBlock: the f32 copy is the block's residual (modules.py:290)."""
    return F.layer_norm_dual(x, eps=1e-6)


DUAL = dict(raw=False, y16_eps=1e-6)  # output consumed by the next block's norm1


def dual_ctx(cross_blk):
    """Output consumed by a block's norm1 and by `cross_blk`'s norm_context (affine, eps 1e-5)."""
    n = cross_blk.norm_context
    return dict(raw=False, y16_eps=1e-6, z=(n.weight, n.bias, n.eps))


def _mlp_pre(blk, a, o, x32, out):
    # x = x + out_proj(o); x = x + mlp(norm2(x)): norm2 is written by the out_proj epilogue
    h32, h16, _ = _res_ln(o, a.out_proj.weight, a.out_proj.bias, x32, raw=True, y16_eps=1e-6)
    m = blk.mlp
    hid = F.linear(h16, m.fc1.weight, m.fc1.bias, act=L.ACT_GELU)
    return _res_ln(hid, m.fc2.weight, m.fc2.bias, h32, **out)


@torch.no_grad()
def attn_block_pre(blk, pre, out):
    """AttnBlock forward (no grad: the tracker) from its norm1 outputs pre = (x32, x16); the
    output LayerNorms the consumers need are written per `out` (see _res_ln)."""
    x32, x16 = pre
    a = blk.attn
    qkv = F.linear(x16, a.in_proj_weight, a.in_proj_bias)
    o = F.attention(qkv, None, blk.heads, x32.shape[-1])
    return _mlp_pre(blk, a, o, x32, out)


@torch.no_grad()
def cross_block_pre(blk, pre, ctx16, out):
    """CrossAttnBlock forward (no grad) from norm1(x) = pre and norm_context(context) = ctx16."""
    x32, x16 = pre
    C = x32.shape[-1]
    a = blk.cross_attn
    W, b = a.in_proj_weight, a.in_proj_bias
    q = F.linear(x16, W[:C], b[:C])
    kv = F.linear(ctx16, W[C:], b[C:])
    o = F.attention(q, kv, blk.heads, C)
    return _mlp_pre(blk, a, o, x32, out)


class CrossAttnBlock(nn.Module):
    def __init__(self, hidden_size, context_dim, num_heads=1, mlp_ratio=4.0, **kw):
        super().__init__()
        self.norm1 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.norm_context = nn.LayerNorm(hidden_size)
        self.norm2 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.cross_attn = _mha_holder(hidden_size, num_heads)
        self.mlp = Mlp(in_features=hidden_size, hidden_features=int(hidden_size * mlp_ratio), drop=0)
        self.heads = num_heads

    def forward(self, x, context, mask=None):
        C = x.shape[-1]
        a = self.cross_attn
        x, xc = F.layer_norm_dual(x, eps=1e-6)
        ctx = F.layer_norm(context, self.norm_context.weight, self.norm_context.bias, eps=1e-5,
                           out_dtype=F.compute_dtype())
        q, kv = F.linear_pair(xc, ctx, a.in_proj_weight, a.in_proj_bias, C)
        o = F.attention(q, kv, self.heads, C)
        x = F.linear(o, a.out_proj.weight, a.out_proj.bias, resid=x, out_dtype=torch.float32)
        xr, xn = F.res_layer_norm(x, eps=1e-6)
        return self.mlp(xn, resid=xr)


# ------------------------------------------------------------------------------------------
# CNN blocks (no-grad, NHWC activations in the compute dtype)
# ------------------------------------------------------------------------------------------
def conv2d_nhwc(x, conv, stride, pad, out_dtype=None):
    """nn.Conv2d on NHWC x via im2col + MFMA GEMM. conv.weight [Cout, Cin, kh, kw]."""
    w = conv.weight
    cout, cin, kh, kw = w.shape
    cx = x.shape[-1]  # may exceed cin: RGB inputs zero-padded to 8 channels for the implicit GEMM
    wm = F.wcast_conv(w, cin_pad=cx)
    if kh == 1 and kw == 1 and stride == 1 and pad == 0:
        n, h, wd, c = x.shape
        y = F.linear(x.reshape(-1, c), wm, conv.bias, out_dtype=out_dtype)
        return y.reshape(n, h, wd, cout)
    xc = x if x.dtype == wm.dtype else ops.cast(x, wm.dtype)
    if wm.dtype == torch.bfloat16 and cx % 8 == 0:  # implicit GEMM: no im2col matrix in HBM
        return ops.conv2d_nhwc(xc, wm, kh, kw, stride, pad, bias=conv.bias, out_dtype=out_dtype or wm.dtype)
    cols, oh, ow = ops.im2col_nhwc(xc, kh, kw, stride, pad, out_dtype=wm.dtype, ldc=wm.shape[1])
    y = F.linear(cols, wm, conv.bias, out_dtype=out_dtype)
    return y.reshape(x.shape[0], oh, ow, cout)


class ResidualBlock(nn.Module):
    def __init__(self, in_planes, planes, norm_fn="group", stride=1, kernel_size=3):
        super().__init__()
        if norm_fn != "instance":
            raise NotImplementedError("the COMET path only uses norm_fn='instance'")
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=kernel_size, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=kernel_size, padding=1)
        self.relu = nn.ReLU(inplace=True)
        self.norm1 = nn.InstanceNorm2d(planes)
        self.norm2 = nn.InstanceNorm2d(planes)
        self.stride = stride
        if stride != 1:
            self.norm3 = nn.InstanceNorm2d(planes)
            self.downsample = nn.Sequential(nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm3)
        else:
            self.downsample = None

    def forward(self, x):
        """x NHWC -> relu(x' + relu(IN(conv2(relu(IN(conv1(x)))))))."""
        y = ops.instnorm_nhwc(conv2d_nhwc(x, self.conv1, self.stride, 1), relu=True)
        y = conv2d_nhwc(y, self.conv2, 1, 1)
        if self.downsample is not None:
            xd = ops.instnorm_nhwc(conv2d_nhwc(x, self.downsample[0], self.stride, 0))
        else:
            xd = x
        # relu(x' + relu(IN(y))) in one pass
        return ops.instnorm_nhwc(y, res=xd, relu=True, relu_inner=True)
