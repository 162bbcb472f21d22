"""Tracker building blocks (mirror of comet/models/track_modules/blocks.py) on libcomet_hip.so.

The tracker is frozen and always runs under no_grad (E2Epose2.py:176), so these modules are
forward-only. Activations are channels-last (NHWC) in the compute dtype; convolutions are
im2col + MFMA GEMM, InstanceNorm/ReLU/residual tails are fused kernels.

  BasicEncoder   blocks.py:27-111   coarse feature net -> [B*S, H/8, W/8, 128]
  ShallowEncoder blocks.py:114-196  fine patch feature net -> [n, 31, 31, 32]
  EfficientUpdateFormer blocks.py:205-348 (time / virtual-track space attention)
"""

import torch
import torch.nn as nn

from ... import functional as F
from ... import ops
from ..modules import (DUAL, AttnBlock, CrossAttnBlock, ResidualBlock, attn_block_pre, conv2d_nhwc,
                       cross_block_pre, dual_ctx, norm1_dual)


class BasicEncoder(nn.Module):
    def __init__(self, input_dim=3, output_dim=128, stride=4, use_trans=False, cfg=None):
        super().__init__()
        self.stride = stride
        self.norm_fn = "instance"
        self.in_planes = output_dim // 2
        self.norm1 = nn.InstanceNorm2d(self.in_planes)
        self.norm2 = nn.InstanceNorm2d(output_dim * 2)
        self.conv1 = nn.Conv2d(input_dim, self.in_planes, kernel_size=7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.layer1 = self._make_layer(output_dim // 2, stride=1)
        self.layer2 = self._make_layer(output_dim // 4 * 3, stride=2)
        self.layer3 = self._make_layer(output_dim, stride=2)
        self.layer4 = self._make_layer(output_dim, stride=2)
        self.conv2 = nn.Conv2d(output_dim * 3 + output_dim // 4, output_dim * 2, kernel_size=3, padding=1)
        self.relu2 = nn.ReLU(inplace=True)
        self.conv3 = nn.Conv2d(output_dim * 2, output_dim, kernel_size=1)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def _make_layer(self, dim, stride=1):
        layer1 = ResidualBlock(self.in_planes, dim, self.norm_fn, stride=stride)
        layer2 = ResidualBlock(dim, dim, self.norm_fn, stride=1)
        self.in_planes = dim
        return nn.Sequential(layer1, layer2)

    @torch.no_grad()
    def forward(self, x, H, W):
        """x NHWC [n, H, W, 3] (compute dtype) -> fmaps NHWC [n, H/stride, W/stride, 128]."""
        x = ops.instnorm_nhwc(conv2d_nhwc(x, self.conv1, 2, 3), relu=True)
        a = self.layer1(x)
        b = self.layer2(a)
        c = self.layer3(b)
        d = self.layer4(c)
        oh, ow = H // self.stride, W // self.stride
        # the four up-sampled maps are written straight into their concat channel slices
        parts = (a, b, c, d)
        x = torch.empty(a.shape[0], oh, ow, sum(t.shape[-1] for t in parts), device=a.device, dtype=a.dtype)
        c0 = 0
        for t in parts:
            ops.resize_bilinear_into(t, x[..., c0:c0 + t.shape[-1]])
            c0 += t.shape[-1]
        x = ops.instnorm_nhwc(conv2d_nhwc(x, self.conv2, 1, 1), relu=True)
        return conv2d_nhwc(x, self.conv3, 1, 0)


class ShallowEncoder(nn.Module):
    def __init__(self, input_dim=3, output_dim=32, stride=1, norm_fn="instance", cfg=None):
        super().__init__()
        self.stride = stride
        self.norm_fn = norm_fn
        self.in_planes = output_dim
        self.norm1 = nn.InstanceNorm2d(self.in_planes)
        self.norm2 = nn.InstanceNorm2d(output_dim * 2)
        self.conv1 = nn.Conv2d(input_dim, self.in_planes, kernel_size=3, stride=2, padding=1)
        self.relu1 = nn.ReLU(inplace=True)
        self.layer1 = self._make_layer(output_dim, stride=2)
        self.layer2 = self._make_layer(output_dim, stride=2)
        self.conv2 = nn.Conv2d(output_dim, output_dim, kernel_size=1)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")

    def _make_layer(self, dim, stride=1):
        self.in_planes = dim
        return ResidualBlock(self.in_planes, dim, self.norm_fn, stride=stride)

    @torch.no_grad()
    def forward(self, x, with_pool=False):
        """x NHWC [n, P, P, 3] -> NHWC [n, P/stride, P/stride, 32] (with_pool: also its 2x2 average
        pool, the fine correlation pyramid's level 1, and with with_pool=2 that pool's pool, level 2:
        the resize-and-adds, conv2, the residual, the up-sampling and the pools in one kernel,
        comet_conv1x1_resize_pool_nhwc)."""
        _, H, W, _ = x.shape
        x = ops.instnorm_nhwc(conv2d_nhwc(x, self.conv1, 2, 1), relu=True)
        h, w = x.shape[1], x.shape[2]
        n, _, _, c = x.shape
        oh, ow = H // self.stride, W // self.stride
        w2 = F.wcast(self.conv2.weight.reshape(c, c))
        tmp1 = self.layer1(x)
        tmp2 = self.layer2(tmp1)  # (layer2 reads layer1's output, not x: the two adds below can wait)
        if with_pool and ops.conv1x1_resize_pool_ok(x, w2, self.conv2.bias, tmp1, tmp2):
            # both resize-and-adds, conv2 (1x1) + residual, the up-sampling and the pyramid's pools
            # in one kernel (the sums and the conv2 output never in HBM)
            return ops.conv1x1_resize_pool(x, w2, self.conv2.bias, oh, ow, up1=tmp1, up2=tmp2, pool2=with_pool == 2)
        x = ops.resize_bilinear(tmp1, h, w, nhwc=True, out=x, add=True)
        x = ops.resize_bilinear(tmp2, h, w, nhwc=True, out=x, add=True)
        x = F.linear(x.reshape(-1, c), w2, self.conv2.bias, resid=x.reshape(-1, c), out_dtype=x.dtype).reshape(n, h, w, c)
        if with_pool:
            if ops.resize_pool_ok(x):
                y, p = ops.resize_bilinear_pool(x, oh, ow)
            else:
                y = ops.resize_bilinear(x, oh, ow, nhwc=True)
                p = ops.avgpool2_nhwc(y)
            return (y, p, ops.avgpool2_nhwc(p)) if with_pool == 2 else (y, p)
        return ops.resize_bilinear(x, oh, ow, nhwc=True)


class EfficientUpdateFormer(nn.Module):
    def __init__(self, space_depth=6, time_depth=6, input_dim=320, hidden_size=384, num_heads=8, output_dim=130,
                 mlp_ratio=4.0, add_space_attn=True, num_virtual_tracks=64):
        super().__init__()
        self.out_channels = 2
        self.num_heads = num_heads
        self.hidden_size = hidden_size
        self.add_space_attn = add_space_attn
        self.input_transform = torch.nn.Linear(input_dim, hidden_size, bias=True)
        self.flow_head = torch.nn.Linear(hidden_size, output_dim, bias=True)
        self.num_virtual_tracks = num_virtual_tracks
        self.virual_tracks = nn.Parameter(torch.randn(1, num_virtual_tracks, 1, hidden_size)) if add_space_attn else None
        self.time_blocks = nn.ModuleList([AttnBlock(hidden_size, num_heads, mlp_ratio=mlp_ratio) for _ in range(time_depth)])
        if add_space_attn:
            self.space_virtual_blocks = nn.ModuleList(
                [AttnBlock(hidden_size, num_heads, mlp_ratio=mlp_ratio) for _ in range(space_depth)])
            self.space_point2virtual_blocks = nn.ModuleList(
                [CrossAttnBlock(hidden_size, hidden_size, num_heads, mlp_ratio=mlp_ratio) for _ in range(space_depth)])
            self.space_virtual2point_blocks = nn.ModuleList(
                [CrossAttnBlock(hidden_size, hidden_size, num_heads, mlp_ratio=mlp_ratio) for _ in range(space_depth)])
        for m in self.modules():
            if isinstance(m, nn.Linear):
                torch.nn.init.xavier_uniform_(m.weight)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    @torch.no_grad()
    def forward(self, input_tensor, mask=None):
        """input [B, N, T, Din] (compute dtype) -> [B, N, T, Dout] f32.

        The reference concatenates the virtual tracks to the point tracks and permutes
        [B, N, T, C] <-> [B*T, N, C] around every space block (blocks.py:300-345). Here point and
        virtual tokens live in two [B, n, T, C] tensors: the time blocks are per-track (run on
        each), the space blocks attend over the track axis of the 4-D tensors directly (inner-batch
        attention over (b, t)), so no cat / permute copies are made."""
        B, N0, T, _ = input_tensor.shape
        C = self.hidden_size
        w_in = self.input_transform.weight
        if input_tensor.shape[-1] != w_in.shape[1]:  # tokens padded with zero columns to a k-tile multiple
            w_in = F.wcast_kpad(w_in, input_tensor.shape[-1])
        init = F.linear(input_tensor, w_in, self.input_transform.bias, out_dtype=torch.float32)
        # every block below starts with a LayerNorm of its input; except for the first ones, those
        # LayerNorms are written by the epilogue of the GEMM that produces the input (the output
        # specs name the consumers), so the token streams move as norm1 pairs (f32, bf16)
        pts = norm1_dual(init.reshape(B * N0, T, C))
        vts = None
        if self.add_space_attn:
            vts = norm1_dual(self.virual_tracks.detach().float().expand(B, -1, T, -1).reshape(-1, T, C).contiguous())
        Nv = self.num_virtual_tracks if self.add_space_attn else 0
        j = 0
        space_every = len(self.time_blocks) // len(self.space_virtual_blocks) if self.add_space_attn else 0
        nl = len(self.time_blocks)
        for i in range(nl):
            blk = self.time_blocks[i]
            space = self.add_space_attn and i % space_every == 0
            last = i == nl - 1
            if space:
                v2p, vself, p2v = (self.space_virtual2point_blocks[j], self.space_virtual_blocks[j],
                                   self.space_point2virtual_blocks[j])
                # time block on the point tracks: its output is norm1 of point<-virtual and the
                # context of virtual<-point
                p32, p16, pctx = attn_block_pre(blk, pts, dual_ctx(v2p))
                v32, v16, _ = attn_block_pre(blk, vts, DUAL)
                r4 = lambda t, n: t.reshape(B, n, T, C)
                v32, v16, _ = cross_block_pre(v2p, (r4(v32, Nv), r4(v16, Nv)), r4(pctx, N0), DUAL)
                v32, v16, vctx = attn_block_pre(vself, (v32, v16), dual_ctx(p2v))
                p32, p16, _ = cross_block_pre(p2v, (r4(p32, N0), r4(p16, N0)), vctx,
                                              dict(raw=True) if last else DUAL)
                pts = (p32.reshape(B * N0, T, C), None if p16 is None else p16.reshape(B * N0, T, C))
                vts = (v32.reshape(B * Nv, T, C), v16.reshape(B * Nv, T, C))
                j += 1
            else:
                p32, p16, _ = attn_block_pre(blk, pts, dict(raw=True) if last else DUAL)
                pts = (p32, p16)
                if vts is not None:
                    v32, v16, _ = attn_block_pre(blk, vts, DUAL)
                    vts = (v32, v16)
        return _flow(pts[0].reshape(B, N0, T, C), init, self.flow_head)


def _flow(tokens, init, head):
    """flow_head(tokens + init) (blocks.py:347). Without gradients in bf16 compute (the frozen
    tracker) the sum is written straight in bf16, one rounding of the f32 sum as the reference's f32
    add + autocast cast (one pass instead of an f32 add and a cast)."""
    tokens = tokens.contiguous()
    if (F.compute_dtype() == torch.bfloat16 and not torch.is_grad_enabled() and init.dtype == torch.float32
            and init.is_contiguous() and init.shape == tokens.shape):
        C = tokens.shape[-1]
        x = ops.add_rows(tokens, init.reshape(-1, C), period=tokens.numel() // C, out_dtype=torch.bfloat16)
        return F.linear(x, head.weight, head.bias, out_dtype=torch.float32)
    x = ops.add(tokens, init)
    return F.linear(x, head.weight, head.bias, out_dtype=torch.float32)
