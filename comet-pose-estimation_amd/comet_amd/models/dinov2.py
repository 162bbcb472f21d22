"""DINOv2 ViT-B/14 with 4 register tokens (the frozen backbone of camera_predictor10.py:601-617,
fetched there with torch.hub "facebookresearch/dinov2", "dinov2_vitb14_reg").

Parameter names follow facebookresearch DINOv2 so reference checkpoints load unchanged
(camera_predictor.backbone.{cls_token, pos_embed, register_tokens, mask_token,
patch_embed.proj, blocks.i.{norm1, attn.qkv, attn.proj, ls1.gamma, norm2, mlp.fc1, mlp.fc2,
ls2.gamma}, norm}). The backbone is frozen and always runs under no_grad, so its derived
operands are prepared once per weight load and cached:
  * patch-embed weight as a K-padded GEMM operand; the ImageNet normalisation + resize to
    336 + patchify is one kernel (comet_dino_prep) and the patch GEMM writes the token rows
    with bias + interpolated position table fused in its epilogue;
  * LayerScale gammas folded into attn.proj / mlp.fc2 (diag(gamma) W, gamma * b).
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as TF

from .. import _lib as L
from .. import functional as F
from .. import ops


class _PatchEmbed(nn.Module):
    def __init__(self, patch, dim):
        super().__init__()
        self.proj = nn.Conv2d(3, dim, kernel_size=patch, stride=patch)


class _LayerScale(nn.Module):
    def __init__(self, dim, init=1e-5):
        super().__init__()
        self.gamma = nn.Parameter(init * torch.ones(dim))


class _Attn(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.qkv = nn.Linear(dim, 3 * dim, bias=True)
        self.proj = nn.Linear(dim, dim, bias=True)


class _Mlp(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.fc1 = nn.Linear(dim, hidden)
        self.fc2 = nn.Linear(hidden, dim)


class _Block(nn.Module):
    def __init__(self, dim, hidden):
        super().__init__()
        self.norm1 = nn.LayerNorm(dim, eps=1e-6)
        self.attn = _Attn(dim)
        self.ls1 = _LayerScale(dim)
        self.norm2 = nn.LayerNorm(dim, eps=1e-6)
        self.mlp = _Mlp(dim, hidden)
        self.ls2 = _LayerScale(dim)


class DinoVisionTransformer(nn.Module):
    def __init__(self, img_size=518, patch_size=14, embed_dim=768, depth=12, num_heads=12, mlp_ratio=4.0,
                 num_register_tokens=4):
        super().__init__()
        self.patch_size = patch_size
        self.embed_dim = embed_dim
        self.num_heads = num_heads
        self.num_register_tokens = num_register_tokens
        n = (img_size // patch_size) ** 2
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, n + 1, embed_dim))
        self.register_tokens = nn.Parameter(torch.zeros(1, num_register_tokens, embed_dim))
        self.mask_token = nn.Parameter(torch.zeros(1, embed_dim))
        self.patch_embed = _PatchEmbed(patch_size, embed_dim)
        self.blocks = nn.ModuleList([_Block(embed_dim, int(embed_dim * mlp_ratio)) for _ in range(depth)])
        self.norm = nn.LayerNorm(embed_dim, eps=1e-6)
        nn.init.trunc_normal_(self.pos_embed, std=0.02)
        nn.init.normal_(self.cls_token, std=1e-6)
        nn.init.normal_(self.register_tokens, std=1e-6)
        self._prep = None
        self._register_load_state_dict_pre_hook(lambda *a, **k: self.invalidate())

    def invalidate(self):
        self._prep = None

    def _apply(self, fn, *args, **kwargs):
        self._prep = None
        return super()._apply(fn, *args, **kwargs)

    # ---- one-time operand preparation (frozen weights) ----
    def _prepared(self, grid, dtype):
        key = (grid, dtype, self.cls_token.data_ptr())
        if self._prep is not None and self._prep["key"] == key:
            return self._prep
        with torch.no_grad():
            C = self.embed_dim
            p = self.patch_size
            K = 3 * p * p
            Kp = (K + 7) // 8 * 8
            wpe = torch.zeros(C, Kp, device=self.cls_token.device, dtype=dtype)
            wpe[:, :K] = self.patch_embed.proj.weight.reshape(C, K).to(dtype)
            pos = self.pos_embed.float()
            M = int(math.sqrt(pos.shape[1] - 1))
            if M == grid:
                patch_pos = pos[0, 1:]
            else:  # interpolate_pos_encoding: bicubic, antialias=True, size=(grid, grid)
                pp = pos[:, 1:].reshape(1, M, M, C).permute(0, 3, 1, 2)
                pp = TF.interpolate(pp, size=(grid, grid), mode="bicubic", antialias=True, align_corners=False)
                patch_pos = pp.permute(0, 2, 3, 1).reshape(grid * grid, C)
            head = torch.cat([self.cls_token[0].float() + pos[0, :1], self.register_tokens[0].float()], 0)
            blocks = []
            for b in self.blocks:
                g1, g2 = b.ls1.gamma.float(), b.ls2.gamma.float()
                blocks.append(dict(
                    wproj=(b.attn.proj.weight.float() * g1[:, None]).to(dtype).contiguous(),
                    bproj=(b.attn.proj.bias.float() * g1).contiguous(),
                    wfc2=(b.mlp.fc2.weight.float() * g2[:, None]).to(dtype).contiguous(),
                    bfc2=(b.mlp.fc2.bias.float() * g2).contiguous(),
                    wqkv=b.attn.qkv.weight.to(dtype).contiguous(),
                    wfc1=b.mlp.fc1.weight.to(dtype).contiguous(),
                ))
            mean = torch.tensor([0.485, 0.456, 0.406], device=wpe.device)
            std = torch.tensor([0.229, 0.224, 0.225], device=wpe.device)
            self._prep = dict(key=key, wpe=wpe, Kp=Kp, pos=patch_pos.contiguous(), head=head.contiguous(),
                              blocks=blocks, mean=mean, std=std)
        return self._prep

    @torch.no_grad()
    def forward(self, images, is_training=True, down_size=336):
        """images [BS, 3, H, W] f32 (dataset-normalised frames) -> {"x_norm_patchtokens": [BS, g*g, C]}.
        Includes camera_predictor10.py:624-634 (resize to down_size, second ImageNet normalisation)."""
        dtype = F.compute_dtype()
        BS = images.shape[0]
        p = self.patch_size
        g = down_size // p
        P = g * g
        C = self.embed_dim
        nh = 1 + self.num_register_tokens
        Lt = nh + P
        prep = self._prepared(g, dtype)
        cols = ops.dino_prep(images, down_size, p, prep["Kp"], prep["mean"], prep["std"], dtype)
        x = torch.empty(BS, Lt, C, device=images.device, dtype=torch.float32)
        x[:, :nh] = prep["head"]
        # patch rows: x[:, nh:] = cols @ Wpe^T + b + pos   (one batched GEMM, fused epilogue)
        ops.gemm_raw(cols, prep["wpe"], x[:, nh:], m=P, n=C, k=prep["Kp"], layout_a=0, lda=prep["Kp"], layout_b=0,
                     ldb=prep["Kp"], ldc=C, batch=(BS, 1), stride_a=(P * prep["Kp"], 0), stride_c=(Lt * C, 0),
                     bias=self.patch_embed.proj.bias, bias_mode=1, resid=prep["pos"], ldr=C, stride_r=(0, 0))
        for blk, bp in zip(self.blocks, prep["blocks"]):
            h = ops.layernorm(x, blk.norm1.weight, blk.norm1.bias, eps=1e-6, out_dtype=dtype)
            qkv = ops.linear(h, bp["wqkv"], bias=blk.attn.qkv.bias)
            o = ops.attention(qkv[..., :C], qkv[..., C:2 * C], qkv[..., 2 * C:], self.num_heads)
            x = ops.linear(o, bp["wproj"], bias=bp["bproj"], resid=x, out_dtype=torch.float32)
            h = ops.layernorm(x, blk.norm2.weight, blk.norm2.bias, eps=1e-6, out_dtype=dtype)
            h = ops.linear(h, bp["wfc1"], bias=blk.mlp.fc1.bias, act=L.ACT_GELU)
            x = ops.linear(h, bp["wfc2"], bias=bp["bfc2"], resid=x, out_dtype=torch.float32)
        xn = ops.layernorm(x[:, nh:], self.norm.weight, self.norm.bias, eps=1e-6, out_dtype=torch.float32)
        return {"x_norm_patchtokens": xn}


def dinov2_vitb14_reg():
    return DinoVisionTransformer(img_size=518, patch_size=14, embed_dim=768, depth=12, num_heads=12,
                                 num_register_tokens=4)
