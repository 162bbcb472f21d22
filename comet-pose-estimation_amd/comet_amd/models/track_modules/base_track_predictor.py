"""BaseTrackerPredictor (mirror of comet/models/track_modules/base_track_predictor.py).

Iterative CoTracker-style refinement (base_track_predictor.py:95-284), forward-only (the tracker
runs under no_grad). Per iteration, on libcomet_hip.so:
  comet_corr_sample     CorrBlock.corr + .sample fused over the avg-pool pyramid (no [B,S,N,H,W]
                        correlation volume is materialised)
  comet_tracker_tokens  [flow sin/cos embedding | flows | corr | track feats | pad] + sampled
                        2-D sincos position embedding, written in the compute dtype
  EfficientUpdateFormer (MFMA GEMMs + flash attention)
  GroupNorm(1) -> Linear -> GELU -> + track feats (LN kernel + fused GEMM epilogue)
  comet_coords_update   coords += delta (frame 0 pinned), per-iteration predictions
Track state is kept as [B, N, S, .] (the update-former layout) instead of [B, S, N, .].
"""
import torch
import torch.nn as nn

from ... import _lib as L
from ... import functional as F
from ... import ops
from .blocks import EfficientUpdateFormer


class BaseTrackerPredictor(nn.Module):
    def __init__(self, stride=4, corr_levels=5, corr_radius=4, latent_dim=128, hidden_size=384, use_spaceatt=True,
                 depth=6, fine=False, cfg=None):
        super().__init__()
        self.cfg = cfg
        self.stride = stride
        self.latent_dim = latent_dim
        self.corr_levels = corr_levels
        self.corr_radius = corr_radius
        self.hidden_size = hidden_size
        self.fine = fine
        self.flows_emb_dim = latent_dim // 2
        self.transformer_dim = corr_levels * (corr_radius * 2 + 1) ** 2 + latent_dim * 2
        if fine:
            self.transformer_dim += 4 if self.transformer_dim % 2 == 0 else 5
        else:
            self.transformer_dim += (4 - self.transformer_dim % 4) % 4
        space_depth = depth if use_spaceatt else 0
        self.updateformer = EfficientUpdateFormer(space_depth=space_depth, time_depth=depth,
                                                  input_dim=self.transformer_dim, hidden_size=self.hidden_size,
                                                  output_dim=self.latent_dim + 2, mlp_ratio=4.0,
                                                  add_space_attn=use_spaceatt)
        self.norm = nn.GroupNorm(1, self.latent_dim)
        self.ffeat_updater = nn.Sequential(nn.Linear(self.latent_dim, self.latent_dim), nn.GELU())
        track_conf = _get(cfg, "track_conf", False)
        if track_conf:
            self.conf_predictor = nn.Sequential(nn.Linear(self.latent_dim, 1))
        if not self.fine:
            self.vis_predictor = nn.Sequential(nn.Linear(self.latent_dim, 1))
        self._pos = {}

    def _pos_table(self, HH, WW, device):
        key = (HH, WW, device)
        t = self._pos.get(key)
        if t is None:
            t = ops.sincos_2d(self.transformer_dim, HH, WW, device).reshape(1, HH, WW, self.transformer_dim)
            self._pos[key] = t
        return t

    @torch.no_grad()
    def forward(self, query_points, fmaps=None, iters=4, return_feat=False, down_ratio=1, is_train=False,
                track_feats=None, TRACKorPOSE=False, ind=0, pyramid1=None, pyramid2=None):
        """query_points [B, N, 2]; fmaps NHWC [B, S, HH, WW, C] (compute dtype).
        Returns (coord_preds list of [B, S, N, 2], vis [B, S, N] or None, track_feats [B, N, S, C],
        query_track_feat [B, N, C], conf None)."""
        B, N, _ = query_points.shape
        _, S, HH, WW, C = fmaps.shape
        dev = fmaps.device
        q = query_points.float()
        if down_ratio > 1:
            q = q / float(down_ratio)
            q = q / float(self.stride)
        coords = q.reshape(B, N, 1, 2).repeat(1, 1, S, 1).contiguous()  # [B, N, S, 2]
        fm0 = fmaps[:, 0]
        query_feat = ops.sample_bilinear(fm0, q, border=True)  # [B, N, C]
        track_feats = query_feat.reshape(B, N, 1, C).repeat(1, 1, S, 1).contiguous()  # f32 [B, N, S, C]
        pyr = [fmaps.reshape(B * S, HH, WW, C)]
        if pyramid1 is not None and self.corr_levels > 1:  # levels 1 (and 2) already pooled by the producer
            pyr.append(pyramid1)
            if pyramid2 is not None and self.corr_levels > 2:
                pyr.append(pyramid2)
        while len(pyr) < self.corr_levels:
            pyr.append(ops.avgpool2_nhwc(pyr[-1]))
        pos = ops.sample_bilinear(self._pos_table(HH, WW, dev).expand(B, -1, -1, -1), q, border=True)  # [B, N, tdim]
        td = self.transformer_dim
        win = (2 * self.corr_radius + 1) ** 2
        corrdim = self.corr_levels * win
        rows = B * N * S
        corr = torch.empty(rows, corrdim, device=dev, dtype=torch.float32)
        # bf16 tokens: rows padded with zeros to a 64-column multiple (664 -> 704, 216 -> 256), so the
        # update former's input GEMM takes the persistent kernel; the products and sums are unchanged
        tdp = (td + 63) // 64 * 64 if F.compute_dtype() == torch.bfloat16 else td
        x = torch.empty(rows, tdp, device=dev, dtype=F.compute_dtype())
        scale = self.stride * down_ratio if down_ratio > 1 else self.stride
        preds = []
        lat = self.latent_dim
        for _ in range(iters):
            ops.corr_sample(pyr, self.corr_radius, track_feats.reshape(rows, C), coords.reshape(rows, 2), corr, 0, B, N, S)
            ops.tracker_tokens(coords, track_feats, lat, corr, corrdim, pos, td, x, rows, S)
            delta = self.updateformer(x.reshape(B, N, S, tdp)).reshape(rows, lat + 2)
            g = ops.layernorm(delta[:, 2:], self.norm.weight, self.norm.bias, eps=self.norm.eps,
                              out_dtype=torch.float32)
            track_feats = _ffeat(g, self.ffeat_updater[0], track_feats.reshape(rows, lat)).reshape(B, N, S, lat)
            pr = torch.empty(B, S, N, 2, device=dev, dtype=torch.float32)
            ops.coords_update(coords, delta, pr, scale, B, N, S)
            preds.append(pr)
        vis = None
        if not self.fine:
            v = F.linear(track_feats.reshape(rows, lat), self.vis_predictor[0].weight, self.vis_predictor[0].bias,
                         act=L.ACT_SIGMOID, out_dtype=torch.float32)
            vis = v.reshape(B, N, S).permute(0, 2, 1)
        if return_feat:
            return preds, vis, track_feats, query_feat, None
        return preds, vis, None


def _ffeat(g, lin, tf):
    """track_feats += GELU(Linear(GroupNorm(delta_feats))) (base_track_predictor.py:237-239)."""
    return F.linear(g, lin.weight, lin.bias, act=L.ACT_GELU, resid=tf, out_dtype=torch.float32)


def _get(cfg, key, default):
    if cfg is None:
        return default
    if hasattr(cfg, "get"):
        return cfg.get(key, default)
    return getattr(cfg, key, default)
