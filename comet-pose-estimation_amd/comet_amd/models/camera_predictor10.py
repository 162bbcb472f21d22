"""CameraPredictor (mirror of comet/models/camera_predictor10.py) on libcomet_hip.so.

Same constructor signature, submodule names and parameter shapes as the reference (so
checkpoints and the abl_ours.yaml `_target_` load unchanged), including modules that the
reference builds but never executes (embed_pose, feature_fusion, motion encoders, ...): their
parameters exist (and receive no gradient), exactly as in the reference.

forward(...) follows camera_predictor10.py:288-484:
  get_2D_image_features: DINOv2 (no_grad) -> input_transform Mlp -> LN -> + 2-D sincos ->
      prepend pose_token -> 4 x {self_att per frame; cross_att frames 1.. -> frame 0} -> token 0
  T_P: traj_encoder(pixel tracks) * sigmoid-MLP(confidence) -> 4 x CrossAttnBlock(rgb <- traj)
  T_F: + 1-D sincos over the frame index -> trunk (4 x AttnBlock over frames)
  GAPR: pose_branch -> quaternion (F.normalize), fc_translation2d -> (du, dv), fc_depth -> dd,
      pose loss vs camera_to_pose_encoding2(gt), frame-0 reset, pose_encoding_to_camera2.
B > 1: every sequence is its own reference frame; loss = mean over sequences.
"""
import math

import torch
import torch.nn as nn

from .. import _lib as L
from .. import functional as F
from .. import ops
from .dinov2 import dinov2_vitb14_reg
from .modules import AttnBlock, CrossAttnBlock, Mlp
from .utils import INTRINSICS, PredCameras

_RESNET_MEAN = [0.485, 0.456, 0.406]
_RESNET_STD = [0.229, 0.224, 0.225]


class FeatureFusion(nn.Module):
    """Built by the reference (camera_predictor10.py:40-72) but never called on the path."""

    def __init__(self, rgb_dim, fmap_dim, fusion_type="adaptive"):
        super().__init__()
        self.fusion_type = fusion_type
        self.fmap_proj = nn.Sequential(nn.Linear(fmap_dim, rgb_dim), nn.LayerNorm(rgb_dim), nn.ReLU())
        self.fusion_layer = nn.Linear(rgb_dim * 2, rgb_dim)
        self.out_norm = nn.LayerNorm(rgb_dim)


class TrajectoryEncoder(nn.Module):
    """camera_predictor10.py:75-87: LN(Linear(ReLU(LN(Linear(xy)))))."""

    def __init__(self, in_dim, hidden_dim, out_dim):
        super().__init__()
        self.mlp = nn.Sequential(nn.Linear(in_dim, hidden_dim), nn.LayerNorm(hidden_dim), nn.ReLU(inplace=True),
                                 nn.Linear(hidden_dim, out_dim), nn.LayerNorm(out_dim))

    def forward(self, traj):
        m = self.mlp
        h = F.linear(traj, m[0].weight, m[0].bias, out_dtype=torch.float32)
        h = F.layer_norm_relu(h, m[1].weight, m[1].bias, eps=m[1].eps)
        h = F.linear(h, m[3].weight, m[3].bias, out_dtype=torch.float32)
        return F.layer_norm(h, m[4].weight, m[4].bias, eps=m[4].eps)


class SimplePoseEmbedding(nn.Module):
    """utils.py:691-706 (constructed via PoseEmbedding; not executed on the path)."""

    def __init__(self, input_dim, output_dim):
        super().__init__()
        self.fc1 = nn.Linear(input_dim, output_dim // 2)
        self.act = nn.GELU()
        self.norm1 = nn.LayerNorm(output_dim // 2)
        self.fc2 = nn.Linear(output_dim // 2, output_dim)
        self.norm2 = nn.LayerNorm(output_dim)


class PoseEmbedding(nn.Module):
    def __init__(self, target_dim, n_harmonic_functions=10, append_input=True):
        super().__init__()
        self._emb_pose = SimplePoseEmbedding(input_dim=8, output_dim=768)


class CameraPredictor(nn.Module):
    # head variants of the ablation files (camera_predictor_abl_*.py subclass this and flip them)
    USE_TP = True            # T_P trajectory cross-attention runs
    TP_RESIDUAL = True       # ... and its result is added to rgb_feat (abl_track drops the add)
    USE_TIME = True          # T_F: 1-D sincos time embedding + trunk (abl_time / abl_all drop both)
    SINGLE_HEAD = False      # pose_branch -> 7 outputs with encoding 3 (abl_uvz / abl_all)

    def __init__(self, hidden_size=768, num_heads=8, mlp_ratio=4, z_dim=768, down_size=336, att_depth=4,
                 trunk_depth=4, backbone="dinov2b", pose_encoding_type="absT_quaR_OneFL", cfg=None):
        super().__init__()
        self.cfg = cfg
        self.att_depth = att_depth
        self.down_size = down_size
        self.pose_encoding_type = pose_encoding_type
        self.num_heads = num_heads
        self.target_dim = {"absT_quaR": 7, "absT_quaR_OneFL": 8, "absT_quaR_logFL": 9}[pose_encoding_type]
        self.backbone = self.get_backbone(backbone)
        for p in self.backbone.parameters():
            p.requires_grad = False
        self.input_transform = Mlp(in_features=z_dim, out_features=hidden_size, drop=0)
        self.norm1 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.norm2 = nn.LayerNorm(hidden_size, elementwise_affine=False, eps=1e-6)
        self.embed_pose = PoseEmbedding(target_dim=self.target_dim,
                                        n_harmonic_functions=int(hidden_size / self.target_dim / 2),
                                        append_input=False)
        self.pose_token = nn.Parameter(torch.zeros(1, 1, 1, hidden_size))
        self.pose_branch = Mlp(in_features=hidden_size, hidden_features=hidden_size * 2,
                               out_features=7 if self.SINGLE_HEAD else 4, drop=0)
        self.ffeat_updater = nn.Sequential(nn.Linear(hidden_size, hidden_size), nn.GELU(), nn.LayerNorm(hidden_size))
        self.self_att = nn.ModuleList([AttnBlock(hidden_size, num_heads, mlp_ratio=mlp_ratio) for _ in range(att_depth)])
        self.pose_branch_scale = nn.Parameter(torch.ones(1) * 0.1)
        self.cross_att = nn.ModuleList([CrossAttnBlock(hidden_size, hidden_size, num_heads, mlp_ratio=mlp_ratio)
                                        for _ in range(att_depth)])
        self.cross_attn_block = nn.ModuleList([CrossAttnBlock(hidden_size, hidden_size, num_heads, mlp_ratio=mlp_ratio)
                                               for _ in range(att_depth)])
        self.trunk = nn.Sequential(*[AttnBlock(hidden_size, num_heads, mlp_ratio=mlp_ratio) for _ in range(trunk_depth)])
        self.gamma = 0.8
        self.alpha = nn.Parameter(torch.tensor(0.5))
        nn.init.normal_(self.pose_token, std=1e-6)
        for name, value in (("_resnet_mean", _RESNET_MEAN), ("_resnet_std", _RESNET_STD)):
            self.register_buffer(name, torch.FloatTensor(value).view(1, 3, 1, 1), persistent=False)
        self.feature_fusion = FeatureFusion(rgb_dim=768, fmap_dim=128, fusion_type="adaptive")
        self.confidence_attention = nn.Sequential(nn.Linear(1, 32), nn.ReLU(), nn.Linear(32, 1), nn.Sigmoid())
        self.motion_weight = cfg.get("motion_weight", 0.1) if cfg is not None and hasattr(cfg, "get") else 0.1
        self.camera_motion_encoder = nn.Sequential(nn.Linear(7, 32), nn.LayerNorm(32), nn.ReLU(), nn.Linear(32, 2))
        self.motion_encoder = nn.Sequential(nn.Linear(3, 32), nn.LayerNorm(32), nn.ReLU(), nn.Linear(32, 2))
        self.traj_encoder = TrajectoryEncoder(2, 256, 768)
        self.track_context_proj = nn.Sequential(nn.Linear(128, 768), nn.GELU(), nn.LayerNorm(768))
        self.traj_encoder_norm = nn.LayerNorm(128)
        self.traj_context_norm = nn.LayerNorm(768)
        self.pose_embed_norm = nn.LayerNorm(768)
        self.pose_embed_scale = nn.Parameter(torch.ones(1) * 0.05)
        self.fc_translation2d = nn.Linear(768, 2)
        self.fc_depth = nn.Linear(768, 1)
        self._tables = {}
        # compute only the rows of the last attention layer that reach the output (same result)
        self.prune_dead_rows = True

    def get_backbone(self, backbone):
        if backbone == "dinov2b":
            return dinov2_vitb14_reg()
        raise NotImplementedError(f"Backbone '{backbone}' not implemented")

    def _cfg_get(self, key, default):
        cfg = self.cfg
        if cfg is None:
            return default
        if hasattr(cfg, "get"):
            return cfg.get(key, default)
        return getattr(cfg, key, default)

    def _table(self, kind, n, C, device):
        key = (kind, n, C, device)
        t = self._tables.get(key)
        if t is None:
            if kind == "2d":
                g = int(math.isqrt(n))
                t = ops.sincos_2d(C, g, g, device)
            else:
                t = ops.sincos_table(torch.arange(n, device=device, dtype=torch.float32), C)
            self._tables[key] = t
        return t

    # ------------------------------------------------------------------------------------
    def get_2D_image_features(self, reshaped_image, batch_size):
        """camera_predictor10.py:622-687 -> (rgb_feat [B, S, C], B, S, C)."""
        tok = self.backbone(reshaped_image, is_training=True, down_size=self.down_size)["x_norm_patchtokens"]
        tok = self.input_transform(tok)
        tok = F.layer_norm(tok, eps=1e-6)
        BS, P, C = tok.shape
        B = batch_size
        S = BS // B
        tok = F.add_rows(tok, self._table("2d", P, C, tok.device), P)
        tok = tok.reshape(B, S, P, C)
        tok = torch.cat([self.pose_token.expand(B, S, -1, -1), tok], dim=-2)
        P = P + 1
        for idx in range(self.att_depth):
            if idx == self.att_depth - 1 and S > 1 and self.prune_dead_rows:
                return self._last_layer_token0(tok, B, S, P, C), B, S, C
            tok = self.self_att[idx](tok.reshape(B * S, P, C)).reshape(B, S, P, C)
            t0, f0, fo = F.frame_split(tok)
            fo = self.cross_att[idx](fo.reshape(B, (S - 1) * P, C), f0).reshape(B, S - 1, P, C)
            tok = F.frame_join(t0, fo)
        return tok[:, :, 0].contiguous(), B, S, C

    @staticmethod
    def _query_rows(B, S, P, dev):
        """Row indices into [B*S*P] of frame 0's P rows of every sequence, then token 0 of every
        frame (the surviving query rows of _last_layer_token0)."""
        b = torch.arange(B, device=dev)
        f0 = (b[:, None] * (S * P) + torch.arange(P, device=dev)[None]).reshape(-1)
        t0 = (b[:, None] * (S * P) + torch.arange(S, device=dev)[None] * P).reshape(-1)
        return torch.cat([f0, t0])

    def _last_layer_token0(self, tok, B, S, P, C):
        """The last (self_att, cross_att) pair computing only the rows that survive (SURVEY
        Appendix B-8, camera_predictor10.py:666-687): only token 0 of every frame is returned, so
          * self_att on frames 1..S-1 needs query row 0 only (keys / values still from all P rows);
          * frame 0 keeps every row (all P are the cross-attention context);
          * cross_att needs the S-1 query rows that are token 0 of frames 1..S-1.
        Every surviving row goes through exactly the reference's per-row arithmetic (attention
        query rows, LayerNorm, out_proj, Mlp are row-independent), so the result is the same. Per sequence at
        T=16 this drops ~0.23 of the 5.15 TFLOP forward and ~0.47 of the 2.32 TFLOP backward
        (the reported GFLOP/seq stays the reference's). -> rgb_feat [B, S, C]."""
        blk, cblk = self.self_att[-1], self.cross_att[-1]
        a = blk.attn
        x = tok.reshape(B * S, P, C)
        xn, xc = F.layer_norm_dual(x, eps=1e-6)  # every row: K / V need all of them
        # query rows: frame 0 (all P) then token 0 of every frame (frame 0's again: 1 row / sequence)
        idx = self._query_rows(B, S, P, x.device)
        qin = F.gather_rows(xc.reshape(B * S * P, C), idx)
        rin = F.gather_rows(xn.reshape(B * S * P, C), idx)
        q, kv = F.linear_pair(qin, xc, a.in_proj_weight, a.in_proj_bias, C)  # kv [B*S, P, 2C]
        o0 = F.attention(q[:B * P].reshape(B, P, C), kv.reshape(B, S, P, 2 * C)[:, 0], blk.heads, C)
        o1 = F.attention(q[B * P:].reshape(B * S, 1, C), kv, blk.heads, C)
        o = torch.cat([o0.reshape(B * P, C), o1.reshape(B * S, C)])
        y = F.linear(o, a.out_proj.weight, a.out_proj.bias, resid=rin, out_dtype=torch.float32)
        yr, yn = F.res_layer_norm(y, eps=1e-6)
        y = blk.mlp(yn, resid=yr)
        f0 = y[:B * P].reshape(B, P, C)
        rows = y[B * P:].reshape(B, S, C)[:, 1:].contiguous()
        r = cblk(rows, f0)  # [B, S-1, C]
        return torch.cat([f0[:, 0:1], r], dim=1)

    def forward(self, reshaped_image, preliminary_cameras=None, iters=4, batch_size=None, rgb_feat_init=None,
                gt_cameras=None, fmaps=None, pred_trajectories=None, track_confidence=None, debug=False):
        if rgb_feat_init is None:
            rgb_feat, B, S, C = self.get_2D_image_features(reshaped_image, batch_size)
        else:
            rgb_feat = rgb_feat_init
            B, S, C = rgb_feat.shape
        # ---- T_P ----
        # (abl_track computes T_P and discards it: nothing downstream depends on it, so it is skipped
        # -- same outputs, and its parameters get no gradient either way)
        if pred_trajectories is not None and self.USE_TP and self.TP_RESIDUAL:
            traj = self.traj_encoder(pred_trajectories)  # [B, S, N, C] f32
            N = traj.shape[2]
            ca = self.confidence_attention
            w = F.linear(track_confidence.unsqueeze(-1), ca[0].weight, ca[0].bias, act=L.ACT_RELU)
            w = F.linear(w, ca[2].weight, ca[2].bias, act=L.ACT_SIGMOID, out_dtype=torch.float32)
            ctx = F.rowscale(traj, w).reshape(B * S, N, C)
            r = rgb_feat.reshape(B * S, 1, C)
            for blk in self.cross_attn_block:
                r = blk(r, ctx)
            rgb_feat = F.add(rgb_feat, r.reshape(B, S, C))
        # ---- T_F ----
        if self.USE_TIME:
            rgb_feat = F.add_rows(rgb_feat, self._table("1d", S, C, rgb_feat.device), S)
            # the trunk runs in f32 whatever the compute dtype: its attention spans the T = 16 frames
            # of one sequence, whose softmax backward cancels (dS = P (dP - delta) over nearly uniform
            # P), so bf16 operands cost the q-projection gradient several % (the reference's own bf16
            # autocast run: 2.9 %; tests/test_headline_gpu.py). 0.9 of the 7,477 GFLOP per sequence.
            with F.precision(torch.float32):
                for blk in self.trunk:
                    rgb_feat = blk(rgb_feat)
        if self.SINGLE_HEAD:
            return self._single_head(rgb_feat, gt_cameras, B, S)
        gt_enc = None
        if gt_cameras is not None:
            gt_enc = ops.pose_encode(gt_cameras.R.float(), gt_cameras.T_uvz.float(), gt_cameras.focal_length.float(),
                                     _ratio(gt_cameras), B, S)
        # ---- GAPR ----
        rot = self.pose_branch(rgb_feat)
        uv = F.linear(rgb_feat, self.fc_translation2d.weight, self.fc_translation2d.bias, out_dtype=torch.float32)
        dd = F.linear(rgb_feat, self.fc_depth.weight, self.fc_depth.bias, out_dtype=torch.float32)
        enc, losses = F.gapr(rot, uv, dd, gt_enc, B, S, self._cfg_get("weight_trans", 1), self._cfg_get("weight_rot", 2))
        pred_cameras = None
        if gt_cameras is not None:
            intr = INTRINSICS[_dataset(self.cfg)]
            R, T = ops.pose_decode(enc, gt_cameras.R.float(), gt_cameras.T_uvz.float(), _ratio(gt_cameras), intr, B, S)
            pred_cameras = PredCameras(R=R, T=T, focal_length=torch.zeros(B * S, 0, device=R.device))
        out = {"pred_pose_enc": enc, "gt_pose_enc": gt_enc, "pred_cameras": pred_cameras}
        if gt_enc is not None:
            out.update(loss=losses[0], loss_trans=losses[1], loss_rot=losses[2])
        else:
            out.update(loss=0, loss_trans=0, loss_rot=0)
        return out

    def _single_head(self, rgb_feat, gt_cameras, B, S):
        """camera_predictor_abl_uvz.py:379-436 / _abl_all.py: one Mlp predicts (dxyz, q); q is
        F.normalize'd, loss vs camera_to_pose_encoding3 (same weights / x100 MSE form as GAPR), frame 0
        reset, pose_encoding_to_camera3 (focal 2.0). The fused GAPR kernels run on strided views
        of the 7-wide output."""
        pred = self.pose_branch(rgb_feat)  # [B, S, 7] f32
        gt8 = None
        if gt_cameras is not None:
            gt8 = ops.pose_encode3(gt_cameras.R.float(), gt_cameras.T.float(), B, S)
        enc, losses = F.gapr(pred[..., 3:7], pred[..., 0:2], pred[..., 2:3], gt8, B, S,
                             self._cfg_get("weight_trans", 1.0), self._cfg_get("weight_rot", 2.0))
        pred_cameras = None
        if gt_cameras is not None:
            R, T = ops.pose_decode3(enc, gt_cameras.R.float(), gt_cameras.T.float(), B, S)
            pred_cameras = PredCameras(R=R, T=T, focal_length=torch.full((B * S, 1), 2.0, device=R.device))
        out = {"pred_pose_enc": enc, "gt_pose_enc": None if gt8 is None else gt8[:, :7], "pred_cameras": pred_cameras}
        if gt8 is not None:
            out.update(loss=losses[0], loss_trans=losses[1], loss_rot=losses[2])
        else:
            out.update(loss=0, loss_trans=0, loss_rot=0)
        return out


def _ratio(cams):
    """gt_cameras.ratio as the reference divides by it (a collated float64 tensor, B-15); handed to
    the pose codec as is (ops._ratio_args: host value or device pointer, never a device sync)."""
    return cams.ratio


def _dataset(cfg):
    try:
        return cfg.train.dataset
    except AttributeError:
        return cfg["train"]["dataset"]
