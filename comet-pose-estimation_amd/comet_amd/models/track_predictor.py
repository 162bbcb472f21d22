"""TrackerPredictor (mirror of comet/models/track_predictor.py): coarse BasicEncoder +
BaseTrackerPredictor, fine ShallowEncoder + BaseTrackerPredictor, built from the same
COARSE / FINE config dicts (abl_ours.yaml:397-428)."""
import torch
from torch import nn

from .. import functional as F
from .. import ops
from ..config import instantiate


class TrackerPredictor(nn.Module):
    def __init__(self, COARSE, FINE, stride=4, corr_levels=5, corr_radius=4, latent_dim=128, cfg=None, **extra_args):
        super().__init__()
        self.cfg = cfg
        self.coarse_down_ratio = COARSE["down_ratio"]
        self.coarse_fnet = instantiate(COARSE["FEATURENET"], _recursive_=False, stride=COARSE["stride"], cfg=cfg)
        self.coarse_predictor = instantiate(COARSE["PREDICTOR"], _recursive_=False, stride=COARSE["stride"], cfg=cfg)
        self.fine_fnet = instantiate(FINE["FEATURENET"], _recursive_=False, stride=1, cfg=cfg)
        self.fine_predictor = instantiate(FINE["PREDICTOR"], _recursive_=False, stride=1, cfg=cfg)

    @torch.no_grad()
    def process_images_to_fmaps(self, images, training=False):
        """track_predictor.py:117-151: x1/down_ratio bilinear (align_corners) then BasicEncoder.
        images [B, S, 3, H, W] f32 -> fmaps NHWC [B, S, H/(down*stride), W/(down*stride), 128]."""
        B, S, C, H, W = images.shape
        if not training:
            assert B == 1, "now we only support processing one scene during inference"
        x = images.reshape(B * S, C, H, W)
        if self.coarse_down_ratio > 1:
            h, w = int(H / self.coarse_down_ratio), int(W / self.coarse_down_ratio)
        else:
            h, w = H, W
        # resize + NCHW -> NHWC + cast in one pass; bf16 pads RGB to 8 channels so conv1 is an
        # implicit GEMM (zero channels x zero weights)
        cdt = F.compute_dtype()
        x = ops.images_nhwc(x, h, w, cdt, cpad=8 if cdt == torch.bfloat16 else 3)
        fm = self.coarse_fnet(x, h, w)
        return fm.reshape(B, S, fm.shape[1], fm.shape[2], fm.shape[3])
