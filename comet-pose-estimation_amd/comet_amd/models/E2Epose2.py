"""COMET (mirror of comet/models/E2Epose2.py:59-266): tracker (no_grad) -> score inversion ->
camera predictor. Same constructor (TRACK, CAMERA, cfg) and forward signature."""
from typing import Dict

import torch
import torch.nn as nn

from ..config import instantiate
from .refine_track import refine_track


class COMET(nn.Module):
    def __init__(self, TRACK: Dict, CAMERA: Dict, cfg=None):
        super().__init__()
        if cfg is None:
            raise ValueError("cfg must be provided")
        self.cfg = cfg
        self.enable_track = cfg["enable_track"]
        self.enable_pose = cfg["enable_pose"]
        self.window_len = cfg.get("window_len", 8) if hasattr(cfg, "get") else 8
        if not (self.enable_track or self.enable_pose):
            raise ValueError("You have to enable at least tracking or pose estimation.")
        if self.enable_track:
            self.track_predictor = instantiate(TRACK, _recursive_=False, cfg=cfg)
            self._freeze_tracker_params()
        if self.enable_pose:
            self.camera_predictor = instantiate(CAMERA, _recursive_=False, cfg=cfg)

    def _freeze_tracker_params(self):
        if self.cfg.get("freeze_track", False):
            for p in self.track_predictor.parameters():
                p.requires_grad = False

    def forward(self, image, gt_cameras=None, training=True, tracks=None, tracks_visibility=None, crop_params=None,
                epoch=-1):
        if training:
            return self.forward_all(image, gt_cameras=gt_cameras, training=training, tracks=tracks,
                                    tracks_visibility=tracks_visibility)
        assert image.shape[0] == 1, f"evaluation processes one sequence at a time, got batch {image.shape[0]}"
        with torch.no_grad():
            return self.forward_all(image, gt_cameras=gt_cameras, training=training, tracks=tracks,
                                    tracks_visibility=tracks_visibility)

    def forward_all(self, image, preliminary_cameras=None, gt_cameras=None, training=True, tracks=None,
                    tracks_visibility=None):
        """E2Epose2.py:151-266 (fine_tracker=True, softmax_refine=False, track_conf=False)."""
        B, T, C, H, W = image.shape
        cfg = self.cfg
        predictions = {}
        pred_track = inverted_score = None
        with torch.no_grad():
            if self.enable_track:
                tp = self.track_predictor
                fmaps = tp.process_images_to_fmaps(image, training=True)
                coarse_lists, vis_e, _, _, _ = tp.coarse_predictor(query_points=tracks[:, 0], fmaps=fmaps,
                                                                   iters=cfg["track_trainit"],
                                                                   down_ratio=tp.coarse_down_ratio, return_feat=True)
                coarse = coarse_lists[-1]
                if cfg["fine_tracker"]:
                    refined, score, inverted_score = refine_track(image, tp.fine_fnet, tp.fine_predictor, coarse,
                                                                  compute_score=True)
                    predictions["coarse_pred_track"] = coarse
                    predictions["refine_pred_track"] = refined
                    predictions["pred_score"] = inverted_score
                    pred_track = refined
                else:
                    pred_track = coarse
                    predictions["refine_pred_track"] = coarse
        pose_predictions = {}
        if self.enable_pose:
            pose_predictions = self.camera_predictor(image.reshape(-1, C, H, W), preliminary_cameras=None,
                                                     batch_size=B, gt_cameras=gt_cameras, iters=cfg["camera_iter"],
                                                     pred_trajectories=pred_track, track_confidence=inverted_score)
        if self.enable_track:
            pose_predictions["pred_tracks"] = predictions["refine_pred_track"]
            pose_predictions["_track_predictions"] = predictions
        return pose_predictions
