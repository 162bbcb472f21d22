"""T_P ablation head (mirror of comet/models/camera_predictor_abl_track.py, selected by
abl_track.yaml's `_target_: models.camera_predictor_abl_track.CameraPredictor`).

camera_predictor_abl_track.py:348 comments out `rgb_feat = rgb_feat + rgb_flat`: the trajectory
cross-attention result is discarded (computed by the reference, skipped here: output-identical).
Same constructor, submodules and state_dict keys as the reference file; everything else is
camera_predictor10.CameraPredictor.
"""
from .camera_predictor10 import CameraPredictor as _Base


class CameraPredictor(_Base):
    TP_RESIDUAL = False
