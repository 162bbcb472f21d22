"""GAPR ablation head (mirror of comet/models/camera_predictor_abl_uvz.py, selected by
abl_uvz.yaml's `_target_: models.camera_predictor_abl_uvz.CameraPredictor`).

camera_predictor_abl_uvz.py:153,379-436: pose_branch predicts all 7 pose values (dxyz, q) in one
Mlp (out_features=7) against camera_to_pose_encoding3 / pose_encoding_to_camera3 (utils.py:270-310,
591-627) instead of the three GAPR heads over (u, v, depth) encoding 2.
Same constructor, submodules and state_dict keys as the reference file; everything else is
camera_predictor10.CameraPredictor.
"""
from .camera_predictor10 import CameraPredictor as _Base


class CameraPredictor(_Base):
    SINGLE_HEAD = True
