"""T_F ablation head (mirror of comet/models/camera_predictor_abl_time.py, selected by
abl_time.yaml's `_target_: models.camera_predictor_abl_time.CameraPredictor`).

camera_predictor_abl_time.py:364-381 comments out the 1-D time embedding and the trunk:
rgb_feat goes from T_P straight to the GAPR head.
Same constructor, submodules and state_dict keys as the reference file; everything else is
camera_predictor10.CameraPredictor.
"""
from .camera_predictor10 import CameraPredictor as _Base


class CameraPredictor(_Base):
    USE_TIME = False
