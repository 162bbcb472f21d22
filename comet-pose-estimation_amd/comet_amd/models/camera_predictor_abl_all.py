"""All-components ablation head (mirror of comet/models/camera_predictor_abl_all.py, selected by
abl_all.yaml's `_target_: models.camera_predictor_abl_all.CameraPredictor`).

camera_predictor_abl_all.py: T_P, T_F (time embedding + trunk) removed and the single
7-output head with encoding 3 (as abl_uvz).
Same constructor, submodules and state_dict keys as the reference file; everything else is
camera_predictor10.CameraPredictor.
"""
from .camera_predictor10 import CameraPredictor as _Base


class CameraPredictor(_Base):
    USE_TP = False
    USE_TIME = False
    SINGLE_HEAD = True
