"""ORACLE / TEST INFRASTRUCTURE ONLY — the reference COMET state_dict layout (765 keys, checkpoint
naming incl. facebookresearch DINOv2 names), as extracted from the reference model by
tools/gen_golden.py into tests/golden/comet_state_dict_shapes.json."""
import json
import os

_JSON = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                     "comet_state_dict_shapes.json")


def comet_shapes():
    with open(_JSON) as f:
        return {k: tuple(v) for k, v in json.load(f)}


def camera_predictor_trainable(shapes=None):
    shapes = shapes or comet_shapes()
    return [k for k in shapes if k.startswith("camera_predictor.") and not k.startswith("camera_predictor.backbone.")]
