"""CPU checks of the drop-in boundary on the host side: the product COMET builds from the
reference's YAML `_target_` strings and exposes exactly the reference checkpoint layout
(key names + shapes, incl. facebookresearch DINOv2 names and the never-executed modules)."""
import os

import pytest
import torch

from conftest import ROOT


@pytest.fixture(scope="module")
def model():
    from comet_amd.config import instantiate, load_config
    cfg = load_config()
    torch.manual_seed(0)
    return instantiate(cfg.MODEL, _recursive_=False, cfg=cfg), cfg


def test_state_dict_layout_matches_reference(model):
    from oracle.weights import comet_shapes
    m, _ = model
    ref = comet_shapes()
    mine = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert set(mine) == set(ref), f"missing {sorted(set(ref) - set(mine))[:5]} extra {sorted(set(mine) - set(ref))[:5]}"
    bad = [k for k in ref if mine[k] != tuple(ref[k])]
    assert not bad, f"shape mismatch {bad[:5]}"
    assert list(mine) == list(ref), "state_dict key order differs from the reference"


def test_parameter_count_matches_readme(model):
    m, _ = model
    n = sum(p.numel() for p in m.parameters())
    assert n == 253_605_300  # README.md:211 "253.6M", probe count


def test_trainable_set_is_camera_predictor_minus_backbone(model):
    m, _ = model
    trainable = {k for k, p in m.named_parameters() if p.requires_grad}
    assert all(k.startswith("camera_predictor.") and ".backbone." not in k for k in trainable)
    assert sum(p.numel() for k, p in m.named_parameters() if p.requires_grad) == 115_940_968 + 2_280_711


def test_reference_yaml_loads_if_present():
    from comet_amd.config import load_config, resolve_target
    p = "/root/reference/comet/models/abl_ours.yaml"
    if not os.path.exists(p):
        pytest.skip("reference not mounted")
    cfg = load_config(p)
    assert resolve_target(cfg.MODEL._target_).__name__ == "COMET"
    assert resolve_target(cfg.MODEL.CAMERA._target_).__name__ == "CameraPredictor"
