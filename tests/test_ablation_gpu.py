"""the ablation heads (camera_predictor_abl_{time,track,uvz,all}.py, chosen by the
reference's abl_*.yaml `_target_`) on the HIP path vs fixtures generated from the reference itself
(tests/golden/comet_golden_abl.npz, tools/gen_golden.py --ablations): pose encodings, losses, decoded
cameras and the norm of every parameter gradient, fp32, from the forward's rgb_feat_init entry."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
GOLD = os.path.join(ROOT, "tests", "golden", "comet_golden_abl.npz")
VARIANTS = ["ours", "time", "track", "uvz", "all"]


def close(a, b, rtol, atol, what):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(np.asarray(b)).double()
    assert a.shape == b.shape, f"{what}: shape {tuple(a.shape)} vs {tuple(b.shape)}"
    err = (a - b).abs()
    bad = err > atol + rtol * b.abs()
    assert not bool(bad.any()), f"{what}: max err {err.max().item():.3e} ({int(bad.sum())} bad of {bad.numel()})"


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD, allow_pickle=False))


def _head(variant):
    import importlib
    from comet_amd.config import load_config
    from oracle import prng
    mod = "camera_predictor10" if variant == "ours" else f"camera_predictor_abl_{variant}"
    M = importlib.import_module("comet_amd.models." + mod)
    cfg = load_config()
    kw = {k: v for k, v in cfg.MODEL.CAMERA.items() if k != "_target_"}
    cp = M.CameraPredictor(cfg=cfg, **kw)
    shapes = {"camera_predictor." + k: tuple(t.shape) for k, t in cp.state_dict().items() if not k.startswith("backbone.")}
    P = prng.make_state_dict(0, shapes)
    missing, unexpected = cp.load_state_dict({k[len("camera_predictor."):]: t for k, t in P.items()}, strict=False)
    assert not unexpected and all(k.startswith("backbone.") for k in missing)
    return cp.cuda()


@pytest.mark.parametrize("variant", VARIANTS)
def test_ablation_head_matches_reference(variant, gold):
    from comet_amd import functional as F
    from comet_amd.models.utils import QuaternionCameras
    from oracle import prng
    B, S, N, seed_rgb, seed_x = [int(v) for v in gold["abl_cfg"]]
    cp = _head(variant)
    _, _, gt = prng.synthetic_batch(seed_x, B, S, 128, 128, N)
    cams = QuaternionCameras(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
                             principal_point=gt["principal_point"], ratio=gt["ratio"], device="cuda")
    rgb = torch.from_numpy(gold["abl_rgb"]).cuda()
    tracks = torch.from_numpy(gold["abl_tracks"]).cuda()
    conf = torch.from_numpy(gold["abl_conf"]).cuda()
    with F.precision(torch.float32):
        cp.zero_grad(set_to_none=True)
        out = cp(None, batch_size=B, rgb_feat_init=rgb, gt_cameras=cams, pred_trajectories=tracks,
                 track_confidence=conf)
        out["loss"].backward()
    torch.cuda.synchronize()
    pre = f"abl_{variant}_"
    close(out["pred_pose_enc"], gold[pre + "pred_pose_enc"], 1e-4, 1e-4, f"{variant} pred_pose_enc")
    close(out["gt_pose_enc"], gold[pre + "gt_pose_enc"], 1e-6, 1e-6, f"{variant} gt_pose_enc")
    for k in ("loss", "loss_trans", "loss_rot"):
        close(out[k].reshape(1), gold[pre + k], 1e-4, 1e-4, f"{variant} {k}")
    close(out["pred_cameras"].R, gold[pre + "pred_R"], 1e-4, 1e-4, f"{variant} pred R")
    close(out["pred_cameras"].T, gold[pre + "pred_T"], 1e-4, 1e-4, f"{variant} pred T")
    names = [str(n) for n in gold[pre + "grad_names"]]
    got = {k: p.grad for k, p in cp.named_parameters() if p.grad is not None}
    assert sorted(got) == names, f"{variant}: gradient set differs"
    norms = torch.tensor([got[k].double().norm().item() for k in names])
    close(norms, gold[pre + "grad_norms"], 2e-3, 1e-6, f"{variant} grad norms")
