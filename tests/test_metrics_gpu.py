"""evaluation metrics (comet_amd.metrics over csrc/metrics.hip) against the reference
metric.py (tests/golden/comet_golden_metrics.npz, tools/gen_golden.py --metrics: the reference's
camera_to_rel_deg3 / camera_to_rel_deg2 / calculate_auc on synthetic eval outputs with exact-match,
180-degree-flip, Euler-singular and zero-translation frames) and against the oracle at a larger size.

Tolerances: both sides compute in f32 (the reference's autocast(dtype=torch.double) is inactive);
an angle from acos of a value within f32 rounding of 1 carries up to ~0.03 degrees of rounding
noise, so angles match to 0.05 degrees + 1e-4 relative; histogram bins may move by a pair whose
error lies within that noise of an integer edge (at most 2 pairs per bin)."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
GOLD = os.path.join(ROOT, "tests", "golden", "comet_golden_metrics.npz")


class _Cams:
    def __init__(self, M, T):
        self.T, self._M = T, M

    def get_world_to_view_transform(self):
        return self

    def get_matrix(self):
        return self._M


def close(a, b, rtol, atol, what):
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(np.asarray(b)).double()
    assert a.shape == b.shape, f"{what}: shape {tuple(a.shape)} vs {tuple(b.shape)}"
    err = (a - b).abs()
    print(f"{what}: max abs err {err.max().item():.3e}")
    assert bool((err <= atol + rtol * b.abs()).all()), f"{what}: max err {err.max().item():.3e}"


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD, allow_pickle=False))


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_metrics_match_reference(gold, tag):
    from comet_amd import metrics as M
    g = {k[3:]: v for k, v in gold.items() if k.startswith(f"m{tag}_")}
    B = int(g["cfg"][1])
    dev = torch.device("cuda")
    pc = _Cams(torch.from_numpy(g["pred_w2v"]).to(dev), torch.from_numpy(g["pred_T"]).to(dev))
    gc = _Cams(torch.from_numpy(g["gt_w2v"]).to(dev), torch.from_numpy(g["gt_T"]).to(dev))
    r3 = M.camera_to_rel_deg3(pc, gc, dev, B)
    torch.cuda.synchronize()
    close(r3[0], g["d3_rel_rangle"], 1e-4, 5e-2, "camera_to_rel_deg3 rotation (deg)")
    close(r3[1], g["d3_rel_tangle"], 1e-4, 5e-2, "camera_to_rel_deg3 translation (deg)")
    for i, k in enumerate(["T_avg", "Tx", "Ty", "Tz"]):
        close(r3[2 + i].reshape(1), g["d3_" + k].reshape(1), 1e-6, 1e-6, f"camera_to_rel_deg3 {k}")
    ep, eg = torch.from_numpy(g["pred_enc"]).to(dev), torch.from_numpy(g["gt_enc"]).to(dev)
    rr, tt, avg, eul, acc5 = M.camera_to_rel_deg2(ep, eg, dev, B)
    close(rr, g["d2_rel_rangle"], 1e-4, 5e-2, "camera_to_rel_deg2 geodesic (deg)")
    close(tt, g["d2_rel_tangle"], 1e-4, 5e-2, "camera_to_rel_deg2 translation (deg)")
    close(avg.reshape(1), g["d2_avg"], 1e-4, 5e-3, "camera_to_rel_deg2 mean geodesic (deg)")
    close(eul, g["d2_error_euler"], 1e-4, 1e-4, "camera_to_rel_deg2 mean |Euler| (deg)")
    npairs = r3[0].numel()
    close(np.asarray(acc5), g["d2_acc5"], 0, 2.0 / ep.shape[0] + 1e-12, "acc@5deg")
    auc, hist = M.calculate_auc(r3[0], r3[1], max_threshold=30, return_list=True)
    close(hist * npairs, g["hist"] * npairs, 0, 2.01, "AUC histogram (pairs per bin)")
    close(auc.reshape(1), g["auc30"], 0, 2.0 / npairs, "Auc_30")


def test_metrics_large_vs_oracle():
    """B = 8 sequences of 64 frames (16128 pairs): the HIP pair / frame errors against the oracle's
    f32 restatement on the same inputs (pinned to the reference in test_oracle_golden.py)."""
    from comet_amd import metrics as M
    from oracle import comet_oracle as O
    torch.manual_seed(7)
    B, S = 8, 64
    n = B * S
    q = torch.nn.functional.normalize(torch.randn(n, 4), dim=-1)
    qp = torch.nn.functional.normalize(q + 0.2 * torch.randn(n, 4), dim=-1)

    def w2v(qq, T):
        m = torch.zeros(n, 4, 4)
        m[:, :3, :3] = O._quat2mat(qq)
        m[:, 3, :3] = T
        m[:, 3, 3] = 1
        return m
    Tg = torch.randn(n, 3)
    Mp, Mg = w2v(qp, Tg + 0.1 * torch.randn(n, 3)), w2v(q, Tg)
    rot, tr = M.pair_errors(Mp.cuda(), Mg.cuda(), B)
    rot_o, tr_o = O.pose_pair_errors(Mp, Mg, B)
    close(rot, rot_o, 1e-4, 5e-2, "pair rotation (deg)")
    close(tr, tr_o, 1e-4, 5e-2, "pair translation (deg)")
    ep = torch.cat([torch.randn(n, 3), qp], 1)
    eg = torch.cat([torch.randn(n, 3), q, torch.zeros(n, 1)], 1)
    ftr, geo, eul = M.frame_errors(ep.cuda(), eg.cuda())
    ftr_o, geo_o, eul_o = O.pose_frame_errors(ep, eg)
    close(torch.rad2deg(geo), torch.rad2deg(geo_o), 1e-4, 5e-2, "geodesic (deg)")
    close(ftr, ftr_o, 1e-4, 5e-2, "frame translation (deg)")
    close(eul, eul_o, 1e-4, 1e-4, "Euler (rad)")


def test_pose_metrics_on_eval_outputs(gold):
    """The eval block's dict (train_eval_func_new_cp5.py:633-671) from pose_metrics: keys present,
    AUCs monotone in the threshold, consistent with calculate_auc on the same errors."""
    from comet_amd import metrics as M
    g = {k[3:]: v for k, v in gold.items() if k.startswith("mb_")}
    dev = torch.device("cuda")
    B = int(g["cfg"][1])
    preds = {"pred_cameras": _Cams(torch.from_numpy(g["pred_w2v"]).to(dev), torch.from_numpy(g["pred_T"]).to(dev)),
             "pred_pose_enc": torch.from_numpy(g["pred_enc"]).to(dev), "gt_pose_enc": torch.from_numpy(g["gt_enc"]).to(dev)}
    gc = _Cams(torch.from_numpy(g["gt_w2v"]).to(dev), torch.from_numpy(g["gt_T"]).to(dev))
    out = M.pose_metrics(preds, gc, B)
    for k in ["R_avg", "T_avg", "X_err", "Y_err", "Z_err", "Racc_him_5", "Tacc_him_15", "Auc_30", "Auc_3",
              "acc@5deg_x"]:
        assert k in out
    for th in (30, 10, 5, 3):
        close(out[f"Auc_{th}"].reshape(1), g[f"auc_{th}"], 0, 2.0 / 480, f"Auc_{th}")
    close(out["R_avg"].reshape(1), g["d2_avg"], 1e-4, 5e-3, "R_avg")


def test_eval_step_runs_metrics_on_model_output():
    """abl_ours.py test_fn path end to end (BASELINE configs[0] shape, small frames): eval_step ->
    model(..., training=False) -> pose_metrics; R_avg equals the mean geodesic error of the
    returned encodings (oracle restatement on the same tensors)."""
    from comet_amd import functional as F
    from comet_amd.config import instantiate, load_config
    from comet_amd.models.utils import QuaternionCameras
    from comet_amd.train import eval_step
    from oracle import comet_oracle as O
    from oracle import prng
    from oracle.weights import comet_shapes
    cfg = load_config()
    model = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg)
    model.load_state_dict(prng.make_state_dict(0, comet_shapes()), strict=True)
    model = model.cuda()
    img, tracks, gt = prng.synthetic_batch(1, 1, 16, 128, 128, 16)
    cams = QuaternionCameras(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
                             principal_point=gt["principal_point"], ratio=gt["ratio"], device="cuda")
    with F.precision(torch.float32):
        out = eval_step(model, img.cuda(), cams, tracks.cuda())
    torch.cuda.synchronize()
    _, geo, _ = O.pose_frame_errors(out["pred_pose_enc"].float().cpu(), out["gt_pose_enc"].float().cpu())
    close(out["R_avg"].reshape(1), torch.rad2deg(geo).mean().reshape(1), 1e-4, 5e-3, "R_avg vs oracle")
    assert 0.0 <= float(out["Auc_30"]) <= 1.0 and float(out["Auc_3"]) <= float(out["Auc_30"]) + 1e-6
