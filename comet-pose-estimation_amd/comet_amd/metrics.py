"""Evaluation metrics of the COMET eval path: mirror of comet/models/metric.py with
the same names, arguments and return values, as consumed by train_eval_func_new_cp5.py:633-671
(camera_to_rel_deg3, camera_to_rel_deg2, calculate_auc) after model(..., training=False).

The per-pair and per-frame geometry runs in libcomet_hip.so (csrc/metrics.hip:
comet_pose_pair_errors, comet_pose_frame_errors) on the tensors' device; the reductions that the
reference does with torch / numpy (means, RMSE, histogram, thresholds) stay torch / numpy here.
`pose_metrics` reproduces the reference's eval block (its dict keys) for one batch.

Reference behaviours kept on purpose:
  * camera_to_rel_deg2 is the definition metric.py binds LAST (391-451): it returns
    (rel_rangle_deg, rel_tangle_deg, avg_rangle_deg, error_euler [x, y, z] deg, acc@5deg list);
  * translation_angle folds the 180-degree ambiguity (metric.py:680-681);
  * calculate_auc bins with torch.histc(bins=max_threshold + 1, min=0, max=max_threshold) and
    returns the mean of the cumulative normalised histogram (metric.py:524-558);
  * the pair errors take the world-to-view matrices as get_matrix() returns them (f32).
"""
import ctypes

import numpy as np
import torch

from . import _lib as L
from .ops import stream as _stream


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


def _f32(t, dev):
    return t.detach().to(device=dev, dtype=torch.float32).contiguous()


def batched_all_pairs(B, N):
    """metric.py:561-570: frame-index pairs i < j of every sequence, torch.combinations order."""
    i1_, i2_ = torch.combinations(torch.arange(N), 2, with_replacement=False).unbind(-1)
    i1, i2 = [(i[None] + torch.arange(B)[:, None] * N).reshape(-1) for i in [i1_, i2_]]
    return i1, i2


def pair_errors(pred_se3, gt_se3, batch_size):
    """All-pairs relative rotation / translation angle errors (degrees) of world-to-view matrices
    [B*S, 4, 4] (metric.py:214-245) -> (rel_rangle_deg, rel_tangle_deg), [B * S*(S-1)/2] each."""
    dev = gt_se3.device
    if dev.type != "cuda":
        raise L.CometHipError("pose metrics run on the GPU (libcomet_hip.so)")
    S = gt_se3.shape[0] // batch_size
    p, g = _f32(pred_se3, dev), _f32(gt_se3, dev)
    n = batch_size * (S * (S - 1) // 2)
    rot = torch.empty(n, device=dev, dtype=torch.float32)
    tr = torch.empty(n, device=dev, dtype=torch.float32)
    L.check(L.load().comet_pose_pair_errors(_p(p), _p(g), batch_size, S, _p(rot), _p(tr), _stream()),
            "comet_pose_pair_errors")
    return rot, tr


def frame_errors(pred_pose_enc, gt_enc):
    """Per-frame errors of pose encodings (metric.py:391-451 core): translation angle (deg),
    geodesic angle of Rp·Rgᵀ (rad), Euler angles of Rp·Rgᵀ [n, 3] (rad)."""
    dev = gt_enc.device
    if dev.type != "cuda":
        raise L.CometHipError("pose metrics run on the GPU (libcomet_hip.so)")
    p, g = _f32(pred_pose_enc, dev), _f32(gt_enc, dev)
    n = p.shape[0]
    tr = torch.empty(n, device=dev, dtype=torch.float32)
    geo = torch.empty(n, device=dev, dtype=torch.float32)
    eul = torch.empty(n, 3, device=dev, dtype=torch.float32)
    L.check(L.load().comet_pose_frame_errors(_p(p), p.shape[1], _p(g), g.shape[1], n, _p(tr), _p(geo), _p(eul),
                                             _stream()), "comet_pose_frame_errors")
    return tr, geo, eul


def camera_to_rel_deg(pred_cameras, gt_cameras, device, batch_size):
    """metric.py:140-180 -> (rel_rangle_deg, rel_tangle_deg) over all frame pairs."""
    with torch.no_grad():
        gt_se3 = gt_cameras.get_world_to_view_transform().get_matrix()
        pred_se3 = pred_cameras.get_world_to_view_transform().get_matrix()
        return pair_errors(pred_se3.to(device), gt_se3.to(device), batch_size)


def camera_to_rel_deg3(pred_cameras, gt_cameras, device, batch_size):
    """metric.py:183-247 -> (rel_rangle_deg, rel_tangle_deg, translation_err, X_err, Y_err, Z_err):
    pair errors plus the absolute translation RMSE (x 10^3) overall and per axis."""
    with torch.no_grad():
        Tp, Tg = pred_cameras.T, gt_cameras.T
        Tg = Tg.to(device=Tp.device)
        n = Tp.shape[0]

        def rmse(a, b):
            return torch.sqrt(torch.nn.functional.mse_loss(a, b, reduction="sum") / n) * (10 ** 3)
        translation_err = rmse(Tp, Tg)
        X_err, Y_err, Z_err = (rmse(Tp[:, k], Tg[:, k]) for k in range(3))
        rot, tr = camera_to_rel_deg(pred_cameras, gt_cameras, device, batch_size)
    return rot, tr, translation_err, X_err, Y_err, Z_err


def camera_to_rel_deg2(pred_pose_enc, gt_enc, device, batch_size, with_cumulative_err=False):
    """metric.py:391-451 (the binding in effect) -> (rel_rangle_deg [n] deg, rel_tangle_deg [n] deg,
    avg_rangle_deg, error_euler [x, y, z] mean |Euler| deg (numpy), acc@5deg [x, y, z] list)."""
    with torch.no_grad():
        tr, geo, eul = frame_errors(pred_pose_enc.to(device), gt_enc.to(device))
        rel_rangle_deg = torch.rad2deg(geo)
        eulers = eul.double().cpu().numpy()
        error_euler = np.rad2deg(np.mean(np.abs(eulers), axis=0))
        error_eulers = np.rad2deg(eulers)
        avg_rangle_deg = rel_rangle_deg.mean()
        percentages_list = (error_eulers < 5.0).mean(axis=0).tolist()
    return rel_rangle_deg, tr, avg_rangle_deg, error_euler, percentages_list


def calculate_auc(r_error, t_error, max_threshold=30, return_list=False):
    """metric.py:524-558: mean of the cumulative normalised histogram of max(r, t) error."""
    max_errors, _ = torch.max(torch.stack((r_error, t_error), dim=1), dim=1)
    histogram = torch.histc(max_errors, bins=max_threshold + 1, min=0, max=max_threshold)
    normalized_histogram = histogram / float(max_errors.size(0))
    if return_list:
        return torch.cumsum(normalized_histogram, dim=0).mean(), normalized_histogram
    return torch.cumsum(normalized_histogram, dim=0).mean()


def calculate_auc_np(r_error, t_error, max_threshold=30):
    """metric.py:494-521 (numpy histogram with integer bin edges)."""
    max_errors = np.max(np.concatenate((r_error[:, None], t_error[:, None]), axis=1), axis=1)
    histogram, _ = np.histogram(max_errors, bins=np.arange(max_threshold + 1))
    normalized_histogram = histogram.astype(float) / float(len(max_errors))
    return np.mean(np.cumsum(normalized_histogram)), normalized_histogram


def pose_metrics(predictions, gt_cameras, batch_size, device=None):
    """The eval block of train_eval_func_new_cp5.py:633-671 for one batch -> the keys it adds to
    `predictions` (R_avg, T_avg, X/Y/Z_err, Tx/Ty/Tz_mse, acc@5deg_*, Racc_him_*, Tacc_him_*, Auc_*)."""
    device = device or predictions["pred_pose_enc"].device
    out = {}
    rot_him, tr_him, T_avg, Tx, Ty, Tz = camera_to_rel_deg3(predictions["pred_cameras"], gt_cameras, device,
                                                             batch_size)
    _, _, R_avg, error_euler, acc_5 = camera_to_rel_deg2(predictions["pred_pose_enc"], predictions["gt_pose_enc"],
                                                         device, batch_size)
    out.update({"X_err": error_euler[2], "Y_err": error_euler[1], "Z_err": error_euler[0], "R_avg": R_avg,
                "T_avg": T_avg, "Tx_mse": Tx, "Ty_mse": Ty, "Tz_mse": Tz, "acc@5deg_x": acc_5[2],
                "acc@5deg_y": acc_5[1], "acc@5deg_z": acc_5[0]})
    for th in (5, 10, 15):
        out[f"Racc_him_{th}"] = (rot_him < th).float().mean()
        out[f"Tacc_him_{th}"] = (tr_him < th).float().mean()
    _, hist = calculate_auc(rot_him, tr_him, max_threshold=30, return_list=True)
    for th in (30, 10, 5, 3):
        out[f"Auc_{th}"] = torch.cumsum(hist[:th], dim=0).mean()
    return out
