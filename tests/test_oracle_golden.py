"""Pin the oracle (CPU restatement) to golden vectors generated from the reference itself
(tools/gen_golden.py, build container). Runs on CPU; weights/inputs regenerated from seeds."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT
from oracle import comet_oracle as O
from oracle import prng

GOLD = os.path.join(ROOT, "tests", "golden", "comet_golden_v1.npz")


@pytest.fixture(scope="module")
def gold():
    return dict(np.load(GOLD, allow_pickle=False))


def close(a, b, rtol, atol, what):
    a = torch.as_tensor(np.asarray(a), dtype=torch.float64)
    b = torch.as_tensor(np.asarray(b), dtype=torch.float64)
    assert a.shape == b.shape, f"{what}: shape {tuple(a.shape)} vs {tuple(b.shape)}"
    err = (a - b).abs()
    assert bool((err <= atol + rtol * b.abs()).all()), f"{what}: max err {err.max().item():.3e}"


def test_sincos_tables(gold):
    close(O.sincos_1d(768, 16), gold["sincos_1d_768_16"], 0, 1e-7, "1d sincos")
    close(O.sincos_2d(768, 24, 24), gold["sincos_2d_768_24"], 0, 1e-7, "2d sincos 768")
    close(O.sincos_2d(664, 16, 16), gold["sincos_2d_664_16"], 0, 1e-7, "2d sincos 664")
    close(O.embed_2d(torch.from_numpy(gold["embed2d_in"]), 64), gold["embed2d_64"], 0, 1e-6, "flow emb")


def test_harmonic_embedding(gold):
    x = torch.from_numpy(gold["harm_x"])
    cov = torch.from_numpy(gold["harm_cov"])
    for n, om, logs, app in [(6, 1.0, True, True), (48, 1.0, True, False), (10, 0.5, False, True)]:
        tag = f"harm_{n}_{om}_{int(logs)}_{int(app)}"
        close(O.harmonic_embedding(x, n, om, logs, app), gold[tag], 0, 1e-6, tag)
        close(O.harmonic_embedding(x, n, om, logs, app, diag_cov=cov), gold[tag + "_cov"], 0, 1e-6, tag + " cov")


def test_pose_codec(gold):
    R = torch.from_numpy(gold["codec_gt_R"])
    T = torch.from_numpy(gold["codec_gt_Tuvz"])
    ratio = torch.tensor([0.5], dtype=torch.float64)
    enc = O.camera_to_pose_encoding2(R, T, torch.full((R.shape[0], 2), 268.44), ratio)
    close(enc, gold["codec_enc"], 0, 1e-6, "camera_to_pose_encoding2")
    penc = torch.from_numpy(gold["codec_penc"])[0]
    for it in ["AMD_eval", "AMD_test", "spark"]:
        q, t, _ = O.pose_encoding_to_camera2(penc, R[0], T[0], ratio, it)
        close(q, gold[f"codec_dec_R_{it}"], 0, 1e-6, f"decode R {it}")
        close(t, gold[f"codec_dec_T_{it}"], 1e-6, 1e-5, f"decode T {it}")


def _block_params(seed, shapes):
    return {k: v.requires_grad_(True) for k, v in prng.make_state_dict(seed, shapes).items()}


def _attn_shapes(C=768, cross=False):
    a = "cross_attn" if cross else "attn"
    sh = {f"{a}.in_proj_weight": (3 * C, C), f"{a}.in_proj_bias": (3 * C,),
          f"{a}.out_proj.weight": (C, C), f"{a}.out_proj.bias": (C,),
          "mlp.fc1.weight": (4 * C, C), "mlp.fc1.bias": (4 * C,),
          "mlp.fc2.weight": (C, 4 * C), "mlp.fc2.bias": (C,)}
    if cross:
        sh.update({"norm_context.weight": (C,), "norm_context.bias": (C,)})
    return sh


def _check_grads(gold, prefix, P, rtol):
    for k, p in P.items():
        g = p.grad
        close(g.norm().reshape(1), gold[prefix + "norm." + k], rtol, 1e-6, prefix + "norm " + k)
        if g.numel() <= 4096:
            close(g, gold[prefix + k], rtol, 1e-6, prefix + k)
        else:
            close(g.reshape(g.shape[0], -1)[:4], gold[prefix + "head." + k], rtol, 1e-5, prefix + k)


def test_attn_blocks_fwd_bwd(gold):
    P = _block_params(7, _attn_shapes())
    x = torch.from_numpy(prng.normal_like(8, "attn_x", (3, 37, 768))).requires_grad_(True)
    # PRNG values are keyed by the block-local names; the oracle reads them under a prefix
    Pn = {"b." + k: v for k, v in P.items()}
    y = O.attn_block(x, Pn, "b", 8)
    y.backward(torch.from_numpy(prng.normal_like(8, "attn_gy", (3, 37, 768))))
    close(y.detach(), gold["blk_attn_y"], 1e-5, 1e-5, "AttnBlock y")
    close(x.grad, gold["blk_attn_dx"], 1e-4, 1e-5, "AttnBlock dx")
    _check_grads(gold, "blk_attn_grad.", P, 1e-4)

    P = _block_params(8, _attn_shapes(cross=True))
    Pn = {"b." + k: v for k, v in P.items()}
    x = torch.from_numpy(prng.normal_like(9, "cx", (2, 29, 768))).requires_grad_(True)
    c = torch.from_numpy(prng.normal_like(9, "cc", (2, 41, 768))).requires_grad_(True)
    y = O.cross_attn_block(x, c, Pn, "b", 8)
    y.backward(torch.from_numpy(prng.normal_like(9, "cgy", (2, 29, 768))))
    close(y.detach(), gold["blk_cross_y"], 1e-5, 1e-5, "CrossAttnBlock y")
    close(x.grad, gold["blk_cross_dx"], 1e-4, 1e-5, "CrossAttnBlock dx")
    close(c.grad, gold["blk_cross_dctx"], 1e-4, 1e-5, "CrossAttnBlock dctx")
    _check_grads(gold, "blk_cross_grad.", P, 1e-4)


@pytest.fixture(scope="module")
def e2e(gold):
    from oracle.weights import comet_shapes
    seed_w, seed_x, B, T, H, W, N = [int(v) for v in gold["cfg"]]
    P = prng.make_state_dict(seed_w, comet_shapes())
    img, tracks, gt = prng.synthetic_batch(seed_x, B, T, H, W, N)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    names = ["camera_predictor." + str(k) for k in gold["grad_names"]]
    loss, grads, _, _ = O.train_step(names, P, img, tracks, gt)
    with torch.no_grad():
        out = O.comet_forward(P, img, tracks, gt, return_all=True)
    return out, loss, grads


def test_e2e_forward_matches_reference(gold, e2e):
    out, loss, _ = e2e
    close(out["pred_tracks"], gold["e2e_pred_tracks"], 1e-6, 1e-4, "pred_tracks")
    close(out["pred_pose_enc"], gold["e2e_pred_pose_enc"], 1e-5, 1e-5, "pred_pose_enc")
    close(out["gt_pose_enc"], gold["e2e_gt_pose_enc"], 1e-6, 1e-6, "gt_pose_enc")
    close(out["loss"].reshape(1), gold["e2e_loss"], 1e-5, 1e-5, "loss")
    close(out["loss_trans"].reshape(1), gold["e2e_loss_trans"], 1e-5, 1e-5, "loss_trans")
    close(out["loss_rot"].reshape(1), gold["e2e_loss_rot"], 1e-5, 1e-5, "loss_rot")
    close(out["pred_R"], gold["e2e_pred_R"], 1e-5, 1e-5, "pred R")
    close(out["pred_T"], gold["e2e_pred_T"], 1e-5, 1e-4, "pred T")
    close(out["fmaps"].reshape(gold["e2e_fmaps"].shape), gold["e2e_fmaps"], 1e-5, 1e-5, "coarse fmaps")


def test_e2e_grads_match_reference(gold, e2e):
    _, _, grads = e2e
    names = [str(k) for k in gold["grad_names"]]
    norms = np.array([grads["camera_predictor." + k].double().norm().item() for k in names])
    close(norms, gold["grad_norms"], 2e-4, 1e-6, "grad norms")
    for k in gold:
        if k.startswith("grad_full."):
            ref = gold[k]
            close(grads["camera_predictor." + k[len("grad_full."):]], ref, 2e-4, 2e-5 * float(np.abs(ref).max()), k)


# ------------------------------------------------------------------------------------------
# round-2 fixtures: eval path at T=16 (v2) and the headline workload, stage by stage
# ------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def gold2():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "comet_golden_v2.npz"), allow_pickle=False))


@pytest.fixture(scope="module")
def full_params():
    from oracle.weights import comet_shapes
    return prng.make_state_dict(0, comet_shapes())


def test_eval_T16_matches_reference(gold2, full_params):
    seed_w, seed_x, B, T, H, W, N = [int(v) for v in gold2["eval_cfg"]]
    img, tracks, gt = prng.synthetic_batch(seed_x, B, T, H, W, N)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    with torch.no_grad():
        out = O.comet_forward(full_params, img, tracks, gt, return_all=True)
    close(out["pred_tracks"], gold2["eval_pred_tracks"], 1e-6, 1e-4, "eval tracks")
    close(out["inv_score"], gold2["eval_pred_score"], 1e-5, 1e-6, "eval pred_score")
    close(out["pred_pose_enc"], gold2["eval_pred_pose_enc"], 1e-5, 1e-5, "eval pose enc")
    close(out["loss"].reshape(1), gold2["eval_loss"], 1e-5, 1e-6, "eval loss")
    close(out["pred_T"], gold2["eval_pred_T"], 1e-5, 1e-4, "eval pred T")


def test_small_pred_score_matches_reference(gold2, full_params):
    gold1 = dict(np.load(GOLD, allow_pickle=False))
    seed_w, seed_x, B, T, H, W, N = [int(v) for v in gold1["cfg"]]
    img, tracks, gt = prng.synthetic_batch(seed_x, B, T, H, W, N)
    with torch.no_grad():
        out = O.comet_forward(full_params, img, tracks, gt, return_all=True)
    close(out["score"], gold2["e2e_track_score"], 1e-5, 1e-6, "track score")
    close(out["inv_score"], gold2["e2e_pred_score"], 1e-5, 1e-6, "pred_score")


@pytest.fixture(scope="module")
def headline():
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "comet_golden_headline.npz"), allow_pickle=False))
    seed_w, seed_x, B, T, H, W, N = [int(v) for v in g["head_cfg"]]
    img, tracks, gt = prng.synthetic_batch(seed_x, B, T, H, W, N)
    return g, img, tracks, gt


def test_headline_stages_match_reference(headline, full_params):
    """T=16, 512^2, N=512 (the bench workload per sequence): coarse tracker from scratch, refine on
    the reference's coarse tracks, camera predictor on the reference's refined tracks / scores."""
    g, img, tracks, gt = headline
    P = full_params
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    import torch.nn.functional as TF
    B, T, C, H, W = img.shape
    with torch.no_grad():
        x = TF.interpolate(img.reshape(B * T, C, H, W), scale_factor=0.5, mode="bilinear", align_corners=True)
        fm = O.basic_encoder(x, P, "track_predictor.coarse_fnet", 4)
        fm = fm.reshape(B, T, -1, fm.shape[-2], fm.shape[-1])
        preds = O.tracker_predictor(tracks[:, 0], fm, P, "track_predictor.coarse_predictor", 4, 4, 2, 5, 4, 128,
                                    False, True)[0]
        close(preds[-1], g["head_coarse"], 1e-6, 1e-3, "headline coarse tracks")
        coarse = torch.from_numpy(g["head_coarse"])
        refined, score = O.refine_track(img, P, coarse)
        close(refined, g["head_refined"], 1e-6, 1e-3, "headline refined tracks")
        close(score, g["head_score"], 1e-4, 1e-5, "headline score")
        out = O.camera_predictor(img.reshape(-1, C, H, W), B, P, gt, torch.from_numpy(g["head_refined"]),
                                 torch.from_numpy(g["head_pred_score"]))
    close(out["pred_pose_enc"], g["head_pred_pose_enc"], 1e-5, 1e-5, "headline pose enc")
    close(out["loss"].reshape(1), g["head_loss"], 1e-5, 1e-6, "headline loss")
    close(out["pred_T"], g["head_pred_T"], 1e-5, 1e-4, "headline pred T")


# ---- §8(f3) evaluation metrics: oracle vs the reference metric.py (comet_golden_metrics.npz) ----
@pytest.fixture(scope="module")
def gold_metrics():
    return dict(np.load(os.path.join(ROOT, "tests", "golden", "comet_golden_metrics.npz"), allow_pickle=False))


@pytest.mark.parametrize("tag", ["a", "b", "c"])
def test_metrics_oracle_matches_reference(gold_metrics, tag):
    g = {k[3:]: v for k, v in gold_metrics.items() if k.startswith(f"m{tag}_")}
    B = int(g["cfg"][1])
    rot, tr = O.pose_pair_errors(torch.from_numpy(g["pred_w2v"]), torch.from_numpy(g["gt_w2v"]), B)
    close(rot, g["d3_rel_rangle"], 1e-5, 1e-3, "pair rotation error (deg)")
    close(tr, g["d3_rel_tangle"], 1e-5, 1e-3, "pair translation error (deg)")
    ftr, geo, eul = O.pose_frame_errors(torch.from_numpy(g["pred_enc"]), torch.from_numpy(g["gt_enc"]))
    close(torch.rad2deg(geo), g["d2_rel_rangle"], 1e-5, 1e-3, "geodesic error (deg)")
    close(ftr, g["d2_rel_tangle"], 1e-5, 1e-3, "frame translation error (deg)")
    close(np.rad2deg(np.abs(eul.numpy()).mean(0)), g["d2_error_euler"], 1e-6, 1e-6, "mean |Euler| (deg)")


@pytest.mark.parametrize("variant", ["ours", "time", "track", "uvz", "all"])
def test_oracle_ablation_heads_match_reference(variant):
    """oracle.ablation_head (camera_predictor10 / _abl_* restated) vs the reference's
    own ablation heads (tests/golden/comet_golden_abl.npz)."""
    from oracle import prng
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "comet_golden_abl.npz"), allow_pickle=False))
    B, S, N, seed_rgb, seed_x = [int(v) for v in g["abl_cfg"]]
    shapes = {k: tuple(v) for k, v in __import__("oracle.weights", fromlist=["x"]).comet_shapes().items()
              if k.startswith("camera_predictor.") and not k.startswith("camera_predictor.backbone.")}
    if variant in ("uvz", "all"):
        shapes["camera_predictor.pose_branch.fc2.weight"] = (7, 1536)
        shapes["camera_predictor.pose_branch.fc2.bias"] = (7,)
    P = prng.make_state_dict(0, shapes)
    _, _, gt = prng.synthetic_batch(seed_x, B, S, 128, 128, N)
    o = O.ablation_head(torch.from_numpy(g["abl_rgb"]), P, variant, gt=gt,
                        pred_trajectories=torch.from_numpy(g["abl_tracks"]),
                        track_confidence=torch.from_numpy(g["abl_conf"]))
    pre = f"abl_{variant}_"
    np.testing.assert_allclose(o["pred_pose_enc"].numpy(), g[pre + "pred_pose_enc"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(o["gt_pose_enc"].numpy(), g[pre + "gt_pose_enc"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(float(o["loss"]), float(g[pre + "loss"][0]), rtol=1e-5)
    np.testing.assert_allclose(o["pred_R"].numpy(), g[pre + "pred_R"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(o["pred_T"].double().numpy(), g[pre + "pred_T"], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("variant", ["time", "track", "uvz", "all"])
def test_ablation_targets_resolve(variant):
    """The reference's abl_*.yaml `_target_` strings resolve to the build's ablation heads with the
    reference's parameter layout (pose_branch 7 outputs for the single-head variants)."""
    from comet_amd.config import resolve_target
    C = resolve_target(f"models.camera_predictor_abl_{variant}.CameraPredictor")
    assert C.__module__ == f"comet_amd.models.camera_predictor_abl_{variant}"
    assert C.SINGLE_HEAD == (variant in ("uvz", "all"))


def test_oracle_keypoint_helpers_match_reference():
    """oracle.simple_nms vs glue-factory's batched_nms and oracle.filter_keypoints vs
    the reference's filter_and_pad (RNG-free cases), tests/golden/comet_golden_kp.npz."""
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "comet_golden_kp.npz"), allow_pickle=False))
    for t in "abc":
        got = O.simple_nms(torch.from_numpy(g[f"nms{t}_in"])[:, None], int(g[f"nms{t}_r"][0]))[:, 0]
        np.testing.assert_array_equal(got.numpy(), g[f"nms{t}_out"])
    for t in "ab":
        got = O.filter_keypoints(torch.from_numpy(g[f"fp{t}_pts"]), torch.from_numpy(g[f"fp{t}_mask"]))
        np.testing.assert_array_equal(got.numpy(), g[f"fp{t}_out"])
