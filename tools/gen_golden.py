"""Generate tests/golden/*.npz from the REFERENCE itself (build container only).

    PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py

Refuses to run without /root/reference. Weights come from oracle/prng.py (seeded; fixtures
store only seeds and outputs), inputs from oracle.prng.synthetic_batch. Also cross-checks the
oracle restatement against the reference on the same inputs and prints the max differences.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import ref_harness as H  # noqa: E402
from oracle import prng  # noqa: E402
from oracle import comet_oracle as O  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden")
SEED_W, SEED_X = 0, 1
CFG_SMALL = dict(B=1, T=4, H=128, W=128, N=16)


def reference_shapes(model):
    """state_dict layout of the reference COMET in checkpoint (facebookresearch DINOv2) naming."""
    shapes = {}
    for k, v in model.state_dict().items():
        if k.startswith("camera_predictor.backbone."):
            if k == "camera_predictor.backbone.model.embeddings.cls_token":
                shapes.update(H.dinov2_fb_shapes())
            continue
        shapes[k] = tuple(v.shape)
    return shapes


def reference_state(model, seed):
    """PRNG state dict in facebookresearch naming (= product naming) + its stand-in conversion."""
    P = prng.make_state_dict(seed, reference_shapes(model))
    return P, H.fb_to_hf(P)


def np32(t):
    return t.detach().float().cpu().numpy().astype(np.float32)


def put_grad(out, prefix, k, g):
    """small grads in full; large ones as L2 norm + the first 4 rows."""
    out[prefix + "norm." + k] = np.array([g.double().norm().item()])
    out[prefix + ("" if g.numel() <= 4096 else "head.") + k] = np32(g if g.numel() <= 4096 else g.reshape(g.shape[0], -1)[:4])


def gen_end_to_end(out):
    torch.manual_seed(0)
    cfg = H.load_cfg()
    model = H.build_reference_comet(cfg)
    P, P_hf = reference_state(model, SEED_W)
    missing, unexpected = model.load_state_dict(P_hf, strict=True), None
    q = CFG_SMALL
    img, tracks, gt = prng.synthetic_batch(SEED_X, q["B"], q["T"], q["H"], q["W"], q["N"])
    QC = H.reference_module("train_eval_func_new_cp5").QuaternionCameras
    cams = QC(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
              principal_point=gt["principal_point"], ratio=gt["ratio"])
    cap = {}

    def hook(name):
        def f(m, i, o):
            cap[name] = o["x_norm_patchtokens"] if isinstance(o, dict) else o
        return f
    model.track_predictor.coarse_fnet.register_forward_hook(hook("fmaps"))
    model.track_predictor.fine_fnet.register_forward_hook(hook("patch_feat"))
    model.camera_predictor.backbone.register_forward_hook(hook("tokens"))
    model.camera_predictor.trunk.register_forward_hook(hook("trunk_out"))
    model.camera_predictor.cross_attn_block[0].register_forward_hook(hook("tp0_out"))

    pred = model(img, gt_cameras=cams, training=True, tracks=tracks,
                 tracks_visibility=torch.ones(q["B"], q["T"], q["N"], dtype=torch.bool))
    loss = pred["loss"].mean()
    model.zero_grad()
    loss.backward()
    grads = {k: p.grad for k, p in model.camera_predictor.named_parameters() if p.grad is not None}

    out["e2e_pred_pose_enc"] = np32(pred["pred_pose_enc"])
    out["e2e_gt_pose_enc"] = np32(pred["gt_pose_enc"])
    out["e2e_loss"] = np32(pred["loss"].reshape(1))
    out["e2e_loss_trans"] = np32(pred["loss_trans"].reshape(1))
    out["e2e_loss_rot"] = np32(pred["loss_rot"].reshape(1))
    out["e2e_pred_R"] = np32(pred["pred_cameras"].R)
    out["e2e_pred_T"] = np32(pred["pred_cameras"].T)
    out["e2e_pred_tracks"] = np32(pred["pred_tracks"])
    out["e2e_fmaps"] = np32(cap["fmaps"])
    pf = cap["patch_feat"]
    out["e2e_patch_feat_head"] = np32(pf[:8])
    out["e2e_patch_feat_sum"] = np32(pf.double().sum().reshape(1))
    out["e2e_patch_feat_abssum"] = np32(pf.double().abs().sum().reshape(1))
    tok = cap["tokens"]
    out["e2e_tokens_head"] = np32(tok[:, :8])
    out["e2e_tokens_sum"] = np32(tok.double().sum(dim=(1, 2)))
    out["e2e_trunk_out"] = np32(cap["trunk_out"])
    out["e2e_tp0_out"] = np32(cap["tp0_out"])
    names = sorted(grads)
    out["grad_names"] = np.array(names)
    out["grad_norms"] = np.array([grads[k].double().norm().item() for k in names])
    for k in ["fc_depth.weight", "fc_translation2d.weight", "pose_branch.fc2.weight", "pose_token",
              "trunk.3.mlp.fc2.bias", "confidence_attention.0.weight", "traj_encoder.mlp.0.weight"]:
        out["grad_full." + k] = np32(grads[k])

    # --- cross-check the oracle restatement on the same inputs ---
    gt_o = dict(gt)
    res = O.comet_forward(P, img, tracks, gt_o, return_all=True)
    diffs = {
        "pred_pose_enc": (res["pred_pose_enc"] - pred["pred_pose_enc"]).abs().max().item(),
        "loss": abs(res["loss"].item() - loss.item()),
        "pred_tracks": (res["pred_tracks"] - pred["pred_tracks"]).abs().max().item(),
        "pred_T": (res["pred_T"] - pred["pred_cameras"].T).abs().max().item(),
        "fmaps": (res["fmaps"].reshape(cap["fmaps"].shape) - cap["fmaps"]).abs().max().item(),
    }
    print("oracle vs reference (fp32):", {k: f"{v:.2e}" for k, v in diffs.items()})
    train_names = ["camera_predictor." + k for k in names]
    _, g_o, _, _ = O.train_step(train_names, P, img, tracks, gt_o)
    gd = max((g_o["camera_predictor." + k] - grads[k]).abs().max().item() / (grads[k].abs().max().item() + 1e-12) for k in names)
    print(f"oracle vs reference grads: max rel-to-max diff {gd:.2e}")

    # --- bf16 autocast run of the reference (accelerate mixed_precision='bf16') ---
    with torch.autocast("cpu", dtype=torch.bfloat16):
        pb = model(img, gt_cameras=cams, training=True, tracks=tracks,
                   tracks_visibility=torch.ones(q["B"], q["T"], q["N"], dtype=torch.bool))
    out["bf16_pred_pose_enc"] = np32(pb["pred_pose_enc"].float())
    out["bf16_loss"] = np32(pb["loss"].float().reshape(1))
    out["bf16_pred_tracks"] = np32(pb["pred_tracks"].float())
    out["cfg"] = np.array([SEED_W, SEED_X, q["B"], q["T"], q["H"], q["W"], q["N"]])
    return model, P


def gen_blocks(out):
    """G1: AttnBlock / CrossAttnBlock of modules.py with PRNG weights: outputs + all grads."""
    mod = H.reference_module("models.modules")
    torch.manual_seed(0)
    blk = mod.AttnBlock(768, 8, mlp_ratio=4)
    P = prng.make_state_dict(SEED_W + 7, {k: tuple(v.shape) for k, v in blk.state_dict().items()})
    blk.load_state_dict(P)
    x = torch.from_numpy(prng.normal_like(SEED_X + 7, "attn_x", (3, 37, 768))).requires_grad_(True)
    y = blk(x)
    gy = torch.from_numpy(prng.normal_like(SEED_X + 7, "attn_gy", (3, 37, 768)))
    y.backward(gy)
    out["blk_attn_y"] = np32(y)
    out["blk_attn_dx"] = np32(x.grad)
    for k, p in blk.named_parameters():
        put_grad(out, "blk_attn_grad.", k, p.grad)
    cblk = mod.CrossAttnBlock(768, 768, 8, mlp_ratio=4)
    P = prng.make_state_dict(SEED_W + 8, {k: tuple(v.shape) for k, v in cblk.state_dict().items()})
    cblk.load_state_dict(P)
    x = torch.from_numpy(prng.normal_like(SEED_X + 8, "cx", (2, 29, 768))).requires_grad_(True)
    c = torch.from_numpy(prng.normal_like(SEED_X + 8, "cc", (2, 41, 768))).requires_grad_(True)
    y = cblk(x, c)
    gy = torch.from_numpy(prng.normal_like(SEED_X + 8, "cgy", (2, 29, 768)))
    y.backward(gy)
    out["blk_cross_y"] = np32(y)
    out["blk_cross_dx"] = np32(x.grad)
    out["blk_cross_dctx"] = np32(c.grad)
    for k, p in cblk.named_parameters():
        put_grad(out, "blk_cross_grad.", k, p.grad)


def gen_exact(out):
    """G5: sincos tables, HarmonicEmbedding, pose codec vectors straight from the reference."""
    ut = H.reference_module("utils")
    he = H.reference_module("minipytorch3d.harmonic_embedding")
    out["sincos_1d_768_16"] = np32(ut.get_1d_sincos_pos_embed(768, 16))
    out["sincos_2d_768_24"] = np32(ut.get_2d_sincos_pos_embed(768, (24, 24)))
    out["sincos_2d_664_16"] = np32(ut.get_2d_sincos_pos_embed(664, (16, 16)))
    xy = torch.from_numpy(prng.uniform(SEED_X, "flows", (5, 7, 2)) * 20)
    out["embed2d_in"] = np32(xy)
    out["embed2d_64"] = np32(ut.get_2d_embedding(xy, 64, cat_coords=False))
    x = torch.from_numpy(prng.uniform(SEED_X, "harm_x", (4, 5, 8)) * 3)
    cov = torch.from_numpy(np.abs(prng.uniform(SEED_X, "harm_cov", (4, 5, 8))) * 0.1)
    out["harm_x"] = np32(x)
    out["harm_cov"] = np32(cov)
    for n, om, logs, app in [(6, 1.0, True, True), (48, 1.0, True, False), (10, 0.5, False, True)]:
        m = he.HarmonicEmbedding(n_harmonic_functions=n, omega_0=om, logspace=logs, append_input=app)
        tag = f"harm_{n}_{om}_{int(logs)}_{int(app)}"
        out[tag] = np32(m(x))
        out[tag + "_cov"] = np32(m(x, diag_cov=cov))
    # pose codec (utils.py:312-403, 631-688) for one 6-frame sequence
    _, _, gt = prng.synthetic_batch(SEED_X + 3, 1, 6, 64, 64, 4)
    QC = H.reference_module("train_eval_func_new_cp5").QuaternionCameras
    cams = QC(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
              principal_point=gt["principal_point"], ratio=gt["ratio"])
    enc = ut.camera_to_pose_encoding2(cams)
    out["codec_gt_R"] = np32(gt["R"])
    out["codec_gt_Tuvz"] = np32(gt["T_uvz"])
    out["codec_enc"] = np32(enc)
    penc = torch.from_numpy(prng.uniform(SEED_X + 3, "penc", (1, 6, 7)) * 0.3)
    penc[..., 3:7] = torch.nn.functional.normalize(penc[..., 3:7] + torch.tensor([1.0, 0, 0, 0]), dim=-1)
    out["codec_penc"] = np32(penc)
    for it in ["AMD_eval", "AMD_test", "spark"]:
        pc = ut.pose_encoding_to_camera2(penc, gt_cameras=cams, pose_encoding_type="absT_quaR_OneFL",
                                         to_OpenCV=False, intri_type=it)
        out[f"codec_dec_R_{it}"] = np32(pc.R)
        out[f"codec_dec_T_{it}"] = np32(pc.T)


CFG_EVAL = dict(B=1, T=16, H=128, W=128, N=16)


def _capture_score(E2E):
    """Wrap the reference's refine_track (as E2Epose2 imported it) to record track_score."""
    cap = {}
    orig = E2E.refine_track

    def wrapped(*a, **k):
        r = orig(*a, **k)
        cap["score"] = r[1]
        return r
    E2E.refine_track = wrapped
    return cap, orig


def gen_v2(out):
    """Round-2 fixtures (tests/golden/comet_golden_v2.npz):
    * e2e (CFG_SMALL, fp32): the reference's predictions["pred_score"] (inverted, normalised score);
    * e2e bf16 autocast: pose enc, loss and the camera-predictor gradients (norms + a few full);
    * eval path (BASELINE configs[0] shape: abl_ours.py test_fn -> model(..., training=False), B=1,
      T=16; frames 128^2, N=16): pose enc, tracks, loss, and get_world_to_view_transform().get_matrix()
      of the predicted and GT cameras (metric.py:155-156, 219-221);
    * WarmupCosineRestarts (train_util.py:2099-2128) lr sequences for three settings."""
    E2E = H.reference_module("E2Epose2")
    cap, orig = _capture_score(E2E)
    try:
        torch.manual_seed(0)
        cfg = H.load_cfg()
        model = H.build_reference_comet(cfg)
        P, P_hf = reference_state(model, SEED_W)
        model.load_state_dict(P_hf, strict=True)
        QC = H.reference_module("train_eval_func_new_cp5").QuaternionCameras
        q = CFG_SMALL
        img, tracks, gt = prng.synthetic_batch(SEED_X, q["B"], q["T"], q["H"], q["W"], q["N"])
        cams = QC(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
                  principal_point=gt["principal_point"], ratio=gt["ratio"])
        vis = torch.ones(q["B"], q["T"], q["N"], dtype=torch.bool)
        with torch.no_grad():
            model(img, gt_cameras=cams, training=True, tracks=tracks, tracks_visibility=vis)
        s = cap["score"]
        inv = 1.0 / (s + 1e-6)
        out["e2e_track_score"] = np32(s)
        out["e2e_pred_score"] = np32(inv / inv.max(dim=1, keepdim=True)[0])
        # bf16 autocast forward + backward (accelerate mixed_precision="bf16")
        model.zero_grad()
        with torch.autocast("cpu", dtype=torch.bfloat16):
            pb = model(img, gt_cameras=cams, training=True, tracks=tracks, tracks_visibility=vis)
        pb["loss"].float().mean().backward()
        grads = {k: p.grad.float() for k, p in model.camera_predictor.named_parameters() if p.grad is not None}
        names = sorted(grads)
        out["bf16_grad_names"] = np.array(names)
        out["bf16_grad_norms"] = np.array([grads[k].double().norm().item() for k in names])
        for k in ["fc_depth.weight", "fc_translation2d.weight", "pose_branch.fc2.weight", "trunk.3.mlp.fc2.bias",
                  "confidence_attention.0.weight"]:
            out["bf16_grad_full." + k] = np32(grads[k])
        out["bf16_pred_pose_enc"] = np32(pb["pred_pose_enc"].float())
        out["bf16_loss"] = np32(pb["loss"].float().reshape(1))
        model.zero_grad()
        # eval path at T=16
        e = CFG_EVAL
        img, tracks, gt = prng.synthetic_batch(SEED_X + 20, e["B"], e["T"], e["H"], e["W"], e["N"])
        cams = QC(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
                  principal_point=gt["principal_point"], ratio=gt["ratio"])
        pe = model(img, gt_cameras=cams, training=False, tracks=tracks,
                   tracks_visibility=torch.ones(e["B"], e["T"], e["N"], dtype=torch.bool))
        out["eval_cfg"] = np.array([SEED_W, SEED_X + 20, e["B"], e["T"], e["H"], e["W"], e["N"]])
        out["eval_pred_pose_enc"] = np32(pe["pred_pose_enc"])
        out["eval_gt_pose_enc"] = np32(pe["gt_pose_enc"])
        out["eval_pred_tracks"] = np32(pe["pred_tracks"])
        out["eval_loss"] = np32(pe["loss"].reshape(1))
        out["eval_pred_R"] = np32(pe["pred_cameras"].R)
        out["eval_pred_T"] = pe["pred_cameras"].T.detach().double().cpu().numpy()
        out["eval_pred_w2v"] = np32(pe["pred_cameras"].get_world_to_view_transform().get_matrix())
        out["eval_gt_w2v"] = np32(cams.get_world_to_view_transform().get_matrix())
        inv = 1.0 / (cap["score"] + 1e-6)
        out["eval_pred_score"] = np32(inv / inv.max(dim=1, keepdim=True)[0])
        # oracle cross-check on the eval inputs
        res = O.comet_forward(P, img, tracks, dict(gt))
        print("oracle vs reference (eval T=16):",
              f"pose enc {(res['pred_pose_enc'] - pe['pred_pose_enc']).abs().max().item():.2e}",
              f"tracks {(res['pred_tracks'] - pe['pred_tracks']).abs().max().item():.2e}")
    finally:
        E2E.refine_track = orig
    # lr schedule
    tu = _reference_train_util()
    for tag, kw, n in [("a", dict(T_0=3, iters_per_epoch=4, warmup_ratio=0.25, warmup_lr_init=1e-7), 30),
                       ("b", dict(T_0=320, iters_per_epoch=2, warmup_ratio=0.0, warmup_lr_init=1e-7), 50),
                       ("c", dict(T_0=2, iters_per_epoch=3, T_mult=2, warmup_ratio=0.1, warmup_lr_init=1e-6,
                                  eta_min=1e-7), 40)]:
        opt = torch.optim.AdamW([torch.nn.Parameter(torch.zeros(1))], lr=1e-5)
        sch = tu.WarmupCosineRestarts(opt, **kw)
        lrs = []
        for _ in range(n):
            lrs.append(sch.get_last_lr()[0])
            opt.step()
            sch.step()
        out[f"lr_sched_{tag}"] = np.array(lrs, dtype=np.float64)


def _reference_train_util():
    """train_util.py imports heavy optional packages at module level; load only the scheduler class
    source out of it (the class body is executed in a namespace with math + torch)."""
    import ast
    import math
    src = open(os.path.join(H.REF, "comet", "models", "train_util.py")).read()
    tree = ast.parse(src)
    node = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "WarmupCosineRestarts")
    ns = {"math": math, "torch": torch}
    exec(compile(ast.Module(body=[node], type_ignores=[]), "train_util.py", "exec"), ns)
    return types_ns(WarmupCosineRestarts=ns["WarmupCosineRestarts"])


def types_ns(**kw):
    import types
    return types.SimpleNamespace(**kw)


CFG_HEAD = dict(B=1, T=16, H=512, W=512, N=512)


def gen_headline(out):
    """Headline workload (BASELINE configs[1]/[2] per sequence: T=16, 512^2, N=512), B=1 (the
    reference cannot run B>1), PRNG weights seed 0, inputs seed 1 (tests/golden/comet_golden_headline.npz).
    Stage tensors are stored so the GPU test can pin each stage on the reference's own inputs
    (the refine step floors coarse tracks: an fp32 ulp near an integer picks another patch):
      coarse tracks -> (refine_track) refined tracks, raw + inverted score -> (camera_predictor)
      pose enc, loss, gradients; plus the bf16-autocast end-to-end pose enc / loss."""
    E2E = H.reference_module("E2Epose2")
    cap = {}
    orig = E2E.refine_track

    def wrapped(images, fnet, fpred, coarse, **k):
        r = orig(images, fnet, fpred, coarse, **k)
        cap["coarse"] = coarse.detach().clone()
        cap["refined"], cap["score"] = r[0].detach().clone(), r[1].detach().clone()
        return r
    E2E.refine_track = wrapped
    try:
        torch.manual_seed(0)
        cfg = H.load_cfg()
        model = H.build_reference_comet(cfg)
        P, P_hf = reference_state(model, SEED_W)
        model.load_state_dict(P_hf, strict=True)
        del P, P_hf
        QC = H.reference_module("train_eval_func_new_cp5").QuaternionCameras
        q = CFG_HEAD
        img, tracks, gt = prng.synthetic_batch(SEED_X, q["B"], q["T"], q["H"], q["W"], q["N"])
        cams = QC(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
                  principal_point=gt["principal_point"], ratio=gt["ratio"])
        vis = torch.ones(q["B"], q["T"], q["N"], dtype=torch.bool)
        import time
        t0 = time.time()
        pred = model(img, gt_cameras=cams, training=True, tracks=tracks, tracks_visibility=vis)
        model.zero_grad()
        pred["loss"].mean().backward()
        print(f"reference fp32 train step at headline size: {time.time() - t0:.1f} s")
        grads = {k: p.grad for k, p in model.camera_predictor.named_parameters() if p.grad is not None}
        names = sorted(grads)
        inv = 1.0 / (cap["score"] + 1e-6)
        out["head_cfg"] = np.array([SEED_W, SEED_X, q["B"], q["T"], q["H"], q["W"], q["N"]])
        out["head_coarse"] = np32(cap["coarse"])
        out["head_refined"] = np32(cap["refined"])
        out["head_score"] = np32(cap["score"])
        out["head_pred_score"] = np32(inv / inv.max(dim=1, keepdim=True)[0])
        out["head_pred_pose_enc"] = np32(pred["pred_pose_enc"])
        out["head_gt_pose_enc"] = np32(pred["gt_pose_enc"])
        out["head_loss"] = np32(pred["loss"].reshape(1))
        out["head_loss_trans"] = np32(pred["loss_trans"].reshape(1))
        out["head_loss_rot"] = np32(pred["loss_rot"].reshape(1))
        out["head_pred_T"] = pred["pred_cameras"].T.detach().double().numpy()
        out["head_grad_names"] = np.array(names)
        out["head_grad_norms"] = np.array([grads[k].double().norm().item() for k in names])
        for k in ["fc_depth.weight", "fc_translation2d.weight", "pose_branch.fc2.weight", "trunk.3.mlp.fc2.bias",
                  "confidence_attention.0.weight", "traj_encoder.mlp.0.weight", "pose_token"]:
            out["head_grad_full." + k] = np32(grads[k])
        del pred, grads
        model.zero_grad(set_to_none=True)
        t0 = time.time()
        with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
            pb = model(img, gt_cameras=cams, training=True, tracks=tracks, tracks_visibility=vis)
        print(f"reference bf16 forward at headline size: {time.time() - t0:.1f} s")
        out["head_bf16_pred_pose_enc"] = np32(pb["pred_pose_enc"].float())
        out["head_bf16_loss"] = np32(pb["loss"].float().reshape(1))
        out["head_bf16_refined"] = np32(pb["pred_tracks"].float())
    finally:
        E2E.refine_track = orig


HEAD_BF16_FULL = ["fc_depth.weight", "fc_translation2d.weight", "pose_branch.fc2.weight", "trunk.3.mlp.fc2.bias",
                  "confidence_attention.0.weight", "traj_encoder.mlp.0.weight", "pose_token",
                  "trunk.0.attn.in_proj_weight", "cross_att.3.cross_attn.in_proj_weight", "self_att.0.mlp.fc1.weight"]


def _rows(g, n=48):
    """a gradient in full when small, else its first n rows (the fixture stays small)"""
    return np32(g if g.numel() <= 65536 else g.reshape(g.shape[0], -1)[:n])


def gen_headline_bf16_head(out):
    """The product's training precision at the headline size: the reference camera head
    (camera_predictor10.py:288-460) forward under torch.autocast(bfloat16) -- accelerate's
    mixed_precision="bf16" wraps the forward only -- and the backward of its loss, on the
    reference's own fp32 stage inputs stored by gen_headline (refined tracks, pred_score), PRNG
    weights seed 0: pose enc, loss, the 169 gradient norms and selected full gradients."""
    torch.manual_seed(0)
    cfg = H.load_cfg()
    model = H.build_reference_comet(cfg)
    P, P_hf = reference_state(model, SEED_W)
    model.load_state_dict(P_hf, strict=True)
    del P, P_hf
    QC = H.reference_module("train_eval_func_new_cp5").QuaternionCameras
    q = CFG_HEAD
    img, tracks, gt = prng.synthetic_batch(SEED_X, q["B"], q["T"], q["H"], q["W"], q["N"])
    cams = QC(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
              principal_point=gt["principal_point"], ratio=gt["ratio"])
    refined = torch.from_numpy(out["head_refined"])
    conf = torch.from_numpy(out["head_pred_score"])
    cp = model.camera_predictor
    import time
    t0 = time.time()
    with torch.autocast("cpu", dtype=torch.bfloat16):
        pred = cp(img.reshape(-1, *img.shape[2:]), batch_size=q["B"], gt_cameras=cams, iters=cfg.camera_iter,
                  pred_trajectories=refined, track_confidence=conf)
    model.zero_grad()
    pred["loss"].mean().float().backward()
    print(f"reference bf16 camera head fwd+bwd at headline size: {time.time() - t0:.1f} s")
    grads = {k: p.grad for k, p in cp.named_parameters() if p.grad is not None}
    names = sorted(grads)
    assert names == [str(k) for k in out["head_grad_names"]], "bf16 and fp32 runs must grade the same params"
    out["head_bf16h_pred_pose_enc"] = np32(pred["pred_pose_enc"].float())
    out["head_bf16h_loss"] = np32(pred["loss"].float().reshape(1))
    out["head_bf16h_loss_trans"] = np32(pred["loss_trans"].float().reshape(1))
    out["head_bf16h_loss_rot"] = np32(pred["loss_rot"].float().reshape(1))
    out["head_bf16h_grad_norms"] = np.array([grads[k].double().norm().item() for k in names])
    for k in HEAD_BF16_FULL:
        out["head_bf16h_grad_full." + k] = _rows(grads[k])
    # the same selection from an fp32 pass, so the test can bound the reference's own bf16 deviation
    model.zero_grad()
    pred32 = cp(img.reshape(-1, *img.shape[2:]), batch_size=q["B"], gt_cameras=cams, iters=cfg.camera_iter,
                pred_trajectories=refined, track_confidence=conf)
    pred32["loss"].mean().backward()
    for k in HEAD_BF16_FULL:
        out["head_fp32h_grad_full." + k] = _rows(cp.get_parameter(k).grad)


def main_headline_bf16_head():
    """Adds the head_bf16h_* arrays to the existing comet_golden_headline.npz (its fp32 stage
    tensors are the inputs)."""
    H.require_reference()
    torch.set_num_threads(8)
    path = os.path.join(OUT, "comet_golden_headline.npz")
    out = dict(np.load(path, allow_pickle=False))
    gen_headline_bf16_head(out)
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes,", len(out), "arrays")


def main_headline():
    H.require_reference()
    torch.set_num_threads(8)
    out = {}
    gen_headline(out)
    path = os.path.join(OUT, "comet_golden_headline.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes,", len(out), "arrays")


def main_v2():
    H.require_reference()
    torch.set_num_threads(8)
    out = {}
    gen_v2(out)
    path = os.path.join(OUT, "comet_golden_v2.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes,", len(out), "arrays")


def _metric_case(seed, B, S):
    """Synthetic eval outputs for the metric fixtures: world-to-view matrices [[R, 0], [T, 1]] (f32)
    of GT and predicted cameras, absolute T, and 7/8-column pose encodings, with edge cases: exact
    matches (zero error), a 180-degree flip, a 90-degree pitch (Euler singularity) and a zero
    translation."""
    from minipytorch3d import rotation_conversions as rc
    g = torch.Generator().manual_seed(seed)
    n = B * S
    qg = torch.randn(n, 4, generator=g)
    qg = qg / qg.norm(dim=-1, keepdim=True)
    dq = torch.randn(n, 4, generator=g) * torch.rand(n, 1, generator=g) * 0.3
    qp = qg + dq
    qp = qp / qp.norm(dim=-1, keepdim=True)
    qp[0] = qg[0]                                     # exact match
    qp[3] = torch.tensor([qg[3, 1], -qg[3, 0], qg[3, 3], -qg[3, 2]])  # 180-degree relative flip
    qp[5] = torch.tensor([0.7071068, 0.0, 0.7071068, 0.0])            # 90-degree pitch
    Tg = torch.randn(n, 3, generator=g) * 2
    Tp = Tg + torch.randn(n, 3, generator=g) * 0.2
    Tp[0] = Tg[0]
    Tp[7] = 0.0                                       # zero translation
    def w2v(q, T):
        M = torch.zeros(n, 4, 4)
        M[:, :3, :3] = rc.quaternion_to_matrix(q)
        M[:, 3, :3] = T
        M[:, 3, 3] = 1.0
        return M
    enc_g = torch.cat([torch.randn(n, 3, generator=g), qg, torch.zeros(n, 1)], 1)
    enc_p = torch.cat([enc_g[:, :3] + torch.randn(n, 3, generator=g) * 0.1, qp], 1)
    enc_p[0] = enc_g[0, :7]
    enc_p[2, :3] = 0.0
    return w2v(qp, Tp), w2v(qg, Tg), Tp.double(), Tg, enc_p, enc_g


class _Cams:
    """The two camera attributes metric.py reads: .T and get_world_to_view_transform().get_matrix()."""
    def __init__(self, M, T):
        self.T, self._M = T, M

    def get_world_to_view_transform(self):
        return self

    def get_matrix(self):
        return self._M


def gen_metrics(out):
    """SURVEY §8(f3) fixtures (tests/golden/comet_golden_metrics.npz): the reference metric.py on
    synthetic eval outputs -- camera_to_rel_deg3, camera_to_rel_deg2 (the binding metric.py leaves in
    effect), calculate_auc, and the eval block of train_eval_func_new_cp5.py:633-671."""
    H.install_stubs()
    M = H.reference_module("metric")
    cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self  # metric.py:337-338 hard-codes .cuda()
    try:
        for tag, (seed, B, S) in {"a": (11, 1, 16), "b": (12, 4, 16), "c": (13, 2, 64)}.items():
            Mp, Mg, Tp, Tg, ep, eg = _metric_case(seed, B, S)
            pc, gc = _Cams(Mp, Tp), _Cams(Mg, Tg)
            r3 = M.camera_to_rel_deg3(pc, gc, "cpu", B)
            r2 = M.camera_to_rel_deg2(ep, eg, "cpu", B)
            auc, hist = M.calculate_auc(r3[0], r3[1], max_threshold=30, return_list=True)
            pre = f"m{tag}_"
            out[pre + "cfg"] = np.array([seed, B, S])
            out[pre + "pred_w2v"], out[pre + "gt_w2v"] = np32(Mp), np32(Mg)
            out[pre + "pred_T"], out[pre + "gt_T"] = Tp.numpy(), np32(Tg)
            out[pre + "pred_enc"], out[pre + "gt_enc"] = np32(ep), np32(eg)
            for k, v in zip(["rel_rangle", "rel_tangle", "T_avg", "Tx", "Ty", "Tz"], r3):
                out[pre + "d3_" + k] = np.asarray(v.detach().double().numpy())
            out[pre + "d2_rel_rangle"] = r2[0].double().numpy()
            out[pre + "d2_rel_tangle"] = r2[1].double().numpy()
            out[pre + "d2_avg"] = np.array([float(r2[2])])
            out[pre + "d2_error_euler"] = np.asarray(r2[3], dtype=np.float64)
            out[pre + "d2_acc5"] = np.asarray(r2[4], dtype=np.float64)
            out[pre + "auc30"] = np.array([float(auc)])
            out[pre + "hist"] = hist.double().numpy()
            for th in (30, 10, 5, 3):
                out[pre + f"auc_{th}"] = np.array([float(torch.cumsum(hist[:th], dim=0).mean())])
            print(tag, "pairs", r3[0].numel(), "auc30", float(auc), "R_avg", float(r2[2]))
    finally:
        torch.Tensor.cuda = cuda


CFG_LOOP = dict(B=1, T=4, H=128, W=128, N=256, steps=2)


def _reference_functions(names):
    """Top-level functions / classes of train_util.py (whose module imports heavy optional
    packages) executed from their source in a namespace with math + torch + F."""
    import ast
    import math
    import torch.nn.functional as Fn
    src = open(os.path.join(H.REF, "comet", "models", "train_util.py")).read()
    tree = ast.parse(src)
    nodes = [n for n in tree.body if isinstance(n, (ast.ClassDef, ast.FunctionDef)) and n.name in names]
    ns = {"math": math, "torch": torch, "F": Fn, "np": np}
    exec(compile(ast.Module(body=nodes, type_ignores=[]), "train_util.py", "exec"), ns)
    return ns


def gen_loop(out):
    """SURVEY §8(c) caller counterpart: the reference's own train_or_eval_fn
    (train_eval_func_new_cp5.py:514-823, training branch) for two steps at the golden size -- keypoint
    tracks from a SuperPoint stub with fixed keypoints (lightglue is absent; SIFT stubbed empty),
    process_spark_data2, QuaternionCameras, forward, loss.mean(), the eval-metric block, then
    zero_grad -> backward (anomaly mode at step 0) -> clip_grad_norm_(1.0) -> AdamW -> scheduler
    (train_util.build_optimizer), PRNG weights seed 0, fp32. Records the per-step losses, the pre-clip
    gradient norms, the learning rates and the parameter updates of the camera predictor."""
    H.install_stubs()
    q = CFG_LOOP
    cfg = H.load_cfg()
    cfg["track_by_spsg"] = True
    cfg["enable_track"] = True
    cfg["labor_input_traj"] = False
    cfg["visual_track"] = False
    cfg["visual_pose"] = False
    cfg["train"]["track_num"] = q["N"]
    cfg["train"]["print_interval"] = 1
    cfg["train"]["dataset"] = "AMD"
    torch.manual_seed(0)
    model = H.build_reference_comet(cfg)
    P, P_hf = reference_state(model, SEED_W)
    model.load_state_dict(P_hf, strict=True)
    M = H.reference_module("train_eval_func_new_cp5")
    ns = _reference_functions({"process_spark_data2", "WarmupCosineRestarts", "build_optimizer"})
    M.process_spark_data2 = ns["process_spark_data2"]
    batches = prng.loop_batches(SEED_X, **{k: q[k] for k in ("B", "T", "H", "W", "N", "steps")})
    kp_iter = iter([b.pop("kp0") for b in batches])

    class SP:  # lightglue.SuperPoint stand-in: the fixed keypoints of each batch
        def __init__(self, *a, **k):
            pass

        def cuda(self):
            return self

        def eval(self):
            return self

        def extract(self, img):
            return {"keypoints": next(kp_iter)[None]}

    class SIFT(SP):
        def extract(self, img):
            return {"keypoints": torch.zeros(1, 0, 2)}

    M.SuperPoint, M.SIFT = SP, SIFT

    class Stats:
        def update(self, *a, **k):
            pass

        def get_status_string(self, *a, **k):
            return ""

    rec = {"loss": [], "norm": [], "lr": []}

    class Acc:
        device = torch.device("cpu")

        def print(self, *a, **k):
            pass

        def backward(self, loss):
            rec["loss"].append(float(loss.detach()))
            loss.backward()

        def clip_grad_norm_(self, params, max_norm):
            n = torch.nn.utils.clip_grad_norm_(params, max_norm)
            rec["norm"].append(float(n))
            return n

    optimizer, sched = ns["build_optimizer"](cfg, model, batches)
    before = {k: p.detach().clone() for k, p in model.camera_predictor.named_parameters()}
    orig_step = sched.step

    def step_rec(*a, **k):
        orig_step(*a, **k)
        rec["lr"].append(sched.get_last_lr()[0])
    sched.step = step_rec
    cuda = torch.Tensor.cuda
    torch.Tensor.cuda = lambda self, *a, **k: self  # metric.py:337-338 hard-codes .cuda()
    try:
        M.train_or_eval_fn(model, batches, cfg, optimizer, Stats(), Acc(), sched, training=True, epoch=0)
    finally:
        torch.Tensor.cuda = cuda
    names = [k for k, p in model.camera_predictor.named_parameters()]
    delta = {k: (p.detach().double() - before[k].double()) for k, p in model.camera_predictor.named_parameters()}
    out["loop_cfg"] = np.array([SEED_W, SEED_X, q["B"], q["T"], q["H"], q["W"], q["N"], q["steps"]])
    out["loop_loss"] = np.array(rec["loss"])
    out["loop_grad_norm"] = np.array(rec["norm"])
    out["loop_lr"] = np.array(rec["lr"])
    out["loop_names"] = np.array(names)
    out["loop_delta_norms"] = np.array([delta[k].norm().item() for k in names])
    for k in ["fc_depth.weight", "pose_token", "trunk.3.mlp.fc2.bias", "confidence_attention.0.weight",
              "traj_encoder.mlp.0.weight", "pose_branch.fc2.weight"]:
        out["loop_delta." + k] = delta[k].numpy()
    print("loop golden: losses", rec["loss"], "pre-clip norms", rec["norm"], "lr", rec["lr"],
          "updated params", int(sum(d.abs().max().item() > 0 for d in delta.values())), "of", len(names))


def main_loop():
    H.require_reference()
    torch.set_num_threads(8)
    out = {}
    gen_loop(out)
    path = os.path.join(OUT, "comet_golden_loop.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes,", len(out), "arrays")


def main_metrics():
    H.require_reference()
    torch.set_num_threads(8)
    out = {}
    gen_metrics(out)
    path = os.path.join(OUT, "comet_golden_metrics.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes,", len(out), "arrays")


ABL_CFG = dict(B=1, S=4, N=16, seed_rgb=21, seed_x=1)


def gen_ablations(out):
    """SURVEY §8(f4) fixtures (tests/golden/comet_golden_abl.npz): the reference's ablation heads
    (camera_predictor_abl_{time,track,uvz,all}.py, selected by abl_*.yaml) and camera_predictor10
    itself, from a PRNG rgb_feat_init (the forward's own entry for precomputed image features,
    camera_predictor_abl_*.py forward), PRNG tracks / confidences / GT cameras: outputs, losses,
    decoded cameras and every parameter gradient's norm. Weights: oracle.prng per key name (same
    values as the COMET goldens for shared keys)."""
    H.install_stubs()
    q = ABL_CFG
    B, S, N = q["B"], q["S"], q["N"]
    rgb = torch.from_numpy(prng.normal_like(q["seed_rgb"], "rgb_feat", (B, S, 768)))
    _, tracks, gt = prng.synthetic_batch(q["seed_x"], B, S, 128, 128, N)
    conf = torch.from_numpy((prng.uniform(q["seed_rgb"], "conf", (B, S, N)) + 1.0) * 0.5)
    QC = H.reference_module("train_eval_func_new_cp5").QuaternionCameras
    out["abl_cfg"] = np.array([B, S, N, q["seed_rgb"], q["seed_x"]])
    out["abl_rgb"], out["abl_tracks"], out["abl_conf"] = np32(rgb), np32(tracks), np32(conf)
    for v, (mod, yml) in {"ours": ("models.camera_predictor10", "abl_ours.yaml"),
                          "time": ("models.camera_predictor_abl_time", "abl_time.yaml"),
                          "track": ("models.camera_predictor_abl_track", "abl_track.yaml"),
                          "uvz": ("models.camera_predictor_abl_uvz", "abl_uvz.yaml"),
                          "all": ("models.camera_predictor_abl_all", "abl_all.yaml")}.items():
        cfg = H.load_cfg(yml)
        M = H.reference_module(mod)
        M.CameraPredictor.get_backbone = lambda self, b: H.make_standin()
        kw = {k: val for k, val in cfg.MODEL.CAMERA.items() if k != "_target_"}
        torch.manual_seed(0)
        cp = M.CameraPredictor(cfg=cfg, **kw)
        shapes = {"camera_predictor." + k: tuple(t.shape) for k, t in cp.state_dict().items()
                  if not k.startswith("backbone.")}
        P = prng.make_state_dict(SEED_W, shapes)
        cp.load_state_dict({k[len("camera_predictor."):]: t for k, t in P.items()}, strict=False)
        cams = QC(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
                  principal_point=gt["principal_point"], ratio=gt["ratio"])
        pred = cp(None, batch_size=B, rgb_feat_init=rgb, gt_cameras=cams, pred_trajectories=tracks,
                  track_confidence=conf)
        cp.zero_grad()
        pred["loss"].backward()
        grads = {k: p.grad for k, p in cp.named_parameters() if p.grad is not None}
        pre = f"abl_{v}_"
        out[pre + "pred_pose_enc"] = np32(pred["pred_pose_enc"])
        out[pre + "gt_pose_enc"] = np32(pred["gt_pose_enc"])
        for k in ("loss", "loss_trans", "loss_rot"):
            out[pre + k] = np32(pred[k].reshape(1))
        out[pre + "pred_R"] = np32(pred["pred_cameras"].R)
        out[pre + "pred_T"] = np32(pred["pred_cameras"].T)
        names = sorted(grads)
        out[pre + "grad_names"] = np.array(names)
        out[pre + "grad_norms"] = np.array([grads[k].double().norm().item() for k in names])
        o = O.ablation_head(rgb, P, v, gt=gt, pred_trajectories=tracks, track_confidence=conf)
        diffs = {"pred_pose_enc": (o["pred_pose_enc"] - pred["pred_pose_enc"]).abs().max().item(),
                 "loss": abs(o["loss"].item() - pred["loss"].item()),
                 "pred_R": (o["pred_R"] - pred["pred_cameras"].R).abs().max().item(),
                 "pred_T": (o["pred_T"].double() - pred["pred_cameras"].T.double()).abs().max().item()}
        print(v, "grads", len(names), "loss", float(pred["loss"]), "oracle vs reference:",
              {k: f"{x:.2e}" for k, x in diffs.items()})


DATA_CASES = {"a": (0, "model0/seq_0", (64, 64), 4), "b": (5, "model0/seq_1", (64, 64), 4),
              "c": (7, "model0/seq_0", (48, 80), 6), "d": (3, "model0/seq_1", (32, 32), 12)}


def gen_data(out):
    """SURVEY §8(f2) fixtures (tests/golden/comet_golden_data.npz): the reference's
    YTDataset.load_images_from_folder (kubric_movif_SFM_dataset_YT.py:160-266) on the synthetic
    sequences of tests/yt_fixture.py (PNG frames / masks, GT text), np.random seeded per case."""
    import tempfile
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import yt_fixture
    H.install_stubs()
    Y = H.reference_module("kubric_movif_SFM_dataset_YT")
    with tempfile.TemporaryDirectory() as root:
        yt_fixture.make_dataset(root)
        for tag, (seed, seq, crop, T) in DATA_CASES.items():
            ds = Y.YTDataset(root, crop_size=crop, seq_len=T)
            np.random.seed(seed)
            smp = ds.load_images_from_folder(seq)
            pre = f"d{tag}_"
            out[pre + "cfg"] = np.array([seed, crop[0], crop[1], T])
            out[pre + "seq"] = np.array(seq)
            for k in ("images", "T", "R", "T_uvz", "R_matrix"):
                out[pre + k] = np32(smp[k])
            out[pre + "first_mask"] = smp["first_mask"].numpy()
            out[pre + "ratio"] = np.array([smp["ratio"]], dtype=np.float64)
            out[pre + "image_names"] = np.array(smp["image_names"])
            print(tag, seq, tuple(smp["images"].shape), "ratio", smp["ratio"], smp["image_names"])


def main_data():
    H.require_reference()
    out = {}
    gen_data(out)
    path = os.path.join(OUT, "comet_golden_data.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes,", len(out), "arrays")


def gen_keypoints(out):
    """SURVEY §8(f1) fixtures (tests/golden/comet_golden_kp.npz): glue-factory's batched_nms (the
    reference tree's copy of LightGlue's simple_nms, gluefactory/models/extractors/superpoint_open.py)
    on score maps with plateaus, and the reference's filter_and_pad
    (train_eval_func_new_cp5.py:261-314) on keypoint sets whose kept count needs no random padding
    or subsetting (the RNG-free branch; the random branches are checked by property)."""
    import importlib.util
    import types
    H.install_stubs()
    # load superpoint_open.py alone: its package imports (base_model -> OmegaConf) are stubbed
    for name in ("gluefactory", "gluefactory.models", "gluefactory.models.extractors", "gluefactory.models.utils"):
        mod = types.ModuleType(name)
        mod.__path__ = []
        sys.modules.setdefault(name, mod)
    sys.modules["gluefactory.models.base_model"] = types.SimpleNamespace(BaseModel=torch.nn.Module)
    sys.modules["gluefactory.models.utils.misc"] = types.SimpleNamespace(pad_and_stack=None)
    path = os.path.join(H.REF, "gluefactory", "models", "extractors", "superpoint_open.py")
    spec = importlib.util.spec_from_file_location("gluefactory.models.extractors.superpoint_open", path)
    sp_mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sp_mod)
    batched_nms = sp_mod.batched_nms
    g = torch.Generator().manual_seed(31)
    for tag, (B, Hh, Ww, r) in {"a": (2, 48, 64, 4), "b": (1, 40, 40, 1), "c": (1, 33, 70, 2)}.items():
        sc = torch.rand(B, Hh, Ww, generator=g)
        sc = torch.where(sc < 0.3, torch.zeros_like(sc), (sc * 8).floor() / 8)  # plateaus and ties
        out[f"nms{tag}_in"] = sc.numpy()
        out[f"nms{tag}_r"] = np.array([r])
        out[f"nms{tag}_out"] = batched_nms(sc, r).numpy()
    T = H.reference_module("train_eval_func_new_cp5")
    for tag, (Hh, Ww, n, lo, hi) in {"a": (64, 80, 300, 10, 400), "b": (50, 50, 120, 5, 200)}.items():
        pts = torch.rand(n, 2, generator=g) * torch.tensor([Ww + 6.0, Hh + 6.0]) - 3.0
        m = torch.zeros(Hh, Ww, dtype=torch.bool)
        m[Hh // 5:Hh * 3 // 4, Ww // 4:Ww * 4 // 5] = True
        kept = T.filter_and_pad(pts, m, lo, hi, "fixture")
        out[f"fp{tag}_pts"], out[f"fp{tag}_mask"] = pts.numpy(), m.numpy()
        out[f"fp{tag}_cfg"] = np.array([lo, hi])
        out[f"fp{tag}_out"] = kept.numpy()
        print("filter_and_pad", tag, tuple(kept.shape))


SP_NET = os.path.join(H.REF, "comet", "models", "dependency", "glue-factory", "gluefactory_nonfree", "superpoint.py")


def gen_superpoint_net(out, seed=7, K=64):
    """The SuperPoint network (magicleap superpoint_v1 architecture, the reference tree's
    gluefactory_nonfree/superpoint.py:152-350, which is the network LightGlue's SuperPoint wraps)
    with PRNG weights (oracle/prng.py, seed `seed`) on three RGB images at identity resize: the
    dense keypoint probabilities (softmax, dustbin dropped, depth-to-space) and the sparse output
    (simple_nms r=4, 4-px borders, threshold 0.005, top-K). Only the config plumbing of glue-factory's
    BaseModel is stubbed (OmegaConf is not installed): the network and the keypoint selection run
    as the reference file defines them; torch.hub's checkpoint download returns the PRNG state dict."""
    import importlib.util
    import types
    H.install_stubs()

    class _Conf(dict):
        __getattr__ = dict.__getitem__

    class _BaseModel(torch.nn.Module):  # glue-factory BaseModel's conf merge, without OmegaConf
        default_conf = {}

        def __init__(self, conf):
            super().__init__()
            self.conf = _Conf({**type(self).default_conf, **conf})
            self._init(self.conf)

        def forward(self, data):
            return self._forward(data)

    for name in ("gluefactory", "gluefactory.models", "gluefactory.models.utils"):
        mod = types.ModuleType(name)
        mod.__path__ = []
        sys.modules.setdefault(name, mod)
    sys.modules["gluefactory.models.base_model"] = types.SimpleNamespace(BaseModel=_BaseModel)
    sys.modules["gluefactory.models.utils.misc"] = types.SimpleNamespace(pad_and_stack=None)
    spec = importlib.util.spec_from_file_location("gluefactory_nonfree.superpoint", SP_NET)
    sp_mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sp_mod)
    shapes = {}
    c = {"conv1a": (64, 1, 3), "conv1b": (64, 64, 3), "conv2a": (64, 64, 3), "conv2b": (64, 64, 3),
         "conv3a": (128, 64, 3), "conv3b": (128, 128, 3), "conv4a": (128, 128, 3), "conv4b": (128, 128, 3),
         "convPa": (256, 128, 3), "convPb": (65, 256, 1), "convDa": (256, 128, 3), "convDb": (256, 256, 1)}
    for n, (co, ci, k) in c.items():
        shapes[n + ".weight"] = (co, ci, k, k)
        shapes[n + ".bias"] = (co,)
    sd = dict(prng.make_state_dict(seed, shapes))
    # fan-in-scaled PRNG weights leave the 65 detector logits within ~1e-3 of each other (near-uniform
    # softmax, top-k decided by float ties): the detector head and the encoder are scaled up so the
    # scores spread over orders of magnitude and the selection is well conditioned
    for n in c:
        sd[n + ".weight"] = sd[n + ".weight"] * (40.0 if n == "convPb" else 2.0)
    orig = torch.hub.load_state_dict_from_url
    torch.hub.load_state_dict_from_url = lambda *a, **k: sd
    try:
        dense = sp_mod.SuperPoint({"sparse_outputs": False, "has_descriptor": True}).eval()
        sparse = sp_mod.SuperPoint({"max_num_keypoints": K, "detection_threshold": 0.005}).eval()
    finally:
        torch.hub.load_state_dict_from_url = orig
    g = torch.Generator().manual_seed(seed + 1)
    for tag, (Hh, Ww) in {"a": (64, 96), "b": (80, 80), "c": (48, 120)}.items():
        img = torch.rand(1, 3, Hh // 4, Ww // 4, generator=g)
        img = torch.nn.functional.interpolate(img, size=(Hh, Ww), mode="bilinear", align_corners=False)
        img = (img + 0.05 * torch.rand(1, 3, Hh, Ww, generator=g)).clamp(0, 1)  # smooth structure + texture
        with torch.no_grad():
            pd = dense({"image": img})
            ps = sparse({"image": img})
        out[f"spn{tag}_img"] = img.numpy()
        out[f"spn{tag}_prob"] = pd["keypoint_scores"].numpy()
        # glue-factory returns pixel (x, y) + 0.5; LightGlue (the reference loop's extractor) the pixel
        out[f"spn{tag}_kp"] = (ps["keypoints"] - 0.5).numpy()
        out[f"spn{tag}_kps"] = ps["keypoint_scores"].numpy()
        print("superpoint", tag, tuple(ps["keypoints"].shape))
    out["spn_cfg"] = np.array([seed, K])


def main_keypoints():
    H.require_reference()
    out = {}
    gen_keypoints(out)
    gen_superpoint_net(out)
    path = os.path.join(OUT, "comet_golden_kp.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes,", len(out), "arrays")


def main_ablations():
    H.require_reference()
    torch.set_num_threads(8)
    out = {}
    gen_ablations(out)
    path = os.path.join(OUT, "comet_golden_abl.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes,", len(out), "arrays")


def main():
    H.require_reference()
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(8)
    out = {}
    gen_exact(out)
    gen_blocks(out)
    gen_end_to_end(out)
    import json
    cfg = H.load_cfg()
    shapes = reference_shapes(H.build_reference_comet(cfg))
    with open(os.path.join(OUT, "comet_state_dict_shapes.json"), "w") as f:
        json.dump([[k, list(v)] for k, v in shapes.items()], f, indent=0)
    path = os.path.join(OUT, "comet_golden_v1.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes,", len(out), "arrays")


if __name__ == "__main__":
    if "--v2" in sys.argv:
        main_v2()
    elif "--loop" in sys.argv:
        main_loop()
    elif "--ablations" in sys.argv:
        main_ablations()
    elif "--data" in sys.argv:
        main_data()
    elif "--keypoints" in sys.argv:
        main_keypoints()
    elif "--metrics" in sys.argv:
        main_metrics()
    elif "--headline-bf16-head" in sys.argv:
        main_headline_bf16_head()
    elif "--headline" in sys.argv:
        main_headline()
    else:
        main()
