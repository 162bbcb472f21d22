"""End-to-end parity of the HIP path (comet_amd on libcomet_hip.so) against the golden vectors
produced by the reference itself and against the oracle, at the golden configuration
(B=1, T=4, 128x128 frames, N=16 tracks, PRNG weights seed 0, inputs seed 1).

Tolerances (north star): fp32 1e-4 on quaternion / uvz outputs; bf16 1e-2 vs the reference's own
bf16-autocast run."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu
GOLD = os.path.join(ROOT, "tests", "golden", "comet_golden_v1.npz")


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


@pytest.fixture(scope="module")
def setup(gold):
    from comet_amd.config import instantiate, load_config
    from comet_amd.models.utils import QuaternionCameras
    from oracle import prng
    from oracle.weights import comet_shapes
    seed_w, seed_x, B, T, H, W, N = [int(v) for v in gold["cfg"]]
    cfg = load_config()
    torch.manual_seed(0)
    model = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg)
    P = prng.make_state_dict(seed_w, comet_shapes())
    model.load_state_dict(P, strict=True)
    model = model.cuda()
    img, tracks, gt = prng.synthetic_batch(seed_x, B, T, H, W, N)
    cams = QuaternionCameras(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
                             principal_point=gt["principal_point"], ratio=gt["ratio"], device="cuda")
    return model, cfg, P, img.cuda(), tracks.cuda(), gt, cams


def _run(setup, dtype, backward=False):
    from comet_amd import functional as F
    model, cfg, P, img, tracks, gt, cams = setup
    with F.precision(dtype):
        model.zero_grad(set_to_none=True)
        out = model(img, gt_cameras=cams, training=True, tracks=tracks)
        if backward:
            out["loss"].backward()
    torch.cuda.synchronize()
    return out


def test_e2e_fp32_forward_matches_reference(setup, gold):
    out = _run(setup, torch.float32)
    tp = out["_track_predictions"]
    close(tp["refine_pred_track"], gold["e2e_pred_tracks"], 1e-5, 1e-3, "refined tracks")
    enc = out["pred_pose_enc"]
    close(enc[:, :3], gold["e2e_pred_pose_enc"][:, :3], 1e-4, 1e-4, "uvz (fp32)")
    close(enc[:, 3:], gold["e2e_pred_pose_enc"][:, 3:], 1e-4, 1e-4, "quaternion (fp32)")
    close(out["gt_pose_enc"], gold["e2e_gt_pose_enc"], 1e-6, 1e-6, "gt_pose_enc")
    close(out["loss"].reshape(1), gold["e2e_loss"], 1e-4, 1e-4, "loss")
    close(out["loss_trans"].reshape(1), gold["e2e_loss_trans"], 1e-4, 1e-4, "loss_trans")
    close(out["loss_rot"].reshape(1), gold["e2e_loss_rot"], 1e-4, 1e-4, "loss_rot")
    close(out["pred_cameras"].R, gold["e2e_pred_R"], 1e-4, 1e-4, "pred R")
    close(out["pred_cameras"].T, gold["e2e_pred_T"], 1e-4, 1e-3, "pred T")


def test_e2e_fp32_grads_match_reference(setup, gold):
    model = setup[0]
    _run(setup, torch.float32, backward=True)
    named = dict(model.camera_predictor.named_parameters())
    names = [str(k) for k in gold["grad_names"]]
    got = [named[k].grad for k in names]
    assert all(g is not None for g in got), [k for k, g in zip(names, got) if g is None][:5]
    norms = np.array([g.double().norm().item() for g in got])
    close(norms, gold["grad_norms"], 2e-3, 1e-5, "grad norms")
    for k in gold:
        if k.startswith("grad_full."):
            ref = gold[k]
            close(named[k[len("grad_full."):]].grad, ref, 2e-3, 2e-4 * float(np.abs(ref).max()), k)
    # parameters the reference never executes receive no gradient
    unused = [k for k, p in named.items() if p.requires_grad and k not in set(names)]
    assert all(named[k].grad is None for k in unused)


def test_e2e_bf16_matches_reference_bf16(setup, gold):
    out = _run(setup, torch.bfloat16)
    enc = out["pred_pose_enc"]
    ref = gold["bf16_pred_pose_enc"]
    close(enc[:, :3], ref[:, :3], 0, 1e-2, "uvz (bf16)")
    close(enc[:, 3:], ref[:, 3:], 0, 1e-2, "quaternion (bf16)")
    close(out["loss"].reshape(1), gold["bf16_loss"], 2e-2, 1e-2, "loss (bf16)")


def test_batch_semantics_per_sequence(setup):
    """B=2 batch of two different sequences == two B=1 runs (SURVEY Appendix B-1 definition)."""
    from comet_amd import functional as F
    from comet_amd.models.utils import QuaternionCameras
    from oracle import prng
    model = setup[0]
    outs = []
    with F.precision(torch.float32), torch.no_grad():
        ims, trs, gts = [], [], []
        for seed in (11, 12):
            img, tr, gt = prng.synthetic_batch(seed, 1, 4, 128, 128, 16)
            cams = QuaternionCameras(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
                                     ratio=gt["ratio"], device="cuda")
            outs.append(model(img.cuda(), gt_cameras=cams, training=True, tracks=tr.cuda()))
            ims.append(img); trs.append(tr); gts.append(gt)
        cams = QuaternionCameras(R=torch.cat([g["R"] for g in gts]), T_uvz=torch.cat([g["T_uvz"] for g in gts]),
                                 T=torch.cat([g["T"] for g in gts]), focal_length=torch.cat([g["focal_length"] for g in gts]),
                                 ratio=gts[0]["ratio"], device="cuda")
        both = model(torch.cat(ims).cuda(), gt_cameras=cams, training=True, tracks=torch.cat(trs).cuda())
    torch.cuda.synchronize()
    ref = torch.cat([o["pred_pose_enc"] for o in outs])
    close(both["pred_pose_enc"], ref.cpu(), 1e-5, 1e-5, "B=2 vs 2xB=1 pose enc")
    close(both["loss"].reshape(1), ((outs[0]["loss"] + outs[1]["loss"]) / 2).reshape(1).cpu(), 1e-5, 1e-5, "B=2 loss")


def _block_params(seed, shapes):
    from oracle import prng
    return prng.make_state_dict(seed, shapes)


def test_attn_blocks_against_reference_vectors(gold):
    from comet_amd import functional as F
    from comet_amd.models.modules import AttnBlock, CrossAttnBlock
    from oracle import prng
    blk = AttnBlock(768, 8, mlp_ratio=4)
    blk.load_state_dict(_block_params(7, {k: tuple(v.shape) for k, v in blk.state_dict().items()}))
    blk = blk.cuda()
    x = torch.from_numpy(prng.normal_like(8, "attn_x", (3, 37, 768))).cuda().requires_grad_(True)
    with F.precision(torch.float32):
        y = blk(x)
        y.backward(torch.from_numpy(prng.normal_like(8, "attn_gy", (3, 37, 768))).cuda())
    close(y, gold["blk_attn_y"], 1e-4, 1e-4, "AttnBlock y")
    close(x.grad, gold["blk_attn_dx"], 1e-3, 1e-4, "AttnBlock dx")
    for k, p in blk.named_parameters():
        close(p.grad.norm().reshape(1), gold["blk_attn_grad.norm." + k], 1e-3, 1e-5, "AttnBlock grad " + k)
    cb = CrossAttnBlock(768, 768, 8, mlp_ratio=4)
    cb.load_state_dict(_block_params(8, {k: tuple(v.shape) for k, v in cb.state_dict().items()}))
    cb = cb.cuda()
    x = torch.from_numpy(prng.normal_like(9, "cx", (2, 29, 768))).cuda().requires_grad_(True)
    c = torch.from_numpy(prng.normal_like(9, "cc", (2, 41, 768))).cuda().requires_grad_(True)
    with F.precision(torch.float32):
        y = cb(x, c)
        y.backward(torch.from_numpy(prng.normal_like(9, "cgy", (2, 29, 768))).cuda())
    close(y, gold["blk_cross_y"], 1e-4, 1e-4, "CrossAttnBlock y")
    close(x.grad, gold["blk_cross_dx"], 1e-3, 1e-4, "CrossAttnBlock dx")
    close(c.grad, gold["blk_cross_dctx"], 1e-3, 1e-4, "CrossAttnBlock dctx")
    for k, p in cb.named_parameters():
        close(p.grad.norm().reshape(1), gold["blk_cross_grad.norm." + k], 1e-3, 1e-5, "CrossAttnBlock grad " + k)


def test_harmonic_embedding_against_reference(gold):
    from comet_amd.minipytorch3d.harmonic_embedding import HarmonicEmbedding
    x = torch.from_numpy(gold["harm_x"]).cuda()
    cov = torch.from_numpy(gold["harm_cov"]).cuda()
    for n, om, logs, app in [(6, 1.0, True, True), (48, 1.0, True, False), (10, 0.5, False, True)]:
        tag = f"harm_{n}_{om}_{int(logs)}_{int(app)}"
        m = HarmonicEmbedding(n, om, logs, app).cuda()
        close(m(x), gold[tag], 0, 2e-5 * max(1.0, n / 6), tag)
        close(m(x, diag_cov=cov), gold[tag + "_cov"], 0, 2e-5 * max(1.0, n / 6), tag + " cov")
    # backward vs torch autograd of the oracle restatement
    from oracle import comet_oracle as O
    xr = x.detach().cpu().double().requires_grad_(True)
    cr = cov.detach().cpu().double().requires_grad_(True)
    y = O.harmonic_embedding(xr, 10, 0.5, False, True, diag_cov=cr)
    g = torch.randn(y.shape, dtype=torch.float64)
    y.backward(g)
    xx = x.clone().requires_grad_(True)
    cc = cov.clone().requires_grad_(True)
    m = HarmonicEmbedding(10, 0.5, False, True).cuda()
    m(xx, diag_cov=cc).backward(g.float().cuda())
    # f32 evaluation (the reference's own dtype) vs f64: f^2 up to 6.6e4 amplifies the argument's f32
    # rounding, so the reference itself is 5e-5 x max|grad| away from f64; tolerance scales with max
    close(xx.grad, xr.grad, 1e-4, 1e-4 * xr.grad.abs().max().item(), "harmonic dx")
    close(cc.grad, cr.grad, 1e-4, 2e-4 * cr.grad.abs().max().item(), "harmonic dcov")


def test_train_step_matches_oracle_adamw(setup):
    """One clip + AdamW step on the camera-predictor params vs torch.optim.AdamW on the same grads."""
    from comet_amd import functional as F
    from comet_amd.train import CometAdamW
    model = setup[0]
    _run(setup, torch.float32, backward=True)
    ps = [p for p in model.camera_predictor.parameters() if p.requires_grad and p.grad is not None]
    ref = [p.detach().clone().cpu() for p in ps]
    grads = [p.grad.detach().clone().cpu() for p in ps]
    total = torch.norm(torch.stack([g.norm() for g in grads]))
    coef = min(1.0, 1.0 / (total.item() + 1e-6))
    refp = [r.clone().requires_grad_(False) for r in ref]
    opt_ref = torch.optim.AdamW(refp, lr=1e-5)
    for r, g in zip(refp, grads):
        r.grad = g * coef
    opt_ref.step()
    before = [p.detach().clone() for p in ps]
    opt = CometAdamW(model.camera_predictor.parameters(), lr=1e-5)
    opt.step(max_norm=1.0)
    torch.cuda.synchronize()
    for p, r, b in zip(ps, refp, before):
        close(p.detach(), r, 1e-6, 1e-7, "AdamW param")
        p.data.copy_(b)  # restore for other tests
    F.invalidate_weight_cache()
