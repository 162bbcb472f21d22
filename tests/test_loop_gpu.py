"""The loop-side caller counterpart on the GPU: train_or_eval_fn's train and eval
branches (train_eval_func_new_cp5.py:514-823) over YTDataset batches from forked DataLoader
workers, with SuperPoint keypoint tracks, QuaternionCameras from process_spark_data2, the bf16
mixed-precision forward, backward, clip + AdamW + LR schedule, the eval metrics and Stats; then the
ckpt_DDDDDD directory of the trained model / optimizer / scheduler round-trips on the device."""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT

import yt_fixture

pytestmark = pytest.mark.gpu


def test_train_or_eval_fn_and_checkpoint_resume(tmp_path):
    from torch.utils.data import DataLoader
    from comet_amd import checkpoint as C
    from comet_amd.config import instantiate, load_config
    from comet_amd.data import DeviceLoader, YTDataset, collate_host
    from comet_amd.loop import TO_PLOT_METRICS, CometAccelerator, Stats, train_or_eval_fn
    from comet_amd.train import build_optimizer
    root = yt_fixture.make_dataset(str(tmp_path / "yt"))
    cfg = load_config(**{"train.track_num": 64, "train.img_size": 128, "seqlen": 4})
    cfg["track_by_spsg"] = True
    cfg["train"]["print_interval"] = 1
    cfg["train"]["eval_print_interval"] = 1
    torch.manual_seed(0)
    ds = YTDataset(root, crop_size=[128, 128], seq_len=4)
    dl = DeviceLoader(DataLoader(ds, batch_size=1, num_workers=2, collate_fn=collate_host), "cuda")
    model = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg)
    opt, sched = build_optimizer(cfg, model, dl)
    acc = CometAccelerator(mixed_precision="bf16")
    model, dl, opt, sched = acc.prepare(model, dl, opt, sched)
    assert next(model.parameters()).is_cuda
    frozen = {k: p.detach().clone() for k, p in model.track_predictor.named_parameters()}
    head = {k: p.detach().clone() for k, p in model.camera_predictor.named_parameters()}
    stats = Stats(TO_PLOT_METRICS)
    stats.new_epoch()
    train_or_eval_fn(model, dl, cfg, opt, stats, acc, sched, training=True, epoch=0)
    assert acc.step == len(ds) == 2 and sched.last_epoch == 2
    tr = stats.get_epoch_averages()["train"]
    for k in ("R_avg", "T_avg", "Auc_30", "Racc_him_5", "acc@5deg_x", "sec/it"):
        assert k in tr and tr[k] == tr[k], k  # present and not NaN
    assert all(torch.equal(p, frozen[k]) for k, p in model.track_predictor.named_parameters())
    moved = [k for k, p in model.camera_predictor.named_parameters() if not torch.equal(p, head[k])]
    assert "pose_token" in moved and len(moved) > 100
    assert all(torch.isfinite(p).all() for p in model.camera_predictor.parameters())
    train_or_eval_fn(model, dl, cfg, opt, stats, acc, sched, training=False, epoch=0)
    ev = stats.get_epoch_averages()["eval"]
    assert ev["it"] == 1 and "Auc_10" in ev
    # checkpoint directory of the trained state, loaded into fresh objects
    path = C.checkpoint_path(str(tmp_path / "exp"), 1)
    acc.save_state(path, model, opt, sched)
    C.save_tdict(path, 1, cfg)
    stats.save(os.path.join(path, "train_stats.jgz"))
    torch.manual_seed(1)
    model2 = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg).cuda()
    opt2, sched2 = build_optimizer(cfg, model2, dl)
    acc2 = CometAccelerator(mixed_precision="bf16")
    last = C.find_last_checkpoint(str(tmp_path / "exp"))
    assert C.resume_epoch(last) == (1, 2)
    acc2.load_state(last, model2, opt2, sched2)
    assert acc2.step == 2
    sd1, sd2 = model.state_dict(), model2.state_dict()
    assert all(torch.equal(sd1[k], sd2[k]) for k in sd1)
    s1, s2 = opt.state_dict()["state"], opt2.state_dict()["state"]
    assert s1.keys() == s2.keys() and all(torch.equal(s1[i]["exp_avg"], s2[i]["exp_avg"]) for i in s1)
    assert all(s2[i]["step"].device.type == "cpu" for i in s2)
    assert sched2.get_last_lr() == sched.get_last_lr()
    assert Stats.load(os.path.join(last, "train_stats.jgz")).get_epoch_averages() == stats.get_epoch_averages()


def test_abl_ours_test_fn_end_to_end(tmp_path):
    """abl_ours.py:24-88 through comet_amd.loop.test_fn: the AMD_eval loader over an on-disk
    YTDataset, drop_last on its batch sampler, load_model_weights2 of a checkpoint file, one
    bf16 eval pass of train_or_eval_fn with SuperPoint keypoint tracks, and one row of
    output_dir/test_results.csv with the reference's fields."""
    import csv
    from comet_amd import loop
    from comet_amd.config import instantiate, load_config
    root = tmp_path / "AMD"
    yt_fixture.make_dataset(str(root / "AMD_eval"))
    cfg = load_config(**{"train.track_num": 64, "train.img_size": 128, "seqlen": 4})
    torch.manual_seed(3)
    ref_model = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg)
    wpath = str(tmp_path / "weights.bin")
    torch.save(ref_model.state_dict(), wpath)
    cfg["track_by_spsg"] = True
    cfg["output_dir"] = str(tmp_path / "abl_ours_eval_fold")
    cfg["train"]["dataset"] = "AMD_eval"
    cfg["train"]["num_workers"] = 2
    cfg["train"]["resume_ckpt"] = wpath
    cfg["train"]["eval_print_interval"] = 1
    assert loop.test_fn(cfg, data_root=str(root)) is True
    with open(tmp_path / "abl_ours_eval_fold" / "test_results.csv") as f:
        rows = list(csv.DictReader(f))
    assert len(rows) == 1
    r = rows[0]
    assert list(r.keys()) == ["epoch", "it", "mode"] + list(loop.TO_PLOT_METRICS)
    from comet_amd.data import YTDataset
    n = len(YTDataset(str(root / "AMD_eval"), crop_size=[128, 128], seq_len=4, split="valid"))
    assert r["mode"] == "eval" and int(r["epoch"]) == -1
    # "it" is PARITY UNPINNED: its value comes from pytorch3d implicitron's Stats, the base class of
    # the reference's VizStats (train_util.py:1914), which is not in the reference tree. What is
    # asserted here is this build's own Stats semantics (one iteration per sample of the pass, plus
    # the lr update test_fn makes after it, abl_ours.py:69), not a reference value.
    assert int(r["it"]) == n
    for k in ("Auc_30", "R_avg", "T_avg", "acc@5deg_x", "lr"):
        v = float(r[k])
        assert v == v, k   # logged and not NaN
    assert float(r["lr"]) == pytest.approx(cfg["train"]["lr"])   # warmup_ratio 0: the base lr at step 0


def test_train_or_eval_fn_matches_reference_loop_golden():
    """The composed training loop against the reference's own train_or_eval_fn run for two steps
    (tests/golden/comet_golden_loop.npz, tools/gen_golden.py --loop: T=4, 128^2, N=256 fixed
    keypoint tracks through the loop's keypoint path and filter_and_pad, PRNG weights, fp32):
    per-step loss and pre-clip gradient norm, the scheduler's learning rates, and the camera
    predictor's parameter updates after zero_grad -> backward -> clip 1.0 -> AdamW -> scheduler
    (this build defers the clip scaling into the AdamW kernel). AdamW's first steps move every
    element by about lr * sign(grad), so the updates are compared by per-parameter norms (2e-2) and
    element-wise on selected tensors, where elements whose gradient sits at the noise floor may take
    the other sign (at most 1 % of them)."""
    from comet_amd.config import instantiate, load_config
    from comet_amd.loop import CometAccelerator, Stats, TO_PLOT_METRICS, train_or_eval_fn
    from comet_amd.train import build_optimizer
    from oracle import prng
    from oracle.weights import comet_shapes
    gold = dict(np.load(os.path.join(ROOT, "tests", "golden", "comet_golden_loop.npz"), allow_pickle=False))
    seed_w, seed_x, B, T, H, W, N, steps = [int(v) for v in gold["loop_cfg"]]
    cfg = load_config(**{"train.track_num": N, "train.img_size": H, "seqlen": T})
    cfg["track_by_spsg"] = True
    cfg["train"]["print_interval"] = 1
    torch.manual_seed(0)
    model = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg)
    model.load_state_dict(prng.make_state_dict(seed_w, comet_shapes()), strict=True)
    batches = prng.loop_batches(seed_x, B, T, H, W, N, steps)
    kps = iter([b.pop("kp0").cuda() for b in batches])

    class SP:  # the generator's SuperPoint stub: the fixed keypoints of each batch
        def extract(self, img):
            return {"keypoints": next(kps)[None]}

    acc = CometAccelerator(mixed_precision="no")
    opt, sched = build_optimizer(cfg, model, batches)
    model, dl, opt, sched = acc.prepare(model, batches, opt, sched)
    rec = {"loss": [], "norm": [], "lr": []}
    backward, clip, sstep = acc.backward, acc.clip_grad_norm_, sched.step

    def rec_backward(loss):
        rec["loss"].append(float(loss.detach()))
        backward(loss)

    def rec_clip(params, max_norm, optimizer=None):
        n = clip(params, max_norm, optimizer=optimizer)
        rec["norm"].append(float(n))
        return n

    def rec_step(*a, **k):
        sstep(*a, **k)
        rec["lr"].append(sched.get_last_lr()[0])
    acc.backward, acc.clip_grad_norm_, sched.step = rec_backward, rec_clip, rec_step
    before = {k: p.detach().double().clone() for k, p in model.camera_predictor.named_parameters()}
    train_or_eval_fn(model, dl, cfg, opt, Stats(TO_PLOT_METRICS), acc, sched, training=True, epoch=0, sp=SP())
    torch.cuda.synchronize()
    print("losses", rec["loss"], "ref", gold["loop_loss"], "norms", rec["norm"], "ref", gold["loop_grad_norm"])
    np.testing.assert_allclose(rec["loss"][0], gold["loop_loss"][0], rtol=2e-4)
    np.testing.assert_allclose(rec["loss"][1], gold["loop_loss"][1], rtol=1e-3)
    np.testing.assert_allclose(rec["norm"], gold["loop_grad_norm"], rtol=2e-3)
    np.testing.assert_allclose(rec["lr"], gold["loop_lr"], rtol=1e-12)
    named = dict(model.camera_predictor.named_parameters())
    # the reference's names include its DINOv2 stand-in (transformers naming); the frozen backbone
    # never moves, so the comparison runs over the updated parameters, which share names
    ref_moved = {str(k): v for k, v in zip(gold["loop_names"], gold["loop_delta_norms"]) if v > 0}
    ours = {k: (p.detach().double() - before[k]).norm().item() for k, p in named.items()}
    ours_moved = {k for k, v in ours.items() if v > 0}
    assert ours_moved == set(ref_moved), (sorted(ours_moved ^ set(ref_moved)))[:8]
    names = sorted(ref_moved)
    dn = np.array([ours[k] for k in names])
    ref = np.array([ref_moved[k] for k in names])
    moved = ref > 0
    rel = np.abs(dn[moved] - ref[moved]) / ref[moved]
    print(f"{int(moved.sum())} updated params: max rel diff of the update norms {rel.max():.3e}")
    assert rel.max() < 2e-2
    lr = float(gold["loop_lr"][0])
    for k in gold:
        if not k.startswith("loop_delta."):
            continue
        name = k[len("loop_delta."):]
        d = (named[name].detach().double() - before[name]).cpu().numpy()
        off = np.abs(d - gold[k]) > 0.1 * lr
        print(f"{name}: {off.mean():.2e} of the elements off by > 0.1 lr")
        assert off.mean() < 1e-2, name
