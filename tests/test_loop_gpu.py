"""The loop-side caller counterpart on the GPU: train_or_eval_fn's train and eval
branches (train_eval_func_new_cp5.py:514-823) over YTDataset batches from forked DataLoader
workers, with SuperPoint keypoint tracks, QuaternionCameras from process_spark_data2, the bf16
mixed-precision forward, backward, clip + AdamW + LR schedule, the eval metrics and Stats; then the
ckpt_DDDDDD directory of the trained model / optimizer / scheduler round-trips on the device."""
import os

import pytest
import torch

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
    assert r["mode"] == "eval" and int(r["epoch"]) == -1 and int(r["it"]) == n - 1   # one iteration per sample
    for k in ("Auc_30", "R_avg", "T_avg", "acc@5deg_x", "lr"):
        v = float(r[k])
        assert v == v, k   # logged and not NaN
    assert float(r["lr"]) == pytest.approx(cfg["train"]["lr"])   # warmup_ratio 0: the base lr at step 0
