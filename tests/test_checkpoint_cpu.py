"""Checkpoint boundary and loop-side batch unpacking, CPU only.

* load_model_weights (train_util.py:165-253) / load_model_weights2 (train_util.py:256-309) on the
  full reference-layout COMET state_dict saved with a `module.` prefix (what a DDP run writes):
  prefix stripped, pose_branch.fc2 dropped by v1 (so a strict v1 load raises, as in the
  reference), relax_load -> non-strict, v2's strict-then-relaxed retry; the prefix added for a
  DDP-wrapped model.
* the ckpt_DDDDDD directory (accelerate.save_state file names, train_e2epose2.py:157-163) round
  trips model, optimizer (torch AdamW state layout), scheduler and RNG state; find_last_checkpoint
  and the tdict epoch resume (train_e2epose2.py:92-103).
* process_spark_data2 (train_util.py:637-667) defaults.
"""
import os
import pickle
import random

import numpy as np
import pytest
import torch

from conftest import PKG  # noqa: F401  (sys.path)


@pytest.fixture(scope="module")
def comet_ckpt(tmp_path_factory):
    from comet_amd.config import instantiate, load_config
    cfg = load_config()
    torch.manual_seed(0)
    m = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg)
    sd = m.state_dict()
    torch.manual_seed(1)
    saved = {k: (v + torch.randn_like(v) * 1e-3 if v.is_floating_point() else v) for k, v in sd.items()}
    path = str(tmp_path_factory.mktemp("ck") / "ddp_model.bin")
    torch.save({"module." + k: v for k, v in saved.items()}, path)
    return cfg, m, saved, path


def test_load_model_weights_strips_prefix_and_drops_fc2(comet_ckpt):
    from comet_amd.checkpoint import DROPPED_V1, load_model_weights
    cfg, m, saved, path = comet_ckpt
    # relax_load False: the two dropped tensors are missing -> strict load fails, like the reference
    with pytest.raises(RuntimeError, match="pose_branch.fc2"):
        load_model_weights(m, path, "cpu", relax_load=False)
    before = {k: m.state_dict()[k].clone() for k in DROPPED_V1}
    load_model_weights(m, path, "cpu", relax_load=True)
    now = m.state_dict()
    for k, v in saved.items():
        if k in DROPPED_V1:
            assert torch.equal(now[k], before[k]), k  # kept the model's own values
        else:
            assert torch.equal(now[k], v), k


def test_load_model_weights2_keeps_every_key_and_retries_relaxed(comet_ckpt, tmp_path):
    from comet_amd.checkpoint import load_model_weights2
    cfg, m, saved, path = comet_ckpt
    load_model_weights2(m, path, "cpu", relax_load=False)
    now = m.state_dict()
    assert all(torch.equal(now[k], v) for k, v in saved.items())
    # an extra key: the strict attempt fails, the reference's except-branch loads non-strict
    extra = dict(saved)
    extra["camera_predictor.not_a_param"] = torch.zeros(3)
    p2 = str(tmp_path / "extra.bin")
    torch.save(extra, p2)
    load_model_weights2(m, p2, "cpu", relax_load=False)
    with pytest.raises(ValueError, match="not found"):
        load_model_weights2(m, str(tmp_path / "missing.bin"), "cpu")


def test_prefix_added_for_ddp_wrapped_model(tmp_path):
    import socket
    import torch.distributed as dist
    from comet_amd.checkpoint import load_model_weights, load_model_weights2
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        net = torch.nn.Sequential(torch.nn.Linear(4, 4), torch.nn.Linear(4, 2))
        ddp = torch.nn.parallel.DistributedDataParallel(net)
        ref = {k: torch.randn_like(v) for k, v in net.state_dict().items()}
        p = str(tmp_path / "plain.bin")
        torch.save(ref, p)  # no prefix; the wrapped model's keys have one
        load_model_weights(ddp, p, "cpu", relax_load=False)
        assert all(torch.equal(net.state_dict()[k], v) for k, v in ref.items())
        ref2 = {k: v + 1 for k, v in ref.items()}
        torch.save(ref2, p)
        load_model_weights2(ddp, p, "cpu")
        assert all(torch.equal(net.state_dict()[k], v) for k, v in ref2.items())
    finally:
        dist.destroy_process_group()


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.camera_predictor = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.ReLU(), torch.nn.Linear(16, 4))


def _torch_adamw_state(net, steps=3):
    opt = torch.optim.AdamW(net.camera_predictor.parameters(), lr=1e-3)
    for i in range(steps):
        opt.zero_grad()
        net.camera_predictor(torch.randn(5, 8, generator=torch.Generator().manual_seed(i))).square().mean().backward()
        opt.step()
    return opt.state_dict()


def test_checkpoint_directory_round_trip(tmp_path):
    from comet_amd import checkpoint as C
    from comet_amd.train import CometAdamW, WarmupCosineRestarts
    torch.manual_seed(0)
    net = _Net()
    opt = CometAdamW(net.camera_predictor.parameters(), lr=1e-3)
    opt.load_state_dict(_torch_adamw_state(net))  # a torch AdamW checkpoint loads into CometAdamW
    assert all(st["step"].device.type == "cpu" and st["step"].dtype == torch.float32 for st in opt.state.values())
    sched = WarmupCosineRestarts(opt, T_0=2, iters_per_epoch=5, warmup_ratio=0.1, warmup_lr_init=1e-7)
    for _ in range(4):
        sched.step()
    path = C.checkpoint_path(str(tmp_path), 7)
    random.seed(5)
    np.random.seed(5)
    torch.manual_seed(5)
    C.save_state(path, net, opt, sched, step=42)
    C.save_tdict(path, 7, {"seed": 0, "train": {"lr": 1e-5}})
    assert sorted(os.listdir(path)) == ["optimizer.bin", "pytorch_model.bin", "random_states_0.pkl",
                                        "scheduler.bin", "tdict.pkl"]
    draws = (random.random(), np.random.rand(), torch.rand(1).item())
    # fresh objects
    torch.manual_seed(1)
    net2 = _Net()
    opt2 = CometAdamW(net2.camera_predictor.parameters(), lr=1e-3)
    sched2 = WarmupCosineRestarts(opt2, T_0=2, iters_per_epoch=5, warmup_ratio=0.1, warmup_lr_init=1e-7)
    step = C.load_state(path, net2, opt2, sched2)
    assert step == 42
    assert (random.random(), np.random.rand(), torch.rand(1).item()) == draws
    for (k, a), b in zip(net.state_dict().items(), net2.state_dict().values()):
        assert torch.equal(a, b), k
    s1, s2 = opt.state_dict(), opt2.state_dict()
    assert s1["param_groups"] == s2["param_groups"]
    for i in s1["state"]:
        for k in ("step", "exp_avg", "exp_avg_sq"):
            assert torch.equal(s1["state"][i][k], s2["state"][i][k])
    assert sched2.last_epoch == sched.last_epoch and sched2.get_last_lr() == sched.get_last_lr()
    # discovery and resume epoch
    C.save_state(C.checkpoint_path(str(tmp_path), 12), net, opt, sched)
    os.makedirs(os.path.join(str(tmp_path), "ckpt_12"))  # not six digits: ignored
    assert C.find_last_checkpoint(str(tmp_path)).endswith("ckpt_000012")
    assert len(C.find_last_checkpoint(str(tmp_path), all_checkpoints=True)) == 2
    assert C.find_last_checkpoint(str(tmp_path / "none")) is None
    assert C.resume_epoch(path) == (7, 8)                     # tdict epoch + 1
    assert C.resume_epoch(C.find_last_checkpoint(str(tmp_path))) == (12, 13)  # no tdict: name + 1
    assert C.load_tdict(path) == {"epoch": 7, "cfg": {"seed": 0, "train": {"lr": 1e-5}}}


def test_load_state_accepts_ddp_prefixed_model_file(tmp_path):
    """accelerate 1.x saves get_state_dict(model, unwrap=False): a reference run under DDP writes
    `module.`-prefixed keys into pytorch_model.bin; load_state strips them for the plain model."""
    from collections import OrderedDict
    from comet_amd import checkpoint as C
    torch.manual_seed(0)
    net = _Net()
    path = str(tmp_path / "ckpt_000003")
    os.makedirs(path)
    torch.save(OrderedDict(("module." + k, v) for k, v in net.state_dict().items()),
               os.path.join(path, C.MODEL_FILE))
    torch.manual_seed(1)
    net2 = _Net()
    C.load_state(path, net2)
    for (k, a), b in zip(net.state_dict().items(), net2.state_dict().values()):
        assert torch.equal(a, b), k


def test_save_state_other_ranks_write_only_their_rng_file(tmp_path):
    """accelerate.utils.save writes the model / optimizer / scheduler archives on the main process
    only; every rank writes random_states_<rank>.pkl (no torn concurrent writes of one file)."""
    from comet_amd import checkpoint as C
    from comet_amd.train import CometAdamW
    net = _Net()
    opt = CometAdamW(net.camera_predictor.parameters(), lr=1e-3)
    path = str(tmp_path / "ckpt_000001")
    C.save_state(path, net, opt, None, step=3, process_index=1)
    assert sorted(os.listdir(path)) == ["random_states_1.pkl"]
    C.save_state(path, net, opt, None, step=3, process_index=0)
    assert sorted(os.listdir(path)) == ["optimizer.bin", "pytorch_model.bin", "random_states_0.pkl",
                                        "random_states_1.pkl"]


def test_step_drops_pending_clip_on_every_path():
    """clip_grad_norm_'s stored (max_norm, norm) is consumed by the next step() even when that
    step returns early because no parameter has a gradient, so it never leaks into a later step."""
    from comet_amd.train import CometAdamW
    net = _Net()
    opt = CometAdamW(net.camera_predictor.parameters(), lr=1e-3)
    opt._pending = (1.0, torch.ones(1))
    opt.step()  # no gradients: early return
    assert opt._pending is None


def test_tdict_refuses_objects(tmp_path):
    from comet_amd.checkpoint import load_tdict

    with open(tmp_path / "tdict.pkl", "wb") as f:
        pickle.dump({"epoch": 3, "cfg": _Net}, f)  # any class reference (an OmegaConf DictConfig in the reference)
    assert load_tdict(str(tmp_path)) is None


def test_process_spark_data2_defaults():
    from comet_amd.config import AttrDict
    from comet_amd.loop import process_spark_data2
    B, S = 2, 3
    batch = {"images": torch.zeros(B, S, 3, 40, 60), "T": torch.zeros(B, S, 3), "R": torch.zeros(B, S, 4),
             "T_uvz": torch.ones(B, S, 3), "ratio": torch.tensor([0.5, 0.25], dtype=torch.float64),
             "seq_name": ["a", "b"]}
    cfg = AttrDict.wrap({"default_focal_length": 1745, "train": {"dataset": "AMD"}})
    out = process_spark_data2(batch, "cpu", cfg)
    images, T_xyz, T_uvz, R, fl, pp, ratio, names, image_names, mask, Rm = out
    assert torch.equal(fl, torch.full((B, S, 2), 1745.0))
    assert torch.equal(pp, torch.tensor([30.0, 20.0]).expand(B, S, 2))
    assert ratio.dtype == torch.float64 and names == ["a", "b"] and image_names is None and mask is None and Rm is None


def test_batch_shard_partitions_batches():
    """drop_last=True on the wrapped sampler: 11 batches over 4 ranks -> the incomplete last round
    (3 batches) is dropped, every rank runs 2 full batches, all distinct."""
    from comet_amd.loop import _BatchShard
    bs = torch.utils.data.BatchSampler(range(23), batch_size=2, drop_last=True)  # 11 batches
    shards = [list(_BatchShard(bs, r, 4)) for r in range(4)]
    assert all(len(s) == len(_BatchShard(bs, 0, 4)) == 2 for s in shards)
    flat = [tuple(b) for s in shards for b in s]
    assert len(set(flat)) == 8 and set(flat) <= {tuple(b) for b in bs}


def test_batch_shard_even_batches_cycles_from_start():
    """even_batches=True, drop_last=False (accelerate's default; the reference's entry points pass
    even_batches=False, train_e2epose2.py:47 -- this pins the default path of _BatchShard): 23 samples in
    batches of 2 (the last one short) over 4 ranks -> 3 full batches per rank; the short batch is
    completed and the round filled with indices cycled from the start of the epoch."""
    from comet_amd.loop import _BatchShard
    bs = torch.utils.data.BatchSampler(range(23), batch_size=2, drop_last=False)  # 12 batches, last [22]
    shards = [list(_BatchShard(bs, r, 4)) for r in range(4)]
    assert [len(s) for s in shards] == [3, 3, 3, 3] == [len(_BatchShard(bs, r, 4)) for r in range(4)]
    assert all(len(b) == 2 for s in shards for b in s)
    assert shards[3][2] == [22, 0]  # the short last batch completed from index 0
    assert sorted(i for s in shards for b in s for i in b) == sorted(list(range(23)) + [0])


@pytest.mark.parametrize("n,bsz,world,drop_last,even", [
    (23, 2, 4, False, True), (23, 2, 4, False, False), (23, 2, 4, True, True), (24, 2, 4, False, True),
    (5, 1, 2, False, True), (5, 1, 2, False, False), (3, 4, 4, False, True), (7, 3, 2, False, True),
    (100, 8, 8, False, True), (100, 8, 8, True, True), (1, 2, 3, False, True), (9, 2, 8, False, False)])
def test_batch_shard_matches_accelerate(n, bsz, world, drop_last, even):
    """_BatchShard restates accelerate's BatchSamplerShard (split_batches=False): the same batches on
    every rank, in order, and the same lengths, against the installed accelerate (the reference pins
    0.24.0; the algorithm for a fixed batch size is unchanged since)."""
    acc = pytest.importorskip("accelerate.data_loader")
    from comet_amd.loop import _BatchShard
    bs = torch.utils.data.BatchSampler(range(n), batch_size=bsz, drop_last=drop_last)
    for r in range(world):
        ours, ref = _BatchShard(bs, r, world, even), acc.BatchSamplerShard(bs, world, r, False, even)
        assert [list(b) for b in ours] == [list(b) for b in ref], (r, list(ours), list(ref))
        assert len(ours) == len(ref)


def test_batch_shard_uneven_keeps_tail():
    """even_batches=False (abl_ours.py:28): 5 batches over 2 ranks -> 3 + 2, nothing dropped."""
    from comet_amd.loop import _BatchShard
    bs = [[i] for i in range(5)]
    r0, r1 = _BatchShard(bs, 0, 2, False), _BatchShard(bs, 1, 2, False)
    assert list(r0) == [[0], [2], [4]] and len(r0) == 3
    assert list(r1) == [[1], [3]] and len(r1) == 2


def test_csv_logger(tmp_path):
    """abl_ours.py:9-22: header once, then one row per log(); reopening appends."""
    import csv
    from comet_amd.loop import CsvLogger
    p = str(tmp_path / "out" / "test_results.csv")
    CsvLogger(p, ["epoch", "it", "mode"]).log({"epoch": -1, "it": 3, "mode": "eval"})
    CsvLogger(p, ["epoch", "it", "mode"]).log({"epoch": 0, "it": 1, "mode": "eval"})
    with open(p) as f:
        rows = list(csv.DictReader(f))
    assert rows == [{"epoch": "-1", "it": "3", "mode": "eval"}, {"epoch": "0", "it": "1", "mode": "eval"}]


def test_stats_round_trip(tmp_path):
    from comet_amd.loop import Stats, TO_PLOT_METRICS
    st = Stats(TO_PLOT_METRICS)
    st.new_epoch()
    for i in range(3):
        st.update({"R_avg": torch.tensor(float(i)), "T_avg": 2.0 * i}, time_start=0.0, stat_set="train")
    av = st.get_epoch_averages()["train"]
    assert av["R_avg"] == 1.0 and av["T_avg"] == 2.0 and av["it"] == 2 and av["epoch"] == 0
    st.save(str(tmp_path / "s"))
    st2 = Stats.load(str(tmp_path / "s"))
    assert st2.get_epoch_averages() == st.get_epoch_averages()
