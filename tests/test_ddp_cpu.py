"""World-size-2 gloo tests of the data-parallel gradient exchange (comet_amd/ddp.py), CPU only.

Checks what DistributedDataParallel guarantees for the reference (train_e2epose2.py:83): after
backward every rank holds the mean of the per-rank gradients, parameters that took no part in the
loss keep grad=None, and the buckets are re-armed every step.
"""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _Net(torch.nn.Module):
    def __init__(self):
        super().__init__()
        torch.manual_seed(0)
        self.a = torch.nn.Linear(16, 32)
        self.b = torch.nn.Linear(32, 32)
        self.unused = torch.nn.Linear(32, 8)  # never executed, like FeatureFusion in the head
        self.c = torch.nn.Linear(32, 4)

    def forward(self, x):
        return self.c(torch.relu(self.b(torch.relu(self.a(x)))))


class _NetUnusedLast(_Net):
    """The never-executed module registered last: with reverse-registration buckets it sits in the
    FIRST bucket (like the head's fc_depth ... pose_embed_scale block)."""

    def __init__(self):
        super().__init__()
        del self.unused
        torch.manual_seed(1)
        self.unused = torch.nn.Linear(32, 8)


def _data(rank, step):
    g = torch.Generator().manual_seed(100 * step + rank)
    return torch.randn(8, 16, generator=g), torch.randn(8, 4, generator=g)


def _worker(rank, world, port, bucket_mb, q, paths, net_cls=_Net, steps=2):
    import sys
    sys.path[:0] = paths
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from comet_amd.ddp import GradBucketer
        net = net_cls()
        bk = GradBucketer(net.parameters(), bucket_mb=bucket_mb)
        out, logs = [], []
        for step in range(steps):
            bk.prepare_backward()
            x, y = _data(rank, step)
            loss = ((net(x) - y) ** 2).mean()
            loss.backward()
            bk.finish_backward()
            out.append({k: (None if p.grad is None else p.grad.detach().numpy().copy()) for k, p in net.named_parameters()})
            logs.append(list(bk.launch_log))
        q.put((rank, len(bk.buckets), out, logs))
    finally:
        dist.destroy_process_group()


def _expected(world, net_cls=_Net, steps=2):
    net = net_cls()
    res = []
    for step in range(steps):
        acc = {k: torch.zeros_like(p) for k, p in net.named_parameters()}
        for r in range(world):
            net.zero_grad(set_to_none=True)
            x, y = _data(r, step)
            ((net(x) - y) ** 2).mean().backward()
            for k, p in net.named_parameters():
                if p.grad is not None:
                    acc[k] += p.grad / world
        res.append(acc)
    return res


@pytest.mark.parametrize("bucket_mb", [64, 0.004])  # one bucket / several buckets
def test_bucketed_allreduce_matches_mean_grad(bucket_mb):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, q, [ROOT, PKG])) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        rank, nb, out, _ = q.get(timeout=120)
        results[rank] = (nb, out)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = _expected(world)
    if bucket_mb < 1:
        assert results[0][0] > 1
    for rank in range(world):
        for step in range(2):
            got = results[rank][1][step]
            for k, g in got.items():
                if k.startswith("unused."):
                    assert g is None, k
                else:
                    torch.testing.assert_close(torch.from_numpy(g), exp[step][k], rtol=1e-5, atol=1e-6)


def test_unused_param_in_first_bucket_does_not_delay_allreduce():
    """the never-executed params are excluded from the buckets after the discovery
    step, so from step 2 on every bucket's all-reduce is launched during the backward (before
    finish_backward), including the one that held the unused module in the provisional layout."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 0.004, q, [ROOT, PKG], _NetUnusedLast, 3))
             for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        rank, nb, out, logs = q.get(timeout=120)
        results[rank] = (nb, out, logs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = _expected(world, _NetUnusedLast, 3)
    for rank in range(world):
        nb, out, logs = results[rank]
        assert nb > 1
        assert all(not during for _, during in logs[0])          # discovery: reduced at finish
        for step in (1, 2):
            assert len(logs[step]) == nb and all(during for _, during in logs[step]), logs[step]
            assert logs[step][0][0] == 0   # first bucket (the head's last layer) goes first
        for step in range(3):
            for k, g in out[step].items():
                if k.startswith("unused."):
                    assert g is None, k
                else:
                    torch.testing.assert_close(torch.from_numpy(g), exp[step][k], rtol=1e-5, atol=1e-6)


def _prepare_worker(rank, world, port, q, paths):
    import sys
    sys.path[:0] = paths
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from comet_amd.loop import CometAccelerator
        torch.manual_seed(1000 + rank)  # seed + rank, as set_seed_and_print(device_specific=True)
        net = torch.nn.Sequential(torch.nn.Linear(16, 32), torch.nn.BatchNorm1d(32), torch.nn.Linear(32, 4))
        net[1].running_mean.normal_()
        before = {k: v.clone() for k, v in net.state_dict().items()}
        opt = torch.optim.SGD(net.parameters(), lr=0.1)
        acc = CometAccelerator(device="cpu")
        net, _, opt, _ = acc.prepare(net, None, opt, None)
        q.put((rank, {k: v.numpy().copy() for k, v in before.items()},
               {k: v.detach().numpy().copy() for k, v in net.state_dict().items()}))
    finally:
        dist.destroy_process_group()


def test_prepare_broadcasts_rank0_weights():
    """CometAccelerator.prepare with world > 1 starts every rank from rank 0's parameters and
    buffers (DDP's _sync_module_states under accelerate.prepare), whatever each rank's seed."""
    import numpy as np
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_prepare_worker, args=(r, world, port, q, [ROOT, PKG])) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(world):
        rank, before, after = q.get(timeout=120)
        res[rank] = (before, after)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert not np.array_equal(res[0][0]["0.weight"], res[1][0]["0.weight"])  # the inits differed
    for k in res[0][1]:
        assert np.array_equal(res[0][1][k], res[0][0][k]), k     # rank 0 kept its own
        assert np.array_equal(res[1][1][k], res[0][0][k]), k     # rank 1 got rank 0's


def _local_worker(rank, world, port, q, paths):
    import sys
    sys.path[:0] = paths
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from comet_amd.ddp import GradBucketer
        net = _Net()
        bk = GradBucketer(net.parameters(), bucket_mb=0.004)
        for step in range(2):  # discovery + one bucketed step
            net.zero_grad(set_to_none=True)
            bk.prepare_backward()
            x, y = _data(rank, step)
            ((net(x) - y) ** 2).mean().backward()
            bk.finish_backward()
        net.zero_grad(set_to_none=True)
        x, y = _data(rank, 5)
        try:  # outside prepare / finish without the opt-in: refused (ranks would diverge unnoticed)
            ((net(x) - y) ** 2).mean().backward()
            raise AssertionError("a backward outside prepare/finish was accepted without bucketer.local")
        except RuntimeError as e:
            assert "outside prepare_backward" in str(e)
        net.zero_grad(set_to_none=True)
        bk.local = True
        ((net(x) - y) ** 2).mean().backward()  # explicit opt-in: local gradients
        bk.local = False
        q.put((rank, {k: p.grad.numpy().copy() for k, p in net.named_parameters() if p.grad is not None},
               len(bk.launch_log)))
    finally:
        dist.destroy_process_group()


def test_backward_outside_prepare_stays_local():
    """A backward outside prepare_backward / finish_backward raises unless `bucketer.local` is set;
    with it, it launches no collective and leaves each rank its own gradient (bench.py times the
    step that way to price the exposed all-reduce)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_local_worker, args=(r, world, port, q, [ROOT, PKG])) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, g, nlog = q.get(timeout=120)
        got[rank] = g
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank in range(world):
        net = _Net()
        x, y = _data(rank, 5)
        ((net(x) - y) ** 2).mean().backward()
        for k, p in net.named_parameters():
            if p.grad is not None:
                torch.testing.assert_close(torch.from_numpy(got[rank][k]), p.grad, rtol=1e-6, atol=1e-7)


def _record_worker(rank, world, port, q, paths):
    import sys
    sys.path[:0] = paths
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from comet_amd.ddp import GradBucketer
        net = _Net()
        bk = GradBucketer(net.parameters(), bucket_mb=0.004)
        res = []
        for step in range(2):  # discovery, then the rebuilt buckets
            bk.record = True
            bk.prepare_backward()
            x, y = _data(rank, step)
            ((net(x) - y) ** 2).mean().backward()
            bk.finish_backward()
            if step == 1:
                pre = {k: bk.pre_reduce_grad(p).detach().numpy().copy() for k, p in net.named_parameters()
                       if p.grad is not None}
                red = {k: p.grad.detach().numpy().copy() for k, p in net.named_parameters() if p.grad is not None}
                res = (pre, red)
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def test_record_keeps_pre_reduce_gradients():
    """GradBucketer.record: each bucket's copy taken just before its all-reduce holds this rank's own
    (local) gradient, and the reduced gradient is the mean of those copies over the ranks -- the
    exact exchange check the GPU simulated-ranks test uses (tests/test_configs_gpu.py)."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_record_worker, args=(r, world, port, q, [ROOT, PKG])) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, res = q.get(timeout=120)
        got[rank] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the local gradient of each rank at step 1
    net = _Net()
    local = {}
    for r in range(world):
        net.zero_grad(set_to_none=True)
        x, y = _data(r, 1)
        ((net(x) - y) ** 2).mean().backward()
        local[r] = {k: p.grad.clone() for k, p in net.named_parameters() if p.grad is not None}
    assert set(got[0][0]) == set(local[0])
    for r in range(world):
        pre, red = got[r]
        for k in pre:
            torch.testing.assert_close(torch.from_numpy(pre[k]), local[r][k], rtol=1e-6, atol=1e-7)
            mean = (torch.from_numpy(got[0][0][k]) + torch.from_numpy(got[1][0][k])) / 2
            torch.testing.assert_close(torch.from_numpy(red[k]), mean, rtol=1e-6, atol=1e-7)
