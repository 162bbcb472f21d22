"""bench.py's multi-rank launcher (BASELINE configs[3]; the reference trains data-parallel through
`accelerate launch`, train_e2epose2.py:47,83), exercised on CPU:

* `--gpus 2` without a launcher spawns two ranks (gloo here via --launcher-check), both join one
  process group and a bucketed gradient all-reduce gives every rank the mean gradient;
* `--gpus N` with fewer than N visible GPUs refuses (exit 2) instead of reporting a 1-GPU run;
* under a launcher, WORLD_SIZE must agree with --gpus.
"""
import json
import os
import subprocess
import sys

from conftest import ROOT

BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=e)


def test_launcher_spawns_two_ranks_and_reduces():
    r = _run(["--gpus", "2", "--launcher-check"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    j = json.loads(lines[0])
    assert j["n_gpus"] == 2 and j["backend"] == "gloo" and j["reduced"] is True and j["buckets"] > 1


def _bench_module():
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_under_test", BENCH)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_refuses_more_gpus_than_visible():
    r = _run(["--gpus", "2", "--no-cpu-baseline"])
    b = _bench_module()
    have = b.visible_gpu_count()
    if have is not None and have >= 2:  # pragma: no cover - a multi-GPU host
        return
    assert r.returncode == 2
    assert "refusing" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_parent_counts_gpus_without_hip(tmp_path, monkeypatch):
    """The --gpus N parent never calls into HIP: torch's own device counters are made to raise,
    amdsmi is hidden, and the count comes from a fake KFD topology (a CPU node, two GPU nodes of
    which one render device is accessible), capped by *_VISIBLE_DEVICES; an unreadable topology
    makes main() refuse (exit 2) instead of falling back to hipGetDeviceCount."""
    import torch
    b = _bench_module()

    def boom(*a, **k):
        raise AssertionError("HIP device count called in the --gpus N parent")
    monkeypatch.setattr(torch._C, "_cuda_getDeviceCount", boom, raising=False)
    monkeypatch.setattr(torch.cuda, "device_count", boom)
    monkeypatch.setitem(sys.modules, "amdsmi", None)
    nodes, dri = tmp_path / "nodes", tmp_path / "dri"
    dri.mkdir()
    for i, (simd, minor) in enumerate([(0, None), (1024, 128), (1024, 129), (1024, 130)]):
        d = nodes / str(i)
        d.mkdir(parents=True)
        lines = [f"simd_count {simd}"] + ([f"drm_render_minor {minor}"] if minor is not None else [])
        (d / "properties").write_text("\n".join(lines) + "\n")
    for minor in (128, 130):
        (dri / f"renderD{minor}").write_text("")
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(var, raising=False)
    assert b.visible_gpu_count(str(nodes), str(dri)) == 2
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "0")
    assert b.visible_gpu_count(str(nodes), str(dri)) == 1
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    assert b.visible_gpu_count(str(tmp_path / "missing"), str(dri)) is None
    monkeypatch.setattr(b, "visible_gpu_count", lambda *a, **k: None)
    monkeypatch.setattr(b, "spawn_ranks", boom)
    monkeypatch.setattr(sys, "argv", [BENCH, "--gpus", "2", "--no-cpu-baseline"])
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        monkeypatch.delenv(k, raising=False)
    assert b.main() == 2


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4", "--launcher-check"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr


def test_gather_ops_count_the_bytes_they_read():
    """The bench line's TB/s for the gather ops uses the bytes the kernels read, not the whole map:
    CorrBlock sampling counts each track's (2r+4)^2 grid per level, at most every pixel of a frame
    once (the coarse 64 x 64 maps are covered by 512 tracks; the fine 31 x 31 patch maps are read only
    in their 10 x 10 windows)."""
    import torch
    sys.path.insert(0, os.path.join(ROOT, "comet-pose-estimation_amd"))
    from comet_amd import ops
    B, N, S, C, r = 2, 512, 3, 128, 4
    pyr = [torch.zeros(B * S, 64 >> l, 64 >> l, C, dtype=torch.bfloat16) for l in range(4)]
    rows = B * N * S
    feats, coords = torch.zeros(rows, C), torch.zeros(rows, 2)
    out = torch.zeros(rows, 4 * 81)
    n = ops._gather_bytes("corr_sample", (pyr, r, feats, coords, out, 0, B, N, S), None)
    maps = sum(p.numel() * 2 for p in pyr)  # every pixel once
    assert n == maps + feats.numel() * 4 + coords.numel() * 4 + out.numel() * 4
    fine = [torch.zeros(rows, 31 >> l, 31 >> l, 32, dtype=torch.bfloat16) for l in range(3)]
    o2 = torch.zeros(rows, 3 * 49)
    n2 = ops._gather_bytes("corr_sample", (fine, 3, torch.zeros(rows, 32), coords, o2, 0, rows, 1, 1), None)
    win = rows * (100 + 100 + 49) * 32 * 2
    assert n2 == win + rows * 32 * 4 + coords.numel() * 4 + o2.numel() * 4
    assert n2 < sum(p.numel() * 2 for p in fine) / 2
