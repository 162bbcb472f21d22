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


def test_refuses_more_gpus_than_visible():
    r = _run(["--gpus", "2", "--no-cpu-baseline"])
    import torch
    if torch.cuda.device_count() >= 2:  # pragma: no cover - a multi-GPU host
        return
    assert r.returncode == 2
    assert "refusing" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "4", "--launcher-check"], env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "WORLD_SIZE=2" in r.stderr
