"""Checkpoint boundary of the COMET path (SURVEY §8(b) "Checkpoint layout").

  load_model_weights      train_util.py:165-253 (train_e2epose2.py:81): add / strip the `module.`
                          prefix to match a DDP-wrapped / plain model, drop
                          camera_predictor.pose_branch.fc2.{weight,bias}, strict = not relax_load
  load_model_weights2     train_util.py:256-309 (abl_ours.py:56): the same prefix handling, no key
                          dropped; strict = not relax_load, and on a key mismatch a second
                          non-strict load (the reference's try / except)
  find_last_checkpoint    train_util.py:1852-1862: newest exp_dir/ckpt_DDDDDD (or all of them)
  save_state / load_state the accelerate.save_state(output_dir, safe_serialization=False) /
                          load_state directory the reference writes every ckpt_interval epochs and
                          auto-resumes from (train_e2epose2.py:92-113, 157-163, 185): the files
                          pytorch_model.bin (model state_dict; `module.` keys of a
                          DDP run's file accepted on load), optimizer.bin,
                          scheduler.bin and random_states_<rank>.pkl (step, python / numpy / torch
                          CPU / torch device RNG states), all torch.save archives, as accelerate
                          1.x names and fills them
  save_tdict / load_tdict tdict.pkl ({"epoch", "cfg"}, train_e2epose2.py:161); read back with an
                          unpickler that admits plain containers and scalars only

Every torch.load here is weights_only=True (RNG archives admit numpy's array reconstruction and
nothing else), so a checkpoint cannot execute code on load.
"""
import glob
import os
import pickle
import random
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn

MODEL_FILE = "pytorch_model.bin"
OPTIMIZER_FILE = "optimizer.bin"
SCHEDULER_FILE = "scheduler.bin"
RNG_FILE = "random_states_{}.pkl"
TDICT_FILE = "tdict.pkl"
DROPPED_V1 = ("camera_predictor.pose_branch.fc2.weight", "camera_predictor.pose_branch.fc2.bias")


def _load(path, device="cpu"):
    return torch.load(path, map_location=device, weights_only=True)


def _unwrap(model):
    return model.module if isinstance(model, (nn.parallel.DistributedDataParallel, nn.parallel.DataParallel)) else model


def _with_prefix(state_dict, want_prefix):
    keys = list(state_dict.keys())
    has = bool(keys) and keys[0].startswith("module.")
    if want_prefix and not has:
        return OrderedDict(("module." + k, v) for k, v in state_dict.items())
    if has and not want_prefix:
        return OrderedDict(((k[7:] if k.startswith("module.") else k), v) for k, v in state_dict.items())
    return state_dict


def load_model_weights(model, weights_path, device, relax_load):
    """train_util.py:165-253. The prefix decision looks at the first key only, as the reference
    does; the two pose_branch.fc2 tensors are always dropped, so a strict load (relax_load False)
    of a model that has them raises, exactly like the reference."""
    if not os.path.isfile(weights_path):
        raise ValueError(f"Weight file not found: {weights_path}")
    is_ddp = isinstance(model, nn.parallel.DistributedDataParallel)
    state_dict = _with_prefix(_load(weights_path, device), is_ddp)
    for name in DROPPED_V1:
        state_dict.pop(name, None)
    model.load_state_dict(state_dict, strict=not relax_load)
    return model.to(device)


def load_model_weights2(model, weights_path, device, relax_load=False):
    """train_util.py:256-309 (evaluation): prefix handled for DDP and DataParallel wrappers, every
    key kept; a strict load that fails on mismatched keys is retried non-strict."""
    if not os.path.isfile(weights_path):
        raise ValueError(f"Weight file not found: {weights_path}")
    is_ddp = isinstance(model, (nn.parallel.DistributedDataParallel, nn.parallel.DataParallel))
    state_dict = _with_prefix(_load(weights_path, device), is_ddp)
    try:
        model.load_state_dict(state_dict, strict=not relax_load)
    except RuntimeError as e:
        print(f"Weights loaded with strict=False. Error: {e}")
        model.load_state_dict(state_dict, strict=False)
    return model.to(device)


def find_last_checkpoint(exp_dir, all_checkpoints=False):
    """train_util.py:1852-1862."""
    fls = sorted(glob.glob(os.path.join(glob.escape(exp_dir), "ckpt_" + "[0-9]" * 6)))
    if not fls:
        return None
    return fls if all_checkpoints else fls[-1]


def checkpoint_path(exp_dir, epoch):
    """train_e2epose2.py:156: exp_dir/ckpt_{epoch:06}."""
    return os.path.join(exp_dir, f"ckpt_{epoch:06}")


def _rng_states(step):
    s = {"step": step, "random_state": random.getstate(), "numpy_random_seed": np.random.get_state(),
         "torch_manual_seed": torch.get_rng_state()}
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        s["torch_cuda_manual_seed"] = torch.cuda.get_rng_state_all()
    return s


def _numpy_safe_globals():
    mods = [np.ndarray, np.dtype]
    core = getattr(np, "_core", None) or np.core
    mods.append(core.multiarray._reconstruct)
    mods.extend(type(np.dtype(t)) for t in (np.uint32, np.float64, np.int64))
    return mods


def save_state(output_dir, model, optimizer=None, scheduler=None, step=0, process_index=0):
    """accelerate.Accelerator.save_state(output_dir, safe_serialization=False) for one model /
    optimizer / scheduler. pytorch_model.bin holds the model's state_dict without a `module.`
    prefix (this build never wraps the model; accelerate 1.x itself saves
    get_state_dict(model, unwrap=False), so the reference's multi-GPU runs write `module.` keys,
    which load_state accepts). As accelerate does, only process 0 writes the model, optimizer and
    scheduler files (accelerate.utils.save on the main process); every rank writes its own
    random_states_<rank>.pkl. No barrier, as accelerate's save_state without automatic naming has
    none: train_e2epose2.py:157-163 calls it from the main process alone."""
    os.makedirs(output_dir, exist_ok=True)
    if process_index == 0:
        torch.save(_unwrap(model).state_dict(), os.path.join(output_dir, MODEL_FILE))
        if optimizer is not None:
            torch.save(optimizer.state_dict(), os.path.join(output_dir, OPTIMIZER_FILE))
        if scheduler is not None:
            torch.save(scheduler.state_dict(), os.path.join(output_dir, SCHEDULER_FILE))
    torch.save(_rng_states(step), os.path.join(output_dir, RNG_FILE.format(process_index)))
    return output_dir


def load_state(input_dir, model, optimizer=None, scheduler=None, process_index=0, device=None, strict=True):
    """accelerate.Accelerator.load_state(input_dir): model (strict; a `module.` prefix written by
    a DDP-wrapped reference run is stripped), optimizer (state moved to the params' device),
    scheduler, RNG states of this process. -> the saved step counter."""
    if not os.path.isdir(input_dir):
        raise ValueError(f"Tried to find {input_dir} but folder does not exist")
    m = _unwrap(model)
    dev = device if device is not None else next(m.parameters()).device
    m.load_state_dict(_with_prefix(_load(os.path.join(input_dir, MODEL_FILE), dev), False), strict=strict)
    if optimizer is not None:
        optimizer.load_state_dict(_load(os.path.join(input_dir, OPTIMIZER_FILE), dev))
    if scheduler is not None:
        scheduler.load_state_dict(_load(os.path.join(input_dir, SCHEDULER_FILE)))
    step = 0
    rng = os.path.join(input_dir, RNG_FILE.format(process_index))
    if os.path.isfile(rng):
        with torch.serialization.safe_globals(_numpy_safe_globals()):
            s = torch.load(rng, map_location="cpu", weights_only=True)
        step = int(s.get("step", 0))
        random.setstate(tuple(tuple(x) if isinstance(x, list) else x for x in s["random_state"]))
        np.random.set_state(s["numpy_random_seed"])
        torch.set_rng_state(s["torch_manual_seed"])
        if "torch_cuda_manual_seed" in s and torch.cuda.is_available():
            torch.cuda.set_rng_state_all(s["torch_cuda_manual_seed"])
    return step


def _plain(x):
    if isinstance(x, dict):
        return {k: _plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_plain(v) for v in x]
    return x


def save_tdict(ckpt_path, epoch, cfg):
    """train_e2epose2.py:161: pickle.dump({"epoch": epoch, "cfg": cfg}); the config is stored as
    plain dicts / lists / scalars."""
    with open(os.path.join(ckpt_path, TDICT_FILE), "wb") as f:
        pickle.dump({"epoch": int(epoch), "cfg": _plain(cfg)}, f)


class _PlainUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        raise pickle.UnpicklingError(f"tdict.pkl: refusing to load {module}.{name}")


def load_tdict(ckpt_path):
    """tdict.pkl -> dict, or None when it is missing or holds anything but plain data (an
    OmegaConf object from the reference's writer): the caller then falls back to the directory
    name's epoch, as train_e2epose2.py:98-103 does on any load error."""
    try:
        with open(os.path.join(ckpt_path, TDICT_FILE), "rb") as f:
            return _PlainUnpickler(f).load()
    except (OSError, pickle.UnpicklingError, EOFError, AttributeError, ValueError):
        return None


def resume_epoch(last_checkpoint):
    """train_e2epose2.py:94-103: (epoch parsed from ckpt_DDDDDD or -1, start epoch from tdict or
    that epoch + 1)."""
    try:
        ep = int(os.path.basename(last_checkpoint)[5:])
    except (TypeError, ValueError):
        ep = -1
    td = load_tdict(last_checkpoint) if last_checkpoint else None
    start = td["epoch"] + 1 if td and "epoch" in td else ep + 1
    return ep, start
