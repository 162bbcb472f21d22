"""Config boundary: the reference's OmegaConf YAML + Hydra `instantiate(_target_)`
(abl_ours.yaml:395-431, E2Epose2.py:78,91, track_predictor.py:43-56) without omegaconf/hydra.

`load_config` reads any of the reference YAML files (or configs/abl_ours.yaml here) into an
attribute dict; `instantiate` resolves the reference's `_target_` strings
(E2Epose2.COMET, models.track_predictor.TrackerPredictor, models.camera_predictor10.CameraPredictor,
models.track_modules.blocks.{BasicEncoder,ShallowEncoder},
models.track_modules.base_track_predictor.BaseTrackerPredictor) to this package's classes.
"""
import importlib
import os

import yaml


class AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            raise AttributeError(k) from None

    def __setattr__(self, k, v):
        self[k] = v

    @staticmethod
    def wrap(x):
        if isinstance(x, dict):
            return AttrDict({k: AttrDict.wrap(v) for k, v in x.items()})
        if isinstance(x, list):
            return [AttrDict.wrap(v) for v in x]
        return x


def load_config(path=None, **overrides):
    if path is None:
        path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "configs", "abl_ours.yaml")
    with open(path) as f:
        cfg = AttrDict.wrap(yaml.safe_load(f))
    for k, v in overrides.items():
        cur = cfg
        parts = k.split(".")
        for p in parts[:-1]:
            cur = cur[p]
        cur[parts[-1]] = v
    return cfg


def resolve_target(target):
    """Map a reference `_target_` string onto comet_amd.models.*."""
    t = target
    for pre in ("comet.models.", "models."):
        if t.startswith(pre):
            t = t[len(pre):]
            break
    mod, cls = t.rsplit(".", 1)
    return getattr(importlib.import_module("comet_amd.models." + mod), cls)


def instantiate(config, *args, _recursive_=False, **kwargs):
    C = resolve_target(config["_target_"])
    params = {k: v for k, v in config.items() if k != "_target_"}
    params.update(kwargs)
    return C(*args, **params)
