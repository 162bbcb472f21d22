"""Training step of the COMET path (train_e2epose2.py:45-186, train_eval_func_new_cp5.py:608-618,
790-803, train_util.py:311-332, 2099-2128) on libcomet_hip.so + RCCL.

  build_optimizer      AdamW(camera_predictor.parameters(), lr=cfg.train.lr) (torch defaults:
                       betas (0.9, 0.999), eps 1e-8, weight_decay 0.01) + WarmupCosineRestarts
  CometAdamW.step      clip_grad_norm_(max_norm) + AdamW as two kernels: comet_sq_norm_multi
                       (device scalar) and comet_adamw_multi (clip coefficient applied in-kernel,
                       no host sync); params without a gradient are skipped, as torch does
  train_step           forward -> loss.mean() -> backward -> (DDP all-reduce) -> clip + AdamW -> lr step
"""
import ctypes
import math

import torch

from . import _lib as L
from . import functional as F
from . import ops


class WarmupCosineRestarts:
    """train_util.py:2099-2128 (T_mult=1 path; the reference only uses T_mult=1)."""

    def __init__(self, optimizer, T_0, iters_per_epoch, T_mult=1, eta_min=0.0, warmup_ratio=0.1,
                 warmup_lr_init=1e-7, last_epoch=-1):
        self.optimizer = optimizer
        self.T_0 = T_0 * iters_per_epoch
        self.T_mult = T_mult
        self.eta_min = eta_min
        self.warmup_iters = int(T_0 * warmup_ratio * iters_per_epoch)
        self.warmup_lr_init = warmup_lr_init
        self.base_lrs = [optimizer.lr]
        self.last_epoch = last_epoch
        self.step()

    def get_lr(self):
        i_restart = self.last_epoch // self.T_0
        T_cur = self.last_epoch - i_restart * self.T_0
        if T_cur < self.warmup_iters:
            r = T_cur / self.warmup_iters
            return [self.warmup_lr_init + (b - self.warmup_lr_init) * r for b in self.base_lrs]
        tc = T_cur - self.warmup_iters
        Ti = self.T_0 - self.warmup_iters
        return [self.eta_min + (b - self.eta_min) * (1 + math.cos(math.pi * tc / Ti)) / 2 for b in self.base_lrs]

    def step(self):
        self.last_epoch += 1
        self.optimizer.lr = self.get_lr()[0]

    def get_last_lr(self):
        return [self.optimizer.lr]


class CometAdamW:
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, max_norm=None):
        self.params = [p for p in params if p.requires_grad]
        self.lr = lr
        self.betas = betas
        self.eps = eps
        self.weight_decay = weight_decay
        self.max_norm = max_norm
        self.state = {}
        self.step_count = 0
        self.last_sqnorm = None

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    def _with_grad(self):
        return [p for p in self.params if p.grad is not None]

    def grad_sqnorm(self, ps=None):
        ps = ps if ps is not None else self._with_grad()
        out = torch.zeros(1, device=ps[0].device, dtype=torch.float32)
        arr = (ctypes.c_void_p * len(ps))(*[p.grad.data_ptr() for p in ps])
        sz = (ctypes.c_int64 * len(ps))(*[p.numel() for p in ps])
        L.check(L.load().comet_sq_norm_multi(arr, sz, len(ps), out.data_ptr(), ops.stream()), "sq_norm")
        return out

    @torch.no_grad()
    def step(self, max_norm=None):
        """clip_grad_norm_(max_norm) (if given) then one AdamW step; returns the pre-clip grad
        squared norm as a device tensor (no host sync)."""
        ps = self._with_grad()
        if not ps:
            return None
        max_norm = max_norm if max_norm is not None else self.max_norm
        self.step_count += 1
        for p in ps:
            if p not in self.state:
                self.state[p] = (torch.zeros_like(p, dtype=torch.float32), torch.zeros_like(p, dtype=torch.float32))
        sq = self.grad_sqnorm(ps) if max_norm is not None and max_norm > 0 else None
        n = len(ps)
        P = (ctypes.c_void_p * n)(*[p.data_ptr() for p in ps])
        G = (ctypes.c_void_p * n)(*[p.grad.data_ptr() for p in ps])
        M = (ctypes.c_void_p * n)(*[self.state[p][0].data_ptr() for p in ps])
        V = (ctypes.c_void_p * n)(*[self.state[p][1].data_ptr() for p in ps])
        S = (ctypes.c_int64 * n)(*[p.numel() for p in ps])
        L.check(L.load().comet_adamw_multi(P, G, M, V, S, n, float(self.lr), float(self.betas[0]), float(self.betas[1]),
                                           float(self.eps), float(self.weight_decay), self.step_count,
                                           None if sq is None else sq.data_ptr(), float(max_norm or 0.0), ops.stream()),
                "adamw")
        F.refresh_weight_cache(ps)
        self.last_sqnorm = sq
        return sq


def build_optimizer(cfg, model, iters_per_epoch=1):
    """train_util.py:311-332: AdamW over camera_predictor.parameters() + WarmupCosineRestarts."""
    m = model.module if hasattr(model, "module") else model
    opt = CometAdamW(m.camera_predictor.parameters(), lr=cfg.train.lr, max_norm=cfg.train.get("clip_grad", 1.0))
    sched = WarmupCosineRestarts(opt, T_0=cfg.train.restart_num, iters_per_epoch=iters_per_epoch,
                                 warmup_ratio=cfg.warmup_ratio, warmup_lr_init=cfg.warmup_lr_init)
    return opt, sched


def train_step(model, images, gt_cameras, tracks, optimizer, lr_scheduler, cfg, ddp=None):
    """One optimisation step (train_eval_func_new_cp5.py:608-618, 790-803)."""
    preds = model(images, gt_cameras=gt_cameras, training=True, tracks=tracks)
    loss = preds["loss"]
    optimizer.zero_grad()
    if ddp is not None:
        ddp.prepare_backward()
    loss.backward()
    if ddp is not None:
        ddp.finish_backward()
    clip = cfg.train.get("clip_grad", 1.0)
    optimizer.step(max_norm=clip if clip and clip > 0 else None)
    lr_scheduler.step()
    return loss.detach(), preds
