"""Training step of the COMET path (train_e2epose2.py:45-186, train_eval_func_new_cp5.py:608-618,
790-803, train_util.py:311-332, 2099-2128) on libcomet_hip.so + RCCL.

  build_optimizer      train_util.py:311-332: AdamW(camera_predictor.parameters(), lr=cfg.train.lr)
                       (torch defaults: betas (0.9, 0.999), eps 1e-8, weight_decay 0.01) +
                       WarmupCosineRestarts(T_0=cfg.train.restart_num, iters_per_epoch=len(dataloader))
  CometAdamW           a torch.optim.Optimizer (param_groups, state_dict / load_state_dict with
                       torch.optim.AdamW's state layout {step, exp_avg, exp_avg_sq}, so
                       accelerate.save_state / load_state round-trip it and an AdamW checkpoint of
                       the reference loads into it). step(): clip_grad_norm_(max_norm) + AdamW as
                       two kernels, comet_sq_norm_multi (device scalar) and comet_adamw_multi (clip
                       coefficient applied in-kernel, no host sync); params without a gradient are
                       skipped, as torch does
  WarmupCosineRestarts a torch LRScheduler (state_dict / get_last_lr like the reference's)
  train_step           forward -> loss.mean() -> backward -> (DDP all-reduce) -> clip + AdamW -> lr step
"""
import ctypes
import math

import torch

from . import _lib as L
from . import functional as F
from . import ops
from .profiler import PROF


class WarmupCosineRestarts(torch.optim.lr_scheduler.LRScheduler):
    """train_util.py:2099-2128: linear warmup from warmup_lr_init over warmup_ratio of each
    period, then cosine to eta_min; restarts every T_0 epochs (T_mult = 1) or geometrically
    growing periods (T_mult > 1)."""

    def __init__(self, optimizer, T_0, iters_per_epoch, T_mult=1, eta_min=0, warmup_ratio=0.1,
                 warmup_lr_init=1e-7, last_epoch=-1):
        self.T_0 = T_0 * iters_per_epoch
        self.T_mult = T_mult
        self.eta_min = eta_min
        self.warmup_iters = int(T_0 * warmup_ratio * iters_per_epoch)
        self.warmup_lr_init = warmup_lr_init
        super().__init__(optimizer, last_epoch)

    def _t_cur(self):
        e = self.last_epoch
        if self.T_mult == 1:
            return e - (e // self.T_0) * self.T_0
        n = int(math.log((e / self.T_0 * (self.T_mult - 1) + 1), self.T_mult))
        return e - self.T_0 * (self.T_mult ** n - 1) // (self.T_mult - 1)

    def get_lr(self):
        t = self._t_cur()
        if t < self.warmup_iters:
            r = t / self.warmup_iters
            return [self.warmup_lr_init + (b - self.warmup_lr_init) * r for b in self.base_lrs]
        tc = t - self.warmup_iters
        ti = self.T_0 - self.warmup_iters
        return [self.eta_min + (b - self.eta_min) * (1 + math.cos(math.pi * tc / ti)) / 2 for b in self.base_lrs]


class CometAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, max_norm=None):
        # like torch.optim.AdamW(model.camera_predictor.parameters()) in the reference, frozen
        # params (the DINOv2 backbone) are members that never receive a gradient
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.max_norm = max_norm
        self.last_sqnorm = None
        self._pending = None  # (max_norm, squared norm) from clip_grad_norm_, used by the next step

    def clip_grad_norm_(self, max_norm):
        """accelerator.clip_grad_norm_(params, max_norm) of the reference loop
        (train_eval_func_new_cp5.py:797): the total gradient norm now (device scalar, no sync);
        the scaling itself is applied inside the next step()'s AdamW kernel, so between this call
        and step() p.grad still holds the unclipped gradient (unlike accelerate, which scales in
        place); the stored norm belongs to the gradients of this moment and is dropped by the next
        step() whatever path it takes. Code that changes the gradients in between (accumulation,
        another backward) must call clip_grad_norm_ again."""
        sq = self.grad_sqnorm()
        self._pending = (float(max_norm), sq)
        return sq.sqrt()

    @property
    def lr(self):
        return self.param_groups[0]["lr"]

    @lr.setter
    def lr(self, v):
        for g in self.param_groups:
            g["lr"] = v

    def _with_grad(self):
        return [p for g in self.param_groups for p in g["params"] if p.grad is not None]

    def load_state_dict(self, state_dict):
        """torch.optim.Optimizer.load_state_dict, then every per-param `step` as a host float32
        scalar: a capturable / fused AdamW checkpoint keeps it on the device, and reading it there
        would cost one device sync per param and step."""
        super().load_state_dict(state_dict)
        for st in self.state.values():
            s = st.get("step")
            if torch.is_tensor(s) and (s.device.type != "cpu" or s.dtype != torch.float32):
                st["step"] = s.detach().to("cpu", torch.float32)

    @staticmethod
    def _check(p, st):
        """comet_adamw_multi takes raw f32 pointers: param, grad and both moments must be
        contiguous f32 tensors on the param's device, or the kernel would stride wrongly."""
        ts = (p, p.grad, st["exp_avg"], st["exp_avg_sq"])
        for t in ts:
            if t.dtype != torch.float32 or not t.is_contiguous() or t.device != p.device or t.shape != p.shape:
                raise L.CometHipError(f"CometAdamW: param / grad / moments must be contiguous float32 of the param's "
                                      f"shape on {p.device}; got {t.dtype} {tuple(t.shape)} on {t.device} "
                                      f"(contiguous={t.is_contiguous()})")

    def grad_sqnorm(self, ps=None):
        ps = ps if ps is not None else self._with_grad()
        for p in ps:
            g = p.grad
            if g.dtype != torch.float32 or not g.is_contiguous() or g.device != ps[0].device:
                raise L.CometHipError(f"CometAdamW: gradients must be contiguous float32 on {ps[0].device}; got "
                                      f"{g.dtype} on {g.device} (contiguous={g.is_contiguous()})")
        # out[0] and the per-workgroup partials of the fixed-order reduction in one allocation
        buf = torch.zeros(1 + L.SQ_NORM_PARTIALS, device=ps[0].device, dtype=torch.float32)
        out = buf[:1]
        arr = (ctypes.c_void_p * len(ps))(*[p.grad.data_ptr() for p in ps])
        sz = (ctypes.c_int64 * len(ps))(*[p.numel() for p in ps])
        e0 = PROF.start()
        L.check(L.load().comet_sq_norm_multi(arr, sz, len(ps), out.data_ptr(), buf[1:].data_ptr(), ops.stream()),
                "sq_norm")
        PROF.stop(e0, "comet_sq_norm_multi", 0.0, 4.0 * sum(p.numel() for p in ps))
        return out

    @torch.no_grad()
    def step(self, closure=None, max_norm=None):
        """clip_grad_norm_(max_norm) (if given) then one AdamW step; returns the pre-clip grad
        squared norm as a device tensor (no host sync)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        pend, self._pending = self._pending, None  # consumed on every path, the early return too
        ps = self._with_grad()
        if not ps:
            return loss
        if max_norm is None and pend is not None:
            max_norm, sq = pend
        else:
            max_norm = max_norm if max_norm is not None else self.max_norm
            sq = None
        clip = max_norm is not None and max_norm > 0
        if clip and sq is None:
            sq = self.grad_sqnorm(ps)
        for g in self.param_groups:
            # params of one launch share lr / betas / step count (torch keeps `step` per param;
            # params that skipped earlier steps form their own launch)
            by_step = {}
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                self._check(p, st)
                st["step"] += 1  # a host scalar (load_state_dict keeps it there): no device sync
                by_step.setdefault(int(st["step"].item()), []).append(p)
            b1, b2 = g["betas"]
            for step, plist in by_step.items():
                n = len(plist)
                P = (ctypes.c_void_p * n)(*[p.data_ptr() for p in plist])
                G = (ctypes.c_void_p * n)(*[p.grad.data_ptr() for p in plist])
                M = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg"].data_ptr() for p in plist])
                V = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg_sq"].data_ptr() for p in plist])
                S = (ctypes.c_int64 * n)(*[p.numel() for p in plist])
                e0 = PROF.start()
                L.check(L.load().comet_adamw_multi(P, G, M, V, S, n, float(g["lr"]), float(b1), float(b2),
                                                   float(g["eps"]), float(g["weight_decay"]), step,
                                                   None if sq is None else sq.data_ptr(),
                                                   float(max_norm) if clip else 0.0, ops.stream()), "adamw")
                # param, m, v read + written, grad read: 7 x 4 bytes per element
                PROF.stop(e0, "comet_adamw_multi", 0.0, 28.0 * sum(p.numel() for p in plist))
        F.refresh_weight_cache(ps)
        self.last_sqnorm = sq
        return loss if closure is not None else sq


def build_optimizer(cfg, model, dataloader):
    """train_util.py:311-332: AdamW over camera_predictor.parameters() + WarmupCosineRestarts
    with iters_per_epoch = len(dataloader) (an int is accepted as the length)."""
    m = model.module if hasattr(model, "module") else model
    iters = dataloader if isinstance(dataloader, int) else len(dataloader)
    clip = cfg.train.get("clip_grad", 1.0) if hasattr(cfg.train, "get") else 1.0
    opt = CometAdamW(m.camera_predictor.parameters(), lr=cfg.train.lr, max_norm=clip)
    sched = WarmupCosineRestarts(opt, T_0=cfg.train.restart_num, iters_per_epoch=iters,
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


def eval_step(model, images, gt_cameras, tracks, batch_size=None):
    """One evaluation step (train_eval_func_new_cp5.py:619-671, the test_fn branch abl_ours.py
    drives): model(..., training=False) under no_grad, loss.mean(), then the eval block's pose
    metrics (comet_amd.metrics.pose_metrics: R_avg, T_avg, Racc / Tacc, Auc_30/10/5/3, ...)
    added to the prediction dict."""
    from .metrics import pose_metrics
    with torch.no_grad():
        preds = model(images, gt_cameras=gt_cameras, training=False, tracks=tracks)
        loss = preds["loss"]
        preds["loss"] = loss.mean() if torch.is_tensor(loss) else loss
        if "gt_pose_enc" in preds and preds["gt_pose_enc"] is not None:
            preds.update(pose_metrics(preds, gt_cameras, batch_size or images.shape[0]))
    return preds
