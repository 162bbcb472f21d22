"""Debug mode of the COMET path (device-side bounds checks and a NaN / Inf check mode).

  * `make -C comet-pose-estimation_amd DEBUG=1` builds libcomet_hip_debug.so (COMET_DEBUG): every
    launch is followed by a device synchronise -- a fault is reported by the op that caused it --
    and a read of the device assertion word that COMET_DASSERT index checks inside the kernels set
    (patch origins inside the frame, ring rows of the row-resident convolution, ...). A failed check
    makes that op's C-ABI call return an error, which the Python wrapper raises as CometHipError
    naming the op. COMET_DEBUG=1 in the environment loads that library (comet_amd/_lib.py).
  * FiniteCheck(model): forward hooks on every submodule count NaN / Inf elements of each floating
    output on the device (comet_count_nonfinite) and raise naming the first module that produced
    one; check_grads(model) does the same for the parameters' gradients after a backward. Works
    with either library; it synchronises after every module, so use it for diagnosis, not timing.
"""
import ctypes

import torch

from . import _lib as L
from . import ops


def debug_library():
    """True when the loaded libcomet_hip is a `make DEBUG=1` build."""
    return L.load().comet_debug_flags(0) >= 0


def debug_flags(clear=True):
    """OR of the device assertion words read so far (debug library), or -1 (release library)."""
    return int(L.load().comet_debug_flags(1 if clear else 0))


def count_nonfinite(t):
    """Number of NaN / Inf elements of a CUDA f32 / bf16 tensor (one kernel + one sync)."""
    if not t.is_cuda or t.dtype not in (torch.float32, torch.bfloat16):
        raise L.CometHipError("count_nonfinite: a CUDA float32 / bfloat16 tensor is required")
    x = t.contiguous()
    cnt = torch.zeros(1, dtype=torch.int32, device=t.device)
    L.check(L.load().comet_count_nonfinite(ops.dt(x), x.data_ptr(), x.numel(), cnt.data_ptr(), ops.stream()),
            "comet_count_nonfinite")
    return int(cnt.item())


def _tensors(out):
    if torch.is_tensor(out):
        yield out
    elif isinstance(out, dict):
        for v in out.values():
            yield from _tensors(v)
    elif isinstance(out, (list, tuple)):
        for v in out:
            yield from _tensors(v)


class FiniteCheck:
    """with FiniteCheck(model): ... -- raise at the first submodule whose output holds a NaN / Inf."""

    def __init__(self, model, modules=None):
        self.model = model
        self.modules = modules
        self.handles = []

    def _hook(self, name):
        def f(mod, inp, out):
            for t in _tensors(out):
                if t.is_cuda and t.dtype in (torch.float32, torch.bfloat16) and t.numel():
                    n = count_nonfinite(t.detach())
                    if n:
                        raise L.CometHipError(f"non-finite values ({n} of {t.numel()}) in the output of "
                                              f"{name or 'the model'} ({type(mod).__name__})")
        return f

    def __enter__(self):
        for name, m in self.model.named_modules():
            if self.modules is None or name in self.modules:
                self.handles.append(m.register_forward_hook(self._hook(name)))
        return self

    def __exit__(self, *exc):
        for h in self.handles:
            h.remove()
        self.handles = []
        return False


def check_grads(model):
    """Raise naming the first parameter whose gradient holds a NaN / Inf."""
    for name, p in model.named_parameters():
        if p.grad is not None and p.grad.is_cuda:
            n = count_nonfinite(p.grad.detach())
            if n:
                raise L.CometHipError(f"non-finite values ({n} of {p.grad.numel()}) in the gradient of {name}")
