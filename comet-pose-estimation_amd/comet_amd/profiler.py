"""Live per-kernel timing with HIP events (used by bench.py for the roofline numbers).

When enabled, ops.gemm_raw / ops.attention bracket each libcomet_hip launch with a pair of
events on the launching (current) stream and record the op's ALGORITHMIC work (2*M*N*K*batch
for GEMM, 4*B*H*Lq*Lk*D for attention). summary() resolves the events after a sync.
"""
import torch


class _Prof:
    def __init__(self):
        self.enabled = False
        self.detail = False  # key GEMM records by shape/layout (tools/gemm_shapes.py)
        self.records = []
        self._pool = []

    def _ev(self):
        if self._pool:
            return self._pool.pop()
        return torch.cuda.Event(enable_timing=True)

    def start(self):
        if not self.enabled:
            return None
        e = self._ev()
        e.record()
        return e

    def stop(self, e0, name, flops=0.0, nbytes=0.0):
        if e0 is None:
            return
        e1 = self._ev()
        e1.record()
        self.records.append((name, e0, e1, flops, nbytes))

    def reset(self):
        for _, a, b, _, _ in self.records:
            self._pool += [a, b]
        self.records = []

    def summary(self, instances=False):
        """{entry point: {launches, ms, flops, bytes}}; with instances=True keyed by the kernel
        instance a call landed on ("comet_gemm|big256.L00.bf16") instead of the entry point."""
        torch.cuda.synchronize()
        out = {}
        for name, a, b, fl, nb in self.records:
            if not instances:
                name = name.split("|", 1)[0]
            d = out.setdefault(name, {"launches": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0})
            d["launches"] += 1
            d["ms"] += a.elapsed_time(b)
            d["flops"] += fl
            d["bytes"] += nb
        return out


PROF = _Prof()
