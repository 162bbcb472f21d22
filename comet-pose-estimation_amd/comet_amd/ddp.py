"""Data-parallel gradient exchange for the COMET train step (replaces accelerate.prepare ->
DistributedDataParallel, train_e2epose2.py:83).

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI). Sequences shard over
ranks; the only exchange is the average of the camera-predictor gradients (115.9 M f32 values,
463.8 MB). Gradients live in flat buckets (~bucket_mb each, reverse registration order so the
first buckets to complete are the head's last layers); each param's .grad is a view into its
bucket, a post-accumulate-grad hook counts arrivals and launches an async all-reduce as soon as a
bucket is complete, overlapping RCCL with the rest of the backward. Parameters that receive no
gradient (the reference's unused modules) keep .grad = None afterwards, so AdamW skips them as
torch does; their (zero) slots are reduced with the last incomplete buckets.
"""
import torch
import torch.distributed as dist


class GradBucketer:
    def __init__(self, params, bucket_mb=64, group=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.backend = dist.get_backend(group) if dist.is_initialized() else None
        cap = int(bucket_mb * 1024 * 1024 // 4)
        self.buckets = []  # list of (flat tensor, [(param, offset, numel)])
        cur, size = [], 0
        for p in reversed(self.params):
            if cur and size + p.numel() > cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += p.numel()
        if cur:
            self.buckets.append(cur)
        self.flat = []
        self.slot = {}
        for bi, plist in enumerate(self.buckets):
            n = sum(p.numel() for p in plist)
            buf = torch.zeros(n, device=plist[0].device, dtype=torch.float32)
            off = 0
            for p in plist:
                self.slot[p] = (bi, off)
                off += p.numel()
            self.flat.append(buf)
        self.pending = [0] * len(self.buckets)
        self.launched = [False] * len(self.buckets)
        self.works = []
        self.arrived = set()
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    def _view(self, p):
        bi, off = self.slot[p]
        return self.flat[bi][off:off + p.numel()].view_as(p)

    def prepare_backward(self):
        for buf in self.flat:
            buf.zero_()
        for p in self.params:
            p.grad = self._view(p)
        self.pending = [len(pl) for pl in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.works = []
        self.arrived = set()

    def _launch(self, bi):
        if self.launched[bi]:
            return
        self.launched[bi] = True
        if self.world == 1:
            return
        op = dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM
        self.works.append((bi, dist.all_reduce(self.flat[bi], op=op, group=self.group, async_op=True)))

    def _on_grad(self, p):
        if p in self.arrived or p not in self.slot:
            return
        self.arrived.add(p)
        bi = self.slot[p][0]
        self.pending[bi] -= 1
        if self.pending[bi] == 0:
            self._launch(bi)

    def finish_backward(self):
        for bi in range(len(self.buckets)):
            self._launch(bi)
        for bi, w in self.works:
            w.wait()
            if self.backend != "nccl":
                self.flat[bi].mul_(1.0 / self.world)
        for p in self.params:
            if p not in self.arrived:
                p.grad = None

    def remove(self):
        for h in self._hooks:
            h.remove()
