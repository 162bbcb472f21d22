"""Data-parallel gradient exchange for the COMET train step (replaces accelerate.prepare ->
DistributedDataParallel, train_e2epose2.py:83).

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI). Sequences shard over
ranks; the only exchange is the average of the camera-predictor gradients (115.9 M f32 values,
463.8 MB). Gradients live in flat f32 buckets (~25 MB); each param's .grad is a view into its
bucket and a post-accumulate-grad hook counts arrivals and launches an async all-reduce
(ReduceOp.AVG) as soon as its bucket is complete, overlapping RCCL with the rest of the backward.

Bucket layout (what torch DDP does with find_unused_parameters + bucket rebuilding):
  * step 1 ("discovery"): one provisional layout over every trainable param in reverse
    registration order; all buckets are reduced at finish_backward. The hooks record the order in
    which gradients arrive.
  * afterwards the buckets are rebuilt over the params that did receive a gradient, in rank 0's
    arrival order (broadcast once, so every rank cuts identical buckets). The reference's 2.28 M
    never-executed params (FeatureFusion, motion encoders, ...) are excluded, so no bucket waits
    on a gradient that never comes: each bucket's all-reduce starts during the backward.
    Excluded params keep .grad = None, so AdamW skips them as torch does.
Buckets launch in index order (a completed bucket waits for the lower ones), as torch's Reducer
does, so every rank issues the same sequence of collectives.
`static_used` (the params that receive gradients, in bucket order) skips discovery when the set is
known up front.
"""
import torch
import torch.distributed as dist


class GradBucketer:
    def __init__(self, params, bucket_mb=25, group=None, static_used=None):
        self.params = [p for p in params if p.requires_grad]
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.backend = dist.get_backend(group) if dist.is_initialized() else None
        self.cap = max(1, int(bucket_mb * 1024 * 1024 // 4))
        self.index = {p: i for i, p in enumerate(self.params)}
        self.discovering = static_used is None
        order = list(reversed(self.params)) if static_used is None else list(static_used)
        self._build(order)
        self.arrival = []
        self.launch_log = []  # (bucket, during_backward) of the last step, for tests / tracing
        self.in_backward = False
        # a backward outside prepare_backward / finish_backward raises unless `local` is set (the
        # bench's timing pass without the exchange): an unreduced gradient would let ranks diverge
        self.local = False
        # tests: keep a copy of every bucket as it was just before its all-reduce (pre_reduce[bi])
        self.record = False
        self.pre_reduce = {}
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self.params]

    # ---------------------------------------------------------------------------------------
    def _build(self, order):
        self.buckets = []
        cur, size = [], 0
        for p in order:
            if cur and size + p.numel() > self.cap:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += p.numel()
        if cur:
            self.buckets.append(cur)
        self.flat, self.slot = [], {}
        for bi, plist in enumerate(self.buckets):
            n = sum(p.numel() for p in plist)
            self.flat.append(torch.zeros(n, device=plist[0].device, dtype=torch.float32))
            off = 0
            for p in plist:
                self.slot[p] = (bi, off)
                off += p.numel()

    def _rebuild_from_arrival(self):
        idx = torch.tensor([self.index[p] for p in self.arrival], dtype=torch.int64)
        if self.world > 1:
            dev = self.flat[0].device if self.backend == "nccl" else torch.device("cpu")
            # every rank must have used the same set of params: MIN and MAX of the per-param
            # 'used' mask over ranks agree only then; all ranks see the same verdict and raise
            # together (instead of one rank raising next step while the others block in all_reduce)
            used = torch.zeros(len(self.params), dtype=torch.int32)
            used[idx] = 1
            lo, hi = used.to(dev), used.to(dev).clone()
            dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=self.group)
            dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=self.group)
            if not torch.equal(lo.cpu(), hi.cpu()):
                diff = (lo != hi).nonzero().flatten().tolist()
                raise RuntimeError(f"GradBucketer: ranks used different parameter sets in the discovery step "
                                   f"(param indices {diff[:8]}{'...' if len(diff) > 8 else ''})")
            n = torch.tensor([idx.numel()], dtype=torch.int64)
            n = n.to(dev)
            dist.broadcast(n, 0, group=self.group)
            buf = torch.zeros(int(n.item()), dtype=torch.int64, device=dev)
            if dist.get_rank(self.group) == 0:
                buf.copy_(idx.to(dev))
            dist.broadcast(buf, 0, group=self.group)
            idx = buf.cpu()
        used = [self.params[i] for i in idx.tolist()]
        grads = {p: p.grad for p in used}
        self._build(used)
        for p in used:  # keep this step's reduced values in the new layout
            v = self._view(p)
            if grads[p] is not None:
                v.copy_(grads[p])
            p.grad = v
        self.discovering = False

    def _view(self, p):
        bi, off = self.slot[p]
        return self.flat[bi][off:off + p.numel()].view_as(p)

    def pre_reduce_grad(self, p):
        """This rank's gradient of p as its bucket held it before the all-reduce (record=True)."""
        bi, off = self.slot[p]
        return self.pre_reduce[bi][off:off + p.numel()].view_as(p)

    # ---------------------------------------------------------------------------------------
    def prepare_backward(self):
        for buf in self.flat:
            buf.zero_()
        for p in self.params:
            p.grad = self._view(p) if p in self.slot else None
        self.pending = [len(pl) for pl in self.buckets]
        self.launched = [False] * len(self.buckets)
        self.next_launch = 0  # buckets launch in index order on every rank (RCCL needs one order)
        self.works = []
        self.arrived = set()
        self.arrival = []
        self.launch_log = []
        self.in_backward = True

    def _launch(self, bi):
        if self.launched[bi]:
            return
        self.launched[bi] = True
        self.launch_log.append((bi, self.in_backward))
        if self.record:  # enqueued before the collective, which waits for this stream's work
            self.pre_reduce[bi] = self.flat[bi].clone()
        if self.world == 1:
            return
        op = dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM
        self.works.append((bi, dist.all_reduce(self.flat[bi], op=op, group=self.group, async_op=True)))

    def _on_grad(self, p):
        if not self.in_backward:
            if self.local:  # explicit opt-in: the backward stays local (no bucket, no collective)
                return
            raise RuntimeError("GradBucketer: a gradient arrived outside prepare_backward/finish_backward "
                               "(use the accelerator's backward, or set bucketer.local = True for a "
                               "deliberately rank-local backward)")
        if p in self.arrived:
            return
        self.arrived.add(p)
        self.arrival.append(p)
        if p not in self.slot:
            raise RuntimeError("GradBucketer: a parameter that received no gradient in the discovery step now "
                               "has one (the graph changed); build the bucketer with static_used")
        bi = self.slot[p][0]
        self.pending[bi] -= 1
        if not self.discovering:
            # like torch's Reducer: a completed bucket waits for every lower-index bucket, so all
            # ranks issue their collectives in the same order whatever order the grads arrive in
            while self.next_launch < len(self.buckets) and self.pending[self.next_launch] == 0:
                self._launch(self.next_launch)
                self.next_launch += 1

    def finish_backward(self):
        self.in_backward = False
        for bi in range(len(self.buckets)):
            self._launch(bi)
        self.next_launch = len(self.buckets)
        for bi, w in self.works:
            w.wait()
            if self.backend != "nccl":
                self.flat[bi].mul_(1.0 / self.world)
        for p in self.params:
            if p not in self.arrived:
                p.grad = None
        if self.discovering:
            self._rebuild_from_arrival()

    def remove(self):
        for h in self._hooks:
            h.remove()
