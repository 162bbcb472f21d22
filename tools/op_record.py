"""Locate the first op whose output differs between repeated forward passes, with where it differs.

Every public function of comet_amd.ops is wrapped: pass 0 keeps a device copy of each tensor the
call returns (and of its `out=` tensor); passes 1 and 2 compare each call with pass 0 as it happens
(bit for bit) and record, for a differing call, its op name, argument shapes, the GEMM plan of the
call, the count / maximum of the differences and, for 2-D outputs, the rows and columns they occupy
(and which 256- / 128-row blocks). Outputs are allocated zeroed (torch.empty -> torch.zeros) so
rows or columns an op does not write compare equal. Run two at once to reproduce the two-ranks-on-
one-GPU variation (tools/gpu/steps.sh rec2).

    python tools/op_record.py [bf16|fp32] [B]
"""
import functools
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "comet-pose-estimation_amd")]

STATE = {"pass": 0, "i": 0}
KEEP = []      # pass 0: (name, shapes, plan, [tensors])
DIFFS = []     # passes 1..: (pass, call, name, shapes, plan, detail)


def _shape(a):
    return tuple(a.shape) if torch.is_tensor(a) else (a if isinstance(a, (int, float, str, type(None))) else type(a).__name__)


def _where(a, b):
    d = a != b
    if a.dtype.is_floating_point:
        d &= ~(torch.isnan(a) & torch.isnan(b))
    n = int(d.sum())
    if n == 0:
        return None
    diff = (a.float() - b.float()).abs()
    diff = torch.where(d, diff, torch.zeros_like(diff))
    info = f"{n} of {a.numel()} elements differ, max |diff| {diff.max().item():.3e} (max |ref| {b.float().abs().max().item():.3e})"
    if a.dim() >= 2:
        d2 = d.reshape(-1, a.shape[-1])
        rows = d2.any(1).nonzero().flatten()
        cols = d2.any(0).nonzero().flatten()
        info += (f"; rows {rows.numel()} in [{rows.min().item()}, {rows.max().item()}] of {d2.shape[0]},"
                 f" cols {cols.numel()} in [{cols.min().item()}, {cols.max().item()}] of {d2.shape[1]}")
        for tb in (256, 128, 32):
            blk = torch.unique(rows // tb)
            info += f"; {tb}-row blocks {blk.numel()}: {blk[:12].tolist()}"
        cb = torch.unique(cols // 64)
        info += f"; 64-col blocks {cb[:16].tolist()}"
        per_row = d2.sum(1)[rows]
        info += f"; per differing row {per_row.min().item()}..{per_row.max().item()} elements"
    return info


def wrap(name, fn, ops):
    @functools.wraps(fn)
    def w(*args, **kw):
        r = fn(*args, **kw)
        outs = list(r) if isinstance(r, (tuple, list)) else [r]
        if "out" in kw:
            outs.append(kw["out"])
        outs = [o for o in outs if torch.is_tensor(o) and o.is_cuda]
        shapes = [_shape(a) for a in args[:5]]
        plan = tuple(ops._PLAN) if "gemm" in name or "linear" in name else None
        i = STATE["i"]
        STATE["i"] += 1
        if STATE["pass"] < 0:
            pass  # warm-up pass: first-use weight casts and tables make extra calls
        elif STATE["pass"] == 0:
            KEEP.append((name, shapes, plan, [o.detach().clone() for o in outs]))
        elif i < len(KEEP) and sum(1 for d in DIFFS if d[0] == STATE["pass"]) < 20:
            ref = KEEP[i][3]
            for k, (o, rr) in enumerate(zip(outs, ref)):
                if o.shape != rr.shape:
                    DIFFS.append((STATE["pass"], i, name, shapes, plan, f"output {k} shape {tuple(o.shape)} vs {tuple(rr.shape)}"))
                    continue
                wh = _where(o.detach(), rr)
                if wh is not None:
                    DIFFS.append((STATE["pass"], i, name, shapes, plan, f"output {k}: {wh}"))
        return r
    return w


def main():
    from comet_amd import functional as F, ops
    from comet_amd.config import instantiate, load_config
    from comet_amd.models.utils import QuaternionCameras
    from oracle import prng
    from oracle.weights import comet_shapes
    _zeros, _zeros_like = torch.zeros, torch.zeros_like
    torch.empty = lambda *a, **k: _zeros(*a, **{x: y for x, y in k.items() if x != "memory_format"})
    torch.empty_like = lambda t, **k: _zeros_like(t, **k)
    for k in dir(ops):
        v = getattr(ops, k)
        if callable(v) and not k.startswith("_") and getattr(v, "__module__", "") == ops.__name__ and k not in ("stream", "dt"):
            setattr(ops, k, wrap(k, v, ops))
    dtype = torch.float32 if len(sys.argv) > 1 and sys.argv[1] == "fp32" else torch.bfloat16
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    T, S, N = 16, 512, 512
    cfg = load_config()
    torch.manual_seed(0)
    model = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg)
    model.load_state_dict(prng.make_state_dict(0, comet_shapes()), strict=True)
    model = model.cuda()
    img, tracks, gt = prng.synthetic_batch(37, B, T, S, S, N)
    img, tracks = img.cuda(), tracks.cuda()
    cams = QuaternionCameras(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"],
                             principal_point=gt["principal_point"], ratio=gt["ratio"], device="cuda")
    for it in range(-1, 3):
        STATE["pass"], STATE["i"] = it, 0
        with F.precision(dtype), torch.no_grad():
            model(img, gt_cameras=cams, training=True, tracks=tracks)
        torch.cuda.synchronize()
        n = STATE["i"]
        nd = sum(1 for d in DIFFS if d[0] == it)
        print(f"pass {it}: {n} op calls, {nd} differing outputs recorded", flush=True)
    print(f"pass 0 kept {sum(t.numel() * t.element_size() for k in KEEP for t in k[3]) / 2**30:.1f} GiB", flush=True)
    for p, i, name, shapes, plan, det in DIFFS:
        print(f"pass {p} call {i} {name} args {shapes} plan {plan}\n    {det}", flush=True)


if __name__ == "__main__":
    main()
