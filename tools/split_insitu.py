"""Which split-K GEMMs of the camera head (headline bf16 fwd+bwd, tests/test_headline_gpu.py) differ
from their unsplit form, and by how much: every comet_gemm call whose plan splits K is re-run with
COMET_GEMM_NO_SMALLSPLIT=1 on a copy of its output and the two results are compared in place."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "comet-pose-estimation_amd"), os.path.join(ROOT, "tests")]
from comet_amd import _lib as L, ops  # noqa: E402

_orig = ops.gemm_raw
LOG = []


def gemm_raw(a, b, c, **kw):
    c0 = torch.empty_strided(c.shape, c.stride(), device=c.device, dtype=c.dtype).copy_(c)
    out = _orig(a, b, c, **kw)
    if ops._PLAN[0] == 2:  # 128 x 128 kernel: split when the workspace was requested
        os.environ["COMET_GEMM_NO_SMALLSPLIT"] = "1"
        try:
            kw2 = dict(kw)
            if kw.get("resid") is not None and kw["resid"].data_ptr() == c.data_ptr():
                kw2["resid"] = torch.empty_strided(c.shape, c.stride(), device=c.device, dtype=c.dtype).copy_(c0)
            if kw.get("aux") is not None:
                kw2["aux"] = kw["aux"].clone()
            c1 = torch.empty_strided(c.shape, c.stride(), device=c.device, dtype=c.dtype).copy_(c0)
            _orig(a, b, c1, **kw2)
            plan_unsplit = tuple(ops._PLAN)
        finally:
            del os.environ["COMET_GEMM_NO_SMALLSPLIT"]
        d = (c.double() - c1.double()).abs().max().item()
        m = c1.double().abs().max().item()
        if d / max(m, 1e-30) > 1e-2:
            import traceback
            print("".join(traceback.format_stack(limit=8)[:-1]))
            print({k: (v.shape, v.stride(), v.dtype) if torch.is_tensor(v) else v for k, v in kw.items()},
                  "a", a.shape, a.stride(), a.dtype, "b", b.shape, b.stride(), b.dtype, "c", c.shape, c.stride(),
                  "ptrs a b c resid", a.data_ptr(), b.data_ptr(), c.data_ptr(),
                  kw["resid"].data_ptr() if kw.get("resid") is not None else None)
        LOG.append((d / max(m, 1e-30), d, m, kw["m"], kw["n"], kw["k"], kw.get("layout_a"), kw.get("layout_b"),
                    str(a.dtype), str(c.dtype), plan_unsplit))
    return out


ops.gemm_raw = gemm_raw


def main():
    from comet_amd import functional as F
    from test_headline_gpu import GOLD, _cams
    from comet_amd.config import instantiate, load_config
    from oracle import prng
    from oracle.weights import comet_shapes
    gold = dict(np.load(GOLD, allow_pickle=False))
    seed_w, seed_x, B, T, H, W, N = [int(v) for v in gold["head_cfg"]]
    cfg = load_config()
    torch.manual_seed(0)
    model = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg)
    model.load_state_dict(prng.make_state_dict(seed_w, comet_shapes()), strict=True)
    model = model.cuda()
    img, tracks, gt = prng.synthetic_batch(seed_x, B, T, H, W, N)
    img = img.cuda()
    cp = model.camera_predictor
    refined = torch.from_numpy(gold["head_refined"]).cuda()
    conf = torch.from_numpy(gold["head_pred_score"]).cuda()
    with F.precision(torch.bfloat16):
        out = cp(img.reshape(-1, *img.shape[2:]), batch_size=B, gt_cameras=_cams(gt), iters=cfg["camera_iter"],
                 pred_trajectories=refined, track_confidence=conf)
        out["loss"].backward()
    torch.cuda.synchronize()
    print(f"{len(LOG)} calls on the 128 x 128 kernel")
    for r in sorted(LOG, reverse=True)[:40]:
        print(f"rel {r[0]:.3e} abs {r[1]:.3e} max {r[2]:.3e}  M{r[3]} N{r[4]} K{r[5]} L{r[6]}{r[7]} {r[8]}->{r[9]} unsplit plan {r[10]}")


if __name__ == "__main__":
    main()
