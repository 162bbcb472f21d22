"""Run-to-run determinism of the training step: the same model, inputs and weights through
forward + backward three times; every output tensor and every camera-predictor gradient compared
bit for bit against the first run (max |a - b| per key, only keys that differ are printed).

    python tools/determinism.py [B] [bf16|fp32]

Environment switches of the product (COMET_*) select the paths under test.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "comet-pose-estimation_amd")]


def flat(prefix, x, out):
    if torch.is_tensor(x):
        out[prefix] = x.detach().float().clone()
    elif isinstance(x, dict):
        for k, v in x.items():
            flat(f"{prefix}.{k}", v, out)
    elif isinstance(x, (list, tuple)):
        for i, v in enumerate(x):
            flat(f"{prefix}[{i}]", v, out)


def main():
    from comet_amd import functional as F
    from comet_amd.config import instantiate, load_config
    from comet_amd.models.utils import QuaternionCameras
    from oracle import prng
    from oracle.weights import comet_shapes
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    dtype = torch.float32 if len(sys.argv) > 2 and sys.argv[2] == "fp32" else torch.bfloat16
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
    runs = []
    for it in range(3):
        model.zero_grad(set_to_none=True)
        with F.precision(dtype):
            out = model(img, gt_cameras=cams, training=True, tracks=tracks)
            out["loss"].backward()
        torch.cuda.synchronize()
        rec = {}
        flat("out", out, rec)
        for k, p in model.named_parameters():
            if p.grad is not None:
                rec["grad." + k] = p.grad.detach().float().clone()
        runs.append(rec)
    for it in (1, 2):
        diff = []
        for k, v in runs[0].items():
            w = runs[it].get(k)
            if w is None or w.shape != v.shape:
                diff.append((float("inf"), k))
                continue
            d = (v - w).abs().max().item() if v.numel() else 0.0
            if d != 0.0 or torch.isnan(v).any().item() != torch.isnan(w).any().item():
                diff.append((d / max(v.abs().max().item(), 1e-30), k))
        diff.sort(reverse=True)
        print(f"run {it} vs run 0: {len(diff)} of {len(runs[0])} keys differ", flush=True)
        for d, k in diff[:25]:
            print(f"   {d:.3e} (rel to max)  {k}")


if __name__ == "__main__":
    main()
