import sys, os, numpy as np, torch
sys.path.insert(0, "."); sys.path.insert(0, "comet-pose-estimation_amd")
from comet_amd.config import instantiate, load_config
from comet_amd.models.utils import QuaternionCameras
from comet_amd import functional as F
from oracle import prng
from oracle.weights import comet_shapes
g = dict(np.load("tests/golden/comet_golden_v1.npz"))
cfg = load_config(); torch.manual_seed(0)
m = instantiate(cfg.MODEL, _recursive_=False, cfg=cfg); m.load_state_dict(prng.make_state_dict(0, comet_shapes())); m = m.cuda()
img, tr, gt = prng.synthetic_batch(1, 1, 4, 128, 128, 16)
cams = QuaternionCameras(R=gt["R"], T_uvz=gt["T_uvz"], T=gt["T"], focal_length=gt["focal_length"], ratio=gt["ratio"], device="cuda")
cap = {}
def hook(n):
    def f(mod, i, o): cap[n] = o["x_norm_patchtokens"] if isinstance(o, dict) else o
    return f
cp = m.camera_predictor
cp.backbone.register_forward_hook(hook("tokens")); cp.trunk[3].register_forward_hook(hook("trunk")); cp.cross_attn_block[0].register_forward_hook(hook("tp0"))
m.track_predictor.fine_fnet.register_forward_hook(hook("pf")); cp.self_att[3].register_forward_hook(hook("sa3"))
with F.precision(torch.float32):
    out = m(img.cuda(), gt_cameras=cams, training=True, tracks=tr.cuda())
torch.cuda.synchronize()
def rel(a, b):
    a = a.detach().double().cpu(); b = torch.as_tensor(b).double()
    return f"max abs {(a-b).abs().max().item():.3e} / max ref {b.abs().max().item():.3e}"
print("tokens head", rel(cap["tokens"][:, :8], g["e2e_tokens_head"]))
print("tokens sums", rel(cap["tokens"].double().sum(dim=(1,2)), g["e2e_tokens_sum"]))
print("tp0", rel(cap["tp0"], g["e2e_tp0_out"]))
print("trunk", rel(cap["trunk"], g["e2e_trunk_out"]))
pf = cap["pf"]; S, N = 4, 16
mine = pf.reshape(N, S, 31, 31, 32)[:8, 0].permute(0, 3, 1, 2)
print("patch feat head", rel(mine, g["e2e_patch_feat_head"]))
print("pred enc", rel(out["pred_pose_enc"], g["e2e_pred_pose_enc"]))
print("score", out["_track_predictions"]["pred_score"].flatten()[:8])
