import sys, numpy as np, torch
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
m.camera_predictor.trunk[3].register_forward_hook(lambda mod, i, o: cap.__setitem__("h", o))
with F.precision(torch.float32):
    out = m(img.cuda(), gt_cameras=cams, training=True, tracks=tr.cuda())
    out["loss"].backward()
torch.cuda.synchronize()
h = cap["h"].detach().double().cpu().reshape(4, 768)
enc = out["pred_pose_enc"].detach().double().cpu(); gte = out["gt_pose_enc"].double().cpu()
d = enc[:, 2]; ct = 200.0 / 9.0
exp = sum(ct * (d[t] - gte[t, 2]) * h[t] for t in range(1, 4))
got = m.camera_predictor.fc_depth.weight.grad.double().cpu()[0]
ref = torch.from_numpy(g["grad_full.fc_depth.weight"]).double()[0]
print("expected vs got", (exp - got).abs().max().item(), "expected vs ref", (exp - ref).abs().max().item(), "max", ref.abs().max().item())
print("loss", out["loss"].item(), g["e2e_loss"], "trans", out["loss_trans"].item(), g["e2e_loss_trans"], "rot", out["loss_rot"].item(), g["e2e_loss_rot"])
print("d", d.tolist(), "gt d", gte[:, 2].tolist())
print("ref enc d", g["e2e_pred_pose_enc"][:, 2].tolist())
