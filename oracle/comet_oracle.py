"""ORACLE / TEST INFRASTRUCTURE ONLY — CPU fp32 restatement of COMET's hot path.

Only tests/, tools/gen_golden.py, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
import this module; the product (comet-pose-estimation_amd/) never does. It restates, as pure
functions over a state_dict `P`, what the reference computes (file:line cited per function,
paths relative to wulibingbinglin/COMET-Pose-Estimation/comet/models/ unless noted), so that:
  * parity of the HIP path is checked against it on identical inputs;
  * it is itself pinned to the reference by tests/golden/ (vectors produced by importing the
    reference in the build container, tools/gen_golden.py);
  * it is the CPU baseline timed by bench.py ("kind": "port").

B > 1 semantics: every sequence is processed exactly as a B = 1 reference
call would process it (per-sequence reference frame, per-sequence score quirks); the loss is the
mean over sequences of the per-sequence loss.
"""
import math

import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------------------
# sin/cos tables — utils.py:724-871
# ----------------------------------------------------------------------------------------


def sincos_1d_from_grid(embed_dim, pos):
    """utils.py:807-832 (float64 omega, fp32 result)."""
    omega = torch.arange(embed_dim // 2, dtype=torch.double)
    omega /= embed_dim / 2.0
    omega = 1.0 / 10000 ** omega
    out = torch.einsum("m,d->md", pos.reshape(-1), omega)
    return torch.cat([torch.sin(out), torch.cos(out)], dim=1)[None].float()


def sincos_1d(embed_dim, length):
    """utils.py:758-777: get_1d_sincos_pos_embed -> (1, length, D)."""
    return sincos_1d_from_grid(embed_dim, torch.arange(length, dtype=torch.float))


def sincos_2d(embed_dim, gh, gw):
    """utils.py:724-755, 780-804: -> (1, D, gh, gw); first D/2 channels encode the column."""
    grid_h = torch.arange(gh, dtype=torch.float)
    grid_w = torch.arange(gw, dtype=torch.float)
    grid = torch.stack(torch.meshgrid(grid_w, grid_h, indexing="xy"), dim=0).reshape(2, 1, gh, gw)
    emb_h = sincos_1d_from_grid(embed_dim // 2, grid[0])
    emb_w = sincos_1d_from_grid(embed_dim // 2, grid[1])
    emb = torch.cat([emb_h, emb_w], dim=2)
    return emb.reshape(1, gh, gw, -1).permute(0, 3, 1, 2)


def embed_2d(xy, C):
    """utils.py:835-871 get_2d_embedding(cat_coords=False): [B,N,2] -> [B,N,2C]."""
    B, N, _ = xy.shape
    x, y = xy[:, :, 0:1], xy[:, :, 1:2]
    div = (torch.arange(0, C, 2, dtype=torch.float32) * (1000.0 / C)).reshape(1, 1, C // 2)
    pe_x = torch.zeros(B, N, C)
    pe_y = torch.zeros(B, N, C)
    pe_x[:, :, 0::2] = torch.sin(x * div)
    pe_x[:, :, 1::2] = torch.cos(x * div)
    pe_y[:, :, 0::2] = torch.sin(y * div)
    pe_y[:, :, 1::2] = torch.cos(y * div)
    return torch.cat([pe_x, pe_y], dim=2)


def harmonic_embedding(x, n_harmonic_functions=6, omega_0=1.0, logspace=True, append_input=True,
                       diag_cov=None):
    """minipytorch3d/harmonic_embedding.py:14-158."""
    if logspace:
        freqs = 2.0 ** torch.arange(n_harmonic_functions, dtype=torch.float32)
    else:
        freqs = torch.linspace(1.0, 2.0 ** (n_harmonic_functions - 1), n_harmonic_functions,
                               dtype=torch.float32)
    freqs = freqs * omega_0
    zero_half_pi = torch.tensor([0.0, 0.5 * torch.pi])
    embed = x[..., None] * freqs
    embed = embed[..., None, :, :] + zero_half_pi[..., None, None]
    embed = embed.sin()
    if diag_cov is not None:
        x_var = diag_cov[..., None] * torch.pow(freqs, 2)
        embed = embed * torch.exp(-0.5 * x_var)[..., None, :, :]
    embed = embed.reshape(*x.shape[:-1], -1)
    if append_input:
        return torch.cat([embed, x], dim=-1)
    return embed


# ----------------------------------------------------------------------------------------
# samplers — utils.py:874-974
# ----------------------------------------------------------------------------------------


def bilinear_sampler(inp, coords, padding_mode="border"):
    """utils.py:874-948 (align_corners=True, pixel coordinates, 2-D case)."""
    sizes = inp.shape[2:]
    coords = coords * torch.tensor([2 / max(s - 1, 1) for s in reversed(sizes)])
    coords = coords - 1
    return F.grid_sample(inp, coords, align_corners=True, padding_mode=padding_mode)


def sample_features4d(inp, coords):
    """utils.py:951-974: [B,C,H,W], [B,R,2] -> [B,R,C] (border padding)."""
    B = inp.shape[0]
    feats = bilinear_sampler(inp, coords.unsqueeze(2))
    return feats.permute(0, 2, 1, 3).reshape(B, -1, feats.shape[1] * feats.shape[3])


# ----------------------------------------------------------------------------------------
# transformer blocks — modules.py:119-344 over nn.MultiheadAttention(batch_first=True)
# ----------------------------------------------------------------------------------------


def linear(x, P, name, act=None):
    y = F.linear(x, P[name + ".weight"], P.get(name + ".bias"))
    if act == "gelu":
        y = F.gelu(y)
    elif act == "relu":
        y = F.relu(y)
    return y


def mlp(x, P, name):
    """modules.py:119-154 (GELU erf)."""
    return linear(linear(x, P, name + ".fc1", "gelu"), P, name + ".fc2")


def mha(xq, xkv, P, name, heads):
    """torch.nn.MultiheadAttention(batch_first=True) explicit path (need_weights=True):
    q*(1/sqrt(d)) then bmm, softmax, bmm, out_proj."""
    W = P[name + ".in_proj_weight"]
    b = P[name + ".in_proj_bias"]
    C = W.shape[1]
    d = C // heads
    q = F.linear(xq, W[:C], b[:C])
    k = F.linear(xkv, W[C:2 * C], b[C:2 * C])
    v = F.linear(xkv, W[2 * C:], b[2 * C:])
    B, Lq, _ = q.shape
    Lk = k.shape[1]
    q = q.reshape(B, Lq, heads, d).transpose(1, 2)
    k = k.reshape(B, Lk, heads, d).transpose(1, 2)
    v = v.reshape(B, Lk, heads, d).transpose(1, 2)
    q = q * math.sqrt(1.0 / float(d))
    a = torch.softmax(q @ k.transpose(-1, -2), dim=-1)
    o = (a @ v).transpose(1, 2).reshape(B, Lq, C)
    return F.linear(o, P[name + ".out_proj.weight"], P[name + ".out_proj.bias"])


def attn_block(x, P, name, heads):
    """modules.py:248-295: residual on the NORMED input (B-2)."""
    C = x.shape[-1]
    x = F.layer_norm(x, (C,), eps=1e-6)
    x = x + mha(x, x, P, name + ".attn", heads)
    return x + mlp(F.layer_norm(x, (C,), eps=1e-6), P, name + ".mlp")


def cross_attn_block(x, ctx, P, name, heads):
    """modules.py:298-344: norm_context affine eps 1e-5."""
    C = x.shape[-1]
    x = F.layer_norm(x, (C,), eps=1e-6)
    ctx = F.layer_norm(ctx, (C,), P[name + ".norm_context.weight"], P[name + ".norm_context.bias"], 1e-5)
    x = x + mha(x, ctx, P, name + ".cross_attn", heads)
    return x + mlp(F.layer_norm(x, (C,), eps=1e-6), P, name + ".mlp")


# ----------------------------------------------------------------------------------------
# DINOv2 ViT-B/14 with 4 registers (facebookresearch layout; camera_predictor10.py:601-617)
# ----------------------------------------------------------------------------------------


def dinov2_pos_embed(P, pre, gh, gw):
    """interpolate_pos_encoding: bicubic, antialias=True, size=(gh, gw) (dinov2_vitb14_reg)."""
    pos = P[pre + ".pos_embed"].float()
    cls_pos, patch_pos = pos[:, 0], pos[:, 1:]
    N = patch_pos.shape[1]
    M = int(math.sqrt(N))
    dim = pos.shape[-1]
    if M == gh and M == gw:
        return pos
    pp = F.interpolate(patch_pos.reshape(1, M, M, dim).permute(0, 3, 1, 2), size=(gh, gw),
                       mode="bicubic", antialias=True, align_corners=False)
    pp = pp.permute(0, 2, 3, 1).reshape(1, -1, dim)
    return torch.cat([cls_pos.unsqueeze(0), pp], dim=1)


def dinov2(img, P, pre="camera_predictor.backbone", heads=12, n_reg=4):
    """-> x_norm_patchtokens [B, gh*gw, 768]."""
    w = P[pre + ".patch_embed.proj.weight"]
    x = F.conv2d(img, w, P[pre + ".patch_embed.proj.bias"], stride=w.shape[-1])
    B, C, gh, gw = x.shape
    x = x.flatten(2).transpose(1, 2)
    x = torch.cat([P[pre + ".cls_token"].expand(B, -1, -1), x], dim=1)
    x = x + dinov2_pos_embed(P, pre, gh, gw)
    x = torch.cat([x[:, :1], P[pre + ".register_tokens"].expand(B, -1, -1), x[:, 1:]], dim=1)
    nb = len({k.split(".")[3] for k in P if k.startswith(pre + ".blocks.")})
    for i in range(nb):
        bp = f"{pre}.blocks.{i}"
        h = F.layer_norm(x, (C,), P[bp + ".norm1.weight"], P[bp + ".norm1.bias"], 1e-6)
        qkv = F.linear(h, P[bp + ".attn.qkv.weight"], P[bp + ".attn.qkv.bias"])
        L = qkv.shape[1]
        qkv = qkv.reshape(B, L, 3, heads, C // heads).permute(2, 0, 3, 1, 4)
        q, k, v = qkv[0], qkv[1], qkv[2]
        a = torch.softmax((q * (C // heads) ** -0.5) @ k.transpose(-1, -2), dim=-1)
        o = (a @ v).transpose(1, 2).reshape(B, L, C)
        o = F.linear(o, P[bp + ".attn.proj.weight"], P[bp + ".attn.proj.bias"])
        x = x + o * P[bp + ".ls1.gamma"]
        h = F.layer_norm(x, (C,), P[bp + ".norm2.weight"], P[bp + ".norm2.bias"], 1e-6)
        h = mlp(h, P, bp + ".mlp")
        x = x + h * P[bp + ".ls2.gamma"]
    x = F.layer_norm(x, (C,), P[pre + ".norm.weight"], P[pre + ".norm.bias"], 1e-6)
    return x[:, 1 + n_reg:]


# ----------------------------------------------------------------------------------------
# camera predictor — camera_predictor10.py
# ----------------------------------------------------------------------------------------
RESNET_MEAN = torch.tensor([0.485, 0.456, 0.406]).view(1, 3, 1, 1)
RESNET_STD = torch.tensor([0.229, 0.224, 0.225]).view(1, 3, 1, 1)


def image_features(images_flat, B, P, pre="camera_predictor", down_size=336, att_depth=4, heads=8):
    """camera_predictor10.py:622-687 -> rgb_feat [B, S, 768] (token 0 of every frame)."""
    x = images_flat
    if x.shape[-1] != down_size:
        x = F.interpolate(x, (down_size, down_size), mode="bilinear", align_corners=True)
    with torch.no_grad():
        x = (x - RESNET_MEAN) / RESNET_STD
        tok = dinov2(x, P, pre + ".backbone")
    tok = mlp(tok, P, pre + ".input_transform")
    C = tok.shape[-1]
    tok = F.layer_norm(tok, (C,), eps=1e-6)
    BS, Pn, _ = tok.shape
    S = BS // B
    tok = tok.reshape(B, S, Pn, C)
    g = int(math.sqrt(Pn))
    pos = sincos_2d(C, g, g).permute(0, 2, 3, 1)[None].reshape(1, 1, g * g, C)
    tok = tok + pos
    tok = torch.cat([P[pre + ".pose_token"].expand(B, S, -1, -1), tok], dim=-2)
    Pn = tok.shape[2]
    for i in range(att_depth):
        tok = attn_block(tok.reshape(B * S, Pn, C), P, f"{pre}.self_att.{i}", heads).reshape(B, S, Pn, C)
        f0 = tok[:, 0]
        fo = tok[:, 1:].reshape(B, (S - 1) * Pn, C)
        fo = cross_attn_block(fo, f0, P, f"{pre}.cross_att.{i}", heads).reshape(B, S - 1, Pn, C)
        tok = torch.cat([tok[:, 0:1], fo], dim=1)
    return tok[:, :, 0]


def quat_raw_mul(a, b):
    """minipytorch3d/rotation_conversions.py:398-417."""
    aw, ax, ay, az = torch.unbind(a, -1)
    bw, bx, by, bz = torch.unbind(b, -1)
    return torch.stack((aw * bw - ax * bx - ay * by - az * bz,
                        aw * bx + ax * bw + ay * bz - az * by,
                        aw * by - ax * bz + ay * bw + az * bx,
                        aw * bz + ax * by - ay * bx + az * bw), -1)


def quat_mul(a, b):
    """rotation_conversions.py:420-432 (standardised: w >= 0)."""
    ab = quat_raw_mul(a, b)
    return torch.where(ab[..., 0:1] < 0, -ab, ab)


def quat_inv(q):
    """rotation_conversions.py:435-449."""
    return q * torch.tensor([1, -1, -1, -1], dtype=q.dtype)


def camera_to_pose_encoding2(R, T_uvz, focal_length, ratio, min_fl=0.1, max_fl=30.0):
    """utils.py:631-688 for one sequence: R [S,4] (w,x,y,z), T_uvz [S,3] -> [S,8]."""
    S = R.shape[0]
    enc = torch.zeros(S, 8)
    enc[0, 3:7] = torch.tensor([1.0, 0.0, 0.0, 0.0])
    enc[..., 7:] = torch.clamp(focal_length, min=min_fl, max=max_fl)[..., 0:1]
    q_ref, t_ref = R[0], T_uvz[0]
    for i in range(1, S):
        q_rel = quat_mul(R[i], quat_inv(q_ref))
        du = (T_uvz[i, 0] - t_ref[0]) * ratio / (256 / 2)
        dv = (T_uvz[i, 1] - t_ref[1]) * ratio / (256 / 2)
        dd = ((T_uvz[i, 2] / t_ref[2]) - 1) * ratio
        enc[i, :3] = torch.stack([torch.as_tensor(du).reshape(()), torch.as_tensor(dv).reshape(()),
                                  torch.as_tensor(dd).reshape(())]).float()
        enc[i, 3:7] = q_rel
    return enc


INTRINSICS = {
    "spark": (1744.92206139719, 1746.58640701753, 737.272795902663, 528.471960188736),
    "AMD": (268.44444444, 268.44444444, 320.0, 240.0),
    "AMD_eval": (268.44444444, 268.44444444, 320.0, 240.0),
    "AMD_test": (214.75555555, 286.34074074, 256.0, 256.0),
}


def pose_encoding_to_camera2(enc, R_ref, T_ref, ratio, intri_type="AMD_eval"):
    """utils.py:312-403 for one sequence: enc [S,7] -> (R [S,4], T [S,3], focal [S,0])."""
    fx, fy, cx, cy = INTRINSICS[intri_type]
    n = enc.shape[0]
    u_ref = T_ref[0].expand(n, 1) if T_ref.dim() == 1 else T_ref[:, :1]
    t_ref = T_ref.unsqueeze(0).expand(n, 3)
    u_ref, v_ref, d_ref = t_ref[:, :1], t_ref[:, 1:2], t_ref[:, 2:]
    du = enc[:, :1] / ratio * (256 / 2)
    dv = enc[:, 1:2] / ratio * (256 / 2)
    dd = enc[:, 2:3] / ratio
    u = u_ref + du
    v = v_ref + dv
    d = d_ref * (dd + 1)
    T = torch.cat([(u - cx) * d / fx, (v - cy) * d / fy, d], dim=1)
    q = quat_mul(enc[:, 3:7], R_ref.unsqueeze(0).expand(n, 4))
    focal = torch.clamp(enc[:, 7:8], min=0.1, max=30)
    return q, T, focal


def camera_head(rgb_feat, P, pred_trajectories, track_confidence, pre="camera_predictor", heads=8):
    """camera_predictor10.py:329-413: T_P, T_F, trunk, GAPR -> (pred_uvd [B,S,3], quat [B,S,4])."""
    B, S, C = rgb_feat.shape
    if pred_trajectories is not None:
        t = linear(pred_trajectories, P, pre + ".traj_encoder.mlp.0")
        t = F.layer_norm(t, (t.shape[-1],), P[pre + ".traj_encoder.mlp.1.weight"], P[pre + ".traj_encoder.mlp.1.bias"], 1e-5)
        t = F.relu(t)
        t = linear(t, P, pre + ".traj_encoder.mlp.3")
        t = F.layer_norm(t, (C,), P[pre + ".traj_encoder.mlp.4.weight"], P[pre + ".traj_encoder.mlp.4.bias"], 1e-5)
        N = t.shape[2]
        w = linear(track_confidence.unsqueeze(-1), P, pre + ".confidence_attention.0", "relu")
        w = torch.sigmoid(linear(w, P, pre + ".confidence_attention.2"))
        ctx = (t * w).reshape(B * S, N, C)
        r = rgb_feat.reshape(B * S, 1, C)
        for i in range(4):
            r = cross_attn_block(r, ctx, P, f"{pre}.cross_attn_block.{i}", heads)
        rgb_feat = rgb_feat + r.reshape(B, S, C)
    rgb_feat = rgb_feat + sincos_1d(C, S).expand(B, -1, -1)
    for i in range(4):
        rgb_feat = attn_block(rgb_feat, P, f"{pre}.trunk.{i}", heads)
    rot = mlp(rgb_feat, P, pre + ".pose_branch")
    uv = linear(rgb_feat, P, pre + ".fc_translation2d")
    d = linear(rgb_feat, P, pre + ".fc_depth")
    uvd = torch.cat([uv, d], dim=-1)
    rot = F.normalize(rot, p=2, dim=-1, eps=1e-8)
    return uvd, rot


def pose_loss(uvd, rot, gt_enc_list, weight_trans=1.0, weight_rot=2.0):
    """camera_predictor10.py:420-438 per sequence; mean over sequences (B-1)."""
    losses, lt, lr = [], [], []
    for b, gt in enumerate(gt_enc_list):
        tl = F.mse_loss(uvd[b, 1:].reshape(-1, 3), gt[1:, :3]) * 100
        rl = F.mse_loss(rot[b, 1:].reshape(-1, 4), gt[1:, 3:7]) * 100
        losses.append(weight_trans * tl + weight_rot * rl)
        lt.append(tl)
        lr.append(rl)
    n = len(losses)
    return sum(losses) / n, sum(lt) / n, sum(lr) / n


def camera_predictor(images_flat, B, P, gt=None, pred_trajectories=None, track_confidence=None,
                     intri_type="AMD_eval", pre="camera_predictor"):
    """camera_predictor10.py:288-484 (gt = dict(R [B*S,4], T_uvz [B*S,3], focal_length [B*S,2], ratio))."""
    rgb = image_features(images_flat, B, P, pre)
    S = rgb.shape[1]
    uvd, rot = camera_head(rgb, P, pred_trajectories, track_confidence, pre)
    out = {}
    gt_encs = None
    if gt is not None:
        gt_encs = [camera_to_pose_encoding2(gt["R"][b * S:(b + 1) * S], gt["T_uvz"][b * S:(b + 1) * S],
                                            gt["focal_length"][b * S:(b + 1) * S], gt["ratio"]) for b in range(B)]
        loss, lt, lr = pose_loss(uvd, rot, gt_encs)
        out.update(loss=loss, loss_trans=lt, loss_rot=lr, gt_pose_enc=torch.cat(gt_encs, 0))
    uvd = uvd.clone()
    rot = rot.clone()
    uvd[:, 0, :] = 0
    rot[:, 0, :] = torch.tensor([1.0, 0.0, 0.0, 0.0])
    enc = torch.cat([uvd, rot], dim=-1)
    out["pred_pose_enc"] = enc.reshape(-1, 7)
    if gt is not None:
        Rs, Ts = [], []
        for b in range(B):
            q, T, _ = pose_encoding_to_camera2(enc[b], gt["R"][b * S], gt["T_uvz"][b * S], gt["ratio"], intri_type)
            Rs.append(q)
            Ts.append(T)
        out["pred_R"] = torch.cat(Rs, 0)
        out["pred_T"] = torch.cat(Ts, 0)
    return out


# ----------------------------------------------------------------------------------------
# ablation heads — camera_predictor_abl_{time,track,uvz,all}.py (abl_*.yaml), from rgb_feat
# ----------------------------------------------------------------------------------------
ABLATIONS = {
    # (use T_P, add its result, time embedding + trunk, single 7-output head with encoding 3)
    "ours": (True, True, True, False),     # camera_predictor10.py
    "time": (True, True, False, False),    # camera_predictor_abl_time.py:364-381 (T_F commented out)
    "track": (True, False, True, False),   # camera_predictor_abl_track.py:348 (residual commented out)
    "uvz": (True, True, True, True),       # camera_predictor_abl_uvz.py:153, 379-436
    "all": (False, False, False, True),    # camera_predictor_abl_all.py
}


def camera_to_pose_encoding3(R, T):
    """utils.py:591-627 for one sequence: R [S,4], T (xyz) [S,3] -> [S,7]."""
    S = R.shape[0]
    enc = torch.zeros(S, 7)
    enc[0, 3:7] = torch.tensor([1.0, 0.0, 0.0, 0.0])
    for i in range(1, S):
        enc[i, :3] = T[i] - T[0]
        enc[i, 3:7] = quat_mul(R[i], quat_inv(R[0]))
    return enc


def pose_encoding_to_camera3(enc, R_ref, T_ref):
    """utils.py:270-310 for one sequence: enc [S,7] -> (R = dq * q0, T = T0 + dxyz, focal 2.0)."""
    n = enc.shape[0]
    T = T_ref.unsqueeze(0).expand(n, 3) + enc[:, :3]
    q = quat_mul(enc[:, 3:7], R_ref.unsqueeze(0).expand(n, 4))
    return q, T, torch.full((n, 1), 2.0)


def ablation_head(rgb_feat, P, variant, gt=None, pred_trajectories=None, track_confidence=None,
                  intri_type="AMD_eval", pre="camera_predictor", heads=8):
    """CameraPredictor.forward from rgb_feat_init for one of ABLATIONS (camera_predictor10.py:288-484
    and the abl_* files): dict(pred_pose_enc [B*S,7], gt_pose_enc, loss, loss_trans, loss_rot,
    pred_R, pred_T)."""
    use_tp, tp_res, use_time, single = ABLATIONS[variant]
    B, S, C = rgb_feat.shape
    if use_tp and tp_res and pred_trajectories is not None:
        t = linear(pred_trajectories, P, pre + ".traj_encoder.mlp.0")
        t = F.layer_norm(t, (t.shape[-1],), P[pre + ".traj_encoder.mlp.1.weight"], P[pre + ".traj_encoder.mlp.1.bias"], 1e-5)
        t = linear(F.relu(t), P, pre + ".traj_encoder.mlp.3")
        t = F.layer_norm(t, (C,), P[pre + ".traj_encoder.mlp.4.weight"], P[pre + ".traj_encoder.mlp.4.bias"], 1e-5)
        N = t.shape[2]
        w = linear(track_confidence.unsqueeze(-1), P, pre + ".confidence_attention.0", "relu")
        w = torch.sigmoid(linear(w, P, pre + ".confidence_attention.2"))
        ctx = (t * w).reshape(B * S, N, C)
        r = rgb_feat.reshape(B * S, 1, C)
        for i in range(4):
            r = cross_attn_block(r, ctx, P, f"{pre}.cross_attn_block.{i}", heads)
        rgb_feat = rgb_feat + r.reshape(B, S, C)
    if use_time:
        rgb_feat = rgb_feat + sincos_1d(C, S).expand(B, -1, -1)
        for i in range(4):
            rgb_feat = attn_block(rgb_feat, P, f"{pre}.trunk.{i}", heads)
    out = {}
    if single:
        pred = mlp(rgb_feat, P, pre + ".pose_branch")
        uvd, rot = pred[..., :3], F.normalize(pred[..., 3:7], p=2, dim=-1, eps=1e-8)
    else:
        rot = F.normalize(mlp(rgb_feat, P, pre + ".pose_branch"), p=2, dim=-1, eps=1e-8)
        uvd = torch.cat([linear(rgb_feat, P, pre + ".fc_translation2d"), linear(rgb_feat, P, pre + ".fc_depth")], -1)
    if gt is not None:
        if single:
            encs = [camera_to_pose_encoding3(gt["R"][b * S:(b + 1) * S], gt["T"][b * S:(b + 1) * S]) for b in range(B)]
        else:
            encs = [camera_to_pose_encoding2(gt["R"][b * S:(b + 1) * S], gt["T_uvz"][b * S:(b + 1) * S],
                                             gt["focal_length"][b * S:(b + 1) * S], gt["ratio"]) for b in range(B)]
        loss, lt, lr = pose_loss(uvd, rot, encs)
        out.update(loss=loss, loss_trans=lt, loss_rot=lr, gt_pose_enc=torch.cat(encs, 0))
    uvd, rot = uvd.clone(), rot.clone()
    uvd[:, 0, :] = 0
    rot[:, 0, :] = torch.tensor([1.0, 0.0, 0.0, 0.0])
    enc = torch.cat([uvd, rot], dim=-1)
    out["pred_pose_enc"] = enc.reshape(-1, 7)
    if gt is not None:
        Rs, Ts = [], []
        for b in range(B):
            if single:
                q, T, _ = pose_encoding_to_camera3(enc[b], gt["R"][b * S], gt["T"][b * S])
            else:
                q, T, _ = pose_encoding_to_camera2(enc[b], gt["R"][b * S], gt["T_uvz"][b * S], gt["ratio"], intri_type)
            Rs.append(q)
            Ts.append(T)
        out["pred_R"], out["pred_T"] = torch.cat(Rs, 0), torch.cat(Ts, 0)
    return out


# ----------------------------------------------------------------------------------------
# keypoint initialisation helpers
# ----------------------------------------------------------------------------------------
def simple_nms(scores, r):
    """LightGlue simple_nms / glue-factory batched_nms (superpoint_open.py:34-48) on [B, H, W]."""
    mp = lambda t: F.max_pool2d(t, kernel_size=2 * r + 1, stride=1, padding=r)  # noqa: E731
    zeros = torch.zeros_like(scores)
    max_mask = scores == mp(scores)
    for _ in range(2):
        supp = mp(max_mask.float()) > 0
        supp_scores = torch.where(supp, zeros, scores)
        max_mask = max_mask | ((supp_scores == mp(supp_scores)) & ~supp)
    return torch.where(max_mask, scores, zeros)


def filter_keypoints(pts, mask):
    """RNG-free part of filter_and_pad (train_eval_func_new_cp5.py:272-282): keypoints whose rounded,
    clamped pixel lies in the mask, in input order."""
    H, W = mask.shape
    xs = pts[:, 0].round().clamp(0, W - 1).long()
    ys = pts[:, 1].round().clamp(0, H - 1).long()
    return pts[mask.bool()[ys, xs]]


# ----------------------------------------------------------------------------------------
# tracker CNNs — modules.py:39-116, blocks.py:27-202 (NCHW, InstanceNorm2d affine=False)
# ----------------------------------------------------------------------------------------


def conv(x, P, name, stride=1, padding=0):
    return F.conv2d(x, P[name + ".weight"], P[name + ".bias"], stride=stride, padding=padding)


def residual_block(x, P, name, stride):
    """modules.py:39-116 with norm_fn='instance', kernel 3, padding 1."""
    y = F.relu(F.instance_norm(conv(x, P, name + ".conv1", stride, 1)))
    y = F.relu(F.instance_norm(conv(y, P, name + ".conv2", 1, 1)))
    if stride != 1:
        x = F.instance_norm(conv(x, P, name + ".downsample.0", stride, 0))
    return F.relu(x + y)


def basic_encoder(x, P, name, stride=4):
    """blocks.py:27-111."""
    _, _, H, W = x.shape
    x = F.relu(F.instance_norm(conv(x, P, name + ".conv1", 2, 3)))
    a = residual_block(x, P, name + ".layer1.0", 1)
    a = residual_block(a, P, name + ".layer1.1", 1)
    b = residual_block(a, P, name + ".layer2.0", 2)
    b = residual_block(b, P, name + ".layer2.1", 1)
    c = residual_block(b, P, name + ".layer3.0", 2)
    c = residual_block(c, P, name + ".layer3.1", 1)
    d = residual_block(c, P, name + ".layer4.0", 2)
    d = residual_block(d, P, name + ".layer4.1", 1)
    size = (H // stride, W // stride)
    a, b, c, d = [F.interpolate(t, size, mode="bilinear", align_corners=True) for t in (a, b, c, d)]
    x = conv(torch.cat([a, b, c, d], dim=1), P, name + ".conv2", 1, 1)
    x = F.relu(F.instance_norm(x))
    return conv(x, P, name + ".conv3")


def shallow_encoder(x, P, name, stride=1):
    """blocks.py:114-196."""
    _, _, H, W = x.shape
    x = F.relu(F.instance_norm(conv(x, P, name + ".conv1", 2, 1)))
    tmp = residual_block(x, P, name + ".layer1", 2)
    x = x + F.interpolate(tmp, x.shape[-2:], mode="bilinear", align_corners=True)
    tmp = residual_block(tmp, P, name + ".layer2", 2)
    x = x + F.interpolate(tmp, x.shape[-2:], mode="bilinear", align_corners=True)
    x = conv(x, P, name + ".conv2") + x
    return F.interpolate(x, (H // stride, W // stride), mode="bilinear", align_corners=True)


# ----------------------------------------------------------------------------------------
# tracker predictor — track_modules/base_track_predictor.py, blocks.py:205-429
# ----------------------------------------------------------------------------------------


def update_former(x, P, name, space, heads=8, n_virtual=64):
    """blocks.py:205-348: [B, N, T, Din] -> [B, N, T, Dout]."""
    tokens = linear(x, P, name + ".input_transform")
    init = tokens
    B, _, T, C = tokens.shape
    if space:
        vt = P[name + ".virual_tracks"].repeat(B, 1, T, 1)
        tokens = torch.cat([tokens, vt], dim=1)
    N = tokens.shape[1]
    depth = len({k.split(".")[len(name.split(".")) + 1] for k in P if k.startswith(name + ".time_blocks.")})
    for i in range(depth):
        tt = attn_block(tokens.reshape(B * N, T, C), P, f"{name}.time_blocks.{i}", heads)
        tokens = tt.view(B, N, T, C)
        if space:
            st = tokens.permute(0, 2, 1, 3).reshape(B * T, N, C)
            pt, vt = st[:, :N - n_virtual], st[:, N - n_virtual:]
            vt = cross_attn_block(vt, pt, P, f"{name}.space_virtual2point_blocks.{i}", heads)
            vt = attn_block(vt, P, f"{name}.space_virtual_blocks.{i}", heads)
            pt = cross_attn_block(pt, vt, P, f"{name}.space_point2virtual_blocks.{i}", heads)
            st = torch.cat([pt, vt], dim=1)
            tokens = st.view(B, T, N, C).permute(0, 2, 1, 3)
    if space:
        tokens = tokens[:, :N - n_virtual]
    tokens = tokens + init
    return linear(tokens, P, name + ".flow_head")


def corr_pyramid(fmaps, levels):
    """blocks.py:351-374: average-pool pyramid."""
    B, S, C, H, W = fmaps.shape
    pyr = [fmaps]
    for _ in range(levels - 1):
        f = F.avg_pool2d(fmaps.reshape(B * S, C, H, W), 2, stride=2)
        _, _, H, W = f.shape
        fmaps = f.reshape(B, S, C, H, W)
        pyr.append(fmaps)
    return pyr


def corr_sample(pyr, targets, coords, radius):
    """blocks.py:376-429 (CorrBlock.corr then .sample, zeros padding)."""
    B, S, N, C = targets.shape
    r = radius
    out = []
    for i, fm in enumerate(pyr):
        H, W = fm.shape[-2:]
        corrs = torch.matmul(targets, fm.view(B, S, C, H * W)).view(B, S, N, H, W)
        corrs = corrs / torch.sqrt(torch.tensor(C).float())
        dx = torch.linspace(-r, r, 2 * r + 1)
        dy = torch.linspace(-r, r, 2 * r + 1)
        delta = torch.stack(torch.meshgrid(dy, dx, indexing="ij"), axis=-1)
        c = coords.reshape(B * S * N, 1, 1, 2) / 2 ** i + delta.view(1, 2 * r + 1, 2 * r + 1, 2)
        s = bilinear_sampler(corrs.reshape(B * S * N, 1, H, W), c, padding_mode="zeros")
        out.append(s.view(B, S, N, -1))
    return torch.cat(out, dim=-1)


def tracker_predictor(query_points, fmaps, P, name, iters, stride, down_ratio, corr_levels,
                      corr_radius, latent_dim, fine, space):
    """base_track_predictor.py:95-284 with TRACKorPOSE=False (query_points [B,N,2])."""
    B, N, _ = query_points.shape
    _, S, C, HH, WW = fmaps.shape
    if down_ratio > 1:
        query_points = query_points / float(down_ratio)
        query_points = query_points / float(stride)
    coords = query_points.clone().reshape(B, 1, N, 2).repeat(1, S, 1, 1)
    query_feat = sample_features4d(fmaps[:, 0], coords[:, 0])
    track_feats = query_feat.unsqueeze(1).repeat(1, S, 1, 1)
    coords_backup = coords.clone()
    pyr = corr_pyramid(fmaps, corr_levels)
    tdim = corr_levels * (corr_radius * 2 + 1) ** 2 + latent_dim * 2
    if fine:
        tdim += 4 if tdim % 2 == 0 else 5
    else:
        tdim += (4 - tdim % 4) % 4
    preds = []
    pos = sincos_2d(tdim, HH, WW)
    for _ in range(iters):
        fcorrs = corr_sample(pyr, track_feats, coords, corr_radius)
        cd = fcorrs.shape[3]
        fcorrs_ = fcorrs.permute(0, 2, 1, 3).reshape(B * N, S, cd)
        flows = (coords - coords[:, 0:1]).permute(0, 2, 1, 3).reshape(B * N, S, 2)
        flows_emb = torch.cat([embed_2d(flows, latent_dim // 2), flows], dim=-1)
        tf_ = track_feats.permute(0, 2, 1, 3).reshape(B * N, S, latent_dim)
        x = torch.cat([flows_emb, fcorrs_, tf_], dim=2)
        if x.shape[2] < tdim:
            x = torch.cat([x, torch.zeros(B * N, S, tdim - x.shape[2])], dim=2)
        spe = sample_features4d(pos.expand(B, -1, -1, -1), coords[:, 0]).reshape(B * N, 1, tdim)
        x = (x + spe).reshape(B, N, S, tdim)
        delta = update_former(x, P, name + ".updateformer", space).reshape(B * N, S, -1)
        dcoords, dfeats = delta[:, :, :2], delta[:, :, 2:]
        tf_ = tf_.reshape(B * N * S, latent_dim)
        dfeats = dfeats.reshape(B * N * S, latent_dim)
        g = F.group_norm(dfeats, 1, P[name + ".norm.weight"], P[name + ".norm.bias"])
        tf_ = F.gelu(linear(g, P, name + ".ffeat_updater.0")) + tf_
        track_feats = tf_.reshape(B, N, S, latent_dim).permute(0, 2, 1, 3)
        coords = coords + dcoords.reshape(B, N, S, 2).permute(0, 2, 1, 3)
        coords[:, 0] = coords_backup[:, 0]
        preds.append(coords * stride * down_ratio if down_ratio > 1 else coords * stride)
    vis = None
    if not fine:
        vis = torch.sigmoid(linear(track_feats.reshape(B * S * N, latent_dim), P, name + ".vis_predictor.0").reshape(B, S, N))
    return preds, vis, track_feats, query_feat


def compute_score(query_feat, patch_feat, fine_track, sradius, psize, B, N, S, Cout):
    """refine_track.py:174-278, including the reference's indexing quirk: the feature map is
    selected with batch_indices = arange(B) (flat (b, s, n) index b, i.e. patch (s=0, n=b) of
    sequence 0 at B>1 — per-sequence semantics: patch (s=0, n=0) of the sequence), while the
    window origins are read in (b n s) order from fine_track [B*N, S, 1, 2]."""
    qf = query_feat.reshape(B, N, Cout).unsqueeze(1).expand(-1, S - 1, -1, -1).reshape(B * (S - 1) * N, Cout)
    ssize = 2 * sradius + 1
    pf = patch_feat.reshape(B, N, S, Cout, psize, psize).permute(0, 2, 1, 3, 4, 5)  # b s n c p q
    tl = (fine_track.floor().int() - sradius).clamp(0, psize - ssize).squeeze(2)  # [B*N, S, 2]
    y_idx = tl[..., 0].flatten()
    x_idx = tl[..., 1].flatten()
    flat = pf.reshape(B * S * N, Cout, psize, psize)
    feats = []
    for m in range(B * S * N):
        f = flat[m // (S * N) * S * N] if B > 1 else flat[0]  # per-sequence: (b, s=0, n=0)
        xi, yi = int(x_idx[m]), int(y_idx[m])
        feats.append(f[:, xi:xi + ssize, yi:yi + ssize])
    ref = torch.stack(feats).reshape(B, S, N, Cout, ssize, ssize)[:, 1:].reshape(B * (S - 1) * N, Cout, ssize * ssize)
    sim = torch.einsum("mc,mcr->mr", qf, ref)
    heat = torch.softmax(sim * (1.0 / Cout ** 0.5), dim=1).reshape(-1, ssize, ssize)
    lin = torch.linspace(-1.0, 1.0, ssize)
    gy, gx = torch.meshgrid(lin, lin, indexing="ij")
    grid = torch.stack([gx, gy], dim=-1).reshape(1, -1, 2)  # kornia create_meshgrid (x, y)
    hv = heat.reshape(-1, ssize * ssize, 1)
    mean = torch.stack([(heat.reshape(-1, ssize * ssize) * grid[0, :, 0]).sum(-1),
                        (heat.reshape(-1, ssize * ssize) * grid[0, :, 1]).sum(-1)], dim=-1)
    var = torch.sum(grid ** 2 * hv, dim=1) - mean ** 2
    std = torch.sum(torch.sqrt(torch.clamp(var, min=1e-10)), -1)
    score = std.reshape(B, S - 1, N)
    return torch.cat([torch.ones_like(score[:, 0:1]), score], dim=1)


def refine_track(images, P, coarse, pradius=15, sradius=2, fine_iters=6):
    """refine_track.py:26-170 (+ compute_score_fn)."""
    B, S, N, _ = coarse.shape
    H, W = images.shape[-2:]
    psize = 2 * pradius + 1
    query_points = coarse[:, 0]
    track_int = coarse.floor().int()
    track_frac = coarse - track_int
    topleft = track_int - pradius
    topleft_bsn = topleft.clone()
    topleft = topleft.clamp(0, H - psize).reshape(B * S, N, 2)
    img = images.reshape(B * S, 3, H, W)
    ar = torch.arange(psize)
    ys = (topleft[..., 1].long()[..., None] + ar)  # [BS, N, p]
    xs = (topleft[..., 0].long()[..., None] + ar)
    bi = torch.arange(B * S)[:, None, None, None]
    patches = img.permute(0, 2, 3, 1)[bi, ys[..., :, None], xs[..., None, :]]  # [BS,N,p,q,3]
    patch_in = patches.permute(0, 1, 4, 2, 3).reshape(B * S * N, 3, psize, psize)
    feat = shallow_encoder(patch_in, P, "track_predictor.fine_fnet")
    Cout = feat.shape[1]
    feat = feat.reshape(B, S, N, Cout, psize, psize).permute(0, 2, 1, 3, 4, 5).reshape(B * N, S, Cout, psize, psize)
    pq = (track_frac[:, 0] + pradius).reshape(B * N, 2).unsqueeze(1)
    preds, _, _, qfeat = tracker_predictor(pq, feat, P, "track_predictor.fine_predictor", fine_iters, 1, 1,
                                           3, 3, 32, True, False)
    fine_last = preds[-1].clone()  # [B*N, S, 1, 2]
    lv = preds[-1].reshape(B, N, S, 1, 2).permute(0, 2, 1, 3, 4).squeeze(-2) + topleft_bsn
    refined = lv.clone()
    refined[:, 0] = query_points
    score = compute_score(qfeat, feat, fine_last, sradius, psize, B, N, S, Cout)
    return refined, score


def comet_forward(P, image, tracks, gt=None, track_iters=4, intri_type="AMD_eval", return_all=False):
    """E2Epose2.py:151-266 forward_all (fine_tracker=True, softmax_refine=False)."""
    B, T, C, H, W = image.shape
    res = {}
    with torch.no_grad():
        x = F.interpolate(image.reshape(B * T, C, H, W), scale_factor=1 / 2, mode="bilinear", align_corners=True)
        fmaps = basic_encoder(x, P, "track_predictor.coarse_fnet", 4)
        fmaps = fmaps.reshape(B, T, -1, fmaps.shape[-2], fmaps.shape[-1])
        preds, vis, _, _ = tracker_predictor(tracks[:, 0], fmaps, P, "track_predictor.coarse_predictor",
                                             track_iters, 4, 2, 5, 4, 128, False, True)
        coarse = preds[-1]
        refined, score = refine_track(image, P, coarse)
        inv = 1.0 / (score + 1e-6)
        inv = inv / inv.max(dim=1, keepdim=True)[0]
        res.update(fmaps=fmaps, coarse_preds=preds, vis=vis, coarse=coarse, refined=refined, score=score,
                   inv_score=inv)
    out = camera_predictor(image.reshape(-1, C, H, W), B, P, gt, refined, inv, intri_type)
    out["pred_tracks"] = refined
    if return_all:
        out.update(res)
    return out


# ----------------------------------------------------------------------------------------
# train step — train_eval_func_new_cp5.py:790-803, train_util.py:311-332
# ----------------------------------------------------------------------------------------


def train_step(P_train, P_all, image, tracks, gt, lr=1e-5, state=None, max_norm=1.0):
    """One fwd+bwd+clip+AdamW step on the camera_predictor params (names in P_train)."""
    params = {k: P_all[k].detach().clone().requires_grad_(True) for k in P_train}
    P = dict(P_all)
    P.update(params)
    out = comet_forward(P, image, tracks, gt)
    loss = out["loss"].mean()
    names = list(params)
    grads = torch.autograd.grad(loss, [params[k] for k in names], allow_unused=True)
    grads = [torch.zeros_like(params[k]) if g is None else g for k, g in zip(names, grads)]
    total = torch.norm(torch.stack([torch.norm(g, 2.0) for g in grads]), 2.0)
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    opt_params = [params[k].detach().clone() for k in names]
    opt = torch.optim.AdamW(opt_params, lr=lr)
    for p, g in zip(opt_params, grads):
        p.grad = g * coef
    opt.step()
    return loss.detach(), dict(zip(names, grads)), dict(zip(names, opt_params)), total


# ----------------------------------------------------------------------------------------
# evaluation metrics — metric.py; f32 like the reference
# ----------------------------------------------------------------------------------------


def _mat2quat(m):
    """minipytorch3d/rotation_conversions.py:104-172 (best-conditioned candidate, w >= 0)."""
    m00, m01, m02, m10, m11, m12, m20, m21, m22 = m.reshape(-1, 9).unbind(-1)
    a = torch.stack([1 + m00 + m11 + m22, 1 + m00 - m11 - m22, 1 - m00 + m11 - m22, 1 - m00 - m11 + m22], -1)
    a = torch.where(a > 0, a.clamp_min(0).sqrt(), torch.zeros_like(a))
    cand = torch.stack([
        torch.stack([a[:, 0] ** 2, m21 - m12, m02 - m20, m10 - m01], -1),
        torch.stack([m21 - m12, a[:, 1] ** 2, m10 + m01, m02 + m20], -1),
        torch.stack([m02 - m20, m10 + m01, a[:, 2] ** 2, m12 + m21], -1),
        torch.stack([m10 - m01, m20 + m02, m21 + m12, a[:, 3] ** 2], -1)], -2)
    cand = cand / (2.0 * a[..., None].clamp_min(0.1))
    q = cand[torch.arange(a.shape[0]), a.argmax(-1)]
    return torch.where(q[:, :1] < 0, -q, q)


def _quat2mat(q):
    r, i, j, k = q.unbind(-1)
    two_s = 2.0 / (q * q).sum(-1)
    return torch.stack([1 - two_s * (j * j + k * k), two_s * (i * j - k * r), two_s * (i * k + j * r),
                        two_s * (i * j + k * r), 1 - two_s * (i * i + k * k), two_s * (j * k - i * r),
                        two_s * (i * k - j * r), two_s * (j * k + i * r), 1 - two_s * (i * i + j * j)],
                       -1).reshape(q.shape[:-1] + (3, 3))


def translation_angle(tg, tp):
    """metric.py:675-701 (ambiguity folded), degrees."""
    tp = tp / (tp.norm(dim=1, keepdim=True) + 1e-15)
    tg = tg / (tg.norm(dim=1, keepdim=True) + 1e-15)
    loss = torch.clamp_min(1.0 - (tp * tg).sum(1) ** 2, 1e-15)
    err = torch.acos(torch.sqrt(1 - loss))
    err[torch.isnan(err) | torch.isinf(err)] = 1e6
    deg = err * 180.0 / math.pi
    return torch.min(deg, (180 - deg).abs())


def pose_pair_errors(pred_w2v, gt_w2v, B):
    """metric.py:214-245 (batched_all_pairs 561-570, closed_form_inverse 611-642, rotation_angle
    645-659) -> (rel_rangle_deg, rel_tangle_deg)."""
    S = gt_w2v.shape[0] // B
    i1_, i2_ = torch.combinations(torch.arange(S), 2).unbind(-1)
    i1 = (i1_[None] + torch.arange(B)[:, None] * S).reshape(-1)
    i2 = (i2_[None] + torch.arange(B)[:, None] * S).reshape(-1)

    def inv(se3):
        Rt = se3[:, :3, :3].transpose(1, 2)
        left = torch.cat((Rt, -se3[:, 3:, :3].bmm(Rt)), 1)
        return torch.cat((left, se3[:, :, 3:]), -1)
    rg = inv(gt_w2v[i1]).bmm(gt_w2v[i2])
    rp = inv(pred_w2v[i1]).bmm(pred_w2v[i2])
    qg, qp = _mat2quat(rg[:, :3, :3]), _mat2quat(rp[:, :3, :3])
    loss = (1 - (qp * qg).sum(1) ** 2).clamp(min=1e-15)
    return torch.arccos(1 - 2 * loss) * 180 / math.pi, translation_angle(rg[:, 3, :3], rp[:, 3, :3])


def pose_frame_errors(pred_enc, gt_enc):
    """metric.py:391-451 core -> (translation angle deg, geodesic rad, Euler [n, 3] rad float64)."""
    tr = translation_angle(gt_enc[:, :3], pred_enc[:, :3])
    m = torch.bmm(_quat2mat(pred_enc[:, 3:7]), _quat2mat(gt_enc[:, 3:7]).transpose(1, 2))
    cos = ((m[:, 0, 0] + m[:, 1, 1] + m[:, 2, 2] - 1) / 2).clamp(-1, 1)
    md = m.double()
    sy = torch.sqrt(md[:, 0, 0] ** 2 + md[:, 1, 0] ** 2)
    sing = sy < 1e-6
    z = torch.where(sing, torch.atan2(-md[:, 1, 2], md[:, 1, 1]), torch.atan2(md[:, 2, 1], md[:, 2, 2]))
    y = torch.atan2(-md[:, 2, 0], sy)
    x = torch.where(sing, torch.zeros_like(sy), torch.atan2(md[:, 1, 0], md[:, 0, 0]))
    return tr, torch.acos(cos), torch.stack([x, y, z], -1)
