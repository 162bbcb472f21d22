"""Keypoint initialisation of the training loop (train_eval_func_new_cp5.py:527-595).

The reference builds `lightglue.SuperPoint(max_num_keypoints=cfg.train.track_num,
detection_threshold=0.005)` and `lightglue.SIFT(max_num_keypoints=track_num)`, runs `.extract()` on
frame 0 of every sequence, concatenates both keypoint sets and keeps / pads them with
`filter_and_pad` against the sequence's first object mask (train_eval_func_new_cp5.py:249-314);
the result, broadcast over the T frames, is the `tracks` input of COMET.

Here:
  * SuperPoint: LightGlue's network (magicleap SuperPoint v1: VGG encoder conv1a..conv4b, detector
    convPa/convPb, descriptor convDa/convDb -- same parameter names, so `superpoint_v1.pth` loads)
    and its extract() pipeline (resize to `resize` on the long side, grayscale, simple_nms radius 4,
    4-px border removal, threshold, top-k, keypoints rescaled to the input). Every dense stage runs
    on libcomet_hip.so (comet_sp_preprocess, comet_conv2d_nhwc with fused ReLU,
    comet_maxpool2_nhwc, comet_sp_scores, comet_maxfilt2d); candidate selection / top-k are device
    torch ops. The descriptor head is not evaluated: COMET uses only the keypoints.
  * filter_and_pad: the reference's rules, on the device, with the same torch RNG calls
    (torch.randint / torch.randperm on the keypoints' device) -- so a run seeded like the reference
    on the same device draws the same padding points -- and the 3x3 dilation on comet_maxfilt2d.
  * SIFT: LightGlue's SIFT wraps OpenCV / pycolmap, neither of which exists here; `sift=None`
    uses the SuperPoint keypoints alone.
Parity: the NMS and filter_and_pad are pinned to fixtures generated from the reference tree
(glue-factory's batched_nms = LightGlue's simple_nms; the reference's filter_and_pad), and the
network + keypoint selection to the reference tree's copy of the same magicleap network
(gluefactory_nonfree/superpoint.py) run with PRNG weights (the trained superpoint_v1.pth is a
download that is not available here); SIFT stays unpinned (absent).
"""
import torch
import torch.nn as nn

from . import _lib as L
from . import functional as F
from . import ops


def _maxfilt(x, r):
    """(2r+1)^2 stride-1 max filter of [B, H, W] f32 (comet_maxfilt2d)."""
    x = x.contiguous().float()
    B, H, W = x.shape
    y = torch.empty_like(x)
    tmp = torch.empty_like(x)
    L.check(L.load().comet_maxfilt2d(x.data_ptr(), y.data_ptr(), tmp.data_ptr(), B, H, W, r, ops.stream()),
            "comet_maxfilt2d")
    return y


def simple_nms(scores, nms_radius):
    """LightGlue superpoint.simple_nms (= glue-factory batched_nms, superpoint_open.py:34-48):
    local maxima of a (2r+1)^2 window, two rounds of re-admitting maxima outside suppressed areas."""
    zeros = torch.zeros_like(scores)
    max_mask = scores == _maxfilt(scores, nms_radius)
    for _ in range(2):
        supp_mask = _maxfilt(max_mask.float(), nms_radius) > 0
        supp_scores = torch.where(supp_mask, zeros, scores)
        new_max_mask = supp_scores == _maxfilt(supp_scores, nms_radius)
        max_mask = max_mask | (new_max_mask & (~supp_mask))
    return torch.where(max_mask, scores, zeros)


def sp_scores(logits_nhwc):
    """Detector logits [B, h, w, 65] -> dense keypoint scores [B, 8h, 8w] (softmax, dustbin dropped,
    depth-to-space; comet_sp_scores)."""
    lg = logits_nhwc.contiguous().float()
    B, h, w, _ = lg.shape
    out = torch.empty(B, 8 * h, 8 * w, device=lg.device, dtype=torch.float32)
    L.check(L.load().comet_sp_scores(lg.data_ptr(), out.data_ptr(), B, h, w, ops.stream()), "comet_sp_scores")
    return out


class SuperPoint(nn.Module):
    """LightGlue's SuperPoint (superpoint_v1 architecture and parameter names) with extract()."""

    default_conf = {"descriptor_dim": 256, "nms_radius": 4, "max_num_keypoints": None,
                    "detection_threshold": 0.0005, "remove_borders": 4, "resize": 1024}

    def __init__(self, **conf):
        super().__init__()
        self.conf = {**self.default_conf, **conf}
        mk = self.conf["max_num_keypoints"]
        if mk is not None and mk <= 0:
            raise ValueError("max_num_keypoints must be positive or None")
        c1, c2, c3, c4, c5 = 64, 64, 128, 128, 256
        self.conv1a = nn.Conv2d(1, c1, 3, 1, 1)
        self.conv1b = nn.Conv2d(c1, c1, 3, 1, 1)
        self.conv2a = nn.Conv2d(c1, c2, 3, 1, 1)
        self.conv2b = nn.Conv2d(c2, c2, 3, 1, 1)
        self.conv3a = nn.Conv2d(c2, c3, 3, 1, 1)
        self.conv3b = nn.Conv2d(c3, c3, 3, 1, 1)
        self.conv4a = nn.Conv2d(c3, c4, 3, 1, 1)
        self.conv4b = nn.Conv2d(c4, c4, 3, 1, 1)
        self.convPa = nn.Conv2d(c4, c5, 3, 1, 1)
        self.convPb = nn.Conv2d(c5, 65, 1, 1, 0)
        self.convDa = nn.Conv2d(c4, c5, 3, 1, 1)
        self.convDb = nn.Conv2d(c5, self.conf["descriptor_dim"], 1, 1, 0)

    def _conv(self, x, conv, relu=True, out_dtype=None):
        k, pad = conv.kernel_size[0], conv.padding[0]
        if x.dtype == torch.bfloat16:  # implicit GEMM with the bias + ReLU epilogue
            w = F.wcast_conv(conv.weight, cin_pad=x.shape[-1])
            return ops.conv2d_nhwc(x, w, k, k, 1, pad, bias=conv.bias,
                                   act=L.ACT_RELU if relu else L.ACT_NONE, out_dtype=out_dtype or x.dtype)
        from .models.modules import conv2d_nhwc  # f32: im2col + GEMM
        y = conv2d_nhwc(x, conv, 1, pad, out_dtype=out_dtype or x.dtype)
        return torch.relu_(y) if relu else y

    def _pool(self, x):
        n, H, W, C = x.shape
        y = torch.empty(n, H // 2, W // 2, C, device=x.device, dtype=x.dtype)
        L.check(L.load().comet_maxpool2_nhwc(ops.dt(x), x.data_ptr(), y.data_ptr(), n, H, W, C, ops.stream()),
                "comet_maxpool2_nhwc")
        return y

    @torch.no_grad()
    def dense_probs(self, x):
        """Preprocessed NHWC image [B, H, W, 8] -> dense keypoint probabilities [B, H, W] (encoder,
        detector head, softmax with the dustbin dropped, depth-to-space; superpoint.py:202-233)."""
        for a, b in (("conv1a", "conv1b"), ("conv2a", "conv2b"), ("conv3a", "conv3b")):
            x = self._conv(self._conv(x, getattr(self, a)), getattr(self, b))
            x = self._pool(x)
        x = self._conv(self._conv(x, self.conv4a), self.conv4b)
        logits = self._conv(self._conv(x, self.convPa), self.convPb, relu=False, out_dtype=torch.float32)
        return sp_scores(logits)

    @torch.no_grad()
    def dense_scores(self, x):
        """Preprocessed NHWC image [B, H, W, 8] -> keypoint scores [B, H', W'] after the NMS and the
        border removal (LightGlue SuperPoint.forward up to the candidate selection)."""
        scores = simple_nms(self.dense_probs(x), self.conf["nms_radius"])
        pad = self.conf["remove_borders"]
        if pad:
            scores[:, :pad] = -1
            scores[:, :, :pad] = -1
            scores[:, -pad:] = -1
            scores[:, :, -pad:] = -1
        return scores

    def _preprocess(self, image, OH, OW):
        B, _, H, W = image.shape
        dt = F.compute_dtype()
        y = torch.empty(B, OH, OW, 8, device=image.device, dtype=dt)
        L.check(L.load().comet_sp_preprocess(ops.dt(y), image.contiguous().float().data_ptr(), y.data_ptr(), B, H, W,
                                             OH, OW, 8, ops.stream()), "comet_sp_preprocess")
        return y

    @torch.no_grad()
    def extract(self, img):
        """LightGlue Extractor.extract: img [3, H, W] or [1, 3, H, W] -> {"keypoints" [1, K, 2]
        (x, y in input pixels), "keypoint_scores" [1, K]}."""
        if img.dim() == 3:
            img = img[None]
        if img.dim() != 4 or img.shape[0] != 1:
            raise ValueError("extract takes one image")
        _, _, H, W = img.shape
        r = self.conf["resize"]
        if r is not None:  # resize so that the long side is `resize` (ImagePreprocessor side="long")
            s = r / max(H, W)
            OH, OW = int(round(H * s)), int(round(W * s))
        else:
            OH, OW = H, W
        scores = self.dense_scores(self._preprocess(img, OH, OW))
        idx = torch.nonzero(scores[0] > self.conf["detection_threshold"])  # (i, j), row-major
        sc = scores[0][idx[:, 0], idx[:, 1]]
        mk = self.conf["max_num_keypoints"]
        if mk is not None and mk < idx.shape[0]:
            sc, order = torch.topk(sc, mk, dim=0, sorted=True)
            idx = idx[order]
        kp = torch.flip(idx, [1]).float()
        scale = torch.tensor([OW / W, OH / H], device=kp.device, dtype=kp.dtype)
        kp = (kp + 0.5) / scale - 0.5
        return {"keypoints": kp[None], "keypoint_scores": sc[None]}


def sample_extra_points(mask, need_extra, device):
    """need_extra random pixels (x, y) of a bool mask (train_eval_func_new_cp5.py:249-259)."""
    ys, xs = torch.where(mask)
    if ys.numel() == 0:
        return None
    idx = torch.randint(0, ys.shape[0], (need_extra,), device=device)
    return torch.stack([xs[idx], ys[idx]], dim=1).float().to(device)


def filter_and_pad(pts, mask0, min_pts, max_pts, sel_first_name=None):
    """Keypoints inside the first object mask, padded to at least min_pts with random mask pixels,
    then pixels of the mask's 1-px dilation ring, then any pixel; at most max_pts (random subset)
    (train_eval_func_new_cp5.py:261-314, same RNG calls in the same order)."""
    H, W = mask0.shape
    device = pts.device
    xs = pts[:, 0].round().clamp(0, W - 1).long()
    ys = pts[:, 1].round().clamp(0, H - 1).long()
    region = mask0.to(device).bool()
    keep = pts[region[ys, xs]]
    if keep.shape[0] < min_pts:
        need = min_pts - keep.shape[0]
        extra = sample_extra_points(region, need, device)
        if extra is None or extra.shape[0] < need:
            ring = (_maxfilt(region.float()[None], 1)[0] > 0) & (~region)
            remain = need if extra is None else need - extra.shape[0]
            extra2 = sample_extra_points(ring, remain, device)
            if extra2 is not None:
                extra = extra2 if extra is None else torch.cat([extra, extra2], 0)
        if extra is None or extra.shape[0] < need:
            gy, gx = torch.meshgrid(torch.arange(H, device=device), torch.arange(W, device=device), indexing="ij")
            grid = torch.stack([gx.flatten(), gy.flatten()], dim=1).float()
            remain = need if extra is None else need - extra.shape[0]
            extra3 = grid[torch.randint(0, grid.shape[0], (remain,), device=device)]
            extra = extra3 if extra is None else torch.cat([extra, extra3], 0)
        keep = torch.cat([keep, extra], 0)
    if keep.shape[0] > max_pts:
        keep = keep[torch.randperm(keep.shape[0], device=device)[:max_pts]]
    return keep


@torch.no_grad()
def keypoint_tracks(sp, images, mask, track_num, sift=None, min_required=256, names=None):
    """train_eval_func_new_cp5.py:560-592: frame-0 keypoints of every sequence (SuperPoint, plus
    SIFT when given), filtered / padded against the first mask, broadcast over the T frames ->
    (tracks [B, T, N, 2], tracks_visibility [B, T, N] bool). images [B, T, 3, H, W]; mask [B, H, W]."""
    B, T = images.shape[:2]
    sel = []
    for i in range(B):
        pts = sp.extract(images[i, 0])["keypoints"][0]
        if sift is not None:
            pts = torch.cat([pts, sift.extract(images[i, 0])["keypoints"][0]], 0)
        sel.append(filter_and_pad(pts, mask[i].bool(), min_required, track_num, names))
    kp0 = torch.stack(sel, 0)  # the reference stacks too: equal counts per sequence required
    tracks = kp0.unsqueeze(1).expand(B, T, -1, -1)
    vis = torch.ones(B, T, kp0.shape[1], device=images.device, dtype=torch.bool)
    return tracks, vis
