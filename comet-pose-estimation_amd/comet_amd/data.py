"""Data path: mirror of comet/models/kubric_movif_SFM_dataset_YT.py's YTDataset.

On-disk format (kubric_movif_SFM_dataset_YT.py:113-140, 160-172):
    data_root/modelX/seq_Y/frames/frame_*      RGB frames
    data_root/modelX/seq_Y/GroundTruth/obj_w2c_*.txt   4x4 object-to-camera pose
    data_root/modelX/seq_Y/Mask/mask_*         object masks

load_images_from_folder does what the reference does per sequence -- frame selection
(sample_with_max_gap, same numpy RNG calls), mask bounding boxes, GT pose -> (quaternion, T, uvz),
the sequence's square crop box and `ratio` -- on the host (these are a few hundred scalars), and
moves the pixel work to the GPU: the decoded uint8 frames are uploaded once and
comet_lanczos_crop_resize (libcomet_hip.so) crops, LANCZOS-resizes (byte-exact with Pillow's
Resample.c) and ImageNet-normalises all T frames into the model's [T, 3, H, W] float32 input on
the device, instead of T PIL crops + resizes + a float normalisation on the CPU
(kubric_movif_SFM_dataset_YT.py:236-260). Decoding stays with PIL (the reference's decoder).

Two stages, so the dataset sits behind forked DataLoader workers as the reference's does
(num_workers 8, train_util.py:829-840): `__getitem__` is host-only (decode, masks, GT, crop box;
returns the uint8 `frames` [T, H, W, 3] and `crop_box` instead of `images`), `collate_host` batches
such samples, and the device stage (`to_device` / `DeviceLoader`, in the main process) uploads the
frames and produces `images` [B, T, 3, h, w]. `load_images_from_folder` is both stages in one call
(the reference's per-sequence function, for in-process use).
"""
import ctypes
import os

import numpy as np
import torch
from PIL import Image

from . import _lib as L
from . import ops

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
# AMD dataset intrinsics used for the uvz ground truth (kubric_movif_SFM_dataset_YT.py:205-208)
FX, FY, CX, CY = 268.44444444, 268.44444444, 320, 240


def make_bbox_square(old_bbox, size_to_fit):
    """kubric_movif_SFM_dataset_YT.py:37-57 (float32 box, centred padding, int truncation)."""
    new_bbox = np.array(old_bbox, dtype=np.float32)
    old_w = old_bbox[2] - old_bbox[0]
    old_h = old_bbox[3] - old_bbox[1]
    pad_h = (size_to_fit - old_h) / 2
    pad_w = (size_to_fit - old_w) / 2
    new_bbox[1] -= pad_h
    new_bbox[3] += pad_h
    new_bbox[0] -= pad_w
    new_bbox[2] += pad_w
    return new_bbox.astype(int)


def sample_with_max_gap(total_frames, seq_len):
    """kubric_movif_SFM_dataset_YT.py:67-91: evenly strided frames, stride <= 8, random start
    (the same numpy global-RNG calls, so a seeded run selects the same frames)."""
    if total_frames < seq_len:
        return np.linspace(0, total_frames - 1, seq_len, dtype=int).tolist()
    max_step = min(8, (total_frames - 1) // (seq_len - 1))
    max_step = max(max_step, 1)
    step = np.random.randint(1, max_step + 1)
    max_start = total_frames - (seq_len - 1) * step
    start = np.random.randint(0, max_start)
    return [start + i * step for i in range(seq_len)]


def mask_bbox(mask):
    """[xmin, ymin, xmax + 1, ymax + 1] of the nonzero pixels (cv2.boundingRect of cv2.findNonZero,
    kubric_movif_SFM_dataset_YT.py:182-188); the whole frame for an empty mask."""
    ys, xs = np.nonzero(mask)
    if xs.size == 0:
        h, w = mask.shape[:2]
        return [0, 0, w, h]
    return [int(xs.min()), int(ys.min()), int(xs.max()) + 1, int(ys.max()) + 1]


def pose_from_w2c(pose_matrix):
    """(R 3x3, T, quaternion (w, x, y, z), uvz) of a 4x4 GT pose (kubric_movif_SFM_dataset_YT.py:190-219)."""
    from scipy.spatial.transform import Rotation
    if pose_matrix.shape != (4, 4):
        raise ValueError("GT pose is not a 4x4 matrix")
    R_mat = pose_matrix[:3, :3]
    T_vec = pose_matrix[:3, 3]
    quat = Rotation.from_matrix(R_mat).as_quat(scalar_first=True)
    if abs(T_vec[2]) < 1e-6:
        raise ZeroDivisionError("Tz ~ 0")
    u = (FX * T_vec[0] + CX * T_vec[2]) / T_vec[2]
    v = (FY * T_vec[1] + CY * T_vec[2]) / T_vec[2]
    return R_mat, T_vec, quat, [u, v, T_vec[2]]


class ResamplePlan:
    """Pillow's LANCZOS coefficient tables for one (crop, output) size pair, on the device
    (comet_resample_coeffs computes them on the host exactly as Resample.c does)."""

    def __init__(self, cw, ch, ow, oh, device):
        lib = L.load()
        self.need_h, self.need_v = ow != cw, oh != ch
        self.bx = self.kx = self.by = self.ky = None
        self.ksx = self.ksy = 0
        if self.need_h:
            self.bx, self.kx, self.ksx = self._table(lib, cw, ow, device)
        self.ybase, self.rows = 0, ch
        if self.need_v:
            by, ky, self.ksy = self._table(lib, ch, oh, device, host=True)
            # Resample.c: the horizontal pass covers only the source rows the vertical pass reads
            first, last = int(by[0]), int(by[2 * oh - 2] + by[2 * oh - 1])
            self.ybase, self.rows = first, last - first
            by[0::2] -= first
            self.by, self.ky = torch.from_numpy(by).to(device), torch.from_numpy(ky).to(device)

    @staticmethod
    def _table(lib, n_in, n_out, device, host=False):
        ks = ctypes.c_int(0)
        L.check(lib.comet_resample_coeffs(n_in, 0.0, float(n_in), n_out, None, None, 0, ctypes.byref(ks)), "resample")
        bounds = np.zeros(2 * n_out, dtype=np.int32)
        coeffs = np.zeros(n_out * ks.value, dtype=np.int32)
        L.check(lib.comet_resample_coeffs(n_in, 0.0, float(n_in), n_out, bounds.ctypes.data, coeffs.ctypes.data,
                                          ks.value, ctypes.byref(ks)), "resample")
        if host:
            return bounds, coeffs, ks.value
        return torch.from_numpy(bounds).to(device), torch.from_numpy(coeffs).to(device), ks.value


_PLANS = {}


def crop_resize_normalize(frames, box, crop_size, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    """frames: uint8 [T, H, W, 3] on the device; box (x0, y0, x1, y1) ints (may leave the frame);
    crop_size (width, height) as PIL's resize takes it -> [T, 3, height, width] f32 on the device,
    equal to torch.from_numpy(np.stack([PIL crop + LANCZOS resize])).permute(0,3,1,2).float() / 255
    then (x - mean) / std (kubric_movif_SFM_dataset_YT.py:236-260)."""
    if not frames.is_cuda or frames.dtype != torch.uint8 or frames.dim() != 4 or frames.shape[-1] != 3:
        raise L.CometHipError("crop_resize_normalize: frames must be a uint8 [T, H, W, 3] device tensor")
    frames = frames.contiguous()
    T, H, W, _ = frames.shape
    x0, y0, x1, y1 = (int(v) for v in box)
    cw, ch = x1 - x0, y1 - y0
    ow, oh = int(crop_size[0]), int(crop_size[1])
    key = (cw, ch, ow, oh, frames.device)
    plan = _PLANS.get(key)
    if plan is None:
        plan = _PLANS[key] = ResamplePlan(cw, ch, ow, oh, frames.device)
    dev = frames.device
    stats = _PLANS.get(("stats", mean, std, dev))
    if stats is None:
        stats = _PLANS[("stats", mean, std, dev)] = (torch.tensor(mean, dtype=torch.float32, device=dev),
                                                      torch.tensor(std, dtype=torch.float32, device=dev))
    tmp = torch.empty(T, plan.rows, ow if plan.need_h else cw, 3, dtype=torch.uint8, device=dev)
    out = torch.empty(T, 3, oh, ow, dtype=torch.float32, device=dev)
    p = lambda t: None if t is None else t.data_ptr()  # noqa: E731
    L.check(L.load().comet_lanczos_crop_resize(
        frames.data_ptr(), T, H, W, H * W * 3, x0, y0, cw, ch, ow, oh, p(plan.bx), p(plan.kx), plan.ksx,
        p(plan.by), p(plan.ky), plan.ksy, plan.ybase, plan.rows, tmp.data_ptr(), stats[0].data_ptr(),
        stats[1].data_ptr(), out.data_ptr(), ops.stream()), "comet_lanczos_crop_resize")
    return out


class YTDataset(torch.utils.data.Dataset):
    """kubric_movif_SFM_dataset_YT.py:94-300 (same constructor and sample fields). Indexing is
    host-only (worker-safe); `images` is produced on `device` by load_images_from_folder or, for
    DataLoader batches, by to_device / DeviceLoader in the main process."""

    def __init__(self, data_root, crop_size=(256, 256), seq_len=24, use_augs=False, split="train", device="cuda"):
        super().__init__()
        self.seq_len = seq_len
        self.crop_size = crop_size
        self.split = split
        self.device = device
        if not os.path.exists(data_root):
            raise ValueError(f"Data root path does not exist: {data_root}")
        self.images_path = data_root
        if self.split == "valid":
            assert use_augs is False, "the validation split takes no augmentation"
        self.random_frame_rate = use_augs
        self.seq_names = self.process_dataset_txt(self.images_path)

    @staticmethod
    def process_dataset_txt(image_path):
        """modelX/seq_Y directories, numerically sorted (kubric_movif_SFM_dataset_YT.py:113-140)."""
        out = []
        models = sorted((d for d in os.listdir(image_path)
                         if os.path.isdir(os.path.join(image_path, d)) and d.startswith("model")),
                        key=lambda x: int(x[5:]))
        for m in models:
            mp = os.path.join(image_path, m)
            seqs = sorted((s for s in os.listdir(mp) if os.path.isdir(os.path.join(mp, s)) and s.startswith("seq_")),
                          key=lambda x: int(x[4:]))
            out.extend(os.path.join(m, s) for s in seqs)
        return out

    def load_images_from_folder(self, seq_name):
        frames, square, meta = self.load_host(seq_name)
        dev = torch.device(self.device)
        up = torch.from_numpy(np.stack(frames, 0))
        if dev.type == "cuda":
            up = up.pin_memory().to(dev, non_blocking=True)
        meta["images"] = crop_resize_normalize(up, square, self.crop_size)
        return meta

    def load_host(self, seq_name):
        """Everything of load_images_from_folder except the pixel work: (decoded uint8 frames,
        square crop box, sample dict without "images")."""
        seq_path = os.path.join(self.images_path, seq_name)
        images_path = os.path.join(seq_path, "frames")
        gts_path = os.path.join(seq_path, "GroundTruth")
        masks_path = os.path.join(seq_path, "Mask")
        image_names = sorted(f for f in os.listdir(images_path) if f.startswith("frame_"))
        gt_names = sorted(f for f in os.listdir(gts_path) if f.startswith("obj_w2c_"))
        mask_names = sorted(f for f in os.listdir(masks_path) if f.startswith("mask_"))
        if len(image_names) < self.seq_len:
            raise ValueError(f"Need {self.seq_len} frames, got {len(image_names)}")
        sel = sample_with_max_gap(len(image_names), self.seq_len)
        frames, boxes, positions, quats, uvzs, rmats, names, masks = [], [], [], [], [], [], [], []
        for ind in sel:
            img = Image.open(os.path.join(images_path, image_names[ind])).convert("RGB")
            frames.append(np.asarray(img))
            mask = np.array(Image.open(os.path.join(masks_path, mask_names[ind])).convert("L"), dtype=np.uint8)
            masks.append(mask)
            boxes.append(mask_bbox(mask))
            R_mat, T_vec, quat, uvz = pose_from_w2c(np.loadtxt(os.path.join(gts_path, gt_names[ind])))
            rmats.append(R_mat)
            uvzs.append(uvz)
            positions.append(T_vec.tolist())
            quats.append(quat.tolist())
            names.append(image_names[ind])
        xmins, ymins, xmaxs, ymaxs = zip(*boxes)
        bbox = np.array([min(xmins), min(ymins), max(xmaxs), max(ymaxs)], dtype=np.float64)
        bbox_size = np.max([bbox[2] - bbox[0], bbox[3] - bbox[1]])
        max_size_with_margin = bbox_size * 1.3
        margin = bbox_size * 0.15
        bbox = bbox + np.array([-margin, -margin, margin, margin])
        square = tuple(int(v) for v in make_bbox_square(bbox, max_size_with_margin))
        ratio = self.crop_size[0] / max_size_with_margin
        if len({f.shape for f in frames}) != 1:
            raise ValueError("frames of one sequence must share a size")
        # first mask: crop + NEAREST resize (one single-channel image, on the host as in the reference)
        m0 = Image.fromarray(masks[0]).crop(square).resize(tuple(self.crop_size), Image.Resampling.NEAREST)
        meta = {"T": torch.from_numpy(np.array(positions)).float(), "R": torch.from_numpy(np.array(quats)).float(),
                "seq_name": seq_name, "T_uvz": torch.from_numpy(np.array(uvzs)).float(), "ratio": ratio,
                "image_names": names, "first_mask": torch.from_numpy(np.array(m0, dtype=np.uint8) > 0),
                "R_matrix": torch.from_numpy(np.array(rmats)).float()}
        return frames, square, meta

    def __len__(self):
        return len(self.seq_names)

    def __getitem__(self, index):
        """Host stage only (no HIP call: safe in forked workers): the sample dict with `frames`
        (uint8 [T, H, W, 3]) and `crop_box` (int64 [4]) in place of `images`."""
        frames, square, meta = self.load_host(self.seq_names[index])
        meta["frames"] = torch.from_numpy(np.stack(frames, 0))
        meta["crop_box"] = torch.tensor(square, dtype=torch.int64)
        meta["crop_size"] = torch.tensor([int(self.crop_size[0]), int(self.crop_size[1])], dtype=torch.int64)
        return meta


def collate_host(samples):
    """DataLoader collate_fn for YTDataset samples (runs in the workers): `frames` stay a list
    (sequences may differ in frame size), every other field through default_collate."""
    from torch.utils.data import default_collate
    frames = [s["frames"] for s in samples]
    rest = default_collate([{k: v for k, v in s.items() if k != "frames"} for s in samples])
    rest["frames"] = frames
    return rest


def to_device(batch, device="cuda", keep_frames=False):
    """Device stage of a collate_host batch (main process): uploads each sequence's frames and
    crops / LANCZOS-resizes / normalises them -> batch["images"] [B, T, 3, h, w] f32 on `device`
    (the reference loader's collated `images`)."""
    dev = torch.device(device)
    imgs = []
    for b, fr in enumerate(batch["frames"]):
        up = fr.pin_memory().to(dev, non_blocking=True) if dev.type == "cuda" and not fr.is_cuda else fr.to(dev)
        box = [int(v) for v in batch["crop_box"][b]]
        size = [int(v) for v in batch["crop_size"][b]]
        imgs.append(crop_resize_normalize(up, box, size))
    out = dict(batch)
    out["images"] = torch.stack(imgs, 0)
    if not keep_frames:
        out.pop("frames")
    return out


class DeviceLoader:
    """Wraps a DataLoader of collate_host batches and applies to_device in the consuming process,
    so the workers never touch the GPU; len() and iteration as the wrapped loader's."""

    def __init__(self, loader, device="cuda"):
        self.loader, self.device = loader, device

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for batch in self.loader:
            yield to_device(batch, self.device)

    def __getattr__(self, k):
        return getattr(self.loader, k)
