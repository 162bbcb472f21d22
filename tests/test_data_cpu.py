"""SURVEY §8(f2) data path, CPU side: the LANCZOS coefficient tables of comet_resample_coeffs (a
host entry of libcomet_hip.so) driven through the same two integer passes as the HIP kernels
(numpy, test-only) equal Pillow's Image.crop + resize(LANCZOS) byte for byte, and the host part of
comet_amd.data.YTDataset reproduces the reference loader's fixtures
(tests/golden/comet_golden_data.npz from tools/gen_golden.py --data)."""
import ctypes
import os
import sys

import numpy as np
import pytest
import torch
from PIL import Image

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tests"))
import yt_fixture  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "comet_golden_data.npz")
MEAN = np.array([0.485, 0.456, 0.406], np.float32)
STD = np.array([0.229, 0.224, 0.225], np.float32)


def _tables(n_in, n_out):
    from comet_amd import _lib as L
    lib = L.load()
    ks = ctypes.c_int(0)
    L.check(lib.comet_resample_coeffs(n_in, 0.0, float(n_in), n_out, None, None, 0, ctypes.byref(ks)), "coeffs")
    b = np.zeros(2 * n_out, np.int32)
    k = np.zeros(n_out * ks.value, np.int32)
    L.check(lib.comet_resample_coeffs(n_in, 0.0, float(n_in), n_out, b.ctypes.data, k.ctypes.data, ks.value,
                                      ctypes.byref(ks)), "coeffs")
    return b.reshape(n_out, 2), k.reshape(n_out, ks.value)


def _clip8(s):
    """Resample.c clip8: 255 at or above 256 << 22, 0 at or below 0, else s >> 22."""
    return np.where(s >= (256 << 22), 255, np.where(s <= 0, 0, s >> 22)).astype(np.uint8)


def resample_like_kernels(crop, ow, oh):
    """The integer passes of comet_lanczos_crop_resize on a cropped uint8 [ch, cw, 3] image."""
    ch, cw = crop.shape[:2]
    img = crop.astype(np.int64)
    if oh != ch:
        by, ky = _tables(ch, oh)
        first, last = by[0, 0], by[-1, 0] + by[-1, 1]
    else:
        first, last = 0, ch
    if ow != cw:
        bx, kx = _tables(cw, ow)
        tmp = np.empty((last - first, ow, 3), np.uint8)
        for xx in range(ow):
            x0, n = bx[xx]
            s = (1 << 21) + np.einsum("rxc,x->rc", img[first:last, x0:x0 + n], kx[xx, :n].astype(np.int64))
            tmp[:, xx] = _clip8(s)
    else:
        tmp = crop[first:last].copy()
    if oh == ch:
        return tmp
    t = tmp.astype(np.int64)
    out = np.empty((oh, tmp.shape[1], 3), np.uint8)
    for yy in range(oh):
        y0, n = by[yy]
        s = (1 << 21) + np.einsum("yxc,y->xc", t[y0 - first:y0 - first + n], ky[yy, :n].astype(np.int64))
        out[yy] = _clip8(s)
    return out


def pil_crop(frame, box):
    x0, y0, x1, y1 = box
    h, w = frame.shape[:2]
    out = np.zeros((y1 - y0, x1 - x0, 3), np.uint8)
    sx0, sy0, sx1, sy1 = max(x0, 0), max(y0, 0), min(x1, w), min(y1, h)
    if sx1 > sx0 and sy1 > sy0:
        out[sy0 - y0:sy1 - y0, sx0 - x0:sx1 - x0] = frame[sy0:sy1, sx0:sx1]
    return out


@pytest.mark.parametrize("case", [((90, 70), (64, 64), (-12, 5)), ((40, 40), (128, 96), (3, -7)),
                                  ((64, 64), (64, 64), (0, 0)), ((300, 200), (256, 256), (20, -30)),
                                  ((57, 131), (57, 40), (-5, 9)), ((120, 33), (80, 33), (10, 2))])
def test_resample_tables_match_pillow(case):
    (cw, ch), (ow, oh), (x0, y0) = case
    rng = np.random.default_rng(cw * 1000 + ow)
    frame = rng.integers(0, 256, size=(150, 200, 3), dtype=np.uint8)
    box = (x0, y0, x0 + cw, y0 + ch)
    ref = np.asarray(Image.fromarray(frame).crop(box).resize((ow, oh), Image.Resampling.LANCZOS))
    np.testing.assert_array_equal(pil_crop(frame, box), np.asarray(Image.fromarray(frame).crop(box)))
    got = resample_like_kernels(pil_crop(frame, box), ow, oh)
    np.testing.assert_array_equal(got, ref)


@pytest.fixture(scope="module")
def dataset_root(tmp_path_factory):
    return yt_fixture.make_dataset(str(tmp_path_factory.mktemp("yt")))


@pytest.mark.parametrize("tag", ["a", "b", "c", "d"])
def test_ytdataset_host_part_matches_reference(tag, dataset_root):
    from comet_amd.data import YTDataset
    g = dict(np.load(GOLD, allow_pickle=False))
    pre = f"d{tag}_"
    seed, cw, chh, T = (int(v) for v in g[pre + "cfg"])
    ds = YTDataset(dataset_root, crop_size=(cw, chh), seq_len=T, device="cpu")
    np.random.seed(seed)
    frames, square, meta = ds.load_host(str(g[pre + "seq"]))
    assert meta["image_names"] == [str(n) for n in g[pre + "image_names"]]
    for k in ("T", "R", "T_uvz", "R_matrix"):
        np.testing.assert_array_equal(meta[k].numpy(), g[pre + k], err_msg=k)
    assert meta["ratio"] == float(g[pre + "ratio"][0])
    np.testing.assert_array_equal(meta["first_mask"].numpy(), g[pre + "first_mask"])
    # the pixels through the kernels' integer passes, then the reference's float32 normalisation
    imgs = np.stack([resample_like_kernels(pil_crop(f, square), cw, chh) for f in frames])
    video = torch.from_numpy(imgs).permute(0, 3, 1, 2).float() / 255.0
    video = (video - torch.from_numpy(MEAN)[None, :, None, None]) / torch.from_numpy(STD)[None, :, None, None]
    np.testing.assert_array_equal(video.numpy(), g[pre + "images"])


def test_ytdataset_behind_forked_dataloader_workers(dataset_root):
    """The reference loads with DataLoader(num_workers=8) (train_util.py:829-840): __getitem__ is
    host-only, so forked workers work; each worker's sample equals the in-process host stage.
    seq_len = the sequence length (12 frames) makes the frame choice RNG-free (start 0, stride 1)."""
    from torch.utils.data import DataLoader
    from comet_amd.data import YTDataset, collate_host
    ds = YTDataset(dataset_root, crop_size=(64, 48), seq_len=12, device="cpu")
    dl = DataLoader(ds, batch_size=2, num_workers=2, collate_fn=collate_host,
                    multiprocessing_context="fork")
    batches = list(dl)
    assert len(batches) == 1
    b = batches[0]
    assert len(b["frames"]) == 2 and "images" not in b
    for i, name in enumerate(ds.seq_names):
        frames, square, meta = ds.load_host(name)
        assert torch.equal(b["frames"][i], torch.from_numpy(np.stack(frames, 0)))
        assert b["crop_box"][i].tolist() == list(square)
        assert b["seq_name"][i] == name
        for k in ("T", "R", "T_uvz", "first_mask"):
            assert torch.equal(b[k][i], meta[k]), k
        assert float(b["ratio"][i]) == meta["ratio"]
