"""SURVEY §8(f2) data path on the GPU: comet_lanczos_crop_resize equals Pillow's crop +
resize(LANCZOS) + the reference's float32 ImageNet normalisation bit for bit (frames at the
dataset's 640 x 480, crops leaving the frame, up- and down-sampling), and YTDataset on the device
reproduces the reference loader's fixtures (tests/golden/comet_golden_data.npz)."""
import os
import sys

import numpy as np
import pytest
import torch
from PIL import Image

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tests"))
import yt_fixture  # noqa: E402

pytestmark = pytest.mark.gpu
GOLD = os.path.join(ROOT, "tests", "golden", "comet_golden_data.npz")
MEAN = torch.tensor([0.485, 0.456, 0.406])[None, :, None, None]
STD = torch.tensor([0.229, 0.224, 0.225])[None, :, None, None]


def pil_reference(frames, box, size):
    rgbs = [np.asarray(Image.fromarray(f).crop(box).resize(size, Image.Resampling.LANCZOS)) for f in frames]
    video = torch.from_numpy(np.stack(rgbs, 0)).permute(0, 3, 1, 2).float() / 255.0
    return (video - MEAN) / STD


@pytest.mark.parametrize("box,size", [((100, 40, 460, 400), (512, 512)), ((-60, -20, 500, 540), (512, 512)),
                                      ((200, 150, 328, 278), (512, 512)), ((300, 100, 812, 612), (512, 512)),
                                      ((10, 10, 250, 130), (96, 64)), ((0, 0, 640, 480), (640, 480))])
def test_crop_resize_normalize_matches_pillow(box, size):
    from comet_amd.data import crop_resize_normalize
    rng = np.random.default_rng(box[0] + 7 * size[0])
    frames = rng.integers(0, 256, size=(16, 480, 640, 3), dtype=np.uint8)
    frames[:, ::5] //= 2
    got = crop_resize_normalize(torch.from_numpy(frames).cuda(), box, size)
    torch.cuda.synchronize()
    ref = pil_reference(frames, box, size)
    assert torch.equal(got.cpu(), ref), f"max diff {(got.cpu() - ref).abs().max().item()}"


@pytest.fixture(scope="module")
def dataset_root(tmp_path_factory):
    return yt_fixture.make_dataset(str(tmp_path_factory.mktemp("yt")))


@pytest.mark.parametrize("tag", ["a", "b", "c", "d"])
def test_ytdataset_on_device_matches_reference(tag, dataset_root):
    from comet_amd.data import YTDataset
    g = dict(np.load(GOLD, allow_pickle=False))
    pre = f"d{tag}_"
    seed, cw, chh, T = (int(v) for v in g[pre + "cfg"])
    ds = YTDataset(dataset_root, crop_size=(cw, chh), seq_len=T)
    np.random.seed(seed)
    smp = ds.load_images_from_folder(str(g[pre + "seq"]))
    assert smp["images"].is_cuda
    np.testing.assert_array_equal(smp["images"].cpu().numpy(), g[pre + "images"])
    for k in ("T", "R", "T_uvz"):
        np.testing.assert_array_equal(smp[k].numpy(), g[pre + k], err_msg=k)
    assert smp["ratio"] == float(g[pre + "ratio"][0])


def test_device_loader_after_cuda_init_with_forked_workers(dataset_root):
    """with HIP already initialised in the parent, forked DataLoader workers must not
    touch the GPU. The host stage runs in the workers, DeviceLoader's device stage in this process;
    the images equal the in-process load_images_from_folder bit for bit."""
    from torch.utils.data import DataLoader
    from comet_amd.data import DeviceLoader, YTDataset, collate_host
    torch.zeros(1, device="cuda")  # HIP initialised before the workers fork
    ds = YTDataset(dataset_root, crop_size=(64, 48), seq_len=12)
    dl = DeviceLoader(DataLoader(ds, batch_size=2, num_workers=2, collate_fn=collate_host,
                                 multiprocessing_context="fork"), "cuda")
    assert len(dl) == 1
    (b,) = list(dl)
    assert b["images"].is_cuda and tuple(b["images"].shape) == (2, 12, 3, 48, 64)
    for i, name in enumerate(ds.seq_names):
        ref = ds.load_images_from_folder(name)
        assert torch.equal(b["images"][i], ref["images"])
