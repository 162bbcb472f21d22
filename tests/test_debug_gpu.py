"""Debug mode: the `make DEBUG=1` library's device-side index checks and the NaN / Inf
check hooks (comet_amd/debug.py).

* In a fresh process with COMET_DEBUG=1 (libcomet_hip_debug.so): a patch gather inside the frame
  passes; one whose patch leaves a W < H frame (the reference clamps both axes with H,
  refine_track.py) fails its COMET_DASSERT and the op raises CometHipError naming it -- the
  reads stay inside the allocation (the frames are a slice of a larger buffer).
* FiniteCheck names the first submodule whose output holds a NaN; check_grads the first
  parameter whose gradient does."""
import os
import subprocess
import sys

import pytest
import torch

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

SCRIPT = r"""
import sys
sys.path.insert(0, {pkg!r})
import torch
from comet_amd import _lib as L, debug, ops
assert L.LIB_PATH.endswith("libcomet_hip_debug.so"), L.LIB_PATH
assert debug.debug_library() and debug.debug_flags() == 0
big = torch.rand(2, 2, 3, 40, 32, device="cuda")   # H = 40 > W = 32
imgs = big[:1]                                       # B = 1, S = 2; reads past it stay in `big`
coarse = torch.full((1, 2, 4, 2), 16.0, device="cuda")
ops.patch_gather(imgs, coarse, 15, torch.float32)  # x0 = 1, 1 + 31 <= 32: inside
torch.cuda.synchronize()
coarse[..., 0] = 30.0                                # x0 = min(15, H - 31 = 9) = 9: 9 + 31 > W
try:
    ops.patch_gather(imgs, coarse, 15, torch.float32)
except L.CometHipError as e:
    assert "index check failed" in str(e), str(e)
    assert debug.debug_flags() != 0
    print("DEBUG-OK", e)
else:
    raise SystemExit("the out-of-frame patch was not reported")
"""


def test_debug_library_reports_failed_index_check():
    lib = os.path.join(PKG, "libcomet_hip_debug.so")
    if not os.path.isfile(lib):
        pytest.fail("libcomet_hip_debug.so missing: build it with `make -C comet-pose-estimation_amd DEBUG=1`")
    env = dict(os.environ, COMET_DEBUG="1")
    env.pop("COMET_HIP_LIB", None)
    r = subprocess.run([sys.executable, "-c", SCRIPT.format(pkg=PKG)], capture_output=True, text=True, env=env,
                       timeout=240, cwd=ROOT)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0 and "DEBUG-OK" in r.stdout


def test_finite_check_names_the_module_and_the_gradient():
    from comet_amd import debug
    from comet_amd import functional as F
    from comet_amd._lib import CometHipError
    from comet_amd.models.modules import AttnBlock
    torch.manual_seed(0)
    blk = AttnBlock(128, 4).cuda()
    x = torch.randn(2, 20, 128, device="cuda")
    with F.precision(torch.float32), debug.FiniteCheck(blk):
        blk(x).sum().backward()  # finite: no error
    debug.check_grads(blk)
    assert not debug.debug_library() or debug.debug_flags() == 0
    x[1, 3, 5] = float("nan")
    with pytest.raises(CometHipError, match="non-finite values .* output of"):
        with F.precision(torch.float32), debug.FiniteCheck(blk):
            blk(x)
    blk.zero_grad()
    with F.precision(torch.float32):
        blk(x).sum().backward()
    with pytest.raises(CometHipError, match="gradient of"):
        debug.check_grads(blk)
    y = torch.tensor([1.0, float("inf"), float("nan"), 2.0], device="cuda")
    assert debug.count_nonfinite(y) == 2 and debug.count_nonfinite(y.to(torch.bfloat16)) == 2
