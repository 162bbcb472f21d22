"""CPU-side checks of the drop-in boundary: libcomet_hip.so loads (no GPU needed) and exports
every entry point declared in include/comet_hip.h; the ctypes signatures cover them all."""
import os
import re

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "comet_hip.h")).read()
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(comet_\w+)\(", src, re.M)))


def test_header_declares_core_entry_points():
    names = _declared()
    for n in ["comet_version", "comet_last_error", "comet_gemm", "comet_attention_fwd",
              "comet_layernorm_fwd", "comet_layernorm_bwd", "comet_adamw_multi"]:
        assert n in names


def test_library_exports_every_declared_symbol():
    from comet_amd import _lib
    lib = _lib.load()
    for n in _declared():
        assert hasattr(lib, n), f"missing export {n}"
    assert set(_declared()) == set(_lib.SIGNATURES), "ctypes SIGNATURES out of sync with header"
    assert lib.comet_version() >= 1


def test_error_path_reports_message():
    import ctypes
    from comet_amd import _lib
    lib = _lib.load()
    g = _lib.GemmArgs()
    g.layout_a = 7
    rc = lib.comet_gemm(ctypes.byref(g), None)
    assert rc == -1
    assert b"layout" in lib.comet_last_error() or b"batch" in lib.comet_last_error()


def test_library_has_no_packed_fp32_high_src1_reads():
    """The built library holds no packed-FP32 VOP3P instruction whose low result reads the high dword
    of its second / third source (op_sel:[x,1,..]): on gfx950 those return wrong values beside a
    co-resident MFMA wave (round 6, tools/isa_hazard.py; the Makefile builds with
    -fno-slp-vectorize). The probe kernel that reproduces the hazard on purpose is exempt."""
    import os
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_hazard
    bad = isa_hazard.check()
    assert not bad, {k[:80]: len(v) for k, v in bad.items()}


def test_round6_entry_points_reject_bad_arguments_before_launching():
    """The round-6 entry points check their arguments on the host and report them through
    comet_last_error without touching the GPU: the fused fine-encoder tail rejects channel counts
    its MFMA tile does not cover and an LDS footprint above 64 KiB, the fused resize + pool rejects
    channel counts whose column pairs would straddle a wave, and the token kernel a row pitch below
    the token width."""
    import ctypes
    from comet_amd import _lib
    lib = _lib.load()
    buf = ctypes.create_string_buffer(1 << 16)
    p = ctypes.addressof(buf) + (-ctypes.addressof(buf)) % 256  # 256-B aligned host address (never read)
    # c = 48: not 32 / 64
    rc = lib.comet_conv1x1_resize_pool_nhwc(p, None, 0, 0, None, 0, 0, p, None, p, p, None, 4, 48, 16, 16, 31, 31,
                                            None)
    assert rc != 0 and b"c in {32, 64}" in lib.comet_last_error()
    # 64 x 64 x 32 input: 256 KiB of LDS
    rc = lib.comet_conv1x1_resize_pool_nhwc(p, None, 0, 0, None, 0, 0, p, None, p, p, None, 4, 32, 64, 64, 31, 31,
                                            None)
    assert rc != 0 and b"64 KiB" in lib.comet_last_error()
    # c = 24: 2 x 3 lanes per column pair does not divide a wave
    rc = lib.comet_resize_bilinear_pool_nhwc(1, 1, p, p, p, 4, 24, 8, 8, 15, 15, None)
    assert rc != 0 and b"c in {8, 16, 32, 64, 128, 256}" in lib.comet_last_error()
    # row pitch below the token width
    rc = lib.comet_tracker_tokens(1, p, p, 32, p, 147, 147, p, 216, p, 200, 16, 4, None)
    assert rc != 0 and b"bad args" in lib.comet_last_error()
