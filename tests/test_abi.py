"""The C-ABI library (include/mjgpu.h) on a machine without a GPU: it loads, exports every
declared entry point, its device-free calls work, and GPU calls fail loudly with an
error code instead of falling back to anything."""
import ctypes as C
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from ffmpeg_distributed_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = open(os.path.join(ROOT, "include", "mjgpu.h")).read()


def declared():
    body = re.sub(r"/\*.*?\*/", "", HEADER, flags=re.S)
    return sorted(set(re.findall(r"\b(mjg_[a-z_]+)\s*\(", body)))


def test_header_declarations_match_binding_list():
    assert declared() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    so = _lib.LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", so], capture_output=True, text=True, check=True).stdout
    syms = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = [s for s in declared() if s not in syms]
    assert not missing
    L = _lib.load()
    for s in declared():
        assert getattr(L, s) is not None


def test_header_constants_match_python():
    for name in ("MJG_OK", "MJG_E_INVALID", "MJG_E_HIP", "MJG_E_NOMEM", "MJG_E_CAPACITY", "MJG_E_STATE",
                 "MJG_F_TIMING", "MJG_F_DEBUG_COEFS", "MJG_F_SWS_NO_BITEXACT", "MJG_F_COM_ITU601"):
        m = re.search(r"#define\s+" + name + r"\s+\(?(-?\d+)u?\)?", HEADER)
        assert m, name
        assert int(m.group(1)) == getattr(_lib, name), name
    m = re.search(r"#define\s+MJG_NUM_KERNELS\s+(\d+)", HEADER)
    assert m and int(m.group(1)) == _lib.MJG_NUM_KERNELS


def test_version_and_error_string():
    L = _lib.load()
    assert L.mjg_version() > 0
    assert isinstance(L.mjg_last_error(), bytes)


def test_build_header_size_query_and_capacity_error():
    L = _lib.load()
    cfg = _lib.MjgConfig(1920, 1080, 1920, 1080, 1, 5, 1, 1, 1, 0)
    n = C.c_size_t()
    assert L.mjg_build_header(C.byref(cfg), None, 0, C.byref(n)) == 0 and n.value > 500
    small = (C.c_uint8 * 10)()
    assert L.mjg_build_header(C.byref(cfg), small, 10, C.byref(n)) == _lib.MJG_E_CAPACITY


@pytest.mark.parametrize("bad", [dict(qscale=0), dict(qscale=32), dict(dst_w=0), dict(sar_num=70000)])
def test_build_header_rejects_bad_config(bad):
    L = _lib.load()
    kw = dict(src_w=64, src_h=48, dst_w=64, dst_h=48, in_full_range=1, qscale=5, sar_num=1, sar_den=1,
              max_batch=1, flags=0)
    kw.update(bad)
    cfg = _lib.MjgConfig(**kw)
    n = C.c_size_t()
    assert L.mjg_build_header(C.byref(cfg), None, 0, C.byref(n)) == _lib.MJG_E_INVALID
    assert L.mjg_last_error()


def test_sws_filter_is_device_free():
    coeff, pos = _lib.sws_filter(3840, 1920, 1 << 14, 4)
    assert coeff.shape[0] == 1920 and (coeff.sum(axis=1) == 1 << 14).all()
    assert (np.diff(pos) >= 0).all()


def test_open_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    from ffmpeg_distributed_amd.encoder import MjpegEncoder
    with pytest.raises(_lib.MjgError):
        MjpegEncoder(0, 64, 48)


def test_product_kernels_carry_no_experiment_switches():
    """The shipped kernel sources hold no preprocessor branches (experiments live as source
    patches in tools/patches.py, applied to a copy for tools/variants.py A/Bs)."""
    import glob
    import re
    csrc = os.path.join(ROOT, "ffmpeg_distributed_amd", "csrc")
    bad = []
    for p in sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h"))
                    + glob.glob(os.path.join(csrc, "*.cpp"))):
        for i, line in enumerate(open(p), 1):
            if re.match(r"\s*#\s*(if|ifdef|ifndef|elif)\b", line):
                bad.append(f"{os.path.basename(p)}:{i}: {line.strip()}")
    assert not bad, bad


@pytest.mark.skipif(os.environ.get("MJG_TOOLS_TESTS") != "1",
                    reason="research tooling, not the product: MJG_TOOLS_TESTS=1 checks the experiment anchors")
def test_experiment_patches_still_apply():
    """Every tools/patches.py experiment anchors exactly once in the product source (a check of
    the A/B tooling, run with MJG_TOOLS_TESTS=1; product edits may retire experiments)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import patches
    res = patches.check_all()
    assert all(res.values()), [k for k, v in res.items() if not v]
