"""ctypes binding of libmjgpu.so (C-ABI declared in include/mjgpu.h).

There is no fallback: if the HIP library is missing or cannot be loaded, every entry
point raises MjgError.  Build it with `python -m ffmpeg_distributed_amd.build`
(or `__graft_entry__.build()`).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MJG_LIBRARY", os.path.join(_PKG, "libmjgpu.so"))

MJG_OK = 0
MJG_E_INVALID = -1
MJG_E_HIP = -2
MJG_E_NOMEM = -3
MJG_E_CAPACITY = -4
MJG_E_STATE = -5

MJG_F_TIMING = 1
MJG_F_DEBUG_COEFS = 2
MJG_F_SWS_NO_BITEXACT = 4
MJG_F_COM_ITU601 = 8
MJG_F_HUFFMAN_OPTIMAL = 16
MJG_F_RST = 32
MJG_F_TIMING_DETAIL = 64
MJG_F_MERGE = 1024

# mjg_config.chroma_format
CHROMA_FORMATS = {"420": 0, "422": 1, "444": 2}

KERNEL_NAMES = ("scale", "encode", "scan_bits", "count_ff", "scan_ff", "write", "huff", "tail")
MJG_NUM_KERNELS = len(KERNEL_NAMES)

# Every symbol include/mjgpu.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "mjg_version", "mjg_last_error", "mjg_device_count", "mjg_device_numa_node", "mjg_open", "mjg_close",
    "mjg_frame_bytes", "mjg_header", "mjg_submit", "mjg_sync", "mjg_fetch", "mjg_fetch_host",
    "mjg_output_device", "mjg_stream", "mjg_queue_depth", "mjg_ctx_queue_depth", "mjg_submit_segments", "mjg_max_segments", "mjg_host_alloc", "mjg_host_free",
    "mjg_kernel_times", "mjg_build_header", "mjg_sws_filter", "mjg_debug_coefs",
    "mjg_debug_planes", "mjg_debug_filter", "mjg_debug_huff_build",
)


class MjgError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mjgpu error {code}: {msg}")
        self.code = code


class MjgConfig(C.Structure):
    _fields_ = [
        ("src_w", C.c_int32), ("src_h", C.c_int32),
        ("dst_w", C.c_int32), ("dst_h", C.c_int32),
        ("in_full_range", C.c_int32), ("qscale", C.c_int32),
        ("sar_num", C.c_int32), ("sar_den", C.c_int32),
        ("max_batch", C.c_int32), ("flags", C.c_uint32),
        ("chroma_format", C.c_int32),
    ]


_lib = None
_lock = threading.Lock()


def load():
    """Load libmjgpu.so (raises MjgError if it is absent: no CPU fallback exists)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise MjgError(MJG_E_STATE, f"{LIB_PATH} not built; run python -m ffmpeg_distributed_amd.build")
        L = C.CDLL(LIB_PATH)
        vp, u8p, sz = C.c_void_p, C.POINTER(C.c_uint8), C.c_size_t
        L.mjg_version.restype = C.c_int
        L.mjg_last_error.restype = C.c_char_p
        L.mjg_device_count.restype = C.c_int
        L.mjg_device_numa_node.argtypes = [C.c_int]
        L.mjg_device_numa_node.restype = C.c_int
        L.mjg_open.argtypes = [C.c_int, C.POINTER(MjgConfig), C.POINTER(vp)]
        L.mjg_close.argtypes = [vp]
        L.mjg_close.restype = None
        L.mjg_frame_bytes.argtypes = [vp]
        L.mjg_frame_bytes.restype = sz
        L.mjg_header.argtypes = [vp, u8p, sz, C.POINTER(sz)]
        L.mjg_submit.argtypes = [vp, vp, C.c_int, C.c_int]
        L.mjg_sync.argtypes = [vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]
        L.mjg_fetch.argtypes = [vp, vp, sz]
        L.mjg_fetch_host.argtypes = [vp, C.POINTER(vp), C.POINTER(sz)]
        L.mjg_output_device.argtypes = [vp, C.POINTER(vp), C.POINTER(vp)]
        L.mjg_stream.argtypes = [vp]
        L.mjg_stream.restype = vp
        if hasattr(L, "mjg_queue_depth"):  # absent from libraries built before r04 (A/B builds)
            L.mjg_queue_depth.argtypes = []
            L.mjg_queue_depth.restype = C.c_int
        if hasattr(L, "mjg_ctx_queue_depth"):  # absent from libraries built before r05 (A/B builds)
            L.mjg_ctx_queue_depth.argtypes = [vp]
            L.mjg_ctx_queue_depth.restype = C.c_int
        if hasattr(L, "mjg_submit_segments"):  # absent from libraries built before r04 (A/B builds)
            L.mjg_submit_segments.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_int), C.c_int]
            L.mjg_max_segments.argtypes = []
            L.mjg_max_segments.restype = C.c_int
        L.mjg_host_alloc.argtypes = [sz, C.POINTER(vp)]
        L.mjg_host_free.argtypes = [vp]
        L.mjg_kernel_times.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_int), C.c_int]
        L.mjg_debug_coefs.argtypes = [vp, C.c_int, C.POINTER(C.c_int16), sz]
        L.mjg_debug_planes.argtypes = [vp, C.c_int, u8p, sz]
        L.mjg_debug_filter.argtypes = [vp, C.c_int, C.c_int, C.POINTER(C.c_int16),
                                       C.POINTER(C.c_int32), C.POINTER(C.c_int), C.POINTER(C.c_int)]
        if hasattr(L, "mjg_debug_huff_build"):  # absent from libraries built before r05 (A/B builds)
            L.mjg_debug_huff_build.argtypes = [C.c_int, C.POINTER(C.c_uint32), C.c_int, u8p, C.POINTER(C.c_uint32)]
        L.mjg_build_header.argtypes = [C.POINTER(MjgConfig), u8p, sz, C.POINTER(sz)]
        L.mjg_sws_filter.argtypes = [C.c_int] * 7 + [C.POINTER(C.c_int16), sz, C.POINTER(C.c_int32),
                                                     C.POINTER(C.c_int)]
        # fail loudly on a stale / partial build (an A/B library from before r04/r05 named by
        # MJG_LIBRARY may lack mjg_queue_depth / mjg_ctx_queue_depth: the queue is then two
        # deep, no merging; and the multi-segment submit, which encoder.submit_segments guards)
        late = (("mjg_queue_depth", "mjg_ctx_queue_depth", "mjg_submit_segments", "mjg_max_segments",
                 "mjg_debug_huff_build")
                if os.environ.get("MJG_LIBRARY") else ())
        for name in EXPORTS:
            if name not in late:
                getattr(L, name)
        _lib = L
        return L


def check(rc: int) -> int:
    if rc < 0:
        msg = load().mjg_last_error().decode(errors="replace")
        raise MjgError(rc, msg)
    return rc


def device_count() -> int:
    return check(load().mjg_device_count())


def device_numa_node(device: int) -> int:
    """NUMA node of the device (-1: unknown)."""
    return check(load().mjg_device_numa_node(int(device)))


def build_header(dst_w: int, dst_h: int, qscale: int, sar=(1, 1), com_itu601: bool = False,
                 chroma: str = "420", rst: bool = False) -> bytes:
    """The per-config JPEG header, computed on the host (no GPU needed)."""
    L = load()
    flags = (MJG_F_COM_ITU601 if com_itu601 else 0) | (MJG_F_RST if rst else 0)
    cfg = MjgConfig(dst_w, dst_h, dst_w, dst_h, 1, qscale, sar[0], sar[1], 1, flags,
                    CHROMA_FORMATS[str(chroma)])
    n = C.c_size_t()
    check(L.mjg_build_header(C.byref(cfg), None, 0, C.byref(n)))
    buf = (C.c_uint8 * n.value)()
    check(L.mjg_build_header(C.byref(cfg), buf, n.value, C.byref(n)))
    return bytes(buf)


def sws_filter(src_len, dst_len, one, align, bitexact=True, src_pos=128, dst_pos=128):
    """swscale bicubic filter table as the library generates it (host side)."""
    import numpy as np
    L = load()
    taps = C.c_int()
    check(L.mjg_sws_filter(src_len, dst_len, one, align, int(bitexact), src_pos, dst_pos, None, 0,
                           None, C.byref(taps)))
    coeff = np.zeros(dst_len * taps.value, np.int16)
    pos = np.zeros(dst_len, np.int32)
    check(L.mjg_sws_filter(src_len, dst_len, one, align, int(bitexact), src_pos, dst_pos,
                           coeff.ctypes.data_as(C.POINTER(C.c_int16)), coeff.size,
                           pos.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(taps)))
    return coeff.reshape(dst_len, taps.value), pos
