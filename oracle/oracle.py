"""ctypes front-end of oracle/liboracle.so (TEST INFRASTRUCTURE ONLY; see __init__.py)."""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build(force: bool = False) -> str:
    """Compile the C restatement with the committed Makefile (gcc only)."""
    src = os.path.join(_HERE, "mjpeg_oracle.c")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE, "-B" if force else "liboracle.so"],
                       check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        u8p = C.POINTER(C.c_uint8)
        L.or_fdct_islow.argtypes = [C.POINTER(C.c_int16)]
        L.or_effective_qscale.argtypes = [C.c_double]
        L.or_effective_qscale.restype = C.c_int
        L.or_build_matrix.argtypes = [C.c_int, u8p, C.POINTER(C.c_int32)]
        L.or_quantize.argtypes = [C.POINTER(C.c_int16), C.POINTER(C.c_int32)]
        L.or_quantize.restype = C.c_int
        L.or_huff_table.argtypes = [C.c_int, u8p, C.POINTER(C.c_uint16)]
        L.or_header.argtypes = [C.c_int] * 7 + [u8p, C.c_size_t]
        L.or_header.restype = C.c_size_t
        L.or_frame_coeffs.argtypes = [u8p, C.c_int, u8p, C.c_int, u8p, C.c_int, C.c_int, C.c_int,
                                      C.c_int, C.POINTER(C.c_int16), C.POINTER(C.c_int8)]
        L.or_encode_planes.argtypes = [u8p, C.c_int, u8p, C.c_int, u8p, C.c_int] + [C.c_int] * 6 + \
            [u8p, C.c_size_t]
        L.or_encode_planes.restype = C.c_size_t
        L.or_sws_init_filter.argtypes = [C.c_int] * 7 + [C.POINTER(C.c_int16), C.POINTER(C.c_int32),
                                                         C.POINTER(C.c_int), C.c_int]
        L.or_sws_init_filter.restype = C.c_int
        L.or_scale_plane.argtypes = [u8p, C.c_int, C.c_int, C.c_int, u8p] + [C.c_int] * 9
        L.or_scale_plane.restype = C.c_int
        L.or_local_pos.argtypes = [C.c_int, C.c_int]
        L.or_local_pos.restype = C.c_int
        L.or_encode_frame.argtypes = [u8p, C.c_int, u8p, C.c_int, u8p, C.c_int] + [C.c_int] * 9 + \
            [u8p, C.c_size_t]
        L.or_encode_frame.restype = C.c_size_t
        L.or_encode_frame_ex.argtypes = [u8p, C.c_int, u8p, C.c_int, u8p, C.c_int] + [C.c_int] * 10 + \
            [u8p, C.c_size_t]
        L.or_encode_frame_ex.restype = C.c_size_t
        L.or_header_cfmt.argtypes = [C.c_int] * 8 + [u8p, C.c_size_t]
        L.or_header_cfmt.restype = C.c_size_t
        L.or_frame_coeffs_cfmt.argtypes = [u8p, C.c_int, u8p, C.c_int, u8p, C.c_int] + [C.c_int] * 4 + \
            [C.POINTER(C.c_int16), C.POINTER(C.c_int8)]
        L.or_mcu_grid.argtypes = [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.or_mcu_grid.restype = None
        L.or_encode_frame_cfmt.argtypes = [u8p, C.c_int, u8p, C.c_int, u8p, C.c_int] + [C.c_int] * 12 + \
            [u8p, C.c_size_t]
        L.or_encode_frame_cfmt.restype = C.c_size_t
        L.or_huff_optimal.argtypes = [C.POINTER(C.c_uint32), u8p, u8p]
        L.or_huff_optimal.restype = C.c_int
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def fdct(block) -> np.ndarray:
    b = np.ascontiguousarray(np.asarray(block, dtype=np.int16).reshape(64)).copy()
    lib().or_fdct_islow(_p(b, C.c_int16))
    return b


def effective_qscale(q: float) -> int:
    return int(lib().or_effective_qscale(float(q)))


def matrix(qscale: int):
    m = np.zeros(64, np.uint8)
    qm = np.zeros(64, np.int32)
    lib().or_build_matrix(int(qscale), _p(m, C.c_uint8), _p(qm, C.c_int32))
    return m, qm


def quantize(coefs, qscale: int):
    b = np.ascontiguousarray(np.asarray(coefs, dtype=np.int16).reshape(64)).copy()
    _, qm = matrix(qscale)
    last = lib().or_quantize(_p(b, C.c_int16), _p(qm, C.c_int32))
    return b, int(last)


def huff_table(table_id: int):
    size = np.zeros(256, np.uint8)
    code = np.zeros(256, np.uint16)
    if lib().or_huff_table(int(table_id), _p(size, C.c_uint8), _p(code, C.c_uint16)):
        raise ValueError(table_id)
    return size, code


CHROMA_FORMATS = {"420": 0, "422": 1, "444": 2}


def _cfmt(chroma) -> int:
    return CHROMA_FORMATS[str(chroma)] if not isinstance(chroma, int) else int(chroma)


def header(width, height, qscale, sar=(1, 1), com_itu601=False, dri=0, chroma="420",
           rst=False) -> bytes:
    """Per-config header.  dri: an explicit DRI interval (4:2:0 only); rst: the DRI slice
    threading writes for `chroma` (MCUs per MCU row)."""
    buf = np.zeros(4096, np.uint8)
    if dri:
        n = lib().or_header(int(width), int(height), int(qscale), int(sar[0]), int(sar[1]),
                            int(bool(com_itu601)), int(dri), _p(buf, C.c_uint8), buf.size)
    else:
        n = lib().or_header_cfmt(int(width), int(height), _cfmt(chroma), int(qscale), int(sar[0]),
                                 int(sar[1]), int(bool(com_itu601)), int(bool(rst)),
                                 _p(buf, C.c_uint8), buf.size)
    if n == 0:
        raise RuntimeError("or_header failed")
    return buf[:n].tobytes()


def mcu_grid(width, height, chroma="420"):
    """(MCUs per row, MCU rows) of a frame."""
    a, b = C.c_int(), C.c_int()
    lib().or_mcu_grid(_cfmt(chroma), int(width), int(height), C.byref(a), C.byref(b))
    return a.value, b.value


def blocks_per_mcu(chroma="420") -> int:
    return (6, 8, 6)[_cfmt(chroma)]


def _planes(y, u, v):
    y = np.ascontiguousarray(y, dtype=np.uint8)
    u = np.ascontiguousarray(u, dtype=np.uint8)
    v = np.ascontiguousarray(v, dtype=np.uint8)
    return y, u, v


def frame_coeffs(y, u, v, qscale, chroma="420"):
    """Quantized coefficients (natural order) of every block in coding order + last index."""
    y, u, v = _planes(y, u, v)
    h, w = y.shape
    mcw, mch = mcu_grid(w, h, chroma)
    nblk = mcw * mch * blocks_per_mcu(chroma)
    coef = np.zeros((nblk, 64), np.int16)
    last = np.zeros(nblk, np.int8)
    lib().or_frame_coeffs_cfmt(_p(y, C.c_uint8), y.strides[0], _p(u, C.c_uint8), u.strides[0],
                               _p(v, C.c_uint8), v.strides[0], w, h, _cfmt(chroma), int(qscale),
                               _p(coef, C.c_int16), _p(last, C.c_int8))
    return coef, last


def _cap(w, h):
    return 4096 + ((w + 15) // 16) * ((h + 15) // 16) * 12 * 420 + 64


def encode_planes(y, u, v, qscale, sar=(1, 1), com_itu601=False) -> bytes:
    """JPEG bytes of one already-full-range 4:2:0 frame (no swscale)."""
    y, u, v = _planes(y, u, v)
    h, w = y.shape
    out = np.zeros(_cap(w, h), np.uint8)
    n = lib().or_encode_planes(_p(y, C.c_uint8), y.strides[0], _p(u, C.c_uint8), u.strides[0],
                               _p(v, C.c_uint8), v.strides[0], w, h, int(qscale), int(sar[0]),
                               int(sar[1]), int(bool(com_itu601)), _p(out, C.c_uint8), out.size)
    if n == 0:
        raise RuntimeError("or_encode_planes failed")
    return out[:n].tobytes()


def sws_filter(src_w, dst_w, one, align, bitexact=True, src_pos=128, dst_pos=128):
    f = np.zeros(dst_w * 256, np.int16)
    pos = np.zeros(dst_w, np.int32)
    size = C.c_int(0)
    rc = lib().or_sws_init_filter(int(src_w), int(dst_w), int(one), int(align), int(bool(bitexact)),
                                  int(src_pos), int(dst_pos), _p(f, C.c_int16), _p(pos, C.c_int32),
                                  C.byref(size), 256)
    if rc:
        raise RuntimeError("or_sws_init_filter failed")
    return f[:dst_w * size.value].reshape(dst_w, size.value).copy(), pos


def local_pos(sub, pos=-513):
    return int(lib().or_local_pos(int(sub), int(pos)))


def scale_plane(src, dst_w, dst_h, range_mode=0, bitexact=True, chroma=False):
    src = np.ascontiguousarray(src, dtype=np.uint8)
    sh, sw = src.shape
    dst = np.zeros((dst_h, dst_w), np.uint8)
    p = local_pos(1, -513) if chroma else local_pos(0, 0)
    rc = lib().or_scale_plane(_p(src, C.c_uint8), src.strides[0], sw, sh, _p(dst, C.c_uint8),
                              dst.strides[0], dst_w, dst_h, int(range_mode), int(bool(bitexact)),
                              p, p, p, p)
    if rc:
        raise RuntimeError("or_scale_plane failed")
    return dst


def encode_frame(y, u, v, dst_w=None, dst_h=None, full_range=False, qscale=5, sar=(1, 1),
                 bitexact_sws=True, huffman="default", chroma="420", rst=False) -> bytes:
    """Whole worker path for one frame: [bicubic resize] + tv->pc + mjpeg encode with
    -huffman default (Annex K tables) or optimal (per-frame tables, mjpegenc_huffman.c),
    chroma format 420/422/444, and rst=True for the slice-threaded layout (DRI, one
    restart interval per MCU row)."""
    if huffman not in ("default", "optimal"):
        raise ValueError(huffman)
    y, u, v = _planes(y, u, v)
    sh, sw = y.shape
    dw = sw if dst_w is None else dst_w
    dh = sh if dst_h is None else dst_h
    out = np.zeros(_cap(dw, dh), np.uint8)
    n = lib().or_encode_frame_cfmt(_p(y, C.c_uint8), y.strides[0], _p(u, C.c_uint8), u.strides[0],
                                   _p(v, C.c_uint8), v.strides[0], sw, sh, dw, dh, _cfmt(chroma),
                                   int(bool(full_range)), int(qscale), int(sar[0]), int(sar[1]),
                                   int(bool(bitexact_sws)), int(huffman == "optimal"), int(bool(rst)),
                                   _p(out, C.c_uint8), out.size)
    if n == 0:
        raise RuntimeError("or_encode_frame_cfmt failed")
    return out[:n].tobytes()


def huff_optimal(counts):
    """BITS[1..16] and HUFFVAL of -huffman optimal for one table's 256 symbol counts
    (ff_mjpeg_encode_huffman_close)."""
    c = np.ascontiguousarray(np.asarray(counts, dtype=np.uint32).reshape(256))
    bits = np.zeros(17, np.uint8)
    vals = np.zeros(256, np.uint8)
    n = lib().or_huff_optimal(_p(c, C.c_uint32), _p(bits, C.c_uint8), _p(vals, C.c_uint8))
    return bits, vals[:n].copy()
