"""GPU MJPEG encoder: the per-segment encode that the reference's worker runs
(`ffmpeg -f matroska -i pipe: <remote_args> -f matroska pipe:`,
ffmpeg_distributed.py:131-141), restricted to the profile
`[-vf scale=W:H:flags=bicubic] -c:v mjpeg -q:v N -dct int [-huffman default|optimal] -bitexact`
(+ `-slices N` / `-thread_type slice` for the RST layout).

Host-side wrapper over libmjgpu.so; frames are packed planar YUV (yuv420p / yuvj420p by
default, 4:2:2 and 4:4:4 with `chroma=`), i.e. what `ffmpeg -f rawvideo -pix_fmt yuv4xxp`
writes.  No CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from collections import deque
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from ._lib import MjgConfig, MjgError, check


CHROMA_SHIFTS = {"420": (1, 1), "422": (1, 0), "444": (0, 0)}


def chroma_size(w: int, h: int, chroma: str = "420"):
    """(width, height) of a chroma plane: ((w + hs) >> hs, (h + vs) >> vs)."""
    hs, vs = CHROMA_SHIFTS[str(chroma)]
    return (w + hs) >> hs, (h + vs) >> vs


def i420_frame_bytes(w: int, h: int, chroma: str = "420") -> int:
    cw, ch = chroma_size(w, h, chroma)
    return w * h + 2 * cw * ch


def split_i420(frame: np.ndarray, w: int, h: int, chroma: str = "420"):
    """Views (Y, U, V) of one packed planar frame (I420 unless `chroma` says otherwise)."""
    cw, ch = chroma_size(w, h, chroma)
    f = np.asarray(frame, dtype=np.uint8).reshape(-1)
    y = f[: w * h].reshape(h, w)
    u = f[w * h: w * h + cw * ch].reshape(ch, cw)
    v = f[w * h + cw * ch: w * h + 2 * cw * ch].reshape(ch, cw)
    return y, u, v


def pack_i420(y, u, v) -> np.ndarray:
    return np.concatenate([np.asarray(p, np.uint8).reshape(-1) for p in (y, u, v)])


class MjpegEncoder:
    """One encoder context on one GPU (owns a HIP stream and device buffers)."""

    def __init__(self, device: int, src_w: int, src_h: int, dst_w: Optional[int] = None,
                 dst_h: Optional[int] = None, full_range: bool = False, qscale: int = 5,
                 sar=(1, 1), max_batch: int = 16, timing: bool = False,
                 debug_coefs: bool = False, sws_bitexact: bool = True, com_itu601: bool = False,
                 huffman: str = "default", chroma: str = "420", rst: bool = False,
                 merge: bool = False):
        self._L = _lib.load()
        self.device = int(device)
        self.src_w, self.src_h = int(src_w), int(src_h)
        self.dst_w = int(dst_w if dst_w is not None else src_w)
        self.dst_h = int(dst_h if dst_h is not None else src_h)
        self.max_batch = int(max_batch)
        flags = 0
        if timing == "detail":
            flags |= _lib.MJG_F_TIMING_DETAIL
        elif timing:
            flags |= _lib.MJG_F_TIMING
        if debug_coefs:
            flags |= _lib.MJG_F_DEBUG_COEFS
        if not sws_bitexact:
            flags |= _lib.MJG_F_SWS_NO_BITEXACT
        if com_itu601:
            flags |= _lib.MJG_F_COM_ITU601
        if huffman == "optimal":
            flags |= _lib.MJG_F_HUFFMAN_OPTIMAL
        elif huffman != "default":
            raise ValueError(f"huffman {huffman!r}")
        if rst:
            flags |= _lib.MJG_F_RST
        # library-side merging of single-segment device submits (MJG_F_MERGE, opt-in): a device
        # submit is held and launched with the next one, so its frames must stay unchanged until
        # its own sync; merge=False: every submit is a launch of its own, launched in submit()
        if merge:
            flags |= _lib.MJG_F_MERGE
        self.huffman = huffman
        self.chroma = str(chroma)
        if self.chroma not in _lib.CHROMA_FORMATS:
            raise ValueError(f"chroma {chroma!r}")
        self.rst = bool(rst)
        sar = sar or (0, 0)
        cfg = MjgConfig(self.src_w, self.src_h, self.dst_w, self.dst_h, int(bool(full_range)),
                        int(qscale), int(sar[0]), int(sar[1]), self.max_batch, flags,
                        _lib.CHROMA_FORMATS[self.chroma])
        h = C.c_void_p()
        check(self._L.mjg_open(self.device, C.byref(cfg), C.byref(h)))
        self._h = h
        self.frame_bytes = int(self._L.mjg_frame_bytes(h))
        self._queued = deque()        # (nframes, host buffer kept alive) per queued submit
        self._synced_since_submit = False
        self._last_sizes = np.zeros(0, np.uint64)
        self._sizes = np.zeros(self.max_batch + 1, np.uint64)

    # ------------------------------------------------------------------ basics
    def close(self):
        if getattr(self, "_h", None):
            self._L.mjg_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return int(self._L.mjg_stream(self._h) or 0)

    def header(self) -> bytes:
        n = C.c_size_t()
        check(self._L.mjg_header(self._h, None, 0, C.byref(n)))
        buf = (C.c_uint8 * n.value)()
        check(self._L.mjg_header(self._h, buf, n.value, C.byref(n)))
        return bytes(buf)

    # ------------------------------------------------------------------ encode
    @property
    def pending(self) -> int:
        """Submits queued and not yet synced (at most `depth`)."""
        return len(self._queued)

    @property
    def depth(self) -> int:
        """Device-pointer submits (submit(device_ptr=...)) pending at most before one must be
        synced (mjg_ctx_queue_depth: two launches, of up to two merged submits each with
        merge=True)."""
        if hasattr(self._L, "mjg_ctx_queue_depth"):
            return int(self._L.mjg_ctx_queue_depth(self._h))
        return self.host_depth

    @property
    def host_depth(self) -> int:
        """Host-buffer submits and submit_segments() calls pending at most before one must be
        synced: each takes a launch of its own (mjg_queue_depth)."""
        return int(self._L.mjg_queue_depth()) if hasattr(self._L, "mjg_queue_depth") else 2

    def submit(self, frames=None, nframes: Optional[int] = None, device_ptr: Optional[int] = None):
        """Queue `nframes` packed frames: a host buffer (numpy / bytes) or a device pointer
        (`device_ptr`, e.g. torch_tensor.data_ptr() on this GPU, kept alive until its sync).
        Up to `host_depth` host submits may be queued (each one's k_encode runs beside the
        previous one's drain and tail kernels), up to `depth` device submits: with merge=True the
        library holds a device submit and launches it with the next one."""
        if device_ptr is not None:
            if nframes is None:
                raise ValueError("nframes is required with device_ptr")
            check(self._L.mjg_submit(self._h, C.c_void_p(int(device_ptr)), int(nframes), 1))
            self._queued.append((int(nframes), None))
            self._synced_since_submit = False
            return
        arr = np.ascontiguousarray(np.frombuffer(frames, dtype=np.uint8)
                                   if isinstance(frames, (bytes, bytearray, memoryview))
                                   else np.asarray(frames, dtype=np.uint8))
        if arr.size % self.frame_bytes:
            raise ValueError(f"buffer of {arr.size} bytes is not a whole number of "
                             f"{self.frame_bytes}-byte frames")
        n = arr.size // self.frame_bytes if nframes is None else int(nframes)
        check(self._L.mjg_submit(self._h, C.c_void_p(arr.ctypes.data), n, 0))
        self._queued.append((n, arr))  # the async H2D copy reads arr until its sync
        self._synced_since_submit = False

    def submit_segments(self, segments):
        """Queue several segments as ONE submit (mjg_submit_segments): `segments` is a list of
        (device_ptr, nframes) on this GPU, at most mjg_max_segments() of them, totalling at
        most max_batch frames.  One launch per kernel covers them
        all; sync() then returns the frames' sizes in segment order and fetch() their JPEGs,
        the same bytes as one submit() per segment.  Every segment's device buffer must stay
        alive until this submit is synced (the kernels read it in place)."""
        if not hasattr(self._L, "mjg_submit_segments"):
            raise MjgError(_lib.MJG_E_STATE, "library lacks mjg_submit_segments")
        k = len(segments)
        ptrs = (C.c_void_p * max(k, 1))(*[C.c_void_p(int(p)) for p, _ in segments])
        ns = (C.c_int * max(k, 1))(*[int(n) for _, n in segments])
        check(self._L.mjg_submit_segments(self._h, ptrs, ns, k))
        self._queued.append((sum(int(n) for _, n in segments), None))
        self._synced_since_submit = False

    @property
    def max_segments(self) -> int:
        """Most segments one submit_segments() may carry (mjg_max_segments)."""
        if not hasattr(self._L, "mjg_max_segments"):
            raise MjgError(_lib.MJG_E_STATE, "library lacks mjg_max_segments")
        return int(self._L.mjg_max_segments())

    def sync(self) -> np.ndarray:
        """Complete the oldest queued submit; its per-frame JPEG sizes."""
        if not self._queued:
            return self._last_sizes.copy()
        total = C.c_uint64()
        check(self._L.mjg_sync(self._h, self._sizes.ctypes.data_as(C.POINTER(C.c_uint64)),
                               C.byref(total)))
        n, _ = self._queued.popleft()
        self._synced_since_submit = True
        self._last_sizes = self._sizes[:n].copy()
        return self._last_sizes.copy()

    def fetch(self) -> List[bytes]:
        """Packed JPEGs of the last synced submit (syncing the oldest queued one first when
        sync() was not called since the last submit)."""
        if self._queued and not self._synced_since_submit:
            self.sync()
        sizes = self._last_sizes
        data, n = C.c_void_p(), C.c_size_t()
        check(self._L.mjg_fetch_host(self._h, C.byref(data), C.byref(n)))  # page-locked copy
        if int(n.value) != int(sizes.sum()):
            raise MjgError(_lib.MJG_E_STATE, "fetch size mismatch")
        out, o = [], int(data.value or 0)
        for s in sizes:
            out.append(C.string_at(o, int(s)))
            o += int(s)
        return out

    def fetch_views(self) -> List[memoryview]:
        """fetch() with one copy: the packed JPEGs copied once out of the page-locked buffer,
        returned as memoryview slices (valid as long as the views are referenced)."""
        if self._queued and not self._synced_since_submit:
            self.sync()
        sizes = self._last_sizes
        data, n = C.c_void_p(), C.c_size_t()
        check(self._L.mjg_fetch_host(self._h, C.byref(data), C.byref(n)))
        if int(n.value) != int(sizes.sum()):
            raise MjgError(_lib.MJG_E_STATE, "fetch size mismatch")
        mv = memoryview(C.string_at(int(data.value or 0), int(n.value)) if n.value else b"")
        out, o = [], 0
        for s in sizes:
            out.append(mv[o:o + int(s)])
            o += int(s)
        return out

    def fetch_into(self, buf: "PinnedBuffer") -> List[memoryview]:
        """The packed JPEGs of the last synced submit DMA'd straight into `buf` (page-locked,
        PinnedBuffer: mjg_fetch's one-DMA path, no host copy), returned as memoryview slices of
        it; MjgError(MJG_E_CAPACITY) when `buf` is too small (see last_total)."""
        if self._queued and not self._synced_since_submit:
            self.sync()
        sizes = self._last_sizes
        total = int(sizes.sum())
        check(self._L.mjg_fetch(self._h, C.c_void_p(buf.ptr), int(buf.nbytes)))
        mv = memoryview(buf.array)[:total]
        out, o = [], 0
        for s in sizes:
            out.append(mv[o:o + int(s)])
            o += int(s)
        return out

    @property
    def last_total(self) -> int:
        """Packed bytes of the last synced submit."""
        return int(self._last_sizes.sum())

    def encode(self, frames) -> List[bytes]:
        """Encode host frames (any count; split into max_batch submits)."""
        arr = np.ascontiguousarray(np.asarray(frames, dtype=np.uint8)).reshape(-1)
        n = arr.size // self.frame_bytes
        out: List[bytes] = []
        for i in range(0, n, self.max_batch):
            k = min(self.max_batch, n - i)
            self.submit(arr[i * self.frame_bytes:(i + k) * self.frame_bytes], k)
            out.extend(self.fetch())
        return out

    def output_device(self):
        data, offs = C.c_void_p(), C.c_void_p()
        check(self._L.mjg_output_device(self._h, C.byref(data), C.byref(offs)))
        return int(data.value or 0), int(offs.value or 0)

    # ------------------------------------------------------------------ timing/debug
    def kernel_times(self, reset: bool = False):
        ms = (C.c_double * _lib.MJG_NUM_KERNELS)()
        n = C.c_int()
        check(self._L.mjg_kernel_times(self._h, ms, C.byref(n), int(bool(reset))))
        return {k: ms[i] for i, k in enumerate(_lib.KERNEL_NAMES)}, n.value

    def debug_coefs(self, frame: int = 0) -> np.ndarray:
        mcu_w = 8 if self.chroma == "444" else 16
        nmcu = ((self.dst_w + mcu_w - 1) // mcu_w) * ((self.dst_h + 15) // 16)
        out = np.zeros((nmcu * (8 if self.chroma == "422" else 6), 64), np.int16)
        check(self._L.mjg_debug_coefs(self._h, int(frame), out.ctypes.data_as(C.POINTER(C.c_int16)),
                                      out.shape[0]))
        return out

    def debug_planes(self, frame: int = 0) -> np.ndarray:
        n = i420_frame_bytes(self.dst_w, self.dst_h, self.chroma)
        out = np.zeros(n, np.uint8)
        check(self._L.mjg_debug_planes(self._h, int(frame), out.ctypes.data_as(C.POINTER(C.c_uint8)), n))
        return out

    def debug_filter(self, plane: int, direction: int):
        taps, ln = C.c_int(), C.c_int()
        check(self._L.mjg_debug_filter(self._h, plane, direction, None, None, C.byref(taps),
                                       C.byref(ln)))
        coeff = np.zeros((ln.value, taps.value), np.int16)
        pos = np.zeros(ln.value, np.int32)
        check(self._L.mjg_debug_filter(self._h, plane, direction,
                                       coeff.ctypes.data_as(C.POINTER(C.c_int16)),
                                       pos.ctypes.data_as(C.POINTER(C.c_int32)),
                                       C.byref(taps), C.byref(ln)))
        return coeff, pos


class PinnedBuffer:
    """Page-locked host buffer from mjg_host_alloc (fast async H2D for submits)."""

    def __init__(self, nbytes: int):
        self._L = _lib.load()
        p = C.c_void_p()
        check(self._L.mjg_host_alloc(int(nbytes), C.byref(p)))
        self.ptr = int(p.value)
        self.nbytes = int(nbytes)
        self.array = np.ctypeslib.as_array((C.c_uint8 * self.nbytes).from_address(self.ptr))

    def free(self):
        if self.ptr:
            self._L.mjg_host_free(C.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


__all__ = ["MjpegEncoder", "MjgError", "PinnedBuffer", "i420_frame_bytes", "split_i420",
           "pack_i420"]
