"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle, byte for byte.

The oracle restates FFmpeg's mjpeg encoder / swscale (oracle/mjpeg_oracle.c); parity
against FFmpeg itself is unpinned (FFmpeg is absent on this pool).
"""
import io

import os

import numpy as np
import pytest

import oracle
from ffmpeg_distributed_amd.encoder import (MjpegEncoder, split_i420, pack_i420, i420_frame_bytes,
                                            chroma_size)
from ffmpeg_distributed_amd.testsrc import testsrc2_i420 as make_testsrc

pytestmark = pytest.mark.gpu


def rand_frames(w, h, n, seed, kind="noise", chroma="420"):
    rng = np.random.default_rng(seed)
    fb = i420_frame_bytes(w, h, chroma)
    cw, ch = chroma_size(w, h, chroma)
    if kind == "noise":
        return rng.integers(0, 256, (n, fb), dtype=np.uint8)
    if kind == "smooth":
        out = []
        for i in range(n):
            yy, xx = np.mgrid[0:h, 0:w]
            cy, cx = np.mgrid[0:ch, 0:cw]
            y = (128 + 90 * np.sin(xx / (5 + i) + yy / 9) + rng.normal(0, 3, (h, w))).clip(0, 255)
            u = (128 + 50 * np.cos(cx / 4 + i)).clip(0, 255) + 0 * cy
            v = (128 + 50 * np.sin(cy / 3 - i)).clip(0, 255) + 0 * cx
            out.append(pack_i420(y.astype(np.uint8), u.astype(np.uint8), v.astype(np.uint8)))
        return np.stack(out)
    if kind == "flat":
        return np.full((n, fb), 255 if seed % 2 else 0, np.uint8)
    if kind == "checker":
        out = []
        for i in range(n):
            yy, xx = np.mgrid[0:h, 0:w]
            y = np.where(((xx + yy + i) & 1) == 0, 255, 0).astype(np.uint8)
            cy, cx = np.mgrid[0:ch, 0:cw]
            u = np.where(((cx // 2 + cy // 2) & 1) == 0, 255, 0).astype(np.uint8)
            v = (255 - u).astype(np.uint8)
            out.append(pack_i420(y, u, v))
        return np.stack(out)
    if kind == "patches":  # flat picture with noisy 8x8 patches: a few long blocks per chunk
        out = []
        for i in range(n):
            f = np.full(fb, 96, np.uint8)
            y = f[: w * h].reshape(h, w)
            for _ in range(max(1, (w // 8) * (h // 8) // 12)):
                by, bx = rng.integers(0, max(1, h // 8)), rng.integers(0, max(1, w // 8))
                y[by * 8:by * 8 + 8, bx * 8:bx * 8 + 8] = rng.integers(0, 256, (8, 8))[: h - by * 8, : w - bx * 8]
            out.append(f)
        return np.stack(out)
    if kind == "testsrc":
        out = []
        for i in range(n):
            y, u, v = split_i420(make_testsrc(w, h, seed + i), w, h)
            if chroma != "420":  # the 4:2:0 chroma, replicated to the format's plane size
                rr = 1 if chroma == "422" else 2
                u = np.repeat(np.repeat(u, 2, 0), rr, 1)[:ch, :cw]
                v = np.repeat(np.repeat(v, 2, 0), rr, 1)[:ch, :cw]
            out.append(pack_i420(y, u, v))
        return np.stack(out)
    raise ValueError(kind)


def oracle_frames(frames, w, h, q, full_range, dw=None, dh=None, sar=(1, 1), huffman="default",
                  chroma="420", rst=False):
    out = []
    for f in frames:
        y, u, v = split_i420(f, w, h, chroma)
        out.append(oracle.encode_frame(y, u, v, dst_w=dw, dst_h=dh, full_range=full_range,
                                       qscale=q, sar=sar, huffman=huffman, chroma=chroma, rst=rst))
    return out


def first_diff(a: bytes, b: bytes):
    n = min(len(a), len(b))
    for i in range(n):
        if a[i] != b[i]:
            return i
    return n if len(a) != len(b) else -1


CASES = [
    # (w, h, q, full_range, kind)
    (72, 40, 5, False, "smooth"),
    (64, 48, 5, True, "smooth"),
    (72, 40, 2, False, "noise"),
    (72, 40, 31, True, "noise"),
    (16, 16, 5, True, "flat"),
    (8, 8, 3, False, "smooth"),
    (130, 66, 4, False, "checker"),
    (101, 57, 7, True, "smooth"),
    (1920, 1080, 5, False, "testsrc"),
    (1280, 720, 2, True, "noise"),
    # blocks past 128 bits staged in HBM among short ones (k_encode ShiftSink spill/flush)
    (256, 128, 1, True, "patches"),
    (200, 72, 2, False, "patches"),
    # a short last chunk (2 / 6 blocks) that starts and ends inside the frame's last word:
    # the byte padding must still be applied (the word's owner is the chunk before it)
    (176, 16, 5, True, "flat"),
    (176, 16, 5, False, "patches"),
]


@pytest.mark.parametrize("w,h,q,full,kind", CASES)
def test_encode_matches_oracle(w, h, q, full, kind):
    n = 3
    frames = rand_frames(w, h, n, seed=w * 31 + h + q, kind=kind)
    with MjpegEncoder(0, w, h, qscale=q, full_range=full, max_batch=4) as enc:
        got = enc.encode(frames)
    ref = oracle_frames(frames, w, h, q, full)
    for i in range(n):
        assert got[i] == ref[i], (i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


@pytest.mark.parametrize("w,h,q,full,kind", CASES)
def test_encode_huffman_optimal_matches_oracle(w, h, q, full, kind):
    """-huffman optimal (FFmpeg's default): per-frame tables from GPU symbol counts."""
    n = 3
    frames = rand_frames(w, h, n, seed=w * 17 + h + q, kind=kind)
    with MjpegEncoder(0, w, h, qscale=q, full_range=full, max_batch=4, huffman="optimal") as enc:
        got = enc.encode(frames)
    ref = oracle_frames(frames, w, h, q, full, huffman="optimal")
    for i in range(n):
        assert got[i] == ref[i], (i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


@pytest.mark.parametrize("kind,full", [("noise", False), ("checker", True), ("testsrc", False), ("smooth", True)])
def test_scale_2to1_matrix_core_hpass(kind, full):
    """Exact 2:1 downscales take k_scale's matrix-core h-pass on their interior tile columns
    (every column but the first and last 64): extreme pixels (noise, checker: the largest h sums
    and the range clamps) and smooth content, tv and pc range, byte-equal to the oracle."""
    w, h, n = 1536, 768, 2
    frames = rand_frames(w, h, n, seed=91, kind=kind)
    with MjpegEncoder(0, w, h, w // 2, h // 2, qscale=4, full_range=full, max_batch=n) as enc:
        got = enc.encode(frames)
    ref = oracle_frames(frames, w, h, 4, full, w // 2, h // 2)
    for i in range(n):
        assert got[i] == ref[i], (i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


def _extreme_2to1_frame(w, h, seed, full):
    """Pixels that drive both passes of a 2:1 bicubic to their extremes: horizontal bands of
    0 / 255 rows (the v filter's negative lobes against the largest h values, 32767 after the
    clamp, and the smallest), vertical full-swing stripes, a pixel checker and noise, each in a
    region several 64-row tiles tall; tv range input keeps 0..255 (swscale clamps it)."""
    rng = np.random.default_rng(seed)
    y = np.zeros((h, w), np.uint8)
    q = w // 4
    rows = np.arange(h)[:, None]
    cols = np.arange(q)[None, :]
    y[:, :q] = np.where((rows // (1 + seed % 3)) % 2 + 0 * cols, 255, 0)  # horizontal bands
    y[:, q:2 * q] = np.where((cols // 2) % 2 + 0 * rows, 255, 0)          # vertical stripes
    y[:, 2 * q:3 * q] = np.where((rows + cols) % 2, 255, 0)               # pixel checker
    y[:, 3 * q:] = rng.integers(0, 256, (h, w - 3 * q))                   # noise
    y[h // 3: h // 3 + 70, :] = 255                                  # a white band across
    y[2 * h // 3: 2 * h // 3 + 5, :] = 0
    cw, ch = (w + 1) // 2, (h + 1) // 2
    u = np.where((np.arange(ch)[:, None] // 3) % 2, 255, 0).astype(np.uint8).repeat(cw, 1)
    v = rng.integers(0, 256, (ch, cw)).astype(np.uint8)
    v[:, : cw // 2] = np.where((np.arange(cw // 2)[None, :] + np.arange(ch)[:, None]) % 2, 0, 255)
    return pack_i420(y, u, v)


@pytest.mark.parametrize("full", [False, True])
def test_scale_2to1_matrix_core_vpass(full):
    """Exact 2:1 downscales also take k_scale's matrix-core v-pass on their interior tiles (tile
    rows but the first and last, h values split into signed hi / offset lo bytes, taps into
    128 fh + fl): content at both passes' extremes, tv and pc range; the scaled planes equal the
    oracle's swscale restatement and the JPEGs its encoder, byte for byte."""
    w, h, n = 1536, 896, 2
    frames = np.stack([_extreme_2to1_frame(w, h, s, full) for s in range(n)])
    with MjpegEncoder(0, w, h, w // 2, h // 2, qscale=4, full_range=full, max_batch=n) as enc:
        enc.submit(frames)
        enc.sync()
        planes = [enc.debug_planes(i) for i in range(n)]
        got = enc.fetch()
    for i in range(n):
        y, u, v = split_i420(frames[i], w, h)
        gy, gu, gv = split_i420(planes[i], w // 2, h // 2)
        ry = oracle.scale_plane(y, w // 2, h // 2, 0 if full else 1)
        assert (gy == ry).all(), (i, np.argwhere(gy != ry)[:5])
        for g, p in ((gu, u), (gv, v)):
            r = oracle.scale_plane(p, w // 4, h // 4, 0 if full else 2, chroma=True)
            assert (g == r).all(), (i, np.argwhere(g != r)[:5])
    assert got == oracle_frames(frames, w, h, 4, full, w // 2, h // 2)


def test_huffman_optimal_scaled_batches():
    """optimal tables with -vf scale, ragged batches and a reused context."""
    sw, sh, dw, dh, q = 160, 96, 80, 48, 3
    frames = rand_frames(sw, sh, 5, seed=3, kind="smooth")
    with MjpegEncoder(0, sw, sh, dw, dh, qscale=q, max_batch=3, huffman="optimal") as enc:
        got = enc.encode(frames[:3]) + enc.encode(frames[3:])
    assert got == oracle_frames(frames, sw, sh, q, False, dw, dh, huffman="optimal")


@pytest.mark.parametrize("w,h,q,full", [(72, 40, 5, False), (1920, 1080, 3, True)])
def test_coefficients_match_oracle(w, h, q, full):
    frames = rand_frames(w, h, 2, seed=1, kind="smooth" if w < 200 else "testsrc")
    with MjpegEncoder(0, w, h, qscale=q, full_range=True, max_batch=2, debug_coefs=True) as enc:
        enc.submit(frames)
        enc.sync()
        for i in range(2):
            y, u, v = split_i420(frames[i], w, h)
            ref, _ = oracle.frame_coeffs(y, u, v, q)
            got = enc.debug_coefs(i)
            bad = np.nonzero((got != ref).any(1))[0]
            assert bad.size == 0, (i, bad[:10])


def test_batching_and_reuse():
    w, h, q = 96, 64, 6
    frames = rand_frames(w, h, 7, seed=3, kind="smooth")
    ref = oracle_frames(frames, w, h, q, False)
    with MjpegEncoder(0, w, h, qscale=q, max_batch=3) as enc:
        got = enc.encode(frames)          # 3 + 3 + 1 frames
        got2 = enc.encode(frames[::-1])   # context reuse, different order
    assert got == ref
    assert got2 == ref[::-1]


def test_sar_and_header():
    w, h = 48, 32
    frames = rand_frames(w, h, 1, seed=9, kind="smooth")
    for sar in [(1, 1), (0, 0), (4, 3)]:
        with MjpegEncoder(0, w, h, qscale=5, sar=sar, max_batch=1) as enc:
            got = enc.encode(frames)[0]
            hdr = enc.header()
        ref = oracle_frames(frames, w, h, 5, False, sar=sar)[0]
        assert got == ref
        assert got.startswith(hdr)
        assert hdr == oracle.header(w, h, 5, sar=sar)


def test_output_overflow_regrow():
    # noise at q=2 compresses worse than raw: exercises the grow-and-rewrite path
    w, h = 256, 128
    frames = rand_frames(w, h, 4, seed=5, kind="noise")
    with MjpegEncoder(0, w, h, qscale=2, full_range=True, max_batch=4) as enc:
        got = enc.encode(frames)
    assert got == oracle_frames(frames, w, h, 2, True)


@pytest.mark.parametrize("sw,sh,dw,dh,full", [
    (3840, 2160, 1920, 1080, False),
    (160, 96, 80, 48, False),
    (160, 96, 80, 48, True),
    (100, 60, 64, 40, False),
    (64, 48, 100, 70, True),
    # one axis unscaled: swscale's 1-tap filter (odd v taps; h taps padded to 4 with zeros)
    (1920, 1080, 1280, 1080, False),
    (1920, 1080, 1920, 720, True),
    # sources narrower than the filter: windows past the row end (zeroed coefficients)
    (9, 8, 30, 8, False),
    (12, 10, 8, 9, True),
])
def test_scale_matches_oracle(sw, sh, dw, dh, full):
    n = 2
    kind = "testsrc" if sw >= 1000 else "smooth"
    frames = rand_frames(sw, sh, n, seed=11, kind=kind)
    q = 3
    with MjpegEncoder(0, sw, sh, dw, dh, qscale=q, full_range=full, max_batch=2) as enc:
        enc.submit(frames)
        enc.sync()
        planes = [enc.debug_planes(i) for i in range(n)]
        for p in range(2):
            for d in range(2):
                coeff, pos = enc.debug_filter(p, d)
                src = (sw if p == 0 else (sw + 1) // 2) if d == 0 else (sh if p == 0 else (sh + 1) // 2)
                dst = (dw if p == 0 else (dw + 1) // 2) if d == 0 else (dh if p == 0 else (dh + 1) // 2)
                rc, rp = oracle.sws_filter(src, dst, 1 << (14 if d == 0 else 12), 4 if d == 0 else 2,
                                           src_pos=128, dst_pos=128)
                assert (coeff == rc).all() and (pos == rp).all(), (p, d)
        got = enc.fetch()
    for i in range(n):
        y, u, v = split_i420(frames[i], sw, sh)
        ry = oracle.scale_plane(y, dw, dh, 0 if full else 1)
        ru = oracle.scale_plane(u, (dw + 1) // 2, (dh + 1) // 2, 0 if full else 2, chroma=True)
        rv = oracle.scale_plane(v, (dw + 1) // 2, (dh + 1) // 2, 0 if full else 2, chroma=True)
        gy, gu, gv = split_i420(planes[i], dw, dh)
        assert (gy == ry).all() and (gu == ru).all() and (gv == rv).all()
    assert got == oracle_frames(frames, sw, sh, q, full, dw, dh)


SCALE_CASES = [
    # (sw, sh, dw, dh, q, full, kind, n, huffman): k_scale + k_encode vs the oracle (the cases
    # of the one-kernel k_scale_encode, retired in r05, kept for the two-kernel path)
    (3840, 2160, 1920, 1080, 3, False, "testsrc", 3, "default"),   # BASELINE configs[3]
    (3840, 2160, 1920, 1080, 3, True, "noise", 2, "default"),
    (3840, 2160, 1920, 1080, 5, False, "testsrc", 2, "optimal"),
    (1920, 1080, 1280, 720, 4, False, "smooth", 2, "default"),      # 1.5:1
    (1280, 720, 640, 360, 2, True, "patches", 3, "default"),
    (640, 360, 1280, 720, 5, False, "testsrc", 2, "default"),       # upscale: 4 taps
    (400, 300, 200, 150, 6, False, "checker", 3, "optimal"),        # < 32 MCUs per row
    (96, 64, 48, 32, 3, True, "noise", 2, "default"),
    (1040, 530, 520, 265, 5, False, "smooth", 3, "default"),        # 33 MCUs per row, odd height
    (1030, 520, 515, 260, 4, True, "checker", 2, "optimal"),        # edge MCU column, partial group
    (2200, 1300, 1100, 650, 7, False, "patches", 1, "default"),     # nmcu % 32 != 0
    (1200, 700, 1023, 600, 3, False, "noise", 2, "default"),        # mild downscale
]


@pytest.mark.parametrize("sw,sh,dw,dh,q,full,kind,n,huffman", SCALE_CASES)
def test_scale_encode_cases_match_oracle(sw, sh, dw, dh, q, full, kind, n, huffman):
    """k_scale + k_encode byte-equal to the oracle's scale_plane + encode_frame (2:1, 1.5:1,
    upscale, odd sizes, partial MCU rows, both Huffman modes)."""
    frames = rand_frames(sw, sh, n, seed=sw + dh + q, kind=kind)
    with MjpegEncoder(0, sw, sh, dw, dh, qscale=q, full_range=full, max_batch=2, huffman=huffman) as enc:
        got = enc.encode(frames)
    ref = _oracle_many(frames, sw, sh, dst_w=dw, dst_h=dh, full_range=full, qscale=q, huffman=huffman)
    for i in range(n):
        assert got[i] == ref[i], (i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


def test_scaled_4k_segment_batch_from_device_memory():
    """BASELINE configs[3] as bench.py submits it: 120 4K frames by device pointer through
    k_scale + k_encode, every frame equal to the oracle."""
    import torch
    from ffmpeg_distributed_amd.testsrc import testsrc2_i420_torch
    w, h, n = 3840, 2160, 120
    dev = torch.device("cuda", 0)
    pool = torch.empty((n, i420_frame_bytes(w, h)), dtype=torch.uint8, device=dev)
    for i in range(0, n, 20):
        pool[i:i + 20] = testsrc2_i420_torch(w, h, 500 + i, 20, dev)
    torch.cuda.synchronize()
    host = pool.cpu().numpy()
    with MjpegEncoder(0, w, h, 1920, 1080, qscale=3, max_batch=n) as enc:
        enc.submit(device_ptr=pool.data_ptr(), nframes=n)
        got = enc.fetch()
    ref = _oracle_many(host, w, h, dst_w=1920, dst_h=1080, qscale=3)
    for i in range(n):
        assert got[i] == ref[i], (i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


def _oracle_many(frames, w, h, **kw):
    """The oracle over many frames on a thread pool (ctypes releases the GIL)."""
    from concurrent.futures import ThreadPoolExecutor

    def one(f):
        y, u, v = split_i420(f, w, h)
        return oracle.encode_frame(y, u, v, **kw)

    with ThreadPoolExecutor(16) as ex:
        return list(ex.map(one, frames))


def test_4k_full_size_properties():
    """BASELINE config 2 size: every frame equal to the oracle, decodable, deterministic."""
    from PIL import Image
    w, h = 3840, 2160
    frames = np.stack([make_testsrc(w, h, t) for t in range(4)])
    with MjpegEncoder(0, w, h, qscale=5, max_batch=4) as enc:
        a = enc.encode(frames)
        b = enc.encode(frames)
    assert a == b
    for j in a:
        im = Image.open(io.BytesIO(j))
        im.load()
        assert im.size == (w, h)
    ref = _oracle_many(frames, w, h, qscale=5)
    for i in range(4):
        assert a[i] == ref[i], (i, len(a[i]), len(ref[i]), first_diff(a[i], ref[i]))


def test_4k_segment_batch_from_device_memory():
    """The bench's exact submission: one 120-frame 4K segment (BASELINE configs[1], a 2 s
    segment at 60 fps) generated in HBM and submitted by device pointer, two submits
    queued; every frame of both submits byte-equal to the oracle."""
    import torch
    from ffmpeg_distributed_amd.testsrc import testsrc2_i420_torch
    w, h, n = 3840, 2160, 120
    dev = torch.device("cuda", 0)
    pool = torch.empty((n, i420_frame_bytes(w, h)), dtype=torch.uint8, device=dev)
    for i in range(0, n, 20):
        pool[i:i + 20] = testsrc2_i420_torch(w, h, 1000 + i, 20, dev)
    torch.cuda.synchronize()
    host = pool.cpu().numpy()
    assert (host[59] == make_testsrc(w, h, 1059)).all()  # the device generator = the host one
    with MjpegEncoder(0, w, h, qscale=5, max_batch=n, merge=True) as enc:
        enc.submit(device_ptr=pool.data_ptr(), nframes=n)
        enc.submit(device_ptr=pool[60].data_ptr(), nframes=60)
        s0 = enc.sync()
        a = enc.fetch()
        s1 = enc.sync()
        b = enc.fetch()
    ref = _oracle_many(host, w, h, qscale=5)
    assert list(s0) == [len(r) for r in ref]
    for i in range(n):
        assert a[i] == ref[i], (i, len(a[i]), len(ref[i]), first_diff(a[i], ref[i]))
    assert list(s1) == [len(r) for r in ref[60:]] and b == ref[60:]


@pytest.mark.parametrize("w,h,full,huff", [(72, 40, False, "default"), (333, 177, True, "default"),
                                            (1920, 1080, False, "optimal")])
def test_submit_segments_matches_oracle(w, h, full, huff):
    """mjg_submit_segments: three segments of 3, 1 and 4 frames in separate device buffers
    as ONE submit (one k_encode launch); every frame byte-equal to the oracle, in segment
    order, and the same bytes again from a second queued multi-segment submit."""
    import torch
    dev = torch.device("cuda", 0)
    counts = [3, 1, 4]
    frames = np.stack([make_testsrc(w, h, 7 * t + 3, full_range=full) for t in range(sum(counts))])
    segs, o = [], 0
    for k in counts:  # separate allocations: the segments are not contiguous in memory
        segs.append(torch.from_numpy(frames[o:o + k].copy()).to(dev))
        o += k
    torch.cuda.synchronize()
    ref = _oracle_many(frames, w, h, qscale=5, full_range=full, huffman=huff)
    with MjpegEncoder(0, w, h, qscale=5, full_range=full, max_batch=sum(counts), huffman=huff) as enc:
        assert enc.max_segments >= len(counts)
        enc.submit_segments([(t.data_ptr(), t.shape[0]) for t in segs])
        enc.submit_segments([(segs[2].data_ptr(), 4), (segs[0].data_ptr(), 3)])
        s0 = enc.sync()
        a = enc.fetch()
        s1 = enc.sync()
        b = enc.fetch()
    assert list(s0) == [len(r) for r in ref]
    for i in range(len(ref)):
        assert a[i] == ref[i], (i, len(a[i]), len(ref[i]), first_diff(a[i], ref[i]))
    assert b == ref[4:] + ref[:3] and list(s1) == [len(r) for r in b]


def test_4k_submit_segments_equals_per_segment_submits():
    """BASELINE configs[1]'s segments (120 4K frames) two per submit: the bytes of each are
    those of one submit per segment (which test_4k_segment_batch_from_device_memory pins to
    the oracle), with two multi-segment submits queued."""
    import torch
    from ffmpeg_distributed_amd.testsrc import testsrc2_i420_torch
    w, h, n = 3840, 2160, 120
    dev = torch.device("cuda", 0)
    pools = []
    for j in range(3):
        p = torch.empty((n, i420_frame_bytes(w, h)), dtype=torch.uint8, device=dev)
        for i in range(0, n, 20):
            p[i:i + 20] = testsrc2_i420_torch(w, h, 2000 + j * n + i, 20, dev)
        pools.append(p)
    torch.cuda.synchronize()
    with MjpegEncoder(0, w, h, qscale=5, max_batch=2 * n) as enc:
        per = []
        for p in pools:
            enc.submit(device_ptr=p.data_ptr(), nframes=n)
            enc.sync()
            per.append(enc.fetch())
        enc.submit_segments([(pools[0].data_ptr(), n), (pools[1].data_ptr(), n)])
        enc.submit_segments([(pools[2].data_ptr(), n), (pools[0].data_ptr(), 60)])
        enc.sync()
        a = enc.fetch()
        enc.sync()
        b = enc.fetch()
    assert a == per[0] + per[1]
    assert b == per[2] + per[0][:60]


@pytest.mark.parametrize("chroma,rst", [("420", True), ("422", False), ("444", True)])
def test_submit_segments_rst_and_chroma_match_oracle(chroma, rst):
    """mjg_submit_segments with the RST layout (one entropy-coded segment per MCU row) and
    4:2:2 / 4:4:4 input: two segments of 2 and 1 frames, byte-equal to the oracle."""
    import torch
    w, h, q = 200, 72, 4
    frames = rand_frames(w, h, 3, seed=w + h + len(chroma), kind="smooth", chroma=chroma)
    segs = [torch.from_numpy(frames[:2].copy()).to("cuda:0"), torch.from_numpy(frames[2:].copy()).to("cuda:0")]
    torch.cuda.synchronize()
    with MjpegEncoder(0, w, h, qscale=q, full_range=True, max_batch=3, chroma=chroma, rst=rst) as enc:
        enc.submit_segments([(t.data_ptr(), t.shape[0]) for t in segs])
        enc.sync()
        got = enc.fetch()
    ref = oracle_frames(frames, w, h, q, True, chroma=chroma, rst=rst)
    for i in range(3):
        assert got[i] == ref[i], (i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


@pytest.mark.parametrize("w,h,dw,dh,q", [(640, 360, 320, 180, 3), (330, 190, 500, 260, 5)])
def test_submit_segments_scaled_match_oracle(w, h, dw, dh, q):
    """-vf scale with segments (k_scale reads each segment's frames from its own buffer):
    segments of 2, 1 and 2 frames, downscale (BASELINE configs[3]'s 2:1 filters) and an
    upscale, byte-equal to the oracle (swscale bicubic + encode)."""
    import torch
    frames = rand_frames(w, h, 5, seed=w + dh, kind="smooth")
    segs = [torch.from_numpy(frames[a:b].copy()).to("cuda:0") for a, b in ((0, 2), (2, 3), (3, 5))]
    torch.cuda.synchronize()
    with MjpegEncoder(0, w, h, dw, dh, qscale=q, max_batch=5) as enc:
        enc.submit_segments([(t.data_ptr(), t.shape[0]) for t in segs])
        enc.sync()
        got = enc.fetch()
    ref = oracle_frames(frames, w, h, q, False, dw, dh)
    for i in range(5):
        assert got[i] == ref[i], (i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


def test_submit_segments_rejects_bad_lists():
    """Errors, not undefined behaviour: no segments, more than mjg_max_segments(), a total
    over max_batch and an empty segment."""
    import torch
    from ffmpeg_distributed_amd._lib import MjgError
    w, h = 64, 48
    t = torch.zeros((4, i420_frame_bytes(w, h)), dtype=torch.uint8, device="cuda:0")
    with MjpegEncoder(0, w, h, qscale=5, max_batch=4) as enc:
        k = enc.max_segments
        for bad in ([], [(t.data_ptr(), 1)] * (k + 1), [(t.data_ptr(), 3), (t.data_ptr(), 2)],
                    [(t.data_ptr(), 0)]):
            with pytest.raises(MjgError):
                enc.submit_segments(bad)
        enc.submit_segments([(t.data_ptr(), 2), (t.data_ptr(), 2)])  # still usable
        assert len(enc.sync()) == 4


def test_8k_yuvj420p_matches_oracle():
    """BASELINE configs[4]: 7680x4320 yuvj420p q=5 (no range conversion), every frame of a
    3-frame batch (and a ragged second submit) byte-equal to the oracle."""
    w, h = 7680, 4320
    frames = np.stack([make_testsrc(w, h, 40 + t, full_range=True) for t in range(3)])
    with MjpegEncoder(0, w, h, qscale=5, full_range=True, max_batch=2) as enc:
        got = enc.encode(frames)
    ref = _oracle_many(frames, w, h, qscale=5, full_range=True)
    for i in range(3):
        assert got[i] == ref[i], (i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


# ------------------------------------------------ 4:2:2 / 4:4:4 and the RST layout (§8f row 4)
FMT_CASES = [
    # (w, h, q, full_range, kind, chroma)
    (72, 40, 5, False, "smooth", "422"),
    (72, 40, 5, False, "smooth", "444"),
    (101, 57, 3, True, "noise", "422"),
    (101, 57, 3, True, "noise", "444"),
    (130, 66, 4, False, "checker", "444"),
    (16, 16, 5, True, "flat", "422"),
    (8, 8, 3, False, "smooth", "444"),
    (9, 17, 2, True, "noise", "444"),
    (1920, 1080, 5, False, "testsrc", "422"),
    (1280, 720, 3, True, "testsrc", "444"),
]


@pytest.mark.parametrize("w,h,q,full,kind,chroma", FMT_CASES)
def test_chroma_formats_match_oracle(w, h, q, full, kind, chroma):
    n = 3
    frames = rand_frames(w, h, n, seed=w * 7 + h + q, kind=kind, chroma=chroma)
    with MjpegEncoder(0, w, h, qscale=q, full_range=full, max_batch=2, chroma=chroma) as enc:
        got = enc.encode(frames)
    ref = oracle_frames(frames, w, h, q, full, chroma=chroma)
    for i in range(n):
        assert got[i] == ref[i], (i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


@pytest.mark.parametrize("w,h,q,full,kind,chroma", [c + ("420",) for c in CASES] + FMT_CASES)
def test_rst_layout_matches_oracle(w, h, q, full, kind, chroma):
    """Slice-threaded layout: DRI, one entropy-coded segment per MCU row, RST0..7."""
    n = 3
    frames = rand_frames(w, h, n, seed=w * 5 + h + q, kind=kind, chroma=chroma)
    with MjpegEncoder(0, w, h, qscale=q, full_range=full, max_batch=3, chroma=chroma, rst=True) as enc:
        got = enc.encode(frames)
    ref = oracle_frames(frames, w, h, q, full, chroma=chroma, rst=True)
    for i in range(n):
        assert got[i] == ref[i], (i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


@pytest.mark.parametrize("chroma", ["422", "444"])
def test_coefficients_match_oracle_422_444(chroma):
    w, h, q = 101, 57, 4
    frames = rand_frames(w, h, 2, seed=3, kind="smooth", chroma=chroma)
    with MjpegEncoder(0, w, h, qscale=q, full_range=True, max_batch=2, debug_coefs=True,
                      chroma=chroma, rst=True) as enc:
        enc.submit(frames)
        enc.sync()
        for i in range(2):
            y, u, v = split_i420(frames[i], w, h, chroma)
            ref, _ = oracle.frame_coeffs(y, u, v, q, chroma)
            got = enc.debug_coefs(i)
            bad = np.nonzero((got != ref).any(1))[0]
            assert bad.size == 0, (i, bad[:10])


@pytest.mark.parametrize("chroma,rst", [("422", False), ("444", True), ("420", True)])
def test_scale_422_444_rst_matches_oracle(chroma, rst):
    sw, sh, dw, dh, q = 160, 96, 80, 48, 3
    frames = rand_frames(sw, sh, 3, seed=13, kind="smooth", chroma=chroma)
    with MjpegEncoder(0, sw, sh, dw, dh, qscale=q, max_batch=2, chroma=chroma, rst=rst) as enc:
        got = enc.encode(frames)
    assert got == oracle_frames(frames, sw, sh, q, False, dw, dh, chroma=chroma, rst=rst)


def test_rst_4k_full_size():
    """4K with RST (135 restart intervals per frame, 23 chunks per row): every frame equal
    to the oracle, decodable, same pixels as the plain layout."""
    from PIL import Image
    w, h = 3840, 2160
    frames = np.stack([make_testsrc(w, h, t) for t in range(3)])
    with MjpegEncoder(0, w, h, qscale=5, max_batch=3, rst=True) as enc:
        a = enc.encode(frames)
    with MjpegEncoder(0, w, h, qscale=5, max_batch=3) as enc:
        b = enc.encode(frames)
    ref = _oracle_many(frames, w, h, qscale=5, rst=True)
    for i in range(3):
        assert a[i] == ref[i], (i, len(a[i]), len(ref[i]), first_diff(a[i], ref[i]))
    for ja, jb in zip(a, b):
        ia, ib = Image.open(io.BytesIO(ja)), Image.open(io.BytesIO(jb))
        assert np.array_equal(np.asarray(ia), np.asarray(ib))


def test_rst_with_optimal_is_rejected():
    from ffmpeg_distributed_amd._lib import MjgError
    with pytest.raises(MjgError):
        MjpegEncoder(0, 64, 64, huffman="optimal", rst=True)


def test_pipelined_submits():
    """mjg_queue_depth() (2) submits queued at once (each with its own scratch/output slot and
    stream); sync completes them oldest first; one more queued submit is refused; overflow
    regrowth works on a queued slot.  A light stream (smooth) and a heavy one (noise at q=2)
    take both branches of the stuffing tail's wave priority (kernels.hip tail_priority)."""
    from ffmpeg_distributed_amd._lib import MjgError
    w, h, q = 96, 64, 4
    frames = rand_frames(w, h, 7, seed=21, kind="smooth")
    ref = oracle_frames(frames, w, h, q, False)
    with MjpegEncoder(0, w, h, qscale=q, max_batch=3) as enc:
        assert enc.host_depth == 2 and enc.depth == 2  # host submits: one launch each
        enc.submit(frames[0:3])
        enc.submit(frames[3:5])
        with pytest.raises(MjgError):
            enc.submit(frames[5:7])
        s0 = enc.sync()
        got0 = enc.fetch()
        enc.submit(frames[5:7])
        s1 = enc.sync()
        got1 = enc.fetch()
        enc.sync()
        got2 = enc.fetch()
    assert got0 == ref[0:3] and list(s0) == [len(x) for x in ref[0:3]]
    assert got1 == ref[3:5] and list(s1) == [len(x) for x in ref[3:5]]
    assert got2 == ref[5:7]
    # noise at q=2 overflows the packed output: regrow while the other slot is queued
    nz = rand_frames(256, 128, 4, seed=5, kind="noise")
    with MjpegEncoder(0, 256, 128, qscale=2, full_range=True, max_batch=2) as enc:
        enc.submit(nz[:2])
        enc.submit(nz[2:])
        enc.sync()
        a = enc.fetch()
        enc.sync()
        b = enc.fetch()
    assert a + b == oracle_frames(nz, 256, 128, 2, True)


MERGE_CFGS = {"default": (200, 120, 200, 120, "default", False), "optimal": (200, 120, 200, 120, "optimal", False),
              "scale": (240, 136, 120, 68, "default", False), "rst": (200, 120, 200, 120, "default", True)}


@pytest.mark.parametrize("cfg", sorted(MERGE_CFGS))
def test_library_merges_queued_device_submits(cfg):
    """Library-side merging (mjg_submit, r05): a device submit is held and launched together with
    the next one as a segment list; each submit stays a job of its own.  Seven ragged
    single-segment submits (separate device buffers) in the bench's pattern and out of it: pairs
    merge, a held job is launched with its partner or alone at its own sync.  Every job's sizes
    and JPEGs byte-equal to the oracle; four launches for seven jobs ([0 1] [2 3] [4 5] [6]); a
    fifth pending submit is refused; merge=False gives one launch per submit and the same
    bytes."""
    import torch
    from ffmpeg_distributed_amd._lib import MjgError
    sw, sh, dw, dh, huff, rst = MERGE_CFGS[cfg]
    counts = [3, 2, 3, 1, 3, 2, 3]
    frames = rand_frames(sw, sh, sum(counts), seed=404, kind="testsrc")
    ref = oracle_frames(frames, sw, sh, 4, False, dw, dh, huffman=huff, rst=rst)
    segs, o = [], 0
    for k in counts:
        segs.append((torch.from_numpy(frames[o:o + k].copy()).to("cuda:0"), o, k))
        o += k
    torch.cuda.synchronize()

    def run(merge):
        out = {}
        with MjpegEncoder(0, sw, sh, dw, dh, qscale=4, max_batch=3, huffman=huff, rst=rst, timing=True,
                          merge=merge) as enc:
            def sub(j):
                enc.submit(device_ptr=segs[j][0].data_ptr(), nframes=counts[j])

            def done(j):
                sizes = enc.sync()
                out[j] = (list(sizes), enc.fetch())
            if merge:
                assert enc.depth == 4 and enc.host_depth == 2
                for j in range(4):  # [0, 1] and [2, 3] merged
                    sub(j)
                with pytest.raises(MjgError):
                    sub(4)
                done(0)
                sub(4)      # held
                done(1)
                done(2)
                sub(5)      # [4, 5] merged
                done(3)
                done(4)
                done(5)
                sub(6)      # held on the idle GPU
                done(6)     # launched alone at its own sync
            else:
                assert enc.depth == 2
                sub(0)
                sub(1)
                for j in range(len(counts)):
                    done(j)
                    if j + 2 < len(counts):
                        sub(j + 2)
            launches = enc.kernel_times()[1]
        return out, launches

    for merge, want in ((True, 4), (False, len(counts))):
        out, launches = run(merge)
        assert launches == want, (merge, launches)
        for j, (_, o0, k) in enumerate(segs):
            sizes, got = out[j]
            assert sizes == [len(r) for r in ref[o0:o0 + k]], (cfg, merge, j)
            for i in range(k):
                assert got[i] == ref[o0 + i], (cfg, merge, j, i, first_diff(got[i], ref[o0 + i]))


def test_merged_4k_segments_equal_unmerged():
    """BASELINE configs[1] segments (120 4K frames) in the bench's pattern (four device submits
    pending, synced when four are): the merged launches' per-segment bytes equal those of
    unmerged launches (which test_4k_segment_batch_from_device_memory pins to the oracle)."""
    import torch
    from ffmpeg_distributed_amd.testsrc import testsrc2_i420_torch
    w, h, n = 3840, 2160, 120
    dev = torch.device("cuda", 0)
    pools = []
    for j in range(3):
        p = torch.empty((n, i420_frame_bytes(w, h)), dtype=torch.uint8, device=dev)
        for i in range(0, n, 20):
            p[i:i + 20] = testsrc2_i420_torch(w, h, 5000 + j * n + i, 20, dev)
        pools.append(p)
    torch.cuda.synchronize()
    res = {}
    for merge in (False, True):
        got = []
        with MjpegEncoder(0, w, h, qscale=5, max_batch=n, merge=merge, timing=True) as enc:
            for s in range(7):
                enc.submit(device_ptr=pools[s % 3].data_ptr(), nframes=n)
                if enc.pending == enc.depth:
                    enc.sync()
                    got.append(enc.fetch())
            while enc.pending:
                enc.sync()
                got.append(enc.fetch())
            res[merge] = (got, enc.kernel_times()[1])
    assert res[False][1] == 7 and res[True][1] == 4  # merged: [0 1] [2 3] [4 5] [6]
    assert res[True][0] == res[False][0]


@pytest.mark.parametrize("depth", [3, 4])
def test_merge_depth_env_keeps_queue_depth(depth, monkeypatch):
    """MJG_MERGE=3 / 4 (jobs per merged launch, an A/B switch read at mjg_open): 23 ragged device
    submits in the bench's pattern (sync when enc.depth are pending) and in an eager pattern
    (sync after every second submit), never refused while fewer than enc.depth are pending (a
    full held group waiting at mjg_sync is launched by the next submit), every job's
    JPEGs byte-equal to the oracle."""
    import torch
    monkeypatch.setenv("MJG_MERGE", str(depth))
    w, h = 72, 40
    counts = [1 + (7 * j) % 3 for j in range(23)]
    frames = rand_frames(w, h, sum(counts), seed=505, kind="testsrc")
    ref = oracle_frames(frames, w, h, 4, False)
    dev_frames = torch.from_numpy(frames.copy()).to("cuda:0")
    torch.cuda.synchronize()
    offs = np.concatenate([[0], np.cumsum(counts)])
    fb = frames.shape[1]
    for eager in (False, True):
        got = []
        with MjpegEncoder(0, w, h, qscale=4, max_batch=3, merge=True) as enc:
            assert enc.depth == 2 * depth
            for j, k in enumerate(counts):
                enc.submit(device_ptr=dev_frames.data_ptr() + int(offs[j]) * fb, nframes=k)
                if enc.pending == enc.depth or (eager and j % 2 == 1):
                    enc.sync()
                    got += enc.fetch()
            while enc.pending:
                enc.sync()
                got += enc.fetch()
        assert len(got) == len(ref)
        for i in range(len(ref)):
            assert got[i] == ref[i], (depth, eager, i, first_diff(got[i], ref[i]))


@pytest.mark.parametrize("cfg", ["optimal", "scale", "scale_optimal", "default"])
def test_pipelined_submits_two_streams(cfg):
    """Every context runs its two slots on two streams (consecutive submits' launches overlap,
    csrc/api.hip alloc_slot): five submits, two queued at a time so every slot is reused on its
    own stream, from host memory (per-slot H2D staging) and with ragged batches; every frame
    byte-equal to the oracle."""
    sw, sh = 200, 120
    dw, dh = (100, 60) if cfg.startswith("scale") else (sw, sh)
    huffman = "optimal" if cfg.endswith("optimal") else "default"
    frames = rand_frames(sw, sh, 13, seed=77, kind="testsrc")
    ref = oracle_frames(frames, sw, sh, 4, False, dw, dh, huffman=huffman)
    cuts = [(0, 3), (3, 5), (5, 8), (8, 11), (11, 13)]
    got = []
    with MjpegEncoder(0, sw, sh, dw, dh, qscale=4, max_batch=3, huffman=huffman) as enc:
        for i, (a, b) in enumerate(cuts):
            enc.submit(frames[a:b])
            if i >= 1:
                enc.sync()
                got += enc.fetch()
        enc.sync()
        got += enc.fetch()
    assert len(got) == len(ref)
    for i in range(len(ref)):
        assert got[i] == ref[i], (cfg, i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


def _sweep_cases(seed=2026, n=600, wmax=420, hmax=260, nmax=3):
    """Seeded random configurations over every option of the GPU profile at once."""
    rng = np.random.default_rng(seed)
    kinds = ["noise", "smooth", "checker", "patches", "testsrc", "flat"]
    out = []
    for i in range(n):
        w, h = int(rng.integers(8, wmax + 1)), int(rng.integers(8, hmax + 1))
        chroma = ["420", "422", "444"][int(rng.integers(0, 3))]
        rst = bool(rng.integers(0, 2))
        huffman = "default" if rst else ["default", "optimal"][int(rng.integers(0, 2))]
        scale = None
        if rng.integers(0, 3) == 0:
            # downscales up to 4:1 (one k_scale LDS tile), upscales up to 2:1
            scale = (int(rng.integers(max(8, w // 4), 2 * w + 1)), int(rng.integers(max(8, h // 4), 2 * h + 1)))
        out.append(dict(w=w, h=h, q=int(rng.integers(1, 32)), full=bool(rng.integers(0, 2)),
                        kind=kinds[int(rng.integers(0, len(kinds)))], chroma=chroma, rst=rst,
                        huffman=huffman, scale=scale, n=int(rng.integers(1, nmax + 1)),
                        batch=int(rng.integers(1, 4)), seed=i))
    return out


SWEEP = _sweep_cases()
SWEEP_LARGE = _sweep_cases(seed=7, n=48, wmax=2200, hmax=1300, nmax=1)  # up to past 1080p


@pytest.mark.parametrize("part", range(12))
def test_random_sweep_matches_oracle(part):
    """600 seeded random configurations (size 8..420 x 8..260, q 1..31, tv/pc range, six
    content kinds, 4:2:0/4:2:2/4:4:4, plain/RST layout, default/optimal tables, up- and
    down-scaling, ragged batches): every frame byte-identical to the oracle."""
    _sweep(SWEEP[part::12])


@pytest.mark.parametrize("part", range(4))
def test_random_sweep_large_matches_oracle(part):
    """48 more seeded random configurations at 8..2200 x 8..1300 (one frame each)."""
    _sweep(SWEEP_LARGE[part::4])


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_random_sweep_more_seeds(seed):
    """600 more seeded random configurations per seed, as the sweep above (~3 s each)."""
    _sweep(_sweep_cases(seed=seed))


def _sweep(cases, **opts):
    for c in cases:
        w, h = c["w"], c["h"]
        dw, dh = c["scale"] or (None, None)
        frames = rand_frames(w, h, c["n"], seed=c["seed"], kind=c["kind"], chroma=c["chroma"])
        with MjpegEncoder(0, w, h, dw, dh, qscale=c["q"], full_range=c["full"], max_batch=c["batch"],
                          huffman=c["huffman"], chroma=c["chroma"], rst=c["rst"], **opts) as enc:
            got = enc.encode(frames)
        ref = oracle_frames(frames, w, h, c["q"], c["full"], dw, dh, huffman=c["huffman"],
                            chroma=c["chroma"], rst=c["rst"])
        for i in range(c["n"]):
            assert got[i] == ref[i], (c, i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


@pytest.mark.parametrize("huffman", ["default", "optimal"])
@pytest.mark.parametrize("q,full", [(1, False), (3, True), (8, False), (20, True)])
def test_wave_parallel_blocks_match_oracle(q, full, huffman):
    """k_encode's wave-parallel emission (emit_block_wave, default tables) and the counting
    pass's wave-parallel counting (count_block_wave, -huffman optimal): chunks with 1..14
    heavy blocks among flat ones -- noise of amplitudes 2..128 (dense blocks with coefficient
    63 set, and sparse ones with long zero runs, i.e. ZRLs), luma and chroma -- byte-equal to
    the oracle."""
    w, h, n = 512, 256, 2
    rng = np.random.default_rng(1000 + q)
    frames = []
    for i in range(n):
        y = np.full((h, w), 100, np.int32)
        u = np.full((h // 2, w // 2), 120, np.int32)
        v = np.full((h // 2, w // 2), 140, np.int32)
        nmcu = (w // 16) * (h // 16)
        for chunk0 in range(0, nmcu * 6, 64):  # per chunk of 64 blocks: 1..14 heavy blocks
            for _ in range(int(rng.integers(1, 15))):
                b = chunk0 + int(rng.integers(0, 64))
                m, k = divmod(b, 6)
                if m >= nmcu:
                    continue
                my, mx = divmod(m, w // 16)
                amp = int(rng.choice([2, 4, 8, 32, 128]))
                blk = rng.integers(-amp, amp + 1, (8, 8))
                if k < 4:
                    yy, xx = my * 16 + (k >> 1) * 8, mx * 16 + (k & 1) * 8
                    y[yy:yy + 8, xx:xx + 8] += blk
                else:
                    c = u if k == 4 else v
                    c[my * 8:my * 8 + 8, mx * 8:mx * 8 + 8] += blk
        frames.append(pack_i420(y.clip(0, 255).astype(np.uint8), u.clip(0, 255).astype(np.uint8),
                                v.clip(0, 255).astype(np.uint8)))
    frames = np.stack(frames)
    with MjpegEncoder(0, w, h, qscale=q, full_range=full, max_batch=n, huffman=huffman) as enc:
        got = enc.encode(frames)
    ref = oracle_frames(frames, w, h, q, full, huffman=huffman)
    for i in range(n):
        assert got[i] == ref[i], (i, len(got[i]), len(ref[i]), first_diff(got[i], ref[i]))


# ------------------------------------------- extreme blocks at the quantiser's ends
@pytest.mark.parametrize("q,full", [(1, False), (31, True)])
def test_extreme_blocks(q, full):
    """Extreme blocks for the fp32 row pass and the column screen's margins: full-swing
    checkers (row-pass outputs near 2^14), black/white blocks, noise, at the finest and
    coarsest quantiser."""
    w, h = 256, 128
    rng = np.random.default_rng(q)
    y = np.where((np.arange(w)[None, :] // 1 + np.arange(h)[:, None]) % 2, 255, 0).astype(np.uint8)
    y[:, 64:128] = rng.integers(0, 256, (h, 64))
    y[:, 128:160] = 255
    y[:, 160:192] = 0
    y[:, 192:] = np.where((np.arange(64)[None, :] // 4) % 2, 255, 0)
    u = rng.integers(0, 256, (h // 2, w // 2)).astype(np.uint8)
    v = np.where(np.arange(w // 2)[None, :] % 2, 0, 255).repeat(h // 2, 0).astype(np.uint8)
    frames = np.stack([pack_i420(y, u, v)])
    with MjpegEncoder(0, w, h, qscale=q, full_range=full, max_batch=1) as enc:
        got = enc.encode(frames)
    assert got[0] == oracle_frames(frames, w, h, q, full)[0]


# ------------------------------------------- a long -huffman optimal launch
def test_optimal_long_launch_matches_oracle():
    """120 1080p frames in one -huffman optimal launch (8 distinct testsrc2 frames, plus noise
    frames, cycled): ~92K chunks, so the counting pass's waves take several units each and flush
    their 16-bit counters every 16 chunks within a frame as well as at frame changes; every frame
    byte-equal to the oracle's encoding of its source."""
    w, h, n = 1920, 1080, 120
    src = [make_testsrc(w, h, t) for t in range(6)] + list(rand_frames(w, h, 2, seed=77, kind="noise"))
    frames = np.stack([src[i % len(src)] for i in range(n)])
    ref = oracle_frames(np.stack(src), w, h, 5, False, huffman="optimal")
    with MjpegEncoder(0, w, h, qscale=5, max_batch=n, huffman="optimal") as enc:
        got = enc.encode(frames)
    for i in range(n):
        r = ref[i % len(src)]
        assert got[i] == r, (i, len(got[i]), len(r), first_diff(got[i], r))


# ------------------------------------------- k_huff_build on given counts (mjg_debug_huff_build)
def test_huff_build_matches_oracle_tables():
    """-huffman optimal's table builder alone, on the 153 count vectors the CPU tests pin the
    oracle with (random, tie-heavy, 16-bit-limit-forcing, edge cases; those summing past int range
    scaled down): every frame's four
    BITS/HUFFVAL equal oracle.huff_optimal (ff_mjpeg_encode_huffman_close: AV_QSORT's tie order
    decides which equal-count symbols get the longer codes)."""
    import ctypes as C
    from ffmpeg_distributed_amd import _lib
    from test_huffman_optimal import count_vectors
    L = _lib.load()
    cv = []
    for c in count_vectors():
        # FFmpeg sums counts as int in package weights (<= 16 x the total): a frame's counts
        # (<= its blocks x 64, 8.3M per 4K table) keep them below 2**31; the geometric vectors
        # that would not are scaled into that domain.
        while 16 * int(c.sum()) >= 2 ** 31:
            c = np.where(c > 0, np.maximum(c >> 4, 1), 0)
        cv.append(c)
    n = len(cv)
    hist = np.zeros((n, 544), np.uint32)
    for i in range(n):
        hist[i, 0:256] = cv[i]                      # AC luma
        hist[i, 256:512] = cv[(i + 1) % n]          # AC chroma
        hist[i, 512:528] = cv[(i + 2) % n][:16]     # DC luma
        hist[i, 528:544] = cv[(i + 3) % n][16:32]   # DC chroma
    dht = np.zeros((n, 4, 272), np.uint8)
    nval = np.zeros((n, 4), np.uint32)
    rc = L.mjg_debug_huff_build(0, hist.ctypes.data_as(C.POINTER(C.c_uint32)), n,
                                dht.ctypes.data_as(C.POINTER(C.c_uint8)), nval.ctypes.data_as(C.POINTER(C.c_uint32)))
    assert rc == 0, L.mjg_last_error()
    for i in range(n):
        for t, sl in ((0, slice(512, 528)), (1, slice(528, 544)), (2, slice(0, 256)), (3, slice(256, 512))):
            c = np.zeros(256, np.uint32)
            c[:sl.stop - sl.start] = hist[i, sl]
            bits, vals = oracle.huff_optimal(c)
            k = int(nval[i, t])
            assert list(dht[i, t, :16]) == list(bits[1:17]), (i, t)
            assert k == len(vals) and list(dht[i, t, 16:16 + k]) == list(vals), (i, t)
