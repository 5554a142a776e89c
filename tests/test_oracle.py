"""CPU tests of the oracle (oracle/mjpeg_oracle.c) and of the library's device-free host
logic.  The oracle restates FFmpeg's mjpeg encoder / swscale; FFmpeg itself is absent on
this pool, so these pin what can be pinned independently:
  - Annex K Huffman tables against libjpeg-turbo's standard tables (via Pillow),
  - bitstream validity + quality by decoding with Pillow (libjpeg-turbo),
  - known-answer properties of the FDCT / quantiser / stuffing / header,
  - the folded tv->pc range formulas the kernel uses, exhaustively,
  - the library's host-side header and swscale filter tables == the oracle's.
"""
import io

import numpy as np
import pytest
from PIL import Image

import oracle
from ffmpeg_distributed_amd import _lib
from ffmpeg_distributed_amd.encoder import pack_i420, split_i420
from ffmpeg_distributed_amd.testsrc import testsrc2_i420 as make_testsrc

ZIGZAG = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48,
          41, 34, 27, 20, 13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15,
          23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]
MPEG1 = [8, 16, 19, 22, 26, 27, 29, 34, 16, 16, 22, 24, 27, 29, 34, 37, 19, 22, 26, 27, 29,
         34, 34, 38, 22, 22, 26, 27, 29, 34, 37, 40, 22, 26, 27, 29, 32, 35, 40, 48, 26, 27,
         29, 32, 35, 40, 48, 58, 26, 27, 29, 34, 38, 46, 56, 69, 27, 29, 35, 38, 46, 56, 69, 83]


def segments(jpg: bytes):
    """(marker, payload) list up to SOS, then ('scan', bytes up to EOI)."""
    assert jpg[:2] == b"\xff\xd8"
    out, i = [], 2
    while True:
        assert jpg[i] == 0xFF
        m = jpg[i + 1]
        ln = (jpg[i + 2] << 8) | jpg[i + 3]
        out.append((m, jpg[i + 4: i + 2 + ln]))
        i += 2 + ln
        if m == 0xDA:
            break
    assert jpg[-2:] == b"\xff\xd9"
    out.append(("scan", jpg[i:-2]))
    return out


def float_dct8x(block):
    """8 x orthonormal 2-D DCT-II (what jfdctint approximates)."""
    n = np.arange(8)
    c = np.cos((2 * n[None, :] + 1) * n[:, None] * np.pi / 16)
    a = np.where(n == 0, 1 / np.sqrt(2), 1.0)[:, None] * c / 2
    return 8 * (a @ block.astype(float) @ a.T)


def smooth_frame(w, h, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    y = (128 + 80 * np.sin(xx / 6) * np.cos(yy / 9) + rng.normal(0, 2, (h, w))).clip(0, 255)
    cw, ch = (w + 1) // 2, (h + 1) // 2
    cy, cx = np.mgrid[0:ch, 0:cw]
    u = (128 + 40 * np.sin(cx / 5)).clip(0, 255) + 0 * cy
    v = (128 + 40 * np.cos(cy / 4)).clip(0, 255) + 0 * cx
    return y.astype(np.uint8), u.astype(np.uint8), v.astype(np.uint8)


# ----------------------------------------------------------------------------- FDCT
def test_fdct_constant_block_is_dc_only():
    for val in (0, 1, 77, 128, 255):
        out = oracle.fdct(np.full(64, val, np.int16))
        assert out[0] == 64 * val
        assert not out[1:].any()


def test_fdct_dc_is_exact_pixel_sum():
    rng = np.random.default_rng(1)
    for _ in range(200):
        b = rng.integers(0, 256, 64)
        assert oracle.fdct(b)[0] == b.sum()


def test_fdct_tracks_float_dct():
    rng = np.random.default_rng(2)
    for _ in range(200):
        b = rng.integers(0, 256, (8, 8))
        got = oracle.fdct(b.reshape(-1)).reshape(8, 8)
        assert np.abs(got - float_dct8x(b)).max() <= 2.0


# ------------------------------------------------------------------------ quantiser
def test_qscale_mapping():
    # mpegvideo_enc.c update_qscale: lambda = q*118, (lambda*139 + 8192) >> 14, clip [2,31]
    assert [oracle.effective_qscale(q) for q in (1, 2, 3, 5, 31, 40)] == [2, 2, 3, 5, 31, 31]


@pytest.mark.parametrize("q", [2, 3, 5, 13, 31])
def test_matrix_formula(q):
    m, qm = oracle.matrix(q)
    assert m[0] == 8
    for i in range(1, 64):
        assert m[i] == min(255, (MPEG1[i] * q) >> 3)
        assert qm[i] == (1 << 22) // (16 * int(m[i]))


def test_quantize_known_answer():
    coefs = np.zeros(64, np.int16)
    coefs[0] = 64 * 100 + 31      # DC: (c + 32) / 64 -> 100
    coefs[1] = 100                # |c| * qmat: qm[1] = 2^18 / 10 at q=5
    coefs[8] = -100
    coefs[63] = 3                 # rounds to zero
    out, last = oracle.quantize(coefs, 5)
    _, qm = oracle.matrix(5)
    expect = (100 * int(qm[1]) + (3 << 18)) >> 21
    assert out[0] == 100 and out[1] == expect and out[8] == -((100 * int(qm[8]) + (3 << 18)) >> 21)
    assert out[63] == 0
    assert last == ZIGZAG.index(8) if out[8] else ZIGZAG.index(1)


def test_ac_magnitude_bound_keeps_clip_coeffs_inactive():
    # the kernel drops clip_coeffs: |q| stays far below 1023 for 8-bit input
    worst = 0
    rng = np.random.default_rng(3)
    for _ in range(300):
        b = np.where(rng.random(64) < 0.5, 0, 255).astype(np.int16)
        out, _ = oracle.quantize(oracle.fdct(b), 2)
        worst = max(worst, int(np.abs(out[1:]).max()))
    assert worst < 512


# --------------------------------------------------------------------- Huffman / header
def pillow_dht_tables():
    """Standard (Annex K) tables as libjpeg-turbo writes them (optimize=False)."""
    buf = io.BytesIO()
    Image.new("YCbCr", (16, 16)).save(buf, "JPEG", quality=90, optimize=False, subsampling=2)
    tabs = {}
    for m, p in segments(buf.getvalue())[:-1]:
        if m != 0xC4:
            continue
        i = 0
        while i < len(p):
            tc_th = p[i]
            bits = list(p[i + 1: i + 17])
            n = sum(bits)
            tabs[tc_th] = (bits, list(p[i + 17: i + 17 + n]))
            i += 17 + n
    return tabs


def test_huffman_tables_match_libjpeg_standard_tables():
    std = pillow_dht_tables()
    hdr = oracle.header(64, 48, 5)
    dht = [p for m, p in segments(hdr + b"\xff\xd9")[:-1] if m == 0xC4]
    assert len(dht) == 1       # FFmpeg writes one DHT with four tables
    p, i, order = dht[0], 0, []
    while i < len(p):
        tc_th = p[i]
        bits = list(p[i + 1: i + 17])
        n = sum(bits)
        assert (bits, list(p[i + 17: i + 17 + n])) == std[tc_th]
        order.append(tc_th)
        i += 17 + n
    assert order == [0x00, 0x01, 0x10, 0x11]   # DC0, DC1, AC0, AC1


def test_huffman_codes_are_canonical_prefix_codes():
    for tid in range(4):
        size, code = oracle.huff_table(tid)
        syms = [s for s in range(256) if size[s]]
        words = sorted(format(int(code[s]), f"0{int(size[s])}b") for s in syms)
        for a, b in zip(words, words[1:]):
            assert not b.startswith(a)
        assert not any(set(w) == {"1"} for w in words)   # no all-ones code


@pytest.mark.parametrize("q,sar", [(5, (1, 1)), (2, (0, 0)), (31, (16, 11))])
def test_header_layout(q, sar):
    hdr = oracle.header(1920, 1080, q, sar=sar)
    segs = segments(hdr + b"\xff\xd9")
    markers = [m for m, _ in segs]
    expect = ([0xE0] if sar[0] else []) + [0xDB, 0xC4, 0xC0, 0xDA, "scan"]
    assert markers == expect
    d = dict(segs[:-1])
    if sar[0]:
        assert d[0xE0] == b"JFIF\x00\x01\x02\x00" + bytes([sar[0] >> 8, sar[0] & 255,
                                                             sar[1] >> 8, sar[1] & 255, 0, 0])
    m, _ = oracle.matrix(q)
    assert d[0xDB] == bytes([0] + [int(m[ZIGZAG[i]]) for i in range(64)])
    assert d[0xC0] == bytes([8, 1080 >> 8, 1080 & 255, 1920 >> 8, 1920 & 255, 3,
                             1, 0x22, 0, 2, 0x11, 0, 3, 0x11, 0])
    assert d[0xDA] == bytes([3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 63, 0])


def test_library_header_equals_oracle():
    for (w, h, q, sar) in [(1920, 1080, 5, (1, 1)), (72, 40, 2, (0, 0)), (3840, 2160, 31, (4, 3))]:
        assert _lib.build_header(w, h, q, sar) == oracle.header(w, h, q, sar=sar)
        assert _lib.build_header(w, h, q, sar, com_itu601=True) == \
            oracle.header(w, h, q, sar=sar, com_itu601=True)


# -------------------------------------------------------------------- full frames
@pytest.mark.parametrize("w,h,q", [(64, 48, 2), (72, 40, 5), (101, 57, 3), (16, 16, 31)])
def test_oracle_jpeg_decodes_with_libjpeg(w, h, q):
    y, u, v = smooth_frame(w, h)
    j = oracle.encode_planes(y, u, v, q)
    im = Image.open(io.BytesIO(j))
    im.draft("YCbCr", None)
    im.load()
    assert im.size == (w, h)
    got = np.asarray(im.convert("YCbCr"))[..., 0].astype(float)
    psnr = 10 * np.log10(255 ** 2 / np.mean((got - y) ** 2))
    assert psnr > {2: 40, 3: 38, 5: 35, 31: 22}[q]


def test_stuffing_every_ff_in_scan_is_followed_by_zero():
    rng = np.random.default_rng(7)
    w, h = 128, 64
    y = rng.integers(0, 256, (h, w), dtype=np.uint8)
    u = rng.integers(0, 256, (h // 2, w // 2), dtype=np.uint8)
    j = oracle.encode_planes(y, u, u[::-1].copy(), 2)
    scan = segments(j)[-1][1]
    ff = [i for i in range(len(scan)) if scan[i] == 0xFF]
    assert ff, "noise at q=2 should produce 0xFF bytes in the scan"
    assert all(i + 1 < len(scan) and scan[i + 1] == 0 for i in ff)
    Image.open(io.BytesIO(j)).load()


def test_coefficients_roundtrip_through_frame_coeffs():
    y, u, v = smooth_frame(72, 40, 3)
    coef, last = oracle.frame_coeffs(y, u, v, 5)
    assert coef.shape == (5 * 3 * 6, 64)
    # block 0 of MCU 0 is the top-left luma block: its DC is round(mean)
    assert coef[0, 0] == (int(y[:8, :8].astype(int).sum()) + 32) // 64
    for b in range(coef.shape[0]):
        nz = [k for k in range(1, 64) if coef[b, ZIGZAG[k]] != 0]
        assert last[b] == (nz[-1] if nz else 0)


# ------------------------------------------------------------------------- swscale
def test_folded_range_formulas_exhaustive():
    p = np.arange(256, dtype=np.int64)
    lum = np.clip((2441856 * p - 38008785) >> 21, 0, 255)
    chrm = np.clip((596864 * p - 9027848) >> 19, 0, 255)
    src = p.astype(np.uint8).reshape(1, 256).repeat(2, 0)
    assert (oracle.scale_plane(src, 256, 2, 1)[0] == lum).all()
    assert (oracle.scale_plane(src, 256, 2, 2, chroma=True)[0] == chrm).all()
    # classic swscale constants, restated
    v = np.minimum(p << 7, 30189)
    assert (np.clip((((v * 19077 - 39057361) >> 14) + 64) >> 7, 0, 255) == lum).all()


@pytest.mark.parametrize("src,dst,one,align", [(3840, 1920, 1 << 14, 4), (2160, 1080, 1 << 12, 2),
                                               (1920, 960, 1 << 14, 4), (100, 64, 1 << 14, 4),
                                               (48, 70, 1 << 12, 2), (1080, 1080, 1 << 12, 2)])
def test_sws_filter_properties_and_library_agreement(src, dst, one, align):
    f, pos = oracle.sws_filter(src, dst, one, align)
    assert (f.sum(1) == one).all()
    assert (pos >= 0).all() and (pos + f.shape[1] <= src).all()
    assert (np.diff(pos) >= 0).all()
    lf, lp = _lib.sws_filter(src, dst, one, align)
    assert (lf == f).all() and (lp == pos).all()
    if src == dst:
        assert f.shape[1] == 1 and (pos == np.arange(dst)).all()


def test_oracle_scaled_frame_decodes():
    fr = make_testsrc(320, 180, 3)
    y, u, v = split_i420(fr, 320, 180)
    j = oracle.encode_frame(y, u, v, dst_w=160, dst_h=90, qscale=3)
    im = Image.open(io.BytesIO(j))
    im.load()
    assert im.size == (160, 90)


def test_pack_split_roundtrip():
    fr = make_testsrc(101, 57, 2)
    assert (pack_i420(*split_i420(fr, 101, 57)) == fr).all()


# ------------------------------------------------ 4:2:2 / 4:4:4 and the RST layout
SHIFTS = {"420": (1, 1), "422": (1, 0), "444": (0, 0)}


def smooth_planes(w, h, chroma, seed=0):
    hs, vs = SHIFTS[chroma]
    cw, ch = (w + hs) >> hs, (h + vs) >> vs
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    y = (128 + 80 * np.sin(xx / 6) * np.cos(yy / 9) + rng.normal(0, 2, (h, w))).clip(0, 255)
    cy, cx = np.mgrid[0:ch, 0:cw]
    u = (128 + 40 * np.sin(cx / 5) + 20 * np.cos(cy / 7)).clip(0, 255)
    v = (128 + 40 * np.cos(cy / 4) - 15 * np.sin(cx / 3)).clip(0, 255)
    return y.astype(np.uint8), u.astype(np.uint8), v.astype(np.uint8)


@pytest.mark.parametrize("chroma,sof", [("420", (0x22, 0x11, 0x11)), ("422", (0x22, 0x12, 0x12)),
                                        ("444", (0x12, 0x12, 0x12))])
@pytest.mark.parametrize("rst", [False, True])
def test_header_sampling_and_dri(chroma, sof, rst):
    """SOF0 factors follow ff_mjpeg_init_hvsample (4:4:4 is 1x2 for every component); DRI
    (slice threading) sits between DQT and DHT with interval = MCUs per MCU row."""
    w, h = 101, 57
    segs = segments(oracle.header(w, h, 5, chroma=chroma, rst=rst) + b"\xff\xd9")
    markers = [m for m, _ in segs]
    assert markers == [0xE0, 0xDB] + ([0xDD] if rst else []) + [0xC4, 0xC0, 0xDA, "scan"]
    d = dict(segs[:-1])
    assert d[0xC0][6:] == bytes([1, sof[0], 0, 2, sof[1], 0, 3, sof[2], 0])
    if rst:
        mcw, _ = oracle.mcu_grid(w, h, chroma)
        assert d[0xDD] == bytes([mcw >> 8, mcw & 255]) and mcw == -(-w // (8 if chroma == "444" else 16))
    assert _lib.build_header(w, h, 5, (1, 1), chroma=chroma, rst=rst) == \
        oracle.header(w, h, 5, chroma=chroma, rst=rst)


def test_luma_blocks_do_not_depend_on_chroma_format():
    """The luma blocks of a 4:2:2 frame are the 4:2:0 ones; 4:4:4 codes each 16x16 macroblock
    as two 8x16 MCUs (left: Y TL, Y BL; right: Y TR, Y BR)."""
    w, h = 48, 32
    y, u, v = smooth_planes(w, h, "420", 1)
    c420, _ = oracle.frame_coeffs(y, u, v, 4, "420")
    y2, u2, v2 = smooth_planes(w, h, "422", 1)
    c422, _ = oracle.frame_coeffs(y, u2, v2, 4, "422")
    y4, u4, v4 = smooth_planes(w, h, "444", 1)
    c444, _ = oracle.frame_coeffs(y, u4, v4, 4, "444")
    lum420 = c420.reshape(-1, 6, 64)[:, :4]
    np.testing.assert_array_equal(c422.reshape(-1, 8, 64)[:, :4], lum420)
    l444 = c444.reshape(-1, 2, 6, 64)[:, :, :2]          # [MB, left/right MCU, Y top/bottom]
    np.testing.assert_array_equal(l444[:, 0, 0], lum420[:, 0])
    np.testing.assert_array_equal(l444[:, 0, 1], lum420[:, 2])
    np.testing.assert_array_equal(l444[:, 1, 0], lum420[:, 1])
    np.testing.assert_array_equal(l444[:, 1, 1], lum420[:, 3])
    # chroma: 4:2:2 Cb top / Cb bottom of MCU 0 are the first two 8x8 blocks of the Cb column
    assert c422[4, 0] == (int(u2[:8, :8].astype(int).sum()) + 32) // 64
    assert c422[5, 0] == (int(u2[8:16, :8].astype(int).sum()) + 32) // 64
    assert c422[6, 0] == (int(v2[:8, :8].astype(int).sum()) + 32) // 64


@pytest.mark.parametrize("chroma", ["420", "422", "444"])
@pytest.mark.parametrize("w,h", [(72, 40), (101, 57), (64, 48), (8, 8), (200, 130)])
def test_chroma_formats_and_rst_decode(chroma, w, h):
    """Each format decodes with libjpeg to the expected sampling at high PSNR; the RST
    layout decodes to exactly the same pixels (same coefficients, rows as restart
    intervals), carries RST0..7 cyclically after every MCU row but the last, and every
    restart interval is byte aligned with its 0xFF bytes stuffed."""
    y, u, v = smooth_planes(w, h, chroma, 2)
    plain = oracle.encode_frame(y, u, v, full_range=True, qscale=3, chroma=chroma)
    rst = oracle.encode_frame(y, u, v, full_range=True, qscale=3, chroma=chroma, rst=True)
    a, b = Image.open(io.BytesIO(plain)), Image.open(io.BytesIO(rst))
    a.load()
    b.load()
    hv = {"420": ((2, 2), (1, 1)), "422": ((2, 2), (1, 2)), "444": ((1, 2), (1, 2))}[chroma]
    assert a.layer == [(1, *hv[0], 0), (2, *hv[1], 0), (3, *hv[1], 0)]
    np.testing.assert_array_equal(np.asarray(a), np.asarray(b))
    got = np.asarray(a.convert("YCbCr"))[..., 0].astype(float)
    assert 10 * np.log10(255 ** 2 / np.mean((got - y) ** 2)) > 30
    _, mch = oracle.mcu_grid(w, h, chroma)
    scan = segments(rst)[-1][1]
    marks = [scan[i + 1] for i in range(len(scan) - 1) if scan[i] == 0xFF and scan[i + 1] != 0]
    assert marks == [0xD0 + (r & 7) for r in range(mch - 1)]
    if mch == 1:
        assert rst == plain                      # one MCU row: no DRI, no RST


def test_rst_restarts_dc_prediction():
    """A flat frame: every MCU row after the first restarts its DC predictors at 128, so with
    RST every row codes the same bits (plain mode codes DC differences of 0 after row 0)."""
    w, h = 64, 64
    y = np.full((h, w), 200, np.uint8)
    u = np.full((h // 2, w // 2), 90, np.uint8)
    j = oracle.encode_frame(y, u, u.copy(), full_range=True, qscale=5, rst=True)
    scan = segments(j)[-1][1]
    rows, cur = [], bytearray()
    i = 0
    while i < len(scan):
        if scan[i] == 0xFF and 0xD0 <= scan[i + 1] <= 0xD7:
            rows.append(bytes(cur))
            cur = bytearray()
            i += 2
            continue
        cur.append(scan[i])
        i += 1
    rows.append(bytes(cur))
    assert len(rows) == 4 and len(set(rows)) == 1


def test_rst_and_optimal_are_exclusive():
    y, u, v = smooth_planes(32, 32, "420")
    with pytest.raises(RuntimeError):
        oracle.encode_frame(y, u, v, full_range=True, huffman="optimal", rst=True)


@pytest.mark.parametrize("chroma", ["422", "444"])
def test_tv_range_and_scale_for_422_444(chroma):
    """yuv422p/yuv444p (tv) input: swscale's per-plane path with the format's chroma plane
    sizes and siting; the frame decodes and scaled frames keep the sampling."""
    w, h, dw, dh = 96, 64, 48, 40
    y, u, v = smooth_planes(w, h, chroma, 5)
    j = oracle.encode_frame(y, u, v, dst_w=dw, dst_h=dh, full_range=False, qscale=3, chroma=chroma)
    im = Image.open(io.BytesIO(j))
    im.load()
    assert im.size == (dw, dh)
    j2 = oracle.encode_frame(y, u, v, full_range=False, qscale=3, chroma=chroma)
    im2 = Image.open(io.BytesIO(j2))
    im2.load()
    got = np.asarray(im2.convert("YCbCr"))[..., 0].astype(float)
    ref = np.clip((y.astype(float) - 16) * 255 / 219, 0, 255)     # tv -> pc luma
    assert 10 * np.log10(255 ** 2 / np.mean((got - ref) ** 2)) > 30


def test_oracle_is_thread_safe():
    """The parity tests run the oracle on a thread pool (ctypes releases the GIL): concurrent
    calls, -huffman optimal included, equal the serial results."""
    from concurrent.futures import ThreadPoolExecutor
    from ffmpeg_distributed_amd.testsrc import testsrc2_i420
    from ffmpeg_distributed_amd.encoder import split_i420
    w, h = 200, 120
    frames = [split_i420(testsrc2_i420(w, h, t), w, h) for t in range(16)]
    args = [dict(huffman="optimal", qscale=3), dict(huffman="default", qscale=5, dst_w=130, dst_h=70)]
    for kw in args:
        serial = [oracle.encode_frame(*f, **kw) for f in frames]
        with ThreadPoolExecutor(8) as ex:
            for _ in range(3):
                assert list(ex.map(lambda f: oracle.encode_frame(*f, **kw), frames)) == serial
