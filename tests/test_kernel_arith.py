"""CPU proofs for the fp32 exact-integer arithmetic of k_encode (csrc/kernels.hip).

The kernel carries jfdctint's integer pass 1 in fp32 mantissas and uses fp32 only as a
*screen* in pass 2 (exact values come from integer dot products).  These tests restate
those steps in numpy (fp32 FMA = exact float64 product-sum rounded once to fp32) and pin
them against the C oracle's FDCT (oracle/mjpeg_oracle.c, a restatement of FFmpeg's
jfdctint_template.c) and swscale's range converters:
  - the fp32 tv->pc range conversion equals the integer formula for all 256 inputs,
  - the fp32 row pass equals jfdctint pass 1 for random and extreme rows,
  - kPass2Dot/kPass2Add (pass 2 as one dot product per output row) equal the oracle FDCT,
  - the screening thresholds never drop a coefficient that quantises to nonzero.
Constants are parsed from the kernel source so the test cannot drift from it.
"""
import os
import re

import numpy as np
import pytest

import oracle

SRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "ffmpeg_distributed_amd", "csrc", "kernels.hip")
M = np.float32(12582912.0)
MC = np.float32(12599296.0)  # kMc = kM + 16384
BIAS = np.array([0] + [16384] * 7, np.int64)  # the row image's bias per row-pass output
RND = np.float32(2.0 ** -10)


def _src():
    with open(SRC) as f:
        return f.read()


def _int_array(name):
    src = _src().replace("\\\n", "\n")  # join macro continuation lines
    m = re.search(name + r"\[\d+\]\s*=\s*\{([^}]*)\}", src)
    if m is None:  # initialised from a macro: `kName[N] = MACRO;` and `#define MACRO {...}`
        macro = re.search(name + r"\[\d+\]\s*=\s*(\w+)\s*;", src).group(1)
        m = re.search(r"#define\s+" + macro + r"\s*\{([^}]*)\}", src)
    body = m.group(1)
    return [int(eval(x)) for x in body.replace("\n", " ").split(",") if x.strip()]


def fma32(a, b, c):
    """fp32 fused multiply-add: exact in float64 for these magnitudes, one rounding."""
    return (np.float64(np.float32(a)) * np.float64(np.float32(b)) + np.float64(np.float32(c))).astype(np.float32)


def range_int(p, chroma):
    if chroma:
        return np.clip((p * 2387456 - 36111392) >> 21, 0, 255)
    return np.clip((p * 2441856 - 38008785) >> 21, 0, 255)


def range_f32(p, chroma):
    """k_encode's [RC] pixel: the LDS table byte range(p) OR'ed into the mantissa of
    M = 1.5 * 2^23, i.e. the fp32 value M + range(p)."""
    byte = range_int(p, chroma).astype(np.uint32)
    return (np.uint32(0x4B400000) | byte).view(np.float32)


@pytest.mark.parametrize("chroma", [False, True])
def test_range_lut_in_mantissa_exhaustive(chroma):
    """The table (range_luma / range_chroma in kernels.hip) OR'ed into M's mantissa is the
    fp32 value M + range(p) for all 256 inputs, and range() is swscale's tv->pc converter."""
    p = np.arange(256, dtype=np.int64)
    got = (range_f32(p, chroma).astype(np.float64) - float(M)).astype(np.int64)
    assert (got == range_int(p, chroma)).all()
    src = _src()
    a, b, sh = (596864, 9027848, 19) if chroma else (2441856, 38008785, 21)
    assert f"__mul24(p, {a}) - {b}) >> {sh}" in src
    assert (np.clip((p * a - b) >> sh, 0, 255) == range_int(p, chroma)).all()


def pass1_int(p):
    """jfdctint pass 1 (CONST_BITS 13, PASS1_BITS 4) on rows of 8, int64."""
    D = lambda x, n: (x + (1 << (n - 1))) >> n
    p = p.astype(np.int64)
    t0, t7 = p[:, 0] + p[:, 7], p[:, 0] - p[:, 7]
    t1, t6 = p[:, 1] + p[:, 6], p[:, 1] - p[:, 6]
    t2, t5 = p[:, 2] + p[:, 5], p[:, 2] - p[:, 5]
    t3, t4 = p[:, 3] + p[:, 4], p[:, 3] - p[:, 4]
    t10, t13, t11, t12 = t0 + t3, t0 - t3, t1 + t2, t1 - t2
    o = np.zeros_like(p)
    o[:, 0] = (t10 + t11) * 16
    o[:, 4] = (t10 - t11) * 16
    z1 = (t12 + t13) * 4433
    o[:, 2] = D(z1 + t13 * 6270, 9)
    o[:, 6] = D(z1 - t12 * 15137, 9)
    z1, z2, z3, z4 = t4 + t7, t5 + t6, t4 + t6, t5 + t7
    z5 = (z3 + z4) * 9633
    t4, t5, t6, t7 = t4 * 2446, t5 * 16819, t6 * 25172, t7 * 12299
    z1, z2, z3, z4 = z1 * -7373, z2 * -20995, z3 * -16069 + z5, z4 * -3196 + z5
    o[:, 7] = D(t4 + z1 + z3, 9)
    o[:, 5] = D(t5 + z2 + z4, 9)
    o[:, 3] = D(t6 + z2 + z3, 9)
    o[:, 1] = D(t7 + z1 + z4, 9)
    return o


def pass1_f32(p, rc_chroma=None):
    """The kernel's fp32 row pass; returns the u16 image values (value + BIAS[output])."""
    f = lambda a: np.asarray(a, np.float32)
    if rc_chroma is None:
        x = [f(p[:, i]) for i in range(8)]
        t0, t1, t2, t3 = (f(x[0] + x[7]), f(x[1] + x[6]), f(x[2] + x[5]), f(x[3] + x[4]))
    else:
        x = [range_f32(p[:, i].astype(np.int64), rc_chroma) for i in range(8)]
        t0 = f(f(x[0] - f(2 * M)) + x[7])
        t1 = f(f(x[1] - f(2 * M)) + x[6])
        t2 = f(f(x[2] - f(2 * M)) + x[5])
        t3 = f(f(x[3] - f(2 * M)) + x[4])
    t7, t6, t5, t4 = f(x[0] - x[7]), f(x[1] - x[6]), f(x[2] - x[5]), f(x[3] - x[4])
    t10, t13, t11, t12 = f(t0 + t3), f(t0 - t3), f(t1 + t2), f(t1 - t2)
    c = lambda v: np.float32(v / 512)
    o = [None] * 8
    o[0] = fma32(f(t10 + t11), 16.0, M)
    o[4] = fma32(f(t10 - t11), 16.0, MC)
    o[2] = f(fma32(t13, c(10703), fma32(t12, c(4433), RND)) + MC)
    o[6] = f(fma32(t13, c(4433), fma32(t12, c(-10704), RND)) + MC)
    odd = {1: (2260, 6437, 9633, 11363), 3: (-6436, -11362, -2259, 9633),
           5: (9633, 2261, -11362, 6437), 7: (-11363, 9633, -6436, 2260)}
    for k, (c4, c5, c6, c7) in odd.items():
        a = fma32(t4, c(c4), RND)
        a = fma32(t5, c(c5), a)
        a = fma32(t6, c(c6), a)
        a = fma32(t7, c(c7), a)
        o[k] = f(a + MC)
    bits = np.stack([v.view(np.uint32) for v in o], 1)
    return (bits & 0xFFFF).astype(np.int64)


def _rows(rng, n):
    r = rng.integers(0, 256, (n, 8))
    r[: n // 4] = rng.choice([0, 255], (n // 4, 8))  # extremes stress the magnitudes
    r[n // 4: n // 4 + 2] = [[0, 255] * 4, [255, 0] * 4]
    return r


def test_fp32_row_pass_equals_jfdctint_pass1():
    rng = np.random.default_rng(1)
    p = _rows(rng, 200000)
    img = pass1_f32(p)
    assert (img - BIAS == pass1_int(p)).all()
    assert ((img >= 0) & (img < 32768)).all()  # reads as the same value in int16 (exact_coef)


@pytest.mark.parametrize("chroma", [False, True])
def test_fp32_row_pass_with_range_convert(chroma):
    rng = np.random.default_rng(2 + chroma)
    p = _rows(rng, 100000)
    ref = pass1_int(range_int(p.astype(np.int64), chroma))
    assert (pass1_f32(p, rc_chroma=chroma) - BIAS == ref).all()


def test_pass2_dot_rows_equal_oracle_fdct():
    dot = np.array(_int_array("kPass2Dot"), np.int64).reshape(8, 8)
    add = np.array([8, 1 << 16, 1 << 16, 1 << 16, 8, 1 << 16, 1 << 16, 1 << 16], np.int64)
    sh = np.array([4, 17, 17, 17, 4, 17, 17, 17])
    rng = np.random.default_rng(3)
    for it in range(300):
        blk = rng.integers(0, 256, (8, 8)) if it % 3 else rng.choice([0, 255], (8, 8))
        ref = oracle.fdct(blk.astype(np.int16)).reshape(8, 8).astype(np.int64)
        img = pass1_f32(blk) - BIAS  # rows -> row-pass values, [row][col]
        for c in range(8):
            col = img[:, c]
            acc = (dot @ col + add).astype(np.int64)
            acc = ((acc + 2 ** 31) % 2 ** 32) - 2 ** 31  # int32 wraparound, as on the GPU
            assert ((acc >> sh) == ref[:, c]).all(), (it, c)


def test_pass2_scaled_dc_rows_equal_oracle_fdct():
    """exact_coef as k_encode runs it: s_m2 rows 0 and 4 scaled by kPass2DcScale, the biased
    u16 image read as int16, the accumulator started at 2^16 (2^16 + kRow0Bias for row 0,
    columns 1-7), int32 wraparound, descaled by 17 -- equal to the oracle FDCT, and the true
    accumulator never leaves int32 (extreme blocks)."""
    scale = int(re.search(r"constexpr int kPass2DcScale = (\d+);", _src()).group(1))
    row0 = int(re.search(r"constexpr uint32_t kRow0Bias = (0x[0-9A-Fa-f]+)u;", _src()).group(1), 16)
    row0 -= 1 << 32
    dot = np.array(_int_array("kPass2Dot"), np.int64).reshape(8, 8)
    dot[[0, 4]] *= scale
    start = np.full((8, 8), 1 << 16, np.int64)
    start[0, 1:] += row0
    rng = np.random.default_rng(5)
    blocks = [np.full((8, 8), 255), np.zeros((8, 8), np.int64)]
    blocks += [rng.choice([0, 255], (8, 8)) for _ in range(100)] + [rng.integers(0, 256, (8, 8)) for _ in range(200)]
    for blk in blocks:
        ref = oracle.fdct(blk.astype(np.int16)).reshape(8, 8).astype(np.int64)
        img = pass1_f32(blk)
        true = dot @ (img - BIAS) + (1 << 16)
        assert (np.abs(true) < 2 ** 31).all()
        acc = dot @ img + start
        acc = ((acc + 2 ** 31) % 2 ** 32) - 2 ** 31  # int32 wraparound, as on the GPU
        assert (acc == true).all()
        assert ((acc >> 17) == ref).all()


def test_screen_thresholds_are_conservative():
    """Every coefficient that quantises to nonzero passes the fp32 screen (q = 1..31)."""
    dot = np.array(_int_array("kPass2Dot"), np.int64).reshape(8, 8)
    rng = np.random.default_rng(4)
    blocks = rng.integers(0, 256, (400, 8, 8))
    blocks[:100] = rng.choice([0, 255], (100, 8, 8))
    for q in (1, 2, 5, 13, 31):
        qm = oracle.matrix(q)[1].astype(np.int64)  # natural order
        T = ((5 << 18) + qm - 1) // qm
        for blk in blocks:
            img = pass1_f32(blk)
            coefs = oracle.quantize(oracle.fdct(blk.astype(np.int16)), q)[0].reshape(8, 8)
            for c in range(8):
                s_exact = dot @ (img[:, c] - BIAS[c])
                for r in range(8):
                    n = r * 8 + c
                    if n == 0 or coefs[r, c] == 0:
                        continue
                    B = 16.0 * T[n] - 8.5 if r in (0, 4) else T[n] * 131072.0 - 65536.0 - 2048.0
                    # the kernel's fp32 sum differs from s_exact by < 2^9 (see kernels.hip)
                    slack = 0 if r in (0, 4) else 512  # rows 0/4 are exact in fp32
                    assert abs(s_exact[r]) - slack > B, (q, n, s_exact[r], B)


def _skip_limits(q, col):
    """Python restatement of open_ctx's k_encode column-skip limits (Rmax, A) for a column."""
    dot = np.array(_int_array("kPass2Dot"), np.int64).reshape(8, 8)
    qm = oracle.matrix(q)[1].astype(np.int64)
    rmax, amax = 65535, 0
    for ro in range(8):
        T = ((5 << 18) + qm[ro * 8 + col] - 1) // qm[ro * 8 + col]
        if ro == 0:
            amax = max(0, 2 * T - 2)
        elif ro == 4:
            rmax = min(rmax, 4 * T - 3)
        else:
            rmax = min(rmax, (2 * (T * 131072 - 65536 - 1)) // int(np.abs(dot[ro]).sum()))
    return max(0, rmax), amax


@pytest.mark.parametrize("q", [1, 2, 3, 5, 8, 13, 31])
def test_column_skip_limits_are_sound(q):
    """A column whose row-pass values satisfy k_encode's skip test (max - min <= Rmax,
    |u| <= A) has every pass-2 output quantising to zero: checked on the extreme columns
    (values at the box corners with the sign pattern of each output row) and random ones."""
    dot = np.array(_int_array("kPass2Dot"), np.int64).reshape(8, 8)
    add = np.array([8, 1 << 16, 1 << 16, 1 << 16, 8, 1 << 16, 1 << 16, 1 << 16], np.int64)
    sh = np.array([4, 17, 17, 17, 4, 17, 17, 17])
    qm = oracle.matrix(q)[1].astype(np.int64)
    rng = np.random.default_rng(q)
    for col in range(2, 8):
        rmax, a = _skip_limits(q, col)
        r = min(rmax, 2 * a)
        T = ((5 << 18) + qm[np.arange(8) * 8 + col] - 1) // qm[np.arange(8) * 8 + col]
        cols = []
        for k in range(8):
            s = dot[k] > 0
            for lo in (-a, a - r, (a - r - a) // 2):
                cols += [lo + r * s, lo + r * ~s]
        cols += list(rng.integers(-a, a + 1, (200, 8)))
        for u in cols:
            u = np.asarray(u, np.int64)
            assert u.max() - u.min() <= rmax and np.abs(u).max() <= a
            v = (dot @ u + add) >> sh
            assert (np.abs(v) < T).all(), (q, col, u, v, T)
        # and the limits are not vacuous at typical quality
        if q <= 8:
            assert rmax > 0 and a > 0
