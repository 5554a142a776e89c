"""-huffman optimal (FFmpeg's default Huffman mode for mjpeg): CPU checks of the oracle's
restatement of libavcodec/mjpegenc_huffman.c (ff_mjpegenc_huffman_compute_bits,
ff_mjpeg_encode_huffman_close) and libavutil/qsort.h (AV_QSORT).

FFmpeg is absent on this pool (parity unpinned against it).  What is
pinned here:
  - a second, independent transcription (Python, below) of the same published algorithm
    gives identical BITS/HUFFVAL for random, tie-heavy and edge-case count vectors,
  - every table is a complete-or-valid prefix code with lengths <= 16 whose total cost
    equals the length-limited optimum (an independent package-merge cost),
  - optimal-mode JPEGs decode (libjpeg-turbo via Pillow) to exactly the pixels of the
    default-mode JPEGs (only the entropy coding differs) and are never larger.
"""
import io

import numpy as np
import pytest
from PIL import Image

import oracle
from ffmpeg_distributed_amd.encoder import split_i420
from ffmpeg_distributed_amd.testsrc import testsrc2_i420 as make_testsrc


def av_qsort(a, cmp):
    """libavutil/qsort.h AV_QSORT, transcribed independently of oracle/mjpeg_oracle.c."""
    n = len(a)
    stack = [(0, n - 1)]
    while stack:
        start, end = stack.pop()
        while start < end:
            if start < end - 1:
                checksort = False
                right, left = end - 2, start + 1
                mid = start + ((end - start) >> 1)
                if cmp(a[start], a[end]) > 0:
                    if cmp(a[end], a[mid]) > 0:
                        a[start], a[mid] = a[mid], a[start]
                    else:
                        a[start], a[end] = a[end], a[start]
                else:
                    if cmp(a[start], a[mid]) > 0:
                        a[start], a[mid] = a[mid], a[start]
                    else:
                        checksort = True
                if cmp(a[mid], a[end]) > 0:
                    a[mid], a[end] = a[end], a[mid]
                    checksort = False
                if start == end - 2:
                    break
                a[end - 1], a[mid] = a[mid], a[end - 1]
                while left <= right:
                    while left <= right and cmp(a[left], a[end - 1]) < 0:
                        left += 1
                    while left <= right and cmp(a[right], a[end - 1]) > 0:
                        right -= 1
                    if left <= right:
                        a[left], a[right] = a[right], a[left]
                        left += 1
                        right -= 1
                a[end - 1], a[left] = a[left], a[end - 1]
                if checksort and (mid == left - 1 or mid == left):
                    mid = start
                    while mid < end and cmp(a[mid], a[mid + 1]) <= 0:
                        mid += 1
                    if mid == end:
                        break
                if end - left < left - start:
                    stack.append((start, right))
                    start = left + 1
                else:
                    stack.append((left + 1, end))
                    end = right
            else:
                if cmp(a[start], a[end]) > 0:
                    a[start], a[end] = a[end], a[start]
                break


def huff_close(counts, max_length=16):
    """ff_mjpeg_encode_huffman_close + ff_mjpegenc_huffman_compute_bits (item lists)."""
    pt = [[v, int(c)] for v, c in enumerate(counts) if c] + [[256, 0]]
    nval = len(pt) - 1
    av_qsort(pt, lambda x, y: x[1] - y[1])
    frm = []  # list of (probability, items)
    i = 0
    for times in range(max_length + 1):
        to = []
        j = 0
        if times < max_length:
            i = 0
        while i < len(pt) or j + 1 < len(frm):
            if i < len(pt) and (j + 1 >= len(frm) or pt[i][1] < frm[j][0] + frm[j + 1][0]):
                to.append((pt[i][1], [pt[i][0]]))
                i += 1
            else:
                to.append((frm[j][0] + frm[j + 1][0], frm[j][1] + frm[j + 1][1]))
                j += 2
        frm = to
    m = min(len(pt) - 1, len(frm))
    nbits = [0] * 257
    for _, items in frm[:m]:
        for it in items:
            nbits[it] += 1
    dist = [[s, nbits[s]] for s in range(256) if nbits[s] > 0]
    av_qsort(dist, lambda x, y: (x[0] - y[0]) if x[1] == y[1] else (x[1] - y[1]))
    bits = [0] * 17
    for _, ln in dist:
        bits[ln] += 1
    return bits, [s for s, _ in dist][:nval]


def optimal_cost(counts, L=16):
    """Minimum total bits of a prefix code with lengths <= L over the symbols plus one
    zero-weight symbol (FFmpeg's dummy 256, which keeps the all-ones code unused):
    the textbook package-merge cost, independent of tie order."""
    w = sorted([int(c) for c in counts if c] + [0])
    cur = list(w)
    for _ in range(L - 1):
        pk = [cur[k] + cur[k + 1] for k in range(0, len(cur) - 1, 2)]
        cur = sorted(w + pk)
    return sum(cur[: 2 * (len(w) - 1)])


def lengths_of(bits, vals):
    ln, k = {}, 0
    for L in range(1, 17):
        for _ in range(bits[L]):
            ln[int(vals[k])] = L
            k += 1
    return ln


def count_vectors():
    rng = np.random.default_rng(7)
    out = []
    for it in range(150):
        c = np.zeros(256, np.int64)
        nsym = int(rng.integers(1, 200))
        idx = rng.choice(256, nsym, replace=False)
        kind = it % 3
        if kind == 0:
            c[idx] = rng.integers(1, 100000, nsym)
        elif kind == 1:  # heavy ties
            c[idx] = rng.integers(1, 4, nsym)
        else:  # geometric: forces the 16-bit limit
            c[idx] = (2.0 ** rng.integers(0, 30, nsym)).astype(np.int64)
        out.append(c)
    dc = np.zeros(256, np.int64)
    dc[:12] = [5000, 3000, 2500, 900, 400, 100, 30, 8, 2, 1, 1, 1]
    out += [dc, np.eye(256, dtype=np.int64)[0] * 7, np.zeros(256, np.int64)]
    return out


def test_oracle_tables_equal_independent_transcription():
    for c in count_vectors():
        bits, vals = oracle.huff_optimal(c)
        rb, rv = huff_close(c)
        assert list(bits) == rb and list(vals) == rv


def test_tables_are_length_limited_optimal_prefix_codes():
    for c in count_vectors():
        bits, vals = oracle.huff_optimal(c)
        nz = [s for s in range(256) if c[s]]
        assert sorted(int(v) for v in vals) == nz
        assert bits[0] == 0 and max((L for L in range(17) if bits[L]), default=0) <= 16
        assert sum(int(bits[L]) * 2.0 ** -L for L in range(1, 17)) < 1.0  # all-ones code reserved
        ln = lengths_of(bits, vals)
        if len(nz) >= 2:
            assert sum(int(c[s]) * ln[s] for s in nz) == optimal_cost(c)


@pytest.mark.parametrize("w,h,q,full", [(352, 288, 5, False), (72, 40, 2, True), (101, 57, 31, False),
                                        (640, 360, 3, True)])
def test_optimal_jpeg_decodes_to_default_pixels(w, h, q, full):
    f = make_testsrc(w, h, 5, full_range=full)
    y, u, v = split_i420(f, w, h)
    a = oracle.encode_frame(y, u, v, full_range=full, qscale=q)
    b = oracle.encode_frame(y, u, v, full_range=full, qscale=q, huffman="optimal")
    assert len(b) <= len(a)
    ia = np.asarray(Image.open(io.BytesIO(a)).convert("YCbCr"))
    ib = np.asarray(Image.open(io.BytesIO(b)).convert("YCbCr"))
    assert (ia == ib).all()
