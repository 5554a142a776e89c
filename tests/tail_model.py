"""Lane-level model of k_count_ff / k_write's word fetch (csrc/kernels.hip `group_words`,
`group_values`) in numpy, for tests/test_tail_model.py: 64 lanes as arrays, ballots as bit
masks, shuffles as index gathers.  It records every slot word the kernel's loads touch, so
the CPU test checks both the words produced (against the plain concatenation of the chunks'
bits plus the 1-bit padding) and that no load leaves the words k_encode wrote.  Test
infrastructure: it restates the kernel's indexing, not FFmpeg."""
from __future__ import annotations

import numpy as np

G = 32          # kChunksPerWave
R = 4           # kTailRounds
SLOT = 3328     # kSlotWords
M32 = 0xFFFFFFFF
LANES = np.arange(64)


def _shfl(x, src):
    src = np.asarray(src)
    return x[np.clip(src, 0, 63)]


class Seg:
    """One entropy-coded segment: chunk bit lengths and their slot words (bits MSB first)."""

    def __init__(self, lengths, rng):
        self.L = np.asarray(lengths, np.int64)
        self.n = len(self.L)
        self.O = np.concatenate([[0], np.cumsum(self.L)[:-1]]).astype(np.int64)
        self.T = int(self.L.sum())
        self.slots = np.zeros((self.n + 1) * SLOT, np.uint64)  # one spare slot past the end
        self.bits = []
        for c, L in enumerate(self.L):
            b = rng.integers(0, 2, int(L), dtype=np.uint8)
            self.bits.append(b)
            nw = (int(L) + 31) // 32
            pad = np.zeros(nw * 32, np.uint8)
            pad[:L] = b
            words = np.packbits(pad).view(">u4").astype(np.uint64)
            self.slots[c * SLOT:c * SLOT + nw] = words
        self.touched = []

    def expected_words(self):
        b = np.concatenate(self.bits) if self.bits else np.zeros(0, np.uint8)
        nbytes = (self.T + 7) // 8
        allb = np.ones(nbytes * 8, np.uint8)  # padding 1s
        allb[:self.T] = b
        nw = (len(allb) + 31) // 32
        full = np.zeros(nw * 32, np.uint8)
        full[:len(allb)] = allb
        return np.packbits(full).view(">u4").astype(np.uint64)

    def load(self, idx, mask):
        idx = np.asarray(idx, np.int64)
        for i in idx[mask]:
            c, w = divmod(int(i), SLOT)
            ok = c < self.n and w < (int(self.L[c]) + 31) // 32
            self.touched.append((c, w, ok))
        return np.where(mask, self.slots[np.clip(idx, 0, len(self.slots) - 1)], 0).astype(np.uint64)


def group_words(seg: Seg, gi: int):
    c0 = gi * G
    n = min(G, seg.n - c0)
    O = np.zeros(64, np.int64)
    L = np.zeros(64, np.int64)
    O[:n] = seg.O[c0:c0 + n]
    L[:n] = seg.L[c0:c0 + n]
    end = O + L
    k0 = (int(O[0]) + 31) >> 5
    k1 = (int(end[n - 1]) + 31) >> 5
    sw = (O + 31) >> 5
    lw = (end + 31) >> 5
    rem = end - 32 * (lw - 1)
    has_next = (c0 + LANES + 1 < seg.n).astype(np.int64)
    info = np.zeros(64, np.int64)
    j = LANES < n
    info[j] = ((sw - k0) | ((32 * sw - O) << 17) | ((rem - 1) << 22) | (has_next << 27))[j]
    info[n] = k1 - k0
    assert np.all((sw - k0)[j] < (1 << 17))
    return dict(c0=c0, n=n, info=info, k0=k0, k1=k1, T=seg.T)


def group_values(seg: Seg, g, kb):
    span = 64 * R
    n, k0, k1 = g["n"], g["k0"], g["k1"]
    rsw = g["info"] & 0x1FFFF
    wk = kb - k0
    ch = (LANES >= 1) & (LANES < n)
    marks = np.zeros(span, bool)
    mk = ch & (rsw >= wk) & (rsw < wk + span)
    marks[rsw[mk] - wk] = True
    base = int(np.sum(ch & (rsw < wk)))
    own = []
    for i in range(R):
        m = marks[64 * i:64 * i + 64]
        own.append(base + np.cumsum(m))
        base += int(m.sum())
    out = []
    for i in range(R):
        r = wk + 64 * i + LANES
        valid = r < k1 - k0
        c = np.where(valid, own[i], 0)
        inf = _shfl(g["info"], c)
        nsw = _shfl(g["info"], c + 1) & 0x1FFFF
        wi = np.where(valid, r - (inf & 0x1FFFF), 0)
        assert np.all(wi >= 0), "negative slot word"
        off = (inf >> 17) & 31
        rem = ((inf >> 22) & 31) + 1
        bnd = valid & (r + 1 == nsw)
        own_nx = valid & ((LANES == 63) | (r + 1 == k1 - k0))
        has_next = ((inf >> 27) & 1) == 1
        slot = (g["c0"] + c) * SLOT
        A = seg.load(slot + wi, np.ones(64, bool))
        X = seg.load(slot + wi + 1, bnd & (off != 0) & (rem > 32 - off))
        bmask = own_nx & (~bnd | ((rem < 32) & has_next))
        B = seg.load(np.where(bnd, slot + SLOT, slot + wi + 1), bmask)
        k = kb + 64 * i + LANES
        nx = np.append(A[1:], np.uint64(0))
        nxt = np.where(own_nx, B, nx).astype(np.uint64)
        lo = np.where(off != 0, np.where(bnd, X, nxt), A).astype(np.uint64)
        sh = ((32 - off) & 31).astype(np.uint64)
        w = (((A << np.uint64(32)) | lo) >> sh) & M32
        remc = np.clip(rem, 0, 31).astype(np.uint64)
        w = np.where(bnd & (rem < 32), w | (nxt >> remc), w)
        endk = g["T"] - 32 * k
        pad = (8 - (g["T"] & 7)) & 7
        e = np.clip(endk, 0, 31).astype(np.uint64)
        ep = np.clip(endk + pad, 0, 32)
        tailmask = np.where(ep >= 32, 0, np.uint64(M32) >> np.clip(ep, 0, 31).astype(np.uint64))
        w = np.where((endk >= 0) & (endk < 32), w | ((np.uint64(M32) >> e) & ~tailmask & M32), w)
        out.append((k, valid, w.astype(np.uint64)))
    return out


def segment_words(seg: Seg):
    """The words every group of the segment produces, in order (k, value)."""
    gps = (seg.n + G - 1) // G
    got = {}
    for gi in range(gps):
        g = group_words(seg, gi)
        for kb in range(g["k0"], g["k1"], 64 * R):
            for k, valid, w in group_values(seg, g, kb):
                for kk, vv, ww in zip(k[valid], valid[valid], w[valid]):
                    assert int(kk) not in got, "word produced twice"
                    got[int(kk)] = int(ww)
    return got
