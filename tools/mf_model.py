#!/usr/bin/env python3
"""Numpy model of k_encode's MFMA DCT stage (kernels.hip dct_mfma, api.hip mf_fragments) with
the documented gfx950 v_mfma_f32_32x32x16_f16 operand maps, checked against exact jfdctint +
quantiser arithmetic: the u16 row image, the DC and the candidate mask (a superset of the
nonzero coefficients).  CPU only; a development check of the index algebra."""


import numpy as np
D8 = np.array([1,1,1,1,1,1,1,1, 11363,9633,6437,2260,-2260,-6437,-9633,-11363,
  10703,4433,-4433,-10703,-10703,-4433,4433,10703, 9633,-2259,-11362,-6436,6436,11362,2259,-9633,
  1,-1,-1,1,1,-1,-1,1, 6437,-11362,2261,9633,-9633,-2261,11362,-6437,
  4433,-10704,10704,-4433,-4433,10704,-10704,4433, 2260,-6436,9633,-11363,11363,-9633,6436,-2260]).reshape(8,8)
ZZ = [0,1,8,16,9,2,3,10,17,24,32,25,18,11,4,5,12,19,26,33,40,48,41,34,27,20,13,6,7,14,21,28,
      35,42,49,56,57,50,43,36,29,22,15,23,30,37,44,51,58,59,52,45,38,31,39,46,53,60,61,54,47,55,62,63]
intra = [8,16,19,22,26,27,29,34,16,16,22,24,27,29,34,37,19,22,26,27,29,34,34,38,22,22,26,27,29,34,37,40,
 22,26,27,29,32,35,40,48,26,27,29,32,35,40,48,58,26,27,29,34,38,46,56,69,27,29,35,38,46,56,69,83]
def c1(i, x): return 16*D8[i][x] if i in (0,4) else D8[i][x]
def f16up(v):
    h = np.float16(v)
    if abs(float(h)) < abs(v): h = np.nextafter(h, np.float16(np.sign(v)*np.inf))
    return h
def fragments(q):
    mp = [8 if i == 0 else min(255, (intra[i]*q) >> 3) for i in range(64)]
    qmat = [(2**22)//(16*m) for m in mp]
    f = np.zeros((12, 64, 8), np.float16)
    for l in range(64):
        m, h = l & 31, l >> 5
        for P in range(2):
            for d in range(2):
                for j in range(8):
                    rl, i = m >> 3, m & 7
                    if rl != 2*P + h: continue
                    cv = c1(i, j)
                    if i in (0,4): v = cv if d == 0 else 0
                    else:
                        hi = int(round(cv/64.0))*64  # C++ lround: half away from zero
                        hi = int(np.sign(cv)*np.floor(abs(cv)/64.0+0.5))*64
                        v = (hi if d == 0 else cv - hi)/512.0
                    f[2*P+d][l][j] = np.float16(v)
        for t in range(2):
            hz, qq = (m >> 2) & 1, (m & 3) + 4*(m >> 3)
            z = 32*hz + 31 - 16*t - qq
            nat = ZZ[z]; io, col = nat >> 3, nat & 7
            scale, up = 1.0, False
            if z:
                qm = qmat[nat]; T = ((5 << 18) + qm - 1)//qm
                dcrow = io in (0,4)
                l1 = sum(abs(D8[io][r]) for r in range(8)); l1c = sum(abs(c1(col, x)) for x in range(8))
                ex = col in (0,4)
                ymax = 16384.0 if ex else 128.0*l1c/512 + 1
                eb = 0.0 if ex else 0.502 + (ymax+1)/2048
                B = 16.0*T - 8.5 if dcrow else T*131072.0 - 65536 - 0.5
                E = l1*eb + (0 if dcrow else l1*(ymax+eb)/2048) + l1*ymax/262144
                scale = 1024.0/(B - E); up = dcrow
            for s in range(4):
                for j in range(8):
                    nd = 16*(s & 1) + 8*(j >> 2) + 4*h + (j & 3)
                    r, i = 4*(s >> 1) + (nd >> 3), nd & 7
                    if i != col: continue
                    v = D8[io][r]*scale
                    f[4+4*t+s][l][j] = f16up(v) if up else np.float16(v)
    return f, qmat
def mfma(a, b, c):  # a,b [64][8] f16, c [64][16] f32
    A = np.zeros((32,16)); B = np.zeros((16,32))
    for l in range(64):
        for j in range(8):
            A[l & 31][8*(l >> 5)+j] = float(a[l][j]); B[8*(l >> 5)+j][l & 31] = float(b[l][j])
    Dm = A @ B
    out = np.array(c, np.float64).copy()
    for l in range(64):
        for q in range(16):
            out[l][q] += Dm[(q & 3) + 8*(q >> 2) + 4*(l >> 5)][l & 31]
    return out.astype(np.float32)
kRnd = 2.0**-10; kMb = np.float32(12615680.0)
def emulate(blocks, q):  # blocks [64][8][8] uint8 (already range-converted)
    f, qmat = fragments(q)
    spk = np.zeros((32, 64), np.uint32)
    W = np.zeros((2, 64), np.uint32); DZ = np.zeros((2, 64), np.float32)
    for g in range(2):
        bp = np.zeros((4, 64, 8), np.float16)
        for s in range(4):
            for l in range(64):
                bp[s][l] = (blocks[32*g + (l & 31)][2*s + (l >> 5)].astype(np.float64) - 128).astype(np.float16)
        d = []
        for t in range(2):
            c = np.array([[0.0 if (qq & 3) == 0 else kRnd for qq in range(16)]]*64, np.float32)
            c = mfma(f[0], bp[2*t], c); c = mfma(f[1], bp[2*t], c); x16 = np.arange(64) ^ 16  # the kernel reads pattern P1 as P0 at lane l ^ 16
            assert (f[2] == f[0][x16]).all() and (f[3] == f[1][x16]).all()
            c = mfma(f[0][x16], bp[2*t+1], c); c = mfma(f[1][x16], bp[2*t+1], c)
            d.append(c)
        b2 = []
        for t in range(2):
            for l in range(64):
                for qq in range(0, 16, 2):
                    o0 = (np.float32(d[t][l][qq]) + kMb).view(np.uint32); o1 = (np.float32(d[t][l][qq+1]) + kMb).view(np.uint32)
                    r = 4*t + (qq >> 2); wi = 2*(l >> 5) + ((qq & 3) >> 1)
                    spk[r*4 + wi][32*g + (l & 31)] = (int(o0) & 0xffff) | ((int(o1) & 0xffff) << 16)
            for s in range(2):
                b2.append(np.array([[np.float16(d[t][l][8*s+j]) for j in range(8)] for l in range(64)]))
        w = np.zeros(64, np.uint64)
        for t in range(2):
            z = np.zeros((64, 16), np.float32)
            for s in range(4): z = mfma(f[4+4*t+s], b2[s], z)
            for qq in range(16):
                neg = np.float32(-z[:, qq]*z[:, qq] + 1048576.0)  # fma sign
                w = (w << np.uint64(1)) | (neg < 0).astype(np.uint64)
            if t == 1: DZ[g] = z[:, 15]
        W[g] = (w & np.uint64(0xffffffff)).astype(np.uint32)
    # swap: lane L<32 (W0[L], W0[L+32]); L>=32 (W1[L-32], W1[L])
    mask = np.zeros(64, np.uint64); dc = np.zeros(64, np.int64)
    for L in range(64):
        lo, hi = (W[0][L], W[0][L+32]) if L < 32 else (W[1][L-32], W[1][L])
        mask[L] = (np.uint64(lo) | (np.uint64(hi) << np.uint64(32))) & ~np.uint64(1)
        dz = DZ[0][L] if L < 32 else DZ[1][L-32]
        dc[L] = int(np.floor(np.float64(dz)/1024 + 128 + 2**-7 + 2**-11 + 0.5))  # RNE approx (ties impossible)
    return spk, mask, dc, qmat
def exact(blocks, qmat):
    x = blocks.astype(np.int64)
    C1 = np.array([[c1(i, xx) for xx in range(8)] for i in range(8)])
    s1 = np.einsum('ix,nrx->nri', C1, x)
    y = np.where(np.isin(np.arange(8), [0,4])[None,None,:], s1, (s1 + 256) >> 9)
    S = np.einsum('or,nrc->noc', D8, y)
    ro = np.arange(8)[:, None]
    sh = np.where((ro == 0) | (ro == 4), 4, 17)
    u = (S + (1 << (sh - 1))) >> sh
    qm = np.array(qmat).reshape(8,8)
    lvl = np.sign(u)*((np.abs(u)*qm + (3 << 18)) >> 21)
    return y, lvl
rng = np.random.default_rng(1)
for trial, q in enumerate([5, 1, 3, 31]):
    kind = trial % 2
    blocks = rng.integers(0, 256, (64, 8, 8)).astype(np.uint8) if kind else \
        np.clip(128 + rng.normal(0, 40, (64,1,1)) + rng.normal(0, 12, (64, 8, 8)), 0, 255).astype(np.uint8)
    blocks[3] = 255; blocks[4] = 0; blocks[5, :, ::2] = 255; blocks[5, :, 1::2] = 0
    spk, mask, dc, qmat = emulate(blocks, q)
    y, lvl = exact(blocks, qmat)
    yc = y.copy(); yc[:, :, 0] -= 16384
    ok_pk = all(((int(spk[r*4 + c//2][b]) >> (16*(c & 1))) & 0xffff) == yc[b][r][c] + 32768 for b in range(64) for r in range(8) for c in range(8))
    nzm = np.zeros(64, np.uint64); ncand = 0
    for b in range(64):
        for z in range(1, 64):
            if lvl[b].reshape(64)[ZZ[z]] != 0: nzm[b] |= np.uint64(1) << np.uint64(z)
        ncand += bin(int(mask[b])).count('1')
    sup = all((int(nzm[b]) & ~int(mask[b])) == 0 for b in range(64))
    ok_dc = all(dc[b] == (int(y[b][:,0].sum()) + 520)//1024 for b in range(64))
    print(f"q{q} {'noise' if kind else 'smooth'}: s_pk {ok_pk} mask superset {sup} dc {ok_dc}; nonzero {sum(bin(int(v)).count('1') for v in nzm)} cand {ncand}")
