// Bicubic resize of one plane for the `-vf scale=W:H:flags=bicubic` leg of the
// reference worker's remote_args (ffmpeg_distributed.py:134).  Applies swscale's
// fixed-point tables (sws_filter.cpp) exactly as libswscale's C path does:
//   hScale8To15_c: min((sum src*f) >> 7, 32767)            (14-bit coeffs)
//   lumRangeToJpeg_c / chrRangeToJpeg_c on that int16       (tv -> pc, if requested)
//   yuv2planeX_8_c: clip_u8(((64 << 12) + sum h*f) >> 19)  (12-bit coeffs, flat dither)
//
// One workgroup = a 64 x TH output tile (4 waves, lane = output column).  TH = 64 for the 2:1
// filters (8 h taps, 5 v pairs: 4K -> 1080p, windows of <= 36 dwords x 140 rows; the host
// checks) with the row-pair image written over the window rows it was computed from (a
// pair's two rows are read only by the wave that writes it, in program order), so the LDS of
// a 64-row tile is that of the 32-row one, and rows at a fixed 36-dword stride (pair stride
// 72: constant LDS offsets in the v-pass); TH = 32 otherwise.
//   load:   the tile's source window (rows x dword-aligned columns, rows padded to 16-byte
//           pieces) is staged in LDS from 16-byte loads, 7 rows x 9 pieces per wave-instruction,
//           all issued before any is waited on.  (Measured on MI355X, c4: a persistent
//           variant that loads the next tile's window during this tile's passes ran ~20%
//           slower -- tile index arithmetic, and 7 instead of 8 workgroups per CU -- and
//           unaligned ds_read_b64 tap reads instead of the funnel shifts ran ~2x slower.)
//   h-pass: wave w computes source row pairs p0+w, p0+w+4, ... of the window for its lane's
//           column: taps funnel-shifted out of aligned LDS dwords (v_alignbit), widened to
//           u16 pairs with v_perm and multiplied with v_dot2_i32_i16 against the column's
//           coefficient pairs (registers).  Rows 2p and 2p+1 go to LDS as one int16 pair.
//           D4 (every coefficient c = 128 ch + cl with int8 ch, cl in [-64, 64)): the window
//           is staged level-shifted (byte ^ 0x80 = p - 128 as int8) and four taps are one
//           v_dot4_i32_i8 against the hi and one against the lo bytes, no widening:
//           sum p c >> 7 = ah + (al >> 7) + sum c (exact: 128 (ah + sum c) is a multiple of 128).
//   v-pass: output row y reads the pairs [vps[y], vps[y] + npv) of its column and dot2s
//           them against that row's coefficient pairs, which the host pre-shifts by the
//           parity of the first tap row (zero-padded), so odd and even starts cost the same.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mjg {

typedef short short2_t __attribute__((ext_vector_type(2)));
typedef int v4i __attribute__((ext_vector_type(4)));

constexpr int kScaleTileW = 64;
constexpr int kScaleLoadRows = 7;  // fast window path: rows x 9 pieces per wave-instruction
__host__ __device__ constexpr int scale_loads_per_wave(int th) { return th >= 64 ? 5 : 3; }
// waves per workgroup for a tile height (128-row tiles: 8 waves, 512 threads)
__host__ __device__ constexpr int scale_waves(int th) { return th == 128 ? 8 : 4; }
constexpr int kScaleAliasWords = 36;  // TH 64: LDS row stride (dwords), the widest fast window
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef u32x4 u32x4_a1 __attribute__((aligned(1)));  // window pieces start at any byte

struct ScaleGeom {
  int sw, sh, dw, dh;            // plane sizes
  int s_stride, d_stride;
  long long s_off, d_off;        // plane offset inside a frame
  long long s_fstride, d_fstride;  // frame strides
  int nf;                        // frames per plane: blockIdx.z >= nf is the next plane (U, V in one launch)
  long long s_poff, d_poff;      // that plane's offset from this one
  int htaps, vtaps;              // htaps multiple of 4 (filterAlign 4), vtaps even
  int npv;                       // coefficient pairs per output row (vtaps/2 + 1)
  int range;                     // 0 none, 1 luma tv->pc, 2 chroma tv->pc
  int lds_pairs;                 // max row pairs any tile needs
  int lds_win_words;             // max source-window dwords any tile needs (TH 64: rows at
                                 // kScaleAliasWords, the pair image inside it)
  // the launch is a 1-D grid of gx * gy * (planes x frames) tiles; tile t -> (bx, by, z) by
  // multiply-high with ceil(2^32 / d), not by two scalar divisions (div_magic)
  int gx, gxy;
  uint32_t gx_magic, gxy_magic;  // 0 when the divisor is 1
  int mf_bx0, mf_bx1, mf_hs;     // tile columns [mf_bx0, mf_bx1) take the matrix-core h-pass
                                 // (one filter, hsum mf_hs; the host checks: api.hip)
  int mv_by0, mv_by1, mv_k;      // of those, tile rows [mv_by0, mv_by1) take the matrix-core v-pass
                                 // (one filter; mv_k = 128 * its tap sum + (64 << 12))
};

// The matrix-core v-pass's byte planes (k_scale): per output column, the h values of the tile's
// window rows as hi bytes ([col][row], this stride) and then as lo bytes ^ 0x80
constexpr int kPlaneStride = 144;  // >= the 136 window rows of a 64-row 2:1 tile, 16-byte multiple
constexpr int kMvFragOff = 512;    // words of mfb before the v-pass A fragments (3 x 64 lanes x 16 B)

// t / d for 0 <= t < 2^31: with m = ceil(2^32 / d), umulhi(t, m) is t / d or one more (the
// error t (m - 2^32/d) / 2^32 < 1), corrected by one compare; d = 1: m = 0
__device__ __forceinline__ int div_magic(int t, uint32_t magic, int d) {
  if (!magic) return t;
  const int q = (int)__umulhi((uint32_t)t, magic);
  return q * d > t ? q - 1 : q;
}

__device__ __forceinline__ int sws_range(int v, int range) {
  if (range == 1) {  // |v| < 2^15: the 24-bit multiply is exact
    v = min(v, 30189);
    return (__mul24(v, 19077) - 39057361) >> 14;
  }
  if (range == 2) {
    v = min(v, 30775);
    return (__mul24(v, 4663) - 9289992) >> 12;
  }
  return v;
}

// hScale8To15 of one source row (taps = the `htaps` bytes at byte offset `off` of an LDS
// row), then range conversion.  Bytes are fetched as aligned dwords and funnel-shifted.
template <int HT, bool D4>  // HT 0: runtime htaps
__device__ __forceinline__ int hscale_lds(const uint32_t *row, int off, const int32_t *hcp, int htaps_rt,
                                          int range, int hs) {
  const int htaps = HT ? HT : htaps_rt;
  const uint32_t *q = row + (off >> 2);
  const uint32_t sh = (uint32_t)(off & 3) * 8;
  uint32_t lo = q[0];
  if (D4) {
    int ah = 0, al = 0;
    for (int k = 0; k < htaps; k += 4) {  // (HT > 0: unrolled by the compiler)
      const uint32_t hi = q[(k >> 2) + 1];
      const int w = (int)__builtin_amdgcn_alignbit(hi, lo, sh);  // taps k..k+3, int8 p - 128
      lo = hi;
      ah = __builtin_amdgcn_sdot4(w, hcp[k >> 1], ah, false);
      al = __builtin_amdgcn_sdot4(w, hcp[(k >> 1) + 1], al, false);
    }
    return sws_range(min(ah + (al >> 7) + hs, 32767), range);
  }
  int acc = 0;
  for (int k = 0; k < htaps; k += 4) {
    const uint32_t hi = q[(k >> 2) + 1];
    const uint32_t w = __builtin_amdgcn_alignbit(hi, lo, sh);  // taps k..k+3 (bytes, LE)
    lo = hi;
    acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, __builtin_amdgcn_perm(0u, w, 0x0c010c00u)),
                                 __builtin_bit_cast(short2_t, hcp[k >> 1]), acc, false);
    acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, __builtin_amdgcn_perm(0u, w, 0x0c030c02u)),
                                 __builtin_bit_cast(short2_t, hcp[(k >> 1) + 1]), acc, false);
  }
  return sws_range(min(acc >> 7, 32767), range);
}

typedef uint32_t u32_unaligned __attribute__((aligned(1)));

// HT / NPV: compile-time tap counts for the common filters (0 = runtime, any ratio); TH: tile
// height (64 only with HT 8, NPV 5)
template <int HT, int NPV, bool D4, int RANGE, int TH>  // RANGE: g.range as a compile-time value
__global__ __launch_bounds__(64 * scale_waves(TH)) void k_scale(const SegList src,  // the submit's input frames (kernels.hip)
                                               uint8_t *__restrict__ dst, ScaleGeom g,
                                               const int32_t *__restrict__ hcp,   // [dw][htaps/2]
                                               const int32_t *__restrict__ hp,    // [dw]
                                               const int32_t *__restrict__ vcp,   // [dh][npv]
                                               const int32_t *__restrict__ vps,   // [dh] pair start
                                               const int32_t *__restrict__ hsum,  // D4: [dw] sum of taps
                                               const int32_t *__restrict__ mfb) {  // matrix-core h-pass B fragments
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  constexpr int LPW = scale_loads_per_wave(TH), NWV = scale_waves(TH), NT = 64 * NWV;
  constexpr bool ALIAS = TH >= 64;
  static_assert(!ALIAS || (HT == 8 && NPV == 5), "64/128-row tiles: 2:1 filters only");
  // wave index as a uniform value: the v-pass rows (and their filter rows) are wave-uniform
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  int t = blockIdx.x;  // the tile, raster order within a (plane, frame), then z
  if (ALIAS) {
    // XCD-contiguous tile order: workgroup i runs on XCD i % 8 (round-robin dispatch), so XCD
    // j takes the j-th eighth of the tiles in raster order and horizontally adjacent tiles --
    // whose windows share the 128-byte lines at their edges -- meet in the same L2
    const int i = t, n = gridDim.x, j = i & 7, q = n >> 3, r = n & 7;
    t = j * q + min(j, r) + (i >> 3);
  }
  const int z = div_magic(t, g.gxy_magic, g.gxy), rem = t - z * g.gxy;
  const int by = div_magic(rem, g.gx_magic, g.gx), bx = rem - by * g.gx;
  const int x0 = bx * kScaleTileW, y0 = by * TH;
  const int pl = z >= g.nf, f = z - (pl ? g.nf : 0);
  const uint8_t *s = seg_frame(src, f, g.s_fstride) + g.s_off + (pl ? g.s_poff : 0);
  uint8_t *d = dst + (size_t)f * g.d_fstride + g.d_off + (pl ? g.d_poff : 0);
  const int xe = min(x0 + kScaleTileW, g.dw), ye = min(y0 + TH, g.dh);
  const int p0 = vps[y0], p1 = vps[ye - 1] + g.npv;  // row pairs [p0, p1)
  const int nrows = 2 * (p1 - p0);
  const int npv = NPV ? NPV : g.npv;
  // source window: dwords [cb, cb + nw) of rows [2 p0, 2 p1) (rows clamped to the plane;
  // the rows past it only meet zero coefficients), staged with coalesced dword loads
  const int cb = hp[x0] & ~3;
  // +1: the funnel shift reads one past; rows padded to whole 16-byte pieces
  const int nw = ((((hp[xe - 1] + g.htaps - cb + 3) >> 2) + 1) + 3) & ~3;
  const int rs = ALIAS ? kScaleAliasWords : nw;  // LDS row stride (dwords)
  uint32_t *win = smem;                                       // [nrows][rs]
  // [p1 - p0][ps]: ALIAS, pair p over window rows 2p, 2p+1; else after the window
  const int ps = ALIAS ? 2 * rs : 64;
  uint32_t *pairs = ALIAS ? smem : smem + g.lds_win_words;
  uint32_t *vtab = smem + g.lds_win_words + g.lds_pairs * kScaleTileW;  // !ALIAS: [ye - y0][1 + npv]
  // ALIAS: wave w owns the row pairs [w ppw, (w + 1) ppw) of the window: it loads their rows
  // itself and runs their h-pass with no workgroup barrier in between (its own LDS stores and
  // loads are ordered), so the waves of a tile start computing as their own rows land
  const int np = p1 - p0, ppw = ALIAS ? (np + NWV - 1) / NWV : 0;
  const bool fast = nw <= 36 && g.sw >= 16 &&
                    (ALIAS ? 2 * ppw <= LPW * kScaleLoadRows : nrows <= NWV * LPW * kScaleLoadRows);
  const int rr = lane / 9, pc = lane - 9 * rr, col = cb + 16 * pc;  // fast loads: row, piece
  // The matrix-core h-pass (2:1 interior tiles): the window is loaded as on the VALU path, then
  // wave w computes column block w (16 output columns) of every 16-row block of the window as
  // v_mfma_i32_16x16x64_i8 products: A = 16 window rows x 64 bytes from the column block's
  // aligned byte 32 w (one ds_read_b128 per lane: lane l row l & 15, bytes 16 (l >> 4) .. +15),
  // B = the shared filter's hi / lo tap bytes on the band (host-built, the same k map), so D =
  // ah / al of hscale_lds for rows 4 (l >> 4) + i, column l & 15.  Every wave reads every row,
  // so the pairs are written over the window after a barrier.
  if (TH == 64 && D4 && HT == 8 && fast && bx >= g.mf_bx0 && bx < g.mf_bx1) {
    const int ppw2 = (p1 - p0 + NWV - 1) / NWV;  // the VALU path's row split for the loads
    u32x4 wv[LPW];
#pragma unroll
    for (int i = 0; i < LPW; i++) {
      const int r = 2 * ppw2 * wave + kScaleLoadRows * i + rr;
      const uint8_t *rp = s + (size_t)min(2 * p0 + r, g.sh - 1) * g.s_stride;
      if (col + 16 <= g.sw) {
        wv[i] = *(const u32x4_a1 *)(rp + col);
      } else {
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int cc = col + 4 * k, lc = min(cc, g.sw - 4);
          w[k] = cc < g.sw ? *(const u32_unaligned *)(rp + lc) >> ((cc - lc) * 8) : 0u;
        }
        wv[i] = u32x4{w[0], w[1], w[2], w[3]};
      }
    }
    const u32x4 bhi = ((const u32x4 *)mfb)[2 * lane], blo = ((const u32x4 *)mfb)[2 * lane + 1];
#pragma unroll
    for (int i = 0; i < LPW; i++) {
      const int r = 2 * ppw2 * wave + kScaleLoadRows * i + rr;
      if (rr < kScaleLoadRows && r < nrows && 4 * pc < nw && kScaleLoadRows * i + rr < 2 * ppw2)
        *(u32x4 *)(win + r * rs + 4 * pc) = wv[i] ^ 0x80808080u;
    }
    __syncthreads();
    const int g4 = lane >> 4, n = lane & 15;
    constexpr int kMfBlocks = 9;  // 16-row blocks: >= the 136 rows of a 64-row tile
    uint32_t pk[kMfBlocks][2];
#pragma unroll
    for (int m = 0; m < kMfBlocks; m++) {
      pk[m][0] = pk[m][1] = 0u;
      if (16 * m < nrows) {
        const int row = min(16 * m + n, nrows - 1);
        const v4i av = __builtin_bit_cast(v4i, *(const u32x4 *)(win + row * rs + 8 * wave + 4 * g4)), z = {0, 0, 0, 0};
        const v4i hi = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, __builtin_bit_cast(v4i, bhi), z, 0, 0, 0);
        const v4i lo = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, __builtin_bit_cast(v4i, blo), z, 0, 0, 0);
        int h[4];
#pragma unroll
        for (int i = 0; i < 4; i++) h[i] = sws_range(min(hi[i] + (lo[i] >> 7) + g.mf_hs, 32767), RANGE);
        pk[m][0] = ((uint32_t)h[0] & 0xffffu) | ((uint32_t)h[1] << 16);
        pk[m][1] = ((uint32_t)h[2] & 0xffffu) | ((uint32_t)h[3] << 16);
      }
    }
    __syncthreads();  // every wave's window reads done: the pairs go over the rows
    if (by >= g.mv_by0 && by < g.mv_by1) {
      // The v-pass on the matrix cores as well (interior tile rows: one v filter, pos[y] = 2y + c).
      // With h = 256 hi + lo (hi: the int16's high byte as int8; lo its low byte, stored as
      // lo ^ 0x80 = lo - 128) and each tap f = 128 fh + fl (fl in [-64, 64)):
      //   sum h f = 32768 S1 + 128 X + S4 + 128 F,  S1 = sum hi fh,  X = sum hi (2 fl) + sum lo' fh,
      //   S4 = sum lo' fl  (F = the tap sum),
      // four v_mfma_i32_16x16x64_i8 per 16 x 16 block of outputs, every product exact in i32:
      // A = 64 plane bytes (window rows 32 rb ..) of 16 columns, B = the filter's band (host-built:
      // output row n of the block reads window rows 2n + delta + j), so D's lane (n, g4) holds
      // output row n, columns 4 g4 .. 4 g4 + 3 of the block.  Each wave writes the planes of the
      // columns it computed in the h-pass, then (after a barrier) takes row block rb = wave.
      uint8_t *phi = (uint8_t *)smem, *plo = phi + 64 * kPlaneStride;
      const int colw = 16 * wave + n;
#pragma unroll
      for (int m = 0; m < kMfBlocks; m++) {
        if (16 * m < nrows) {  // (rows past nrows repeat the last one: finite, met by zero taps)
          const uint32_t hw = __builtin_amdgcn_perm(pk[m][1], pk[m][0], 0x07050301u);
          const uint32_t lw = __builtin_amdgcn_perm(pk[m][1], pk[m][0], 0x06040200u) ^ 0x80808080u;
          *(uint32_t *)(phi + colw * kPlaneStride + 16 * m + 4 * g4) = hw;
          *(uint32_t *)(plo + colw * kPlaneStride + 16 * m + 4 * g4) = lw;
        }
      }
      const u32x4 *mva = (const u32x4 *)(mfb + kMvFragOff);
      const v4i bfh = __builtin_bit_cast(v4i, mva[lane]), bfl = __builtin_bit_cast(v4i, mva[64 + lane]),
                b2fl = __builtin_bit_cast(v4i, mva[128 + lane]);
      const v4i z = {0, 0, 0, 0}, kv = {g.mv_k, g.mv_k, g.mv_k, g.mv_k};
      __syncthreads();  // every column's planes written
      uint32_t W[4];  // W[cb]: output row n, columns 16 cb + 4 g4 .. + 3 (bytes)
#pragma unroll
      for (int cb = 0; cb < 4; cb++) {
        // rows 32 wave .. 32 wave + 63 of column 16 cb + n (the last block's reads run past the
        // column into the next one: bytes met by zero taps)
        const int off = (16 * cb + n) * kPlaneStride + 32 * wave + 16 * g4;
        const v4i ah = __builtin_bit_cast(v4i, *(const u32x4 *)(phi + off));
        const v4i al = __builtin_bit_cast(v4i, *(const u32x4 *)(plo + off));
        const v4i s1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, bfh, z, 0, 0, 0);
        v4i x = __builtin_amdgcn_mfma_i32_16x16x64_i8(ah, b2fl, z, 0, 0, 0);
        x = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, bfh, x, 0, 0, 0);
        const v4i s4 = __builtin_amdgcn_mfma_i32_16x16x64_i8(al, bfl, kv, 0, 0, 0);
        uint32_t v[4];
#pragma unroll
        for (int i = 0; i < 4; i++) v[i] = (uint32_t)min(max(((s1[i] << 15) + (x[i] << 7) + s4[i]) >> 19, 0), 255);
        W[cb] = __builtin_amdgcn_perm(v[1], v[0], 0x0c0c0400u) | __builtin_amdgcn_perm(v[3], v[2], 0x04000c0cu);
      }
      // 4 x 4 transpose of (cb, g4) across lanes n, n + 16, n + 32, n + 48: then lane (n, g4)
      // holds columns 16 g4 .. 16 g4 + 15 of row n, one 16-byte store (a wave: 16 full rows)
      auto swap32 = [](uint32_t &a_, uint32_t &b_) {
        const auto r = __builtin_amdgcn_permlane32_swap(a_, b_, false, false);
        a_ = r[0];
        b_ = r[1];
      };
      auto swap16 = [](uint32_t &a_, uint32_t &b_) {
        const auto r = __builtin_amdgcn_permlane16_swap(a_, b_, false, false);
        a_ = r[0];
        b_ = r[1];
      };
      swap32(W[0], W[2]);
      swap32(W[1], W[3]);
      swap16(W[0], W[1]);
      swap16(W[2], W[3]);
      *(u32x4 *)(d + (size_t)(y0 + 16 * wave + n) * g.d_stride + x0 + 16 * g4) = u32x4{W[0], W[1], W[2], W[3]};
      return;
    }
#pragma unroll
    for (int m = 0; m < kMfBlocks; m++) {
      const int pa = 8 * m + 2 * g4;  // the pairs of D rows 4 g4 .. 4 g4 + 3 of block m
      if (pa < np) pairs[pa * ps + 16 * wave + n] = pk[m][0];
      if (pa + 1 < np) pairs[(pa + 1) * ps + 16 * wave + n] = pk[m][1];
    }
  } else {
  // Every global load of the tile is issued before any is waited on: the window rows, this
  // lane's h filter (column x), and the tile's v filter rows (one entry per thread).
  // fast path: 16-byte pieces, 7 rows of 9 pieces per wave-instruction, 3 per wave (84 rows
  // of <= 144 bytes)
  u32x4 v[LPW];
  if (fast) {
#pragma unroll
    for (int i = 0; i < LPW; i++) {
      const int r = ALIAS ? 2 * ppw * wave + kScaleLoadRows * i + rr : kScaleLoadRows * (LPW * wave + i) + rr;
      const uint8_t *rp = s + (size_t)min(2 * p0 + r, g.sh - 1) * g.s_stride;
      if (col + 16 <= g.sw) {
        v[i] = *(const u32x4_a1 *)(rp + col);
      } else {  // the piece crosses the row end: dwords loaded in-row and shifted down (bytes
                // >= sw meet no tap)
        uint32_t w[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int cc = col + 4 * k, lc = min(cc, g.sw - 4);
          w[k] = cc < g.sw ? *(const u32_unaligned *)(rp + lc) >> ((cc - lc) * 8) : 0u;
        }
        v[i] = u32x4{w[0], w[1], w[2], w[3]};
      }
    }
  }
  const int x = min(x0 + lane, g.dw - 1);  // clamped: tail lanes redo the last column
  const int32_t *hc = hcp + (size_t)x * (g.htaps >> 1);
  int32_t hreg[HT ? HT / 2 : 8];  // HT taps (or up to 16 at runtime) in registers
#pragma unroll
  for (int k = 0; k < (HT ? HT / 2 : 8); k++) hreg[k] = (2 * k < g.htaps) ? hc[k] : 0;
  const int hpx = hp[x];
  const int hs = D4 ? hsum[x] : 0;
  // v filter rows staged in LDS (ALIAS: read per output row with scalar loads instead -- the
  // row is wave-uniform -- so the tile's LDS is the window alone: 8 workgroups per CU)
  const int nvt = ALIAS ? 0 : (ye - y0) * (npv + 1);
  uint32_t vt = 0;
  int vi = tid;
  if (vi < nvt) {
    const int yy = vi / (npv + 1), k = vi - yy * (npv + 1);
    vt = k == 0 ? (uint32_t)vps[y0 + yy] : (uint32_t)vcp[(size_t)(y0 + yy) * g.npv + (k - 1)];
  }
  if (fast) {
#pragma unroll
    for (int i = 0; i < LPW; i++) {
      const int r = ALIAS ? 2 * ppw * wave + kScaleLoadRows * i + rr : kScaleLoadRows * (LPW * wave + i) + rr;
      const u32x4 w = D4 ? v[i] ^ 0x80808080u : v[i];
      // (ALIAS: only this wave's rows -- a neighbour may already have its pairs over its own)
      if (rr < kScaleLoadRows && r < nrows && 4 * pc < nw && (!ALIAS || kScaleLoadRows * i + rr < 2 * ppw))
        *(u32x4 *)(win + r * rs + 4 * pc) = w;
    }
  } else {
    for (int i = tid; i < nrows * nw; i += NT) {
      const int r = i / nw, c = i - r * nw;  // (LDS word r * rs + c)
      const uint8_t *rp = s + (size_t)min(2 * p0 + r, g.sh - 1) * g.s_stride;
      const int cc = cb + 4 * c;
      uint32_t w = 0;
      for (int bb = 0; bb < 4; bb++)
        if (cc + bb < g.sw) w |= (uint32_t)rp[cc + bb] << (8 * bb);
      win[r * rs + c] = w ^ (D4 ? 0x80808080u : 0u);
    }
  }
#pragma unroll 1
  for (; vi < nvt; vi += NT) {  // (one pass unless npv > 7)
    if (vi != tid) {
      const int yy = vi / (npv + 1), k = vi - yy * (npv + 1);
      vt = k == 0 ? (uint32_t)vps[y0 + yy] : (uint32_t)vcp[(size_t)(y0 + yy) * g.npv + (k - 1)];
    }
    vtab[vi] = vt;
  }
  const int off = hpx - cb;
  if (!(ALIAS && fast)) __syncthreads();  // (uniform: the tile's geometry)
  const int pb = ALIAS ? ppw * wave : wave, pe = ALIAS ? min(pb + ppw, np) : np, pstep = ALIAS ? 1 : NWV;
#pragma unroll 2
  for (int p = pb; p < pe; p += pstep) {
    int a, b;
    if (HT || g.htaps <= 16) {
      a = hscale_lds<HT, D4>(win + (2 * p) * rs, off, hreg, g.htaps, RANGE, hs);
      b = hscale_lds<HT, D4>(win + (2 * p + 1) * rs, off, hreg, g.htaps, RANGE, hs);
    } else {
      a = hscale_lds<0, D4>(win + (2 * p) * rs, off, hc, g.htaps, RANGE, hs);
      b = hscale_lds<0, D4>(win + (2 * p + 1) * rs, off, hc, g.htaps, RANGE, hs);
    }
    pairs[p * ps + lane] = ((uint32_t)a & 0xffffu) | ((uint32_t)b << 16);
  }
  }  // (the VALU h-pass)
  __syncthreads();
  if (x0 + lane >= g.dw) return;
  for (int y = y0 + wave; y < ye; y += NWV) {
    const uint32_t *vr = vtab + (y - y0) * (npv + 1);  // uniform address: LDS broadcast
    const int32_t *vg = vcp + (size_t)y * npv;         // ALIAS: uniform address: scalar loads
    const uint32_t *cp = pairs + ((ALIAS ? vps[y] : (int)vr[0]) - p0) * ps + lane;
    int acc = 64 << 12;
#pragma unroll
    for (int k = 0; k < npv; k++)
      acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, cp[k * ps]),
                                   __builtin_bit_cast(short2_t, ALIAS ? (uint32_t)vg[k] : vr[1 + k]), acc, false);
    d[(size_t)y * g.d_stride + x0 + lane] = (uint8_t)min(max(acc >> 19, 0), 255);
  }
}

}  // namespace mjg
