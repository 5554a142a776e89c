#pragma once
// gfx950 kernels of the MJPEG segment encoder (see include/mjgpu.h for the boundary).
//
// Pipeline per submit (B frames, one launch per stage, all on the ctx stream):
//   k_scale       [only with -vf scale] bicubic hscale -> tv->pc range -> vscale, LDS-staged
//   k_encode      one workgroup = one chunk of 64 MCUs (384 blocks, one 8x8 block per
//                 thread): coalesced 8-byte row loads with edge replication, [tv->pc range],
//                 integer jfdctint, quantiser, zigzag, DC prediction through LDS,
//                 Huffman bit-length pass -> wave prefix-sum -> bit-pack pass into an
//                 LDS window (ds_or_b32) -> chunk bitstream to a scratch slot
//   k_scan_bits   per frame: exclusive scan of chunk bit lengths
//   k_count_ff    per chunk: realign its bits to the frame offset, pad with 1s, count 0xFF
//   k_scan_ff     per frame: exclusive scan of 0xFF counts -> stuffed frame size
//   k_write       per chunk: header / stuffed scan bytes / EOI into the packed output
//
// Arithmetic follows FFmpeg (see oracle/mjpeg_oracle.c for the per-function citations):
// libavcodec/jfdctint_template.c, mpegvideo_enc.c dct_quantize_c, mjpegenc.c
// encode_block, mjpegenc_common.c escape/stuffing; libswscale hscale/range/vscale.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jpeg_tables.h"

namespace mjg {

constexpr int kMcuPerChunk = 64;
constexpr int kEncThreads = 6 * 64;  // 6 blocks per MCU x 64 MCUs, one block per thread
constexpr int kWinWords = 4096;      // LDS bit-pack window (16 KiB)
constexpr int kMaxBlockBits = 1664;  // >= DC 16 + 63 * (16 + 10) bits
constexpr int kSlotWords = (kMcuPerChunk * 6 * kMaxBlockBits + 31) / 32;

struct EncGeom {
  int w, h;            // encoded size
  int cw, ch;          // chroma plane size
  int mbw, nmcu, nchunks;
  int y_stride, c_stride;
  long long frame_stride, u_off, v_off;
  int range_convert;   // 1: yuv420p (tv) input without scale -> swscale tv->pc per pixel
  int debug_coefs;
};

struct QuantTab {
  int32_t qmat[64];  // natural order, floor(2^18 / m'[i])
};

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ int range_luma(int p) {
  // hScale8To15 (1 tap, 1<<14) -> lumRangeToJpeg_c -> yuv2plane1_8_c (flat 64 dither)
  int v = min(p << 7, 30189);
  v = (v * 19077 - 39057361) >> 14;
  v = (v + 64) >> 7;
  return min(max(v, 0), 255);
}
__device__ __forceinline__ int range_chroma(int p) {
  int v = min(p << 7, 30775);
  v = (v * 4663 - 9289992) >> 12;
  v = (v + 64) >> 7;
  return min(max(v, 0), 255);
}

#define MJG_DESCALE(x, n) (((x) + (1 << ((n) - 1))) >> (n))

// One 8-point jfdctint butterfly on p[0], p[S], ... p[7S] (CONST_BITS 13, PASS1_BITS 4).
// ROW: pass 1 (d0/d4 << 4, others descale 9); !ROW: pass 2 (descale 4 / 17).  Every
// stored value fits int16 for 8-bit input, so FFmpeg's int16 stores are identities here.
template <int S, bool ROW>
__device__ __forceinline__ void fdct8(int *p) {
  int t0 = p[0 * S] + p[7 * S], t7 = p[0 * S] - p[7 * S];
  int t1 = p[1 * S] + p[6 * S], t6 = p[1 * S] - p[6 * S];
  int t2 = p[2 * S] + p[5 * S], t5 = p[2 * S] - p[5 * S];
  int t3 = p[3 * S] + p[4 * S], t4 = p[3 * S] - p[4 * S];
  const int t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
  constexpr int SH = ROW ? 9 : 17;
  if (ROW) {
    p[0 * S] = (t10 + t11) * 16;
    p[4 * S] = (t10 - t11) * 16;
  } else {
    p[0 * S] = MJG_DESCALE(t10 + t11, 4);
    p[4 * S] = MJG_DESCALE(t10 - t11, 4);
  }
  int z1 = (t12 + t13) * 4433;
  p[2 * S] = MJG_DESCALE(z1 + t13 * 6270, SH);
  p[6 * S] = MJG_DESCALE(z1 - t12 * 15137, SH);
  z1 = t4 + t7;
  int z2 = t5 + t6, z3 = t4 + t6, z4 = t5 + t7;
  const int z5 = (z3 + z4) * 9633;
  t4 *= 2446;
  t5 *= 16819;
  t6 *= 25172;
  t7 *= 12299;
  z1 *= -7373;
  z2 *= -20995;
  z3 *= -16069;
  z4 *= -3196;
  z3 += z5;
  z4 += z5;
  p[7 * S] = MJG_DESCALE(t4 + z1 + z3, SH);
  p[5 * S] = MJG_DESCALE(t5 + z2 + z4, SH);
  p[3 * S] = MJG_DESCALE(t6 + z2 + z3, SH);
  p[1 * S] = MJG_DESCALE(t7 + z1 + z4, SH);
}

__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    uint32_t t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Load an 8x8 block at (x0, y0) of a plane with coordinate clamping (FFmpeg
// emulated_edge_mc / draw_edges replicate the last row/column).
template <int CHROMA>
__device__ __forceinline__ void load_block(int (&c)[64], const uint8_t *plane, int stride, int pw,
                                           int ph, int x0, int y0, int rc) {
  const uint8_t *base = plane + (size_t)y0 * stride + x0;
  const bool fast = (x0 + 8 <= pw) && (y0 + 8 <= ph) &&
                    ((((uintptr_t)base) | (uintptr_t)stride) & 7) == 0;
  if (fast) {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const uint64_t v = __builtin_nontemporal_load((const uint64_t *)(base + (size_t)r * stride));
#pragma unroll
      for (int b = 0; b < 8; b++) c[r * 8 + b] = (int)((v >> (8 * b)) & 255u);
    }
  } else {
#pragma unroll
    for (int r = 0; r < 8; r++) {
      const int sy = min(y0 + r, ph - 1);
#pragma unroll
      for (int b = 0; b < 8; b++) {
        const int sx = min(x0 + b, pw - 1);
        c[r * 8 + b] = plane[(size_t)sy * stride + sx];
      }
    }
  }
  if (rc) {
#pragma unroll
    for (int i = 0; i < 64; i++) c[i] = CHROMA ? range_chroma(c[i]) : range_luma(c[i]);
  }
}

struct BitSink {
  uint64_t acc;
  int nacc;        // bits held in acc (< 32 between emits)
  uint32_t widx;   // chunk-relative index of the word being filled
  uint32_t wbase;  // first word of the LDS window
  uint32_t *win;
  __device__ __forceinline__ void put(uint32_t w) {
    const uint32_t i = widx - wbase;
    if (i < (uint32_t)kWinWords) atomicOr(&win[i], w);
    widx++;
  }
  __device__ __forceinline__ void emit(uint32_t v, int n) {
    acc = (acc << n) | v;
    nacc += n;
    if (nacc >= 32) {
      nacc -= 32;
      put((uint32_t)(acc >> nacc));
    }
  }
  __device__ __forceinline__ void finish() {
    if (nacc > 0) put((uint32_t)(acc << (32 - nacc)));
  }
};

// Huffman coding of one block, FFmpeg mjpegenc.c encode_block / ff_mjpeg_encode_dc.
// EMIT=false returns the bit length only.
template <bool EMIT>
__device__ __forceinline__ uint32_t code_block(const int (&qz)[64], int diff, const uint32_t *ac,
                                               const uint32_t *dc, BitSink *sink) {
  uint32_t bits;
  {
    const int a = diff < 0 ? -diff : diff;
    const int cat = diff == 0 ? 0 : 32 - __clz(a);
    const uint32_t e = dc[cat];
    bits = (e >> 16) + cat;
    if (EMIT) {
      const uint32_t mant = (uint32_t)(diff < 0 ? diff - 1 : diff) & ((1u << cat) - 1u);
      sink->emit(((e & 0xffffu) << cat) | mant, (int)bits);
    }
  }
  const uint32_t zrl = ac[0xf0];
  int prev = 0;
#pragma unroll
  for (int k = 1; k < 64; k++) {
    const int v = qz[k];
    if (v != 0) {
      int run = k - prev - 1;
      const int a = v < 0 ? -v : v;
      const int cat = 32 - __clz(a);
      const uint32_t e = ac[((run & 15) << 4) | cat];
      const int len = (int)(e >> 16) + cat;
      if (EMIT) {
        while (run >= 16) {
          sink->emit(zrl & 0xffffu, (int)(zrl >> 16));
          run -= 16;
        }
        const uint32_t mant = (uint32_t)(v < 0 ? v - 1 : v) & ((1u << cat) - 1u);
        sink->emit(((e & 0xffffu) << cat) | mant, len);
      } else {
        bits += (uint32_t)(run >> 4) * (zrl >> 16);
      }
      bits += len;
      prev = k;
    }
  }
  if (prev != 63) {
    const uint32_t eob = ac[0];
    bits += eob >> 16;
    if (EMIT) sink->emit(eob & 0xffffu, (int)(eob >> 16));
  }
  return bits;
}

// ------------------------------------------------------------------ k_encode
// grid (nchunks, nframes), 384 threads.  Thread roles inside a chunk of 64 MCUs:
//   waves 0,1: Y0/Y1 (top luma row) of MCUs 0-31 / 32-63, lanes interleave Y0,Y1
//   waves 2,3: Y2/Y3 (bottom luma row), same interleave
//   wave 4: Cb, wave 5: Cr of MCU = lane
// so every wave's 8-byte row loads cover 512 contiguous bytes.
__global__ __launch_bounds__(kEncThreads) void k_encode(
    const uint8_t *__restrict__ frames, EncGeom g, QuantTab qt, const uint32_t *__restrict__ tabs,
    uint32_t *__restrict__ scratch, uint32_t *__restrict__ chunk_bits,
    int16_t *__restrict__ dbg_coefs) {
  __shared__ uint32_t s_ac[512];
  __shared__ uint32_t s_dc[32];
  __shared__ int s_dcq[kEncThreads];
  __shared__ int s_pred[4];
  __shared__ uint32_t s_off[kEncThreads];
  __shared__ uint32_t s_total;
  __shared__ uint32_t s_win[kWinWords];

  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int chunk = blockIdx.x, frame = blockIdx.y;
  const uint8_t *fr = frames + (size_t)frame * g.frame_stride;

  for (int i = tid; i < 512; i += kEncThreads) s_ac[i] = tabs[i];
  if (tid < 32) s_dc[tid] = tabs[512 + tid];

  // Predecessor DCs (Y3, Cb, Cr of the MCU before this chunk): the quantised DC of a
  // block is (pixel sum + 32) >> 6 because the FDCT's DC output is the exact sum.
  if (wave < 3) {
    int dc = 128;
    if (chunk > 0) {
      const int m = chunk * kMcuPerChunk - 1;
      const int mx = m % g.mbw, my = m / g.mbw;
      const int px = lane & 7, py = lane >> 3;
      int v;
      if (wave == 0) {
        const int sx = min(mx * 16 + 8 + px, g.w - 1), sy = min(my * 16 + 8 + py, g.h - 1);
        v = fr[(size_t)sy * g.y_stride + sx];
        if (g.range_convert) v = range_luma(v);
      } else {
        const uint8_t *pl = fr + (wave == 1 ? g.u_off : g.v_off);
        const int sx = min(mx * 8 + px, g.cw - 1), sy = min(my * 8 + py, g.ch - 1);
        v = pl[(size_t)sy * g.c_stride + sx];
        if (g.range_convert) v = range_chroma(v);
      }
      dc = (wave_sum(v) + 32) >> 6;
    }
    if (lane == 0) s_pred[wave] = dc;
  }

  int local_mcu, blk;
  if (wave < 4) {
    local_mcu = 32 * (wave & 1) + (lane >> 1);
    blk = ((wave >> 1) << 1) | (lane & 1);
  } else {
    local_mcu = lane;
    blk = wave;
  }
  const int mcu = chunk * kMcuPerChunk + local_mcu;
  const bool active = mcu < g.nmcu;
  const int tab = blk < 4 ? 0 : 1;

  int qz[64];
  int dc = 0;
  if (active) {
    const int mx = mcu % g.mbw, my = mcu / g.mbw;
    int c[64];
    if (blk < 4) {
      load_block<0>(c, fr, g.y_stride, g.w, g.h, mx * 16 + (blk & 1) * 8, my * 16 + (blk >> 1) * 8,
                    g.range_convert);
    } else {
      load_block<1>(c, fr + (blk == 4 ? g.u_off : g.v_off), g.c_stride, g.cw, g.ch, mx * 8, my * 8,
                    g.range_convert);
    }
#pragma unroll
    for (int r = 0; r < 8; r++) fdct8<1, true>(c + r * 8);
#pragma unroll
    for (int col = 0; col < 8; col++) fdct8<8, false>(c + col);

    // dct_quantize_c (intra, MJPEG): DC (c+32)/64; AC (|c|*qmat + 3<<18) >> 21, sign
    // restored, clip_coeffs to +-1023.
    dc = (c[0] + 32) >> 6;
    qz[0] = dc;
#pragma unroll
    for (int k = 1; k < 64; k++) {
      const int j = kZigzag[k];
      const int level = c[j] * qt.qmat[j];
      const int a = level < 0 ? -level : level;
      const int q = min((a + (3 << 18)) >> 21, 1023);
      qz[k] = level < 0 ? -q : q;
    }
    if (g.debug_coefs) {
      int16_t *o = dbg_coefs + (((size_t)frame * g.nmcu + mcu) * 6 + blk) * 64;
#pragma unroll
      for (int k = 0; k < 64; k++) o[kZigzag[k]] = (int16_t)qz[k];
    }
  } else {
#pragma unroll
    for (int k = 0; k < 64; k++) qz[k] = 0;
  }
  s_dcq[local_mcu * 6 + blk] = dc;
  __syncthreads();

  // DC predictor: previous block of the same component in MCU order (FFmpeg last_dc,
  // reset to 128 at the start of the frame).
  int pred;
  if (blk == 0)
    pred = local_mcu == 0 ? s_pred[0] : s_dcq[(local_mcu - 1) * 6 + 3];
  else if (blk < 4)
    pred = s_dcq[local_mcu * 6 + blk - 1];
  else
    pred = local_mcu == 0 ? s_pred[blk - 3] : s_dcq[(local_mcu - 1) * 6 + blk];
  const int diff = dc - pred;

  const uint32_t *ac = s_ac + tab * 256;
  const uint32_t *dct = s_dc + tab * 16;
  const uint32_t nbits = active ? code_block<false>(qz, diff, ac, dct, nullptr) : 0u;
  s_off[local_mcu * 6 + blk] = nbits;
  __syncthreads();

  // Exclusive scan of the 384 block lengths in MCU order (wave 0: 6 per lane).
  if (wave == 0) {
    uint32_t v[6], sum = 0;
#pragma unroll
    for (int i = 0; i < 6; i++) {
      v[i] = s_off[lane * 6 + i];
      sum += v[i];
    }
    const uint32_t incl = wave_incl_scan(sum, lane);
    uint32_t e = incl - sum;
#pragma unroll
    for (int i = 0; i < 6; i++) {
      s_off[lane * 6 + i] = e;
      e += v[i];
    }
    if (lane == 63) s_total = incl;
  }
  __syncthreads();
  const uint32_t off = s_off[local_mcu * 6 + blk];
  const uint32_t total = s_total;
  const uint32_t nwords = (total + 31) >> 5;
  uint32_t *slot = scratch + ((size_t)frame * g.nchunks + chunk) * kSlotWords;

  for (uint32_t wbase = 0; wbase < nwords; wbase += kWinWords) {
    for (int i = tid; i < kWinWords; i += kEncThreads) s_win[i] = 0;
    __syncthreads();
    const uint32_t first_w = off >> 5, last_w = (off + nbits - 1) >> 5;
    if (active && last_w >= wbase && first_w < wbase + kWinWords) {
      BitSink sink;
      sink.acc = 0;
      sink.nacc = (int)(off & 31);
      sink.widx = first_w;
      sink.wbase = wbase;
      sink.win = s_win;
      code_block<true>(qz, diff, ac, dct, &sink);
      sink.finish();
    }
    __syncthreads();
    const uint32_t n = min((uint32_t)kWinWords, nwords - wbase);
    for (uint32_t i = tid; i < n; i += kEncThreads) slot[wbase + i] = s_win[i];
    __syncthreads();
  }
  if (tid == 0) chunk_bits[(size_t)frame * g.nchunks + chunk] = total;
}

// --------------------------------------------------------------- block scan
// Exclusive scan of n uint32 values with one 1024-thread workgroup; returns the total.
__device__ uint32_t block_excl_scan(const uint32_t *in, uint32_t *out, int n) {
  __shared__ uint32_t s_w[16];
  __shared__ uint32_t s_carry;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid == 0) s_carry = 0;
  __syncthreads();
  for (int base = 0; base < n; base += 1024) {
    const int i = base + tid;
    const uint32_t v = i < n ? in[i] : 0u;
    const uint32_t incl = wave_incl_scan(v, lane);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    if (wave == 0) {
      const uint32_t t = lane < 16 ? s_w[lane] : 0u;
      const uint32_t ti = wave_incl_scan(t, lane);
      if (lane < 16) s_w[lane] = ti - t;
    }
    __syncthreads();
    const uint32_t carry = s_carry;
    if (i < n) out[i] = carry + s_w[wave] + incl - v;
    __syncthreads();
    if (tid == 1023) s_carry = carry + s_w[wave] + incl;
    __syncthreads();
  }
  return s_carry;
}

__global__ __launch_bounds__(1024) void k_scan_bits(const uint32_t *__restrict__ chunk_bits,
                                                    uint32_t *__restrict__ chunk_off,
                                                    uint32_t *__restrict__ frame_bits, int nchunks) {
  const int f = blockIdx.x;
  const uint32_t t = block_excl_scan(chunk_bits + (size_t)f * nchunks, chunk_off + (size_t)f * nchunks,
                                     nchunks);
  if (threadIdx.x == 0) frame_bits[f] = t;
}

// Word k (32 bits, MSB first) of frame f's unstuffed scan, for a word owned by chunk c
// (its first bit lies in chunk c).  Bits past the chunk come from chunk c+1, or for the
// frame's last chunk are the 1-bit padding to a byte boundary (ff_mjpeg_escape_FF pad).
__device__ __forceinline__ uint32_t chunk_bits_at(const uint32_t *slot, uint32_t p, uint32_t len) {
  const uint32_t wi = p >> 5, s = p & 31;
  const uint32_t nw = (len + 31) >> 5;
  uint32_t v = slot[wi];
  if (s) {
    const uint32_t w1 = (wi + 1 < nw) ? slot[wi + 1] : 0u;
    v = (v << s) | (w1 >> (32 - s));
  }
  const uint32_t rem = len - p;
  if (rem < 32) v &= ~(0xffffffffu >> rem);
  return v;
}

__device__ __forceinline__ uint32_t aligned_word(const uint32_t *scratch, const uint32_t *cbits,
                                                 int nchunks, int f, int c, uint32_t O, uint32_t L,
                                                 uint32_t T, uint32_t k) {
  const uint32_t *slot = scratch + ((size_t)f * nchunks + c) * kSlotWords;
  const uint32_t p = 32 * k - O;
  uint32_t v = chunk_bits_at(slot, p, L);
  const uint32_t rem = L - p;
  if (rem < 32) {
    if (c + 1 < nchunks) {
      const uint32_t *nslot = slot + kSlotWords;
      const uint32_t nl = cbits[(size_t)f * nchunks + c + 1];
      v |= chunk_bits_at(nslot, 0, nl) >> rem;
    } else {
      const uint32_t pad = (8 - (T & 7)) & 7;
      const uint32_t ones = (0xffffffffu >> rem) & ~(rem + pad >= 32 ? 0u : (0xffffffffu >> (rem + pad)));
      v |= ones;
    }
  }
  return v;
}

__device__ __forceinline__ int ff_in_word(uint32_t v, uint32_t byte0, uint32_t total_bytes) {
  int n = 0;
#pragma unroll
  for (int b = 0; b < 4; b++)
    n += (byte0 + b < total_bytes) && (((v >> (24 - 8 * b)) & 0xffu) == 0xffu);
  return n;
}

__global__ __launch_bounds__(256) void k_count_ff(const uint32_t *__restrict__ scratch,
                                                  const uint32_t *__restrict__ chunk_bits,
                                                  const uint32_t *__restrict__ chunk_off,
                                                  const uint32_t *__restrict__ frame_bits,
                                                  uint32_t *__restrict__ chunk_ff, int nchunks) {
  __shared__ int s_w[4];
  const int c = blockIdx.x, f = blockIdx.y, tid = threadIdx.x;
  const size_t ci = (size_t)f * nchunks + c;
  const uint32_t O = chunk_off[ci], L = chunk_bits[ci], T = frame_bits[f];
  const uint32_t total_bytes = (T + 7) >> 3;
  const uint32_t k0 = (O + 31) >> 5, k1 = (O + L + 31) >> 5;
  int cnt = 0;
  for (uint32_t k = k0 + tid; k < k1; k += 256) {
    const uint32_t v = aligned_word(scratch, chunk_bits, nchunks, f, c, O, L, T, k);
    cnt += ff_in_word(v, 4 * k, total_bytes);
  }
  cnt = wave_sum(cnt);
  if ((tid & 63) == 0) s_w[tid >> 6] = cnt;
  __syncthreads();
  if (tid == 0) chunk_ff[ci] = (uint32_t)(s_w[0] + s_w[1] + s_w[2] + s_w[3]);
}

__global__ __launch_bounds__(1024) void k_scan_ff(const uint32_t *__restrict__ chunk_ff,
                                                  uint32_t *__restrict__ ff_off,
                                                  const uint32_t *__restrict__ frame_bits,
                                                  uint64_t *__restrict__ frame_size, int nchunks,
                                                  int hdr_len) {
  const int f = blockIdx.x;
  const uint32_t t = block_excl_scan(chunk_ff + (size_t)f * nchunks, ff_off + (size_t)f * nchunks,
                                     nchunks);
  if (threadIdx.x == 0) frame_size[f] = (uint64_t)hdr_len + ((frame_bits[f] + 7) >> 3) + t + 2;
}

// grid (nchunks, nframes), 256 threads.  Writes chunk c's owned bytes with a 0x00 after
// every 0xFF; chunk 0 also writes the header, the last chunk the EOI marker.
__global__ __launch_bounds__(256) void k_write(
    const uint32_t *__restrict__ scratch, const uint32_t *__restrict__ chunk_bits,
    const uint32_t *__restrict__ chunk_off, const uint32_t *__restrict__ frame_bits,
    const uint32_t *__restrict__ ff_off, const uint64_t *__restrict__ frame_size,
    const uint8_t *__restrict__ hdr, int hdr_len, int nchunks, uint8_t *__restrict__ out,
    uint64_t out_cap, uint64_t *__restrict__ frame_offsets, uint32_t *__restrict__ status) {
  __shared__ uint32_t s_w[4];
  __shared__ uint64_t s_foff;
  __shared__ uint32_t s_carry;
  const int c = blockIdx.x, f = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (wave == 0) {
    uint64_t s = 0;
    for (int i = lane; i < f; i += 64) s += frame_size[i];
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d, 64);
    if (lane == 0) {
      s_foff = s;
      s_carry = 0;
    }
  }
  __syncthreads();
  const uint64_t foff = s_foff;
  const uint64_t fsize = frame_size[f];
  if (foff + fsize > out_cap) {
    if (tid == 0) atomicOr(status, 1u);
    return;
  }
  if (c == 0 && tid == 0) {
    frame_offsets[f] = foff;
    if (f == (int)gridDim.y - 1) frame_offsets[f + 1] = foff + fsize;
  }
  uint8_t *fo = out + foff;
  if (c == 0)
    for (int i = tid; i < hdr_len; i += 256) fo[i] = hdr[i];
  const size_t ci = (size_t)f * nchunks + c;
  const uint32_t O = chunk_off[ci], L = chunk_bits[ci], T = frame_bits[f];
  const uint32_t total_bytes = (T + 7) >> 3;
  if (c == nchunks - 1 && tid == 0) {
    fo[fsize - 2] = 0xff;
    fo[fsize - 1] = 0xd9;
  }
  const uint32_t k0 = (O + 31) >> 5, k1 = (O + L + 31) >> 5;
  uint8_t *scan = fo + hdr_len;
  const uint32_t ff_before = ff_off[ci];
  for (uint32_t kb = k0; kb < k1; kb += 256) {
    const uint32_t k = kb + tid;
    uint32_t v = 0;
    int cnt = 0;
    if (k < k1) {
      v = aligned_word(scratch, chunk_bits, nchunks, f, c, O, L, T, k);
      cnt = ff_in_word(v, 4 * k, total_bytes);
    }
    const uint32_t incl = wave_incl_scan((uint32_t)cnt, lane);
    if (lane == 63) s_w[wave] = incl;
    __syncthreads();
    uint32_t wpre = 0;
    for (int i = 0; i < wave; i++) wpre += s_w[i];
    const uint32_t carry = s_carry;
    if (k < k1) {
      // stuffed position of this word's first byte
      uint32_t pos = 4 * k + ff_before + carry + wpre + incl - (uint32_t)cnt;
#pragma unroll
      for (int b = 0; b < 4; b++) {
        if (4 * k + b < total_bytes) {
          const uint8_t byte = (uint8_t)(v >> (24 - 8 * b));
          scan[pos++] = byte;
          if (byte == 0xff) scan[pos++] = 0;
        }
      }
    }
    __syncthreads();
    if (tid == 255) s_carry = carry + s_w[0] + s_w[1] + s_w[2] + s_w[3];
    __syncthreads();
  }
}

}  // namespace mjg
