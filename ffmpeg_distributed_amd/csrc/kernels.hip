#pragma once
// gfx950 kernels of the MJPEG segment encoder (see include/mjgpu.h for the boundary).
//
// Pipeline per submit (B frames; see DESIGN.md §4 for the streams they run on):
//   k_scale       [only with -vf scale] bicubic hscale -> tv->pc range -> vscale, LDS-staged
//   k_encode      persistent waves, one chunk of 64 consecutive blocks (MCU coding order) per
//                 wave step, lane = block: 8-byte row loads with edge replication, [tv->pc
//                 range], jfdctint row pass (exact fp32) + column screen, exact quantisation of
//                 the screened candidates, DC prediction by lane shuffles, Huffman coding,
//                 wave prefix-sum bit-pack of the chunk into its scratch slot
//   k_scan_bits   per segment: exclusive scan of chunk bit lengths
//   k_count_ff    per group of 32 chunks: realign the bits to the segment offset (1-bit padding),
//                 count 0xFF bytes
//   k_scan_ff     per frame: scans of the group counts, segment / frame sizes; the last frame to
//                 finish places every frame
//   k_write       per group: header / stuffed scan bytes / RSTn / EOI into the packed output
//
// Arithmetic follows FFmpeg (see oracle/mjpeg_oracle.c for the per-function citations):
// libavcodec/jfdctint_template.c, mpegvideo_enc.c dct_quantize_c, mjpegenc.c
// encode_block, mjpegenc_common.c escape/stuffing; libswscale hscale/range/vscale.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "jpeg_tables.h"

namespace mjg {

constexpr int kEncWavesPerEU = 3;  // k_encode occupancy target (waves per SIMD); measured best (v8)

constexpr int kMaxBlockBits = 1664;  // >= DC 16 + 63 * (16 + 10) bits
constexpr int kSlotWords = (64 * kMaxBlockBits + 31) / 32;  // one chunk = 64 blocks

// fp32 exact-integer arithmetic (k_encode): adding kM = 1.5*2^23 rounds to an integer
// (round-to-nearest-even) and keeps it in the low mantissa bits; kMc = kM + 16384 leaves
// value + 16384 in the low 16 bits.  kRnd = 2^-10 turns floor(x/512 + 1/2) into RNE.
// The row image (s_pk) holds row-pass output 0 (the row sum, 0..32640) unbiased and outputs
// 1-7 (|value| <= 16320) + 16384, so every u16 is below 2^15 and reads as the same value
// when v_dot2_i32_i16 takes it as int16 (exact_coef: no sign fix-up).
constexpr int kTabWords = 704;  // device table block, see open_ctx
constexpr float kM = 12582912.0f;
constexpr float kMc = 12599296.0f;  // kM + 16384: the row image's bias for outputs 1-7
constexpr float kRnd = 0x1p-10f;

// jfdctint pass 2 (CONST_BITS 13, PASS1_BITS 4) per output row as one dot product over
// the 8 column inputs: the LLM butterfly's t/z terms multiplied out (rows 0/4: +-1 with
// DESCALE 4; others: DESCALE 17).
#define MJG_PASS2_DOT                                                  \
  {1, 1, 1, 1, 1, 1, 1, 1,                                             \
   11363, 9633, 6437, 2260, -2260, -6437, -9633, -11363,               \
   10703, 4433, -4433, -10703, -10703, -4433, 4433, 10703,             \
   9633, -2259, -11362, -6436, 6436, 11362, 2259, -9633,               \
   1, -1, -1, 1, 1, -1, -1, 1,                                         \
   6437, -11362, 2261, 9633, -9633, -2261, 11362, -6437,               \
   4433, -10704, 10704, -4433, -4433, 10704, -10704, 4433,             \
   2260, -6436, 9633, -11363, 11363, -9633, 6436, -2260}
__device__ static constexpr int kPass2Dot[64] = MJG_PASS2_DOT;
// The kernel's pass-2 rows (s_m2): rows 0 and 4 scaled by 2^13, so every row is accumulated
// from 2^16 and descaled by 17 (2^13 (S + 8) >> 17 == (S + 8) >> 4; |S| <= 8 * 32640, so
// 2^13 (S + 8) stays below 2^31): no per-row shift in exact_coef.  The image's +16384 of
// columns 1-7 cancels in every row but row 0 (its entries sum to 2^16), where the start value
// is 2^16 - 2^30 instead (kRow0Bias, carried in the descriptor's top bits).
constexpr uint32_t kRow0Bias = 0xC0000000u;  // -2^30 = -16384 * 2^16
constexpr int kPass2DcScale = 8192;
__device__ __forceinline__ uint32_t pass2_pair(int i) {  // int16 pair of entries 2i, 2i + 1
  const int r = i >> 2, f = (r & 3) == 0 ? kPass2DcScale : 1;
  return (uint32_t)(uint16_t)(kPass2Dot[2 * i] * f) | ((uint32_t)(uint16_t)(kPass2Dot[2 * i + 1] * f) << 16);
}
// Frame geometry.  A frame is a raster of MCUs of `bpm` blocks each (4:2:0: 16x16, Y0-3 Cb
// Cr; 4:2:2: 16x16, Y0-3 Cb0 Cb1 Cr0 Cr1; 4:4:4: 8x16, Y0 Y1 Cb0 Cb1 Cr0 Cr1 -- FFmpeg's
// coding order, see oracle/mjpeg_oracle.c or_layouts), split into `nseg` entropy-coded
// segments per frame (1, or one per MCU row in RST mode) of seg_blocks blocks, each cut into
// `nchunks` chunks of 64 blocks.  The per-block-of-MCU descriptors (plane, table, 8x8 offset
// in the MCU, DC predecessor distance) are words [672, 680) of the table block.
struct EncGeom {
  int w, h;            // encoded size
  int cw, ch;          // chroma plane size
  int mbw, nmcu;       // MCUs per row, per frame
  int bpm;             // blocks per MCU (6 or 8)
  uint32_t bpm_magic;  // ceil(2^32 / bpm): b / bpm == umulhi(b, bpm_magic) for b < 2^29
  uint32_t mbw_magic;  // ceil(2^32 / mbw) (0 when mbw == 1): m / mbw == umulhi(m, mbw_magic)
                       // while m * mbw < 2^32 (the host checks (nmcu + 64) * mbw)
  int lmw, cmh;        // luma MCU width (16, 4:4:4: 8), chroma MCU height (8, 4:2:2/4:4:4: 16)
  int nseg, seg_blocks, nchunks;  // segments per frame, blocks / chunks per segment
  unsigned long long nchunks_magic, nseg_magic;  // ceil(2^40 / n): t / n == (t * magic) >> 40
                                                 // for t * n < 2^40 (tasks per launch)
  int y_stride, c_stride;
  long long frame_stride, u_off, v_off;
  int range_convert;   // 1: yuv420p (tv) input without scale -> swscale tv->pc per pixel
  int debug_coefs;
};

// A submit's input frames as up to kMaxSegs segments (mjg_submit_segments): segment k holds
// the submit's frames [f0[k], f0[k + 1]) at p[k], frame_stride apart; unused entries have
// f0 = INT_MAX.  One launch then covers several segments, so their ramp and drain are paid
// once (DESIGN §4 segments).  A kernel argument, resolved with scalar selects per chunk.
constexpr int kMaxSegs = 4;
struct SegList {
  const uint8_t *p[kMaxSegs];
  int f0[kMaxSegs];
};
__device__ __forceinline__ const uint8_t *seg_frame(const SegList &sl, int f, long long stride) {
  const uint8_t *b = sl.p[0];
  int s0 = 0;
#pragma unroll
  for (int k = 1; k < kMaxSegs; k++)
    if (f >= sl.f0[k]) {
      b = sl.p[k];
      s0 = sl.f0[k];
    }
  return b + (size_t)(f - s0) * stride;
}

// block descriptor word: bits 0-1 plane, 2 Huffman table (chroma), 3 dx (8 px), 4 dy (8 px),
// 8-11 distance to the previous block of the same component in coding order
__device__ __forceinline__ int desc_tab(uint32_t d) { return (int)((d >> 2) & 1u); }
__device__ __forceinline__ int desc_delta(uint32_t d) { return (int)(d >> 8); }
__device__ __forceinline__ int block_in_mcu(const EncGeom &g, int b) {
  return b - __mul24(g.bpm, (int)__umulhi((uint32_t)b, g.bpm_magic));
}


// ---------------------------------------------------------------- helpers
// swscale's unscaled yuv420p -> yuvj420p path per sample: hScale8To15 (1 tap, 1<<14)
// -> lumRangeToJpeg_c / chrRangeToJpeg_c -> yuv2plane1_8_c (flat 64 dither), i.e.
//   Y: clip_u8((((min(p<<7, 30189) * 19077 - 39057361) >> 14) + 64) >> 7)
//   C: clip_u8((((min(p<<7, 30775) *  4663 -  9289992) >> 12) + 64) >> 7)
// The nested floors fold to one shift and the input clamps are subsumed by the output
// clamp (checked exhaustively for p = 0..255 in tests/test_oracle.py).
__device__ __forceinline__ int range_luma(int p) {
  return min(max((__mul24(p, 2441856) - 38008785) >> 21, 0), 255);
}
__device__ __forceinline__ int range_chroma(int p) {
  return min(max((__mul24(p, 596864) - 9027848) >> 19, 0), 255);
}

#define MJG_DESCALE(x, n) (((x) + (1 << ((n) - 1))) >> (n))

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ u16x2 as_u16x2(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

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
  int z1 = __mul24(t12 + t13, 4433);
  p[2 * S] = MJG_DESCALE(z1 + __mul24(t13, 6270), SH);
  p[6 * S] = MJG_DESCALE(z1 - __mul24(t12, 15137), SH);
  z1 = t4 + t7;
  int z2 = t5 + t6, z3 = t4 + t6, z4 = t5 + t7;
  const int z5 = __mul24(z3 + z4, 9633);
  t4 = __mul24(t4, 2446);
  t5 = __mul24(t5, 16819);
  t6 = __mul24(t6, 25172);
  t7 = __mul24(t7, 12299);
  z1 = __mul24(z1, -7373);
  z2 = __mul24(z2, -20995);
  z3 = __mul24(z3, -16069);
  z4 = __mul24(z4, -3196);
  z3 += z5;
  z4 += z5;
  p[7 * S] = MJG_DESCALE(t4 + z1 + z3, SH);
  p[5 * S] = MJG_DESCALE(t5 + z2 + z4, SH);
  p[3 * S] = MJG_DESCALE(t6 + z2 + z3, SH);
  p[1 * S] = MJG_DESCALE(t7 + z1 + z4, SH);
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS traffic
// (lgkmcnt) but NOT for outstanding global loads, so a prefetch issued before the
// barrier stays in flight (__syncthreads() would add s_waitcnt vmcnt(0)).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Inclusive wave prefix sum on DPP lane moves (no LDS round trips): Hillis-Steele within
// each 16-lane row (row_shr 1, 2, 4, 8; lanes whose source is outside the row read 0:
// bound_ctrl, so each step is one v_add_u32_dpp), then row_bcast:15 carries row 0 / row 2 totals into rows 1 / 3 and
// row_bcast:31 carries the rows 0-1 total into rows 2-3.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t v, int) {
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);   // row_shr:1
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);   // row_shr:2
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);   // row_shr:4
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);   // row_shr:8
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return v;
}

__device__ __forceinline__ uint32_t lane63(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
  return v;
}

// Symbol -> code lookups shared by the emitting sinks: tables hold (len << 16) | code.
#define MJG_SINK_SYMBOLS                                                              \
  const uint32_t *act, *dct;                                                          \
  __device__ __forceinline__ void dc(int cat, uint32_t mant) {                        \
    const uint32_t e = dct[cat];                                                      \
    emit(((e & 0xffffu) << cat) | mant, (int)(e >> 16) + cat);                        \
  }                                                                                   \
  __device__ __forceinline__ void ac(int sym, int cat, uint32_t mant) {               \
    const uint32_t e = act[sym];                                                      \
    emit(((e & 0xffffu) << cat) | mant, (int)(e >> 16) + cat);                        \
  }                                                                                   \
  /* the AC code of sym (a table read issued early), then its emission */             \
  __device__ __forceinline__ uint32_t lookup(int sym) const { return act[sym]; }      \
  __device__ __forceinline__ void put_ac(uint32_t e, int, int cat, uint32_t mant) {   \
    emit(((e & 0xffffu) << cat) | mant, (int)(e >> 16) + cat);                        \
  }

__device__ __forceinline__ int dc_cat(int diff) {
  const int a = diff < 0 ? -diff : diff;
  return diff == 0 ? 0 : 32 - __clz(a);
}

// JPEG magnitude category and mantissa of v != 0 (mjpegenc.c encode_block: mant = v, or v - 1
// for v < 0, in `cat` bits): t = v - (v < 0) holds the mantissa in its low bits, and cat is
// where t's bits start to differ from its sign (clrsb: v_ffbh_i32), so |v| is never formed.
__device__ __forceinline__ int mag_cat(int v, uint32_t &mant) {
  const int t = v + (v >> 31);
  const int cat = 31 - __builtin_clrsb(t);  // v_ffbh_i32
  mant = __builtin_amdgcn_ubfe((uint32_t)t, 0u, (uint32_t)cat);
  return cat;
}

// v_ffbh_i32: the bit position, counted from the MSB, of the first bit that differs from the
// sign bit; -1 for 0 and -1.  For t = v - (v < 0) of a nonzero v, 32 - ffbh is the category.
__device__ __forceinline__ int ffbh_i32(int t) {
  int r;
  asm("v_ffbh_i32 %0, %1" : "=v"(r) : "v"(t));
  return r;
}

// The emission pass: the block's last 128 bits right-aligned in a 4-register shift register
// (w3 lowest; the block's offset in the chunk is not known yet), and the total bit count.
// Appending n <= 26 bits is four funnel shifts, (w_i << n) | (w_i+1 >> (32 - n)), one
// v_alignbit each.  A block longer than 128 bits (rare: text-like detail) spills its stream
// word by word to the lane's staging column in HBM (stage[j * 64] = stream bits
// [32j, 32j + 32)) just before the word would leave the window; flush() then writes the
// rest, and the pack step copies the staged stream to its place in the slot.
struct ShiftSink {
  MJG_SINK_SYMBOLS
  uint32_t w0 = 0, w1 = 0, w2 = 0, w3 = 0;
  uint32_t bits = 0;     // stream bits (set by finish(), or by emit_block_wave)
  int room = 128;        // free window bits: 128 - (stream bits - spilled)
  uint32_t spilled = 0;  // stream bits already staged (multiple of 32)
  bool staged = false;   // the whole stream is in the staging column (emit_block_wave)
  uint32_t *stage;
  // the staged word at stream bit `spilled`: window offset o = 128 - (bits - spilled) from the top
  __device__ __forceinline__ uint32_t window_word(uint32_t o, uint32_t a, uint32_t b) const {
    return o ? __builtin_amdgcn_alignbit(a, b, 32u - o) : a;
  }
  __device__ __forceinline__ void emit(uint32_t v, int n) {
    room -= n;
    if (room < 0) {  // the oldest unstaged word would be shifted out
      stage[(spilled >> 5) * 64] = window_word((uint32_t)(room + n), w0, w1);
      spilled += 32;
      room += 32;
    }
    const uint32_t sh = 32u - (uint32_t)n;
    w0 = __builtin_amdgcn_alignbit(w0, w1, sh);
    w1 = __builtin_amdgcn_alignbit(w1, w2, sh);
    w2 = __builtin_amdgcn_alignbit(w2, w3, sh);
    w3 = (w3 << n) | v;  // v_lshl_or (n <= 27)
  }
  // the block's bit count; a block past 128 bits stages the rest of its window
  __device__ __forceinline__ void finish() {
    bits = spilled + 128u - (uint32_t)room;
    if (bits > 128u) flush();
  }
  // a block past 128 bits: stage the words still in the window (stream words
  // spilled/32 .. (bits-1)/32, at most 4)
  __device__ __forceinline__ void flush() {
    const uint32_t o = 128u - (bits - spilled), j0 = spilled >> 5, nrem = (bits - spilled + 31) >> 5;
    stage[j0 * 64] = window_word(o, w0, w1);
    if (nrem > 1) stage[(j0 + 1) * 64] = window_word(o, w1, w2);
    if (nrem > 2) stage[(j0 + 2) * 64] = window_word(o, w2, w3);
    if (nrem > 3) stage[(j0 + 3) * 64] = window_word(o, w3, 0u);
  }
};

constexpr int kStageWords = (kMaxBlockBits + 31) / 32;  // staged words per lane
constexpr int kHvWords = kStageWords < 128 ? 128 : kStageWords;  // s_hv: emit_block_wave, pack_chunk_short

// Exact quantised coefficient at natural index n of this lane's block, from the row-pass
// image (pkcol = s_pk + lane: word [c*4 + r/2] holds column c of rows r, r+1 (r even) as u16
// = value, + 16384 for columns 1-7).  jfdctint pass 2 for output row ro is one integer dot
// product over the column (the LLM butterfly's products and sums folded into kPass2Dot[ro][*]):
// v_dot2_i32_i16 multiplies a word (two rows) at a time against the packed coefficient pairs
// m2p[ro][*] (pass2_pair; every u16 is below 2^15, so int16 reads it unchanged, and the bias
// cancels or is started out, see kRow0Bias).  Then DESCALE and dct_quantize_c's intra
// rounding: sign(u) * ((|u| * qmat + 3<<18) >> 21), folded into one signed multiply-add.
typedef short short2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int exact_coef(const uint32_t *pkcol, int n, const uint32_t *m2p,
                                          const int *qc) {
  const int ro = n >> 3, c = n & 7;
  const uint4 mp = *(const uint4 *)(m2p + ro * 4);
  const uint32_t m[4] = {mp.x, mp.y, mp.z, mp.w};
  int acc = (int)((ro == 0 && c != 0 ? kRow0Bias : 0u) | 0x10000u);  // see pass2_pair
#pragma unroll
  for (int i = 0; i < 4; i++)
    acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, pkcol[(c * 4 + i) * 64]),
                                 __builtin_bit_cast(short2_t, m[i]), acc, false);
  const int u = acc >> 17;
  const int qm = qc[c * 8 + ro];
  return (__mul24(u, qm) + (u < 0 ? (1 << 21) - 1 - (3 << 18) : (3 << 18))) >> 21;
}

// exact_coef for zigzag position k from its descriptor (zz_desc, in LDS), returned as
// t = v - (v < 0) (see emit_block): x = the accumulator's start value (2^16, plus kRow0Bias for
// row 0, columns 1-7), y = qmat, z = the pass-2 row's byte offset in s_m2, w = the column's
// byte offset in the row image.  One 16-byte LDS read per candidate replaces the zigzag, qmat
// and row tables and every field extraction.
__device__ __forceinline__ uint4 zz_desc(int k, const uint32_t *tabs) {
  const int n = kZigzag[k], ro = n >> 3, c = n & 7;
  return make_uint4((ro == 0 && c != 0 ? kRow0Bias : 0u) | 0x10000u, tabs[544 + c * 8 + ro],
                    (uint32_t)ro * 16u, (uint32_t)c * 4u * 64u * 4u);
}
__device__ __forceinline__ int exact_coef_t(const uint32_t *pkcol, uint4 d, const uint32_t *m2p) {
  const uint32_t *col = (const uint32_t *)((const uint8_t *)pkcol + d.w);
  const uint4 mp = *(const uint4 *)((const uint8_t *)m2p + d.z);
  const uint32_t m[4] = {mp.x, mp.y, mp.z, mp.w};
  int acc = (int)d.x;
#pragma unroll
  for (int i = 0; i < 4; i++)
    acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, col[i * 64]), __builtin_bit_cast(short2_t, m[i]),
                                 acc, false);
  const int u = acc >> 17;
  // t = v - (v < 0) (mag_cat's t) directly: for u < 0 the rounding constant less 2^21
  return (__mul24(u, (int)d.y) + (u < 0 ? -1 - (3 << 18) : (3 << 18))) >> 21;
}

// Bit-pack one block's Huffman codes, FFmpeg mjpegenc.c encode_block /
// mjpegenc_common.c ff_mjpeg_encode_dc (ZRL 0xF0 per 16 zeros, EOB unless coef 63 != 0).
// `cand` is a superset of the nonzero AC positions in zigzag order (the float screening of
// the column pass); each candidate is quantised exactly and skipped when it is zero, so
// runs and EOB are those of the exact block.  (Mean nonzero AC per block is ~1.3 on
// testsrc2 4K q5, so the loop is short.)
// t: the coefficient v as v - (v < 0) (exact_coef_t), so t is 0 or -1 exactly when v == 0
// and the category is 32 - v_ffbh_i32(t) (no |v|, no sign fix-up).
// Candidates are taken two at a time so the LDS reads of both (their descriptors, the columns
// of the row image, then their AC codes) are in flight together: both symbols are formed
// before either is emitted (the second one's run depends only on whether the first is zero).
template <class Sink>
__device__ __forceinline__ void emit_block(const uint32_t *pkcol, uint64_t cand, int diff,
                                           const uint4 *zd, const uint32_t *m2, Sink &sink) {
  {
    uint32_t mant = 0;
    const int cat = diff ? mag_cat(diff, mant) : 0;
    sink.dc(cat, mant);
  }
  int prev = 0;
  while (cand) {
    const int k1 = (int)__builtin_ctzll(cand);
    cand &= cand - 1;
    const bool two = cand != 0;
    const int k2 = two ? (int)__builtin_ctzll(cand) : k1;
    cand &= cand - 1;  // no-op when cand == 0
    const int t1 = exact_coef_t(pkcol, zd[k1], m2);
    const int t2 = exact_coef_t(pkcol, zd[k2], m2);
    const int fb1 = ffbh_i32(t1), fb2 = two ? ffbh_i32(t2) : -1;  // < 0: quantises to zero
    const bool nz1 = fb1 >= 0, nz2 = fb2 >= 0;
    const int run1 = k1 - prev - 1, p1 = nz1 ? k1 : prev, run2 = k2 - p1 - 1;
    const int cat1 = 32 - fb1, cat2 = 32 - fb2;
    const int s1 = nz1 ? ((run1 & 15) << 4) | cat1 : 0, s2 = nz2 ? ((run2 & 15) << 4) | cat2 : 0;
    const uint32_t e1 = sink.lookup(s1), e2 = sink.lookup(s2);
    if (nz1) {
      for (int r = run1; r >= 16; r -= 16) sink.ac(0xf0, 0, 0u);  // ZRL
      sink.put_ac(e1, s1, cat1, __builtin_amdgcn_ubfe((uint32_t)t1, 0u, (uint32_t)cat1));
    }
    if (nz2) {
      for (int r = run2; r >= 16; r -= 16) sink.ac(0xf0, 0, 0u);
      sink.put_ac(e2, s2, cat2, __builtin_amdgcn_ubfe((uint32_t)t2, 0u, (uint32_t)cat2));
    }
    prev = nz2 ? k2 : p1;
  }
  if (prev != 63) sink.ac(0x00, 0, 0u);  // EOB
}

// Wave-parallel emission of one block h (wave-uniform): lane k codes zigzag coefficient k.
// For blocks with many coefficients (noise, fine texture) the per-lane loop of emit_block
// runs as long as the wave's longest block, with the other lanes idle; here the block's
// symbols are formed side by side and placed by a prefix sum of their lengths.
//   coefficients: exact_coef with the block's row-image words broadcast from lanes 0-31
//                 (one ds_read of column h, then ds_bpermute per word)
//   symbols:      lane k (nonzero) codes ZRL* + (run, size) + mantissa, run from the ballot
//                 of nonzeros; lane 0 the DC; lane 63 the EOB when coefficient 63 is zero
//   bits:         each lane's <= 59 bits ORed into the wave's LDS stream words (<= 3 per
//                 lane), which then go to block h's staging column (pack_chunk reads it)
// Returns the block's bit count.  Same bytes as emit_block (FFmpeg encode_block).
__device__ __noinline__ uint32_t emit_block_wave(const uint32_t *s_pk, int h, int diff_h, int tab_h,
                                                 const uint4 *zd, const uint32_t *m2,
                                                 const uint32_t *s_ac, const uint32_t *s_dc, uint32_t *s_hv,
                                                 uint32_t *stage_w, int lane) {
  const uint32_t wv = lane < 32 ? s_pk[lane * 64 + h] : 0u;
  const uint4 d = zd[lane];
  const uint32_t cw = d.w >> 6;  // byte offset of the column's first word in wv's lanes (4 * c * 4)
  const uint4 mp = *(const uint4 *)((const uint8_t *)m2 + d.z);
  const uint32_t m[4] = {mp.x, mp.y, mp.z, mp.w};
  int acc = (int)d.x;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t pr = (uint32_t)__builtin_amdgcn_ds_bpermute((int)cw + 4 * i, (int)wv);
    acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, pr), __builtin_bit_cast(short2_t, m[i]), acc, false);
  }
  const int u = acc >> 17;
  int t = (__mul24(u, (int)d.y) + (u < 0 ? -1 - (3 << 18) : (3 << 18))) >> 21;  // exact_coef_t
  if (lane == 0) t = 0;  // the DC is coded from diff_h
  const int fb = ffbh_i32(t);
  const uint64_t nz = __ballot(fb >= 0);
  const uint32_t *act = s_ac + tab_h * 256;
  uint64_t V = 0;
  uint32_t L = 0;
  if (fb >= 0) {
    const uint64_t below = nz & ((1ull << lane) - 1ull);
    int run = lane - (below ? 63 - (int)__builtin_clzll(below) : 0) - 1;
    if (run >= 16) {
      const uint32_t ez = act[0xf0];  // ZRL
      const uint32_t zc = ez & 0xffffu, zl = ez >> 16;
      while (run >= 16) {
        V = (V << zl) | zc;
        L += zl;
        run -= 16;
      }
    }
    const int cat = 32 - fb;
    const uint32_t mant = __builtin_amdgcn_ubfe((uint32_t)t, 0u, (uint32_t)cat);
    const uint32_t e = act[((run & 15) << 4) | cat];
    const uint32_t cl = (e >> 16) + (uint32_t)cat;
    V = (V << cl) | (((e & 0xffffu) << cat) | mant);
    L += cl;
  } else if (lane == 63) {  // EOB: coefficient 63 is zero
    const uint32_t e = act[0x00];
    V = e & 0xffffu;
    L = e >> 16;
  } else if (lane == 0) {
    const int cat = dc_cat(diff_h);
    const uint32_t e = s_dc[tab_h * 16 + cat];
    V = ((e & 0xffffu) << cat) | ((uint32_t)(diff_h < 0 ? diff_h - 1 : diff_h) & ((1u << cat) - 1u));
    L = (e >> 16) + (uint32_t)cat;
  }
  const uint32_t incl = wave_incl_scan(L, lane), off = incl - L, total = lane63(incl);
  if (L) {  // bits [off, off + L): V's MSB at bit off & 31 of word off >> 5 (MSB first)
    const uint32_t sh = 96u - (off & 31u) - L;  // 6..95: V << sh fits 96 bits
    const uint64_t hi = sh >= 32u ? V << (sh - 32u) : V >> (32u - sh);
    const uint32_t lo = sh >= 32u ? 0u : (uint32_t)(V << sh);
    uint32_t *d = s_hv + (off >> 5);
    atomicOr(d, (uint32_t)(hi >> 32));
    if ((uint32_t)hi) atomicOr(d + 1, (uint32_t)hi);
    if (lo) atomicOr(d + 2, lo);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const uint32_t nws = (total + 31u) >> 5;
  if ((uint32_t)lane < nws) {
    stage_w[lane * 64 + h] = s_hv[lane];
    s_hv[lane] = 0u;
  }
  return total;
}

// Blocks of a chunk coded by emit_block_wave instead of per lane: the lanes whose candidate
// count exceeds T, for the T in {4, 8, 16, 32} that minimises 4 x (wave-parallel blocks) + T
// (T bounds the per-lane loop that remains; a wave-parallel block costs about four
// candidates of it: factors 1, 2, 4, 6 and 8 were A/B'd on three contents), if that beats
// the per-lane loop alone (bounded by the smallest T no lane exceeds).  0: all per lane.
__device__ __forceinline__ uint64_t wave_parallel_blocks(int ncand) {
  uint64_t hv[4];
  int serial = 64;
#pragma unroll
  for (int k = 3; k >= 0; k--) {
    hv[k] = __ballot(ncand > (4 << k));
    if (!hv[k]) serial = 4 << k;
  }
  uint64_t best = 0ull;
  int best_cost = serial;
#pragma unroll
  for (int k = 0; k < 4; k++) {
    const int cost = 4 * __popcll(hv[k]) + (4 << k);
    if (hv[k] && cost < best_cost) {
      best_cost = cost;
      best = hv[k];
    }
  }
  return best;
}

// -huffman optimal, first pass: count the block's symbols into the wave's LDS histogram,
// mjpegenc.c record_block / ff_mjpeg_encode_huffman_increment.  The histogram is 16-bit
// counters in pairs (kCountWords words: AC table t symbol s at word t*128 + (s & 127), half
// s >> 7; DC table t category c at word 256 + t*8 + (c & 7), half c >> 3: the rare symbols
// share a word with the common ones, so same-address atomics stay those of one symbol), so
// that the counting pass fits 4 workgroups per CU; flushed into the frame's 32-bit table block
// (AC luma 0-255, AC chroma 256-511, DC luma 512-527, DC chroma 528-543) at every frame change
// and at least every kCountFlush chunks (a symbol occurs at most 63 times per block:
// 16 x 64 x 63 < 2^16).
// It also records every symbol with its mantissa in the lane's record column (rec[j * 64]:
// DC flag << 31 | (DC category or AC symbol) << 16 | mantissa), so the emission pass
// replays the symbols (k_emit_syms) instead of recomputing the block.
constexpr int kSymCap = 68;  // symbols per block: DC + 63 AC + 3 ZRL + EOB
constexpr int kCountWords = 272, kCountFlush = 16;
struct CountSink {
  uint32_t *hac, *hdc;
  uint32_t *rec;
  uint32_t n = 0;
  __device__ __forceinline__ void dc(int cat, uint32_t mant) {
    atomicAdd(&hdc[cat & 7], 1u << ((cat >> 3) << 4));
    rec[n * 64] = (1u << 31) | ((uint32_t)cat << 16) | mant;
    n++;
  }
  __device__ __forceinline__ void ac(int sym, int, uint32_t mant) {
    atomicAdd(&hac[sym & 127], 1u << ((sym >> 7) << 4));
    rec[n * 64] = ((uint32_t)sym << 16) | mant;
    n++;
  }
  __device__ __forceinline__ uint32_t lookup(int) const { return 0u; }
  __device__ __forceinline__ void put_ac(uint32_t, int sym, int cat, uint32_t mant) { ac(sym, cat, mant); }
  __device__ __forceinline__ void finish() {}
};

// The wave's 16-bit counter pairs (CountSink) added into the frame's table block hf, and zeroed.
__device__ __forceinline__ void flush_counts(uint32_t *s_cnt, uint32_t *hf, int lane) {
  for (int i = lane; i < kCountWords; i += 64) {
    const uint32_t v = s_cnt[i];
    if (v) {
      const int lo = i < 256 ? (i >> 7) * 256 + (i & 127) : 512 + ((i - 256) >> 3) * 16 + (i & 7);
      const int hi = lo + (i < 256 ? 128 : 8);
      if (v & 0xffffu) atomicAdd(&hf[lo], v & 0xffffu);
      if (v >> 16) atomicAdd(&hf[hi], v >> 16);
      s_cnt[i] = 0;
    }
  }
}

// Wave-parallel counting of one block h (wave-uniform), CountSink's work for the blocks
// wave_parallel_blocks picks: lane k quantises zigzag coefficient k as emit_block_wave does and
// holds its ZRLs + (run, size) symbol (lane 0 the DC, lane 63 the EOB); a prefix sum of the
// lanes' symbol counts places each lane's records in block h's record column (the records and
// order of emit_block with CountSink), and each lane counts its symbols.  Returns the block's
// symbol count.
__device__ __noinline__ uint32_t count_block_wave(const uint32_t *s_pk, int h, int diff_h, int tab_h,
                                                  const uint4 *zd, const uint32_t *m2, uint32_t *s_cnt,
                                                  uint32_t *rec_h, int lane) {
  const uint32_t wv = lane < 32 ? s_pk[lane * 64 + h] : 0u;
  const uint4 d = zd[lane];
  const uint32_t cw = d.w >> 6;
  const uint4 mp = *(const uint4 *)((const uint8_t *)m2 + d.z);
  const uint32_t m[4] = {mp.x, mp.y, mp.z, mp.w};
  int acc = (int)d.x;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const uint32_t pr = (uint32_t)__builtin_amdgcn_ds_bpermute((int)cw + 4 * i, (int)wv);
    acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, pr), __builtin_bit_cast(short2_t, m[i]), acc, false);
  }
  const int u = acc >> 17;
  int t = (__mul24(u, (int)d.y) + (u < 0 ? -1 - (3 << 18) : (3 << 18))) >> 21;  // exact_coef_t
  if (lane == 0) t = 0;
  const int fb = ffbh_i32(t);
  const uint64_t nz = __ballot(fb >= 0);
  uint32_t *hac = s_cnt + tab_h * 128;
  uint32_t nsym = 0, zrl = 0, r = 0;  // this lane's symbols, its ZRLs among them, its last record
  if (fb >= 0) {
    const uint64_t below = nz & ((1ull << lane) - 1ull);
    const int run = lane - (below ? 63 - (int)__builtin_clzll(below) : 0) - 1;
    zrl = (uint32_t)run >> 4;
    const int cat = 32 - fb, sym = ((run & 15) << 4) | cat;
    r = ((uint32_t)sym << 16) | __builtin_amdgcn_ubfe((uint32_t)t, 0u, (uint32_t)cat);
    nsym = zrl + 1;
    atomicAdd(&hac[sym & 127], 1u << ((sym >> 7) << 4));
    if (zrl) atomicAdd(&hac[0xf0 & 127], zrl << 16);  // ZRL 0xf0: word 0x70, high half
  } else if (lane == 63) {  // EOB: coefficient 63 is zero
    nsym = 1;
    atomicAdd(&hac[0], 1u);
  } else if (lane == 0) {
    uint32_t mant = 0;
    const int cat = diff_h ? mag_cat(diff_h, mant) : 0;
    r = (1u << 31) | ((uint32_t)cat << 16) | mant;
    nsym = 1;
    atomicAdd(&s_cnt[256 + tab_h * 8 + (cat & 7)], 1u << ((cat >> 3) << 4));
  }
  const uint32_t incl = wave_incl_scan(nsym, lane), off = incl - nsym;
  for (uint32_t i = 0; i < zrl; i++) rec_h[(off + i) * 64] = 0xf0u << 16;
  if (nsym) rec_h[(off + nsym - 1) * 64] = r;
  return lane63(incl);
}

// Raw 8x8 block as 8 little-endian row words.  Addresses are 32-bit offsets from the frame's
// base, which is wave-uniform (a chunk never spans two frames): the loads take the base from
// SGPRs and one VGPR offset (global_load saddr form), no 64-bit address arithmetic per row.
// A block's plane fields come from the block-of-MCU descriptor table in LDS (BlockDesc, one
// entry per block of the MCU): no per-lane branch on the plane.  fetch_rows issues the 8-byte
// row loads for interior blocks (the prefetch path, 16 VGPRs) and returns false for blocks that
// touch the frame edge or are misaligned; fetch_rows_edge builds those with coordinate clamping
// (FFmpeg emulated_edge_mc / draw_edges replicate the last row/column) at a point where no
// other block data is live.
struct BlockDesc {  // LDS, two uint4 per block of the MCU
  uint32_t poff;    // plane offset in the frame (0, U, V)
  int stride, pw, ph;
  int xs, ys, dx, dy;  // x0 = mx * xs + dx, y0 = my * ys + dy
};

struct BlockPos {
  uint32_t poff;
  int stride, pw, ph, x0, y0;
};

// Position of block b (index in the frame's coding order) in its frame.
__device__ __forceinline__ BlockPos block_pos(const EncGeom &g, int b, const uint4 *s_bd) {
  // (24-bit multiplies: every operand here is below 2^24)
  const int m = (int)__umulhi((uint32_t)b, g.bpm_magic);
  const int i = b - __mul24(m, g.bpm);
  const int my = g.mbw == 1 ? m : (int)__umulhi((uint32_t)m, g.mbw_magic), mx = m - __mul24(my, g.mbw);
  const uint4 a = s_bd[2 * i], c = s_bd[2 * i + 1];
  BlockPos p;
  p.poff = a.x;
  p.stride = (int)a.y;
  p.pw = (int)a.z;
  p.ph = (int)a.w;
  p.x0 = __mul24(mx, (int)c.x) + (int)c.z;
  p.y0 = __mul24(my, (int)c.y) + (int)c.w;
  return p;
}

// The block's 8 rows when it is active, inside its plane and 8-byte aligned (returns true);
// otherwise every row load reads the frame's first bytes (aligned and valid) and the caller
// refetches with fetch_rows_edge.  Unconditional loads: no per-lane branch and no zeroing of
// the row registers around them.  fb: the frame's base (wave-uniform, 8-byte aligned when
// fb_aligned).
__device__ __forceinline__ bool fetch_rows(uint64_t (&raw)[8], const uint8_t *fb, bool fb_aligned, const BlockPos &p,
                                           bool active) {
  // offsets < the frame size < 2^32, operands < 2^24
  const uint32_t off = p.poff + (uint32_t)__umul24((uint32_t)p.y0, (uint32_t)p.stride) + (uint32_t)p.x0;
  const bool fast = fb_aligned && active && (p.x0 + 8 <= p.pw) && (p.y0 + 8 <= p.ph) &&
                    ((off | (uint32_t)p.stride) & 7) == 0;
  uint32_t o = fast ? off : 0u;
  const uint32_t st = fast ? (uint32_t)p.stride : 0u;
  // plain loads: a chunk's row segments straddle 64-B sectors shared with the
  // neighbouring chunk, which L2 keeps for its wave (nontemporal loads read 1.64x)
#pragma unroll
  for (int r = 0; r < 8; r++, o += st) raw[r] = *(const uint64_t *)(fb + o);
  return fast;
}

__device__ __forceinline__ void fetch_rows_edge(uint64_t (&raw)[8], const uint8_t *fb, const BlockPos &p) {
  for (int r = 0; r < 8; r++) {
    const uint8_t *row = fb + p.poff + (size_t)min(p.y0 + r, p.ph - 1) * p.stride;
    uint64_t w = 0;
    for (int b = 0; b < 8; b++) w |= (uint64_t)row[min(p.x0 + b, p.pw - 1)] << (8 * b);
    raw[r] = w;
  }
}

// ------------------------------------------------------------------ k_encode
// Wave-granular chunks, no workgroup barriers.  A chunk is 64 consecutive blocks of a
// frame in MCU-interleaved order (Y0 Y1 Y2 Y3 Cb Cr per MCU), lane = block, so a wave
// owns a contiguous piece of the frame's bitstream:
//   * DC prediction: the predecessor of block b is b-3 (Y0), b-1 (Y1..Y3) or b-6 (Cb,
//     Cr) -- a lane shuffle, or the previous chunk's DCs carried in a register (this
//     wave encoded that chunk in its previous iteration; the first chunk of a wave's
//     range recomputes them from pixel sums: quantised DC = (sum + 32) >> 6 exactly);
//   * bit offsets: wave prefix-sum of the 64 block lengths;
//   * bit-packing: ds_or_b32 into the wave's private LDS window, then coalesced stores
//     of the chunk's words to its HBM slot.
// Persistent grid: wave w encodes chunks [w*T, (w+1)*T) in (frame, chunk) order and
// prefetches the next chunk's pixel rows into registers while encoding the current one.
constexpr int kWavesPerWg = 4;

// The block-of-MCU descriptor table (BlockDesc) from the descriptor words and the geometry.
__device__ __forceinline__ void init_block_desc(const EncGeom &g, const uint32_t *tabs, uint4 *s_bd, int tid) {
  if (tid < 8) {
    const uint32_t d = tabs[672 + tid];
    const uint32_t plane = d & 3u;
    const bool luma = plane == 0;
    uint4 a, c;
    a.x = luma ? 0u : (uint32_t)(plane == 1 ? g.u_off : g.v_off);
    a.y = (uint32_t)(luma ? g.y_stride : g.c_stride);
    a.z = (uint32_t)(luma ? g.w : g.cw);
    a.w = (uint32_t)(luma ? g.h : g.ch);
    c.x = (uint32_t)(luma ? g.lmw : 8);
    c.y = (uint32_t)(luma ? 16 : g.cmh);
    c.z = ((d >> 3) & 1u) * 8u;
    c.w = ((d >> 4) & 1u) * 8u;
    s_bd[2 * tid] = a;
    s_bd[2 * tid + 1] = c;
  }
}

// Task t (one chunk) -> frame, chunk index in its segment, first block of the segment.
__device__ __forceinline__ void task_pos(const EncGeom &g, int t, int &frame, int &chunk, int &bbase) {
  const int seg = (int)(((unsigned long long)(uint32_t)t * g.nchunks_magic) >> 40);
  chunk = t - seg * g.nchunks;
  if (g.nseg == 1) {  // one segment per frame (no RST): skip the second division
    frame = seg;
    bbase = 0;
    return;
  }
  frame = (int)(((unsigned long long)(uint32_t)seg * g.nseg_magic) >> 40);
  bbase = (seg - frame * g.nseg) * g.seg_blocks;
}

// chunks per work unit pulled from the counters: 12 (with the per-XCD counters: c2 -6%, c5 -5%
// against 16; 8 and 24 measured too)
constexpr int kBatch = 12;

// DC predictor carried into a chunk that does not follow this wave's previous chunk: the
// quantised DCs of the 8 blocks before it (every possible predecessor: distance <= 8),
// lane 56+i holding block chunk*64-8+i of the segment.  Quantised DC = (pixel sum + 32) >> 6
// exactly.  carry_row: lane loads row (lane & 7) of block (lane >> 3) of those 8 blocks
// (issued early so the load overlaps a chunk's work); carry_finish reduces them.
__device__ __forceinline__ uint64_t carry_row(const uint8_t *fb, const EncGeom &g, int bbase, int chunk, int lane,
                                              const uint4 *s_bd) {
  if (chunk == 0) return 0;
  const BlockPos p = block_pos(g, bbase + chunk * 64 - 8 + (lane >> 3), s_bd);
  const uint8_t *row = fb + p.poff + (size_t)min(p.y0 + (lane & 7), p.ph - 1) * p.stride;
  if (p.x0 + 8 <= p.pw && (((uintptr_t)(row + p.x0)) & 7) == 0)
    return *(const uint64_t *)(row + p.x0);
  uint64_t w = 0;
  for (int x = 0; x < 8; x++) w |= (uint64_t)row[min(p.x0 + x, p.pw - 1)] << (8 * x);
  return w;
}

__device__ __forceinline__ int carry_finish(uint64_t w, int chunk, int lane, bool rc, const EncGeom &g,
                                            const uint32_t *desc) {
  if (chunk == 0) return 128;
  const bool chroma = desc_tab(desc[block_in_mcu(g, chunk * 64 - 8 + (lane >> 3))]) != 0;
  int sum = 0;
#pragma unroll
  for (int x = 0; x < 8; x++) {
    const int p = (int)((w >> (8 * x)) & 255u);
    sum += !rc ? p : (chroma ? range_chroma(p) : range_luma(p));
  }
  sum += __shfl_xor(sum, 1, 64);
  sum += __shfl_xor(sum, 2, 64);
  sum += __shfl_xor(sum, 4, 64);
  const int d = __shfl((sum + 32) >> 6, max(lane - 56, 0) * 8, 64);
  return lane >= 56 ? d : 128;
}

// MODE: kEmitDefault (-huffman default, Annex K tables), kCount (-huffman optimal pass 1:
// per-frame symbol histograms into hist[frame][544] and each block's symbol records, which
// k_emit_syms replays with the frame's own tables).
constexpr int kEmitDefault = 0, kCount = 1;
constexpr int kFrameTabWords = 544;  // AC luma, AC chroma, DC luma, DC chroma (table block layout)

// Pack a chunk's 64 block codes into its slot: a wave prefix-scan of the block lengths gives
// each block's bit offset; blocks up to 128 bits come from their ShiftSink window, longer
// ones from their staging column.  No LDS atomics: lane L's bits occupy words fw..lw.
// Words strictly inside are L's alone; word fw may be shared with earlier lanes and word lw
// with later ones.  Every word has one writer: the lane whose bits cover its first bit
// ("opener"), which ORs in the heads of the lanes that start inside the word, G = segmented
// suffix-OR of heads over lanes with equal fw.  Lane 0 writes the chunk's bit count.
__device__ __forceinline__ void pack_chunk(const ShiftSink &q, bool cur_active, uint32_t *slot,
                                           uint32_t *chunk_bits_t, int lane) {
  const uint32_t incl = wave_incl_scan(q.bits, lane);
  const uint32_t off = incl - q.bits;
  const uint32_t total = lane63(incl);

  const bool has = cur_active && q.bits != 0;
  const uint32_t sft = off & 31, fw = off >> 5;
  const uint32_t lw = has ? (off + q.bits - 1) >> 5 : fw;
  uint32_t head = 0, tail = 0;
  if (has) {
    if (q.bits <= 128 && !q.staged) {
      // the block's words from its end: d[4] = word lw, d[4 - j] = word lw - j, i.e. the
      // right-aligned 128 bits shifted left by t, the free bits after the block in word lw
      const uint32_t t = (32u - ((off + q.bits) & 31u)) & 31u, sh = 32u - t;  // sh in 1..32
      const uint32_t d[5] = {(uint32_t)((uint64_t)q.w0 >> sh),
                             (uint32_t)((((uint64_t)q.w0 << 32) | q.w1) >> sh),
                             (uint32_t)((((uint64_t)q.w1 << 32) | q.w2) >> sh),
                             (uint32_t)((((uint64_t)q.w2 << 32) | q.w3) >> sh), q.w3 << t};
      const uint32_t nmid = lw - fw;  // 0..4
      tail = d[4];
#pragma unroll
      for (int j = 1; j < 4; j++)
        if ((uint32_t)j < nmid) slot[lw - j] = d[4 - j];
      head = nmid == 0 ? d[4] : nmid == 1 ? d[3] : nmid == 2 ? d[2] : nmid == 3 ? d[1] : d[0];
    } else {  // long block: its staged stream shifted into place, 8 words per step
      const uint32_t nws = (q.bits + 31) >> 5, nw = lw - fw + 1;
      const uint32_t *stg = q.stage;
      for (uint32_t m0 = 0; m0 < nw; m0 += 8) {
        uint32_t S[9];
#pragma unroll
        for (int i = 0; i < 9; i++) {  // stream words m0 - 1 .. m0 + 7 (0 outside the stream)
          const uint32_t j = m0 - 1 + (uint32_t)i;
          S[i] = j < nws ? stg[j * 64] : 0u;
        }
#pragma unroll
        for (int i = 0; i < 8; i++) {
          const uint32_t m = m0 + (uint32_t)i;
          const uint32_t F = sft ? (S[i] << (32u - sft)) | (S[i + 1] >> sft) : S[i + 1];
          if (m == 0) head = F;
          if (m + 1 == nw && m > 0) tail = F;
          if (m > 0 && m + 1 < nw) slot[fw + m] = F;
        }
      }
    }
  }
  // Group OR of the heads of the lanes that start inside word fw, needed at the group's
  // first lane.  Heads of one word occupy disjoint bits, so their OR is their sum: with H
  // the inclusive prefix sum of the heads (mod 2^32), the group's OR is H[last] - H[first]
  // + head[first].  The group's last lane is the lane before the next group's first one
  // (ballot of the group starts; lane 63 when none follows): one bpermute.
  const uint32_t fprev = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)fw, 0x138, 0xf, 0xf, false);  // wave_shr:1
  const uint64_t firsts = __ballot(fprev != fw);
  const uint64_t later = lane < 63 ? firsts >> (lane + 1) : 0ull;
  const int last = later ? lane + (int)__builtin_ctzll(later) : 63;
  const uint32_t H = wave_incl_scan(head, lane);
  const uint32_t grp = (uint32_t)__builtin_amdgcn_ds_bpermute(last << 2, (int)H) - H + head;  // valid at group firsts
  // lane + 1's values (DPP wave_shl:1; lane 63 reads the old 0 / ~0u)
  const uint32_t gnext = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)grp, 0x130, 0xf, 0xf, false);
  const uint32_t fnext = (uint32_t)__builtin_amdgcn_update_dpp(-1, (int)fw, 0x130, 0xf, 0xf, false);
  if (has) {
    if (lw > fw) slot[lw] = tail | ((lane < 63 && fnext == lw) ? gnext : 0u);
    if (sft == 0) slot[fw] = grp;  // word-aligned start: this lane opens word fw
  }
  if (lane == 0) *chunk_bits_t = total;
}

// pack_chunk for a chunk whose blocks are all short and none wave-parallel (window path only):
// each block's bits, right-aligned in the queue, are ORed into the wave's LDS words (s_w, zero
// outside a pack, >= 128 words), which coalesced stores move to the slot.  No per-word opener
// logic; same bytes as pack_chunk.  W = 32: blocks of at most 32 bits (w3; two words at most;
// 96% of testsrc 4K q5 chunks), W = 64: at most 64 bits (w2:w3; three words; 2/3 of the
// fractal content's chunks).  A chunk is then at most 64 x W bits.
template <int W>
__device__ __forceinline__ void pack_chunk_short(const ShiftSink &q, uint32_t bits, uint32_t *s_w, uint32_t *slot,
                                                 uint32_t *chunk_bits_t, int lane) {
  const uint32_t incl = wave_incl_scan(bits, lane), off = incl - bits, total = lane63(incl);
  if (bits) {  // bits [off, off + bits), MSB first
    uint32_t *d = s_w + (off >> 5);
    if (W == 32) {
      const uint64_t x = (uint64_t)q.w3 << (64u - (off & 31u) - bits);
      atomicOr(d, (uint32_t)(x >> 32));
      if ((uint32_t)x) atomicOr(d + 1, (uint32_t)x);
    } else {  // emit_block_wave's placement: V << sh fits 96 bits
      const uint64_t v = ((uint64_t)q.w2 << 32) | q.w3;
      const uint32_t sh = 96u - (off & 31u) - bits;
      const uint64_t hi = sh >= 32u ? v << (sh - 32u) : v >> (32u - sh);
      const uint32_t lo = sh >= 32u ? 0u : (uint32_t)(v << sh);
      atomicOr(d, (uint32_t)(hi >> 32));
      if ((uint32_t)hi) atomicOr(d + 1, (uint32_t)hi);
      if (lo) atomicOr(d + 2, lo);
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  const uint32_t nw = (total + 31u) >> 5;
#pragma unroll
  for (uint32_t w = (uint32_t)lane; w < (uint32_t)(2 * W); w += 64)
    if (w < nw) {
      slot[w] = s_w[w];
      s_w[w] = 0u;
    }
  if (lane == 0) *chunk_bits_t = total;
}

// Row pass of one chunk, lane = block: raw rows (8 little-endian words of 8 pixels) ->
// the wave's LDS row image s_pk ([word][lane]; word c*4 + r/2 = column c of rows r, r+1 as
// u16 pairs; output 0 as is, 1-7 + 16384).
template <bool RC>
__device__ __forceinline__ void row_pass(const uint64_t (&raw)[8], int tab, const uint8_t *s_rc,
                                         uint32_t *s_pk, int lane) {
  // Row pass (jfdctint pass 1) in fp32, exactly: every value is an integer or a multiple
  // of 2^-10 below 2^14 (24 significant bits), each fma rounds nothing, and the DESCALE
  // floor((x + 256) / 512) is the single round-to-nearest-even of (x/512 + 2^-10) + M'
  // (M' = kMc = 1.5*2^23 + 16384; kM for output 0), which also leaves x + 16384 (x) in the
  // low 16 mantissa bits: one v_perm packs an output of two rows as a u16 pair into the
  // wave's LDS row image (rows in pairs: exact_coef then reads two rows of a column per word).
  // [RC] swscale tv->pc per pixel from a 512-byte LDS table (clip_u8((p * A21 - B21) >> 21),
  // checked exhaustively in tests/test_oracle.py), OR'ed into the mantissa of M = 1.5*2^23:
  // values then carry the +M bias, which the butterfly's differences cancel and its sums
  // remove with one -2M.
  auto row = [&](int r, float (&o)[8]) {
    const uint32_t lo = (uint32_t)raw[r], hi = (uint32_t)(raw[r] >> 32);
    float p[8];
    p[0] = (float)((lo >> 0) & 255u);  // v_cvt_f32_ubyte0
    p[1] = (float)((lo >> 8) & 255u);  // v_cvt_f32_ubyte1
    p[2] = (float)((lo >> 16) & 255u);  // v_cvt_f32_ubyte2
    p[3] = (float)((lo >> 24) & 255u);  // v_cvt_f32_ubyte3
    p[4] = (float)((hi >> 0) & 255u);  // v_cvt_f32_ubyte0
    p[5] = (float)((hi >> 8) & 255u);  // v_cvt_f32_ubyte1
    p[6] = (float)((hi >> 16) & 255u);  // v_cvt_f32_ubyte2
    p[7] = (float)((hi >> 24) & 255u);  // v_cvt_f32_ubyte3
    float t0, t1, t2, t3;
    if (RC) {
      // LDS address (tab << 8) | pixel in one v_perm, the table byte OR'ed into kM's
      // mantissa: the fp32 value kM + range(p)
#pragma unroll
      for (int x = 0; x < 8; x++) {
        const uint32_t a = __builtin_amdgcn_perm((uint32_t)tab, x < 4 ? lo : hi,
                                                 0x0c0c0400u | (uint32_t)(x & 3));
        p[x] = __uint_as_float(0x4B400000u | (uint32_t)s_rc[a]);
      }
      t0 = (p[0] - 2.0f * kM) + p[7];
      t1 = (p[1] - 2.0f * kM) + p[6];
      t2 = (p[2] - 2.0f * kM) + p[5];
      t3 = (p[3] - 2.0f * kM) + p[4];
    } else {
      t0 = p[0] + p[7];
      t1 = p[1] + p[6];
      t2 = p[2] + p[5];
      t3 = p[3] + p[4];
    }
    const float t7 = p[0] - p[7], t6 = p[1] - p[6], t5 = p[2] - p[5], t4 = p[3] - p[4];
    const float t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
    o[0] = __builtin_fmaf(t10 + t11, 16.0f, kM);  // the row sum: unbiased (0..32640)
    o[4] = __builtin_fmaf(t10 - t11, 16.0f, kMc);
    o[2] = __builtin_fmaf(t13, 10703.0f / 512, __builtin_fmaf(t12, 4433.0f / 512, kRnd)) + kMc;
    o[6] = __builtin_fmaf(t13, 4433.0f / 512, __builtin_fmaf(t12, -10704.0f / 512, kRnd)) + kMc;
    o[1] = __builtin_fmaf(t7, 11363.0f / 512, __builtin_fmaf(t6, 9633.0f / 512,
           __builtin_fmaf(t5, 6437.0f / 512, __builtin_fmaf(t4, 2260.0f / 512, kRnd)))) + kMc;
    o[3] = __builtin_fmaf(t7, 9633.0f / 512, __builtin_fmaf(t6, -2259.0f / 512,
           __builtin_fmaf(t5, -11362.0f / 512, __builtin_fmaf(t4, -6436.0f / 512, kRnd)))) + kMc;
    o[5] = __builtin_fmaf(t7, 6437.0f / 512, __builtin_fmaf(t6, -11362.0f / 512,
           __builtin_fmaf(t5, 2261.0f / 512, __builtin_fmaf(t4, 9633.0f / 512, kRnd)))) + kMc;
    o[7] = __builtin_fmaf(t7, 2260.0f / 512, __builtin_fmaf(t6, -6436.0f / 512,
           __builtin_fmaf(t5, 9633.0f / 512, __builtin_fmaf(t4, -11363.0f / 512, kRnd)))) + kMc;
  };
#pragma unroll
  for (int rp = 0; rp < 4; rp++) {
    float a[8], b[8];
    row(2 * rp, a);
    row(2 * rp + 1, b);
#pragma unroll
    for (int c = 0; c < 8; c++)
      s_pk[(c * 4 + rp) * 64 + lane] = __builtin_amdgcn_perm(__float_as_uint(b[c]), __float_as_uint(a[c]), 0x05040100u);
    __builtin_amdgcn_sched_barrier(0);
  }
}

  // Column pass (jfdctint pass 2) as a float *screen*: the products of pass 2 need up to
  // 31 bits, so fp32 sums are only approximate (|error| < 2^9 before the 2^17 descale).
  // Each AC coefficient is tested against its quantiser threshold widened by a margin
  // (s_thr = B^2, fma(-s, s, B^2) < 0 <=> |s| > B), giving a candidate mask in zigzag
  // order; emit_block quantises the candidates exactly from the integer row image
  // (exact_coef).  Rows 0 and 4 (sums only) are exact, which gives the DC exactly:
  // (((x + 8) >> 4) + 32) >> 6 == floor((sum + 520) / 1024).
// Adaptive skip test: st bit jp (wave-uniform, carried from chunk to chunk) records whether pair
// jp's test skipped a column on the wave's previous test of it.  A pair is tested when it did,
// or on every fourth chunk (retest); a pair whose columns are rarely skippable (detailed
// content) then costs its test a quarter of the time (the test is ~20 VALU per pair).
// The candidate bits are deposited straight at their zigzag positions (mlo: scan positions 0-31,
// mhi: 32-63; r and col are compile-time after unrolling, so each bit costs a shift and an
// and-or): the emission visits candidates in scan order with no scatter step.
__device__ __forceinline__ void column_screen(const uint32_t *s_pk, int lane, const uint32_t *s_skip,
                                              const float *s_thr, int &dc, uint32_t &mlo, uint32_t &mhi,
                                              uint32_t &st, bool retest) {
#pragma unroll
  for (int jp = 0; jp < 4; jp++) {
    __builtin_amdgcn_sched_barrier(0);  // one column pair in flight at a time
    uint32_t w[8];  // w[4h + i]: column 2jp + h of rows 2i (low half), 2i + 1 (high half)
#pragma unroll
    for (int i = 0; i < 8; i++) w[i] = s_pk[(jp * 8 + i) * 64 + lane];
    // Column skip (pairs 1-3): every AC output of a column quantises to zero when the
    // column's row-pass values are small enough.  Rows 1-7 of pass 2 have coefficient
    // sums 0, so |S_k| <= L1(row k) * R / 2 with R = max - min of the column; row 0 is
    // the plain sum, |S_0| <= 8 max|u|.  open_ctx turns the quantiser thresholds into
    // limits on R, max and min (u16 with the +16384 bias), tested with packed u16
    // max/min and saturating subtracts; a column is skipped when every block of the
    // chunk passes (wave ballot), its 8 screen bits are then 0.
    bool skip0 = false, skip1 = false;
    if (jp > 0 && (((st >> jp) & 1u) || retest)) {
      u16x2 ma = as_u16x2(w[0]), na = ma, mb = as_u16x2(w[4]), nb = mb;
#pragma unroll
      for (int i = 1; i < 4; i++) {
        ma = __builtin_elementwise_max(ma, as_u16x2(w[i]));
        na = __builtin_elementwise_min(na, as_u16x2(w[i]));
        mb = __builtin_elementwise_max(mb, as_u16x2(w[4 + i]));
        nb = __builtin_elementwise_min(nb, as_u16x2(w[4 + i]));
      }
      // (column 2jp, column 2jp + 1): each column's even-row and odd-row halves combined
      const u16x2 mx = __builtin_elementwise_max(as_u16x2(__builtin_amdgcn_perm(as_u32(mb), as_u32(ma), 0x05040100u)),
                                                 as_u16x2(__builtin_amdgcn_perm(as_u32(mb), as_u32(ma), 0x07060302u)));
      const u16x2 mn = __builtin_elementwise_min(as_u16x2(__builtin_amdgcn_perm(as_u32(nb), as_u32(na), 0x05040100u)),
                                                 as_u16x2(__builtin_amdgcn_perm(as_u32(nb), as_u32(na), 0x07060302u)));
      const uint32_t t =
          as_u32(__builtin_elementwise_sub_sat(mx - mn, as_u16x2(s_skip[3 * jp - 3]))) |
          as_u32(__builtin_elementwise_sub_sat(mx, as_u16x2(s_skip[3 * jp - 2]))) |
          as_u32(__builtin_elementwise_sub_sat(as_u16x2(s_skip[3 * jp - 1]), mn));
      skip0 = __ballot((t & 0xffffu) != 0u) == 0;
      skip1 = __ballot((t >> 16) != 0u) == 0;
      st = (skip0 || skip1) ? st | (1u << jp) : st & ~(1u << jp);
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
      __builtin_amdgcn_sched_barrier(0);  // one column at a time
      const int col = 2 * jp + h;
      if (h ? skip1 : skip0) continue;  // wave-uniform: no candidates in this column
      float x[8];
#pragma unroll
      for (int r = 0; r < 8; r++)
        x[r] = __uint_as_float(__builtin_amdgcn_perm(0x4B400000u, w[4 * h + r / 2], (r & 1) ? 0x07060302u : 0x07060100u));
      // x = M' + value (M' = kM for column 0, kMc for the others): differences cancel the
      // bias, sums drop it with one -2M'
      const float kB2 = col == 0 ? 2.0f * kM : 2.0f * kMc;
      const float t0 = (x[0] - kB2) + x[7], t7 = x[0] - x[7];
      const float t1 = (x[1] - kB2) + x[6], t6 = x[1] - x[6];
      const float t2 = (x[2] - kB2) + x[5], t5 = x[2] - x[5];
      const float t3 = (x[3] - kB2) + x[4], t4 = x[3] - x[4];
      const float t10 = t0 + t3, t13 = t0 - t3, t11 = t1 + t2, t12 = t1 - t2;
      float sv[8];
      sv[0] = t10 + t11;
      sv[4] = t10 - t11;
      sv[2] = __builtin_fmaf(t13, 10703.0f, t12 * 4433.0f);
      sv[6] = __builtin_fmaf(t13, 4433.0f, t12 * -10704.0f);
      sv[1] = __builtin_fmaf(t7, 11363.0f, __builtin_fmaf(t6, 9633.0f, __builtin_fmaf(t5, 6437.0f, t4 * 2260.0f)));
      sv[3] = __builtin_fmaf(t7, 9633.0f, __builtin_fmaf(t6, -2259.0f, __builtin_fmaf(t5, -11362.0f, t4 * -6436.0f)));
      sv[5] = __builtin_fmaf(t7, 6437.0f, __builtin_fmaf(t6, -11362.0f, __builtin_fmaf(t5, 2261.0f, t4 * 9633.0f)));
      sv[7] = __builtin_fmaf(t7, 2260.0f, __builtin_fmaf(t6, -6436.0f, __builtin_fmaf(t5, 9633.0f, t4 * -11363.0f)));
      const float4 ta = *(const float4 *)(s_thr + col * 8), tb = *(const float4 *)(s_thr + col * 8 + 4);
      const float thr[8] = {ta.x, ta.y, ta.z, ta.w, tb.x, tb.y, tb.z, tb.w};
#pragma unroll
      for (int r = 0; r < 8; r++) {
        if (col == 0 && r == 0) {
          dc = (int)(__float_as_uint(__builtin_fmaf(sv[0], 1.0f / 1024, 0x1.1p-7f) + kM) - 0x4B400000u);
        } else {
          // the sign of B^2 - s^2 at the coefficient's scan position
          const uint32_t neg = __float_as_uint(__builtin_fmaf(-sv[r], sv[r], thr[r]));
          const int z = kZigzagInv[r * 8 + col];
          if (z < 32)
            mlo |= (neg >> 31) << z;
          else
            mhi |= (neg >> 31) << (z - 32);
        }
      }
    }
  }
}

// DC predictor of this lane's block (FFmpeg last_dc, 128 at every segment start): the block
// `delta` before it in coding order (the previous block of the same component) is in this
// chunk (lane - delta) or among the previous chunk's last 8 blocks, whose DCs lanes 56..63
// carry.  One bpermute for both: quantised DCs and carried DCs fit int16.
__device__ __forceinline__ int dc_predictor(int dc, int carry, int delta, bool first_chunk, int lane) {
  const int src_lane = (lane - delta) & 63;
  const uint32_t both = __builtin_amdgcn_ds_bpermute(
      src_lane << 2, (int)(((uint32_t)dc & 0xffffu) | ((uint32_t)carry << 16)));
  const int from_cur = (int)(int16_t)(both & 0xffffu), from_prev = (int)both >> 16;
  return lane >= delta ? from_cur : (first_chunk ? 128 : from_prev);
}

// k_encode's work units per XCD: workgroup i runs on XCD i % 8 (round-robin dispatch), and
// XCD j's waves take the units of the j-th eighth of the launch first (its own counter,
// work_ctr[j * kCtrStride]: neighbouring chunks share the 64-byte sectors at their edges, so
// they meet in one L2), then the other eighths' leftovers.  Correct for any placement.
// NX = 1: one counter for the whole launch (the -huffman optimal counting pass, where the
// per-XCD split measured 2% slower; c2 2-3% faster with NX = 8).
constexpr int kXcds = 8, kCtrStride = 32;  // one 128-byte line per counter
template <int NX>
struct XcdUnits {
  int j, nbatch;
  __device__ __forceinline__ int start(int x) const { return (int)(((long long)x * nbatch) / NX); }
  __device__ __forceinline__ int nw(int x, int nwg) const {  // waves of XCD x
    return ((nwg - x + NX - 1) / NX) * kWavesPerWg;
  }
  // lane 0: the next unit (>= nbatch: none left)
  __device__ __forceinline__ int next(uint32_t *ctr, int nwg) const {
    for (int k = 0; k < NX; k++) {
      const int x = (j + k) & (NX - 1), e = start(x + 1);
      const int u = start(x) + nw(x, nwg) + (int)atomicAdd(ctr + x * kCtrStride, 1u);
      if (u < e) return u;
    }
    return nbatch;
  }
};

// DBG: the MJG_F_DEBUG_COEFS instantiation (quantised blocks out); the product kernels carry
// neither its branch nor its live scalars (k_encode is short of SGPRs: they spill to VGPR lanes).
// (The DCT stage on the matrix cores, dct_mfma, r02-r05, was retired in r06: slower or equal on
// every BASELINE config once the VALU screen skipped columns, profiles/HISTORY.md §4c.)
template <bool RC, int MODE, bool DBG = false>  // RC: yuv420p (tv) input without scale -> swscale tv->pc per pixel
__global__ __launch_bounds__(64 * kWavesPerWg, MODE == kCount ? 4 : kEncWavesPerEU) void k_encode(
    const SegList frames, EncGeom g, const uint32_t *__restrict__ tabs,
    uint32_t *__restrict__ scratch, uint32_t *__restrict__ chunk_bits,
    int16_t *__restrict__ dbg_coefs, uint32_t *__restrict__ work_ctr, int ntasks,
    uint32_t *__restrict__ hist, uint32_t *__restrict__ stage_all,
    uint32_t *__restrict__ syms, uint32_t *__restrict__ symn) {
  constexpr bool EM = MODE == kEmitDefault;  // the AC / DC codes (the counting pass codes nothing)
  __shared__ uint32_t s_ac[EM ? 512 : 1];
  __shared__ uint32_t s_dc[EM ? 32 : 1];
  __shared__ __attribute__((aligned(16))) int32_t s_qc[64];  // qmat column-major: [col][row]
  __shared__ uint8_t s_zz[64];                                // zigzag -> natural index
  __shared__ uint4 s_zd[64];                                  // zigzag -> exact_coef descriptor (zz_desc)
  __shared__ __attribute__((aligned(16))) float s_thr[64];  // screening thresholds^2 [col][row]
  __shared__ __attribute__((aligned(16))) uint32_t s_m2[32];  // pass-2 dot rows as int16 pairs
  __shared__ uint8_t s_rc[RC ? 512 : 1];  // tv->pc: luma [0,256), chroma [256,512)
  __shared__ uint32_t s_desc[8];                   // block-of-MCU descriptors (EncGeom)
  __shared__ uint4 s_bd[16];                       // their plane fields (BlockDesc)
  __shared__ uint32_t s_skip[12];        // column-skip limits, 3 u16x2 words per pair
  __shared__ uint32_t s_pk_all[kWavesPerWg][32 * 64];  // quantised blocks, [word][lane]
  // emit_block_wave's stream words, pack_chunk_short's chunk words
  __shared__ uint32_t s_hv_all[MODE == kEmitDefault ? kWavesPerWg : 1][kHvWords];
  // per wave: the current frame's histogram (kCount; CountSink's 16-bit pairs)
  __shared__ uint32_t s_aux_all[EM ? 1 : kWavesPerWg][EM ? 1 : kCountWords];

  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  if (EM) {
    for (int i = tid; i < 512; i += 64 * kWavesPerWg) s_ac[i] = tabs[i];
    if (tid < 32) s_dc[tid] = tabs[512 + tid];
  }
  if (tid < 64) {
    s_qc[tid] = (int32_t)tabs[544 + tid];
    s_zz[tid] = kZigzag[tid];
    s_zd[tid] = zz_desc(tid, tabs);
    s_thr[tid] = __uint_as_float(tabs[608 + tid]);
    if (tid < 32)
      s_m2[tid] = pass2_pair(tid);
  }
  if (tid < 8) {
    s_desc[tid] = tabs[672 + tid];
  }
  init_block_desc(g, tabs, s_bd, tid);
  if (tid < 12) s_skip[tid] = tabs[680 + tid];
  if (RC)
    for (int i = tid; i < 512; i += 64 * kWavesPerWg)
      s_rc[i] = (uint8_t)(i < 256 ? range_luma(i) : range_chroma(i - 256));
  uint32_t *s_pk = s_pk_all[wave];
  uint32_t *s_hv = s_hv_all[MODE == kEmitDefault ? wave : 0];
  if (MODE == kEmitDefault)
    for (int i = lane; i < kHvWords; i += 64) s_hv[i] = 0u;
  uint32_t *s_aux = s_aux_all[MODE == kEmitDefault ? 0 : wave];
  if (MODE == kCount)
    for (int i = lane; i < kCountWords; i += 64) s_aux[i] = 0;
  int aux_frame = -1;  // frame whose histogram / tables s_aux holds (wave-uniform)
  int aux_chunks = 0;  // chunks counted into s_aux since its last flush
  __syncthreads();  // tables visible; the only workgroup barrier

  const int gw = blockIdx.x * kWavesPerWg + wave;
  const int nbatch = (ntasks + kBatch - 1) / kBatch;
  constexpr int NX = MODE == kEmitDefault ? kXcds : 1;
  const XcdUnits<NX> xu{(int)(blockIdx.x & (NX - 1)), nbatch};
  const int nwg = gridDim.x;
  int u0 = xu.start(xu.j) + (int)(blockIdx.x / NX) * kWavesPerWg + wave;  // static first unit
  if (u0 >= xu.start(xu.j + 1)) {  // none: straight to the counters
    int v = 0;
    if (lane == 0) v = xu.next(work_ctr, nwg);
    u0 = __builtin_amdgcn_readfirstlane(v);
    if (u0 >= nbatch) return;
  }
  const int nblk = g.seg_blocks;  // blocks of one entropy-coded segment
  constexpr bool rc = RC;

  // Units of kBatch consecutive chunks: the first one static (unit gw), the rest
  // pulled from work_ctr (zeroed by k_scan_bits after every launch), so waves whose
  // picture content is cheap take more batches and all waves finish together.
  int t = u0 * kBatch, tend = min(t + kBatch, ntasks);
  uint32_t nb = 0;  // lane 0: the unit after this one
  int frame, chunk, bbase;
  task_pos(g, t, frame, chunk, bbase);
  int b = chunk * 64 + lane;  // block in the segment
  bool active = b < nblk;
  // the chunk's frame base (wave-uniform) and whether it is 8-byte aligned
  auto frame_base = [&](int f) { return seg_frame(frames, f, g.frame_stride); };
  const uint8_t *fb = frame_base(frame);
  uint64_t raw[8];
  bool fast = fetch_rows(raw, fb, ((uintptr_t)fb & 7) == 0, block_pos(g, bbase + b, s_bd), active);
  int carry = carry_finish(carry_row(fb, g, bbase, chunk, lane, s_bd), chunk, lane, rc, g, s_desc);
  uint32_t skip_st = 0xeu;  // column_screen's adaptive skip test: test every pair first

  while (true) {
    // the next unit is reserved at the top of this unit's last chunk (its rows are prefetched
    // midway through it), not when this unit starts: a wave holding a reserved unit while the
    // counter runs dry left the others idle for up to a whole unit at the end of every launch
    if (t + 1 == tend && lane == 0) nb = (uint32_t)xu.next(work_ctr, nwg);
    const uint32_t dsc = s_desc[block_in_mcu(g, b)];
    const int tab = desc_tab(dsc);
    if (active && !fast) fetch_rows_edge(raw, fb, block_pos(g, bbase + b, s_bd));
    int dc = 0;
    row_pass<RC>(raw, tab, s_rc, s_pk, lane);
    // prefetch the next chunk while this one is encoded
    const int cur_frame = frame, cur_chunk = chunk, cur_bbase = bbase;
    const bool cur_active = active;
    int tn = t + 1;
    const bool new_batch = tn >= tend;
    if (new_batch) {
      const int nbu = __builtin_amdgcn_readfirstlane(nb);
      tn = nbu < nbatch ? nbu * kBatch : -1;
    }
    if (tn >= 0) {
      task_pos(g, tn, frame, chunk, bbase);
      b = chunk * 64 + lane;
      active = b < nblk;
      fb = frame_base(frame);
      fast = fetch_rows(raw, fb, ((uintptr_t)fb & 7) == 0, block_pos(g, bbase + b, s_bd), active);
    }
    // a new batch starts at an arbitrary chunk: fetch its predecessors' rows now
    const uint64_t crow = (new_batch && tn >= 0) ? carry_row(fb, g, bbase, chunk, lane, s_bd) : 0;

    uint32_t mlo = 0, mhi = 0;  // candidate mask, scan positions 0-31 / 32-63 (column_screen)
    if (cur_active) {
      column_screen(s_pk, lane, s_skip, s_thr, dc, mlo, mhi, skip_st, (t & 3) == 0);
      if (DBG && g.debug_coefs) {  // natural-order int16 pairs of the exact quantised block
        uint32_t *dst = (uint32_t *)(dbg_coefs +
                                     ((size_t)cur_frame * g.nmcu * g.bpm + cur_bbase + cur_chunk * 64 + lane) * 64);
#pragma unroll 1
        for (int n = 0; n < 64; n += 2) {
          const int a0 = n == 0 ? dc : exact_coef(s_pk + lane, n, s_m2, s_qc);
          const int a1 = exact_coef(s_pk + lane, n + 1, s_m2, s_qc);
          dst[n >> 1] = ((uint32_t)a0 & 0xffffu) | ((uint32_t)a1 << 16);
        }
      }
    }
    const uint64_t mask = ((uint64_t)mhi << 32) | mlo;

    // DC predictor (FFmpeg last_dc, 128 at every segment start): shuffle within the chunk,
    // else the carried DCs of the previous chunk.
    const int diff = dc - dc_predictor(dc, carry, desc_delta(dsc), cur_chunk == 0, lane);
    carry = dc;

    if (MODE == kCount && (cur_frame != aux_frame || aux_chunks == kCountFlush)) {  // flush the counts
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's LDS traffic is done
      if (aux_frame >= 0) flush_counts(s_aux, hist + (size_t)aux_frame * kFrameTabWords, lane);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      aux_frame = cur_frame;
      aux_chunks = 0;
    }
    if (MODE == kCount) {
      CountSink cs{s_aux + tab * 128, s_aux + 256 + tab * 8, syms + (size_t)t * kSymCap * 64 + lane};
      // the heavy blocks wave-parallel, as the default-table encode codes them
      const uint64_t wide = wave_parallel_blocks(cur_active ? __popcll(mask) : 0);
      if (cur_active && !((wide >> lane) & 1ull)) emit_block(s_pk + lane, mask, diff, s_zd, s_m2, cs);
      uint32_t nsym = cs.n;
      for (uint64_t hw = wide; hw; hw &= hw - 1) {
        const int h = (int)__builtin_ctzll(hw);
        const uint32_t nh = count_block_wave(s_pk, h, __builtin_amdgcn_readlane(diff, h),
                                             __builtin_amdgcn_readlane(tab, h), s_zd, s_m2, s_aux,
                                             syms + (size_t)t * kSymCap * 64 + h, lane);
        if (lane == h) nsym = nh;
      }
      aux_chunks++;
      symn[(size_t)t * 64 + lane] = nsym;
      if (tn < 0) break;
      if (new_batch) {
        carry = carry_finish(crow, chunk, lane, rc, g, s_desc);
        tend = min(tn + kBatch, ntasks);
      }
      t = tn;
      continue;
    }
    ShiftSink q;
    q.act = s_ac + tab * 256;
    q.dct = s_dc + tab * 16;
    uint32_t *stage_w = stage_all + (size_t)gw * 64 * kStageWords;
    q.stage = stage_w + lane;
    const uint64_t wide = wave_parallel_blocks(cur_active ? __popcll(mask) : 0);
    if (cur_active && !((wide >> lane) & 1ull)) {
      emit_block(s_pk + lane, mask, diff, s_zd, s_m2, q);
      q.finish();
    }
    if (wide) {  // the heavy blocks, one wave-parallel block at a time
      for (uint64_t hw = wide; hw; hw &= hw - 1) {
        const int h = (int)__builtin_ctzll(hw);
        const uint32_t nb = emit_block_wave(s_pk, h, __builtin_amdgcn_readlane(diff, h),
                                            __builtin_amdgcn_readlane(tab, h), s_zd, s_m2, s_ac, s_dc,
                                            s_hv, stage_w, lane);
        if (lane == h) {
          q.bits = nb;
          q.staged = true;
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // staged words visible to pack_chunk's lanes
    }
    const uint32_t qbits = cur_active ? q.bits : 0u;
    if (__ballot(qbits > 32u || q.staged) == 0ull)
      pack_chunk_short<32>(q, qbits, s_hv, scratch + (size_t)t * kSlotWords, chunk_bits + t, lane);
    else if (__ballot(qbits > 64u || q.staged) == 0ull)
      pack_chunk_short<64>(q, qbits, s_hv, scratch + (size_t)t * kSlotWords, chunk_bits + t, lane);
    else
      pack_chunk(q, cur_active, scratch + (size_t)t * kSlotWords, chunk_bits + t, lane);
    if (tn < 0) break;
    if (new_batch) {
      carry = carry_finish(crow, chunk, lane, rc, g, s_desc);
      tend = min(tn + kBatch, ntasks);
    }
    t = tn;
  }
  if (MODE == kCount && aux_frame >= 0) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    flush_counts(s_aux, hist + (size_t)aux_frame * kFrameTabWords, lane);
  }
}

// ------------------------------------------------------------ k_emit_syms
// -huffman optimal, emission pass: every block's symbols as the counting pass recorded
// them (CountSink), coded with the frame's tables (k_huff_build) and packed as k_encode
// packs them.  No pixels, no DCT: one wave per chunk, lane = block; the record words are
// loaded 8 per step (4: 2.5% slower on c1).  Persistent waves (the long-block staging columns are per wave).
__global__ __launch_bounds__(64 * kWavesPerWg) void k_emit_syms(
    EncGeom g, const uint32_t *__restrict__ tabs, const uint32_t *__restrict__ ftabs,
    const uint32_t *__restrict__ syms, const uint32_t *__restrict__ symn, uint32_t *__restrict__ scratch,
    uint32_t *__restrict__ chunk_bits, uint32_t *__restrict__ stage_all, int ntasks) {
  __shared__ uint32_t s_aux_all[kWavesPerWg][kFrameTabWords];
  __shared__ uint32_t s_desc[8];
  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  if (tid < 8) s_desc[tid] = tabs[672 + tid];
  __syncthreads();
  uint32_t *s_aux = s_aux_all[wave];
  const int nwaves = gridDim.x * kWavesPerWg, gw = blockIdx.x * kWavesPerWg + wave;
  int aux_frame = -1;
  // the chunk's symbol count and first 8 records are loaded one chunk ahead, only the rows the
  // block has (a 128-byte line of a record row is fetched when one of its 32 lanes needs it:
  // 1.4x the records on testsrc 1080p q5, against 2.6x for 8 rows read unconditionally; k_emit_syms
  // reads 0.34 GB instead of 0.49 per 250-frame launch, c1 -0.7%, natural -1.7%,
  // profiles/r06/c1_emit_predicated_reads_ab.txt)
  uint32_t n_nx = 0, e_nx[8] = {0u, 0u, 0u, 0u, 0u, 0u, 0u, 0u};
  auto head = [&](int tt) {
    int frame, chunk, bbase;
    task_pos(g, tt, frame, chunk, bbase);
    const int b = chunk * 64 + lane;
    n_nx = b < g.seg_blocks ? symn[(size_t)tt * 64 + lane] : 0u;
    const uint32_t *rec = syms + (size_t)tt * kSymCap * 64 + lane;
    e_nx[0] = rec[0];  // every block has >= 2 symbols (the DC, and the EOB or an AC)
    e_nx[1] = rec[64];
#pragma unroll
    for (int i = 2; i < 8; i++)
      if (n_nx > (uint32_t)i) e_nx[i] = rec[i * 64];
  };
  // a wave takes a run of consecutive chunks: one frame's tables serve the whole run (taking
  // every nwaves-th chunk reloaded the tables for every chunk)
  const int per = (ntasks + nwaves - 1) / nwaves, t0 = gw * per, t1 = min(t0 + per, ntasks);
  if (t0 < t1) head(t0);
  for (int t = t0; t < t1; t++) {
    int frame, chunk, bbase;
    task_pos(g, t, frame, chunk, bbase);
    const uint32_t n = n_nx;
    uint32_t e[8] = {e_nx[0], e_nx[1], e_nx[2], e_nx[3], e_nx[4], e_nx[5], e_nx[6], e_nx[7]};
    if (t + 1 < t1) head(t + 1);
    if (frame != aux_frame) {  // the frame's code tables into the wave's LDS
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      for (int i = lane; i < kFrameTabWords; i += 64) s_aux[i] = ftabs[(size_t)frame * kFrameTabWords + i];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      aux_frame = frame;
    }
    const int b = chunk * 64 + lane;
    const bool active = b < g.seg_blocks;
    const int tab = desc_tab(s_desc[block_in_mcu(g, b)]);
    ShiftSink q;
    q.act = s_aux + tab * 256;
    q.dct = s_aux + 512 + tab * 16;
    q.stage = stage_all + (size_t)gw * 64 * kStageWords + lane;
    const uint32_t *rec = syms + (size_t)t * kSymCap * 64 + lane;
    for (uint32_t j0 = 0; j0 < n; j0 += 8) {
      if (j0) {
#pragma unroll
        for (int i = 0; i < 8; i++) e[i] = j0 + i < n ? rec[(j0 + i) * 64] : 0u;
      }
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if (j0 + i >= n) break;
        const uint32_t v = (e[i] >> 16) & 0xffu, mant = e[i] & 0xffffu;
        if (e[i] >> 31)
          q.dc((int)v, mant);
        else
          q.ac((int)v, (int)(v & 15u), mant);
      }
    }
    q.finish();
    pack_chunk(q, active, scratch + (size_t)t * kSlotWords, chunk_bits + t, lane);
  }
}

// ------------------------------------------------------------- k_huff_build
// -huffman optimal tables of one (frame, table) per 64-thread workgroup, restating
// libavcodec/mjpegenc_huffman.c (ff_mjpeg_encode_huffman_close ->
// ff_mjpegenc_huffman_compute_bits) and libavutil/qsort.h AV_QSORT exactly (see
// oracle/mjpeg_oracle.c for the CPU restatement this is tested against):
//   1. nonzero counts in ascending symbol order + the dummy symbol 256 with count 0;
//   2. AV_QSORT by count (lane 0; its tie order decides which equal-count symbols get
//      the longer codes, so it is reproduced step for step);
//   3. package-merge lists X_0..X_15 (X_t = merge of the leaves and the pairwise packages
//      of X_{t-1}, a package first on equal weight), merged in parallel by rank: a leaf
//      lands after the packages of weight <= its own, a package after the leaves lighter
//      than it; only each entry's weight and leaf/package tag are kept;
//   4. X_16 = packages of X_15; its first m = min(n-1, |X_16|) entries are selected, which
//      selects a prefix of every X_t: s_15 = 2m, and s_{t-1} = 2 * (packages among the
//      first s_t entries of X_t).  A leaf's code length is the number of lists whose
//      selected prefix holds it;
//   5. BITS/HUFFVAL ordered by (length, symbol) and canonical codes
//      (ff_mjpeg_build_huffman_codes).
// Table t: 0 DC luma, 1 DC chroma, 2 AC luma, 3 AC chroma.  Outputs: ftabs[f][544]
// ((len << 16) | code, table block layout), dht[f][t][kDhtSlot] (BITS[1..16] then
// HUFFVAL) and dht_nval[f][t].
constexpr int kDhtSlot = 16 + 256;
constexpr int kPmMax = 520;  // >= 257 leaves + 257 packages

__device__ void av_qsort_pairs(int *val, int *key, int num) {
  int stack[64][2];
  int sp = 1;
  stack[0][0] = 0;
  stack[0][1] = num - 1;
#define MJG_SWAP(a, b)                     \
  do {                                     \
    const int ia_ = (a), ib_ = (b);        \
    const int tk_ = key[ia_], tv_ = val[ia_]; \
    key[ia_] = key[ib_];                   \
    val[ia_] = val[ib_];                   \
    key[ib_] = tk_;                        \
    val[ib_] = tv_;                        \
  } while (0)
#define MJG_CMP(a, b) (key[a] - key[b])
  while (sp) {
    int start = stack[--sp][0];
    int end = stack[sp][1];
    while (start < end) {
      if (start < end - 1) {
        bool checksort = false;
        int right = end - 2, left = start + 1;
        int mid = start + ((end - start) >> 1);
        if (MJG_CMP(start, end) > 0) {
          if (MJG_CMP(end, mid) > 0)
            MJG_SWAP(start, mid);
          else
            MJG_SWAP(start, end);
        } else {
          if (MJG_CMP(start, mid) > 0)
            MJG_SWAP(start, mid);
          else
            checksort = true;
        }
        if (MJG_CMP(mid, end) > 0) {
          MJG_SWAP(mid, end);
          checksort = false;
        }
        if (start == end - 2) break;
        MJG_SWAP(end - 1, mid);
        while (left <= right) {
          while (left <= right && MJG_CMP(left, end - 1) < 0) left++;
          while (left <= right && MJG_CMP(right, end - 1) > 0) right--;
          if (left <= right) {
            MJG_SWAP(left, right);
            left++;
            right--;
          }
        }
        MJG_SWAP(end - 1, left);
        if (checksort && (mid == left - 1 || mid == left)) {
          mid = start;
          while (mid < end && MJG_CMP(mid, mid + 1) <= 0) mid++;
          if (mid == end) break;
        }
        if (end - left < left - start) {
          stack[sp][0] = start;
          stack[sp++][1] = right;
          start = left + 1;
        } else {
          stack[sp][0] = left + 1;
          stack[sp++][1] = end;
          end = right;
        }
      } else {
        if (MJG_CMP(start, end) > 0) MJG_SWAP(start, end);
        break;
      }
    }
  }
#undef MJG_SWAP
#undef MJG_CMP
}

__global__ __launch_bounds__(64) void k_huff_build(const uint32_t *__restrict__ hist,
                                                   uint32_t *__restrict__ ftabs,
                                                   uint8_t *__restrict__ dht,
                                                   uint32_t *__restrict__ dht_nval) {
  __shared__ int s_val[260], s_key[260];   // leaves: symbol, count (sorted by count)
  __shared__ int s_w[2][kPmMax];            // weights of X_{t-1} / X_t
  __shared__ uint8_t s_tag[16][kPmMax];     // 1 = leaf entry of X_t
  __shared__ int s_pre[17];                 // leaves in the selected prefix of X_t
  __shared__ int s_len[256];                // code length per symbol
  __shared__ uint32_t s_mask[17][8];        // symbols per length (bitmap)
  __shared__ int s_bits[17], s_off[17], s_first[17];
  __shared__ int s_n;
  const int f = blockIdx.x >> 2, t = blockIdx.x & 3, lane = threadIdx.x;
  const uint32_t *h = hist + (size_t)f * kFrameTabWords + (t < 2 ? 512 + 16 * t : 256 * (t - 2));
  const int nb = t < 2 ? 16 : 256;

  // 1. compaction in ascending symbol order
  int n = 0;
  for (int base = 0; base < nb; base += 64) {
    const int sym = base + lane;
    const uint32_t c = sym < nb ? h[sym] : 0u;
    const uint64_t m = __ballot(c != 0);
    const int pos = n + __popcll(m & ((1ull << lane) - 1ull));
    if (c) {
      s_val[pos] = sym;
      s_key[pos] = (int)c;
    }
    n += __popcll(m);
  }
  for (int i = lane; i < 256; i += 64) s_len[i] = 0;
  for (int i = lane; i < 17 * 8; i += 64) (&s_mask[0][0])[i] = 0;
  if (lane == 0) {
    s_val[n] = 256;
    s_key[n] = 0;
    av_qsort_pairs(s_val, s_key, n + 1);  // 2.
  }
  __syncthreads();
  const int size = n + 1;

  // 3. forward lists
  int len_prev = 0;  // |X_{t-1}|
  for (int lt = 0; lt < 16; lt++) {
    int *prev = s_w[(lt + 1) & 1], *cur = s_w[lt & 1];
    const int np = len_prev >> 1;
    for (int i = lane; i < size; i += 64) {  // leaf i: after the packages with weight <= key
      const int key = s_key[i];
      int lo = 0, hi = np;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (prev[2 * mid] + prev[2 * mid + 1] <= key) lo = mid + 1; else hi = mid;
      }
      cur[i + lo] = key;
      s_tag[lt][i + lo] = 1;
    }
    for (int j = lane; j < np; j += 64) {  // package j: after the leaves lighter than it
      const int w = prev[2 * j] + prev[2 * j + 1];
      int lo = 0, hi = size;
      while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (s_key[mid] < w) lo = mid + 1; else hi = mid;
      }
      cur[j + lo] = w;
      s_tag[lt][j + lo] = 0;
    }
    len_prev = size + np;
    __syncthreads();
  }
  // 4. selection, backwards
  {
    const int m = min(size - 1, len_prev >> 1);  // X_16 = packages of X_15
    int sel = 2 * m;                              // wave-uniform
    for (int lt = 15; lt >= 1; lt--) {
      int leaves = 0;
      for (int k = lane; k < sel; k += 64) leaves += s_tag[lt][k];
      leaves = wave_sum(leaves);
      if (lane == 0) s_pre[lt] = leaves;
      sel = 2 * (sel - leaves);
    }
    if (lane == 0) s_pre[0] = sel;
  }
  __syncthreads();
  for (int i = lane; i < size; i += 64) {
    int L = 0;
#pragma unroll
    for (int lt = 0; lt < 16; lt++) L += i < s_pre[lt] ? 1 : 0;
    const int sym = s_val[i];
    if (sym < 256 && L > 0) {
      s_len[sym] = L;
      atomicOr(&s_mask[L][sym >> 5], 1u << (sym & 31));
    }
  }
  __syncthreads();
  // 5. BITS / HUFFVAL by (length, symbol), canonical codes
  if (lane == 0) {
    int off = 0, code = 0;
    for (int L = 1; L <= 16; L++) {
      int c = 0;
      for (int w = 0; w < 8; w++) c += __popc(s_mask[L][w]);
      s_bits[L] = c;
      s_off[L] = off;
      s_first[L] = code;
      off += c;
      code = (code + c) << 1;
    }
    s_n = off;
  }
  __syncthreads();
  uint8_t *d = dht + ((size_t)f * 4 + t) * kDhtSlot;
  if (lane >= 1 && lane <= 16) d[lane - 1] = (uint8_t)s_bits[lane];
  uint32_t *ft = ftabs + (size_t)f * kFrameTabWords + (t < 2 ? 512 + 16 * t : 256 * (t - 2));
  for (int sym = lane; sym < nb; sym += 64) {
    const int L = s_len[sym];
    uint32_t e = 0;
    if (L) {
      int rank = 0;
      for (int w = 0; w < (sym >> 5); w++) rank += __popc(s_mask[L][w]);
      rank += __popc(s_mask[L][sym >> 5] & ((1u << (sym & 31)) - 1u));
      const int k = s_off[L] + rank;
      d[16 + k] = (uint8_t)sym;
      e = ((uint32_t)L << 16) | (uint32_t)(s_first[L] + rank);
    }
    ft[sym] = e;
  }
  if (lane == 0) dht_nval[(size_t)f * 4 + t] = (uint32_t)s_n;
}

// The stuffing tail's waves (k_scan_bits, k_count_ff, k_scan_ff, k_write) run at wave
// priority 2 when the submit's stream is light.  They share SIMDs with the next submit's
// k_encode waves, which are older, and the SIMD arbiter issues the oldest wave first: at
// priority 0 a submit's tail ended ~590 us after its k_encode (~100 us of work), and the host,
// whose sync of that submit frees the slot the submit after next reuses, waited for it.  At 2
// it ends ~260 us after; c5 +14%, c4 +1%, c2 within noise, but natural -1.3% (bench.py;
// profiles/r04ad_tail_wave_priority.txt, r04ae_tail_wave_priority_levels.txt): a heavy stream's
// tail (2-4x the bytes) then takes that much more issue from k_encode.  So the raise is kept to
// submits whose first segment averages under kTailLightBits per chunk (BASELINE's testsrc
// workloads 740-1440 bits, the fractal content 2190, noise-patches 3340).  The test reads the
// first segment's bit count, so the scans that produce it (k_scan_bits, k_scan_bits_seg: a few
// microseconds, before any count exists) always run at kTailPrio; k_count_ff, k_scan_ff and
// k_write apply the test with the segment's chunk count.
constexpr int kTailPrio = 2;
constexpr uint32_t kTailLightBits = 1800;
__device__ __forceinline__ void tail_priority(const uint32_t *seg_bits, int nchunks) {
  if ((uint32_t)__builtin_amdgcn_readfirstlane((int)seg_bits[0]) < kTailLightBits * (uint32_t)nchunks)
    __builtin_amdgcn_s_setprio(kTailPrio);
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

// Per-frame exclusive scan of the chunk bit lengths.  Lengths are clamped to the slot
// size first, so a corrupted length can never send the realign/stuff kernels outside
// their slots (defence in depth; k_encode never writes more than a slot).
__global__ __launch_bounds__(1024) void k_scan_bits(uint32_t *__restrict__ chunk_bits,
                                                    uint32_t *__restrict__ chunk_off,
                                                    uint32_t *__restrict__ frame_bits, int nchunks,
                                                    uint32_t *__restrict__ work_ctr,
                                                    uint32_t *__restrict__ status,
                                                    uint32_t *__restrict__ done, int ndone) {
  const int f = blockIdx.x;
  __builtin_amdgcn_s_setprio(kTailPrio);
  if (f == 0 && threadIdx.x < kXcds) work_ctr[threadIdx.x * kCtrStride] = 0;  // k_encode's unit counters
  if (f == 0 && threadIdx.x == 0) *status = 0;  // output overflow flag, set by k_write
  {  // k_count_ff's ticket counters
    const int i = f * 1024 + (int)threadIdx.x;
    if (i < ndone) done[i] = 0;
  }
  uint32_t *cb = chunk_bits + (size_t)f * nchunks;
  for (int i = threadIdx.x; i < nchunks; i += 1024) cb[i] = min(cb[i], (uint32_t)kSlotWords * 32u);
  __syncthreads();
  const uint32_t t = block_excl_scan(cb, chunk_off + (size_t)f * nchunks, nchunks);
  if (threadIdx.x == 0) frame_bits[f] = t;
}

// RST mode: the same per segment with one wave per segment (a segment is one MCU row, a
// few dozen chunks), 4 segments per 256-thread workgroup.
__device__ __forceinline__ uint32_t wave_excl_scan_arr(const uint32_t *in, uint32_t *out, int n, int lane) {
  uint32_t carry = 0;
  for (int i0 = 0; i0 < n; i0 += 64) {
    const int i = i0 + lane;
    const uint32_t v = i < n ? in[i] : 0u;
    const uint32_t incl = wave_incl_scan(v, lane);
    if (i < n) out[i] = carry + incl - v;
    carry += lane63(incl);
  }
  return carry;
}

__global__ __launch_bounds__(256) void k_scan_bits_seg(uint32_t *__restrict__ chunk_bits,
                                                       uint32_t *__restrict__ chunk_off,
                                                       uint32_t *__restrict__ seg_bits, int nchunks,
                                                       int nsegs, uint32_t *__restrict__ work_ctr,
                                                       uint32_t *__restrict__ status,
                                                       uint32_t *__restrict__ done, int ndone) {
  const int sg = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  __builtin_amdgcn_s_setprio(kTailPrio);
  if (blockIdx.x == 0 && threadIdx.x < kXcds) work_ctr[threadIdx.x * kCtrStride] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) *status = 0;
  {  // k_count_ff's ticket counters
    const int i = blockIdx.x * 256 + (int)threadIdx.x;
    if (i < ndone) done[i] = 0;
  }
  if (sg >= nsegs) return;
  uint32_t *cb = chunk_bits + (size_t)sg * nchunks;
  for (int i = lane; i < nchunks; i += 64) cb[i] = min(cb[i], (uint32_t)kSlotWords * 32u);
  const uint32_t t = wave_excl_scan_arr(cb, chunk_off + (size_t)sg * nchunks, nchunks, lane);
  if (lane == 0) seg_bits[sg] = t;
}

// ------------------------------------------------------------------ the stuffing tail
// Three launches after k_scan_bits, on *groups* of kChunksPerWave consecutive chunks of an
// entropy-coded segment (the frame unless RST mode), one wave per group:
//   k_count_ff  realigns the group's words to the segment's bit offsets and counts their 0xFF
//               bytes (group_ff)
//   k_scan_ff   per frame: scans of the group counts and segment sizes, the frame's size; the
//               last frame to finish (one ticket per frame) places every frame (frame_offsets)
//   k_write     the same words again, byte-stuffed (ff_mjpeg_escape_FF): a word without 0xFF
//               is one (unaligned) dword store; the frame's first group writes the header, a
//               segment's last group its RSTn / EOI
// The tail runs beside the next submit's k_encode, whose VALU issue it shares, so its cost per
// word is kept to a few dozen VALU instructions per 64-word round (group_values).
constexpr int kChunksPerWave = 32;  // chunks per group (lanes 0..G hold their metadata)
constexpr int kTailRounds = 4;      // 64-word rounds whose slot loads are issued together
static_assert(kChunksPerWave * kSlotWords < (1 << 17), "group word offsets are 17-bit fields");

// A group: chunks c0 .. c0 + n - 1 of segment s, owning words [k0, k1) of the segment's
// unstuffed scan (a word belongs to the chunk holding its first bit: chunk c owns
// [ceil(O_c / 32), ceil(O_{c+1} / 32))).  Lane j < n holds chunk j's packed metadata:
//   bits  0-16  rsw: its first owned word - k0
//   bits 17-21  off: 32 * ceil(O / 32) - O, the slot bit where its first owned word starts
//   bits 22-26  rem - 1: bits of the chunk in its last owned word (1..32)
//   bit  27     a next chunk exists in the segment
// lane n: rsw = k1 - k0 (the end of the group's words).
struct GroupWords {
  int s, c0, n;
  uint32_t T;         // segment bits
  uint32_t k0, k1;
  uint32_t info;
  const uint32_t *slot0;  // scratch slot of chunk c0
};

__device__ __forceinline__ GroupWords group_words(const uint32_t *scratch, const uint32_t *chunk_bits,
                                                  const uint32_t *chunk_off, const uint32_t *seg_bits,
                                                  int nchunks, int gps, int gi, int lane) {
  GroupWords g;
  g.s = gi / gps;
  g.c0 = (gi - g.s * gps) * kChunksPerWave;
  g.n = min(kChunksPerWave, nchunks - g.c0);
  g.T = seg_bits[g.s];
  const size_t i0 = (size_t)g.s * nchunks + g.c0;
  g.slot0 = scratch + i0 * kSlotWords;
  const uint32_t O = lane < g.n ? chunk_off[i0 + lane] : 0u, L = lane < g.n ? chunk_bits[i0 + lane] : 0u;
  const uint32_t end = O + L;
  const uint32_t gend = __builtin_amdgcn_readlane(end, g.n - 1);
  g.k0 = (__builtin_amdgcn_readfirstlane(O) + 31) >> 5;
  g.k1 = (gend + 31) >> 5;
  const uint32_t sw = (O + 31) >> 5, lw = (end + 31) >> 5;  // first owned word, one past the last
  const uint32_t rem = end - 32 * (lw - 1);                    // 1..32
  g.info = lane < g.n ? (sw - g.k0) | ((32 * sw - O) << 17) | ((rem - 1) << 22) |
                            ((uint32_t)(g.c0 + lane + 1 < nchunks) << 27)
         : lane == g.n ? g.k1 - g.k0 : 0u;
  return g;
}

__device__ __forceinline__ uint32_t bperm(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}

// Words kb + 64 i + lane (i < R) of the segment's unstuffed scan, 32 bits MSB first; lanes at
// or past k1 compute garbage the caller masks (their loads stay inside chunk 0's words).
//   owner c: the chunk starts inside the window are marked in the wave's LDS bytes; one ballot
//            per round counts those at or before the lane's word
//   A:       chunk c's slot word under the word's first bit (every lane); lane + 1's A is the
//            next slot word of the chunk, or at the chunk's last owned word the next chunk's
//            first word (it owns word k + 1 from that word's bit 0); lane 63 and the group's last
//            word load that one themselves (B), and a chunk's last word whose bits span two slot
//            words loads the second (X), all in the same batch
//   value:   A:next funnel-shifted by off; at a chunk's last word the next chunk's first bits
//            follow its rem bits, and past the segment's last bit the 1-bit padding to a byte
//            boundary (ff_mjpeg_escape_FF pad).  No masking: k_encode zero-fills every slot word
//            past its chunk's last bit, and X / B are loaded only where they hold chunk bits.
template <int R>
__device__ __forceinline__ void group_values(const GroupWords &g, uint32_t kb, uint8_t *marks, int lane,
                                             uint32_t (&v)[R]) {
  const uint32_t span = 64u * R;
  const uint32_t rsw = g.info & 0x1ffffu, wk = kb - g.k0;  // window start, relative to k0
  const bool mk = lane >= 1 && lane < g.n && rsw >= wk && rsw < wk + span;
  if (mk) marks[rsw - wk] = 1;
  int base = __popcll(__ballot(lane >= 1 && lane < g.n && rsw < wk));
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  int own[R];
#pragma unroll
  for (int i = 0; i < R; i++) {
    const uint32_t mark = marks[64 * i + lane];
    const uint64_t m = __ballot(mark != 0);
    // chunk starts at or before the lane's word: mbcnt counts the ballot bits below the lane
    own[i] = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u)) +
             (int)mark;
    base += __popcll(m);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if (mk) marks[rsw - wk] = 0;
  uint32_t A[R], B[R], X[R], inf[R];
  bool bnd[R], own_nx[R];
#pragma unroll
  for (int i = 0; i < R; i++) {
    const uint32_t r = wk + 64u * i + (uint32_t)lane;  // word - k0
    const bool valid = r < g.k1 - g.k0;  // lanes past k1: chunk 0's first word, no X / B loads
    const int c = valid ? own[i] : 0;
    inf[i] = bperm(g.info, c);
    const uint32_t nsw = bperm(g.info, c + 1) & 0x1ffffu;
    const uint32_t wi = valid ? r - (inf[i] & 0x1ffffu) : 0u;  // slot word under the first bit
    const uint32_t off = (inf[i] >> 17) & 31u, rem = ((inf[i] >> 22) & 31u) + 1u;
    bnd[i] = valid && r + 1 == nsw;  // chunk c's last owned word
    own_nx[i] = valid && (lane == 63 || r + 1 == g.k1 - g.k0);  // lane + 1 does not hold word k + 1
    // 32-bit offsets from the group's first slot (the wave-uniform base: saddr loads)
    const uint8_t *s0 = (const uint8_t *)g.slot0;  // byte offsets < 2^32: one 32-bit VGPR each
    const uint32_t oa = (__umul24((uint32_t)c, (uint32_t)kSlotWords) + wi) << 2;
    A[i] = *(const uint32_t *)(s0 + oa);
    X[i] = (bnd[i] && off && rem > 32u - off) ? *(const uint32_t *)(s0 + oa + 4u) : 0u;
    const bool has_next = (inf[i] >> 27) & 1u;
    B[i] = (own_nx[i] && (!bnd[i] || (rem < 32u && has_next)))
               ? *(const uint32_t *)(s0 + (bnd[i] ? __umul24((uint32_t)c + 1u, (uint32_t)kSlotWords * 4u) : oa + 4u))
               : 0u;
  }
#pragma unroll
  for (int i = 0; i < R; i++) {
    const uint32_t k = kb + 64u * i + (uint32_t)lane;
    const uint32_t nx = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)A[i], 0x130, 0xf, 0xf, false);  // wave_shl:1
    const uint32_t next = own_nx[i] ? B[i] : nx;
    const uint32_t off = (inf[i] >> 17) & 31u, rem = ((inf[i] >> 22) & 31u) + 1u;
    const uint32_t lo = off ? (bnd[i] ? X[i] : next) : A[i];
    uint32_t w = __builtin_amdgcn_alignbit(A[i], lo, (32u - off) & 31u);
    if (bnd[i] && rem < 32u) w |= next >> rem;  // the next chunk's first bits (0 past the segment)
    const uint32_t endk = g.T - 32 * k;  // the segment ends in this word: 1-bit padding
    if (endk < 32u) {
      const uint32_t pad = (8u - (g.T & 7u)) & 7u;
      w |= (0xffffffffu >> endk) & ~(endk + pad >= 32u ? 0u : (0xffffffffu >> (endk + pad)));
    }
    v[i] = w;
  }
}

// 0xFF bytes of a word (exact per byte: no carries between bytes)
__device__ __forceinline__ uint32_t ff_bytes(uint32_t v) {
  const uint32_t y = ~v;
  const uint32_t t = ~(((y & 0x7f7f7f7fu) + 0x7f7f7f7fu) | y | 0x7f7f7f7fu);  // 0x80 per zero byte of y
  return (uint32_t)__popc(t);
}

// agent-scope (all XCDs) store / load of the frame sizes k_scan_ff's last frame reads
__device__ __forceinline__ void st_agent64(uint64_t *p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent64(const uint64_t *p) {
  return __hip_atomic_load(const_cast<uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// frame header length: the default header, or (-huffman optimal) the default header without
// its 348 table values plus the frame's own (k_huff_build's value counts)
__device__ __forceinline__ uint32_t frame_hdr_len(int f, int hdr_len, const uint32_t *dht_nval) {
  if (!dht_nval) return (uint32_t)hdr_len;
  const uint32_t *nv = dht_nval + 4 * (size_t)f;
  return (uint32_t)(hdr_len - 348) + nv[0] + nv[1] + nv[2] + nv[3];
}

// Wave per group: the group's words realigned into the segment's contiguous stream (word k of
// segment s at stream[s * nchunks * kSlotWords + k], coalesced), and the 0xFF bytes among
// them -> group_ff[gi].  (Bytes of the segment's last word past its padding are 0x00, so whole
// words are counted.)
__global__ __launch_bounds__(256) void k_count_ff(const uint32_t *__restrict__ scratch,
                                                  const uint32_t *__restrict__ chunk_bits,
                                                  const uint32_t *__restrict__ chunk_off,
                                                  const uint32_t *__restrict__ seg_bits,
                                                  uint32_t *__restrict__ group_ff, int nchunks, int gps,
                                                  int ngroups, uint32_t *__restrict__ stream) {
  __shared__ uint8_t s_marks[4][64 * kTailRounds];
  tail_priority(seg_bits, nchunks);
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int gi = blockIdx.x * 4 + wave;  // wave-uniform: the group's pointers are scalar
  for (int i = lane; i < 64 * kTailRounds; i += 64) s_marks[wave][i] = 0;
  if (gi >= ngroups) return;
  const GroupWords g = group_words(scratch, chunk_bits, chunk_off, seg_bits, nchunks, gps, gi, lane);
  uint8_t *sw = (uint8_t *)(stream + (size_t)g.s * nchunks * kSlotWords);  // the segment's realigned words
  uint32_t cnt = 0;
  for (uint32_t kb = g.k0; kb < g.k1; kb += 64 * kTailRounds) {
    uint32_t v[kTailRounds];
    group_values<kTailRounds>(g, kb, s_marks[wave], lane, v);
#pragma unroll
    for (int i = 0; i < kTailRounds; i++) {
      const uint32_t k = kb + 64 * i + lane;
      if (k < g.k1) {
        cnt += ff_bytes(v[i]);
        *(uint32_t *)(sw + 4u * k) = v[i];
      }
    }
  }
  cnt = (uint32_t)wave_sum((int)cnt);
  if (lane == 0) group_ff[gi] = cnt;
}

// Workgroup per frame: per segment (wave s % 4), the exclusive scan of its groups' 0xFF counts
// (ff_off) and its stuffed size with the RSTn / EOI trailer; then the frame's size (header +
// segments; RST: the segments' offsets after the header, seg_off).  The last frame to finish
// (one ticket per frame, done[0], zeroed by k_scan_bits) places every frame: frame_offsets.
__global__ __launch_bounds__(256) void k_scan_ff(const uint32_t *__restrict__ group_ff,
                                                 uint32_t *__restrict__ ff_off,
                                                 const uint32_t *__restrict__ seg_bits, int nchunks, int gps, int nseg,
                                                 int hdr_len, const uint32_t *__restrict__ dht_nval,
                                                 uint32_t *__restrict__ hdr_lens, uint32_t *__restrict__ seg_size,
                                                 uint32_t *__restrict__ seg_off, uint64_t *__restrict__ frame_size,
                                                 uint64_t *__restrict__ frame_offsets, uint32_t *__restrict__ done) {
  __shared__ uint32_t s_last;
  tail_priority(seg_bits, nchunks);
  const int f = blockIdx.x, nframes = gridDim.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  uint32_t mine = 0;  // nseg == 1: the segment's size (wave 0)
  for (int si = wave; si < nseg; si += 4) {
    const size_t s = (size_t)f * nseg + si, g0 = s * gps;
    uint32_t carry = 0;
    for (int i0 = 0; i0 < gps; i0 += 64) {
      const int i = i0 + lane;
      const uint32_t v = i < gps ? group_ff[g0 + i] : 0u;
      const uint32_t incl = wave_incl_scan(v, lane);
      if (i < gps) ff_off[g0 + i] = carry + incl - v;
      carry += lane63(incl);
    }
    mine = ((seg_bits[s] + 7) >> 3) + carry + 2;
    if (nseg > 1 && lane == 0) seg_size[s] = mine;
  }
  __syncthreads();  // seg_size of the frame written (RST)
  const uint32_t hl = frame_hdr_len(f, hdr_len, dht_nval);
  if (wave == 0) {
    uint64_t fsz = hl;
    if (nseg == 1) {
      fsz += mine;
    } else {
      uint32_t carry = 0;
      for (int i0 = 0; i0 < nseg; i0 += 64) {
        const int i = i0 + lane;
        const uint32_t v = i < nseg ? seg_size[(size_t)f * nseg + i] : 0u;
        const uint32_t incl = wave_incl_scan(v, lane);
        if (i < nseg) seg_off[(size_t)f * nseg + i] = carry + incl - v;
        carry += lane63(incl);
      }
      fsz += carry;
    }
    if (lane == 0) {
      if (dht_nval) hdr_lens[f] = hl;
      st_agent64(frame_size + f, fsz);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t t = 0;
    // release: this frame's size is visible (agent scope) before its ticket; acquire: the
    // last ticket sees every frame's size
    if (lane == 0) t = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (lane == 0) s_last = t;
  }
  __syncthreads();
  if (s_last != (uint32_t)nframes - 1 || wave != 0) return;
  __threadfence();  // every lane of the placing wave acquires the frame sizes (agent scope)
  // the last frame: packed offsets of every frame
  uint64_t carry = 0;
  for (int i0 = 0; i0 < nframes; i0 += 64) {
    const int i = i0 + lane;
    const uint64_t v = i < nframes ? ld_agent64(frame_size + i) : 0ull;
    uint64_t incl = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint64_t o = __shfl_up(incl, d, 64);
      if (lane >= d) incl += o;
    }
    if (i < nframes) frame_offsets[i] = carry + incl - v;
    carry += __shfl(incl, 63, 64);
  }
  if (lane == 0) frame_offsets[nframes] = carry;
}

// The frame header at fo (hl bytes): the default header, or (-huffman optimal) its bytes
// before and after the DHT around the frame's own DHT (jpeg_table_header: one DHT, tables
// DC0, DC1, AC0, AC1).
__device__ __noinline__ void write_header(uint8_t *fo, int f, const uint8_t *hdr, int hdr_len, int dht_pos,
                                             int dht_end, const uint8_t *dht, const uint32_t *dht_nval, int lane) {
  if (!dht_nval) {
    for (int i = lane; i < hdr_len; i += 64) fo[i] = hdr[i];
    return;
  }
  const uint32_t *nv = dht_nval + 4 * (size_t)f;
  const int len = 2 + 4 * 17 + (int)(nv[0] + nv[1] + nv[2] + nv[3]);
  for (int i = lane; i < dht_pos; i += 64) fo[i] = hdr[i];
  uint8_t *o = fo + dht_pos;
  if (lane == 0) {
    o[0] = 0xff;
    o[1] = 0xc4;
    o[2] = (uint8_t)(len >> 8);
    o[3] = (uint8_t)len;
  }
  o += 4;
  for (int t = 0; t < 4; t++) {
    const uint8_t *src = dht + ((size_t)f * 4 + t) * kDhtSlot;
    const int n = 16 + (int)nv[t];
    if (lane == 0) o[0] = (uint8_t)(t < 2 ? t : 0x10 | (t - 2));
    for (int i = lane; i < n; i += 64) o[1 + i] = src[i];
    o += 1 + n;
  }
  const int tail = hdr_len - dht_end;
  for (int i = lane; i < tail; i += 64) o[i] = hdr[dht_end + i];
}

typedef uint32_t u32_any __attribute__((aligned(1)));  // a dword at any byte address (global memory)

// Wave per chunk group: the group's words from the stream k_count_ff realigned, with a 0x00
// after every 0xFF (ff_mjpeg_escape_FF), at frame offset + header + segment offset + 4 k + the
// 0xFFs before word k in the segment.  A word without 0xFF goes out as one unaligned dword
// store (byte-swapped: the scan is MSB first), a word with 0xFF bytes as byte stores.
__global__ __launch_bounds__(256) void k_write(
    const uint32_t *__restrict__ stream, const uint32_t *__restrict__ chunk_bits,
    const uint32_t *__restrict__ chunk_off, const uint32_t *__restrict__ seg_bits,
    const uint32_t *__restrict__ ff_off, int nchunks, int gps, int nseg, int nframes,
    const uint32_t *__restrict__ seg_size, const uint32_t *__restrict__ seg_off,
    const uint64_t *__restrict__ frame_offsets, const uint8_t *__restrict__ hdr, int hdr_len,
    const uint32_t *__restrict__ hdr_lens, int dht_pos, int dht_end, const uint8_t *__restrict__ dht,
    const uint32_t *__restrict__ dht_nval, uint8_t *__restrict__ out, uint64_t out_cap,
    uint32_t *__restrict__ status) {
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  tail_priority(seg_bits, nchunks);
  const int gi = blockIdx.x * 4 + wave, ngroups = gps * nseg * nframes;
  if (gi >= ngroups) return;
  const int s = gi / gps, gx = gi - s * gps, f = s / nseg, si = s - f * nseg;
  const int c0 = gx * kChunksPerWave, cl = min(c0 + kChunksPerWave, nchunks) - 1;
  const size_t i0 = (size_t)s * nchunks;
  const uint32_t k0 = (chunk_off[i0 + c0] + 31) >> 5, k1 = (chunk_off[i0 + cl] + chunk_bits[i0 + cl] + 31) >> 5;
  const uint32_t total_bytes = (seg_bits[s] + 7) >> 3;
  const uint64_t foff = frame_offsets[f];
  if (frame_offsets[f + 1] > out_cap) {  // the host regrows the output and runs k_write again
    if (lane == 0) atomicOr(status, 1u);
    return;
  }
  const uint32_t hl = hdr_lens ? hdr_lens[f] : (uint32_t)hdr_len;
  const uint64_t sbase = foff + hl + (nseg > 1 ? seg_off[s] : 0u);
  if (si == 0 && gx == 0) write_header(out + foff, f, hdr, hdr_len, dht_pos, dht_end, dht, dht_nval, lane);
  if (gx == gps - 1 && lane == 0) {  // the segment's trailer: RSTn, or EOI after the frame's last
    const uint64_t segsz = nseg > 1 ? seg_size[s] : frame_offsets[f + 1] - foff - hl;
    uint8_t *m = out + sbase + segsz - 2;
    m[0] = 0xff;
    m[1] = si == nseg - 1 ? 0xd9 : (uint8_t)(0xd0 + (si & 7));
  }
  const uint8_t *sw = (const uint8_t *)(stream + i0 * kSlotWords);
  uint8_t *ob = out + sbase + ff_off[gi];  // + 4 k + the word's 0xFF prefix in the group
  uint32_t carry = 0;
  for (uint32_t kb = k0; kb < k1; kb += 64 * kTailRounds) {
    uint32_t v[kTailRounds];
#pragma unroll
    for (int i = 0; i < kTailRounds; i++) v[i] = *(const uint32_t *)(sw + 4u * min(kb + 64 * i + lane, k1 - 1));
#pragma unroll
    for (int i = 0; i < kTailRounds; i++) {
      if (kb + 64 * i >= k1) break;  // wave-uniform
      const uint32_t k = kb + 64 * i + lane;
      const bool valid = k < k1;
      const uint32_t w = v[i];
      const uint32_t ff = valid ? ff_bytes(w) : 0u;
      const uint32_t incl = wave_incl_scan(ff, lane);
      uint8_t *p = ob + 4 * (size_t)k + carry + incl - ff;
      const bool last = valid && 4 * k + 4 > total_bytes;  // the segment's last word: nb < 4 bytes
      if (valid && ff == 0 && !last) {
        *(u32_any *)p = __builtin_bswap32(w);
      } else if (valid) {  // 0xFF bytes (each then 0x00), or the segment's last (short) word
        const uint32_t nb = min(4u, total_bytes - 4 * k);
        uint64_t X = 0;
        uint32_t len = 0;
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const uint32_t byte = (w >> (24 - 8 * b)) & 0xffu;
          if ((uint32_t)b < nb) {
            X |= (uint64_t)byte << (8 * len);
            len += byte == 0xffu ? 2u : 1u;
          }
        }
        const uint32_t first = len >= 4u ? 4u : 0u;
        if (len >= 4u) *(u32_any *)p = (uint32_t)X;
#pragma unroll
        for (uint32_t b = 0; b < 8; b++)
          if (b >= first && b < len) p[b] = (uint8_t)(X >> (8 * b));
      }
      carry += lane63(incl);
    }
  }
}

}  // namespace mjg
