// k_scale_encode: the `-vf scale=W:H:flags=bicubic` resize and the MJPEG encode of the scaled
// frame in one kernel (BASELINE configs[3]: 4K -> 1080p bicubic + q=3, remote_args of
// ffmpeg_distributed.py:134).  The scaled pixels never touch HBM: a workgroup scales a
// group of 32 consecutive MCUs into LDS and its three waves encode the group's three
// chunks of 64 blocks (4:2:0: 32 MCUs x 6 blocks = 3 chunks) from there.
//
// Arithmetic is libswscale's C path, exactly as k_scale applies it (scale.hip), so the
// encoded frame is byte-identical to k_scale + k_encode (and to oracle.scale_plane +
// encode_frame):
//   hScale8To15_c  min((sum src*f) >> 7, 32767), 14-bit coefficients; D4 layout: taps as
//                  int8 (p - 128) against the coefficients' int8 hi / lo bytes, two
//                  v_dot4_i32_i8 per 4 taps: (sum p c) >> 7 = ah + (al >> 7) + sum c
//   [tv input]     lumRangeToJpeg_c / chrRangeToJpeg_c on that int16
//   yuv2planeX_8_c clip_u8(((64 << 12) + sum h*f) >> 19), 12-bit coefficients as pairs
//                  (v_dot2_i32_i16), the host's parity-shifted pair table (k_scale's)
//
// Phase 1 (scale, all waves): column tasks of 64 output columns, lane = column.  A lane
// reads its 8-byte tap window of every source row its MCU row needs straight from global
// memory (unaligned 8-byte loads; a wave's loads of one row span ~130 contiguous bytes),
// runs the h-pass per source row and stores the row pairs (int16 x 2) to the wave's LDS
// h-buffer; the v-pass then reads the pairs of each output row and writes the pixel to
// the group's LDS image (Y: 16 rows x 512, Cb, Cr: 8 rows x 256; rows past the frame
// replicate its last row, columns past it the last column: FFmpeg's edge emulation).
// Phase 2 (encode, wave w = chunk 3g + w): the block rows from the LDS image, then
// k_encode's row pass, column screen, DC prediction (chunk predecessors through LDS),
// Huffman coding and packing into the chunk's slot, unchanged.
//
// Persistent workgroups pull units of groups_per_wg consecutive groups of one frame; a unit's
// first group's predecessor MCU is scaled once more (prologue) for its DCs, later groups take
// them from the previous group's third chunk.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mjg {

constexpr int kFusedWaves = 3;
constexpr int kGroupMcus = 32;           // 4:2:0: 32 MCUs = 192 blocks = 3 chunks
constexpr int kFusedMaxPairs = 21;       // h-pass row pairs per column task (2:1 luma: 20)
constexpr int kFusedGroupsPerWg = 4;     // consecutive groups per workgroup
constexpr int kFusedTabWords = 8;        // words per column (h) / row (v) filter entry
constexpr int kImgY = 16 * 512, kImgC = 8 * 256;           // LDS image bytes per plane
constexpr int kImgWords = (kImgY + 2 * kImgC) / 4;          // 3072
constexpr int kHbufWords = kFusedWaves * kFusedMaxPairs * 64;  // 4032
constexpr int kPkWords = kFusedWaves * 32 * 64;                // 6144
constexpr int kRegionWords = (kHbufWords + kImgWords) > kPkWords ? (kHbufWords + kImgWords) : kPkWords;

struct FusedGeom {
  int sw[2], sh[2];           // source plane sizes: luma, chroma
  int dw[2], dh[2];           // scaled plane sizes (== EncGeom w, h / cw, ch)
  long long s_fstride, s_off[3];  // source frame stride, plane offsets (Y, U, V)
  int gpf, groups_per_wg;     // groups per frame, groups per workgroup
  int npairs[2];              // h-pass row pairs a column task needs, luma / chroma (<= kFusedMaxPairs)
};

// One h-pass output: hScale8To15 of the 8 (HT) taps at src (D4 words c[0..HT/2)), then the
// range conversion.  hs = sum of the taps' coefficients (folded into the hi accumulator).
template <int HT, int RANGE>
__device__ __forceinline__ int fused_hscale(const uint8_t *src, const uint32_t (&c)[HT / 2], int hs) {
  typedef uint64_t u64_unaligned __attribute__((aligned(1)));
  typedef uint32_t u32_unaligned __attribute__((aligned(1)));
  int ah = hs, al = 0;
  if constexpr (HT == 8) {
    const uint64_t w = *(const u64_unaligned *)src;
    const int lo = (int)((uint32_t)w ^ 0x80808080u), hi = (int)((uint32_t)(w >> 32) ^ 0x80808080u);
    ah = __builtin_amdgcn_sdot4(lo, (int)c[0], ah, false);
    al = __builtin_amdgcn_sdot4(lo, (int)c[1], al, false);
    ah = __builtin_amdgcn_sdot4(hi, (int)c[2], ah, false);
    al = __builtin_amdgcn_sdot4(hi, (int)c[3], al, false);
  } else {  // HT == 4
    const int lo = (int)(*(const u32_unaligned *)src ^ 0x80808080u);
    ah = __builtin_amdgcn_sdot4(lo, (int)c[0], ah, false);
    al = __builtin_amdgcn_sdot4(lo, (int)c[1], al, false);
  }
  const int v = ah + (al >> 7);
  if (RANGE == 1) return (__mul24(min(v, 30189), 19077) - 39057361) >> 14;  // min also clips 32767
  if (RANGE == 2) return (__mul24(min(v, 30775), 4663) - 9289992) >> 12;
  return min(v, 32767);
}

// One column task: lane = one scaled column `x` of plane `pl` (0 luma, 1/2 chroma), output rows
// ybase .. ybase + rows - 1 (clamped to the plane), written as bytes to dst[i * dpitch].
// hbuf: the wave's h-buffer ([pair][lane]).  RANGE_ON: tv input (luma 1, chroma 2 per plane).
template <int HT, int NPV, bool RANGE_ON>
__device__ __forceinline__ void fused_column(const uint8_t *frame, const FusedGeom &fg, int pl, int x,
                                             int ybase, int rows, const uint32_t *__restrict__ htab,
                                             const uint32_t *__restrict__ vtab, uint32_t *hbuf,
                                             uint8_t *dst, int dpitch, bool valid, int lane, int np) {
  const int pc = pl ? 1 : 0;
  const int sw = fg.sw[pc], sh = fg.sh[pc], dh = fg.dh[pc];
  const uint8_t *src = frame + fg.s_off[pl];
  const uint32_t *ht = htab + (size_t)x * kFusedTabWords;
  const uint4 h0 = *(const uint4 *)ht, h1 = *(const uint4 *)(ht + 4);
  uint32_t c[HT / 2];
  c[0] = h0.x;
  c[1] = h0.y;
  if constexpr (HT == 8) {
    c[2] = h0.z;
    c[3] = h0.w;
  }
  const int hpos = (int)h1.z, hs = (int)h1.w;
  const int ps0 = (int)vtab[(size_t)min(ybase, dh - 1) * kFusedTabWords];
  const uint8_t *colp = src + hpos;
  // h-pass: source rows 2 (ps0 + p) and 2 (ps0 + p) + 1 of pair p (rows past the plane meet
  // only zero coefficients: clamped)
  const int rmax = sh - 1;
#pragma unroll 2
  for (int p = 0; p < np; p++) {
    const int r0 = min(2 * (ps0 + p), rmax), r1 = min(2 * (ps0 + p) + 1, rmax);
    int a, b;
    if (RANGE_ON) {
      if (pc == 0) {
        a = fused_hscale<HT, 1>(colp + (size_t)r0 * sw, c, hs);
        b = fused_hscale<HT, 1>(colp + (size_t)r1 * sw, c, hs);
      } else {
        a = fused_hscale<HT, 2>(colp + (size_t)r0 * sw, c, hs);
        b = fused_hscale<HT, 2>(colp + (size_t)r1 * sw, c, hs);
      }
    } else {
      a = fused_hscale<HT, 0>(colp + (size_t)r0 * sw, c, hs);
      b = fused_hscale<HT, 0>(colp + (size_t)r1 * sw, c, hs);
    }
    hbuf[p * 64 + lane] = ((uint32_t)a & 0xffffu) | ((uint32_t)b << 16);
  }
  // v-pass: output row y reads the pairs [vps[y], vps[y] + NPV) against its pair coefficients
  for (int i = 0; i < rows; i++) {
    const uint32_t *vr = vtab + (size_t)min(ybase + i, dh - 1) * kFusedTabWords;
    const uint4 v0 = *(const uint4 *)vr, v1 = *(const uint4 *)(vr + 4);
    const uint32_t vc[7] = {v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    const uint32_t *cp = hbuf + ((int)v0.x - ps0) * 64 + lane;
    int acc = 64 << 12;
#pragma unroll
    for (int k = 0; k < NPV; k++)
      acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, cp[k * 64]), __builtin_bit_cast(short2_t, vc[k]),
                                   acc, false);
    if (valid) dst[i * dpitch] = (uint8_t)min(max(acc >> 19, 0), 255);
  }
}

// Column task t (0..15) of a group: 8 luma tasks of 64 columns (4 MCUs each), 4 Cb and 4 Cr
// tasks of 64 columns (8 MCUs each).  Wave order balances the cost (a luma task scales 16
// rows from ~40 source rows, a chroma task 8 rows from ~24): waves get {L0 L3 L6 C0 C3},
// {L1 L4 L7 C1 C4}, {L2 L5 C2 C5 C6 C7} (C0-3 Cb, C4-7 Cr).
__device__ static constexpr int8_t kFusedTasks[3][6] = {
    {0, 3, 6, 8, 11, -1}, {1, 4, 7, 9, 12, -1}, {2, 5, 10, 13, 14, 15}};

template <int HT, int NPV, bool RANGE_ON>
__device__ __forceinline__ void fused_scale_group(const uint8_t *frame, const EncGeom &g, const FusedGeom &fg,
                                                  int grp, const uint32_t *htab0, const uint32_t *vtab0,
                                                  const uint32_t *htab1, const uint32_t *vtab1, uint32_t *hbuf,
                                                  uint8_t *img, int wave, int lane) {
#pragma unroll 1
  for (int k = 0; k < 6; k++) {
    const int t = kFusedTasks[wave][k];
    if (t < 0) break;
    const int pl = t < 8 ? 0 : (t < 12 ? 1 : 2);
    const int j = (t < 8 ? t : (t & 3)) * 64 + lane;  // column within the group's plane strip
    const int mw = pl ? 8 : 16;                         // MCU width in this plane
    const int ml = j / mw, m = grp * kGroupMcus + ml;
    const bool valid = m < g.nmcu;
    const int mm = valid ? m : g.nmcu - 1;
    const int my = mm / g.mbw, mx = mm - my * g.mbw;
    const int pc = pl ? 1 : 0;
    const int x = min(mx * mw + (j - ml * mw), fg.dw[pc] - 1);
    uint8_t *dst = img + (pl == 0 ? j : kImgY + (pl - 1) * kImgC + j);
    fused_column<HT, NPV, RANGE_ON>(frame, fg, pl, x, my * mw, mw, pl ? htab1 : htab0, pl ? vtab1 : vtab0,
                                    hbuf, dst, pl ? 256 : 512, valid, lane, fg.npairs[pc]);
  }
}

template <int HT, int NPV, bool RANGE_ON, int MODE>
__global__ __launch_bounds__(64 * kFusedWaves, 4) void k_scale_encode(
    const uint8_t *__restrict__ frames, EncGeom g, FusedGeom fg, const uint32_t *__restrict__ tabs,
    const uint32_t *__restrict__ htab0, const uint32_t *__restrict__ vtab0,
    const uint32_t *__restrict__ htab1, const uint32_t *__restrict__ vtab1,
    uint32_t *__restrict__ scratch, uint32_t *__restrict__ chunk_bits, uint32_t *__restrict__ stage_all,
    uint32_t *__restrict__ work_ctr, int nframes, uint32_t *__restrict__ hist, uint32_t *__restrict__ syms,
    uint32_t *__restrict__ symn) {
  __shared__ uint32_t s_ac[512];
  __shared__ uint32_t s_dc[32];
  __shared__ __attribute__((aligned(16))) int32_t s_qc[64];
  __shared__ uint8_t s_zz[64];
  __shared__ __attribute__((aligned(16))) float s_thr[64];
  __shared__ __attribute__((aligned(16))) uint32_t s_m2[32];
  __shared__ uint8_t s_scat[64];
  __shared__ uint32_t s_desc[8];
  __shared__ uint32_t s_skip[12];
  __shared__ int s_dcx[2][kFusedWaves][8];  // per group parity: each chunk's last 8 DCs
  __shared__ int s_next;                     // the workgroup's next unit
  __shared__ __attribute__((aligned(16))) uint32_t s_region[kRegionWords];
  __shared__ uint32_t s_aux_all[MODE == kEmitDefault ? 1 : kFusedWaves][kFrameTabWords];

  const int tid = threadIdx.x, wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  for (int i = tid; i < 512; i += 64 * kFusedWaves) s_ac[i] = tabs[i];
  if (tid < 32) s_dc[tid] = tabs[512 + tid];
  if (tid < 64) {
    s_qc[tid] = (int32_t)tabs[544 + tid];
    s_zz[tid] = kZigzag[tid];
    s_thr[tid] = __uint_as_float(tabs[608 + tid]);
    if (tid < 32)
      s_m2[tid] = (uint32_t)(uint16_t)kPass2Dot[2 * tid] | ((uint32_t)(uint16_t)kPass2Dot[2 * tid + 1] << 16);
    s_scat[tid] = kScreenScatter[tid];
  }
  if (tid < 8) s_desc[tid] = tabs[672 + tid];
  if (tid < 12) s_skip[tid] = tabs[680 + tid];
  uint32_t *s_aux = s_aux_all[MODE == kEmitDefault ? 0 : wave];
  if (MODE == kCount)
    for (int i = lane; i < kFrameTabWords; i += 64) s_aux[i] = 0;

  uint32_t *hbuf = s_region + wave * kFusedMaxPairs * 64;
  uint8_t *img = (uint8_t *)(s_region + kHbufWords);
  uint32_t *s_pk = s_region + wave * 32 * 64;
  const int nblk = g.seg_blocks;
  const int runs_pf = (fg.gpf + fg.groups_per_wg - 1) / fg.groups_per_wg;
  const int nunits = runs_pf * nframes;
  uint32_t *stage = stage_all + ((size_t)blockIdx.x * kFusedWaves + wave) * 64 * kStageWords + lane;
  int aux_frame = -1;  // frame whose histogram s_aux holds (kCount)

  // Persistent workgroups: unit = (frame, run of groups_per_wg consecutive groups); the first
  // unit is blockIdx.x, the next ones come from work_ctr (zeroed by the tail's scan kernel).
  for (int unit = blockIdx.x; unit < nunits;) {
    const int frame = unit / runs_pf;
    const int g0 = (unit - frame * runs_pf) * fg.groups_per_wg;
    const int g1 = min(g0 + fg.groups_per_wg, fg.gpf);
    const uint8_t *fr = frames + (size_t)frame * fg.s_fstride;
    // prologue: the DCs of the MCU before this unit's first group (the predecessors of chunk
    // 3 g0's first blocks), into s_dcx[parity of g0 - 1][2][2..7]
    if (g0 > 0) {
      if (wave == 0 && lane < 32) {
        const int pl = lane < 16 ? 0 : (lane < 24 ? 1 : 2);
        const int m = g0 * kGroupMcus - 1, my = m / g.mbw, mx = m - my * g.mbw;
        const int mw = pl ? 8 : 16, c = pl == 0 ? lane : (lane - 16) & 7;
        const int pc = pl ? 1 : 0;
        const int x = min(mx * mw + c, fg.dw[pc] - 1);
        uint8_t *dst = img + (pl == 0 ? c : kImgY + (pl - 1) * kImgC + c);
        fused_column<HT, NPV, RANGE_ON>(fr, fg, pl, x, my * mw, mw, pl ? htab1 : htab0, pl ? vtab1 : vtab0,
                                        hbuf, dst, pl ? 256 : 512, true, lane, fg.npairs[pc]);
      }
      __syncthreads();
      if (wave == 0 && lane < 6) {  // block `lane` of the MCU: 64-pixel sum -> quantised DC
        const uint32_t d = s_desc[lane];
        const int pl = (int)(d & 3u), dx = (int)((d >> 3) & 1u) * 8, dy = (int)((d >> 4) & 1u) * 8;
        const uint8_t *bp = pl == 0 ? img + dy * 512 + dx : img + kImgY + (pl - 1) * kImgC;
        const int pitch = pl ? 256 : 512;
        uint32_t sum = 0;
        for (int r = 0; r < 8; r++) {
          const uint2 w = *(const uint2 *)(bp + r * pitch);
          sum = __builtin_amdgcn_udot4(w.x, 0x01010101u, sum, false);
          sum = __builtin_amdgcn_udot4(w.y, 0x01010101u, sum, false);
        }
        s_dcx[(g0 - 1) & 1][2][2 + lane] = (int)((sum + 32) >> 6);
      }
      __syncthreads();  // the prologue's image is read before phase 1 overwrites it
    }
    if (MODE == kCount && frame != aux_frame) {  // flush the previous frame's counts
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (aux_frame >= 0)
        for (int i = lane; i < kFrameTabWords; i += 64) {
          const uint32_t v = s_aux[i];
          if (v) atomicAdd(&hist[(size_t)aux_frame * kFrameTabWords + i], v);
          s_aux[i] = 0;
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      aux_frame = frame;
    }

    for (int grp = g0; grp < g1; grp++) {
      // phase 1: the group's scaled pixels into the LDS image
      fused_scale_group<HT, NPV, RANGE_ON>(fr, g, fg, grp, htab0, vtab0, htab1, vtab1, hbuf, img, wave, lane);
      __syncthreads();
      // phase 2: chunk 3 grp + wave, lane = block
      const int chunk = grp * kFusedWaves + wave;
      const int b = chunk * 64 + lane;
      const bool active = chunk < g.nchunks && b < nblk;
      const int m = (int)__umulhi((uint32_t)b, g.bpm_magic);
      const uint32_t dsc = s_desc[b - m * g.bpm];
      const int tab = desc_tab(dsc);
      uint64_t raw[8];
      {
        const int ml = m - grp * kGroupMcus;
        const int pl = (int)(dsc & 3u), dx = (int)((dsc >> 3) & 1u) * 8, dy = (int)((dsc >> 4) & 1u) * 8;
        const uint8_t *bp = pl == 0 ? img + dy * 512 + ml * 16 + dx : img + kImgY + (pl - 1) * kImgC + ml * 8;
        const int pitch = pl ? 256 : 512;
#pragma unroll
        for (int r = 0; r < 8; r++) raw[r] = active ? *(const uint64_t *)(bp + r * pitch) : 0ull;
      }
      __syncthreads();  // every wave holds its rows: the region becomes the row images
      row_pass<false>(raw, tab, nullptr, s_pk, lane);
      int dc = 0;
      uint32_t ca = 0, cb = 0;
      if (active) column_screen(s_pk, lane, s_skip, s_thr, dc, ca, cb);
      const uint64_t mask = screen_mask(ca, cb, s_scat);
      const int par = grp & 1;
      if (lane >= 56) s_dcx[par][wave][lane - 56] = dc;
      __syncthreads();
      const int carry =
          lane >= 56 ? (wave ? s_dcx[par][wave - 1][lane - 56] : s_dcx[par ^ 1][2][lane - 56]) : 128;
      const int diff = dc - dc_predictor(dc, carry, desc_delta(dsc), chunk == 0, lane);
      const size_t t = (size_t)frame * g.nchunks + chunk;
      if (MODE == kCount) {
        CountSink cs{s_aux + tab * 256, s_aux + 512 + tab * 16, syms + t * kSymCap * 64 + lane};
        if (active) emit_block(s_pk + lane, mask, diff, s_zz, s_m2, s_qc, cs);
        if (chunk < g.nchunks) symn[t * 64 + lane] = cs.n;
      } else {
        ShiftSink q;
        q.act = s_ac + tab * 256;
        q.dct = s_dc + tab * 16;
        q.stage = stage;
        if (active) {
          emit_block(s_pk + lane, mask, diff, s_zz, s_m2, s_qc, q);
          if (q.bits > 128) q.flush();
        }
        if (chunk < g.nchunks) pack_chunk(q, active, scratch + t * kSlotWords, chunk_bits + t, lane);
      }
      __syncthreads();  // the row images are done with before the next group's phase 1
    }
    if (tid == 0) s_next = (int)gridDim.x + (int)atomicAdd(work_ctr, 1u);
    __syncthreads();
    unit = s_next;
  }
  if (MODE == kCount && aux_frame >= 0) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    for (int i = lane; i < kFrameTabWords; i += 64) {
      const uint32_t v = s_aux[i];
      if (v) atomicAdd(&hist[(size_t)aux_frame * kFrameTabWords + i], v);
    }
  }
}

}  // namespace mjg
