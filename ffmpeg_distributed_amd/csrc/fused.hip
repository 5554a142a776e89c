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
constexpr int kFusedMaxPairs = 20;       // h-pass row pairs per column task (2:1 luma: 20)
constexpr int kFusedBatch = 4;           // h-pass pairs whose loads are in flight together
constexpr int kFusedGroupsPerWg = 4;     // consecutive groups per workgroup
constexpr int kFusedTabWords = 8;        // words per column (h) / row (v) filter entry
constexpr int kImgY = 16 * 512, kImgC = 8 * 256;           // LDS image bytes per plane
constexpr int kImgWords = (kImgY + 2 * kImgC) / 4;          // 3072
constexpr int kHbufWave = kFusedMaxPairs * 64 + 96;             // h-buffer + v-row table
constexpr int kHbufWords = kFusedWaves * kHbufWave;
constexpr int kPkWords = kFusedWaves * 32 * 64;                // 6144
constexpr int kRegionWords = (kHbufWords + kImgWords) > kPkWords ? (kHbufWords + kImgWords) : kPkWords;

struct FusedGeom {
  int sw[2], sh[2];           // source plane sizes: luma, chroma
  int dw[2], dh[2];           // scaled plane sizes (== EncGeom w, h / cw, ch)
  long long s_fstride, s_off[3];  // source frame stride, plane offsets (Y, U, V)
  int gpf, groups_per_wg;     // groups per frame, groups per workgroup
  int npairs[2];              // h-pass row pairs a column task needs, luma / chroma (<= kFusedMaxPairs)
};

__device__ __forceinline__ int dot4_i8(int a, int b, int c) { return __builtin_amdgcn_sdot4(a, b, c, false); }

// One h-pass output: hScale8To15 of the HT (8 or 4) taps in w (little-endian bytes, D4 words
// c[0..HT/2)), then the range conversion.  hs = sum of the taps' coefficients (folded into
// the hi accumulator).
template <int HT, int RANGE>
__device__ __forceinline__ int fused_hscale(uint64_t w, const uint32_t (&c)[HT / 2], int hs) {
  const int lo = (int)((uint32_t)w ^ 0x80808080u);
  int ah = dot4_i8(lo, (int)c[0], hs);
  int al = dot4_i8(lo, (int)c[1], 0);
  if constexpr (HT == 8) {
    const int hi = (int)((uint32_t)(w >> 32) ^ 0x80808080u);
    ah = dot4_i8(hi, (int)c[2], ah);
    al = dot4_i8(hi, (int)c[3], al);
  }
  const int v = ah + (al >> 7);
  if (RANGE == 1) return (__mul24(min(v, 30189), 19077) - 39057361) >> 14;  // min also clips 32767
  if (RANGE == 2) return (__mul24(min(v, 30775), 4663) - 9289992) >> 12;
  return min(v, 32767);
}

// h-table entry of one scaled column: D4 coefficient words, tap position, tap sum.
template <int HT>
struct HCol {
  uint32_t c[HT / 2];
  int hpos, hs;
};

template <int HT>
__device__ __forceinline__ HCol<HT> load_hcol(const uint32_t *__restrict__ htab, int x) {
  const uint32_t *ht = htab + (size_t)x * kFusedTabWords;
  const uint4 h0 = *(const uint4 *)ht, h1 = *(const uint4 *)(ht + 4);
  HCol<HT> r;
  r.c[0] = h0.x;
  r.c[1] = h0.y;
  if constexpr (HT == 8) {
    r.c[2] = h0.z;
    r.c[3] = h0.w;
  }
  r.hpos = (int)h1.z;
  r.hs = (int)h1.w;
  return r;
}

// The rows of MCU row my (wave-uniform) for this lane's column (h entry hc): the ROWS scaled
// rows, bytes to dst[i * dpitch] when `valid`.  Everything row-related is wave-uniform: the
// source row addresses are scalar (the loads take the lane's tap position as their only
// vector operand) and the v rows come by scalar loads.  The tap-window loads (np <=
// kFusedMaxPairs row pairs, 8 B each, np even) go out kFusedBatch pairs ahead of their use.
template <int HT, int NPV, int RANGE, int ROWS>
__device__ __forceinline__ void fused_rows(const uint8_t *__restrict__ src, int sw, int sh, int dh, int my,
                                           const HCol<HT> &hc, const uint32_t *__restrict__ vtab,
                                           uint32_t *hbuf, uint32_t *s_vrow, uint8_t *dst, int dpitch, bool valid,
                                           int lane, int np) {
  typedef uint64_t u64_unaligned __attribute__((aligned(1)));
  typedef uint32_t u32_unaligned __attribute__((aligned(1)));
  const int ybase = my * ROWS;
  const int ps0 = (int)vtab[(size_t)min(ybase, dh - 1) * kFusedTabWords];
  const int rmax = sh - 1;
  // the task's v rows (ROWS x 6 words) into the wave's LDS row table: loaded now, stored after
  // the h-pass (their latency hides behind it), read by the v-pass as uniform broadcasts
  // (a partial wave -- the prologue, or one MCU row of a task that straddles two -- has its
  // active lanes store the table first, each several entries)
  constexpr int kVt = ROWS * 6, kVtPerLane = (kVt + 63) / 64;
  const uint64_t act = __ballot(1);
  const bool full = act == ~0ull;
  uint32_t vtw[kVtPerLane];
  if (full) {
#pragma unroll
    for (int k = 0; k < kVtPerLane; k++) {
      const int e = lane + 64 * k, row = e / 6, wd = e - row * 6;
      vtw[k] = e < kVt ? vtab[(size_t)min(ybase + row, dh - 1) * kFusedTabWords + wd] : 0u;
    }
  } else {
    const int na = __popcll(act), rk = __popcll(act & ((1ull << lane) - 1ull));
    for (int e = rk; e < kVt; e += na) {
      const int row = e / 6, wd = e - row * 6;
      s_vrow[e] = vtab[(size_t)min(ybase + row, dh - 1) * kFusedTabWords + wd];
    }
  }
  const uint32_t hp = (uint32_t)hc.hpos;
  auto load = [&](uint64_t (&w)[2 * kFusedBatch], int p0) {
#pragma unroll
    for (int q = 0; q < 2 * kFusedBatch; q++) {
      const uint8_t *row = src + (size_t)min(2 * (ps0 + p0) + q, rmax) * sw;  // uniform
      if constexpr (HT == 8)
        w[q] = *(const u64_unaligned *)(row + hp);
      else
        w[q] = *(const u32_unaligned *)(row + hp);
    }
  };
  auto compute = [&](const uint64_t (&w)[2 * kFusedBatch], int p0) {
#pragma unroll
    for (int k = 0; k < kFusedBatch; k++) {
      const int a = fused_hscale<HT, RANGE>(w[2 * k], hc.c, hc.hs);
      const int b = fused_hscale<HT, RANGE>(w[2 * k + 1], hc.c, hc.hs);
      hbuf[(p0 + k) * 64 + lane] = ((uint32_t)a & 0xffffu) | ((uint32_t)b << 16);
    }
  };
  // np is a multiple of kFusedBatch (host-rounded); the next batch's loads are issued before
  // the current batch is computed
  // whole batches of kFusedBatch pairs, then a tail of 2 pairs when np % kFusedBatch == 2
  const int nfull = np & ~(kFusedBatch - 1);
  uint64_t wa[2 * kFusedBatch], wb[2 * kFusedBatch];
  if (nfull) load(wa, 0);
#pragma unroll 1
  for (int p0 = 0; p0 < nfull; p0 += 2 * kFusedBatch) {
    if (p0 + kFusedBatch < nfull) load(wb, p0 + kFusedBatch);
    compute(wa, p0);
    if (p0 + kFusedBatch >= nfull) break;
    if (p0 + 2 * kFusedBatch < nfull) load(wa, p0 + 2 * kFusedBatch);
    compute(wb, p0 + kFusedBatch);
  }
  if (np != nfull) {
    uint64_t wt[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
      const uint8_t *row = src + (size_t)min(2 * (ps0 + nfull) + q, rmax) * sw;  // uniform
      if constexpr (HT == 8)
        wt[q] = *(const u64_unaligned *)(row + hp);
      else
        wt[q] = *(const u32_unaligned *)(row + hp);
    }
#pragma unroll
    for (int k = 0; k < 2; k++) {
      const int a = fused_hscale<HT, RANGE>(wt[2 * k], hc.c, hc.hs);
      const int b = fused_hscale<HT, RANGE>(wt[2 * k + 1], hc.c, hc.hs);
      hbuf[(nfull + k) * 64 + lane] = ((uint32_t)a & 0xffffu) | ((uint32_t)b << 16);
    }
  }
  if (full) {
#pragma unroll
    for (int k = 0; k < kVtPerLane; k++)
      if (lane + 64 * k < kVt) s_vrow[lane + 64 * k] = vtw[k];
  }
  // v-pass: output row y reads the pairs [vps[y], vps[y] + NPV) against its pair coefficients
  const uint32_t *hcol = hbuf + lane;
#pragma unroll 2
  for (int i = 0; i < ROWS; i++) {
    const uint32_t *vr = s_vrow + i * 6;  // uniform address: LDS broadcast
    const uint32_t *cp = hcol + ((int)vr[0] - ps0) * 64;
    int acc = 64 << 12;
#pragma unroll
    for (int k = 0; k < NPV; k++)
      acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, cp[k * 64]), __builtin_bit_cast(short2_t, vr[1 + k]),
                                   acc, false);
    if (valid) dst[i * dpitch] = (uint8_t)min(max(acc >> 19, 0), 255);
  }
}

// One column task of plane pl (wave-uniform): lane = scaled column x of MCU (my, ...); the lanes'
// MCU rows are run one at a time (at most two: a 64-column task straddles a row end only when
// the MCUs per row are not a multiple of its 4 / 8 MCUs), so row work stays wave-uniform.
template <int HT, int NPV, bool RANGE_ON>
__device__ __forceinline__ void fused_task_rows(const uint8_t *frame, const FusedGeom &fg, int pl, int my,
                                                const HCol<HT> &hc, const uint32_t *vtab0, const uint32_t *vtab1,
                                                uint32_t *hbuf, uint8_t *dst, bool valid, int lane) {
  const uint8_t *src = frame + fg.s_off[pl];
  uint32_t *s_vrow = hbuf + kFusedMaxPairs * 64;  // the wave's v-row table (after its h-buffer)
  auto run = [&](int my_u) {
    if (pl == 0)
      fused_rows<HT, NPV, RANGE_ON ? 1 : 0, 16>(src, fg.sw[0], fg.sh[0], fg.dh[0], my_u, hc, vtab0, hbuf, s_vrow,
                                                 dst, 512, valid, lane, fg.npairs[0]);
    else
      fused_rows<HT, NPV, RANGE_ON ? 2 : 0, 8>(src, fg.sw[1], fg.sh[1], fg.dh[1], my_u, hc, vtab1, hbuf, s_vrow,
                                                dst, 256, valid, lane, fg.npairs[1]);
  };
  const int my_a = __builtin_amdgcn_readfirstlane(my);
  if (my == my_a) run(my_a);
  const uint64_t rest = __ballot(my != my_a);
  if (rest) {  // the lanes of the second MCU row
    const int my_b = __builtin_amdgcn_readlane(my, (int)__builtin_ctzll(rest));
    if (my == my_b) run(my_b);
  }
}

// Column task t (0..15) of a group: 8 luma tasks of 64 columns (4 MCUs each), 4 Cb and 4 Cr
// tasks of 64 columns (8 MCUs each).  Wave order balances the cost (a luma task scales 16
// rows from ~40 source rows, a chroma task 8 rows from ~24): waves get {L0 L3 L6 C0 C3},
// {L1 L4 L7 C1 C4}, {L2 L5 C2 C5 C6 C7} (C0-3 Cb, C4-7 Cr).
__device__ static constexpr int8_t kFusedTasks[3][7] = {
    {0, 3, 6, 8, 11, -1, -1}, {1, 4, 7, 9, 12, -1, -1}, {2, 5, 10, 13, 14, 15, -1}};

// Task t of group grp: the lane's column x, MCU row, whether its MCU is inside the frame and
// its LDS image byte.  Plane pl = task_plane(t) is wave-uniform.
__device__ __forceinline__ int task_plane(int t) { return t < 8 ? 0 : (t < 12 ? 1 : 2); }

struct FusedTask {
  int x, my, img_off;
  bool valid;
};

__device__ __forceinline__ FusedTask fused_task(const EncGeom &g, const FusedGeom &fg, int grp, int t, int pl,
                                                int lane) {
  FusedTask r;
  const int j = (t < 8 ? t : (t & 3)) * 64 + lane;  // column within the group's plane strip
  const int mw = pl ? 8 : 16;                        // MCU width in this plane
  const int ml = j / mw, m0 = grp * kGroupMcus + ml;
  r.valid = m0 < g.nmcu;
  const int m = r.valid ? m0 : g.nmcu - 1;
  r.my = m / g.mbw;
  const int mx = m - r.my * g.mbw;
  r.x = min(mx * mw + (j - ml * mw), fg.dw[pl ? 1 : 0] - 1);
  r.img_off = pl == 0 ? j : kImgY + (pl - 1) * kImgC + j;
  return r;
}

// Phase 1 of group grp: the wave's column tasks, each task's h entries loaded while the
// previous task runs.
template <int HT, int NPV, bool RANGE_ON>
__device__ __forceinline__ void fused_scale_group(const uint8_t *frame, const EncGeom &g, const FusedGeom &fg,
                                                  int grp, const uint32_t *htab0, const uint32_t *htab1,
                                                  const uint32_t *vtab0, const uint32_t *vtab1, uint32_t *hbuf,
                                                  uint8_t *img, int wave, int lane) {
  int t = kFusedTasks[wave][0];
  int pl = task_plane(t);
  FusedTask tk = fused_task(g, fg, grp, t, pl, lane);
  HCol<HT> hc = load_hcol<HT>(pl ? htab1 : htab0, tk.x);
#pragma unroll 1
  for (int k = 0; k < 6; k++) {
    const int tn = kFusedTasks[wave][k + 1], pn = task_plane(tn);
    FusedTask nk = tk;
    HCol<HT> nc = hc;
    if (tn >= 0) {  // prefetch the next task's h entry
      nk = fused_task(g, fg, grp, tn, pn, lane);
      nc = load_hcol<HT>(pn ? htab1 : htab0, nk.x);
    }
    fused_task_rows<HT, NPV, RANGE_ON>(frame, fg, pl, tk.my, hc, vtab0, vtab1, hbuf, img + tk.img_off, tk.valid,
                                       lane);
    if (tn < 0) break;
    tk = nk;
    hc = nc;
    pl = pn;
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
  __shared__ uint4 s_zd[64];  // zigzag -> exact_coef descriptor (zz_desc)
  __shared__ __attribute__((aligned(16))) float s_thr[64];
  __shared__ __attribute__((aligned(16))) uint32_t s_m2[32];
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
    s_zd[tid] = zz_desc(tid, tabs);
    s_thr[tid] = __uint_as_float(tabs[608 + tid]);
    if (tid < 32)
      s_m2[tid] = pass2_pair(tid);
  }
  if (tid < 8) s_desc[tid] = tabs[672 + tid];
  if (tid < 12) s_skip[tid] = tabs[680 + tid];
  uint32_t *s_aux = s_aux_all[MODE == kEmitDefault ? 0 : wave];
  if (MODE == kCount)
    for (int i = lane; i < kFrameTabWords; i += 64) s_aux[i] = 0;

  uint32_t *hbuf = s_region + wave * kHbufWave;
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
      const int m = g0 * kGroupMcus - 1, myp = m / g.mbw, mx = m - myp * g.mbw;
      if (wave == 0 && lane < 32) {  // lanes 0-15: luma columns, 16-23: Cb, 24-31: Cr of MCU m
        const int pl = lane < 16 ? 0 : (lane < 24 ? 1 : 2);
        const int c = lane < 16 ? lane : (lane - 16) & 7;
        const int x = min(mx * (pl ? 8 : 16) + c, fg.dw[pl ? 1 : 0] - 1);
        const HCol<HT> hc = load_hcol<HT>(pl ? htab1 : htab0, x);
        if (lane < 16)
          fused_task_rows<HT, NPV, RANGE_ON>(fr, fg, 0, myp, hc, vtab0, vtab1, hbuf, img + c, true, lane);
        else if (lane < 24)
          fused_task_rows<HT, NPV, RANGE_ON>(fr, fg, 1, myp, hc, vtab0, vtab1, hbuf, img + kImgY + c, true, lane);
        else
          fused_task_rows<HT, NPV, RANGE_ON>(fr, fg, 2, myp, hc, vtab0, vtab1, hbuf, img + kImgY + kImgC + c,
                                             true, lane);
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
      __syncthreads();  // the prologue's image is done with
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
      fused_scale_group<HT, NPV, RANGE_ON>(fr, g, fg, grp, htab0, htab1, vtab0, vtab1, hbuf, img, wave, lane);
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
      uint32_t mlo = 0, mhi = 0;
      uint32_t skip_st = 0xeu;  // every pair's skip test, every group
      if (active) column_screen(s_pk, lane, s_skip, s_thr, dc, mlo, mhi, skip_st, true);
      const uint64_t mask = ((uint64_t)mhi << 32) | mlo;
      const int par = grp & 1;
      if (lane >= 56) s_dcx[par][wave][lane - 56] = dc;
      __syncthreads();
      const int carry =
          lane >= 56 ? (wave ? s_dcx[par][wave - 1][lane - 56] : s_dcx[par ^ 1][2][lane - 56]) : 128;
      const int diff = dc - dc_predictor(dc, carry, desc_delta(dsc), chunk == 0, lane);
      const size_t t = (size_t)frame * g.nchunks + chunk;
      if (MODE == kCount) {
        CountSink cs{s_aux + tab * 256, s_aux + 512 + tab * 16, syms + t * kSymCap * 64 + lane};
        if (active) emit_block(s_pk + lane, mask, diff, s_zd, s_m2, cs);
        if (chunk < g.nchunks) symn[t * 64 + lane] = cs.n;
      } else {
        ShiftSink q;
        q.act = s_ac + tab * 256;
        q.dct = s_dc + tab * 16;
        q.stage = stage;
        if (active) {
          emit_block(s_pk + lane, mask, diff, s_zd, s_m2, q);
          q.finish();
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
