// C-ABI of libmjgpu.so (declarations and boundary citations: include/mjgpu.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cctype>
#include <climits>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mjgpu.h"
#include "jpeg_tables.h"
#include "kernels.hip"
#include "scale.hip"
#include "sws_filter.h"

using namespace mjg;

namespace {


thread_local std::string g_err = "no error";

int set_err(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                                   \
  do {                                                                                  \
    hipError_t e_ = (expr);                                                             \
    if (e_ != hipSuccess) return set_err(MJG_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
  } while (0)

// JPEG header of the profile: mjpegenc_common.c ff_mjpeg_encode_picture_header for
// AV_CODEC_ID_MJPEG, -bitexact (no COM), equal luma/chroma matrices (one DQT), DRI only
// with slice threading (RST mode), -huffman default (one DHT with DC0, DC1, AC0, AC1);
// SOF0 sampling factors from ff_mjpeg_init_hvsample.
struct ByteWriter {
  std::vector<uint8_t> b;
  void u8(int v) { b.push_back((uint8_t)v); }
  void u16(int v) { u8(v >> 8); u8(v); }
};

// (h, v) sampling factors of Y, Cb, Cr (ff_mjpeg_init_hvsample; 4:4:4 is all 1x2).
void hvsample(int cfmt, int hs[3], int vs[3]) {
  if (cfmt == MJG_CHROMA_444) {
    hs[0] = hs[1] = hs[2] = 1;
    vs[0] = vs[1] = vs[2] = 2;
    return;
  }
  hs[0] = vs[0] = 2;
  hs[1] = hs[2] = 1;
  vs[1] = vs[2] = cfmt == MJG_CHROMA_422 ? 2 : 1;
}

std::vector<uint8_t> build_header(int w, int h, const uint8_t mprime[64], int sar_num, int sar_den,
                                  bool com_itu601, int cfmt, bool rst, size_t *dht_pos = nullptr,
                                  size_t *dht_end = nullptr) {
  int hs[3], vs[3];
  hvsample(cfmt, hs, vs);
  ByteWriter o;
  o.u16(0xFFD8);
  if (sar_num > 0 && sar_den > 0) {
    o.u16(0xFFE0);
    o.u16(16);
    for (char c : {'J', 'F', 'I', 'F', '\0'}) o.u8(c);
    o.u16(0x0102);
    o.u8(0);
    o.u16(sar_num);
    o.u16(sar_den);
    o.u8(0);
    o.u8(0);
  }
  if (com_itu601) {  // jpeg_put_comments: COM "CS=ITU601" when the encoder pix_fmt is yuv420p
    o.u16(0xFFFE);
    o.u16(12);
    for (char ch : {'C', 'S', '=', 'I', 'T', 'U', '6', '0', '1', '\0'}) o.u8(ch);
  }
  o.u16(0xFFDB);
  o.u16(2 + 65);
  o.u8(0x00);
  for (int i = 0; i < 64; i++) o.u8(mprime[kZigzag[i]]);
  if (rst) {  // jpeg_table_header: DRI, interval = MCUs per MCU row
    o.u16(0xFFDD);
    o.u16(4);
    o.u16((w - 1) / (8 * hs[0]) + 1);
  }
  if (dht_pos) *dht_pos = o.b.size();
  o.u16(0xFFC4);
  const size_t len_at = o.b.size();
  o.u16(0);
  auto table = [&](int cls_id, const uint8_t *bits, const uint8_t *vals) {
    o.u8(cls_id);
    int n = 0;
    for (int i = 1; i <= 16; i++) {
      o.u8(bits[i]);
      n += bits[i];
    }
    for (int i = 0; i < n; i++) o.u8(vals[i]);
  };
  table(0x00, kBitsDcLum, kValDc);
  table(0x01, kBitsDcChr, kValDc);
  table(0x10, kBitsAcLum, kValAcLum);
  table(0x11, kBitsAcChr, kValAcChr);
  const size_t dht_len = o.b.size() - len_at;
  o.b[len_at] = (uint8_t)(dht_len >> 8);
  o.b[len_at + 1] = (uint8_t)dht_len;
  if (dht_end) *dht_end = o.b.size();
  o.u16(0xFFC0);
  o.u16(17);
  o.u8(8);
  o.u16(h);
  o.u16(w);
  o.u8(3);
  for (int c = 0; c < 3; c++) {
    o.u8(c + 1);
    o.u8((hs[c] << 4) | vs[c]);
    o.u8(0);
  }
  o.u16(0xFFDA);
  o.u16(12);
  o.u8(3);
  o.u8(1); o.u8(0x00);
  o.u8(2); o.u8(0x11);
  o.u8(3); o.u8(0x11);
  o.u8(0); o.u8(63); o.u8(0);
  return o.b;
}

template <typename T>
int dmalloc(T **p, size_t count) {
  *p = nullptr;
  if (count == 0) return MJG_OK;
  if (hipMalloc((void **)p, count * sizeof(T)) != hipSuccess) {
    *p = nullptr;
    (void)hipGetLastError();
    return set_err(MJG_E_NOMEM, "hipMalloc(%zu bytes) failed", count * sizeof(T));
  }
  return MJG_OK;
}

struct PlaneScale {
  SwsFilter hf, vf;
  int32_t *hcp = nullptr, *hp = nullptr, *vcp = nullptr, *vps = nullptr, *hsum = nullptr;
  int32_t *mfb = nullptr;  // k_scale's matrix-core h-pass: the B fragments (ScaleGeom::mf_*)
  bool d4 = false;  // h coefficients in the v_dot4 hi/lo byte layout (k_scale D4)
  ScaleGeom g{};
  size_t lds = 0;
  dim3 grid;
  int th = 32;  // k_scale tile height (64: the 2:1 filters, scale.hip)
};

// Per-submit state.  A context has kSlots slots so further mjg_submits can be queued before
// the first is synced; everything a submit's results and its overflow re-write need lives
// in its slot.  Slots 1.. are allocated on the first pipelined submits.  Each slot has its
// own stream for H2D, scale and k_encode; the tail stream runs a submit's scan/stuff/write
// kernels after its k_encode (event enc_done), so the latency-bound tail of submit A runs
// beside the VALU-bound k_encode of submit B.  A slot is reused only after the host synced
// its previous submit (mjg_sync waits for `done`), so no device-side wait guards it.
// Two deep: a persistent k_encode holds every CU until its drain, so the host's sync of
// submit s-1 (whose slot submit s+1 reuses) waits for its tail, which gets CUs only as submit
// s's k_encode drains; the tail stream therefore runs at the highest priority (its
// workgroups dispatch before the next k_encode's).  Three slots measured 10% slower: three
// k_encode launches then share the CUs (DESIGN §4 streams; tools/patches.py slots3).
constexpr int kSlots = 2;
// Library-side merging (r05): single-segment device submits are held while the GPU has a
// launch queued and launched kMerge at a time as one segment list (submit_impl's SegList),
// so the launch's ramp and drain (T(n) = 0.115 ms + 4.48 us n per 4K launch) is
// paid once per kMerge submits.  Each submit stays a job of its own for mjg_sync / mjg_fetch.
constexpr int kMerge = 2;
// k_emit_syms workgroups per k_encode workgroup: the replay waits on memory most of its time
// and needs 54 VGPRs and 8.7 KB of LDS, so more waves per SIMD than k_encode's four hide that
// latency.  Since each wave replays a run of consecutive chunks (one table load per frame
// instead of one per chunk), x2 is the best grid: bench c1 x1 / x2 / x4 0.526-0.529 /
// 0.508-0.512 / 0.506-0.522 ms per step (profiles/r05/c1_emit_runs_ab.txt; with strided chunks
// x4 was best, profiles/r05/c1_emit_grid_bench.txt)
constexpr int kEmitGridMul = 2;
// merging is off when the slots' doubled scratch would take more than this share of the
// device's free memory (slot buffers scale with the frames a launch may carry)
constexpr double kMergeMemShare = 0.25;
struct Slot {
  bool alloc = false, pending = false;
  int njobs = 0, nsynced = 0;       // submits (jobs) this launch carries / already synced
  int jf0[kMaxSegs] = {}, jn[kMaxSegs] = {};  // each job's first frame in the launch, frames
  hipStream_t st = nullptr;        // H2D, scale and k_encode of this slot's submits
  uint8_t *d_stage = nullptr;      // H2D staging for host submits (allocated on first use)
  uint8_t *d_scaled = nullptr;     // -vf scale: k_scale's output planes
  uint32_t *d_stage_bits = nullptr;  // k_encode: per wave, lane-major staging of blocks past 128 bits
  int n = 0;  // frames of the launch
  uint32_t *d_scratch = nullptr;
  uint32_t *d_stream = nullptr;  // k_count_ff's realigned words, per segment (k_write reads them)
  uint32_t *d_chunk_bits = nullptr, *d_chunk_off = nullptr, *d_group_ff = nullptr, *d_ff_off = nullptr;
  uint32_t *d_frame_bits = nullptr, *d_status = nullptr;
  uint32_t *d_work = nullptr;  // k_encode's batch counter (zero; reset by the slot's scan kernel)
  uint64_t *d_frame_size = nullptr, *d_frame_offsets = nullptr;
  uint32_t *d_seg_size = nullptr;  // RST mode: stuffed segment sizes and offsets after the header
  uint32_t *d_seg_off = nullptr;
  uint32_t *d_done = nullptr;      // k_scan_ff's frame ticket (one word, zeroed by k_scan_bits)
  uint8_t *d_out = nullptr;
  size_t out_cap = 0;
  uint32_t *d_hist = nullptr, *d_ftabs = nullptr, *d_dht_nval = nullptr, *d_hdr_lens = nullptr;  // optimal
  uint32_t *d_syms = nullptr, *d_symn = nullptr;  // optimal: per block, the symbols the counting pass saw
  uint8_t *d_dht = nullptr;
  int16_t *d_dbg = nullptr;
  uint64_t *h_sizes = nullptr;
  uint32_t *h_status = nullptr;
  hipEvent_t done = nullptr, enc_done = nullptr;
  hipEvent_t ev[MJG_NUM_KERNELS][2] = {};
};

}  // namespace

struct mjg_ctx {
  int device = 0;
  mjg_config cfg{};
  hipStream_t stream = nullptr;  // H2D, scale, k_encode of slot 0's submits
  hipStream_t more[kSlots - 1] = {};  // ... of slots 1..: consecutive submits' k_encode launches
                                      // overlap (the next starts on the CUs the previous drain frees)
  hipStream_t tail = nullptr;    // scans, stuffing, write, D2H of the sizes
  EncGeom geom{};
  int32_t qmat[64];
  int enc_grid = 0;             // persistent k_encode workgroups: every CU full (kEmitDefault)
  int enc_grid_cnt = 0;         // the same for the -huffman optimal counting pass (kCount: more LDS)
  bool scale = false;
  size_t in_frame_bytes = 0, enc_frame_bytes = 0;
  std::vector<uint8_t> hdr;
  uint8_t mprime[64];

  uint32_t *d_tabs = nullptr;
  uint8_t *d_hdr = nullptr;
  size_t stage_cols = 0;       // staging columns per slot (persistent waves of k_encode / k_emit_syms)
  bool rst = false;            // RST mode (MJG_F_RST, more than one MCU row)
  bool optimal = false;        // -huffman optimal
  size_t dht_pos = 0, dht_end = 0;
  PlaneScale ps[2];  // 0 luma, 1 chroma (U and V share)
  size_t slot_B = 0, slot_NC = 0, slot_NS = 0;  // slot sizes: frames, chunks and segments per frame

  Slot slot[kSlots];
  int head = 0;   // slot of the next launch
  int nout = 0;   // launches with jobs not yet synced (0..kSlots)
  int last = -1;  // slot of the last synced job (fetch / output_device / debug read it)
  int last_job = 0;            // that job's index in its launch
  uint64_t last_off = 0, last_total = 0;  // its packed bytes' offset in the launch's d_out, size
  bool synced_since_submit = false;
  int merge = 1;               // jobs per launch for single-segment device submits (kMerge or 1)
  bool hold_idle = true;       // hold a lone device job even on an idle GPU (MJG_MERGE_HOLD=0: launch it)
  int held = 0;                // device jobs held for the next launch (0..merge)
  const uint8_t *held_p[kMaxSegs] = {};
  int held_n[kMaxSegs] = {};
  int launches = 0;            // launches since open (tests / diagnostics)

  bool timing = false, timing_detail = false;
  bool timing_tail = false;  // MJG_F_TIMING's tail interval (MJG_TIMING_NOTAIL=1: off, A/B of the events' cost)
  uint8_t *h_fetch = nullptr;  // page-locked copy of the last fetched output (mjg_fetch_host)
  size_t h_fetch_cap = 0;
  double t_acc[MJG_NUM_KERNELS] = {0};
  int t_n = 0;
};

namespace {

void free_ctx(mjg_ctx *c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (hipStream_t st : c->more)
    if (st) (void)hipStreamSynchronize(st);
  if (c->tail) (void)hipStreamSynchronize(c->tail);
  void *ptrs[] = {c->d_tabs, c->d_hdr, c->ps[0].hcp,
                  c->ps[0].vcp, c->ps[0].hp, c->ps[0].vps, c->ps[1].hcp, c->ps[1].vcp, c->ps[1].hp,
                  c->ps[0].hsum, c->ps[1].hsum, c->ps[1].vps, c->ps[0].mfb, c->ps[1].mfb};
  for (void *p : ptrs)
    if (p) (void)hipFree(p);
  for (Slot &S : c->slot) {
    void *sp[] = {S.d_stage, S.d_scaled, S.d_stage_bits, S.d_scratch, S.d_stream, S.d_work, S.d_chunk_bits, S.d_chunk_off, S.d_group_ff, S.d_ff_off, S.d_frame_bits,
                  S.d_status, S.d_frame_size, S.d_frame_offsets, S.d_seg_size, S.d_seg_off, S.d_done, S.d_out,
                  S.d_hist, S.d_ftabs, S.d_dht_nval, S.d_hdr_lens, S.d_dht, S.d_dbg, S.d_syms, S.d_symn};
    for (void *p : sp)
      if (p) (void)hipFree(p);
    if (S.h_sizes) (void)hipHostFree(S.h_sizes);
    if (S.h_status) (void)hipHostFree(S.h_status);
    if (S.done) (void)hipEventDestroy(S.done);
    if (S.enc_done) (void)hipEventDestroy(S.enc_done);
    for (auto &e : S.ev) {
      if (e[0]) (void)hipEventDestroy(e[0]);
      if (e[1]) (void)hipEventDestroy(e[1]);
    }
  }
  if (c->h_fetch) (void)hipHostFree(c->h_fetch);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  for (hipStream_t st : c->more)
    if (st) (void)hipStreamDestroy(st);
  if (c->tail && c->tail != c->stream) (void)hipStreamDestroy(c->tail);
  delete c;
}

// chroma: plane subsampling shifts (hsub, vsub) select the siting get_local_pos(shift, -513)
int setup_plane_scale(mjg_ctx *c, PlaneScale &p, int sw, int sh, int dw, int dh, int chroma,
                      int hsub, int vsub, bool bitexact) {
  const int hpos = chroma ? sws_local_pos(hsub, -513) : sws_local_pos(0, 0);
  const int vpos = chroma ? sws_local_pos(vsub, -513) : sws_local_pos(0, 0);
  if (!make_sws_filter(sw, dw, 1 << 14, 4, bitexact, hpos, hpos, &p.hf) ||
      !make_sws_filter(sh, dh, 1 << 12, 2, bitexact, vpos, vpos, &p.vf))
    return set_err(MJG_E_INVALID, "scale %dx%d -> %dx%d needs swscale's cascade (unsupported)", sw,
                   sh, dw, dh);
  for (int i = 1; i < dw; i++)
    if (p.hf.pos[i] < p.hf.pos[i - 1]) return set_err(MJG_E_INVALID, "non-monotone hscale");
  for (int i = 1; i < dh; i++)
    if (p.vf.pos[i] < p.vf.pos[i - 1]) return set_err(MJG_E_INVALID, "non-monotone vscale");
  // h taps padded with zero coefficients to a multiple of 4 (k_scale takes 4 taps per step),
  // v taps of any count (the pair table below zero-pads).  A window may run past the row
  // end (tiny sources, padded taps): initFilter zeroes every coefficient past srcW, so the
  // bytes k_scale stages there never count.
  const int ht0 = p.hf.taps, vt = p.vf.taps;
  const int ht = (ht0 + 3) & ~3;
  std::vector<int16_t> hpad((size_t)dw * ht, 0);
  for (int x = 0; x < dw; x++)
    for (int k = 0; k < ht0; k++) hpad[(size_t)x * ht + k] = p.hf.coeff[(size_t)x * ht0 + k];
  // h: coefficient pairs per output column; v: pairs starting at the even row <= pos[y],
  // shifted by its parity and zero-padded to npv = vt/2 + 1 pairs
  const int npv = vt / 2 + 1;
  std::vector<int32_t> hcp((size_t)dw * (ht / 2)), vcp((size_t)dh * npv, 0), vps(dh);
  // D4 layout when every coefficient splits as 128 ch + cl, ch int8, cl in [-64, 64): per 4
  // taps one word of ch bytes and one of cl bytes (else the int16 pair layout)
  std::vector<int32_t> hsum(dw, 0);
  p.d4 = true;
  for (size_t i = 0; i < p.hf.coeff.size(); i++)
    if (p.hf.coeff[i] < -128 * 128 - 64 || p.hf.coeff[i] >= 127 * 128 + 64) p.d4 = false;
  for (int x = 0; x < dw; x++) {
    const int16_t *cx = &hpad[(size_t)x * ht];
    for (int k = 0; k < ht; k++) hsum[x] += cx[k];
    for (int k = 0; k < ht / 2; k++) {
      uint32_t wv;
      if (p.d4) {
        const int g4 = k >> 1, lo_part = k & 1;  // word 2j: ch of taps 4j..4j+3, word 2j+1: cl
        wv = 0;
        for (int b = 0; b < 4; b++) {
          const int cv = cx[4 * g4 + b], cl = ((cv + 64) & 127) - 64, ch = (cv - cl) / 128;
          wv |= (uint32_t)(uint8_t)(int8_t)(lo_part ? cl : ch) << (8 * b);
        }
      } else {
        wv = (uint32_t)(uint16_t)cx[2 * k] | ((uint32_t)(uint16_t)cx[2 * k + 1] << 16);
      }
      hcp[(size_t)x * (ht / 2) + k] = (int32_t)wv;
    }
  }
  for (int y = 0; y < dh; y++) {
    const int r = p.vf.pos[y], par = r & 1;
    vps[y] = r >> 1;
    for (int k = 0; k < npv; k++) {
      const int j0 = 2 * k - par, j1 = j0 + 1;
      const uint16_t c0 = (j0 >= 0 && j0 < vt) ? (uint16_t)p.vf.coeff[(size_t)y * vt + j0] : 0;
      const uint16_t c1 = (j1 >= 0 && j1 < vt) ? (uint16_t)p.vf.coeff[(size_t)y * vt + j1] : 0;
      vcp[(size_t)y * npv + k] = (int32_t)((uint32_t)c0 | ((uint32_t)c1 << 16));
    }
  }
  // k_scale's tile height: 64 rows for the 2:1 filters when every window fits the fast path
  // at a 36-dword row stride (scale.hip), else 32
  auto tile_pairs = [&](int th) {
    int m = 0;
    for (int y0 = 0; y0 < dh; y0 += th) m = std::max(m, vps[std::min(y0 + th, dh) - 1] + npv - vps[y0]);
    return m;
  };
  int max_nw = 0;
  for (int x0 = 0; x0 < dw; x0 += kScaleTileW) {  // same formula as k_scale's window
    const int xe = std::min(x0 + kScaleTileW, dw), cb = p.hf.pos[x0] & ~3;
    max_nw = std::max(max_nw, ((((p.hf.pos[xe - 1] + ht - cb + 3) >> 2) + 1) + 3) & ~3);
  }
  const int th2 = 64;  // tile height for the 2:1 filters
  const int th = (ht == 8 && npv == 5 && max_nw <= kScaleAliasWords && sw >= 16 &&
                  2 * tile_pairs(th2) <= scale_waves(th2) * scale_loads_per_wave(th2) * kScaleLoadRows) ? th2 : 32;
  const int max_pairs = tile_pairs(th);
  p.th = th;
  ScaleGeom &g = p.g;
  g.htaps = ht;
  g.vtaps = vt;
  g.npv = npv;
  g.lds_pairs = max_pairs;
  if (th >= 64) {  // pair image over the window rows (scale.hip: ALIAS)
    g.lds_win_words = 2 * max_pairs * kScaleAliasWords;
    p.lds = (size_t)g.lds_win_words * 4 + 64;  // v filter rows by scalar loads; the matrix-core
                                               // h-pass reads 16 bytes past the last row
  } else {
    g.lds_win_words = 2 * max_pairs * max_nw;
    p.lds = ((size_t)g.lds_win_words + (size_t)max_pairs * kScaleTileW + (size_t)th * (npv + 1)) * 4;
  }
  if (p.lds > 64 * 1024)
    return set_err(MJG_E_INVALID, "scale ratio too large for one LDS tile (%zu B)", p.lds);
  p.grid = dim3((dw + kScaleTileW - 1) / kScaleTileW, (dh + th - 1) / th, 1);
  int rc;
  if ((rc = dmalloc(&p.hcp, hcp.size())) || (rc = dmalloc(&p.hp, (size_t)dw)) ||
      (rc = dmalloc(&p.vcp, vcp.size())) || (rc = dmalloc(&p.vps, (size_t)dh)) ||
      (rc = dmalloc(&p.hsum, (size_t)dw)))
    return rc;
  HIP_TRY(hipMemcpy(p.hsum, hsum.data(), (size_t)dw * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(p.hcp, hcp.data(), hcp.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(p.hp, p.hf.pos.data(), (size_t)dw * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(p.vcp, vcp.data(), vcp.size() * 4, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(p.vps, vps.data(), (size_t)dh * 4, hipMemcpyHostToDevice));
  // The matrix-core h-pass (scale.hip, scale_hpass_mf) for the interior tile columns when they
  // all share one filter at a 2-byte step (exact 2:1): B[k][n] = the hi (lo) byte of tap
  // k - 2n - d of that filter (0 outside the 8 taps), k the byte of a 64-byte window that starts
  // at the column block's aligned byte 32 cj, d = the first column's byte offset in its dword.
  // Lane l holds B[16 (l >> 4) + j][l & 15] in byte j (the same k map as its A fragment).
  g.mf_bx0 = g.mf_bx1 = 0;
  g.mf_hs = 0;
  const int gxt = (dw + kScaleTileW - 1) / kScaleTileW;
  if (p.d4 && ht == 8 && th >= 64 && gxt >= 3) {
    const int xa = kScaleTileW, xb = kScaleTileW * (gxt - 1);
    bool ok = true;
    for (int x = xa; x < xb && ok; x++) {
      ok = p.hf.pos[x] == p.hf.pos[xa] + 2 * (x - xa) && hsum[x] == hsum[xa];
      for (int k = 0; k < ht / 2 && ok; k++) ok = hcp[(size_t)x * (ht / 2) + k] == hcp[(size_t)xa * (ht / 2) + k];
    }
    if (ok) {
      const int d = p.hf.pos[xa] & 3;
      std::vector<int32_t> mfb(kMvFragOff + 3 * 64 * 4, 0);
      for (int l = 0; l < 64; l++)
        for (int j = 0; j < 16; j++) {
          const int k = 16 * (l >> 4) + j, n = l & 15, t = k - 2 * n - d;
          if (t < 0 || t >= 8) continue;
          const uint32_t hi = ((uint32_t)hcp[(size_t)xa * (ht / 2) + 2 * (t >> 2)] >> (8 * (t & 3))) & 255u;
          const uint32_t lo = ((uint32_t)hcp[(size_t)xa * (ht / 2) + 2 * (t >> 2) + 1] >> (8 * (t & 3))) & 255u;
          mfb[(size_t)l * 8 + (j >> 2)] |= (int32_t)(hi << (8 * (j & 3)));
          mfb[(size_t)l * 8 + 4 + (j >> 2)] |= (int32_t)(lo << (8 * (j & 3)));
        }
      // The matrix-core v-pass (scale.hip) for the interior tile rows of those columns when they
      // all share one v filter at a 2-row step: A[m][k] = tap k - 2m - delta of it (0 outside the
      // 8 taps), delta = the parity of its first row (the window starts at the even row below),
      // split as tap = 128 fh + fl: fragments fh, fl and 2 fl, lane l holding A[l & 15][16 (l >> 4)
      // + j] in byte j (the h-pass's k map)
      const int gyt = (dh + th - 1) / th, ya = th, yb = th * (gyt - 1);
      bool vok = gyt >= 3 && vt == 8 && 2 * 64 * kPlaneStride + 16 <= (int)p.lds;
      for (int y = ya; y < yb && vok; y++) {
        vok = p.vf.pos[y] == p.vf.pos[ya] + 2 * (y - ya);
        for (int k = 0; k < vt && vok; k++) vok = p.vf.coeff[(size_t)y * vt + k] == p.vf.coeff[(size_t)ya * vt + k];
      }
      int fsum = 0;
      for (int k = 0; k < vt && vok; k++) {
        const int cv = p.vf.coeff[(size_t)ya * vt + k], fl = ((cv + 64) & 127) - 64;
        vok = (cv - fl) / 128 >= -128 && (cv - fl) / 128 <= 127;
        fsum += cv;
      }
      g.mv_by0 = g.mv_by1 = 0;
      g.mv_k = 0;
      if (vok) {
        const int delta = p.vf.pos[ya] & 1;
        for (int l = 0; l < 64; l++)
          for (int j = 0; j < 16; j++) {
            const int m = l & 15, k = 16 * (l >> 4) + j, t = k - 2 * m - delta;
            const int cv = (t >= 0 && t < 8) ? p.vf.coeff[(size_t)ya * vt + t] : 0;
            const int fl = ((cv + 64) & 127) - 64, fh = (cv - fl) / 128;
            const int vals[3] = {fh, fl, 2 * fl};
            for (int f = 0; f < 3; f++)
              mfb[kMvFragOff + (size_t)(f * 64 + l) * 4 + (j >> 2)] |= (int32_t)((uint32_t)(uint8_t)(int8_t)vals[f] << (8 * (j & 3)));
          }
        g.mv_by0 = 1;
        g.mv_by1 = gyt - 1;
        g.mv_k = 128 * fsum + (64 << 12);
      }
      if ((rc = dmalloc(&p.mfb, mfb.size()))) return rc;
      HIP_TRY(hipMemcpy(p.mfb, mfb.data(), mfb.size() * 4, hipMemcpyHostToDevice));
      g.mf_bx0 = 1;
      g.mf_bx1 = gxt - 1;
      g.mf_hs = hsum[xa];
    }
  }
  (void)c;
  return MJG_OK;
}

hipStream_t slot_stream(const mjg_ctx *c, int i) { return i ? c->more[i - 1] : c->stream; }

int alloc_slot(mjg_ctx *c, Slot &S) {
  const size_t B = c->slot_B, NC = c->slot_NC, NS = c->slot_NS;
  const EncGeom &g = c->geom;
  int rc;
  // Each slot on its own stream: consecutive submits (queued kSlots deep) overlap, so the next
  // submit's launches start on the CUs the previous one's drain frees.  A persistent k_encode's
  // waves finish its last work units over ~140 us (the SIMD arbiter runs its oldest wave 2.2x
  // faster than its youngest), and a workgroup's slot frees when its last wave
  // ends.  A/B: c2 +5.4% (bench.py, r04), c5 +1.6%, c1 +24% and c4 +1.7% (r03, chains of
  // launches).  Each launch's own event interval then includes its neighbour's overlap.
  S.st = slot_stream(c, (int)(&S - c->slot));
  if ((rc = dmalloc(&S.d_stage_bits, c->stage_cols * 64 * kStageWords))) return rc;
  if (c->scale && (rc = dmalloc(&S.d_scaled, B * c->enc_frame_bytes))) return rc;
  if ((rc = dmalloc(&S.d_scratch, B * NC * (size_t)kSlotWords)) ||
      (rc = dmalloc(&S.d_stream, B * NC * (size_t)kSlotWords)) ||
      (rc = dmalloc(&S.d_chunk_bits, B * NC)) || (rc = dmalloc(&S.d_chunk_off, B * NC)) ||
      (rc = dmalloc(&S.d_group_ff, B * NC)) || (rc = dmalloc(&S.d_ff_off, B * NC)) ||
      (rc = dmalloc(&S.d_frame_bits, B * NS)) || (rc = dmalloc(&S.d_status, 4)) ||
      (rc = dmalloc(&S.d_frame_size, B)) || (rc = dmalloc(&S.d_frame_offsets, B + 1)) ||
      (rc = dmalloc(&S.d_done, 1)) ||
      (rc = dmalloc(&S.d_work, (size_t)kXcds * kCtrStride)))
    return rc;
  HIP_TRY(hipMemset(S.d_work, 0, (size_t)kXcds * kCtrStride * sizeof(uint32_t)));
  if (c->rst && ((rc = dmalloc(&S.d_seg_size, B * NS)) || (rc = dmalloc(&S.d_seg_off, B * NS)))) return rc;
  S.out_cap = B * (c->enc_frame_bytes + c->hdr.size() + 4096 + 2 * NS);
  if ((rc = dmalloc(&S.d_out, S.out_cap))) return rc;
  if (c->optimal &&
      ((rc = dmalloc(&S.d_hist, B * kFrameTabWords)) || (rc = dmalloc(&S.d_ftabs, B * kFrameTabWords)) ||
       (rc = dmalloc(&S.d_dht, B * 4 * kDhtSlot)) || (rc = dmalloc(&S.d_dht_nval, B * 4)) ||
       (rc = dmalloc(&S.d_hdr_lens, B)) || (rc = dmalloc(&S.d_syms, B * NC * (size_t)kSymCap * 64)) ||
       (rc = dmalloc(&S.d_symn, B * NC * 64))))
    return rc;
  if (g.debug_coefs && (rc = dmalloc(&S.d_dbg, B * (size_t)g.nmcu * g.bpm * 64))) return rc;
  HIP_TRY(hipHostMalloc((void **)&S.h_sizes, (B + 1) * sizeof(uint64_t), hipHostMallocDefault));
  HIP_TRY(hipHostMalloc((void **)&S.h_status, 16, hipHostMallocDefault));
  HIP_TRY(hipEventCreateWithFlags(&S.done, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&S.enc_done, hipEventDisableTiming));
  if (c->timing)
    for (auto &e : S.ev) {
      HIP_TRY(hipEventCreate(&e[0]));
      HIP_TRY(hipEventCreate(&e[1]));
    }
  S.alloc = true;
  return MJG_OK;
}

int open_ctx(int device, const mjg_config *cfg, mjg_ctx *c) {
  c->device = device;
  c->cfg = *cfg;
  const mjg_config &k = *cfg;
  if (k.src_w < 1 || k.src_h < 1 || k.dst_w < 1 || k.dst_h < 1 || k.src_w > 16384 ||
      k.src_h > 16384 || k.dst_w > 16384 || k.dst_h > 16384)
    return set_err(MJG_E_INVALID, "bad frame size %dx%d -> %dx%d", k.src_w, k.src_h, k.dst_w, k.dst_h);
  if (k.qscale < 1 || k.qscale > 31) return set_err(MJG_E_INVALID, "qscale %d not in 1..31", k.qscale);
  if (k.max_batch < 1 || k.max_batch > 65535)
    return set_err(MJG_E_INVALID, "max_batch %d not in 1..65535", k.max_batch);
  if (k.sar_num < 0 || k.sar_den < 0 || k.sar_num > 65535 || k.sar_den > 65535)
    return set_err(MJG_E_INVALID, "bad SAR %d:%d", k.sar_num, k.sar_den);
  if (k.chroma_format < MJG_CHROMA_420 || k.chroma_format > MJG_CHROMA_444)
    return set_err(MJG_E_INVALID, "chroma_format %d", k.chroma_format);
  constexpr uint32_t kKnownFlags = MJG_F_TIMING | MJG_F_DEBUG_COEFS | MJG_F_SWS_NO_BITEXACT | MJG_F_COM_ITU601 |
                                   MJG_F_HUFFMAN_OPTIMAL | MJG_F_RST | MJG_F_TIMING_DETAIL | MJG_F_MERGE;
  if (k.flags & ~kKnownFlags)  // retired bits (128, 256, 512: r05's FUSED / DCT_MFMA / DCT_VALU) included
    return set_err(MJG_E_INVALID, "unknown flags 0x%x", k.flags & ~kKnownFlags);
  if ((k.flags & MJG_F_RST) && (k.flags & MJG_F_HUFFMAN_OPTIMAL))
    return set_err(MJG_E_INVALID, "RST (slice threading) forces -huffman default");

  int ndev = 0;
  HIP_TRY(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return set_err(MJG_E_INVALID, "device %d of %d", device, ndev);
  HIP_TRY(hipSetDevice(device));
  HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  for (hipStream_t &st : c->more) HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int least = 0, greatest = 0;  // the tail's workgroups first (see kSlots)
  HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
  HIP_TRY(hipStreamCreateWithPriority(&c->tail, hipStreamNonBlocking, greatest));

  c->scale = (k.src_w != k.dst_w || k.src_h != k.dst_h);
  const int cf = k.chroma_format;
  const int hsh = cf == MJG_CHROMA_444 ? 0 : 1, vsh = cf == MJG_CHROMA_420 ? 1 : 0;
  const int scw = (k.src_w + hsh) >> hsh, sch = (k.src_h + vsh) >> vsh;
  const int w = k.dst_w, h = k.dst_h, cw = (w + hsh) >> hsh, ch = (h + vsh) >> vsh;
  c->in_frame_bytes = (size_t)k.src_w * k.src_h + 2 * (size_t)scw * sch;
  c->enc_frame_bytes = (size_t)w * h + 2 * (size_t)cw * ch;

  EncGeom &g = c->geom;
  g.w = w;
  g.h = h;
  g.cw = cw;
  g.ch = ch;
  g.bpm = cf == MJG_CHROMA_422 ? 8 : 6;
  g.bpm_magic = (uint32_t)((((uint64_t)1 << 32) + (uint64_t)g.bpm - 1) / (uint64_t)g.bpm);
  g.lmw = cf == MJG_CHROMA_444 ? 8 : 16;
  g.cmh = cf == MJG_CHROMA_420 ? 8 : 16;
  g.mbw = (w + g.lmw - 1) / g.lmw;
  const int mbh = (h + 15) / 16;
  g.nmcu = g.mbw * mbh;
  g.mbw_magic = g.mbw > 1 ? (uint32_t)((((uint64_t)1 << 32) + (uint64_t)g.mbw - 1) / (uint64_t)g.mbw) : 0u;
  if ((uint64_t)(g.nmcu + 64) * (uint64_t)g.mbw >= ((uint64_t)1 << 32))
    return set_err(MJG_E_INVALID, "frame too large (%d MCUs)", g.nmcu);
  // RST: one segment per MCU row (mpegvideo clips the slice count to mb_height, so a
  // single-row picture has no restart markers)
  c->rst = (k.flags & MJG_F_RST) && mbh > 1;
  g.nseg = c->rst ? mbh : 1;
  g.seg_blocks = (c->rst ? g.mbw : g.nmcu) * g.bpm;
  g.nchunks = (g.seg_blocks + 63) / 64;  // chunks of 64 blocks (one wave each) per segment
  g.nchunks_magic = (((unsigned long long)1 << 40) + (unsigned long long)g.nchunks - 1) / (unsigned long long)g.nchunks;
  g.nseg_magic = (((unsigned long long)1 << 40) + (unsigned long long)g.nseg - 1) / (unsigned long long)g.nseg;
  // task t / nchunks by magic (exact while t * nchunks < 2^40, t < max_batch * nseg * nchunks)
  if ((unsigned long long)k.max_batch * g.nseg * g.nchunks * g.nchunks >= ((unsigned long long)1 << 40))
    return set_err(MJG_E_INVALID, "max_batch %d too large for this frame size", k.max_batch);
  g.y_stride = w;
  g.c_stride = cw;
  g.u_off = (long long)w * h;
  g.v_off = g.u_off + (long long)cw * ch;
  g.frame_stride = (long long)c->enc_frame_bytes;
  if (c->enc_frame_bytes >= ((size_t)1 << 32))  // k_encode addresses a frame with 32-bit offsets
    return set_err(MJG_E_INVALID, "frame of %zu bytes", c->enc_frame_bytes);
  g.range_convert = (!c->scale && !k.in_full_range) ? 1 : 0;
  g.debug_coefs = (k.flags & MJG_F_DEBUG_COEFS) ? 1 : 0;

  // mpegvideo_enc.c encode_picture FMT_MJPEG matrix + ff_convert_matrix (qscale -> 8).
  for (int i = 0; i < 64; i++) {
    int v = i == 0 ? 8 : ((kMpeg1Intra[i] * k.qscale) >> 3);
    v = v > 255 ? 255 : v;
    c->mprime[i] = (uint8_t)v;
    c->qmat[i] = (int32_t)((2ull << 21) / (uint64_t)(16 * v));
  }
  c->hdr = build_header(w, h, c->mprime, k.sar_num, k.sar_den, (k.flags & MJG_F_COM_ITU601) != 0, cf,
                        c->rst, &c->dht_pos, &c->dht_end);
  c->optimal = (k.flags & MJG_F_HUFFMAN_OPTIMAL) != 0;

  // device table block: [0,256) AC luma, [256,512) AC chroma, [512,528) DC luma,
  // [528,544) DC chroma ((len << 16) | code), [544,608) qmat column-major ([col][row]),
  // [608,672) k_encode's screening thresholds B^2 (fp32 bits, [col][row]): a quantised AC
  // coefficient is nonzero iff |u| >= T = ceil(5*2^18 / qmat) (dct_quantize_c intra
  // rounding), i.e. |pass-2 sum| >= 16T - 8 (rows 0, 4: DESCALE 4, exact in fp32) or
  // >= T*2^17 - 2^16 (other rows); the latter is widened by 2048 > the fp32 error (< 2^9).
  uint32_t tabs[kTabWords] = {0};
  build_huffman(tabs, kBitsAcLum, kValAcLum);
  build_huffman(tabs + 256, kBitsAcChr, kValAcChr);
  uint32_t dc[256];
  build_huffman(dc, kBitsDcLum, kValDc);
  for (int i = 0; i < 16; i++) tabs[512 + i] = dc[i];
  build_huffman(dc, kBitsDcChr, kValDc);
  for (int i = 0; i < 16; i++) tabs[528 + i] = dc[i];
  for (int i = 0; i < 64; i++) tabs[544 + (i & 7) * 8 + (i >> 3)] = (uint32_t)c->qmat[i];  // [col][row]
  for (int i = 1; i < 64; i++) {
    const int ro = i >> 3;
    const uint32_t qm = (uint32_t)c->qmat[i];
    const double Ti = (double)(((5u << 18) + qm - 1) / qm);  // ceil(5*2^18 / qmat)
    const double B = (ro == 0 || ro == 4) ? 16.0 * Ti - 8.5 : Ti * 131072.0 - 65536.0 - 2048.0;
    const float b2 = (float)(B * B);
    memcpy(&tabs[608 + (i & 7) * 8 + ro], &b2, 4);
  }
  // [680, 689): k_encode's column-skip limits for column pairs 1-3 (columns 2-7), three u16x2
  // words per pair: Rmax, HI, LO.  A column's AC outputs all quantise to zero if
  //   row 0:  |S| = |sum u_r| <= 16 T - 9          <= 8 max|u_r|, max|u_r| <= 2T - 2
  //   row 4:  |S| = |sum +-u_r| <= 16 T - 9        <= 4 R  (the +-1 row sums to 0)
  //   others: |S| <= T 2^17 - 2^16 - 1             <= L1(row) R / 2
  // (T = ceil(5 2^18 / qmat) of that output, R = max - min of the column's row-pass values
  // u_r, S the pass-2 sum before DESCALE; dct_quantize_c gives 0 iff |DESCALE(S)| < T).  With
  // U = u + 16384 (the u16 image, columns 1-7): skip iff R <= Rmax, max U <= HI, min U >= LO.
  {
    static const int kDot[64] = MJG_PASS2_DOT;
    for (int jp = 1; jp < 4; jp++) {
      uint32_t lim[3] = {0, 0, 0};
      for (int h = 0; h < 2; h++) {
        const int col = 2 * jp + h;
        long long rmax = 65535, amax = 0;
        for (int ro = 0; ro < 8; ro++) {
          const long long qm = c->qmat[ro * 8 + col];
          const long long T = ((5ll << 18) + qm - 1) / qm;
          if (ro == 0) {
            amax = std::max(0ll, 2 * T - 2);
          } else if (ro == 4) {
            rmax = std::min(rmax, 4 * T - 3);
          } else {
            long long l1 = 0;
            for (int r = 0; r < 8; r++) l1 += std::abs(kDot[ro * 8 + r]);
            rmax = std::min(rmax, (2 * (T * 131072 - 65536 - 1)) / l1);
          }
        }
        rmax = std::max(0ll, rmax);
        const long long hi = std::min(65535ll, 16384 + amax), lo = std::max(0ll, 16384 - amax);
        lim[0] |= (uint32_t)rmax << (16 * h);
        lim[1] |= (uint32_t)hi << (16 * h);
        lim[2] |= (uint32_t)lo << (16 * h);
      }
      for (int i = 0; i < 3; i++) tabs[680 + 3 * (jp - 1) + i] = lim[i];
    }
  }
  // [672, 680): block-of-MCU descriptors in coding order (EncGeom): plane | chroma table << 2 |
  // dx8 << 3 | dy8 << 4 | DC predecessor distance << 8 (ff_mjpeg_encode_mb order; the
  // predecessor is the previous block of the same component)
  {
    static const uint8_t kPlane[3][8] = {{0, 0, 0, 0, 1, 2}, {0, 0, 0, 0, 1, 1, 2, 2}, {0, 0, 1, 1, 2, 2}};
    static const uint8_t kDx[3][8] = {{0, 1, 0, 1, 0, 0}, {0, 1, 0, 1, 0, 0, 0, 0}, {0, 0, 0, 0, 0, 0}};
    static const uint8_t kDy[3][8] = {{0, 0, 1, 1, 0, 0}, {0, 0, 1, 1, 0, 1, 0, 1}, {0, 1, 0, 1, 0, 1}};
    for (int j = 0; j < g.bpm; j++) {
      const int pl = kPlane[cf][j];
      int delta = 0;  // distance back to the previous block of plane pl (wrapping to the previous MCU)
      for (int d = 1; d <= g.bpm && !delta; d++)
        if (kPlane[cf][((j - d) % g.bpm + g.bpm) % g.bpm] == pl) delta = d;
      tabs[672 + j] = (uint32_t)pl | (pl ? 4u : 0u) | ((uint32_t)kDx[cf][j] << 3) |
                      ((uint32_t)kDy[cf][j] << 4) | ((uint32_t)delta << 8);
    }
  }

  const size_t NC = (size_t)g.nchunks * g.nseg, NS = (size_t)g.nseg;
  // merging (kMerge): opt-in with MJG_F_MERGE (a held submit's frames are read after mjg_submit
  // returns); MJG_MERGE=1 turns it off for a process (A/B), =2..4 sets the jobs per launch
  c->merge = 1;
  if (k.flags & MJG_F_MERGE) {
    c->merge = kMerge;
    if (const char *e = getenv("MJG_MERGE")) c->merge = std::max(1, std::min(kMaxSegs, atoi(e)));
  }
  if (const char *e = getenv("MJG_MERGE_HOLD")) c->hold_idle = atoi(e) != 0;
  if (c->merge > 1) {  // slot buffers for merge * max_batch frames: within a share of free memory
    size_t fr = 0, tot = 0;
    HIP_TRY(hipMemGetInfo(&fr, &tot));
    const double per_frame = 2.0 * (double)NC * kSlotWords * 4 + 2.0 * (double)c->enc_frame_bytes;
    if (kSlots * (double)c->merge * (double)k.max_batch * per_frame > kMergeMemShare * (double)fr) c->merge = 1;
  }
  if ((unsigned long long)k.max_batch * c->merge * g.nseg * g.nchunks * g.nchunks >= ((unsigned long long)1 << 40))
    c->merge = 1;  // merged launches would overflow k_encode's task magic (checked for max_batch above)
  const size_t B = (size_t)k.max_batch * (size_t)c->merge;  // frames one launch may carry
  int rc;
  if ((rc = dmalloc(&c->d_tabs, kTabWords)) || (rc = dmalloc(&c->d_hdr, c->hdr.size()))) return rc;
  c->slot_B = B;
  c->slot_NC = NC;
  c->slot_NS = NS;
  c->timing = (k.flags & (MJG_F_TIMING | MJG_F_TIMING_DETAIL)) != 0;
  c->timing_detail = (k.flags & MJG_F_TIMING_DETAIL) != 0;
  c->timing_tail = c->timing && !c->timing_detail && !(getenv("MJG_TIMING_NOTAIL") && atoi(getenv("MJG_TIMING_NOTAIL")));
  HIP_TRY(hipMemcpy(c->d_tabs, tabs, sizeof tabs, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(c->d_hdr, c->hdr.data(), c->hdr.size(), hipMemcpyHostToDevice));

  if (c->scale) {
    const bool bitexact = !(k.flags & MJG_F_SWS_NO_BITEXACT);
    if ((rc = setup_plane_scale(c, c->ps[0], k.src_w, k.src_h, w, h, 0, 0, 0, bitexact)) ||
        (rc = setup_plane_scale(c, c->ps[1], scw, sch, cw, ch, 1, hsh, vsh, bitexact)))
      return rc;
    for (int p = 0; p < 2; p++) {
      ScaleGeom &sg = c->ps[p].g;
      sg.sw = p ? scw : k.src_w;
      sg.sh = p ? sch : k.src_h;
      sg.dw = p ? cw : w;
      sg.dh = p ? ch : h;
      sg.s_stride = sg.sw;
      sg.d_stride = sg.dw;
      sg.s_fstride = (long long)c->in_frame_bytes;
      sg.d_fstride = (long long)c->enc_frame_bytes;
      sg.range = k.in_full_range ? 0 : (p ? 2 : 1);
    }
  }

  // persistent k_encode grid: every CU filled with as many workgroups as fit
  int ncu = 0, per_cu = 0;
  HIP_TRY(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device));
  HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(
      &per_cu, (const void *)k_encode<true, kEmitDefault>, 64 * kWavesPerWg, 0));
  c->enc_grid = std::max(1, ncu * std::max(1, per_cu));
  // -huffman optimal's counting pass is launched with the same grid (4 workgroups per CU: its
  // histograms are 16-bit counter pairs, profiles/r05/c1_count_occupancy_ab.txt)
  c->enc_grid_cnt = c->enc_grid;
  c->stage_cols = (size_t)c->enc_grid * kWavesPerWg * (c->optimal ? kEmitGridMul : 1);
  return alloc_slot(c, c->slot[0]);
}

// HIP events: with MJG_F_TIMING around scale, huff, encode and the whole tail (scan .. write,
// reported as MJG_K_TAIL); with MJG_F_TIMING_DETAIL around every kernel (each event record
// costs ~10 us of GPU idle between the short tail kernels).
void tmark(mjg_ctx *c, Slot &S, int k, int end) {
  if (!c->timing) return;
  const bool tail = k == MJG_K_SCAN_BITS || k == MJG_K_COUNT_FF || k == MJG_K_SCAN_FF || k == MJG_K_WRITE;
  if (tail && !c->timing_detail) return;
  (void)hipEventRecord(S.ev[k][end], tail ? c->tail : S.st);
}

// status: reset the overflow flag first (the regrow path; a submit's scan kernel resets it)
int launch_write(mjg_ctx *c, Slot &S, int n, bool reset_status) {
  const EncGeom &g = c->geom;
  const int gps = (g.nchunks + kChunksPerWave - 1) / kChunksPerWave, ngroups = gps * n * g.nseg;
  if (reset_status) HIP_TRY(hipMemsetAsync(S.d_status, 0, 4, c->tail));
  tmark(c, S, MJG_K_WRITE, 0);
  k_write<<<(ngroups + 3) / 4, 256, 0, c->tail>>>(
      S.d_stream, S.d_chunk_bits, S.d_chunk_off, S.d_frame_bits, S.d_ff_off, g.nchunks, gps, g.nseg, n,
      S.d_seg_size, S.d_seg_off, S.d_frame_offsets, c->d_hdr, (int)c->hdr.size(),
      c->optimal ? S.d_hdr_lens : nullptr, (int)c->dht_pos, (int)c->dht_end, S.d_dht,
      c->optimal ? S.d_dht_nval : nullptr, S.d_out, (uint64_t)S.out_cap, S.d_status);
  tmark(c, S, MJG_K_WRITE, 1);
  if (c->timing_tail && !reset_status) (void)hipEventRecord(S.ev[MJG_K_TAIL][1], c->tail);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipMemcpyAsync(S.h_sizes, S.d_frame_size, n * sizeof(uint64_t), hipMemcpyDeviceToHost,
                         c->tail));
  HIP_TRY(hipMemcpyAsync(S.h_status, S.d_status, 4, hipMemcpyDeviceToHost, c->tail));
  HIP_TRY(hipEventRecord(S.done, c->tail));
  return MJG_OK;
}


template <int MODE, bool DBG>
void launch_encode2(mjg_ctx *c, Slot &S, const SegList &enc_in, int wgs, int ntasks) {
  const EncGeom &g = c->geom;
  if (g.range_convert)
    k_encode<true, MODE, DBG><<<wgs, 64 * kWavesPerWg, 0, S.st>>>(
        enc_in, g, c->d_tabs, S.d_scratch, S.d_chunk_bits, S.d_dbg, S.d_work, ntasks, S.d_hist,
        S.d_stage_bits, S.d_syms, S.d_symn);
  else
    k_encode<false, MODE, DBG><<<wgs, 64 * kWavesPerWg, 0, S.st>>>(
        enc_in, g, c->d_tabs, S.d_scratch, S.d_chunk_bits, S.d_dbg, S.d_work, ntasks, S.d_hist,
        S.d_stage_bits, S.d_syms, S.d_symn);
}

template <int MODE>
void launch_encode(mjg_ctx *c, Slot &S, const SegList &enc_in, int wgs, int ntasks) {
  if (c->geom.debug_coefs)
    launch_encode2<MODE, true>(c, S, enc_in, wgs, ntasks);
  else
    launch_encode2<MODE, false>(c, S, enc_in, wgs, ntasks);
}

}  // namespace

extern "C" {

int mjg_version(void) { return 100; }

const char *mjg_last_error(void) { return g_err.c_str(); }

int mjg_device_count(void) {
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n));
  return n;
}

int mjg_device_numa_node(int device) {
  char bus[64] = {0};
  HIP_TRY(hipDeviceGetPCIBusId(bus, (int)sizeof bus, device));
  for (char *p = bus; *p; p++) *p = (char)tolower((unsigned char)*p);
  char path[160];
  snprintf(path, sizeof path, "/sys/bus/pci/devices/%s/numa_node", bus);
  FILE *f = fopen(path, "r");
  if (!f) return -1;
  int node = -1;
  if (fscanf(f, "%d", &node) != 1) node = -1;
  fclose(f);
  return node < 0 ? -1 : node;
}

int mjg_open(int device, const mjg_config *cfg, mjg_ctx **out) {
  if (!cfg || !out) return set_err(MJG_E_INVALID, "null argument");
  *out = nullptr;
  mjg_ctx *c = new mjg_ctx();
  const int rc = open_ctx(device, cfg, c);
  if (rc) {
    const std::string keep = g_err;
    free_ctx(c);
    g_err = keep;
    return rc;
  }
  *out = c;
  return MJG_OK;
}

void mjg_close(mjg_ctx *ctx) { free_ctx(ctx); }

size_t mjg_frame_bytes(const mjg_ctx *ctx) { return ctx ? ctx->in_frame_bytes : 0; }

int mjg_header(const mjg_ctx *ctx, uint8_t *out, size_t cap, size_t *len) {
  if (!ctx) return set_err(MJG_E_INVALID, "null ctx");
  if (len) *len = ctx->hdr.size();
  if (!out) return MJG_OK;
  if (cap < ctx->hdr.size()) return set_err(MJG_E_CAPACITY, "header needs %zu bytes", ctx->hdr.size());
  memcpy(out, ctx->hdr.data(), ctx->hdr.size());
  return MJG_OK;
}

namespace {
// mjg_submit's body; segs (mjg_submit_segments: device frames, no -vf scale) replaces the one
// segment at `frames` as k_encode's input
int submit_impl(mjg_ctx *c, const uint8_t *frames, int n, int src_is_device, const SegList *segs) {
  if (n < 1 || (size_t)n > c->slot_B || (!src_is_device && n > c->cfg.max_batch))
    return set_err(MJG_E_INVALID, "nframes %d not in 1..%d", n, c->cfg.max_batch);
  if (c->nout == kSlots) return set_err(MJG_E_STATE, "%d submits queued: sync one first", kSlots);
  HIP_TRY(hipSetDevice(c->device));
  const EncGeom &g = c->geom;
  Slot &S = c->slot[c->head];
  if (!S.alloc) {  // slots 1.., on the first pipelined submits
    const int rc = alloc_slot(c, S);
    if (rc) return rc;
  }
  const uint8_t *src = frames;
  if (!src_is_device) {
    if (!S.d_stage) {  // staging for host submits, allocated on first use
      const int rc = dmalloc(&S.d_stage, (size_t)c->cfg.max_batch * c->in_frame_bytes);
      if (rc) return rc;
    }
    HIP_TRY(hipMemcpyAsync(S.d_stage, frames, (size_t)n * c->in_frame_bytes, hipMemcpyHostToDevice, S.st));
    src = S.d_stage;
  }
  SegList in_sl;  // the submit's input frames: the caller's segments, or one at src
  if (segs) {
    in_sl = *segs;
  } else {
    for (int k = 0; k < kMaxSegs; k++) {
      in_sl.p[k] = src;
      in_sl.f0[k] = k ? INT_MAX : 0;
    }
  }
  SegList enc_in = in_sl;
  if (c->scale) {
    tmark(c, S, MJG_K_SCALE, 0);
    const ScaleGeom &lg = c->ps[0].g, &cg = c->ps[1].g;
    // luma, then U and V in one launch (same filters; blockIdx.z >= n is V) while 2n fits the
    // grid's z range, else one launch each
    const bool uv1 = 2 * n <= 65535;
    for (int p = 0; p < (uv1 ? 2 : 3); p++) {
      PlaneScale &ps = c->ps[p ? 1 : 0];
      ScaleGeom sg = p ? cg : lg;
      sg.nf = n;
      sg.s_off = sg.d_off = sg.s_poff = sg.d_poff = 0;
      if (p) {
        sg.s_off = (long long)c->cfg.src_w * c->cfg.src_h + (p - 1) * (long long)cg.sw * cg.sh;
        sg.d_off = g.u_off + (p - 1) * (long long)g.cw * g.ch;
        if (uv1) {
          sg.s_poff = (long long)cg.sw * cg.sh;
          sg.d_poff = (long long)g.cw * g.ch;
        }
      }
      // one dimension: tiles x planes x frames (scale.hip decodes it by multiply-high)
      const int nz = p && uv1 ? 2 * n : n;
      sg.gx = (int)ps.grid.x;
      sg.gxy = (int)(ps.grid.x * ps.grid.y);
      auto magic = [](uint32_t d) { return d > 1 ? (uint32_t)((((uint64_t)1 << 32) + d - 1) / d) : 0u; };
      sg.gx_magic = magic((uint32_t)sg.gx);
      sg.gxy_magic = magic((uint32_t)sg.gxy);
      const dim3 grid((unsigned)(sg.gxy * nz), 1, 1);
#define MJG_SCALE_LAUNCH3(HT, NPV, D4, TH)                                                          \
  do {                                                                                              \
    if (sg.range == 1)                                                                              \
      k_scale<HT, NPV, D4, 1, TH><<<grid, 64 * scale_waves(TH), ps.lds, S.st>>>(in_sl, S.d_scaled, sg, ps.hcp,        \
                                                                    ps.hp, ps.vcp, ps.vps, ps.hsum, ps.mfb); \
    else if (sg.range == 2)                                                                         \
      k_scale<HT, NPV, D4, 2, TH><<<grid, 64 * scale_waves(TH), ps.lds, S.st>>>(in_sl, S.d_scaled, sg, ps.hcp,        \
                                                                    ps.hp, ps.vcp, ps.vps, ps.hsum, ps.mfb); \
    else                                                                                            \
      k_scale<HT, NPV, D4, 0, TH><<<grid, 64 * scale_waves(TH), ps.lds, S.st>>>(in_sl, S.d_scaled, sg, ps.hcp,        \
                                                                    ps.hp, ps.vcp, ps.vps, ps.hsum, ps.mfb); \
  } while (0)
#define MJG_SCALE_LAUNCH(HT, NPV, TH)      \
  do {                                     \
    if (ps.d4)                             \
      MJG_SCALE_LAUNCH3(HT, NPV, true, TH);  \
    else                                   \
      MJG_SCALE_LAUNCH3(HT, NPV, false, TH); \
  } while (0)
      if (sg.htaps == 8 && sg.npv == 5 && ps.th == 128)  // 2:1 downscale (4K -> 1080p), tall tiles
        MJG_SCALE_LAUNCH(8, 5, 128);
      else if (sg.htaps == 8 && sg.npv == 5 && ps.th == 64)
        MJG_SCALE_LAUNCH(8, 5, 64);
      else if (sg.htaps == 8 && sg.npv == 5)
        MJG_SCALE_LAUNCH(8, 5, 32);
      else if (sg.htaps == 4 && sg.npv == 3)  // upscale / mild downscale
        MJG_SCALE_LAUNCH(4, 3, 32);
      else
        MJG_SCALE_LAUNCH(0, 0, 32);
#undef MJG_SCALE_LAUNCH
#undef MJG_SCALE_LAUNCH3
    }
    tmark(c, S, MJG_K_SCALE, 1);
    HIP_TRY(hipGetLastError());
    for (int k = 0; k < kMaxSegs; k++) {  // k_encode reads the scaled frames, one buffer
      enc_in.p[k] = S.d_scaled;
      enc_in.f0[k] = k ? INT_MAX : 0;
    }
  }
  const int ntasks = g.nchunks * g.nseg * n;
  const int nsegs = g.nseg * n;  // entropy-coded segments of this submit
  const int wgs = std::min((ntasks + kWavesPerWg - 1) / kWavesPerWg, c->enc_grid);
  if (c->optimal) {  // pass 1: symbol counts per frame, then the frame's tables
    tmark(c, S, MJG_K_HUFF, 0);
    HIP_TRY(hipMemsetAsync(S.d_hist, 0, (size_t)n * kFrameTabWords * 4, S.st));
    launch_encode<kCount>(c, S, enc_in, std::min(wgs, c->enc_grid_cnt), ntasks);
    HIP_TRY(hipMemsetAsync(S.d_work, 0, (size_t)kXcds * kCtrStride * 4, S.st));  // unit counters for pass 2
    k_huff_build<<<n * 4, 64, 0, S.st>>>(S.d_hist, S.d_ftabs, S.d_dht, S.d_dht_nval);
    tmark(c, S, MJG_K_HUFF, 1);
    HIP_TRY(hipGetLastError());
  }
  tmark(c, S, MJG_K_ENCODE, 0);
  if (c->optimal)
    k_emit_syms<<<c->enc_grid * kEmitGridMul, 64 * kWavesPerWg, 0, S.st>>>(g, c->d_tabs, S.d_ftabs, S.d_syms, S.d_symn,
                                                             S.d_scratch, S.d_chunk_bits, S.d_stage_bits,
                                                                  ntasks);
  else
    launch_encode<kEmitDefault>(c, S, enc_in, wgs, ntasks);
  tmark(c, S, MJG_K_ENCODE, 1);
  HIP_TRY(hipGetLastError());
  HIP_TRY(hipEventRecord(S.enc_done, S.st));
  HIP_TRY(hipStreamWaitEvent(c->tail, S.enc_done, 0));
  if (c->timing_tail) (void)hipEventRecord(S.ev[MJG_K_TAIL][0], c->tail);
  tmark(c, S, MJG_K_SCAN_BITS, 0);
  const int ndone = 1;  // k_scan_ff's frame ticket
  if (c->rst)
    k_scan_bits_seg<<<(nsegs + 3) / 4, 256, 0, c->tail>>>(S.d_chunk_bits, S.d_chunk_off, S.d_frame_bits,
                                                            g.nchunks, nsegs, S.d_work, S.d_status, S.d_done,
                                                            ndone);
  else
    k_scan_bits<<<n, 1024, 0, c->tail>>>(S.d_chunk_bits, S.d_chunk_off, S.d_frame_bits, g.nchunks,
                                           S.d_work, S.d_status, S.d_done, ndone);
  tmark(c, S, MJG_K_SCAN_BITS, 1);
  HIP_TRY(hipGetLastError());
  tmark(c, S, MJG_K_COUNT_FF, 0);
  const int gps = (g.nchunks + kChunksPerWave - 1) / kChunksPerWave;
  k_count_ff<<<(gps * nsegs + 3) / 4, 256, 0, c->tail>>>(S.d_scratch, S.d_chunk_bits, S.d_chunk_off,
                                                           S.d_frame_bits, S.d_group_ff, g.nchunks, gps,
                                                           gps * nsegs, S.d_stream);
  tmark(c, S, MJG_K_COUNT_FF, 1);
  HIP_TRY(hipGetLastError());
  // segment and frame sizes, the frames' packed offsets
  tmark(c, S, MJG_K_SCAN_FF, 0);
  k_scan_ff<<<n, 256, 0, c->tail>>>(S.d_group_ff, S.d_ff_off, S.d_frame_bits, g.nchunks, gps, g.nseg, (int)c->hdr.size(),
                                      c->optimal ? S.d_dht_nval : nullptr, S.d_hdr_lens, S.d_seg_size,
                                      S.d_seg_off, S.d_frame_size, S.d_frame_offsets, S.d_done);
  tmark(c, S, MJG_K_SCAN_FF, 1);
  HIP_TRY(hipGetLastError());
  int rc = launch_write(c, S, n, false);
  if (rc) return rc;
  S.n = n;
  S.pending = true;
  S.njobs = 1;  // the caller records a merged launch's jobs
  S.nsynced = 0;
  S.jf0[0] = 0;
  S.jn[0] = n;
  c->head = (c->head + 1) % kSlots;
  c->nout++;
  c->launches++;
  c->synced_since_submit = false;
  return MJG_OK;
}

// Jobs submitted and not yet synced: those of the queued launches plus the held ones.
int pending_jobs(const mjg_ctx *c) {
  int p = c->held;
  for (int i = 0; i < c->nout; i++) {
    const Slot &S = c->slot[(c->head + kSlots - c->nout + i) % kSlots];
    p += S.njobs - S.nsynced;
  }
  return p;
}

// One launch for the held device jobs: their frames as a segment list (one job: the plain
// single-segment launch), each job's frames recorded for mjg_sync.
int launch_held(mjg_ctx *c) {
  SegList sl;
  int n = 0;
  for (int k = 0; k < kMaxSegs; k++) {
    sl.p[k] = c->held_p[k < c->held ? k : 0];
    sl.f0[k] = k < c->held ? n : INT_MAX;
    if (k < c->held) n += c->held_n[k];
  }
  Slot &S = c->slot[c->head];
  const int rc = submit_impl(c, c->held_p[0], n, 1, c->held > 1 ? &sl : nullptr);
  if (rc) return rc;  // the jobs stay held
  S.njobs = c->held;
  for (int k = 0, f = 0; k < c->held; f += c->held_n[k], k++) {
    S.jf0[k] = f;
    S.jn[k] = c->held_n[k];
  }
  c->held = 0;
  return MJG_OK;
}

// Launch the held jobs when a launch slot is free and they are `merge` jobs (with hold_idle off,
// also when the GPU has nothing else queued); a lone held job launches at its own mjg_sync (or
// before a host submit).  Holding even on an idle GPU keeps every launch of a stream of device
// submits a full pair: A/B with prewarmed clocks (profiles/r05/merge_prewarm_ab.txt) c5 +6%, c1 +3.5%,
// c4 +1.5%, c2 +0-1% against no merging; launching a lone job on an idle GPU made the first
// launch a single and lost that gain on c2.  At mjg_sync the slot of the job just synced stays
// untouched: its results are read (mjg_fetch, mjg_output_device) until the caller's next submit.
int try_launch_held(mjg_ctx *c, bool at_sync) {
  if (!c->held || c->nout == kSlots) return MJG_OK;
  if (c->held < c->merge && (c->nout > 0 || c->hold_idle)) return MJG_OK;
  if (at_sync && c->head == c->last) return MJG_OK;
  return launch_held(c);
}
}  // namespace

int mjg_submit(mjg_ctx *c, const uint8_t *frames, int n, int src_is_device) {
  if (!c || !frames) return set_err(MJG_E_INVALID, "null argument");
  if (n < 1 || n > c->cfg.max_batch)
    return set_err(MJG_E_INVALID, "nframes %d not in 1..%d", n, c->cfg.max_batch);
  if (src_is_device && c->merge > 1) {  // held, and launched with the next one(s)
    // a full held group whose launch waited at mjg_sync (its slot was the one just synced, whose
    // results stay readable until this call): launched now, before the new job is held
    if (c->held == c->merge && c->nout < kSlots) {
      const int rc = launch_held(c);
      if (rc) return rc;
    }
    if (pending_jobs(c) >= kSlots * c->merge || c->held == c->merge)
      return set_err(MJG_E_STATE, "%d submits queued: sync one first", pending_jobs(c));
    c->held_p[c->held] = frames;
    c->held_n[c->held] = n;
    c->held++;
    c->synced_since_submit = false;
    const int rc = try_launch_held(c, false);
    if (rc) c->held--;
    return rc;
  }
  // host frames (H2D through the slot's staging) or merging off: a launch of its own, after
  // a launch of the jobs held before it
  if (c->nout + (c->held ? 1 : 0) >= kSlots)
    return set_err(MJG_E_STATE, "%d launches queued: sync one first", kSlots);
  if (c->held) {
    const int rc = launch_held(c);
    if (rc) return rc;
  }
  return submit_impl(c, frames, n, src_is_device, nullptr);
}

int mjg_max_segments(void) { return kMaxSegs; }

int mjg_submit_segments(mjg_ctx *c, const uint8_t *const *seg_frames, const int *seg_nframes, int nsegs) {
  if (!c || !seg_frames || !seg_nframes) return set_err(MJG_E_INVALID, "null argument");
  if (nsegs < 1 || nsegs > kMaxSegs) return set_err(MJG_E_INVALID, "nsegs %d not in 1..%d", nsegs, kMaxSegs);
  SegList sl;
  int n = 0;
  for (int k = 0; k < kMaxSegs; k++) {
    if (k < nsegs) {
      if (!seg_frames[k] || seg_nframes[k] < 1 || seg_nframes[k] > c->cfg.max_batch)
        return set_err(MJG_E_INVALID, "segment %d: null frames or nframes not in 1..%d", k, c->cfg.max_batch);
      sl.p[k] = seg_frames[k];
      sl.f0[k] = n;
      n += seg_nframes[k];
    } else {
      sl.p[k] = seg_frames[0];
      sl.f0[k] = INT_MAX;
    }
  }
  if (n > c->cfg.max_batch) return set_err(MJG_E_INVALID, "%d frames in the segments, max_batch %d", n, c->cfg.max_batch);
  if (c->nout + (c->held ? 1 : 0) >= kSlots)
    return set_err(MJG_E_STATE, "%d launches queued: sync one first", kSlots);
  if (c->held) {
    const int rc = launch_held(c);
    if (rc) return rc;
  }
  return submit_impl(c, seg_frames[0], n, 1, &sl);
}

int mjg_ctx_queue_depth(const mjg_ctx *c) { return c ? kSlots * c->merge : 0; }

// Completes the oldest queued job (or, with none queued, reports the last synced one).  The
// first job of a launch waits for it (and regrows its output on overflow); the others of the
// same launch are then ready.
int mjg_sync(mjg_ctx *c, uint64_t *frame_sizes, uint64_t *total) {
  if (!c) return set_err(MJG_E_INVALID, "null ctx");
  if (c->nout == 0 && c->held == 0 && c->last < 0) return set_err(MJG_E_STATE, "nothing submitted");
  HIP_TRY(hipSetDevice(c->device));
  if (c->nout == 0 && c->held) {  // the oldest job is held: launch it now
    const int rc = launch_held(c);
    if (rc) return rc;
  }
  if (c->nout > 0) {
    const int si = (c->head + kSlots - c->nout) % kSlots;  // oldest queued launch
    Slot &S = c->slot[si];
    if (S.nsynced == 0) {
      HIP_TRY(hipEventSynchronize(S.done));
      const int n = S.n;
      uint64_t t = 0;
      for (int i = 0; i < n; i++) t += S.h_sizes[i];
      if (*S.h_status & 1u) {  // packed output overflowed: grow, re-run the write pass only
        HIP_TRY(hipFree(S.d_out));
        S.d_out = nullptr;
        S.out_cap = t + t / 4 + 4096;
        int rc = dmalloc(&S.d_out, S.out_cap);
        if (rc) return rc;
        if ((rc = launch_write(c, S, n, true))) return rc;
        HIP_TRY(hipEventSynchronize(S.done));
        if (*S.h_status & 1u) return set_err(MJG_E_HIP, "output overflow persisted");
      }
      if (c->timing) {
        for (int k = 0; k < MJG_NUM_KERNELS; k++) {
          if (k == MJG_K_SCALE && !c->scale) continue;
          if (k == MJG_K_HUFF && !c->optimal) continue;
          const bool tail = k == MJG_K_SCAN_BITS || k == MJG_K_COUNT_FF || k == MJG_K_SCAN_FF || k == MJG_K_WRITE;
          if (tail != c->timing_detail && (tail || k == MJG_K_TAIL)) continue;
          if (k == MJG_K_TAIL && !c->timing_tail) continue;
          float ms = 0.f;
          if (hipEventElapsedTime(&ms, S.ev[k][0], S.ev[k][1]) == hipSuccess) c->t_acc[k] += ms;
        }
        c->t_n++;
      }
    }
    const int j = S.nsynced;
    uint64_t off = 0, t = 0;
    for (int i = 0; i < S.jf0[j]; i++) off += S.h_sizes[i];
    for (int i = S.jf0[j]; i < S.jf0[j] + S.jn[j]; i++) t += S.h_sizes[i];
    if (++S.nsynced == S.njobs) {
      S.pending = false;
      c->nout--;
    }
    c->last = si;
    c->last_job = j;
    c->last_off = off;
    c->last_total = t;
    (void)try_launch_held(c, true);  // a failed launch leaves the jobs held: their own sync reports it
  }
  c->synced_since_submit = true;
  const Slot &L = c->slot[c->last];
  if (frame_sizes) memcpy(frame_sizes, L.h_sizes + L.jf0[c->last_job], L.jn[c->last_job] * sizeof(uint64_t));
  if (total) *total = c->last_total;
  return MJG_OK;
}

// The packed JPEGs of the last synced submit, copied D2H into the context's page-locked
// buffer (grown as needed); with no mjg_sync since the last mjg_submit it syncs the oldest
// queued submit first (the submit -> fetch pattern).  A DMA into page-locked memory: a copy
// into pageable memory goes through the runtime's staging and page pinning, which measured
// 0.1 s per 1080p segment in some worker processes and 2 ms in others.
int mjg_fetch_host(mjg_ctx *c, const uint8_t **data, size_t *len) {
  if (!c || !data) return set_err(MJG_E_INVALID, "null argument");
  if (pending_jobs(c) > 0 && !c->synced_since_submit) {
    const int rc = mjg_sync(c, nullptr, nullptr);
    if (rc) return rc;
  }
  if (c->last < 0) return set_err(MJG_E_STATE, "nothing submitted");
  const Slot &L = c->slot[c->last];
  const uint64_t total = c->last_total;
  HIP_TRY(hipSetDevice(c->device));
  if (total > c->h_fetch_cap) {
    if (c->h_fetch) HIP_TRY(hipHostFree(c->h_fetch));
    c->h_fetch = nullptr;
    c->h_fetch_cap = 0;
    const size_t cap = total + total / 4 + 4096;
    if (hipHostMalloc((void **)&c->h_fetch, cap, hipHostMallocDefault) != hipSuccess) {
      c->h_fetch = nullptr;
      (void)hipGetLastError();
      return set_err(MJG_E_NOMEM, "hipHostMalloc(%zu) failed", cap);
    }
    c->h_fetch_cap = cap;
  }
  if (total) HIP_TRY(hipMemcpy(c->h_fetch, L.d_out + c->last_off, total, hipMemcpyDeviceToHost));
  *data = c->h_fetch;
  if (len) *len = total;
  return MJG_OK;
}

// The last synced job's packed JPEGs into the caller's memory: one DMA when it is page-locked
// (mjg_host_alloc), else mjg_fetch_host and a copy.
int mjg_fetch(mjg_ctx *c, uint8_t *out, size_t cap) {
  if (!c || !out) return set_err(MJG_E_INVALID, "null argument");
  if (pending_jobs(c) > 0 && !c->synced_since_submit) {
    const int rc = mjg_sync(c, nullptr, nullptr);
    if (rc) return rc;
  }
  if (c->last < 0) return set_err(MJG_E_STATE, "nothing submitted");
  if (cap < c->last_total) return set_err(MJG_E_CAPACITY, "fetch needs %llu bytes", (unsigned long long)c->last_total);
  HIP_TRY(hipSetDevice(c->device));
  // page-locked caller memory (mjg_host_alloc): one DMA straight into it, no staging copy
  hipPointerAttribute_t at{};
  if (hipPointerGetAttributes(&at, out) == hipSuccess && at.type == hipMemoryTypeHost) {
    if (c->last_total)
      HIP_TRY(hipMemcpy(out, c->slot[c->last].d_out + c->last_off, c->last_total, hipMemcpyDeviceToHost));
    return MJG_OK;
  }
  (void)hipGetLastError();  // pageable memory: not a HIP pointer
  const uint8_t *p = nullptr;
  size_t n = 0;
  const int rc = mjg_fetch_host(c, &p, &n);
  if (rc) return rc;
  if (n) memcpy(out, p, n);
  return MJG_OK;
}

// The launch's packed output and the job's frame offsets into it (data + offsets[i] is the
// job's frame i; with merged launches offsets[0] is the job's place in the launch's output).
int mjg_output_device(mjg_ctx *c, const uint8_t **data, const uint64_t **offsets) {
  if (!c) return set_err(MJG_E_INVALID, "null ctx");
  const Slot &L = c->slot[c->last < 0 ? 0 : c->last];
  if (data) *data = L.d_out;
  if (offsets) *offsets = L.d_frame_offsets + (c->last < 0 ? 0 : L.jf0[c->last_job]);
  return MJG_OK;
}

void *mjg_stream(mjg_ctx *c) {
  if (!c) return nullptr;
  return (void *)slot_stream(c, c->head);
}

int mjg_queue_depth(void) { return kSlots; }

int mjg_host_alloc(size_t bytes, void **ptr) {
  if (!ptr) return set_err(MJG_E_INVALID, "null argument");
  if (hipHostMalloc(ptr, bytes, hipHostMallocDefault) != hipSuccess) {
    *ptr = nullptr;
    (void)hipGetLastError();
    return set_err(MJG_E_NOMEM, "hipHostMalloc(%zu) failed", bytes);
  }
  return MJG_OK;
}

int mjg_host_free(void *ptr) {
  if (ptr) HIP_TRY(hipHostFree(ptr));
  return MJG_OK;
}

int mjg_kernel_times(mjg_ctx *c, double *ms, int *launches, int reset) {
  if (!c) return set_err(MJG_E_INVALID, "null ctx");
  if (!c->timing) return set_err(MJG_E_STATE, "context opened without MJG_F_TIMING");
  for (int k = 0; k < MJG_NUM_KERNELS; k++)
    if (ms) ms[k] = c->t_n ? c->t_acc[k] / c->t_n : 0.0;
  if (launches) *launches = c->t_n;
  if (reset) {
    for (double &t : c->t_acc) t = 0;
    c->t_n = 0;
  }
  return MJG_OK;
}

int mjg_build_header(const mjg_config *cfg, uint8_t *out, size_t cap, size_t *len) {
  if (!cfg) return set_err(MJG_E_INVALID, "null cfg");
  if (cfg->dst_w < 1 || cfg->dst_h < 1 || cfg->dst_w > 65535 || cfg->dst_h > 65535 ||
      cfg->qscale < 1 || cfg->qscale > 31 || cfg->chroma_format < MJG_CHROMA_420 ||
      cfg->chroma_format > MJG_CHROMA_444)
    return set_err(MJG_E_INVALID, "bad size / qscale / chroma_format");
  if (cfg->sar_num < 0 || cfg->sar_den < 0 || cfg->sar_num > 65535 || cfg->sar_den > 65535)
    return set_err(MJG_E_INVALID, "bad SAR %d:%d", cfg->sar_num, cfg->sar_den);
  uint8_t mp[64];
  for (int i = 0; i < 64; i++) {
    const int v = i == 0 ? 8 : ((kMpeg1Intra[i] * cfg->qscale) >> 3);
    mp[i] = (uint8_t)(v > 255 ? 255 : v);
  }
  const bool rst = (cfg->flags & MJG_F_RST) && (cfg->dst_h + 15) / 16 > 1;
  const std::vector<uint8_t> h = build_header(cfg->dst_w, cfg->dst_h, mp, cfg->sar_num, cfg->sar_den,
                                             (cfg->flags & MJG_F_COM_ITU601) != 0, cfg->chroma_format, rst);
  if (len) *len = h.size();
  if (!out) return MJG_OK;
  if (cap < h.size()) return set_err(MJG_E_CAPACITY, "header needs %zu bytes", h.size());
  memcpy(out, h.data(), h.size());
  return MJG_OK;
}

int mjg_sws_filter(int src_len, int dst_len, int one, int align, int bitexact, int src_pos,
                   int dst_pos, int16_t *coeff, size_t coeff_cap, int32_t *pos_out, int *taps) {
  SwsFilter f;
  if (!make_sws_filter(src_len, dst_len, one, align, bitexact != 0, src_pos, dst_pos, &f))
    return set_err(MJG_E_INVALID, "unsupported filter %d -> %d", src_len, dst_len);
  if (taps) *taps = f.taps;
  if (!coeff) return MJG_OK;
  if (coeff_cap < f.coeff.size()) return set_err(MJG_E_CAPACITY, "need %zu taps", f.coeff.size());
  memcpy(coeff, f.coeff.data(), f.coeff.size() * sizeof(int16_t));
  if (pos_out) memcpy(pos_out, f.pos.data(), f.pos.size() * sizeof(int32_t));
  return MJG_OK;
}

int mjg_debug_coefs(mjg_ctx *c, int frame, int16_t *out, size_t nblocks) {
  if (!c || !out) return set_err(MJG_E_INVALID, "null argument");
  if (!c->geom.debug_coefs) return set_err(MJG_E_STATE, "context opened without MJG_F_DEBUG_COEFS");
  if (pending_jobs(c) > 0 && !c->synced_since_submit) {
    const int rc = mjg_sync(c, nullptr, nullptr);
    if (rc) return rc;
  }
  if (c->last < 0) return set_err(MJG_E_STATE, "nothing submitted");
  const Slot &L = c->slot[c->last];
  const size_t nb = (size_t)c->geom.nmcu * c->geom.bpm;  // dbg buffer: frame-major, coding order
  if (frame < 0 || frame >= L.jn[c->last_job]) return set_err(MJG_E_INVALID, "frame %d", frame);
  if (nblocks < nb) return set_err(MJG_E_CAPACITY, "need %zu blocks", nb);
  // the kernel stores each quantised block in natural (raster) order
  const size_t f = (size_t)L.jf0[c->last_job] + (size_t)frame;
  HIP_TRY(hipMemcpy(out, L.d_dbg + f * nb * 64, nb * 64 * sizeof(int16_t), hipMemcpyDeviceToHost));
  return MJG_OK;
}

int mjg_debug_planes(mjg_ctx *c, int frame, uint8_t *out, size_t cap) {
  if (!c || !out) return set_err(MJG_E_INVALID, "null argument");
  if (!c->scale) return set_err(MJG_E_STATE, "context does not scale");
  if (pending_jobs(c) > 0) {  // the latest synced submit's planes
    const int rc = mjg_sync(c, nullptr, nullptr);
    if (rc) return rc;
  }
  if (pending_jobs(c) > 0 || c->last < 0) return set_err(MJG_E_STATE, "sync every queued submit first");
  const Slot &L = c->slot[c->last];
  if (frame < 0 || frame >= L.jn[c->last_job]) return set_err(MJG_E_INVALID, "frame %d", frame);
  if (cap < c->enc_frame_bytes) return set_err(MJG_E_CAPACITY, "need %zu bytes", c->enc_frame_bytes);
  const size_t f = (size_t)L.jf0[c->last_job] + (size_t)frame;
  HIP_TRY(hipMemcpy(out, L.d_scaled + f * c->enc_frame_bytes, c->enc_frame_bytes, hipMemcpyDeviceToHost));
  return MJG_OK;
}

int mjg_debug_huff_build(int device, const uint32_t *hist, int nframes, uint8_t *dht, uint32_t *nval) {
  if (!hist || !dht || !nval || nframes < 1 || nframes > 4096) return set_err(MJG_E_INVALID, "bad arguments");
  HIP_TRY(hipSetDevice(device));
  const size_t nh = (size_t)nframes * kFrameTabWords, nd = (size_t)nframes * 4 * kDhtSlot, nv = (size_t)nframes * 4;
  uint32_t *d_hist = nullptr, *d_ftabs = nullptr, *d_nval = nullptr;
  uint8_t *d_dht = nullptr;
  int rc = MJG_OK;
  if (hipMalloc((void **)&d_hist, nh * 4) != hipSuccess || hipMalloc((void **)&d_ftabs, nh * 4) != hipSuccess ||
      hipMalloc((void **)&d_dht, nd) != hipSuccess || hipMalloc((void **)&d_nval, nv * 4) != hipSuccess) {
    (void)hipGetLastError();
    rc = set_err(MJG_E_NOMEM, "hipMalloc failed");
  }
  if (rc == MJG_OK && (hipMemcpy(d_hist, hist, nh * 4, hipMemcpyHostToDevice) != hipSuccess ||
                       hipMemset(d_dht, 0, nd) != hipSuccess)) rc = set_err(MJG_E_HIP, "copy in failed");
  if (rc == MJG_OK) {
    k_huff_build<<<nframes * 4, 64>>>(d_hist, d_ftabs, d_dht, d_nval);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
        hipMemcpy(dht, d_dht, nd, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(nval, d_nval, nv * 4, hipMemcpyDeviceToHost) != hipSuccess)
      rc = set_err(MJG_E_HIP, "k_huff_build failed");
  }
  (void)hipFree(d_hist);
  (void)hipFree(d_ftabs);
  (void)hipFree(d_dht);
  (void)hipFree(d_nval);
  return rc;
}

int mjg_debug_filter(mjg_ctx *c, int plane, int dir, int16_t *coeff, int32_t *pos, int *taps,
                     int *len) {
  if (!c) return set_err(MJG_E_INVALID, "null ctx");
  if (!c->scale) return set_err(MJG_E_STATE, "context does not scale");
  if (plane < 0 || plane > 1 || dir < 0 || dir > 1) return set_err(MJG_E_INVALID, "plane/dir");
  const SwsFilter &f = dir ? c->ps[plane].vf : c->ps[plane].hf;
  if (taps) *taps = f.taps;
  if (len) *len = f.dst_len;
  if (coeff) memcpy(coeff, f.coeff.data(), f.coeff.size() * sizeof(int16_t));
  if (pos) memcpy(pos, f.pos.data(), f.pos.size() * sizeof(int32_t));
  return MJG_OK;
}

}  // extern "C"

