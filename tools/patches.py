#!/usr/bin/env python3
"""Source patches of the encoder's measured-and-not-kept experiments, applied to a copy of
ffmpeg_distributed_amd/csrc for tools/variants.py A/Bs.  The product kernels carry no
experiment switches (no `#if` but include guards); each former MJG_EXP_* / MJG_TAIL_* /
MJG_SLOT_WORDS branch lives here as exact text replacements, so an old A/B can be re-run
with `VARIANTS="base=:;x=@no_skip"` (several: `@no_sb_row+no_sb_col`, parameters:
`@wide_cost=3`).

A patch is a list of (file, old, new); `old` must occur exactly once (the patch fails loudly
when the product source has moved on)."""
from __future__ import annotations

import os
import shutil

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "ffmpeg_distributed_amd", "csrc")
K = "kernels.hip"


# name -> function(param or None) -> [(file, old, new)]
PATCHES = {
    # the stuffing tail on the submit stream: no co-run with the next submit's k_encode
    # (profiles/r03_ab_serial_tail.txt)
    "serial_tail": lambda a: [("api.hip", "  HIP_TRY(hipStreamCreateWithPriority(&c->tail, hipStreamNonBlocking, greatest));\n",
                               "  c->tail = c->stream;\n")],
    # no column skip test in the VALU column screen (profiles/r03_ab_column_skip.txt)
    "no_skip": lambda a: [(K, "    if (jp > 0 && (((st >> jp) & 1u) || retest)) {\n", "    if (false) {\n")],
    # the column skip test on every chunk (round 3's form, before the adaptive test)
    "always_test": lambda a: [(K, "    if (jp > 0 && (((st >> jp) & 1u) || retest)) {\n", "    if (jp > 0) {\n")],
    # wave-parallel block cost factor (profiles/r03_ab_wide_cost.txt)
    "wide_cost": lambda a: [(K, "const int cost = 4 * __popcll(hv[k])", f"const int cost = {int(a)} * __popcll(hv[k])")],
    # chunks per k_encode work unit, VALU stage (profiles/r03_ab_sched_units.txt)
    "batch": lambda a: [(K, "constexpr int kBatchOf = MF ? 8 : 12;", f"constexpr int kBatchOf = MF ? 8 : {int(a)};")],
    # k_encode scheduling barriers (profiles/r03_ab_sched_units.txt)
    "no_sb_row": lambda a: [(K, "0x05040100u);\n    __builtin_amdgcn_sched_barrier(0);\n", "0x05040100u);\n")],
    "no_sb_pair": lambda a: [(K, "    __builtin_amdgcn_sched_barrier(0);  // one column pair in flight at a time\n", "")],
    "no_sb_col": lambda a: [(K, "      __builtin_amdgcn_sched_barrier(0);  // one column at a time\n", "")],
    # stuffing tail group size / rounds
    "tail_g": lambda a: [(K, "constexpr int kChunksPerWave = 32;", f"constexpr int kChunksPerWave = {int(a)};")],
    "tail_r": lambda a: [(K, "constexpr int kTailRounds = 4;", f"constexpr int kTailRounds = {int(a)};")],
    # slot stride (words per chunk).  UNSAFE below the worst case 3328: layout timing only
    "slot_words": lambda a: [(K, "constexpr int kSlotWords = (64 * kMaxBlockBits + 31) / 32;",
                              f"constexpr int kSlotWords = {int(a)};")],
    # k_count_ff without its realigned-stream stores (timing probe: k_write then reads garbage)
    "count_nostream": lambda a: [(K, "        cnt += ff_bytes(v[i]);\n        *(uint32_t *)(sw + 4u * k) = v[i];\n",
                                  "        cnt += ff_bytes(v[i]);\n")],
    # k_write without its clean-word stores (timing probe: wrong output)
    "write_nostore": lambda a: [(K, "      if (valid && ff == 0 && !last) {\n        *(u32_any *)p = __builtin_bswap32(w);\n      }",
                                 "      if (w == 0x12345678u && k == 7u) *(u32_any *)p = 0u;  // keeps the loads alive\n"
                                 "      else if (valid && ff == 0 && !last) {\n      }")],
    # branch-free slot loads in k_count_ff (measured slower)
    "branchfree": lambda a: [(K, """    // 32-bit offsets from the group's first slot (the wave-uniform base: saddr loads)
    const uint8_t *s0 = (const uint8_t *)g.slot0;  // byte offsets < 2^32: one 32-bit VGPR each
    const uint32_t oa = (__umul24((uint32_t)c, (uint32_t)kSlotWords) + wi) << 2;
    A[i] = *(const uint32_t *)(s0 + oa);
    X[i] = (bnd[i] && off && rem > 32u - off) ? *(const uint32_t *)(s0 + oa + 4u) : 0u;
    const bool has_next = (inf[i] >> 27) & 1u;
    B[i] = (own_nx[i] && (!bnd[i] || (rem < 32u && has_next)))
               ? *(const uint32_t *)(s0 + (bnd[i] ? __umul24((uint32_t)c + 1u, (uint32_t)kSlotWords * 4u) : oa + 4u))
               : 0u;
""", """    // 32-bit byte offsets from the group's first slot; X / B load A's word when not needed
    const uint8_t *s0 = (const uint8_t *)g.slot0;
    const uint32_t oa = __umul24((uint32_t)c, kSlotWords * 4u) + (wi << 2);
    const bool nX = bnd[i] && off && rem > 32u - off;
    const bool has_next = (inf[i] >> 27) & 1u;
    const bool nB = own_nx[i] && (!bnd[i] || (rem < 32u && has_next));
    const uint32_t ob = bnd[i] ? __umul24((uint32_t)c + 1u, kSlotWords * 4u) : oa + 4u;
    A[i] = *(const uint32_t *)(s0 + oa);
    X[i] = *(const uint32_t *)(s0 + (nX ? oa + 4u : oa));
    B[i] = *(const uint32_t *)(s0 + (nB ? ob : oa));
    X[i] = nX ? X[i] : 0u;
    B[i] = nB ? B[i] : 0u;
""")],
    # -huffman optimal counting pass without its LDS histogram atomics / without its symbol
    # record stores (timing probes: wrong tables / wrong replay; c1: 0.753 -> 0.658 / 0.817 ms,
    # profiles/r05/c1_count_ablation.txt).  Counting the DC and EOB symbols per distinct value
    # after the block (a ballot loop) instead of per lane measured slower: 0.791 vs 0.760 ms.
    "cnt_noatomic": lambda a: [(K, "    atomicAdd(&hdc[cat], 1u);\n", ""), (K, "    atomicAdd(&hac[sym], 1u);\n", "")],
    "cnt_norec": lambda a: [(K, "    rec[n * 64] = (1u << 31) | ((uint32_t)cat << 16) | mant;\n", ""),
                            (K, "    rec[n * 64] = ((uint32_t)sym << 16) | mant;\n", "")],
    # occupancy probe: k_encode's workgroup LDS past 40 KB (3 workgroups, 3 waves per SIMD)
    "occ3": lambda a: [(K, "][kHvWords];\n", "][kHvWords + 512];\n")],
}

# ---------------------------------------------------------------- probes (wrong timing, right bytes)
# phase_clock: k_encode<.., kEmitDefault> lane 0 reads the shader clock (s_memtime) at the phase
# boundaries of every chunk and adds the deltas into mjg_phase_acc[8] (one atomic per phase per
# wave at its end); mjg_probe_phase() returns and clears them (tools/phase_probe.py).  The clock
# reads wait for the wave's outstanding LDS / scalar operations (lgkmcnt), so each phase also
# absorbs the LDS latency still open at its end.
_PH_DECL = "constexpr int kWavesPerWg = 4;\n"
_PH_DEVICE = (_PH_DECL + "__device__ unsigned long long mjg_phase_acc[8];\n"
              "__device__ unsigned long long mjg_wave_t0[16384], mjg_wave_t1[16384];\n"
              "__device__ unsigned int mjg_wave_hw[16384], mjg_wave_xcc[16384], mjg_wave_n[16384];\n"
              "#define MJG_PH(i) do { if (MODE == kEmitDefault) { __builtin_amdgcn_sched_barrier(0); "
              "const unsigned long long _t = __builtin_amdgcn_s_memtime(); ph_acc[i] += _t - ph_prev; ph_prev = _t; "
              "__builtin_amdgcn_sched_barrier(0); } } while (0)\n")


def _phase_clock(a):
    return [
        (K, _PH_DECL, _PH_DEVICE),
        (K, "  while (true) {\n    // the next unit is reserved",
         "  unsigned long long ph_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, ph_prev = __builtin_amdgcn_s_memtime();\n"
         "  if (MODE == kEmitDefault && lane == 0 && gw < 16384) mjg_wave_t0[gw] = __builtin_amdgcn_s_memrealtime();\n"
         "  unsigned int ph_n = 0;\n"
         "  while (true) {\n    MJG_PH(7);\n    ph_n++;\n    // the next unit is reserved"),
        (K, "      row_pass<RC>(raw, tab, s_rc, s_pk, lane);\n", "      row_pass<RC>(raw, tab, s_rc, s_pk, lane);\n    MJG_PH(0);\n"),
        (K, "    uint32_t mlo = 0, mhi = 0;  // candidate mask", "    MJG_PH(1);\n    uint32_t mlo = 0, mhi = 0;  // candidate mask"),
        (K, "    if (SCR) mask = ((uint64_t)mhi << 32) | mlo;\n", "    if (SCR) mask = ((uint64_t)mhi << 32) | mlo;\n    MJG_PH(2);\n"),
        (K, "    if (cur_active && !((wide >> lane) & 1ull)) {", "    MJG_PH(3);\n    if (cur_active && !((wide >> lane) & 1ull)) {"),
        (K, "    if (wide) {  // the heavy blocks", "    MJG_PH(4);\n    if (wide) {  // the heavy blocks"),
        (K, "    const uint32_t qbits = cur_active ? q.bits : 0u;\n", "    MJG_PH(5);\n    const uint32_t qbits = cur_active ? q.bits : 0u;\n"),
        (K, "      pack_chunk(q, cur_active, scratch + (size_t)t * kSlotWords, chunk_bits + t, lane);\n    if (tn < 0) break;",
         "      pack_chunk(q, cur_active, scratch + (size_t)t * kSlotWords, chunk_bits + t, lane);\n    MJG_PH(6);\n"
         "    if (tn < 0) break;"),
        (K, "  if (MODE == kCount && aux_frame >= 0) {\n    asm volatile",
         "  if (MODE == kEmitDefault && lane == 0)\n    for (int i = 0; i < 8; i++) atomicAdd(&mjg_phase_acc[i], ph_acc[i]);\n"
         "  if (MODE == kEmitDefault && lane == 0 && gw < 16384) {\n    mjg_wave_t1[gw] = __builtin_amdgcn_s_memrealtime();\n"
         "    mjg_wave_hw[gw] = __builtin_amdgcn_s_getreg((31 << 11) | 4);\n"
         "    mjg_wave_xcc[gw] = __builtin_amdgcn_s_getreg((31 << 11) | 20);\n    mjg_wave_n[gw] = ph_n;\n  }\n"
         "  if (MODE == kCount && aux_frame >= 0) {\n    asm volatile"),
        ("api.hip", "}  // extern \"C\"", "int mjg_probe_phase(unsigned long long *out) {\n"
         "  HIP_TRY(hipDeviceSynchronize());\n  HIP_TRY(hipMemcpyFromSymbol(out, HIP_SYMBOL(mjg_phase_acc), 64));\n"
         "  unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(mjg_phase_acc), z, 64));\n"
         "  return MJG_OK;\n}\n"
         "int mjg_probe_waves(unsigned long long *t0, unsigned long long *t1) {\n"
         "  HIP_TRY(hipDeviceSynchronize());\n"
         "  HIP_TRY(hipMemcpyFromSymbol(t0, HIP_SYMBOL(mjg_wave_t0), 16384 * 8));\n"
         "  HIP_TRY(hipMemcpyFromSymbol(t1, HIP_SYMBOL(mjg_wave_t1), 16384 * 8));\n"
         "  HIP_TRY(hipMemcpyFromSymbol(t0 + 16384, HIP_SYMBOL(mjg_wave_hw), 16384 * 4));\n"
         "  HIP_TRY(hipMemcpyFromSymbol(t0 + 16384 + 8192, HIP_SYMBOL(mjg_wave_xcc), 16384 * 4));\n"
         "  HIP_TRY(hipMemcpyFromSymbol(t1 + 16384, HIP_SYMBOL(mjg_wave_n), 16384 * 4));\n"
         "  std::vector<unsigned long long> z(16384, 0ull);\n"
         "  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(mjg_wave_t0), z.data(), 16384 * 8));\n"
         "  HIP_TRY(hipMemcpyToSymbol(HIP_SYMBOL(mjg_wave_t1), z.data(), 16384 * 8));\n"
         "  return MJG_OK;\n}\n}  // extern \"C\""),
    ]


PATCHES["phase_clock"] = _phase_clock


# ---------------------------------------------------------------- wave priority experiments (r04)
# The SIMD arbiter favours its oldest wave: per chunk, wave slot 0 runs 2.2x faster than slot 3
# (profiles/r04j_drain_by_hw.txt), so at the end of a launch the slowest waves hold the last units.
_NEXT = "      tn = nbu < nbatch ? nbu * kBatch : -1;\n"
PATCHES["prio_late"] = lambda a: [(K, _NEXT, _NEXT +
    "      if (nbu < nbatch) {  // a unit among the last of its eighth: run it at top priority\n"
    "        const int xe = (int)(((long long)nbu * NX) / nbatch);\n"
    "        int e = xu.start(xe + 1);\n"
    "        if (nbu >= e) e = xu.start(xe + 2);\n"
    "        if (e - nbu <= " + str(int(a or 512)) + ") __builtin_amdgcn_s_setprio(3);\n"
    "      }\n")]
PATCHES["prio_slot"] = lambda a: [(K, "  __syncthreads();  // tables visible; the only workgroup barrier\n",
    "  __syncthreads();  // tables visible; the only workgroup barrier\n"
    "  {  // equalise the arbiter: younger wave slots get higher priority\n"
    "    const uint32_t slot = __builtin_amdgcn_readfirstlane(__builtin_amdgcn_s_getreg((3 << 11) | 4)) & 3u;\n"
    "    if (slot == 1) __builtin_amdgcn_s_setprio(1);\n"
    "    if (slot == 2) __builtin_amdgcn_s_setprio(2);\n"
    "    if (slot == 3) __builtin_amdgcn_s_setprio(3);\n"
    "  }\n")]

# every submit on one stream, back to back (round 3's form for default tables; a stream per
# slot since r04, profiles/r04m_ab_two_streams_bench.txt)
PATCHES["one_stream"] = lambda a: [("api.hip", "  S.st = slot_stream(c, (int)(&S - c->slot));", "  S.st = c->stream;")]
# the submit queue three deep, a stream per slot (profiles/r04aa_depth_priority.txt: 10% slower,
# three k_encode launches share the CUs)
PATCHES["slots3"] = lambda a: [("api.hip", "constexpr int kSlots = 2;", "constexpr int kSlots = 3;")]

# probes (wrong output): the stuffing tail's co-run cost on the bench (the kernels launch, and
# return at once)
PATCHES["no_write"] = lambda a: [(K, "  const int gi = blockIdx.x * 4 + wave, ngroups = gps * nseg * nframes;\n  if (gi >= ngroups) return;",
                                  "  const int gi = blockIdx.x * 4 + wave, ngroups = gps * nseg * nframes;\n  if (gi >= 0) return;")]
PATCHES["no_count"] = lambda a: [(K, "  for (int i = lane; i < 64 * kTailRounds; i += 64) s_marks[wave][i] = 0;\n  if (gi >= ngroups) return;",
                                  "  for (int i = lane; i < 64 * kTailRounds; i += 64) s_marks[wave][i] = 0;\n  if (gi >= 0) return;")]


# emit_block taking four candidates per step instead of two (more LDS reads in flight)
_PAIR_OLD = """  while (cand) {
    const int k1 = (int)__builtin_ctzll(cand);"""
_PAIR_END = """    prev = nz2 ? k2 : p1;
  }
"""
_QUAD = """  while (cand) {
    int kq[4], tq[4], fq[4];
    bool hq[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      hq[i] = cand != 0;
      kq[i] = hq[i] ? (int)__builtin_ctzll(cand) : 0;
      cand &= cand - 1;
    }
#pragma unroll
    for (int i = 0; i < 4; i++) tq[i] = exact_coef_t(pkcol, zd[kq[i]], m2);
    int p = prev, sq[4], rq[4];
    uint32_t eq[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      fq[i] = hq[i] ? ffbh_i32(tq[i]) : -1;
      rq[i] = kq[i] - p - 1;
      p = fq[i] >= 0 ? kq[i] : p;
      sq[i] = fq[i] >= 0 ? ((rq[i] & 15) << 4) | (32 - fq[i]) : 0;
      eq[i] = sink.lookup(sq[i]);
    }
#pragma unroll
    for (int i = 0; i < 4; i++)
      if (fq[i] >= 0) {
        for (int r = rq[i]; r >= 16; r -= 16) sink.ac(0xf0, 0, 0u);
        sink.put_ac(eq[i], sq[i], 32 - fq[i], __builtin_amdgcn_ubfe((uint32_t)tq[i], 0u, (uint32_t)(32 - fq[i])));
      }
    prev = p;
  }
"""


def _quad(a):
    src = open(os.path.join(CSRC, K)).read()
    i = src.index(_PAIR_OLD)
    j = src.index(_PAIR_END, i) + len(_PAIR_END)
    return [(K, src[i:j], _QUAD)]


PATCHES["quad"] = _quad


def _quad_adaptive(a):
    """emit_block's four-candidate form only for chunks where some per-lane block has more than
    `a` candidates (natural content), the pair form elsewhere (testsrc)"""
    src = open(os.path.join(CSRC, K)).read()
    i = src.index("template <class Sink>\n__device__ __forceinline__ void emit_block(")
    j = src.index("  if (prev != 63) sink.ac(0x00, 0, 0u);  // EOB\n}\n", i) + len("  if (prev != 63) sink.ac(0x00, 0, 0u);  // EOB\n}\n")
    body = src[i:j]
    k0 = body.index(_PAIR_OLD)
    k1 = body.index(_PAIR_END, k0) + len(_PAIR_END)
    quad = body[:k0] + _QUAD + body[k1:]
    quad = quad.replace("void emit_block(", "void emit_block4(")
    call = "      emit_block(s_pk + lane, mask, diff, s_zd, s_m2, q);\n"
    return [
        (K, body, body + "\n" + quad),
        (K, "    if (cur_active && !((wide >> lane) & 1ull)) {\n" + call,
         f"    const bool quad_h = __ballot(cur_active && !((wide >> lane) & 1ull) && __popcll(mask) > {int(a)}) != 0ull;\n"
         "    if (cur_active && !((wide >> lane) & 1ull)) {\n"
         "      if (quad_h)\n  emit_block4(s_pk + lane, mask, diff, s_zd, s_m2, q);\n      else\n  " + call),
    ]


PATCHES["quad_adaptive"] = _quad_adaptive


# the chunk-parallel coder prototype (tools/cpc_proto.hip) in place of the per-lane emission,
# the wave-parallel blocks and pack_chunk
_CPC_OLD_START = "    const uint64_t wide = wave_parallel_blocks(cur_active ? __popcll(mask) : 0);\n"
_CPC_OLD_END = "      pack_chunk(q, cur_active, scratch + (size_t)t * kSlotWords, chunk_bits + t, lane);\n"


def _cpc(a):
    src = open(os.path.join(CSRC, K)).read()
    i = src.index(_CPC_OLD_START)
    j = src.index(_CPC_OLD_END, i) + len(_CPC_OLD_END)
    proto = open(os.path.join(HERE, "cpc_proto.hip")).read()
    hv = "  uint32_t *s_hv = s_hv_all[MODE == kEmitDefault ? wave : 0];\n"
    return [
        (K, "template <int NX>\nstruct XcdUnits {", proto + "template <int NX>\nstruct XcdUnits {"),
        (K, hv, hv + "  __shared__ uint32_t s_ring_all[MODE == kEmitDefault ? kWavesPerWg : 1][kRingWords];\n"
                     "  if (MODE == kEmitDefault)\n"
                     "    for (int i = lane; i < kRingWords; i += 64) s_ring_all[wave][i] = 0u;\n"),
        (K, src[i:j], "    emit_chunk_cpc(s_pk, lane, cur_active, mask, diff, tab, s_zd, s_m2, s_ac, s_dc,\n"
                      "                   s_ring_all[MODE == kEmitDefault ? wave : 0], stage_w,\n"
                      "                   scratch + (size_t)t * kSlotWords, chunk_bits + t);\n"),
    ]


PATCHES["cpc"] = _cpc


def _cpc_hybrid(a):
    """the prototype only for chunks whose per-lane cost exceeds a * rounds"""
    src = open(os.path.join(CSRC, K)).read()
    i = src.index(_CPC_OLD_START)
    j = src.index(_CPC_OLD_END, i) + len(_CPC_OLD_END)
    p = _cpc(a)
    p[2] = (K, src[i:j],
            "    const int nc_h = cur_active ? __popcll(mask) : 0;\n"
            "    const int rounds_h = (wave_sum(cur_active ? nc_h + 1 : 0) + 63) >> 6;\n"
            f"    if (per_lane_cost(nc_h) > {float(a)}f * rounds_h) {{\n"
            "    emit_chunk_cpc(s_pk, lane, cur_active, mask, diff, tab, s_zd, s_m2, s_ac, s_dc,\n"
            "                   s_ring_all[MODE == kEmitDefault ? wave : 0], stage_w,\n"
            "                   scratch + (size_t)t * kSlotWords, chunk_bits + t);\n"
            "    } else {\n" + src[i:j] + "    }\n")
    return p


PATCHES["cpc_hybrid"] = _cpc_hybrid


# HIP stream priority of the stuffing tail's stream (the product: the highest, since r04;
# profiles/r04s_ab_stream_priority.txt, r04z_ab_tail_high_priority.txt, r04aa_depth_priority.txt):
# "low" = the lowest, "normal" = the default (rounds 1-4 until r04)
PATCHES["stream_prio"] = lambda a: [("api.hip", "  HIP_TRY(hipStreamCreateWithPriority(&c->tail, hipStreamNonBlocking, greatest));\n",
                                     "  HIP_TRY(hipStreamCreateWithPriority(&c->tail, hipStreamNonBlocking, "
                                     + {"low": "least", "normal": "0"}.get(a, "0") + "));\n")]


# pack_chunk for every chunk, without pack_chunk_short's fast path for chunks of short blocks
# (profiles/r04t_ab_short_pack.txt, r04w_bench_ab_short_pack_pack64.txt)
PATCHES["no_short_pack"] = lambda a: [(K, """    if (__ballot(qbits > 32u || q.staged) == 0ull)
      pack_chunk_short<32>(q, qbits, s_hv, scratch + (size_t)t * kSlotWords, chunk_bits + t, lane);
    else if (__ballot(qbits > 64u || q.staged) == 0ull)
      pack_chunk_short<64>(q, qbits, s_hv, scratch + (size_t)t * kSlotWords, chunk_bits + t, lane);
    else
""", "")]
# only the 32-bit fast path (HEAD 2ffb3a0; profiles/r04w_bench_ab_short_pack_pack64.txt)
PATCHES["no_pack64"] = lambda a: [(K, """    else if (__ballot(qbits > 64u || q.staged) == 0ull)
      pack_chunk_short<64>(q, qbits, s_hv, scratch + (size_t)t * kSlotWords, chunk_bits + t, lane);
""", "")]




# the screen's candidate-bit deposit as two forced VALU per coefficient (v_lshrrev of the sign,
# v_lshl_or into the mask) instead of the compiler's shift / and / or3 form
_DEPOSIT = """          if (z < 32)
            mlo |= (neg >> 31) << z;
          else
            mhi |= (neg >> 31) << (z - 32);
"""
PATCHES["deposit_asm"] = lambda a: [(K, _DEPOSIT, """          const uint32_t sb = neg >> 31;
          if (z < 32)
            asm("v_lshl_or_b32 %0, %1, %2, %0" : "+v"(mlo) : "v"(sb), "n"(z));
          else
            asm("v_lshl_or_b32 %0, %1, %2, %0" : "+v"(mhi) : "v"(sb), "n"(z - 32));
""")]


# the stuffing tail's wave priority (the product: kTailPrio = 2 since r04; before: 0).  They
# share SIMDs with the next submit's k_encode waves, which the oldest-first arbiter otherwise
# issues first (profiles/r04ad_tail_wave_priority.txt, r04ae_tail_wave_priority_levels.txt)
PATCHES["tail_prio"] = lambda a: [(K, "constexpr int kTailPrio = 2;", f"constexpr int kTailPrio = {int(a) if a else 0};")]
# the raise for every submit, light or heavy (r04ad/r04ae's form)
PATCHES["tail_prio_always"] = lambda a: [(K, "constexpr uint32_t kTailLightBits = 1800;", "constexpr uint32_t kTailLightBits = 0xffffffffu / 65536u;")]


# -huffman optimal's counting pass sized to its own occupancy (3 workgroups per CU; r04 until
# r04an) instead of the default pass's grid (profiles/r04an_c1_count_grid_tail_prio.txt)
PATCHES["count_grid_own"] = lambda a: [("api.hip", "  c->enc_grid_cnt = c->enc_grid;\n",
                                         "  c->enc_grid_cnt = c->enc_grid;\n  if (c->optimal) {\n    int pc = 0;\n"
                                         "    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&pc, (const void *)k_encode<true, kCount>, 64 * kWavesPerWg, 0));\n"
                                         "    c->enc_grid_cnt = std::max(1, ncu * std::max(1, pc));\n  }\n")]


# k_encode's persistent grid at N workgroups per CU below the occupancy (4): the launch leaves
# CU slots free for the next submit's k_encode and for the tail
PATCHES["enc_grid_per_cu"] = lambda a: [("api.hip", "  c->enc_grid = std::max(1, ncu * std::max(1, per_cu));\n",
                                          f"  c->enc_grid = std::max(1, ncu * std::max(1, std::min(per_cu, {int(a) if a else 3})));\n")]


# young waves (wave slot >= 2 on their SIMD: the oldest-first arbiter runs them ~2x slower) stop
# taking units when fewer than (waves of the XCD) / D remain on their XCD, so the launch's last
# units run on old waves and the drain is shorter; old waves still pull until every counter is dry
def _young_exit(a):
    d = int(a) if a else 2
    return [
        (K, """  __device__ __forceinline__ int next(uint32_t *ctr, int nwg) const {
    for (int k = 0; k < NX; k++) {""", f"""  __device__ __forceinline__ int next(uint32_t *ctr, int nwg, bool young = false) const {{
    if (young) {{
      const int used = (int)__hip_atomic_load(ctr + j * kCtrStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (start(j + 1) - (start(j) + nw(j, nwg) + used) < nw(j, nwg) / {d}) return nbatch;
    }}
    for (int k = 0; k < NX; k++) {{"""),
        (K, "    if (t + 1 == tend && lane == 0) nb = (uint32_t)xu.next(work_ctr, nwg);",
         "    if (t + 1 == tend && lane == 0) nb = (uint32_t)xu.next(work_ctr, nwg, young_w);"),
        (K, "  const int nwg = gridDim.x;\n  int u0 = xu.start(xu.j)",
         "  const int nwg = gridDim.x;\n  const bool young_w = NX > 1 && (__builtin_amdgcn_s_getreg((31 << 11) | 4) & 15) >= 2;\n  int u0 = xu.start(xu.j)"),
    ]


PATCHES["young_exit"] = _young_exit


# young waves (wave slot >= 2 on their SIMD) pull dynamic units of S chunks instead of kBatch,
# so a unit takes about as long on a young wave as a full one on an old wave and the launch's
# last units end closer together; the per-XCD counters count chunks instead of units
# (S = kBatch: the same schedule as HEAD with chunk counters, a control)
def _young_half(a):
    s = int(a) if a else 6
    return [
        (K, """  // lane 0: the next unit (>= nbatch: none left)
  __device__ __forceinline__ int next(uint32_t *ctr, int nwg) const {""",
         """  // lane 0: chunks [p, e) of the next dynamic range of `size` chunks (p >= ntasks: none left)
  __device__ __forceinline__ int next_c(uint32_t *ctr, int nwg, int size, int kb, int ntasks, int &e) const {
    for (int k = 0; k < NX; k++) {
      const int x = (j + k) & (NX - 1), ce = min(start(x + 1) * kb, ntasks);
      const int p = (start(x) + nw(x, nwg)) * kb + (int)atomicAdd(ctr + x * kCtrStride, (uint32_t)size);
      if (p < ce) {
        e = min(p + size, ce);
        return p;
      }
    }
    return ntasks;
  }
  // lane 0: the next unit (>= nbatch: none left)
  __device__ __forceinline__ int next(uint32_t *ctr, int nwg) const {"""),
        (K, """  if (u0 >= xu.start(xu.j + 1)) {  // none: straight to the counters
    int v = 0;
    if (lane == 0) v = xu.next(work_ctr, nwg);
    u0 = __builtin_amdgcn_readfirstlane(v);
    if (u0 >= nbatch) return;
  }""", f"""  const bool young_w = NX > 1 && (__builtin_amdgcn_s_getreg((31 << 11) | 4) & 15) >= 2;
  const int usz = young_w ? {s} : kBatch;
  int t0 = u0 * kBatch, te0 = min(t0 + kBatch, ntasks);
  if (u0 >= xu.start(xu.j + 1)) {{  // none: straight to the counters
    int v = 0, ve = 0;
    if (lane == 0) v = xu.next_c(work_ctr, nwg, usz, kBatch, ntasks, ve);
    t0 = __builtin_amdgcn_readfirstlane(v);
    te0 = __builtin_amdgcn_readfirstlane(ve);
    if (t0 >= ntasks) return;
  }}"""),
        (K, "  int t = u0 * kBatch, tend = min(t + kBatch, ntasks);\n  uint32_t nb = 0;",
         "  int t = t0, tend = te0;\n  uint32_t nb = 0, nbe = 0;"),
        (K, "    if (t + 1 == tend && lane == 0) nb = (uint32_t)xu.next(work_ctr, nwg);",
         """    if (t + 1 == tend && lane == 0) {
      int e_ = 0;
      nb = (uint32_t)xu.next_c(work_ctr, nwg, usz, kBatch, ntasks, e_);
      nbe = (uint32_t)e_;
    }"""),
        (K, """    const bool new_batch = tn >= tend;
    if (new_batch) {
      const int nbu = __builtin_amdgcn_readfirstlane(nb);
      tn = nbu < nbatch ? nbu * kBatch : -1;
    }""", """    const bool new_batch = tn >= tend;
    int nend = 0;
    if (new_batch) {
      const int nbu = __builtin_amdgcn_readfirstlane(nb);
      tn = nbu < ntasks ? nbu : -1;
      nend = __builtin_amdgcn_readfirstlane(nbe);
    }"""),
        (K, "carry = carry_finish(crow, chunk, lane, rc, g, s_desc);\n        tend = min(tn + kBatch, ntasks);",
         "carry = carry_finish(crow, chunk, lane, rc, g, s_desc);\n        tend = nend;"),
        (K, "carry = carry_finish(crow, chunk, lane, rc, g, s_desc);\n      tend = min(tn + kBatch, ntasks);",
         "carry = carry_finish(crow, chunk, lane, rc, g, s_desc);\n      tend = nend;"),
    ]


PATCHES["young_half"] = _young_half


def parse_spec(spec: str):
    """'no_skip+wide_cost=3' -> [('no_skip', None), ('wide_cost', '3')]"""
    out = []
    for item in spec.split("+"):
        name, _, arg = item.partition("=")
        if name not in PATCHES:
            raise KeyError(f"unknown patch {name!r} (known: {', '.join(sorted(PATCHES))})")
        out.append((name, arg or None))
    return out


def apply(spec: str, dst: str, src: str = CSRC) -> str:
    """Copy `src` (the product csrc) to `dst` and apply the patches of `spec`; returns dst."""
    if os.path.isdir(dst):
        shutil.rmtree(dst)
    shutil.copytree(src, dst)
    for name, arg in parse_spec(spec):
        for fname, old, new in PATCHES[name](arg):
            path = os.path.join(dst, fname)
            with open(path) as f:
                text = f.read()
            n = text.count(old)
            if n != 1:
                raise ValueError(f"patch {name}: anchor found {n} times in {fname}")
            with open(path, "w") as f:
                f.write(text.replace(old, new))
    return dst


def check_all() -> dict:
    """Every patch's anchors against the current product source (tests/test_abi.py)."""
    res = {}
    for name, fn in PATCHES.items():
        edits = fn("1")
        ok = True
        for fname, old, _ in edits:
            with open(os.path.join(CSRC, fname)) as f:
                ok &= f.read().count(old) == 1
        res[name] = ok
    return res


if __name__ == "__main__":
    import json
    print(json.dumps(check_all(), indent=1))
