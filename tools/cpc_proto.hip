// Chunk-parallel coder (prototype for A/B only; inserted into kernels.hip by tools/patches.py
// "cpc"; the product kernels code per lane + wave-parallel blocks, see emit_block).
//
// One chunk's 64 blocks as ONE list of items in stream order: per block its DC item, then one
// item per screen candidate (zigzag order).  Rounds of 64 items, lane = item, so the work per
// round does not depend on how the candidates are spread over the blocks (the per-lane loop
// runs as long as the chunk's heaviest block).
//   list:    each lane writes its block's items (b << 6 | k, k = 0 the DC) at its offset, an
//            exclusive scan of 1 + candidates, into the wave's staging area (u16)
//   item:    exact coefficient (exact_coef_t on block b's column, any lane), its category
//   run:     the last nonzero item before it (a wave max-scan of b << 6 | k over the nonzero and
//            DC items; the list is sorted, so the max is the nearest one) and the carried max of
//            the earlier rounds
//   EOB:     appended to the block's last item (the next item belongs to another block) unless
//            that item is a nonzero coefficient 63
//   bits:    a wave sum-scan of the item lengths (<= 63 bits) places them; ORed into a 128-word
//            LDS ring, whose complete words go to the chunk's slot after every round
// Same bytes as emit_block + pack_chunk (FFmpeg encode_block).
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true));   // row_shr:1
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true));   // row_shr:2
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true));   // row_shr:4
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true));   // row_shr:8
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false));  // row_bcast:15
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false));  // row_bcast:31
  return v;
}

constexpr int kRingWords = 128;

__device__ __forceinline__ void emit_chunk_cpc(const uint32_t *s_pk, int lane, bool active, uint64_t mask, int diff,
                                            int tab, const uint4 *zd, const uint32_t *m2, const uint32_t *s_ac,
                                            const uint32_t *s_dc, uint32_t *ring, uint32_t *stage_w,
                                            uint32_t *slot, uint32_t *chunk_bits_t) {
  // the item list
  const uint32_t items = active ? (uint32_t)__popcll(mask) + 1u : 0u;
  const uint32_t incl0 = wave_incl_scan(items, lane);
  const int T = (int)lane63(incl0);
  uint16_t *list = (uint16_t *)stage_w;
  if (active) {
    uint16_t *l = list + (incl0 - items);
    const uint32_t bb = (uint32_t)lane << 6;
    l[0] = (uint16_t)bb;
    int j = 1;
    for (uint64_t m = mask; m; m &= m - 1, j++) l[j] = (uint16_t)(bb | (uint32_t)__builtin_ctzll(m));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the list visible to the other lanes
  // per block, for its items' lanes: diff (int16), table, and the index of its last item
  const uint32_t dpk = ((uint32_t)diff & 0xffffu) | ((uint32_t)tab << 16) | ((incl0 - 1u) << 17);

  uint32_t base = 0, flushed = 0, cmax = 0;
  uint32_t itn = lane < T ? list[lane] : 0xffffu;
  for (int r0 = 0; r0 < T; r0 += 64) {
    const int i = r0 + lane;
    const bool valid = i < T;
    const uint32_t it = itn;
    itn = i + 64 < T ? list[i + 64] : 0xffffu;  // the next round's item, in flight during this one
    const int b = (int)(it >> 6) & 63, k = (int)(it & 63u);
    const uint32_t dd = (uint32_t)__builtin_amdgcn_ds_bpermute(b << 2, (int)dpk);
    const int diff_b = (int)(int16_t)(dd & 0xffffu), tab_b = (int)((dd >> 16) & 1u);
    const bool isdc = k == 0, last = (uint32_t)i == (dd >> 17);
    int t = exact_coef_t(s_pk + b, zd[k], m2);
    if (isdc) t = diff_b + (diff_b >> 31);
    const int fb = ffbh_i32(t);
    const bool nz = fb >= 0;
    const int cat = nz ? 32 - fb : 0;
    const bool mark = valid && (isdc || nz);
    const uint32_t inc = wave_incl_max(mark ? it : 0u);
    const uint32_t exc = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)inc, 0x138, 0xf, 0xf, false);  // wave_shr:1
    const int prevk = (int)(max(exc, cmax) & 63u);
    cmax = max(cmax, lane63(inc));
    const int run = k - prevk - 1;
    const uint32_t *act = s_ac + tab_b * 256;
    const uint32_t e = isdc ? s_dc[tab_b * 16 + cat] : act[((run & 15) << 4) | cat];
    uint64_t V = 0;
    uint32_t L = 0;
    if (valid && !isdc && nz && run >= 16) {
      const uint32_t ez = act[0xf0];  // ZRL
      for (int r = run; r >= 16; r -= 16) {
        V = (V << (ez >> 16)) | (ez & 0xffffu);
        L += ez >> 16;
      }
    }
    if (mark) {
      const uint32_t cl = (e >> 16) + (uint32_t)cat;
      V = (V << cl) | (((e & 0xffffu) << cat) | __builtin_amdgcn_ubfe((uint32_t)t, 0u, (uint32_t)cat));
      L += cl;
    }
    if (valid && last && !(nz && !isdc && k == 63)) {
      const uint32_t eo = act[0x00];  // EOB
      V = (V << (eo >> 16)) | (eo & 0xffffu);
      L += eo >> 16;
    }
    const uint32_t incl = wave_incl_scan(L, lane), off = base + incl - L;
    if (L) {  // bits [off, off + L), MSB first (emit_block_wave's placement)
      const uint32_t sh = 96u - (off & 31u) - L;
      const uint64_t hi = sh >= 32u ? V << (sh - 32u) : V >> (32u - sh);
      const uint32_t lo = sh >= 32u ? 0u : (uint32_t)(V << sh);
      const uint32_t w = off >> 5;
      atomicOr(ring + (w & (kRingWords - 1)), (uint32_t)(hi >> 32));
      if ((uint32_t)hi) atomicOr(ring + ((w + 1) & (kRingWords - 1)), (uint32_t)hi);
      if (lo) atomicOr(ring + ((w + 2) & (kRingWords - 1)), lo);
    }
    base += lane63(incl);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint32_t done = base >> 5;  // complete words: at most 127 new ones per round
#pragma unroll
    for (uint32_t w = flushed + (uint32_t)lane, h = 0; h < 2; h++, w += 64)
      if (w < done) {
        slot[w] = ring[w & (kRingWords - 1)];
        ring[w & (kRingWords - 1)] = 0u;
      }
    flushed = done;
  }
  if ((base & 31u) && lane == 0) {
    slot[flushed] = ring[flushed & (kRingWords - 1)];
    ring[flushed & (kRingWords - 1)] = 0u;
  }
  if (lane == 0) *chunk_bits_t = base;
}

// The per-lane path's cost in candidate steps (wave_parallel_blocks' model): the smallest
// 4 x (wave-parallel blocks) + T, or the longest block when no split pays.
__device__ __forceinline__ int per_lane_cost(int ncand) {
  int serial = 64, best = 64;
#pragma unroll
  for (int k = 3; k >= 0; k--) {
    const uint64_t hv = __ballot(ncand > (4 << k));
    if (!hv) serial = 4 << k;
    else best = min(best, 4 * __popcll(hv) + (4 << k));
  }
  return min(serial, best);
}

