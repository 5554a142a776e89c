// Host-side generation of swscale's fixed-point bicubic filter tables for the
// `-vf scale=W:H:flags=bicubic` leg of the reference worker's remote_args
// (ffmpeg_distributed.py:134 passes them to `ffmpeg`).  Semantics follow
// libswscale/utils.c initFilter (B=0, C=0.6; fixed-point distance math; the
// 0.002 reduce cutoff; x86 filter alignment; border folding; error-diffusion
// normalisation).  The GPU kernels only *apply* these tables.
#pragma once
#include <stdint.h>
#include <vector>

namespace mjg {

struct SwsFilter {
  int dst_len = 0;    // output samples
  int taps = 0;       // filter size per output sample
  std::vector<int16_t> coeff;  // dst_len * taps
  std::vector<int32_t> pos;    // dst_len, first source sample of each tap window
};

// one: 1<<14 (horizontal) or 1<<12 (vertical); align: 4 (horizontal) / 2 (vertical) on
// x86; src_pos/dst_pos: swscale "local position" (128 = centred sample).
// Returns false when the filter would need swscale's cascade path (unsupported).
bool make_sws_filter(int src_len, int dst_len, int one, int align, bool bitexact,
                     int src_pos, int dst_pos, SwsFilter *out);

// swscale get_local_pos() for the default (-513) chroma siting.
int sws_local_pos(int chroma_shift, int pos);

}  // namespace mjg
