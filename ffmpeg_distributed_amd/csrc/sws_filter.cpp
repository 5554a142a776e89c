// See sws_filter.h.  Reference semantics: libswscale/utils.c initFilter (bicubic).
#include "sws_filter.h"

#include <cmath>
#include <cstdlib>

namespace mjg {

namespace {

int ilog2(unsigned v) {
  int n = 0;
  while (v >>= 1) n++;
  return n;
}

// Bicubic kernel in swscale's fixed point: d is |distance| in 1/2^30 source units,
// result scaled by 2^54 / fone.
int64_t bicubic_coeff(int64_t d, int64_t fone) {
  const int64_t B = 0;
  const int64_t C = (int64_t)(0.6 * (1 << 24));
  int64_t c;
  if (d >= (1LL << 31)) {
    c = 0;
  } else {
    const int64_t dd = (d * d) >> 30;
    const int64_t ddd = (dd * d) >> 30;
    if (d < (1LL << 30))
      c = (12 * (1 << 24) - 9 * B - 6 * C) * ddd + (-18 * (1 << 24) + 12 * B + 6 * C) * dd +
          (6 * (1 << 24) - 2 * B) * (1LL << 30);
    else
      c = (-B - 6 * C) * ddd + (6 * B + 30 * C) * dd + (-12 * B - 48 * C) * d +
          (8 * B + 24 * C) * (1LL << 30);
  }
  return c / ((1LL << 54) / fone);
}

}  // namespace

int sws_local_pos(int chroma_shift, int pos) {
  if (pos == -1 || pos <= -513) pos = (128 << chroma_shift) - 128;
  pos += 128;
  return pos >> chroma_shift;
}

bool make_sws_filter(int src_len, int dst_len, int one, int align, bool bitexact, int src_pos,
                     int dst_pos, SwsFilter *out) {
  if (src_len <= 0 || dst_len <= 0) return false;
  const int64_t inc = (((int64_t)src_len << 16) + (dst_len >> 1)) / dst_len;
  const int lg = ilog2((unsigned)(src_len / dst_len));
  const int64_t fone = 1LL << (54 - (lg < 8 ? lg : 8));

  int size;
  std::vector<int64_t> f;
  std::vector<int32_t> pos(dst_len);

  if (std::llabs(inc - 0x10000) < 10 && src_pos == dst_pos) {
    size = 1;
    f.assign((size_t)dst_len, fone);
    for (int i = 0; i < dst_len; i++) pos[i] = i;
  } else {
    const int size_factor = 4;  // bicubic
    size = (inc <= (1 << 16)) ? 1 + size_factor
                              : 1 + (int)((size_factor * (int64_t)src_len + dst_len - 1) / dst_len);
    if (size > src_len - 2) size = src_len - 2;
    if (size < 1) size = 1;
    f.assign((size_t)dst_len * size, 0);
    // centre of output sample i in source coordinates, 1/2^17 units
    int64_t centre = ((dst_pos * inc) >> 7) - ((src_pos * 0x10000LL) >> 7);
    for (int i = 0; i < dst_len; i++, centre += 2 * inc) {
      int xx = (int)((centre - (size - 2) * (1LL << 16)) / (1 << 17));
      pos[i] = xx;
      for (int j = 0; j < size; j++, xx++) {
        int64_t d = std::llabs((int64_t)xx * (1 << 17) - centre) << 13;
        if (inc > (1 << 16)) d = d * dst_len / src_len;
        f[(size_t)i * size + j] = bicubic_coeff(d, fone);
      }
    }
  }

  // Reduce: drop near-zero leading taps (keeping pos monotone), measure trailing ones.
  int min_size = 0;
  const double cutoff_limit = 0.002 * (double)fone;
  for (int i = dst_len - 1; i >= 0; i--) {
    int64_t *row = &f[(size_t)i * size];
    int keep = size;
    int64_t cut = 0;
    for (int j = 0; j < size; j++) {
      cut += std::llabs(row[0]);
      if ((double)cut > cutoff_limit) break;
      if (i < dst_len - 1 && pos[i] >= pos[i + 1]) break;
      for (int k = 1; k < size; k++) row[k - 1] = row[k];
      row[size - 1] = 0;
      pos[i]++;
    }
    cut = 0;
    for (int j = size - 1; j > 0; j--) {
      cut += std::llabs(row[j]);
      if ((double)cut > cutoff_limit) break;
      keep--;
    }
    if (keep > min_size) min_size = keep;
  }
  if (min_size == 1 && align == 2) align = 1;  // x86 unscaled-vertical special case
  const int taps = (min_size + (align - 1)) & ~(align - 1);
  if (taps >= 256) return false;  // would need swscale's cascade

  std::vector<int64_t> g((size_t)dst_len * taps, 0);
  for (int i = 0; i < dst_len; i++)
    for (int j = 0; j < taps; j++) {
      int64_t v = (j < size) ? f[(size_t)i * size + j] : 0;
      if (bitexact && j >= min_size) v = 0;
      g[(size_t)i * taps + j] = v;
    }

  // Fold taps that fall outside [0, src_len) onto the edge samples.
  for (int i = 0; i < dst_len; i++) {
    int64_t *row = &g[(size_t)i * taps];
    if (pos[i] < 0) {
      for (int j = 1; j < taps; j++) {
        const int left = (j + pos[i] > 0) ? j + pos[i] : 0;
        row[left] += row[j];
        row[j] = 0;
      }
      pos[i] = 0;
    }
    if (pos[i] + taps > src_len) {
      const int shift = pos[i] + ((taps - src_len) < 0 ? taps - src_len : 0);
      int64_t acc = 0;
      for (int j = taps - 1; j >= 0; j--)
        if (pos[i] + j >= src_len) {
          acc += row[j];
          row[j] = 0;
        }
      for (int j = taps - 1; j >= 0; j--) row[j] = (j < shift) ? 0 : row[j - shift];
      pos[i] -= shift;
      row[src_len - 1 - pos[i]] += acc;
    }
  }

  // Normalise to `one` with error diffusion (ROUNDED_DIV).
  out->dst_len = dst_len;
  out->taps = taps;
  out->coeff.assign((size_t)dst_len * taps, 0);
  out->pos = pos;
  for (int i = 0; i < dst_len; i++) {
    const int64_t *row = &g[(size_t)i * taps];
    int64_t sum = 0, err = 0;
    for (int j = 0; j < taps; j++) sum += row[j];
    sum = (sum + one / 2) / one;
    if (!sum) sum = 1;
    for (int j = 0; j < taps; j++) {
      const int64_t v = row[j] + err;
      const int64_t q = v >= 0 ? (v + (sum >> 1)) / sum : (v - (sum >> 1)) / sum;
      out->coeff[(size_t)i * taps + j] = (int16_t)q;
      err = v - q * sum;
    }
  }
  return true;
}

}  // namespace mjg
