// Bicubic resize of one plane for the `-vf scale=W:H:flags=bicubic` leg of the
// reference worker's remote_args (ffmpeg_distributed.py:134).  Applies swscale's
// fixed-point tables (sws_filter.cpp) exactly as libswscale's C path does:
//   hScale8To15_c: min((sum src*f) >> 7, 32767)            (14-bit coeffs)
//   lumRangeToJpeg_c / chrRangeToJpeg_c on that int16       (tv -> pc, if requested)
//   yuv2planeX_8_c: clip_u8(((64 << 12) + sum h*f) >> 19)  (12-bit coeffs, flat dither)
// One workgroup = a 64 x 16 output tile: the source window is staged in LDS with
// coalesced byte loads, the horizontal pass fills an int16 LDS tile of every source
// row the tile's vertical taps touch, then the vertical pass writes the output.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mjg {

constexpr int kScaleTileW = 64;
constexpr int kScaleTileH = 16;

struct ScaleGeom {
  int sw, sh, dw, dh;            // plane sizes
  int s_stride, d_stride;
  long long s_off, d_off;        // plane offset inside a frame
  long long s_fstride, d_fstride;  // frame strides
  int htaps, vtaps;
  int range;                     // 0 none, 1 luma tv->pc, 2 chroma tv->pc
  int lds_cols;                  // padded source-window width (multiple of 16)
  int lds_rows;                  // max source rows any tile needs
};

__device__ __forceinline__ int sws_range(int v, int range) {
  if (range == 1) {
    v = min(v, 30189);
    return (v * 19077 - 39057361) >> 14;
  }
  if (range == 2) {
    v = min(v, 30775);
    return (v * 4663 - 9289992) >> 12;
  }
  return v;
}

__global__ __launch_bounds__(256) void k_scale(const uint8_t *__restrict__ src,
                                               uint8_t *__restrict__ dst, ScaleGeom g,
                                               const int16_t *__restrict__ hc,
                                               const int32_t *__restrict__ hp,
                                               const int16_t *__restrict__ vc,
                                               const int32_t *__restrict__ vp) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int tid = threadIdx.x;
  const int x0 = blockIdx.x * kScaleTileW, y0 = blockIdx.y * kScaleTileH, f = blockIdx.z;
  const uint8_t *s = src + (size_t)f * g.s_fstride + g.s_off;
  uint8_t *d = dst + (size_t)f * g.d_fstride + g.d_off;
  const int xe = min(x0 + kScaleTileW, g.dw), ye = min(y0 + kScaleTileH, g.dh);
  const int r0 = vp[y0], r1 = vp[ye - 1] + g.vtaps;
  const int c0 = hp[x0], c1 = hp[xe - 1] + g.htaps;
  const int nr = r1 - r0, nc = c1 - c0;
  uint8_t *st = smem;
  int16_t *ht = (int16_t *)(smem + (size_t)g.lds_rows * g.lds_cols);

  for (int i = tid; i < nr * nc; i += 256) {
    const int r = i / nc, cc = i - r * nc;
    st[r * g.lds_cols + cc] = s[(size_t)(r0 + r) * g.s_stride + c0 + cc];
  }
  __syncthreads();
  for (int i = tid; i < nr * kScaleTileW; i += 256) {
    const int r = i >> 6, x = i & 63, xx = x0 + x;
    if (xx < g.dw) {
      const int16_t *fc = hc + (size_t)xx * g.htaps;
      const uint8_t *row = st + r * g.lds_cols + (hp[xx] - c0);
      int val = 0;
      for (int j = 0; j < g.htaps; j++) val += (int)row[j] * fc[j];
      val = min(val >> 7, 32767);
      ht[r * kScaleTileW + x] = (int16_t)sws_range(val, g.range);
    }
  }
  __syncthreads();
  for (int i = tid; i < kScaleTileH * kScaleTileW; i += 256) {
    const int y = i >> 6, x = i & 63, yy = y0 + y, xx = x0 + x;
    if (yy < g.dh && xx < g.dw) {
      const int16_t *fc = vc + (size_t)yy * g.vtaps;
      const int16_t *col = ht + (vp[yy] - r0) * kScaleTileW + x;
      int val = 64 << 12;
      for (int j = 0; j < g.vtaps; j++) val += (int)col[j * kScaleTileW] * fc[j];
      val >>= 19;
      d[(size_t)yy * g.d_stride + xx] = (uint8_t)min(max(val, 0), 255);
    }
  }
}

}  // namespace mjg
