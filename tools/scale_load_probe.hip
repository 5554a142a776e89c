// Probe (perf tooling, not product): how fast can k_scale's window loads go on their own?
// k_scale (csrc/scale.hip) reads, per 64 x 64 output tile of a 2:1 plane, a window of 136 source
// rows x 144 bytes (16-byte pieces, 7 rows x 9 pieces per wave-instruction, 5 per wave), stages
// it in LDS and computes.  Its SQ counters show ~42% of wave time in s_waitcnt.  This probe runs
// only the loads over the c4 workload's luma planes (120 frames 3840 x 2160, resident in HBM):
//   mode 0  plain streaming read of the same bytes (16 B per lane, grid-stride): the ceiling
//   mode 1  k_scale's window pattern and tile order (XCD-contiguous), loads XOR-reduced
//   mode 2  as 1, plus the LDS staging, a barrier and one LDS read per lane (k_scale's shape)
//   mode 3  as 2 with 128-column x 32-row tiles (272-byte x 72-row windows: longer rows)
//   mode 4  as 2 in plain raster tile order
//   modes 5-9: other tile shapes (columns x rows), XCD order unless noted
// Every tile mode allocates k_scale's 19,584 bytes of LDS per workgroup (8 workgroups per CU).
// Usage: scale_load_probe [reps]   -> one line per mode: ms per 120 frames, GB/s of unique bytes
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr int W = 3840, H = 2160, NF = 120;
constexpr int kLds = 136 * 144;
template <int TW, int TH> constexpr int lds_bytes() { return (2 * TW + 16) * (2 * TH + 8) > kLds ? (2 * TW + 16) * (2 * TH + 8) : kLds; }

__global__ __launch_bounds__(256) void k_stream(const u32x4 *__restrict__ p, size_t n, uint32_t *out) {
  u32x4 acc = {0, 0, 0, 0};
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x5a5a5a5au) out[0] = 1;  // keeps the loads live
}

// TW output columns x TH output rows per tile (2:1: source window 2 TW + 16 bytes x 2 TH + 8 rows)
template <int TW, int TH, bool STAGE, bool XCD>
__global__ __launch_bounds__(256) void k_tiles(const uint8_t *__restrict__ src, uint32_t *out) {
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  constexpr int RB = 2 * TW + 16, PIECES = RB / 16, ROWS = 2 * TH + 8;
  constexpr int RPI = 64 / PIECES;                      // rows per wave-instruction
  constexpr int RPW = (ROWS + 3) / 4;                   // rows per wave
  constexpr int LPW = (RPW + RPI - 1) / RPI;            // loads per lane
  const int gx = W / 2 / TW, gy = (H / 2 + TH - 1) / TH;
  int t = blockIdx.x;
  if (XCD) {
    const int i = t, n = gridDim.x, j = i & 7, q = n >> 3, r = n & 7;
    t = j * q + min(j, r) + (i >> 3);
  }
  const int f = t / (gx * gy), rem = t - f * gx * gy, by = rem / gx, bx = rem - by * gx;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, rr = lane / PIECES, pc = lane - PIECES * rr;
  const int col = max(2 * TW * bx - 4, 0), row0 = 2 * TH * by - 4;
  const uint8_t *fs = src + (size_t)f * W * H;
  u32x4 v[LPW];
#pragma unroll
  for (int i = 0; i < LPW; i++) {
    const int r = RPW * wave + RPI * i + rr;
    const int sr = min(max(row0 + r, 0), H - 1);
    const int c = min(col + 16 * pc, W - 16);
    v[i] = (rr < RPI && RPI * i + rr < RPW && r < ROWS) ? *(const u32x4 *)(fs + (size_t)sr * W + c) : u32x4{0, 0, 0, 0};
  }
  uint32_t acc = 0;
  if (STAGE) {
#pragma unroll
    for (int i = 0; i < LPW; i++) {
      const int r = RPW * wave + RPI * i + rr;
      if (rr < RPI && RPI * i + rr < RPW && r < ROWS) *(u32x4 *)(smem + r * (RB / 4) + 4 * pc) = v[i] ^ 0x80808080u;
    }
    __syncthreads();
    const u32x4 w = *(const u32x4 *)(smem + (lane % ROWS) * (RB / 4) + 4 * (wave % PIECES));
    acc = w.x ^ w.y ^ w.z ^ w.w;
  } else {
#pragma unroll
    for (int i = 0; i < LPW; i++) acc ^= v[i].x ^ v[i].y ^ v[i].z ^ v[i].w;
  }
  if (acc == 0x5a5a5a5au) out[blockIdx.x] = acc;
}

template <int TW, int TH, bool STAGE, bool XCD>
static float run_tiles(const uint8_t *src, uint32_t *out, int reps) {
  const int gx = W / 2 / TW, gy = (H / 2 + TH - 1) / TH, n = gx * gy * NF;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  constexpr int L = lds_bytes<TW, TH>();
  k_tiles<TW, TH, STAGE, XCD><<<n, 256, L>>>(src, out);
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; i++) k_tiles<TW, TH, STAGE, XCD><<<n, 256, L>>>(src, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  const size_t bytes = (size_t)W * H * NF;
  uint8_t *p;
  uint32_t *o;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&o, 1 << 22) != hipSuccess) return 1;
  (void)hipMemset(p, 7, bytes);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  k_stream<<<8192, 256>>>((const u32x4 *)p, bytes / 16, o);
  (void)hipEventRecord(a);
  for (int i = 0; i < reps; i++) k_stream<<<8192, 256>>>((const u32x4 *)p, bytes / 16, o);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  ms /= reps;
  const double gb = bytes / 1e9;
  printf("mode 0 stream            %.4f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
  ms = run_tiles<64, 64, false, true>(p, o, reps);
  printf("mode 1 tiles 64x64 xcd   %.4f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
  ms = run_tiles<64, 64, true, true>(p, o, reps);
  printf("mode 2 +lds 64x64 xcd    %.4f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
  ms = run_tiles<128, 32, true, true>(p, o, reps);
  printf("mode 3 +lds 128x32 xcd   %.4f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
  ms = run_tiles<64, 64, true, false>(p, o, reps);
  printf("mode 4 +lds 64x64 raster %.4f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
  ms = run_tiles<256, 16, true, true>(p, o, reps);
  printf("mode 5 +lds 256x16 xcd   %.4f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
  ms = run_tiles<128, 24, true, true>(p, o, reps);
  printf("mode 6 +lds 128x24 xcd   %.4f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
  ms = run_tiles<96, 40, true, true>(p, o, reps);
  printf("mode 7 +lds 96x40 xcd    %.4f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
  ms = run_tiles<128, 32, true, false>(p, o, reps);
  printf("mode 8 +lds 128x32 raster %.4f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
  ms = run_tiles<32, 64, true, true>(p, o, reps);
  printf("mode 9 +lds 32x64 xcd    %.4f ms  %.0f GB/s\n", ms, gb / ms * 1e3);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
