// PMC calibration (perf tooling, not product): read / write buffers of known size with the
// access widths the encoder's kernels use, so FETCH_SIZE and WRITE_SIZE can be scaled to
// bytes per width on gfx950 (MI355X_MICROARCH.md: FETCH_SIZE is exact only when calibrated;
// it reads 1/2 of the bytes of wide coalesced streams).
//   k_calib_read8   8 B per lane (k_encode's pixel row loads)
//   k_calib_read4   4 B per lane (k_scale's window loads, the realign kernels' slot words)
//   k_calib_write4  4 B per lane (k_encode's slot words)
//   k_calib_write1  1 B per lane (k_scale's output pixels, k_write's bytes)
// Usage: calib_bin BYTES   (each kernel runs 3 times over BYTES bytes)
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

template <typename T>
__device__ void calib_read(const T *__restrict__ p, size_t n, T *out) {
  T acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == (T)0x5a) out[0] = acc;  // keep the loads live
}

template <typename T>
__device__ void calib_write(T *__restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = (T)i;
}

__global__ void k_calib_read8(const uint64_t *p, size_t n, uint64_t *o) { calib_read<uint64_t>(p, n, o); }
__global__ void k_calib_read4(const uint32_t *p, size_t n, uint32_t *o) { calib_read<uint32_t>(p, n, o); }
__global__ void k_calib_write4(uint32_t *p, size_t n) { calib_write<uint32_t>(p, n); }
__global__ void k_calib_write1(uint8_t *p, size_t n) { calib_write<uint8_t>(p, n); }

int main(int argc, char **argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : (size_t)1493 << 20) & ~(size_t)63;
  uint8_t *p, *o;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&o, 64) != hipSuccess) return 1;
  (void)hipMemset(p, 1, bytes);
  for (int it = 0; it < 3; it++) {
    k_calib_read8<<<4096, 256>>>((const uint64_t *)p, bytes / 8, (uint64_t *)o);
    k_calib_read4<<<4096, 256>>>((const uint32_t *)p, bytes / 4, (uint32_t *)o);
    k_calib_write4<<<4096, 256>>>((uint32_t *)p, bytes / 4);
    k_calib_write1<<<4096, 256>>>(p, bytes);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("calib bytes_per_launch %zu\n", bytes);
  return 0;
}
