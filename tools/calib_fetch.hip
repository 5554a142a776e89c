// PMC calibration (perf tooling, not product): read a buffer of known size with
// 8-byte-per-lane fully coalesced loads, so FETCH_SIZE can be scaled to bytes for this
// access width on gfx950 (MI355X_MICROARCH.md: FETCH_SIZE is exact only when calibrated).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

__global__ void k_calib_read8(const uint64_t *__restrict__ p, size_t n, uint64_t *out) {
  uint64_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= p[i];
  if (acc == 0x9e3779b97f4a7c15ull) out[0] = acc;  // keep the loads live
}

int main(int argc, char **argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], 0, 10) : (size_t)1493 << 20);
  uint64_t *p, *o;
  if (hipMalloc(&p, bytes) != hipSuccess || hipMalloc(&o, 8) != hipSuccess) return 1;
  (void)hipMemset(p, 1, bytes);
  for (int it = 0; it < 3; it++) k_calib_read8<<<4096, 256>>>(p, bytes / 8, o);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("calib bytes_per_launch %zu\n", bytes);
  return 0;
}
