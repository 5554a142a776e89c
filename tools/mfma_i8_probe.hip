// Probe (tool): the A/B operand lane maps of v_mfma_i32_16x16x64_i8 on gfx950, checked with
// random int8 matrices against a host product.  C/D: col = lane & 15, row = 4 (lane >> 4) + i
// (cdna_hip_programming.md: dtype-independent).  Hypotheses for the 16 int8 elements j of lane l:
//   H0: k = 16 (l >> 4) + j
//   H1: k = 8 (l >> 4) + j for j < 8, 32 + 8 (l >> 4) + (j - 8) for j >= 8
// usage: hipcc --offload-arch=gfx950 -O2 -o /tmp/probe tools/mfma_i8_probe.hip && /tmp/probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef int v4i __attribute__((ext_vector_type(4)));

__global__ void k_probe(const int8_t *A, const int8_t *B, int *D, int hyp) {
  const int l = threadIdx.x;
  int8_t a[16], b[16];
  for (int j = 0; j < 16; j++) {
    const int k = hyp == 0 ? 16 * (l >> 4) + j : (j < 8 ? 8 * (l >> 4) + j : 32 + 8 * (l >> 4) + (j - 8));
    a[j] = A[(l & 15) * 64 + k];
    b[j] = B[k * 16 + (l & 15)];
  }
  v4i av, bv;
  __builtin_memcpy(&av, a, 16);
  __builtin_memcpy(&bv, b, 16);
  v4i c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
  for (int i = 0; i < 4; i++) D[(4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}

int main() {
  int8_t hA[16 * 64], hB[64 * 16];
  srand(7);
  for (int i = 0; i < 16 * 64; i++) hA[i] = (int8_t)(rand() % 256 - 128);
  for (int i = 0; i < 64 * 16; i++) hB[i] = (int8_t)(rand() % 256 - 128);
  int ref[256];
  for (int r = 0; r < 16; r++)
    for (int c = 0; c < 16; c++) {
      int s = 0;
      for (int k = 0; k < 64; k++) s += hA[r * 64 + k] * hB[k * 16 + c];
      ref[r * 16 + c] = s;
    }
  int8_t *dA, *dB;
  int *dD;
  if (hipMalloc(&dA, sizeof hA) || hipMalloc(&dB, sizeof hB) || hipMalloc(&dD, 256 * sizeof(int))) return 2;
  hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice);
  hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
  for (int hyp = 0; hyp < 2; hyp++) {
    int hD[256];
    k_probe<<<1, 64>>>(dA, dB, dD, hyp);
    if (hipDeviceSynchronize()) return 3;
    hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 256; i++) bad += hD[i] != ref[i];
    printf("hypothesis H%d: %d of 256 outputs differ\n", hyp, bad);
  }
  return 0;
}
