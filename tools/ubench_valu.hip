// VALU issue-rate microbenchmark for the instructions a k_encode redesign would lean on.
// Each kernel runs 8 independent accumulator chains x ITERS iterations of one instruction
// per thread; prints cycles per wave-instruction per SIMD (at the measured clock of
// s_memtime vs wall time is not attempted: reports ns and instr/ns per SIMD).
//   hipcc --offload-arch=gfx950 -O3 -o ubench_valu tools/ubench_valu.hip && ./ubench_valu
#include <hip/hip_runtime.h>
#include <stdio.h>

#define ITERS 4096

#define BODY8(INS)                                                                        \
  asm volatile(INS INS INS INS INS INS INS INS : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3),  \
               "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(x), "v"(y), "s"(s));

// each INS string uses %0..%7 through a macro per chain
#define K(NAME, TEMPLATE)                                                                  \
  __global__ void NAME(int *out, int seed) {                                               \
    int a0 = seed + threadIdx.x, a1 = a0 ^ 3, a2 = a0 * 5, a3 = a0 + 7, a4 = a0 ^ 11,      \
        a5 = a0 * 13, a6 = a0 + 17, a7 = a0 ^ 19;                                          \
    int x = seed * 3 + 1, y = seed ^ 0x55, s = seed + 9;                                   \
    for (int i = 0; i < ITERS; i++) {                                                      \
      asm volatile(TEMPLATE(0) TEMPLATE(1) TEMPLATE(2) TEMPLATE(3) TEMPLATE(4) TEMPLATE(5) \
                       TEMPLATE(6) TEMPLATE(7)                                             \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                     "+v"(a7)                                                              \
                   : "v"(x), "v"(y), "s"(s));                                              \
    }                                                                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;    \
  }

#define T0(i) "v_add_u32 %" #i ", %8, %" #i "\n"
K(k0, T0)
#define T1(i) "v_add_u32 %" #i ", %10, %" #i "\n"
K(k1, T1)
#define T2(i) "v_sub_u32 %" #i ", %8, %" #i "\n"
K(k2, T2)
#define T3(i) "v_and_b32 %" #i ", %8, %" #i "\n"
K(k3, T3)
#define T4(i) "v_or_b32 %" #i ", %8, %" #i "\n"
K(k4, T4)
#define T5(i) "v_xor_b32 %" #i ", %8, %" #i "\n"
K(k5, T5)
#define T6(i) "v_lshlrev_b32 %" #i ", 3, %" #i "\n"
K(k6, T6)
#define T7(i) "v_lshrrev_b32 %" #i ", 3, %" #i "\n"
K(k7, T7)
#define T8(i) "v_ashrrev_i32 %" #i ", 9, %" #i "\n"
K(k8, T8)
#define T9(i) "v_min_i32 %" #i ", %8, %" #i "\n"
K(k9, T9)
#define T10(i) "v_max_u32 %" #i ", %8, %" #i "\n"
K(k10, T10)
#define T11(i) "v_cndmask_b32 %" #i ", %8, %" #i ", vcc\n"
K(k11, T11)
#define T12(i) "v_mov_b32 %" #i ", %8\n"
K(k12, T12)
#define T13(i) "v_mul_i32_i24 %" #i ", %8, %" #i "\n"
K(k13, T13)
#define T14(i) "v_mul_u32_u24 %" #i ", %8, %" #i "\n"
K(k14, T14)
#define T15(i) "v_mad_i32_i24 %" #i ", %8, %9, %" #i "\n"
K(k15, T15)
#define T16(i) "v_mad_u32_u24 %" #i ", %8, %9, %" #i "\n"
K(k16, T16)
#define T17(i) "v_mul_lo_u32 %" #i ", %8, %" #i "\n"
K(k17, T17)
#define T18(i) "v_add3_u32 %" #i ", %8, %9, %" #i "\n"
K(k18, T18)
#define T19(i) "v_lshl_add_u32 %" #i ", %8, 3, %" #i "\n"
K(k19, T19)
#define T20(i) "v_add_lshl_u32 %" #i ", %8, %" #i ", 3\n"
K(k20, T20)
#define T21(i) "v_lshl_or_b32 %" #i ", %8, 3, %" #i "\n"
K(k21, T21)
#define T22(i) "v_and_or_b32 %" #i ", %8, %9, %" #i "\n"
K(k22, T22)
#define T23(i) "v_or3_b32 %" #i ", %8, %9, %" #i "\n"
K(k23, T23)
#define T24(i) "v_bfe_u32 %" #i ", %" #i ", 8, 8\n"
K(k24, T24)
#define T25(i) "v_bfi_b32 %" #i ", %8, %9, %" #i "\n"
K(k25, T25)
#define T26(i) "v_perm_b32 %" #i ", %8, %" #i ", %9\n"
K(k26, T26)
#define T27(i) "v_alignbit_b32 %" #i ", %8, %" #i ", 9\n"
K(k27, T27)
#define T28(i) "v_med3_i32 %" #i ", %" #i ", 0, %8\n"
K(k28, T28)
#define T29(i) "v_ffbh_u32 %" #i ", %" #i "\n"
K(k29, T29)
#define T30(i) "v_dot2_i32_i16 %" #i ", %8, %9, %" #i "\n"
K(k30, T30)
#define T31(i) "v_dot2c_i32_i16 %" #i ", %8, %9\n"
K(k31, T31)
#define T32(i) "v_pk_add_u16 %" #i ", %8, %" #i "\n"
K(k32, T32)
#define T33(i) "v_pk_mad_u16 %" #i ", %8, %9, %" #i "\n"
K(k33, T33)
#define T34(i) "v_pk_min_u16 %" #i ", %8, %" #i "\n"
K(k34, T34)
#define T35(i) "v_ashrrev_i32_sdwa %" #i ", 9, %8 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:DWORD src1_sel:DWORD\n"
K(k35, T35)
#define T36(i) "v_add_u32_sdwa %" #i ", %8, %" #i " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:BYTE_1 src1_sel:DWORD\n"
K(k36, T36)
#define T37(i) "v_add_u32_dpp %" #i ", %8, %" #i " row_shr:1 row_mask:0xf bank_mask:0xf\n"
K(k37, T37)
#define T38(i) "v_cvt_f32_ubyte1 %" #i ", %" #i "\n"
K(k38, T38)
#define T39(i) "v_fmac_f32 %" #i ", %8, %9\n"
K(k39, T39)
#define T40(i) "v_fma_f32 %" #i ", %8, %9, %" #i "\n"
K(k40, T40)
#define T41(i) "v_cvt_pk_i16_i32 %" #i ", %8, %" #i "\n"
K(k41, T41)

#define T42(i) "v_cvt_flr_i32_f32 %" #i ", %" #i "\n"
K(k42, T42)
#define T43(i) "v_cvt_i32_f32 %" #i ", %" #i "\n"
K(k43, T43)
#define T44(i) "v_floor_f32 %" #i ", %" #i "\n"
K(k44, T44)
#define T45(i) "v_med3_f32 %" #i ", %" #i ", %8, %9\n"
K(k45, T45)
#define T46(i) "v_add_f32 %" #i ", %8, %" #i "\n"
K(k46, T46)
#define T47(i) "v_mul_f32 %" #i ", %8, %" #i "\n"
K(k47, T47)
#define T48(i) "v_cvt_f32_i32 %" #i ", %" #i "\n"
K(k48, T48)
#define T49(i) "v_pk_sub_u16 %" #i ", %8, %" #i " clamp\n"
K(k49, T49)
#define T50(i) "v_pk_lshrrev_b16 %" #i ", 3, %" #i "\n"
K(k50, T50)
#define T51(i) "v_sub_co_u32 %" #i ", vcc, %8, %" #i "\n"
K(k51, T51)
#define T52(i) "v_addc_co_u32 %" #i ", vcc, %" #i ", %" #i ", vcc\n"
K(k52, T52)
#define T53(i) "v_mul_hi_u32 %" #i ", %8, %" #i "\n"
K(k53, T53)
#define T54(i) "v_max3_i32 %" #i ", %8, %9, %" #i "\n"
K(k54, T54)
#define T55(i) "v_mad_u32_u16 %" #i ", %8, %9, %" #i "\n"
K(k55, T55)
#define T56(i) "v_cvt_f32_ubyte0_sdwa %" #i ", %8 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD\n"
K(k56, T56)

#define T57(i) "v_cmp_gt_i32 vcc, %8, %" #i "\nv_cndmask_b32 %" #i ", %8, %" #i ", vcc\n"
K(k57, T57)
#define T58(i) "v_cmp_gt_i32 vcc, %8, %" #i "\n"
K(k58, T58)
#define T59(i) "v_cndmask_b32_e64 %" #i ", %8, %" #i ", s[20:21]\n"
K(k59, T59)
#define T60(i) "v_cmp_gt_i32 s[20:21], %8, %" #i "\nv_cndmask_b32_e64 %" #i ", %8, %" #i ", s[20:21]\n"
K(k60, T60)
#define T61(i) "v_sad_u32 %" #i ", %8, %9, %" #i "\n"
K(k61, T61)
#define T62(i) "v_max_f32 %" #i ", %8, %" #i "\n"
K(k62, T62)
#define T63(i) "v_subrev_u32 %" #i ", %8, %" #i "\n"
K(k63, T63)
#define T64(i) "v_sub_f32 %" #i ", %8, %" #i "\n"
K(k64, T64)
#define T65(i) "v_add_u32 %" #i ", 0x4b400000, %" #i "\n"
K(k65, T65)
#define T67(i) "v_mul_f32 %" #i ", 0x3f800001, %" #i "\n"
K(k67, T67)
#define T68(i) "v_add_f32 %" #i ", 0x4b400000, %" #i "\n"
K(k68, T68)
#define T70(i) "v_bitop3_b32 %" #i ", %8, %9, %" #i " bitop3:0xf8\n"
K(k70, T70)
#define T71(i) "v_lshl_add_u64 %" #i ", %8, 0, %" #i "\n"
#define T69(i) "v_add_u32 %" #i ", %" #i ", %" #i "\n"
K(k69, T69)

// LDS LUT lookup throughput: 256-byte table, per-lane random byte index (conflict-free)
__global__ void lut_u8(int *out, int seed) {
  __shared__ unsigned char lut[256];
  __shared__ float flut[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) { lut[i] = (unsigned char)(i * 7); flut[i] = i; }
  __syncthreads();
  unsigned a[8];
  for (int j = 0; j < 8; j++) a[j] = (seed + threadIdx.x * 13 + j * 29) & 255;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) a[j] = lut[a[j]];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a[0] + a[1] + a[2] + a[3] + a[4] + a[5] + a[6] + a[7];
}
__global__ void lut_f32(int *out, int seed) {
  __shared__ float flut[256];
  for (int i = threadIdx.x; i < 256; i += blockDim.x) flut[i] = (float)((i * 7) & 255);
  __syncthreads();
  unsigned a[8];
  for (int j = 0; j < 8; j++) a[j] = (seed + threadIdx.x * 13 + j * 29) & 255;
  for (int i = 0; i < ITERS; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) a[j] = (unsigned)flut[a[j]];
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a[0] + a[1] + a[2] + a[3] + a[4] + a[5] + a[6] + a[7];
}

// 64-bit (register-pair) chains for packed fp32 and 64-bit shifts
#define K64(NAME, TEMPLATE)                                                                \
  __global__ void NAME(int *out, int seed) {                                               \
    long long a0 = seed + threadIdx.x, a1 = a0 ^ 3, a2 = a0 * 5, a3 = a0 + 7, a4 = a0 ^ 11,\
        a5 = a0 * 13, a6 = a0 + 17, a7 = a0 ^ 19;                                          \
    long long x = seed * 3 + 1, y = seed ^ 0x55;                                           \
    for (int i = 0; i < ITERS; i++) {                                                      \
      asm volatile(TEMPLATE(0) TEMPLATE(1) TEMPLATE(2) TEMPLATE(3) TEMPLATE(4) TEMPLATE(5) \
                       TEMPLATE(6) TEMPLATE(7)                                             \
                   : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                     "+v"(a7)                                                              \
                   : "v"(x), "v"(y));                                                      \
    }                                                                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = (int)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7); \
  }
#define P0(i) "v_pk_fma_f32 %" #i ", %8, %9, %" #i "\n"
K64(q0, P0)
#define P1(i) "v_pk_add_f32 %" #i ", %8, %" #i "\n"
K64(q1, P1)
#define P2(i) "v_pk_mul_f32 %" #i ", %8, %" #i "\n"
K64(q2, P2)
#define P3(i) "v_lshlrev_b64 %" #i ", 3, %" #i "\n"
K64(q3, P3)
#define P4(i) "v_pk_mov_b32 %" #i ", %8, %" #i " op_sel:[1,0]\n"
K64(q4, P4)

// clamp semantics of v_pk_mad_i16: is the saturation applied to the full product?
__global__ void clamp_probe(int *out) {
  int r;
  const int a = (200 << 16) | 255, b = (149 << 16) | 149, c = (0xffff & -1000) | ((0xffff & -1000) << 16);
  asm volatile("v_pk_mad_i16 %0, %1, %2, %3 clamp" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  if (threadIdx.x == 0) out[0] = r;
}

typedef void (*kfn)(int *, int);

int main() {
  int dev = 0, ncu = 0;
  hipDeviceProp_t p;
  (void)hipGetDeviceProperties(&p, dev);
  ncu = p.multiProcessorCount;
  const int wg = 256, waves_per_simd = 8;
  const int grid = ncu * waves_per_simd;  // 256-thread WGs: 4 waves -> 1 per SIMD each
  int *out;
  (void)hipMalloc(&out, (size_t)grid * wg * 4);
  struct {
    const char *name;
    kfn f;
  } ks[] = {{"v_add_u32", k0},
{"v_add_u32_sgpr", k1},
{"v_sub_u32", k2},
{"v_and_b32", k3},
{"v_or_b32", k4},
{"v_xor_b32", k5},
{"v_lshlrev_b32", k6},
{"v_lshrrev_b32", k7},
{"v_ashrrev_i32", k8},
{"v_min_i32", k9},
{"v_max_u32", k10},
{"v_cndmask_b32", k11},
{"v_mov_b32", k12},
{"v_mul_i32_i24", k13},
{"v_mul_u32_u24", k14},
{"v_mad_i32_i24", k15},
{"v_mad_u32_u24", k16},
{"v_mul_lo_u32", k17},
{"v_add3_u32", k18},
{"v_lshl_add_u32", k19},
{"v_add_lshl_u32", k20},
{"v_lshl_or_b32", k21},
{"v_and_or_b32", k22},
{"v_or3_b32", k23},
{"v_bfe_u32", k24},
{"v_bfi_b32", k25},
{"v_perm_b32", k26},
{"v_alignbit_b32", k27},
{"v_med3_i32", k28},
{"v_ffbh_u32", k29},
{"v_dot2_i32_i16", k30},
{"v_dot2c_i32_i16", k31},
{"v_pk_add_u16", k32},
{"v_pk_mad_u16", k33},
{"v_pk_min_u16", k34},
{"v_ashrrev_sdwa", k35},
{"v_add_u32_sdwa", k36},
{"v_add_u32_dpp", k37},
{"v_cvt_f32_ubyte1", k38},
{"v_fmac_f32", k39},
{"v_fma_f32", k40},
{"v_cvt_pk_i16_i32", k41},
{"v_cvt_flr_i32_f32", k42},
{"v_cvt_i32_f32", k43},
{"v_floor_f32", k44},
{"v_med3_f32", k45},
{"v_add_f32", k46},
{"v_mul_f32", k47},
{"v_cvt_f32_i32", k48},
{"v_pk_sub_u16_clamp", k49},
{"v_pk_lshrrev_b16", k50},
{"v_sub_co_u32", k51},
{"v_addc_co_u32", k52},
{"v_mul_hi_u32", k53},
{"v_max3_i32", k54},
{"v_mad_u32_u16", k55},
{"v_cvt_f32_ubyte0_sdwa", k56},
{"cmp+cndmask(vcc) pair", k57},
{"v_cmp_gt_i32 (vcc)", k58},
{"v_cndmask_e64 s[20:21]", k59},
{"cmp+cndmask(s pair)", k60},
{"v_sad_u32", k61},
{"v_max_f32", k62},
{"v_subrev_u32", k63},
{"v_sub_f32", k64},
{"v_add_u32 literal", k65},
{"v_mul_f32 literal", k67},
{"v_add_f32 literal", k68},
{"v_add_u32 x+x", k69},
{"v_bitop3_b32", k70},
{"lds lut u8 (per lookup)", lut_u8},
{"lds lut f32 (per lookup, +cvt)", lut_f32},
{"v_pk_fma_f32", q0},
{"v_pk_add_f32", q1},
{"v_pk_mul_f32", q2},
{"v_lshlrev_b64", q3},
{"v_pk_mov_b32", q4}};
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  printf("CUs %d, clock %d kHz, grid %d x %d\n", ncu, p.clockRate, grid, wg);
  for (auto &k : ks) {
    hipLaunchKernelGGL(k.f, dim3(grid), dim3(wg), 0, 0, out, 1);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0, 0);
    for (int r = 0; r < 5; r++) hipLaunchKernelGGL(k.f, dim3(grid), dim3(wg), 0, 0, out, r);
    (void)hipEventRecord(e1, 0);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double wave_instr = 5.0 * grid * (wg / 64) * (double)ITERS * 8;
    const double per_simd = wave_instr / (ncu * 4.0);
    const double ns = ms * 1e6;
    printf("%-18s %8.3f ms  %.3f wave-instr/ns/SIMD  (%.2f cyc @2.4GHz)\n", k.name, ms,
           per_simd / ns, 2.4 * ns / per_simd);
  }
  hipLaunchKernelGGL(clamp_probe, dim3(1), dim3(64), 0, 0, out);
  int r = 0;
  (void)hipMemcpy(&r, out, 4, hipMemcpyDeviceToHost);
  printf("v_pk_mad_i16 clamp probe: lo %d (255*149-1000=%d) hi %d (200*149-1000=%d)\n", (short)(r & 0xffff),
         255 * 149 - 1000, (short)(r >> 16), 200 * 149 - 1000);
  return 0;
}
