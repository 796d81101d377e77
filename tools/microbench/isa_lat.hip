// Throughput of VOP3 integer ops with 16 independent chains per wave and
// 8 waves/SIMD, to separate issue rate from dependent latency.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang diagnostic ignored "-Wunused-result"
#define ITERS 1024
#define B16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)
#define DECL(k) uint32_t a##k = threadIdx.x + k;
#define XOR(k) ^ a##k
#define KERN(name, INSTR)                                                            \
  __global__ __launch_bounds__(1024) void name(uint64_t* out, uint32_t s) {          \
    B16(DECL) uint32_t y = s * 3 + 1;                                                \
    for (int i = 0; i < ITERS; i++) {                                                \
      B16(INSTR)                                                                     \
    }                                                                                \
    out[blockIdx.x * blockDim.x + threadIdx.x] = 0 B16(XOR);                         \
  }
#define I_ALIGN(k) asm volatile("v_alignbit_b32 %0, %1, %0, 29" : "+v"(a##k) : "v"(y));
#define I_MULLO(k) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##k) : "v"(y));
#define I_ADD(k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##k) : "v"(y));
#define I_ADDCO(k) asm volatile("v_add_co_u32 %0, s[40:41], %0, %1" : "+v"(a##k) : "v"(y) : "s40", "s41");
#define I_ADDC(k) asm volatile("v_addc_co_u32 %0, s[40:41], %0, 0, s[40:41]" : "+v"(a##k) :: "s40", "s41");
#define I_AND(k) asm volatile("v_and_b32 %0, %0, %1" : "+v"(a##k) : "v"(y));
#define I_LSHR(k) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(a##k));
#define I_ADD3(k) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(a##k) : "v"(y));
#define I_BFE(k) asm volatile("v_bfe_u32 %0, %0, 3, 29" : "+v"(a##k));
#define I_CND(k) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(a##k) : "v"(y) : "s40", "s41");
#define I_ADDE64(k) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a##k) : "v"(y));
KERN(k_align, I_ALIGN) KERN(k_mullo, I_MULLO) KERN(k_add, I_ADD) KERN(k_addco, I_ADDCO) KERN(k_addc, I_ADDC)
KERN(k_and, I_AND) KERN(k_lshr, I_LSHR) KERN(k_add3, I_ADD3) KERN(k_bfe, I_BFE) KERN(k_cnd, I_CND) KERN(k_adde64, I_ADDE64)
__global__ __launch_bounds__(1024) void k_mad(uint64_t* out, uint32_t s) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint64_t a8 = threadIdx.x, a9 = a0 + 1, a10 = a0 + 2, a11 = a0 + 3, a12 = a0 + 4, a13 = a0 + 5, a14 = a0 + 6, a15 = a0 + 7;
  uint32_t x = s + threadIdx.x, y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(a##k) : "v"(x), "v"(y) : "s40", "s41");
    B16(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7 ^ a8 ^ a9 ^ a10 ^ a11 ^ a12 ^ a13 ^ a14 ^ a15;
}
typedef void (*kfn)(uint64_t*, uint32_t);
static void run(const char* name, kfn k, uint64_t* buf) {
  const int blocks = 256 * 2, threads = 1024;  // 32 waves per CU = 8 per SIMD
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, 7u); hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, 7u);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
  double wave_instr = (double)blocks * (threads / 64) * ITERS * 16;
  printf("%-22s %.2f cycles/wave-instr/SIMD at 2.4GHz\n", name, ms * 1e-3 * 2.4e9 * 1024 / wave_instr);
}
int main() {
  uint64_t* buf; hipMalloc(&buf, 256 * 2 * 1024 * 8);
  run("v_add_u32 (e32)", k_add, buf); run("v_add_u32_e64", k_adde64, buf); run("v_and_b32", k_and, buf);
  run("v_lshrrev_b32", k_lshr, buf); run("v_add3_u32", k_add3, buf); run("v_bfe_u32", k_bfe, buf);
  run("v_alignbit_b32", k_align, buf); run("v_mul_lo_u32", k_mullo, buf); run("v_add_co_u32 sdst", k_addco, buf);
  run("v_addc_co_u32 sdst", k_addc, buf); run("v_cndmask_b32_e64", k_cnd, buf); run("v_mad_u64_u32", k_mad, buf);
  return 0;
}
