// Per-instruction VALU throughput on gfx950 via inline asm (8 independent
// chains per wave, 4 waves/SIMD).  Reports cycles per wave64 instruction
// assuming 2.4 GHz (the clock under load may be lower).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang diagnostic ignored "-Wunused-result"
#define ITERS 2048
#define BODY8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

__global__ void k_mad64(uint64_t* out, uint32_t s) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t x = s + threadIdx.x, y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0" : "+v"(a##k) : "v"(x), "v"(y) : "s40", "s41");
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_lshladd(uint64_t* out, uint32_t s) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint64_t y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_lshl_add_u64 %0, %0, 0, %1" : "+v"(a##k) : "v"(y));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_addc(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_addc_co_u32 %0, vcc, %0, %1, vcc" : "+v"(a##k) : "v"(y) : "vcc");
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_mov(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_mov_b32 %0, %1" : "=v"(a##k) : "v"(y ^ a##k));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_add32(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a##k) : "v"(y));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_mullo(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(a##k) : "v"(y));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_fma64(uint64_t* out, uint32_t s) {
  double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  double y = s * 0.5, z = 0.25;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}
__global__ void k_mad_u32_u24(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(a##k) : "v"(y));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_pk_fma32(uint64_t* out, uint32_t s) {
  float2 a0 = make_float2(threadIdx.x, 1), a1 = a0, a2 = a0, a3 = a0, a4 = a0, a5 = a0, a6 = a0, a7 = a0;
  float2 y = make_float2(s * 0.5f, 0.5f), z = make_float2(0.25f, 0.1f);
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)(a0.x + a1.x + a2.y + a3.x + a4.x + a5.x + a6.x + a7.x);
}

typedef void (*kfn)(uint64_t*, uint32_t);
static void run(const char* name, kfn k, uint64_t* buf) {
  const int blocks = 256 * 4, threads = 1024;  // 16 waves per CU = 4 per SIMD
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, 7u); hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k, dim3(blocks), dim3(threads), 0, 0, buf, 7u);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
  double wave_instr = (double)blocks * (threads / 64) * ITERS * 8;
  double simd_cycles = ms * 1e-3 * 2.4e9 * 256 * 4;
  printf("%-16s %.3f ms  %.2f cycles/wave-instr/SIMD (at 2.4GHz)  %.2f T lane-ops/s\n", name, ms,
         simd_cycles / wave_instr, wave_instr * 64 / (ms * 1e-3) / 1e12);
}
int main() {
  uint64_t* buf; hipMalloc(&buf, 256 * 4 * 1024 * 8);
  run("v_mad_u64_u32", k_mad64, buf);
  run("v_lshl_add_u64", k_lshladd, buf);
  run("v_addc_co_u32", k_addc, buf);
  run("v_mov_b32", k_mov, buf);
  run("v_add_u32", k_add32, buf);
  run("v_mul_lo_u32", k_mullo, buf);
  run("v_fma_f64", k_fma64, buf);
  run("v_mad_u32_u24", k_mad_u32_u24, buf);
  run("v_pk_fma_f32", k_pk_fma32, buf);
  return 0;
}
