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


__global__ void k_addc3(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < ITERS; i++) {
    asm volatile("v_addc_co_u32 %0, s[40:41], %0, 0, s[40:41]\n\tv_addc_co_u32 %1, s[42:43], %1, 0, s[42:43]\n\t"
                 "v_addc_co_u32 %2, s[44:45], %2, 0, s[44:45]\n\tv_addc_co_u32 %3, s[46:47], %3, 0, s[46:47]\n\t"
                 "v_addc_co_u32 %4, s[48:49], %4, 0, s[48:49]\n\tv_addc_co_u32 %5, s[50:51], %5, 0, s[50:51]\n\t"
                 "v_addc_co_u32 %6, s[52:53], %6, 0, s[52:53]\n\tv_addc_co_u32 %7, s[54:55], %7, 0, s[54:55]"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                 :: "s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_addco3(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
    asm volatile("v_add_co_u32 %0, s[40:41], %0, %8\n\tv_add_co_u32 %1, s[42:43], %1, %8\n\t"
                 "v_add_co_u32 %2, s[44:45], %2, %8\n\tv_add_co_u32 %3, s[46:47], %3, %8\n\t"
                 "v_add_co_u32 %4, s[48:49], %4, %8\n\tv_add_co_u32 %5, s[50:51], %5, %8\n\t"
                 "v_add_co_u32 %6, s[52:53], %6, %8\n\tv_add_co_u32 %7, s[54:55], %7, %8"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(y)
                 : "s40","s41","s42","s43","s44","s45","s46","s47","s48","s49","s50","s51","s52","s53","s54","s55");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_addc2vcc(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
    asm volatile("v_add_co_u32 %0, vcc, %0, %8\n\tv_addc_co_u32 %1, vcc, %1, %8, vcc\n\t"
                 "v_addc_co_u32 %2, vcc, %2, %8, vcc\n\tv_addc_co_u32 %3, vcc, %3, %8, vcc\n\t"
                 "v_addc_co_u32 %4, vcc, %4, %8, vcc\n\tv_addc_co_u32 %5, vcc, %5, %8, vcc\n\t"
                 "v_addc_co_u32 %6, vcc, %6, %8, vcc\n\tv_addc_co_u32 %7, vcc, %7, %8, vcc"
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(y) : "vcc");
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_alignbit(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_alignbit_b32 %0, %1, %0, 29" : "+v"(a##k) : "v"(y));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_cndmask(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(a##k) : "v"(y) : "s40", "s41");
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_mad_nodep(uint64_t* out, uint32_t s) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t x = s + threadIdx.x, y = s * 3 + 1;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_mad_u64_u32 %0, s[40:41], %1, %2, %0\n\tv_addc_co_u32 %3, s[40:41], %3, 0, s[40:41]" : "+v"(a##k) : "v"(x), "v"(y), "v"(x) : "s40", "s41");
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

typedef void (*kfn)(uint64_t*, uint32_t);
__global__ void k_perm(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1, z = s ^ 0x5555;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_xor(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1, z = s ^ 0x5555;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_add3(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1, z = s ^ 0x5555;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_lshlor(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1, z = s ^ 0x5555;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_lshl_or_b32 %0, %0, 7, %1" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_bitop3(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1, z = s ^ 0x5555;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_xad(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1, z = s ^ 0x5555;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_pkmov(uint64_t* out, uint32_t s) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1, z = s ^ 0x5555;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_pk_mov_b32 %0, %0, %0 op_sel:[1,0]" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_lshr64(uint64_t* out, uint32_t s) {
  uint64_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1, z = s ^ 0x5555;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_lshrrev_b64 %0, 32, %0" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_alignbyte(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1, z = s ^ 0x5555;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_alignbyte_b32 %0, %0, %0, 1" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_pkadd16(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1, z = s ^ 0x5555;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_pk_add_u16 %0, %0, 0 op_sel:[1,0] op_sel_hi:[0,1]" : "+v"(a##k) : "v"(y), "v"(z));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ void k_xorsdwa(uint64_t* out, uint32_t s) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t y = s * 3 + 1, z = s ^ 0x5555;
  for (int i = 0; i < ITERS; i++) {
#define M(k) asm volatile("v_xor_b32_sdwa %0, %0, %1 dst_sel:WORD_0 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1" : "+v"(a##k) : "v"(y));
    BODY8(M)
#undef M
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
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
  run("v_addc VOP3 sgpr", k_addc3, buf);
  run("v_add_co VOP3 sgpr", k_addco3, buf);
  run("add_co+addc vcc chain", k_addc2vcc, buf);
  run("v_alignbit_b32", k_alignbit, buf);
  run("v_cndmask_e64", k_cndmask, buf);
  run("v_perm_b32", k_perm, buf);
  run("v_xor_b32", k_xor, buf);
  run("v_add3_u32", k_add3, buf);
  run("v_lshl_or_b32", k_lshlor, buf);
  run("v_bitop3_b32", k_bitop3, buf);
  run("v_xad_u32", k_xad, buf);
  run("v_pk_mov_b32", k_pkmov, buf);
  run("v_lshrrev_b64", k_lshr64, buf);
  run("v_alignbyte_b32", k_alignbyte, buf);
  run("v_pk_add_u16 swap", k_pkadd16, buf);
  run("v_xor_b32_sdwa", k_xorsdwa, buf);
  return 0;
}
