// Do cheap VALU instructions (v_mov_b32, v_add_u32, v_xor_b32) cost issue cycles when they are
// interleaved with the slow VOP3 ones (v_mad_u64_u32, v_addc_co_u32)?  Each test runs 8 independent
// chains per kind; cycles per wave64 instruction of the SLOW kind are reported (clock from
// s_memtime / s_memrealtime inside the kernel), so "mad+mov" at the "mad" figure means the moves
// were free.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#define ITERS 512

template <int V>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t s, unsigned long long* clk) {
  uint64_t acc[8];
  uint32_t m[8], x[8];
  for (int i = 0; i < 8; ++i) {
    acc[i] = (uint64_t)(s * (i + 3) + threadIdx.x) << 7;
    m[i] = s ^ (i * 0x9e3779b9u) ^ threadIdx.x;
    x[i] = m[i] + 1;
  }
  const uint32_t y = s | 1u;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (V == 0 || V == 1 || V == 2 || V == 3 || V == 6) {
        uint64_t c;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[i]), "=s"(c) : "v"(m[i]), "v"(y));
      }
      if (V == 1) asm volatile("v_mov_b32 %0, %1" : "=v"(x[i]) : "v"(m[(i + 1) & 7]));
      if (V == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
      if (V == 3) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[i]) : "v"(y));
      if (V == 4 || V == 5 || V == 6) {
        uint64_t c;
        asm volatile("v_add_co_u32 %0, %1, %0, %2\n\tv_addc_co_u32 %0, %1, %0, 0, %1"
                     : "+v"(x[i]), "=&s"(c)
                     : "v"(y));
      }
      if (V == 5) asm volatile("v_mov_b32 %0, %1" : "=v"(m[i]) : "v"(x[(i + 3) & 7]));
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t a = 0;
  for (int i = 0; i < 8; ++i) a ^= (uint32_t)acc[i] ^ (uint32_t)(acc[i] >> 32) ^ x[i] ^ m[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

// slow: slow wave64 instructions per chain per iteration; cheap: cheap ones
template <int V>
void run(const char* name, int slow, int cheap, uint32_t* out, unsigned long long* clk, int waves) {
  const int blocks = 256 * waves;
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, out, 3u, clk);
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, out, 3u, clk);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  unsigned long long h[2];
  (void)hipMemcpy(h, clk, sizeof h, hipMemcpyDeviceToHost);
  const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;  // s_memrealtime: 100 MHz
  const double per = (double)blocks * 4 * ITERS * 8;               // wave-iterations x chains
  const double cyc = ms * 1e-3 * ghz * 1e9 * 1024;
  printf("%-14s waves/SIMD %d: %.2f cycles per slow instr, %.2f per instr (clock %.2f GHz)\n", name, waves,
         cyc / (per * slow), cyc / (per * (slow + cheap)), ghz);
}

int main() {
  uint32_t* out;
  unsigned long long* clk;
  (void)hipMalloc(&out, 256 * 8 * 256 * 4);
  (void)hipMalloc(&clk, 16);
  for (int w : {4, 8}) {
    run<0>("mad", 1, 0, out, clk, w);
    run<1>("mad+mov", 1, 1, out, clk, w);
    run<2>("mad+add_u32", 1, 1, out, clk, w);
    run<3>("mad+xor", 1, 1, out, clk, w);
    run<4>("addco+addc", 2, 0, out, clk, w);
    run<5>("addco+addc+mov", 2, 1, out, clk, w);
    run<6>("mad+addco+addc", 3, 0, out, clk, w);
  }
  return 0;
}
