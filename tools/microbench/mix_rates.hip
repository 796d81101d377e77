// Issue cost of MIXED VALU streams on gfx950 (cycles per wave64 instruction, 1024 SIMDs; the clock
// is read from s_memtime / s_memrealtime inside the kernel, so the cycle figures are real cycles):
//   xor            8 independent v_xor_b32 chains
//   alignbit       8 independent v_alignbit_b32 chains
//   xor+alignbit   alternating, 8 chains (each chain: xor then rotate of its result)
//   blake G        the Blake2s G function, 4 independent G per step (one compression's column step)
//   blake G x2     two compressions interleaved (8 independent G)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>
#define ITERS 1024

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }

#define G(a, b, c, d, x, y)   \
  a = a + b + x;              \
  d = rotr(d ^ a, 16);        \
  c = c + d;                  \
  b = rotr(b ^ c, 12);        \
  a = a + b + y;              \
  d = rotr(d ^ a, 8);         \
  c = c + d;                  \
  b = rotr(b ^ c, 7);

template <int V>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t s, unsigned long long* clk) {
  uint32_t v[16], u[16];
  for (int i = 0; i < 16; ++i) {
    v[i] = s * (i + 1) + threadIdx.x;
    u[i] = v[i] ^ 0x9e3779b9u;
  }
  const uint32_t x = s ^ threadIdx.x, y = s + 7;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < ITERS; ++it) {
    if (V == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[i]) : "v"(x));
    } else if (V == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(v[i]));
    } else if (V == 2) {
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(v[i]) : "v"(x));
#pragma unroll
      for (int i = 0; i < 8; ++i) asm volatile("v_alignbit_b32 %0, %0, %0, 7" : "+v"(v[i]));
    } else if (V == 3) {
      G(v[0], v[4], v[8], v[12], x, y) G(v[1], v[5], v[9], v[13], y, x)
      G(v[2], v[6], v[10], v[14], x, x) G(v[3], v[7], v[11], v[15], y, y)
    } else {
      G(v[0], v[4], v[8], v[12], x, y) G(v[1], v[5], v[9], v[13], y, x)
      G(v[2], v[6], v[10], v[14], x, x) G(v[3], v[7], v[11], v[15], y, y)
      G(u[0], u[4], u[8], u[12], x, y) G(u[1], u[5], u[9], u[13], y, x)
      G(u[2], u[6], u[10], u[14], x, x) G(u[3], u[7], u[11], u[15], y, y)
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t acc = 0;
  for (int i = 0; i < 16; ++i) acc ^= v[i] ^ u[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    clk[0] = t1 - t0;
    clk[1] = r1 - r0;
  }
}

template <int V>
void run(const char* name, int per_iter, uint32_t* out, unsigned long long* clk, int waves) {
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
  const double ghz = (double)h[0] / ((double)h[1] / 100e6) / 1e9;  // s_memrealtime runs at 100 MHz
  const double instr = (double)blocks * 4 * ITERS * per_iter;  // wave-instructions
  const double cyc = ms * 1e-3 * ghz * 1e9 * 1024;
  printf("%-14s waves/SIMD %d: %.2f cycles per wave64 instr (clock %.2f GHz)\n", name, waves, cyc / instr, ghz);
}

int main() {
  uint32_t* out;
  unsigned long long* clk;
  (void)hipMalloc(&out, 256 * 8 * 256 * 4);
  (void)hipMalloc(&clk, 16);
  for (int w : {4, 8}) {
    run<0>("xor", 8, out, clk, w);
    run<1>("alignbit", 8, out, clk, w);
    run<2>("xor+alignbit", 16, out, clk, w);
    run<3>("blake G", 4 * 12, out, clk, w);
    run<4>("blake G x2", 8 * 12, out, clk, w);
  }
  return 0;
}
