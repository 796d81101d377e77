// fe29_mul variants under kernel-like conditions: ONE dependent product chain
// per thread, occupancy limited to 2-4 waves/SIMD by LDS.
#include "fp29_dev.h"
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"
using namespace stark;
#define ITERS 128
// two accumulators per column: a*b products and m*p products are independent chains
__device__ __forceinline__ fe29 fe29_mul2(const fe29& a, const fe29& b) {
  uint32_t m[9];
  fe29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    uint64_t accb = 0;
#pragma unroll
    for (int j = 0; j < k; ++j) {
      acc += (uint64_t)a.l[j] * b.l[k - j];
      accb += (uint64_t)m[j] * p29(k - j);
    }
    acc += (uint64_t)a.l[k] * b.l[0];
    acc += accb;
    const uint32_t t = (uint32_t)acc;
    m[k] = ((t << 28) - t) & kM29;
    acc += (uint64_t)m[k] * p29(0);
    acc >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; ++k) {
    uint64_t accb = 0;
#pragma unroll
    for (int j = k - 8; j < 9; ++j) {
      acc += (uint64_t)a.l[j] * b.l[k - j];
      accb += (uint64_t)m[j] * p29(k - j);
    }
    acc += accb;
    r.l[k - 9] = (uint32_t)acc & kM29;
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}
template <int V>
__global__ __launch_bounds__(256) void k(fe* out, fe a0) {
  extern __shared__ int pad[];
  fe29 y = fe29_from_fe(a0);
  fe b = a0; b.w[0] += threadIdx.x;
  fe29 x = fe29_from_fe(b);
  for (int i = 0; i < ITERS; ++i) x = V == 0 ? fe29_mul(x, y) : fe29_mul2(x, y);
  if (x.l[0] == 0x12345 && threadIdx.x == 0) pad[0] = 1;
  out[blockIdx.x * blockDim.x + threadIdx.x] = fe_from_fe29(x);
}
__global__ __launch_bounds__(256) void k32(fe* out, fe a0) {
  extern __shared__ int pad[];
  fe b = a0; b.w[0] += threadIdx.x;
  for (int i = 0; i < ITERS; ++i) b = fe_mul(b, a0);
  if (b.w[0] == 0x12345 && threadIdx.x == 0) pad[0] = 1;
  out[blockIdx.x * blockDim.x + threadIdx.x] = b;
}
template <typename K> void run(K kern, fe* out, fe a0, const char* name, int wps) {
  size_t lds = (160 * 1024) / wps - 64;
  if (lds > 65536) lds = 65536;
  hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const int blocks = 256 * wps * 8;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, out, a0); hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), lds, 0, out, a0);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
  printf("%-28s waves/SIMD=%d: %.2f Gmodmul/s\n", name, wps, (double)blocks * 256 * ITERS / ms / 1e6);
}
int main() {
  fe* out; hipMalloc(&out, (size_t)256 * 8 * 8 * 256 * sizeof(fe));
  fe a0; for (int i = 0; i < 8; i++) a0.w[i] = 0x12345678u * (i + 1); a0.w[7] = 0x1234567;
  for (int w : {2, 3, 4, 6}) {
    run(k<0>, out, a0, "fe29_mul (1 accumulator)", w);
    run(k<1>, out, a0, "fe29_mul2 (2 accumulators)", w);
    run(k32, out, a0, "fe_mul radix 2^32 asm", w);
  }
  return 0;
}
