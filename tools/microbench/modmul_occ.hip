// Modmul throughput vs occupancy (waves/SIMD), 1 or 2 independent fe_mul
// chains per thread.  Occupancy is limited by dynamic LDS per workgroup.
#include "../../stark-pure-rust_amd/csrc/fp_dev.h"
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"
using namespace stark;
#define ITERS 128
template <int CH>
__global__ __launch_bounds__(256) void k(fe* out, fe a0) {
  extern __shared__ int pad[];
  fe a[CH], b;
  b = a0; b.w[1] ^= threadIdx.x;
#pragma unroll
  for (int c = 0; c < CH; ++c) { a[c] = a0; a[c].w[0] += threadIdx.x + 17 * c; }
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) a[c] = fe_mul(a[c], b);
  }
  fe r = a[0];
#pragma unroll
  for (int c = 1; c < CH; ++c) r = fe_add(r, a[c]);
  if (threadIdx.x == 0 && r.w[0] == 0x12345) pad[0] = 1;
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int CH>
void run(fe* out, fe a0, int waves_per_simd) {
  // 256-thread WG = 4 waves = 1 wave per SIMD; WGs per CU = waves_per_simd
  size_t lds = (160 * 1024) / waves_per_simd - 64;
  if (lds > 65536) lds = 65536;
  hipFuncSetAttribute((const void*)k<CH>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  const int blocks = 256 * waves_per_simd * 8;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(256), lds, 0, out, a0); hipDeviceSynchronize();
  hipEventRecord(e0);
  hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(256), lds, 0, out, a0);
  hipLaunchKernelGGL(k<CH>, dim3(blocks), dim3(256), lds, 0, out, a0);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 2;
  double muls = (double)blocks * 256 * ITERS * CH;
  printf("chains=%d waves/SIMD<=%d lds=%zu: %.2f Gmodmul/s\n", CH, waves_per_simd, lds, muls / ms / 1e6);
}
int main() {
  fe* out; hipMalloc(&out, (size_t)256 * 8 * 8 * 256 * sizeof(fe));
  fe a0; for (int i = 0; i < 8; i++) a0.w[i] = 0x12345678u * (i + 1); a0.w[7] = 0x1234567;
  int occ[] = {1, 2, 3, 4, 5, 6, 8};
  for (int o : occ) run<1>(out, a0, o);
  for (int o : occ) run<2>(out, a0, o);
  for (int o : occ) run<4>(out, a0, o);
  return 0;
}
