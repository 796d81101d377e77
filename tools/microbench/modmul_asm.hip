// fe_mul (per-product asm, fp_dev.h) vs fe_mul_lazy (one asm block,
// fe_mul_asm.h) throughput, 2 independent chains per thread.
#include "../../stark-pure-rust_amd/csrc/fp_dev.h"

#include <cstdio>
using namespace stark;
#define ITERS 128
template <int V, int CH>
__global__ __launch_bounds__(256) void k(fe* out, fe a0) {
  fe a[CH], b;
  b = a0; b.w[1] ^= threadIdx.x;
#pragma unroll
  for (int c = 0; c < CH; ++c) { a[c] = a0; a[c].w[0] += threadIdx.x + 17 * c; }
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if (V == 0) a[c] = fe_mul(a[c], b);
      if (V == 1) { a[c] = fe_mul_lazy(a[c], b); fe_reduce_once(a[c]); }
      if (V == 2) a[c] = fe_mul_lazy(a[c], b);
    }
  }
  fe r = a[0];
#pragma unroll
  for (int c = 1; c < CH; ++c) r = fe_add(r, a[c]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int V, int CH>
float run(fe* out, fe a0) {
  const int blocks = 256 * 8 * 4;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((k<V, CH>), dim3(blocks), dim3(256), 0, 0, out, a0); hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k<V, CH>), dim3(blocks), dim3(256), 0, 0, out, a0);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
  double muls = (double)blocks * 256 * ITERS * CH;
  printf("variant %d chains %d: %.2f Gmodmul/s\n", V, CH, muls / ms / 1e6);
  return ms;
}
int main() {
  fe* out; hipMalloc(&out, (size_t)256 * 8 * 4 * 256 * sizeof(fe));
  fe a0; for (int i = 0; i < 8; i++) a0.w[i] = 0x12345678u * (i + 1); a0.w[7] = 0x1234567;
  // correctness: variants 0 and 1 must agree
  fe* o2; hipMalloc(&o2, (size_t)256 * 8 * 4 * 256 * sizeof(fe));
  hipLaunchKernelGGL((k<0, 1>), dim3(64), dim3(256), 0, 0, out, a0);
  hipLaunchKernelGGL((k<1, 1>), dim3(64), dim3(256), 0, 0, o2, a0);
  static fe h1[64 * 256], h2[64 * 256];
  hipMemcpy(h1, out, sizeof h1, hipMemcpyDeviceToHost); hipMemcpy(h2, o2, sizeof h2, hipMemcpyDeviceToHost);
  int bad = 0; for (int i = 0; i < 64 * 256; ++i) for (int j = 0; j < 8; ++j) bad += h1[i].w[j] != h2[i].w[j];
  printf("mismatches: %d\n", bad);
  run<0, 1>(out, a0); run<1, 1>(out, a0); run<2, 1>(out, a0);
  run<0, 2>(out, a0); run<1, 2>(out, a0); run<2, 2>(out, a0);
  return 0;
}
