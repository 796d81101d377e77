// A/B of the Montgomery product's carry form (tools/gen_fe_mul_asm.py):
//   sgpr: carry-outs in an allocated SGPR pair, every counting v_addc_co_u32 is VOP3 (8 bytes)
//   vcc : carry-outs in VCC, the counting v_addc_co_u32 is VOP2 (e32, 4 bytes)
// Both must give identical limbs; throughput in G products/s at 4 and 8 waves per SIMD.
#include "../../stark-pure-rust_amd/csrc/fp_dev.h"

#include <cstdio>
using namespace stark;
#define ITERS 256
template <int V, int CH>
__global__ __launch_bounds__(256) void k(fe* out, fe a0) {
  fe a[CH], b;
  b = a0;
  b.w[1] ^= threadIdx.x;
  b.w[7] &= 0x0fffffff;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    a[c] = a0;
    a[c].w[0] += threadIdx.x + 17 * c;
  }
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if (V == 0) a[c] = fe_mul_lazy(a[c], b);
      if (V == 1) a[c] = fe_mul_lazy_vcc(a[c], b);
      if (V == 2 && (c & 1)) fe_mul_lazy2(a[c - 1], a[c], a[c - 1], b, a[c], b);
    }
  }
  fe r = a[0];
#pragma unroll
  for (int c = 1; c < CH; ++c) r = fe_add(r, a[c]);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
template <int V, int CH>
void run(fe* out, fe a0, int waves_per_simd) {
  const int blocks = 256 * waves_per_simd;  // 256 threads = 4 waves = 1 per SIMD
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipLaunchKernelGGL((k<V, CH>), dim3(blocks), dim3(256), 0, 0, out, a0);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<V, CH>), dim3(blocks), dim3(256), 0, 0, out, a0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  double muls = (double)blocks * 256 * ITERS * CH;
  printf("%-5s chains %d waves/SIMD %d: %.2f G products/s\n", V == 2 ? "dual" : V ? "vcc" : "sgpr", CH, waves_per_simd,
         muls / ms / 1e6);
}
int main() {
  const size_t cnt = (size_t)256 * 16 * 256;
  fe *out, *o2;
  hipMalloc(&out, cnt * sizeof(fe));
  hipMalloc(&o2, cnt * sizeof(fe));
  fe a0;
  for (int i = 0; i < 8; i++) a0.w[i] = 0x12345678u * (i + 1);
  a0.w[7] = 0x1234567;
  hipLaunchKernelGGL((k<0, 2>), dim3(256), dim3(256), 0, 0, out, a0);
  hipLaunchKernelGGL((k<1, 2>), dim3(256), dim3(256), 0, 0, o2, a0);
  static fe h1[256 * 256], h2[256 * 256];
  hipMemcpy(h1, out, sizeof h1, hipMemcpyDeviceToHost);
  hipMemcpy(h2, o2, sizeof h2, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int i = 0; i < 256 * 256; ++i)
    for (int j = 0; j < 8; ++j) bad += h1[i].w[j] != h2[i].w[j];
  printf("mismatches sgpr vs vcc: %d\n", bad);
  hipLaunchKernelGGL((k<2, 2>), dim3(256), dim3(256), 0, 0, o2, a0);
  hipMemcpy(h2, o2, sizeof h2, hipMemcpyDeviceToHost);
  bad = 0;
  for (int i = 0; i < 256 * 256; ++i)
    for (int j = 0; j < 8; ++j) bad += h1[i].w[j] != h2[i].w[j];
  printf("mismatches sgpr vs dual: %d\n", bad);
  for (int w : {4, 8}) {
    run<0, 1>(out, a0, w);
    run<1, 1>(out, a0, w);
    run<0, 2>(out, a0, w);
    run<1, 2>(out, a0, w);
    run<2, 2>(out, a0, w);
    run<2, 4>(out, a0, w);
  }
  return 0;
}
