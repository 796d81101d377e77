// Microbenchmark: sustained fe_mul (BN254 Montgomery, 8x32 limbs) throughput.
#include "../../stark-pure-rust_amd/csrc/fp_dev.h"
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"
#define ITERS 256
using namespace stark;
// Previous (compiler-scheduled CIOS) version, kept here only for A/B and cross-checking.
__device__ __forceinline__ fe fe_mul_cios(const fe& a, const fe& b) {
  uint32_t t[8];
  for (int i = 0; i < 8; i++) t[i] = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t bi = b.w[i];
    uint64_t A = (uint64_t)a.w[0] * bi + t[0];
    t[0] = (uint32_t)A;
    const uint32_t m = t[0] * STARK_PINV32;
    uint64_t C = (uint64_t)m * STARK_P0 + t[0];
#pragma unroll
    for (int j = 1; j < 8; j++) {
      A = (uint64_t)a.w[j] * bi + t[j] + (A >> 32);
      t[j] = (uint32_t)A;
      C = (uint64_t)m * p_limb(j) + t[j] + (C >> 32);
      t[j - 1] = (uint32_t)C;
    }
    t[7] = (uint32_t)(C >> 32) + (uint32_t)(A >> 32);
  }
  fe r;
  for (int i = 0; i < 8; i++) r.w[i] = t[i];
  fe_reduce_once(r);
  return r;
}
__global__ void k_check(int* bad, const fe* x, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe a = x[i], b = x[(i * 7 + 3) % n];
  fe u = fe_mul(a, b), v = fe_mul_cios(a, b);
  for (int k = 0; k < 8; k++) if (u.w[k] != v.w[k]) atomicAdd(bad, 1);
}
__global__ void k_modmul_cios(fe* out, fe a0) {
  fe a = a0, b = a0, c = a0, d = a0;
  a.w[0] += threadIdx.x; b.w[1] += threadIdx.x; c.w[2] += blockIdx.x; d.w[3] += threadIdx.x * 3;
  for (int i = 0; i < ITERS; ++i) { a = fe_mul_cios(a, b); c = fe_mul_cios(c, d); }
  out[blockIdx.x * blockDim.x + threadIdx.x] = fe_add(a, c);
}
__global__ void k_modmul(fe* out, fe a0) {
  fe a = a0, b = a0, c = a0, d = a0;
  a.w[0] += threadIdx.x; b.w[1] += threadIdx.x; c.w[2] += blockIdx.x; d.w[3] += threadIdx.x * 3;
  for (int i = 0; i < ITERS; ++i) {
    a = fe_mul(a, b);
    c = fe_mul(c, d);
  }
  fe r = fe_add(a, c);
  out[blockIdx.x * blockDim.x + threadIdx.x] = r;
}
int main() {
  const int blocks = 256 * 16, threads = 256;
  fe* out; hipMalloc(&out, (size_t)blocks * threads * sizeof(fe));
  fe a0; for (int i = 0; i < 8; i++) a0.w[i] = 0x12345678u * (i + 1); a0.w[7] = 0x1234567;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  k_modmul<<<blocks, threads>>>(out, a0); hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) k_modmul<<<blocks, threads>>>(out, a0);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
  double muls = (double)blocks * threads * ITERS * 2;
  printf("fe_mul (FIPS asm): %.3f ms, %.2f Gmodmul/s\n", ms, muls / ms / 1e6);
  hipEventRecord(e0);
  for (int r = 0; r < 5; r++) k_modmul_cios<<<blocks, threads>>>(out, a0);
  hipEventRecord(e1); hipEventSynchronize(e1);
  hipEventElapsedTime(&ms, e0, e1); ms /= 5;
  printf("fe_mul (CIOS C++): %.3f ms, %.2f Gmodmul/s\n", ms, muls / ms / 1e6);
  // cross-check on pseudo-random canonical inputs (top limb < 0x30000000 keeps them < p)
  const int n = 1 << 20;
  fe* h = (fe*)malloc(sizeof(fe) * n);
  uint64_t st = 88172645463325252ull;
  for (int i = 0; i < n; i++) for (int k = 0; k < 8; k++) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; h[i].w[k] = (uint32_t)st; }
  for (int i = 0; i < n; i++) h[i].w[7] &= 0x2fffffff;
  fe* dx; hipMalloc(&dx, sizeof(fe) * n); hipMemcpy(dx, h, sizeof(fe) * n, hipMemcpyHostToDevice);
  int* dbad; hipMalloc(&dbad, 4); hipMemset(dbad, 0, 4);
  k_check<<<n / 256, 256>>>(dbad, dx, n);
  int bad = -1; hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
  printf("FIPS vs CIOS mismatches: %d / %d\n", bad, n);
  return 0;
}
