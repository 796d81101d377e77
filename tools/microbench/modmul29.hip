// fe29_mul (radix 2^29, no carry ops) vs fe_mul (radix 2^32 FIPS asm):
// throughput and a cross-check through the radix conversions.
#include "fp29_dev.h"
#include <cstdio>
#pragma clang diagnostic ignored "-Wunused-result"
using namespace stark;
#define ITERS 128
template <int V>
__global__ __launch_bounds__(256) void k(fe* out, fe a0, const Kp29Table* kp) {
  fe a[2], b = a0; b.w[1] ^= threadIdx.x;
  for (int c = 0; c < 2; ++c) { a[c] = a0; a[c].w[0] += threadIdx.x + 17 * c; }
  if (V == 0) {
    for (int i = 0; i < ITERS; ++i)
      for (int c = 0; c < 2; ++c) a[c] = fe_mul(a[c], b);
    out[blockIdx.x * blockDim.x + threadIdx.x] = fe_add(a[0], a[1]);
  } else {
    fe29 x[2], y = fe29_from_fe(b);
    for (int c = 0; c < 2; ++c) x[c] = fe29_from_fe(a[c]);
    for (int i = 0; i < ITERS; ++i)
      for (int c = 0; c < 2; ++c) x[c] = fe29_mul(x[c], y);
    out[blockIdx.x * blockDim.x + threadIdx.x] = fe29_canonical(fe29_add(x[0], x[1]), kp);
  }
}
// check: canonical(fe29_mul(A29, B29)) * 2^261 == A*B (mod p) via fe_mul:
// fe_mul(a, b) = a b 2^-256; fe29 path gives a b 2^-261 -> multiply by 2^5 * ... compare
// canonical(fe29_mul(a,b)) against fe_mul(fe_mul(a,b), c) with c = 2^-5 * 2^256 (Montgomery image of 2^-5).
__global__ void kcheck(int* bad, const fe* x, int n, fe c, const Kp29Table* kp) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe a = x[i], b = x[(i * 7 + 3) % n];
  fe u = fe29_canonical(fe29_mul(fe29_from_fe(a), fe29_from_fe(b)), kp);
  fe v = fe_mul(fe_mul(a, b), c);
  for (int q = 0; q < 8; q++) if (u.w[q] != v.w[q]) { atomicAdd(bad, 1); break; }
}
template <int V> void run(fe* out, fe a0, const char* name, const Kp29Table* kp) {
  const int blocks = 256 * 32;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, out, a0, kp); hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 3; r++) hipLaunchKernelGGL(k<V>, dim3(blocks), dim3(256), 0, 0, out, a0, kp);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 3;
  printf("%s: %.2f Gmodmul/s\n", name, (double)blocks * 256 * ITERS * 2 / ms / 1e6);
}
int main(int argc, char** argv) {
  fe* out; hipMalloc(&out, (size_t)256 * 32 * 256 * sizeof(fe));
  fe a0; for (int i = 0; i < 8; i++) a0.w[i] = 0x12345678u * (i + 1); a0.w[7] = 0x1234567;
  // kp table: q p in radix 2^29 (host, __int128 arithmetic)
  Kp29Table hk;
  const unsigned __int128 P_LO = ((unsigned __int128)0x2833e84879b97091ull << 64) | 0x43e1f593f0000001ull;
  const unsigned __int128 P_HI = ((unsigned __int128)0x30644e72e131a029ull << 64) | 0xb85045b68181585dull;
  for (int q = 0; q < 32; q++) {
    // q*p as 320-bit little-endian bit vector, then 29-bit limbs
    unsigned __int128 lo = P_LO * q, c = 0;
    // hi part with carry from lo: compute via 64-bit pieces
    uint64_t w[5] = {0};
    uint64_t pw[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull, 0x30644e72e131a029ull};
    for (int i = 0; i < 4; i++) { unsigned __int128 t = (unsigned __int128)pw[i] * q + c; w[i] = (uint64_t)t; c = t >> 64; }
    w[4] = (uint64_t)c; (void)lo; (void)P_HI;
    for (int i = 0; i < 9; i++) {
      int bit = 29 * i; uint64_t v = 0;
      for (int b = 0; b < 29; b++) { int bb = bit + b; if (bb < 320 && ((w[bb / 64] >> (bb % 64)) & 1)) v |= 1ull << b; }
      hk.l[q][i] = (uint32_t)v;
    }
  }
  Kp29Table* kp; hipMalloc(&kp, sizeof(hk)); hipMemcpy(kp, &hk, sizeof(hk), hipMemcpyHostToDevice);
  run<0>(out, a0, "fe_mul   radix 2^32 (asm FIPS)", kp);
  run<1>(out, a0, "fe29_mul radix 2^29 (no carries)", kp);
  const int n = 1 << 20;
  fe* h = (fe*)malloc(sizeof(fe) * n);
  uint64_t st = 88172645463325252ull;
  for (int i = 0; i < n; i++) for (int q = 0; q < 8; q++) { st ^= st << 13; st ^= st >> 7; st ^= st << 17; h[i].w[q] = (uint32_t)st; }
  for (int i = 0; i < n; i++) h[i].w[7] &= 0x2fffffff;
  fe* dx; hipMalloc(&dx, sizeof(fe) * n); hipMemcpy(dx, h, sizeof(fe) * n, hipMemcpyHostToDevice);
  int* dbad; hipMalloc(&dbad, 4); hipMemset(dbad, 0, 4);
  fe c; // Montgomery image (R=2^256) of 2^-5 mod p, from argv as 8 hex words
  for (int q = 0; q < 8; q++) c.w[q] = (uint32_t)strtoul(argv[1 + q], 0, 16);
  kcheck<<<n / 256, 256>>>(dbad, dx, n, c, kp);
  int bad = -1; hipMemcpy(&bad, dbad, 4, hipMemcpyDeviceToHost);
  printf("fe29 vs fe mismatches: %d / %d\n", bad, n);
  return 0;
}
