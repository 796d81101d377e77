#include "/root/repo/stark-pure-rust_amd/csrc/fp_dev.h"
#include <cstdio>
using namespace stark;
struct fe29 { uint32_t l[9]; };
// Shoup product by a constant in radix 2^29 (tools/gen_fe29_asm.py): r = a*w mod p in [0, 3p).
__device__ __forceinline__ fe29 fe29_mul_shoup(const fe29& a, const fe29& w, const fe29& wq) {
  fe29 r;
  uint32_t q0, q1, q2, q3, q4, q5, q6, q7, q8;
  const uint32_t N0 = 0x0fffffffu, N1 = 0x00f05360u, N2 = 0x11a3dbafu, N3 = 0x182f6f0cu, N4 = 0x0a7a2d7cu, N5 = 0x1d24bf3fu, N6 = 0x1f591ebeu, N7 = 0x11a3d9cbu, N8 = 0x1fcf9bb1u;
  asm("v_mad_u64_u32 v[2:3], s[100:101], %18, %43, 0\n\tv_mad_u64_u32 v[2:3], s[100:101], %19, %42, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %20, %41, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %21, %40, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %22, %39, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %23, %38, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %24, %37, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %25, %36, v[2:3]\n\tv_lshrrev_b64 v[0:1], 29, v[2:3]\n\tv_mad_u64_u32 v[0:1], s[100:101], %18, %44, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %19, %43, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %20, %42, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %21, %41, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %22, %40, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %23, %39, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %24, %38, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %25, %37, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %26, %36, v[0:1]\n\tv_lshrrev_b64 v[2:3], 29, v[0:1]\n\tv_mad_u64_u32 v[2:3], s[100:101], %19, %44, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %20, %43, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %21, %42, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %22, %41, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %23, %40, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %24, %39, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %25, %38, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %26, %37, v[2:3]\n\tv_lshrrev_b64 v[0:1], 29, v[2:3]\n\tv_and_b32 %9, 0x1fffffff, v2\n\tv_mad_u64_u32 v[0:1], s[100:101], %20, %44, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %21, %43, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %22, %42, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %23, %41, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %24, %40, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %25, %39, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %26, %38, v[0:1]\n\tv_lshrrev_b64 v[2:3], 29, v[0:1]\n\tv_and_b32 %10, 0x1fffffff, v0\n\tv_mad_u64_u32 v[2:3], s[100:101], %21, %44, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %22, %43, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %23, %42, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %24, %41, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %25, %40, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %26, %39, v[2:3]\n\tv_lshrrev_b64 v[0:1], 29, v[2:3]\n\tv_and_b32 %11, 0x1fffffff, v2\n\tv_mad_u64_u32 v[0:1], s[100:101], %22, %44, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %23, %43, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %24, %42, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %25, %41, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %26, %40, v[0:1]\n\tv_lshrrev_b64 v[2:3], 29, v[0:1]\n\tv_and_b32 %12, 0x1fffffff, v0\n\tv_mad_u64_u32 v[2:3], s[100:101], %23, %44, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %24, %43, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %25, %42, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %26, %41, v[2:3]\n\tv_lshrrev_b64 v[0:1], 29, v[2:3]\n\tv_and_b32 %13, 0x1fffffff, v2\n\tv_mad_u64_u32 v[0:1], s[100:101], %24, %44, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %25, %43, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %26, %42, v[0:1]\n\tv_lshrrev_b64 v[2:3], 29, v[0:1]\n\tv_and_b32 %14, 0x1fffffff, v0\n\tv_mad_u64_u32 v[2:3], s[100:101], %25, %44, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %26, %43, v[2:3]\n\tv_lshrrev_b64 v[0:1], 29, v[2:3]\n\tv_and_b32 %15, 0x1fffffff, v2\n\tv_mad_u64_u32 v[0:1], s[100:101], %26, %44, v[0:1]\n\tv_lshrrev_b64 v[2:3], 29, v[0:1]\n\tv_and_b32 %16, 0x1fffffff, v0\n\tv_mov_b32 %17, v2\n\tv_mad_u64_u32 v[0:1], s[100:101], %18, %27, 0\n\tv_mad_u64_u32 v[0:1], s[100:101], %9, %45, v[0:1]\n\tv_lshrrev_b64 v[2:3], 29, v[0:1]\n\tv_and_b32 %0, 0x1fffffff, v0\n\tv_mad_u64_u32 v[2:3], s[100:101], %18, %28, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %19, %27, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %9, %46, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %10, %45, v[2:3]\n\tv_lshrrev_b64 v[0:1], 29, v[2:3]\n\tv_and_b32 %1, 0x1fffffff, v2\n\tv_mad_u64_u32 v[0:1], s[100:101], %18, %29, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %19, %28, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %20, %27, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %9, %47, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %10, %46, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %11, %45, v[0:1]\n\tv_lshrrev_b64 v[2:3], 29, v[0:1]\n\tv_and_b32 %2, 0x1fffffff, v0\n\tv_mad_u64_u32 v[2:3], s[100:101], %18, %30, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %19, %29, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %20, %28, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %21, %27, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %9, %48, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %10, %47, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %11, %46, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %12, %45, v[2:3]\n\tv_lshrrev_b64 v[0:1], 29, v[2:3]\n\tv_and_b32 %3, 0x1fffffff, v2\n\tv_mad_u64_u32 v[0:1], s[100:101], %18, %31, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %19, %30, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %20, %29, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %21, %28, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %22, %27, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %9, %49, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %10, %48, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %11, %47, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %12, %46, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %13, %45, v[0:1]\n\tv_lshrrev_b64 v[2:3], 29, v[0:1]\n\tv_and_b32 %4, 0x1fffffff, v0\n\tv_mad_u64_u32 v[2:3], s[100:101], %18, %32, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %19, %31, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %20, %30, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %21, %29, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %22, %28, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %23, %27, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %9, %50, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %10, %49, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %11, %48, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %12, %47, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %13, %46, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %14, %45, v[2:3]\n\tv_lshrrev_b64 v[0:1], 29, v[2:3]\n\tv_and_b32 %5, 0x1fffffff, v2\n\tv_mad_u64_u32 v[0:1], s[100:101], %18, %33, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %19, %32, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %20, %31, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %21, %30, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %22, %29, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %23, %28, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %24, %27, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %9, %51, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %10, %50, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %11, %49, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %12, %48, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %13, %47, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %14, %46, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %15, %45, v[0:1]\n\tv_lshrrev_b64 v[2:3], 29, v[0:1]\n\tv_and_b32 %6, 0x1fffffff, v0\n\tv_mad_u64_u32 v[2:3], s[100:101], %18, %34, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %19, %33, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %20, %32, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %21, %31, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %22, %30, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %23, %29, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %24, %28, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %25, %27, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %9, %52, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %10, %51, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %11, %50, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %12, %49, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %13, %48, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %14, %47, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %15, %46, v[2:3]\n\tv_mad_u64_u32 v[2:3], s[100:101], %16, %45, v[2:3]\n\tv_lshrrev_b64 v[0:1], 29, v[2:3]\n\tv_and_b32 %7, 0x1fffffff, v2\n\tv_mad_u64_u32 v[0:1], s[100:101], %18, %35, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %19, %34, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %20, %33, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %21, %32, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %22, %31, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %23, %30, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %24, %29, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %25, %28, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %26, %27, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %9, %53, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %10, %52, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %11, %51, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %12, %50, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %13, %49, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %14, %48, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %15, %47, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %16, %46, v[0:1]\n\tv_mad_u64_u32 v[0:1], s[100:101], %17, %45, v[0:1]\n\tv_and_b32 %8, 0x1fffffff, v0"
      : "=&v"(r.l[0]), "=&v"(r.l[1]), "=&v"(r.l[2]), "=&v"(r.l[3]), "=&v"(r.l[4]), "=&v"(r.l[5]), "=&v"(r.l[6]), "=&v"(r.l[7]), "=&v"(r.l[8]), "=&v"(q0), "=&v"(q1), "=&v"(q2), "=&v"(q3), "=&v"(q4), "=&v"(q5), "=&v"(q6), "=&v"(q7), "=&v"(q8)
      : "v"(a.l[0]), "v"(a.l[1]), "v"(a.l[2]), "v"(a.l[3]), "v"(a.l[4]), "v"(a.l[5]), "v"(a.l[6]), "v"(a.l[7]), "v"(a.l[8]), "v"(w.l[0]), "v"(w.l[1]), "v"(w.l[2]), "v"(w.l[3]), "v"(w.l[4]), "v"(w.l[5]), "v"(w.l[6]), "v"(w.l[7]), "v"(w.l[8]), "v"(wq.l[0]), "v"(wq.l[1]), "v"(wq.l[2]), "v"(wq.l[3]), "v"(wq.l[4]), "v"(wq.l[5]), "v"(wq.l[6]), "v"(wq.l[7]), "v"(wq.l[8]),
        "s"(N0), "s"(N1), "s"(N2), "s"(N3), "s"(N4), "s"(N5), "s"(N6), "s"(N7), "s"(N8)
      : "v0", "v1", "v2", "v3", "s100", "s101");
  return r;
}

#define ITERS 256
__constant__ uint32_t W29[9] = {0x117fd374, 0x1e0f51b7, 0x8cc954f, 0xc82714c, 0x16a3b0d4, 0x1446f350, 0x3d8a09d, 0xbe39f62, 0x17cb76};
__constant__ uint32_t WQ29[9] = {0xd92a14, 0x128a5ac6, 0x14340a91, 0x1b76bc7b, 0x1460f49c, 0x5790422, 0x13e6453b, 0x184628f2, 0xfbc1800};
__constant__ uint32_t W32[8] = {0xf17fd374, 0x3fc1ea36, 0xa6233255, 0xd464138, 0xe6a16a3b, 0x2827688d, 0x1cfb10f6, 0x17cb765f};
__constant__ uint32_t WQ32[8] = {0xc606c950, 0x52328a5a, 0xf1ee8681, 0x7a4e6dda, 0x90422a30, 0xcc8a7657, 0x118a3ca7, 0x7de0c006};
template <int V, int CH>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  fe29 a[CH], w, wq; fe b[CH], w2, wq2;
  for (int i = 0; i < 9; ++i) { w.l[i] = W29[i]; wq.l[i] = WQ29[i]; }
  for (int i = 0; i < 8; ++i) { w2.w[i] = W32[i]; wq2.w[i] = WQ32[i]; }
  for (int c = 0; c < CH; ++c) {
    for (int i = 0; i < 9; ++i) a[c].l[i] = (seed * (i + 1) + threadIdx.x * 77 + c) & 0x1fffffff;
    for (int i = 0; i < 8; ++i) b[c].w[i] = seed * (i + 3) + threadIdx.x + c;
    b[c].w[7] &= 0x0fffffff;
  }
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      if (V == 0) a[c] = fe29_mul_shoup(a[c], w, wq);
      else b[c] = fe_mul_shoup(b[c], w2, wq2);
    }
  }
  uint32_t x = 0;
  for (int c = 0; c < CH; ++c) { for (int i = 0; i < 9; ++i) x ^= a[c].l[i]; for (int i = 0; i < 8; ++i) x ^= b[c].w[i]; }
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
}
// correctness: one product per thread, written out
__global__ void chk(const uint32_t* in, uint32_t* out) {
  fe29 a, w, wq;
  for (int i = 0; i < 9; ++i) { a.l[i] = in[threadIdx.x * 9 + i]; w.l[i] = W29[i]; wq.l[i] = WQ29[i]; }
  fe29 r = fe29_mul_shoup(a, w, wq);
  for (int i = 0; i < 9; ++i) out[threadIdx.x * 9 + i] = r.l[i];
}
template <int V, int CH>
void run(uint32_t* out, int waves) {
  const int blocks = 256 * waves;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipLaunchKernelGGL((k<V, CH>), dim3(blocks), dim3(256), 0, 0, out, 3u);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL((k<V, CH>), dim3(blocks), dim3(256), 0, 0, out, 3u);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
  printf("%-8s chains %d waves/SIMD %d: %.2f G products/s\n", V ? "shoup32" : "shoup29", CH, waves, (double)blocks * 256 * ITERS * CH / ms / 1e6);
}
int main() {
  uint32_t* out; hipMalloc(&out, 256 * 16 * 256 * 4 * 9);
  static uint32_t h[256 * 9];
  FILE* f = fopen(getenv("MB_IN"), "rb"); if (f) { fread(h, 4, 256 * 9, f); fclose(f); }
  uint32_t* din; hipMalloc(&din, sizeof h); hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(chk, dim3(1), dim3(256), 0, 0, din, out);
  hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
  f = fopen(getenv("MB_OUT"), "wb"); fwrite(h, 4, 256 * 9, f); fclose(f);
  for (int w : {3, 4, 8}) { run<0, 1>(out, w); run<0, 2>(out, w); run<1, 1>(out, w); run<1, 2>(out, w); }
  return 0;
}
