// Memory-only floor of the NTT pass access patterns: each workgroup moves a
// [R][B] tile of 32-B elements: reads in[j + r n/R] (B adjacent columns j),
// writes out[(j/Ns) Ns R + j%Ns + r Ns] -- the Stockham pass pattern -- with
// no arithmetic.  Compared with a contiguous float4 copy.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#pragma clang diagnostic ignored "-Wunused-result"
struct el { uint4 a, b; };
template <int LOG_R>
__global__ __launch_bounds__(256) void pass_copy(const el* __restrict__ in, el* __restrict__ out, uint32_t log_n,
                                                 uint32_t log_ns, uint32_t log_b) {
  const uint32_t B = 1u << log_b, E = B << LOG_R, T = blockDim.x;
  const size_t j0 = (size_t)blockIdx.x << log_b;
  const uint32_t log_cols = log_n - LOG_R;
  const size_t ns_mask = ((size_t)1 << log_ns) - 1;
  for (uint32_t e = threadIdx.x; e < E; e += T) {
    const uint32_t b = e & (B - 1), r = e >> log_b;
    const size_t j = j0 + b;
    el v = in[j + ((size_t)r << log_cols)];
    size_t dst;
    if (((size_t)1 << log_ns) >= B) dst = ((j >> log_ns) << (log_ns + LOG_R)) + (j & ns_mask) + ((size_t)r << log_ns);
    else dst = (j0 << LOG_R) + e;  // (layout of the Ns < B case is a permutation of the same run)
    out[dst] = v;
  }
}
__global__ void copy4(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n4) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) out[i] = in[i];
}
int main() {
  const uint32_t log_n = 24;
  const size_t n = (size_t)1 << log_n;
  el *a, *b; hipMalloc(&a, n * 32); hipMalloc(&b, n * 32); hipMemset(a, 1, n * 32);
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1); float ms;
  auto time = [&](auto f) { f(); hipDeviceSynchronize(); hipEventRecord(e0); for (int i = 0; i < 10; i++) f(); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms, e0, e1); return ms / 10; };
  float t = time([&] { copy4<<<256 * 8, 256>>>((const uint4*)a, (uint4*)b, n * 2); });
  printf("contiguous copy 512 MiB: %.3f ms  %.2f TB/s\n", t, 2.0 * n * 32 / t / 1e9);
  for (uint32_t lb : {2, 3, 4}) {
    for (uint32_t ns : {0u, 8u, 16u}) {
      const uint32_t E = 1u << (8 + lb);
      const uint32_t T = E / 4 < 256 ? E / 4 : 256;
      t = time([&] { pass_copy<8><<<(unsigned)(n >> (8 + lb)), T>>>(a, b, log_n, ns, lb); });
      printf("R=256 B=%u Ns=2^%u: %.3f ms  %.2f TB/s\n", 1u << lb, ns, t, 2.0 * n * 32 / t / 1e9);
    }
  }
  return 0;
}
