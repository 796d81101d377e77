// Digit-basis constant product (fe_mul_db) vs the Shoup product (fe_mul_shoup):
//   check: reads db_in.bin (n x [a (8 u32), W table (72 u32)], made by tools/db_check.py) and
//          writes db_out.bin (n x fe_mul_db(a, W));
//   rate:  G products/s with the constants in LDS (128 constants, four lanes per constant as in the
//          NTT's radix steps) at 2 and 4 waves per SIMD, and with wave-uniform constants.
#include "../../stark-pure-rust_amd/csrc/fe_db.h"

#include <cstdio>
#include <vector>
using namespace stark;

__global__ void check_k(const uint32_t* in, fe* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t* rec = in + 80 * (size_t)i;
  fe a;
  for (int k = 0; k < 8; ++k) a.w[k] = rec[k];
  out[i] = fe_mul_db(a, rec + 8);
}

#define ITERS 128
#define NCONST 128
// V = 0: digit basis, LDS constants; 1: Shoup, LDS (w, w') pairs; 2: digit basis, uniform constant;
// 3: digit basis, LDS constants, two independent chains (as the NTT's t1/t3 pairs); 4: Shoup, two chains.
template <int V>
__global__ __launch_bounds__(256) void rate_k(fe* out, const uint32_t* tabs, const fe* pairs, fe a0) {
  __shared__ __attribute__((aligned(16))) uint32_t lw[NCONST * 72];
  __shared__ fe lp[NCONST * 2];
  for (int k = threadIdx.x; k < NCONST * 72; k += 256) lw[k] = tabs[k];
  for (int k = threadIdx.x; k < NCONST * 2; k += 256) lp[k] = pairs[k];
  __syncthreads();
  fe a = a0, b = a0;
  a.w[0] += threadIdx.x;
  b.w[1] ^= threadIdx.x;
  const uint32_t g = threadIdx.x >> 2;
  for (int i = 0; i < ITERS; ++i) {
    const uint32_t c = (g + (uint32_t)i) & (NCONST - 1);
    const uint32_t* tw = (const uint32_t*)__builtin_assume_aligned(lw + 72 * c, 16);
    if (V == 0) a = fe_mul_db(a, tw);
    if (V == 1) a = fe_mul_shoup(a, lp[2 * c], lp[2 * c + 1]);
    if (V == 2) a = fe_mul_db(a, lw + 72 * ((uint32_t)i & (NCONST - 1)));
    if (V == 3 && (i & 1) == 0) {
      a = fe_mul_db(a, tw);
      b = fe_mul_db(b, tw);
    }
    if (V == 4 && (i & 1) == 0) {
      a = fe_mul_shoup(a, lp[2 * c], lp[2 * c + 1]);
      b = fe_mul_shoup(b, lp[2 * c], lp[2 * c + 1]);
    }
  }
  if (V >= 3) a = fe_add(a, b);
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}

template <int V>
void rate(fe* out, const uint32_t* tabs, const fe* pairs, fe a0, int waves) {
  const int blocks = 256 * waves;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(rate_k<V>, dim3(blocks), dim3(256), 0, 0, out, tabs, pairs, a0);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(rate_k<V>, dim3(blocks), dim3(256), 0, 0, out, tabs, pairs, a0);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  static const char* names[] = {"db/lds", "shoup/lds", "db/uniform", "db/lds x2", "shoup/lds x2"};
  printf("%-11s waves/SIMD %d: %.2f G products/s\n", names[V], waves, (double)blocks * 256 * ITERS / ms / 1e6);
}

int main(int argc, char** argv) {
  const char* inp = argc > 1 ? argv[1] : "db_in.bin";
  const char* outp = argc > 2 ? argv[2] : "db_out.bin";
  FILE* f = fopen(inp, "rb");
  if (!f) {
    printf("no %s\n", inp);
    return 1;
  }
  fseek(f, 0, SEEK_END);
  const long bytes = ftell(f);
  fseek(f, 0, SEEK_SET);
  const int n = (int)(bytes / (80 * 4));
  std::vector<uint32_t> h(80 * (size_t)n);
  if (fread(h.data(), 4, h.size(), f) != h.size()) return 1;
  fclose(f);
  uint32_t* din;
  fe* dout;
  (void)hipMalloc(&din, h.size() * 4);
  const size_t out_elems = (size_t)256 * 8 * 256 > (size_t)n ? (size_t)256 * 8 * 256 : (size_t)n;
  (void)hipMalloc(&dout, out_elems * sizeof(fe));
  (void)hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(check_k, dim3((n + 255) / 256), dim3(256), 0, 0, din, dout, n);
  std::vector<fe> o(n);
  (void)hipMemcpy(o.data(), dout, (size_t)n * sizeof(fe), hipMemcpyDeviceToHost);
  FILE* g = fopen(outp, "wb");
  fwrite(o.data(), sizeof(fe), o.size(), g);
  fclose(g);
  printf("checked %d products -> %s\n", n, outp);
  // Rate inputs: the first NCONST tables; Shoup pairs are arbitrary (rate only).
  std::vector<uint32_t> tabs(NCONST * 72);
  for (int c = 0; c < NCONST; ++c)
    for (int k = 0; k < 72; ++k) tabs[72 * c + k] = h[80 * (size_t)(c % n) + 8 + k];
  std::vector<fe> pairs(NCONST * 2);
  for (int c = 0; c < 2 * NCONST; ++c)
    for (int k = 0; k < 8; ++k) pairs[c].w[k] = h[80 * (size_t)(c % n) + 8 + k] | (k == 7 ? 0 : 0x80000000u);
  uint32_t* dtabs;
  fe* dpairs;
  (void)hipMalloc(&dtabs, tabs.size() * 4);
  (void)hipMalloc(&dpairs, pairs.size() * sizeof(fe));
  (void)hipMemcpy(dtabs, tabs.data(), tabs.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dpairs, pairs.data(), pairs.size() * sizeof(fe), hipMemcpyHostToDevice);
  fe a0;
  for (int k = 0; k < 8; ++k) a0.w[k] = h[k];
  for (int w : {2, 4, 8}) {
    rate<0>(dout, dtabs, dpairs, a0, w);
    rate<1>(dout, dtabs, dpairs, a0, w);
    rate<2>(dout, dtabs, dpairs, a0, w);
    rate<3>(dout, dtabs, dpairs, a0, w);
    rate<4>(dout, dtabs, dpairs, a0, w);
  }
  return 0;
}
