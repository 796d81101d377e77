// Constant product a * w mod p (BN254 Fr) with the column sums on the int8 matrix cores
// (v_mfma_i32_32x32x32_i8), against the digit-basis VALU product (csrc/fe_db.h) in the same binary.
//
// Form (tools/mfma_mul_check.py builds the constants): a = sum_i a_i 2^(8 i), 32 bytes; a_i' = a_i - 128
// (one XOR per word) is a signed byte.  W_i = w 2^(8 i) mod p is written in 32 balanced signed digits
// d_ij (sum_j d_ij 2^(8 j) = W_i, |d| <= 128).  Then
//   c_j = sum_i a_i' d_ij                  one MFMA: A[j][i] = d_ij (the constant), B[i][e] = a_i'(e)
//   S'  = sum_j c_j 2^(8 j) = sum_i a_i' W_i = a w - 128 sum_i W_i   (|c_j| <= 2^19)
//   T   = S' + K,  K = (128 sum_i W_i mod p) + 2^12 p  (so 0 <= T < 2^13 p + p)
//   r   = T - q p, q = floor(T / p) or one less from the top 64 bits in doubles -> r in [0, 2p).
// A wave multiplies 64 elements by one constant per step: two MFMAs (elements 0-31 and 32-63 of the
// wave's run are the B columns); lane l (half h = l >> 5) holds words 4h..4h+3 of element l & 31 of
// each run (the B operand layout) and gets back the column sums c_j, j = 8m + 4h + (0..3), of element
// l & 31 (C/D layout: col = lane & 31, row = (reg & 3) + 8 (reg >> 2) + 4 h).  The word-g partial sums
// t_g = c_4g + 2^8 c_4g+1, u_g = c_4g+2 + 2^8 c_4g+3 are exchanged between the halves with
// v_permlane32_swap so that lane l ends with all eight for ONE element (run h, column l & 31), the
// carry chain and reduction run once per element, and four more swaps rebuild the B layout for a
// chained product.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -mllvm -amdgpu-mfma-vgpr-form=1 mfma_mul.hip -o mfma_mul
// (the VGPR form of the MFMA: its results feed VALU code, so no v_accvgpr_read per column sum).
//   check: reads mfma_in.bin, writes mfma_out.bin: one product per element (and ITERS chained);
//   rate:  G products/s at 1, 2, 4 waves per SIMD for the MFMA form and for fe_mul_db (uniform constant
//          in LDS, the digit-basis product's best case), both chaining ITERS products per element.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "../../stark-pure-rust_amd/csrc/fe_db.h"
using namespace stark;

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

#define ITERS 256

struct MConst {
  int a[64][4];   // the A operand per lane: lane l holds d_ij for row j = l & 31, i = 16 (l >> 5) + byte
  uint32_t k[9];  // K
  uint32_t pad[3];
  double c224;    // 2^224 / p
  double margin;  // 2^-20
};

__device__ __forceinline__ void pswap(uint32_t& a, uint32_t& b) {
  // lanes 32-63 of a <-> lanes 0-31 of b
  auto s = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = s[0];
  b = s[1];
}

// X: B layout (X[4 t + k] = word 4h + k of element l & 31 of run t) -> F: element (run h, column l & 31)
// as 8 words in [0, 2p).
__device__ __forceinline__ void mfma_mul(uint32_t F[8], const uint32_t X[8], const v4i A, const uint32_t* K,
                                         double c224, double margin) {
  v4i b0, b1;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    b0[k] = (int)(X[k] ^ 0x80808080u);
    b1[k] = (int)(X[4 + k] ^ 0x80808080u);
  }
  const v16i z = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  const v16i d0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, b0, z, 0, 0, 0);
  const v16i d1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(A, b1, z, 0, 0, 0);
  uint32_t t0[4], u0[4], t1[4], u1[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    t0[m] = (uint32_t)d0[4 * m] + ((uint32_t)d0[4 * m + 1] << 8);
    u0[m] = (uint32_t)d0[4 * m + 2] + ((uint32_t)d0[4 * m + 3] << 8);
    t1[m] = (uint32_t)d1[4 * m] + ((uint32_t)d1[4 * m + 1] << 8);
    u1[m] = (uint32_t)d1[4 * m + 2] + ((uint32_t)d1[4 * m + 3] << 8);
  }
  // lower lanes keep run 0's even words and get its odd ones; upper lanes the reverse for run 1
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    pswap(t0[m], t1[m]);
    pswap(u0[m], u1[m]);
  }
  // word g = t_g + 2^16 u_g + carry (signed; |t|, |u| < 2^28): one v_mad_i64_i32 per word
  uint32_t w[9];
  int32_t carry = 0;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const int32_t t = (int32_t)((g & 1) ? t1[g >> 1] : t0[g >> 1]);
    const int32_t u = (int32_t)((g & 1) ? u1[g >> 1] : u0[g >> 1]);
    const int64_t c64 = (int64_t)(t + carry);
    int64_t v;
    uint64_t sd;  // (the carry-out lane mask, unused: an SGPR pair of its own rather than vcc)
    asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(v), "=s"(sd) : "v"(u), "s"(65536), "v"(c64));
    w[g] = (uint32_t)v;
    carry = (int32_t)(v >> 32);
  }
  // T = S' + K: a 9-word non-negative value (K in VGPRs: a VOP2 carry op reads vcc on the constant bus)
  w[8] = (uint32_t)carry;
  asm("v_add_co_u32 %0, vcc, %0, %9\n\t"
      "v_addc_co_u32 %1, vcc, %1, %10, vcc\n\t"
      "v_addc_co_u32 %2, vcc, %2, %11, vcc\n\t"
      "v_addc_co_u32 %3, vcc, %3, %12, vcc\n\t"
      "v_addc_co_u32 %4, vcc, %4, %13, vcc\n\t"
      "v_addc_co_u32 %5, vcc, %5, %14, vcc\n\t"
      "v_addc_co_u32 %6, vcc, %6, %15, vcc\n\t"
      "v_addc_co_u32 %7, vcc, %7, %16, vcc\n\t"
      "v_addc_co_u32 %8, vcc, %8, %17, vcc"
      : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]), "+v"(w[7]), "+v"(w[8])
      : "v"(K[0]), "v"(K[1]), "v"(K[2]), "v"(K[3]), "v"(K[4]), "v"(K[5]), "v"(K[6]), "v"(K[7]), "v"(K[8])
      : "vcc");
  const double f = fmax(fma(fma((double)w[8], 0x1p32, (double)w[7]), c224, -margin), 0.0);
  const uint32_t q = (uint32_t)f;
  // r = T - q p (words 0..7; T - q p < 2p < 2^256)
  const uint32_t P[8] = {STARK_P0, STARK_P1, STARK_P2, STARK_P3, STARK_P4, STARK_P5, STARK_P6, STARK_P7};
  uint32_t m[8];
  uint64_t hi = 0;
#pragma unroll
  for (int g = 0; g < 8; ++g) {
    const uint64_t mm = (uint64_t)q * P[g] + hi;
    m[g] = (uint32_t)mm;
    hi = mm >> 32;
  }
#pragma unroll
  for (int g = 0; g < 8; ++g) F[g] = w[g];
  asm("v_sub_co_u32 %0, vcc, %0, %8\n\t"
      "v_subb_co_u32 %1, vcc, %1, %9, vcc\n\t"
      "v_subb_co_u32 %2, vcc, %2, %10, vcc\n\t"
      "v_subb_co_u32 %3, vcc, %3, %11, vcc\n\t"
      "v_subb_co_u32 %4, vcc, %4, %12, vcc\n\t"
      "v_subb_co_u32 %5, vcc, %5, %13, vcc\n\t"
      "v_subb_co_u32 %6, vcc, %6, %14, vcc\n\t"
      "v_subb_co_u32 %7, vcc, %7, %15, vcc"
      : "+v"(F[0]), "+v"(F[1]), "+v"(F[2]), "+v"(F[3]), "+v"(F[4]), "+v"(F[5]), "+v"(F[6]), "+v"(F[7])
      : "v"(m[0]), "v"(m[1]), "v"(m[2]), "v"(m[3]), "v"(m[4]), "v"(m[5]), "v"(m[6]), "v"(m[7])
      : "vcc");
}

// B layout from the element layout (inverse of the exchange above, four swaps).
__device__ __forceinline__ void to_b_layout(uint32_t X[8], const uint32_t F[8]) {
#pragma unroll
  for (int k = 0; k < 8; ++k) X[k] = F[k];
#pragma unroll
  for (int k = 0; k < 4; ++k) pswap(X[k], X[4 + k]);
}

__device__ __forceinline__ void load_b(uint32_t X[8], const uint32_t* in, size_t base, int lane) {
  const int h = lane >> 5, e = lane & 31;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const uint4 v = *reinterpret_cast<const uint4*>(in + 8 * (base + 32 * t + e) + 4 * h);
    X[4 * t + 0] = v.x;
    X[4 * t + 1] = v.y;
    X[4 * t + 2] = v.z;
    X[4 * t + 3] = v.w;
  }
}

// iters products per element, chained; element base + lane out
__global__ __launch_bounds__(256) void mfma_k(const uint32_t* in, uint32_t* out, const MConst* mc, int n_in,
                                              int iters) {
  const int lane = threadIdx.x & 63;
  const size_t gw = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t base = (gw * 64) % (size_t)n_in;
  const v4i A = {mc->a[lane][0], mc->a[lane][1], mc->a[lane][2], mc->a[lane][3]};
  uint32_t K[9];
#pragma unroll
  for (int g = 0; g < 9; ++g) K[g] = mc->k[g];
  const double c224 = mc->c224, margin = mc->margin;
  uint32_t X[8], F[8];
  load_b(X, in, base, lane);
  for (int it = 0; it < iters; ++it) {  // (X carried: F is dead after each swap back)
    mfma_mul(F, X, A, K, c224, margin);
    to_b_layout(X, F);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) pswap(X[k], X[4 + k]);  // the swaps are their own inverse
#pragma unroll
  for (int k = 0; k < 8; ++k) F[k] = X[k];
  uint32_t* o = out + 8 * (gw * 64 + lane);
#pragma unroll
  for (int g = 0; g < 8; ++g) o[g] = F[g];
}

// fe_mul_db with one constant's table in LDS (wave-uniform reads), iters products per element
__global__ __launch_bounds__(256) void db_k(const uint32_t* in, uint32_t* out, const uint32_t* tab, int n_in,
                                            int iters) {
  __shared__ __attribute__((aligned(16))) uint32_t lw[72];
  if (threadIdx.x < 72) lw[threadIdx.x] = tab[threadIdx.x];
  __syncthreads();
  const size_t gi = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  fe a;
#pragma unroll
  for (int g = 0; g < 8; ++g) a.w[g] = in[8 * (gi % (size_t)n_in) + g];
  for (int it = 0; it < iters; ++it) a = fe_mul_db(a, lw);
#pragma unroll
  for (int g = 0; g < 8; ++g) out[8 * gi + g] = a.w[g];
}

static float time_ms(void (*launch)(int), int waves) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  launch(waves);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 10; ++r) launch(waves);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / 10;
}

static const uint32_t* g_in;
static uint32_t* g_out;
static const MConst* g_mc;
static const uint32_t* g_tab;
static int g_n;

static void launch_mfma(int waves) {
  hipLaunchKernelGGL(mfma_k, dim3(256 * waves), dim3(256), 0, 0, g_in, g_out, g_mc, g_n, ITERS);
}
static void launch_db(int waves) {
  hipLaunchKernelGGL(db_k, dim3(256 * waves), dim3(256), 0, 0, g_in, g_out, g_tab, g_n, ITERS);
}

int main(int argc, char** argv) {
  const char* inp = argc > 1 ? argv[1] : "mfma_in.bin";
  const char* outp = argc > 2 ? argv[2] : "mfma_out.bin";
  FILE* f = fopen(inp, "rb");
  if (!f) {
    printf("no %s\n", inp);
    return 1;
  }
  MConst mc;
  uint32_t tab[72];
  int n = 0;
  if (fread(&mc, sizeof mc, 1, f) != 1 || fread(tab, 4, 72, f) != 72 || fread(&n, 4, 1, f) != 1 || n % 64) {
    printf("bad %s\n", inp);
    return 1;
  }
  std::vector<uint32_t> h(8 * (size_t)n);
  if (fread(h.data(), 4, h.size(), f) != h.size()) return 1;
  fclose(f);
  uint32_t *din, *dout, *dtab;
  MConst* dmc;
  const size_t out_elems = (size_t)256 * 8 * 256 > (size_t)n ? (size_t)256 * 8 * 256 : (size_t)n;
  (void)hipMalloc(&din, h.size() * 4);
  (void)hipMalloc(&dout, out_elems * 32);
  (void)hipMalloc(&dmc, sizeof mc);
  (void)hipMalloc(&dtab, sizeof tab);
  (void)hipMemcpy(din, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(dmc, &mc, sizeof mc, hipMemcpyHostToDevice);
  (void)hipMemcpy(dtab, tab, sizeof tab, hipMemcpyHostToDevice);
  g_in = din;
  g_out = dout;
  g_mc = dmc;
  g_tab = dtab;
  g_n = n;
  // check: 1 product and ITERS chained products per element, MFMA form and digit basis
  FILE* g = fopen(outp, "wb");
  std::vector<uint32_t> o(8 * (size_t)n);
  for (int iters : {1, ITERS}) {
    hipLaunchKernelGGL(mfma_k, dim3(n / 256 + (n % 256 != 0)), dim3(256), 0, 0, din, dout, dmc, n, iters);
    (void)hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
    fwrite(o.data(), 4, o.size(), g);
    hipLaunchKernelGGL(db_k, dim3(n / 256 + (n % 256 != 0)), dim3(256), 0, 0, din, dout, dtab, n, iters);
    (void)hipMemcpy(o.data(), dout, o.size() * 4, hipMemcpyDeviceToHost);
    fwrite(o.data(), 4, o.size(), g);
  }
  fclose(g);
  printf("checked %d elements (1 and %d chained products, mfma and digit basis) -> %s\n", n, ITERS, outp);
  for (int w : {1, 2, 4, 8}) {
    const double prods = (double)256 * w * 256 * ITERS;
    const float mm = time_ms(launch_mfma, w), md = time_ms(launch_db, w);
    printf("waves/SIMD %d: mfma i8 %.2f G products/s (%.4f ms)   digit basis %.2f G products/s (%.4f ms)\n", w,
           prods / mm / 1e6, mm, prods / md / 1e6, md);
  }
  return 0;
}
