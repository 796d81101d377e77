// Field-vector kernels: zero-preserving batch inverse (multi_inv,
// packages/fri/src/poly_utils.rs:38-70) and multi-point polynomial evaluation
// (eval_poly_at over every x, poly_utils.rs:93-102 as called at
// packages/r1cs-stark/src/prove.rs:216-220), plus expand_root_of_unity
// (packages/fri/src/fft.rs:5-14).
#include "internal.h"

namespace stark {

constexpr uint32_t kInvChunk = 32;

// Montgomery constants used below (Montgomery images):
//   r2 = R^2 mod p  -> montmul(x_canon, r2) = x in Montgomery form
struct MontConsts {
  fe r2;   // R^2 mod p as limbs (i.e. Montgomery image of R)
  fe one;  // Montgomery image of 1 (= R mod p)
};

// x^(p-2) for x in Montgomery form (Fermat inverse), fixed exponent.
__device__ fe fe_inv_mont(const fe& x, const fe& one_m) {
  // p - 2 limbs, most significant first.
  const uint32_t e[8] = {STARK_P7, STARK_P6, STARK_P5, STARK_P4, STARK_P3, STARK_P2, STARK_P1, STARK_P0 - 2u};
  fe r = one_m;
  for (int i = 0; i < 8; ++i) {
    for (int b = 31; b >= 0; --b) {
      r = fe_mul(r, r);
      if ((e[i] >> b) & 1u) r = fe_mul(r, x);
    }
  }
  return r;
}

// Phase 1: chunk c of kInvChunk elements -> prefix products (Montgomery,
// zeros skipped) into pref, chunk product into tot[c].  MONT_IN: the input
// already holds Montgomery images (the chunk products of a lower level).
template <bool MONT_IN>
__global__ void inv_prefix_kernel(const fe* __restrict__ v, uint64_t n, fe* __restrict__ pref, fe* __restrict__ tot,
                                  MontConsts mc) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lo = c * kInvChunk;
  if (lo >= n) return;
  const uint64_t hi = lo + kInvChunk < n ? lo + kInvChunk : n;
  fe acc = mc.one;
  for (uint64_t i = lo; i < hi; ++i) {
    pref[i] = acc;  // product of the non-zero elements before i (exclusive)
    const fe x = fe_load(v + i);
    if (!fe_is_zero(x)) acc = fe_mul(acc, MONT_IN ? x : fe_mul(x, mc.r2));
  }
  tot[c] = acc;
}

// Phase 2: invert every chunk product (Fermat; ~380 products per chunk).
__global__ void inv_chunk_kernel(fe* __restrict__ tot, uint64_t chunks, MontConsts mc) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= chunks) return;
  tot[c] = fe_inv_mont(tot[c], mc.one);
}

// Phase 3: walk each chunk backwards (poly_utils.rs:55-67 order).  `tot`
// holds the Montgomery inverse of each chunk product.  Output canonical, or
// Montgomery when MONT_IN.
template <bool MONT_IN>
__global__ void inv_back_kernel(const fe* __restrict__ v, uint64_t n, const fe* __restrict__ pref,
                                const fe* __restrict__ tot, fe* __restrict__ out, MontConsts mc) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lo = c * kInvChunk;
  if (lo >= n) return;
  const uint64_t hi = lo + kInvChunk < n ? lo + kInvChunk : n;
  fe inv = tot[c];  // Montgomery
  fe unit = fe_zero();
  unit.w[0] = 1;
  for (uint64_t i = hi; i-- > lo;) {
    const fe x = fe_load(v + i);
    if (fe_is_zero(x)) {
      fe_store(out + i, fe_zero());
    } else {
      const fe r = fe_mul(pref[i], inv);  // Montgomery x^-1
      fe_store(out + i, MONT_IN ? r : fe_mul(r, unit));
      inv = fe_mul(inv, MONT_IN ? x : fe_mul(x, mc.r2));
    }
  }
}

// Horner evaluation of one polynomial at many points; coefficients canonical.
__global__ void eval_poly_kernel(const fe* __restrict__ poly, uint64_t deg1, const fe* __restrict__ xs, uint64_t n,
                                 fe* __restrict__ out, MontConsts mc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const fe xm = fe_mul(fe_load(xs + i), mc.r2);  // Montgomery image of x
  fe y = fe_zero();
  for (uint64_t k = deg1; k-- > 0;) y = fe_add(fe_mul(y, xm), fe_load(poly + k));
  fe_store(out + i, y);
}

// powers[i] = w^i (canonical) for i < count, from the two-level tables.
__global__ void powers_kernel(const fe* __restrict__ lo, const fe* __restrict__ hi, uint32_t kb, uint64_t count,
                              fe* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= count) return;
  fe unit = fe_zero();
  unit.w[0] = 1;
  // montmul(montmul(lo, hi), 1) = canonical w^i
  fe_store(out + i, fe_mul(fe_mul(lo[i & (((uint64_t)1 << kb) - 1)], hi[i >> kb]), unit));
}

MontConsts mont_consts() {
  const FieldHost& F = FieldHost::get();
  MontConsts mc;
  // Montgomery image of R is R^2 mod p: from_canonical(R mod p).
  uint64_t rmodp[4];
  HostFp one = F.one();  // Montgomery image of 1 = R mod p (as limbs)
  memcpy(rmodp, one.v, 32);
  mc.r2 = to_dev(F.from_canonical(rmodp));
  mc.one = to_dev(one);
  return mc;
}

// Batch inverse (0 -> 0).  Chunk products of kInvChunk elements; when there
// are many chunks their inverses come from a second batch-inverse level, so
// only n / kInvChunk^2 Fermat inversions run.
stark_status multi_inv_device(stark_ctx* ctx, const fe* d_in, fe* d_out, uint64_t n, hipStream_t s) {
  if (n == 0) return STARK_OK;
  const uint64_t c1 = (n + kInvChunk - 1) / kInvChunk;
  const uint64_t c2 = (c1 + kInvChunk - 1) / kInvChunk;
  const bool two = c1 > 4096;
  stark_status st = ensure_buf(ctx, ctx->io2, (n + c1 + (two ? 2 * c1 + c2 : 0)) * sizeof(fe));
  if (st != STARK_OK) return st;
  fe* pref1 = (fe*)ctx->io2.ptr;
  fe* tot1 = pref1 + n;
  const MontConsts mc = mont_consts();
  const unsigned b1 = (unsigned)((c1 + 255) / 256);
  hipLaunchKernelGGL(inv_prefix_kernel<false>, dim3(b1), dim3(256), 0, s, d_in, n, pref1, tot1, mc);
  const fe* tot1_inv = tot1;
  if (two) {
    fe* pref2 = tot1 + c1;
    fe* tot2 = pref2 + c1;
    fe* inv1 = tot2 + c2;
    const unsigned b2 = (unsigned)((c2 + 255) / 256);
    hipLaunchKernelGGL(inv_prefix_kernel<true>, dim3(b2), dim3(256), 0, s, (const fe*)tot1, c1, pref2, tot2, mc);
    hipLaunchKernelGGL(inv_chunk_kernel, dim3(b2), dim3(256), 0, s, tot2, c2, mc);
    hipLaunchKernelGGL(inv_back_kernel<true>, dim3(b2), dim3(256), 0, s, (const fe*)tot1, c1, (const fe*)pref2,
                       (const fe*)tot2, inv1, mc);
    tot1_inv = inv1;
  } else {
    hipLaunchKernelGGL(inv_chunk_kernel, dim3(b1), dim3(256), 0, s, tot1, c1, mc);
  }
  hipLaunchKernelGGL(inv_back_kernel<false>, dim3(b1), dim3(256), 0, s, d_in, n, (const fe*)pref1, tot1_inv, d_out,
                     mc);
  STARK_HIP(ctx, hipGetLastError());
  return STARK_OK;
}

}  // namespace stark

using namespace stark;

extern "C" {

stark_status stark_multi_inv(stark_ctx* ctx, const uint64_t* values, size_t n, uint64_t* out) {
  if (!ctx || (n && (!values || !out))) return STARK_ERR_BAD_ARG;
  if (n == 0) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  stark_status st = ensure_buf(ctx, ctx->io, 2 * n * sizeof(fe));
  if (st != STARK_OK) return st;
  fe* d_in = (fe*)ctx->io.ptr;
  fe* d_out = d_in + n;
  STARK_HIP(ctx, hipMemcpyAsync(d_in, values, n * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
  st = multi_inv_device(ctx, d_in, d_out, n, ctx->stream);
  if (st != STARK_OK) return st;
  STARK_HIP(ctx, hipMemcpyAsync(out, d_out, n * sizeof(fe), hipMemcpyDeviceToHost, ctx->stream));
  STARK_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return STARK_OK;
}

stark_status stark_eval_poly_at_multi(stark_ctx* ctx, const uint64_t* poly, size_t deg_plus_1, const uint64_t* xs,
                                      size_t n, uint64_t* out) {
  if (!ctx || (n && (!xs || !out)) || (deg_plus_1 && !poly)) return STARK_ERR_BAD_ARG;
  if (n == 0) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const size_t d1 = deg_plus_1 ? deg_plus_1 : 1;
  stark_status st = ensure_buf(ctx, ctx->io, (d1 + 2 * n) * sizeof(fe));
  if (st != STARK_OK) return st;
  fe* d_poly = (fe*)ctx->io.ptr;
  fe* d_xs = d_poly + d1;
  fe* d_out = d_xs + n;
  if (deg_plus_1)
    STARK_HIP(ctx, hipMemcpyAsync(d_poly, poly, deg_plus_1 * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
  STARK_HIP(ctx, hipMemcpyAsync(d_xs, xs, n * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
  hipLaunchKernelGGL(eval_poly_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ctx->stream, d_poly,
                     (uint64_t)deg_plus_1, d_xs, (uint64_t)n, d_out, mont_consts());
  STARK_HIP(ctx, hipGetLastError());
  STARK_HIP(ctx, hipMemcpyAsync(out, d_out, n * sizeof(fe), hipMemcpyDeviceToHost, ctx->stream));
  STARK_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return STARK_OK;
}

stark_status stark_expand_root_of_unity(stark_ctx* ctx, const uint64_t root[4], uint64_t* out, size_t cap,
                                        size_t* count) {
  if (!ctx || !root || !count || (cap && !out)) return STARK_ERR_BAD_ARG;
  // Order of root: smallest 2^k with root^(2^k) == 1 (k <= 28).
  const FieldHost& F = FieldHost::get();
  HostFp w = F.from_canonical(root), t = w;
  uint32_t k = 0;
  while (!FieldHost::eq(t, F.one())) {
    if (++k > 28) return STARK_ERR_BAD_ROOT;
    t = F.mul(t, t);
  }
  *count = (size_t)1 << k;
  const size_t m = cap < *count ? cap : *count;
  if (m == 0) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const Twiddles* tw = nullptr;
  uint64_t canon[4];
  F.to_canonical(w, canon);
  stark_status st = get_twiddles(ctx, canon, k, &tw);
  if (st != STARK_OK) return st;
  st = ensure_buf(ctx, ctx->io, m * sizeof(fe));
  if (st != STARK_OK) return st;
  hipLaunchKernelGGL(powers_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, ctx->stream, tw->d_lo, tw->d_hi,
                     tw->kb, (uint64_t)m, (fe*)ctx->io.ptr);
  STARK_HIP(ctx, hipGetLastError());
  STARK_HIP(ctx, hipMemcpyAsync(out, ctx->io.ptr, m * sizeof(fe), hipMemcpyDeviceToHost, ctx->stream));
  STARK_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return STARK_OK;
}

}  // extern "C"
