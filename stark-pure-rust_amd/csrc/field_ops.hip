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

// Phase 1: chunk c of kInvChunk elements -> prefix products (Montgomery,
// zeros skipped) into pref, chunk product into tot[c].  MONT_IN: the input
// already holds Montgomery images (the chunk products of a lower level).
template <bool MONT_IN, uint32_t CHUNK>
__global__ void inv_prefix_kernel(const fe* __restrict__ v, uint64_t n, fe* __restrict__ pref, fe* __restrict__ tot,
                                  MontConsts mc) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lo = c * CHUNK;
  if (lo >= n) return;
  const uint64_t hi = lo + CHUNK < n ? lo + CHUNK : n;
  fe acc = mc.one;
  for (uint64_t i = lo; i < hi; ++i) {
    pref[i] = acc;  // product of the non-zero elements before i (exclusive)
    const fe x = fe_load(v + i);
    if (!fe_is_zero(x)) acc = fe_mul(acc, MONT_IN ? x : fe_mul(x, mc.r2));
  }
  tot[c] = acc;
}

// Phase 3: walk each chunk backwards (poly_utils.rs:55-67 order).  `tot`
// holds the Montgomery inverse of each chunk product.  Output canonical, or
// Montgomery when MONT_IN.
template <bool MONT_IN, uint32_t CHUNK>
__global__ void inv_back_kernel(const fe* __restrict__ v, uint64_t n, const fe* __restrict__ pref,
                                const fe* __restrict__ tot, fe* __restrict__ out, MontConsts mc) {
  const uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t lo = c * CHUNK;
  if (lo >= n) return;
  const uint64_t hi = lo + CHUNK < n ? lo + CHUNK : n;
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

// Batch inverse (0 -> 0), the tree form of multi_inv (poly_utils.rs:38-70):
// chunk products of 32 inputs, then of 16 chunk products per level until at
// most 16 remain.  Those few are inverted on the host (one Fermat inversion
// there takes microseconds; on one GPU lane it is a ~250-product dependent
// chain, a quarter millisecond), and the inverses flow back down the levels.
constexpr uint32_t kInvChunkUp = 16;
constexpr uint64_t kInvTop = 16;

stark_status multi_inv_device(stark_ctx* ctx, const fe* d_in, fe* d_out, uint64_t n, hipStream_t s) {
  if (n == 0) return STARK_OK;
  // Level sizes: c[0] = ceil(n / 32) chunk products, c[i] = ceil(c[i-1] / 16).
  std::vector<uint64_t> c{(n + kInvChunk - 1) / kInvChunk};
  while (c.back() > kInvTop) c.push_back((c.back() + kInvChunkUp - 1) / kInvChunkUp);
  // Scratch: pref0[n], then per level i: tot_i[c_i], inv_i[c_i], pref_{i+1}[c_i] (for i < top).
  size_t total = n;
  for (size_t i = 0; i < c.size(); ++i) total += 3 * c[i];
  stark_status st = ensure_buf(ctx, ctx->io2, total * sizeof(fe));
  if (st != STARK_OK) return st;
  fe* pref0 = (fe*)ctx->io2.ptr;
  std::vector<fe*> tot(c.size()), inv(c.size()), pref(c.size());
  fe* at = pref0 + n;
  for (size_t i = 0; i < c.size(); ++i) {
    tot[i] = at;
    inv[i] = at + c[i];
    pref[i] = at + 2 * c[i];  // prefixes of level i+1's chunks over tot[i]
    at += 3 * c[i];
  }
  const MontConsts mc = mont_consts();
  auto blocks = [](uint64_t chunks) { return (unsigned)((chunks + 255) / 256); };
  hipLaunchKernelGGL((inv_prefix_kernel<false, kInvChunk>), dim3(blocks(c[0])), dim3(256), 0, s, d_in, n, pref0, tot[0],
                     mc);
  for (size_t i = 1; i < c.size(); ++i)
    hipLaunchKernelGGL((inv_prefix_kernel<true, kInvChunkUp>), dim3(blocks(c[i])), dim3(256), 0, s,
                       (const fe*)tot[i - 1], c[i - 1], pref[i - 1], tot[i], mc);
  STARK_HIP(ctx, hipGetLastError());
  // Top level: at most 16 non-zero Montgomery products, inverted on the host.
  const size_t top = c.size() - 1;
  uint8_t* pinned = nullptr;
  st = ctx_pinned(ctx, 1, 4096, (void**)&pinned);
  if (st != STARK_OK) return st;
  fe* h_top = (fe*)(pinned + 2560);  // pinned slot 1 layout: [2560, 3072) batch-inverse top level
  STARK_HIP(ctx, hipMemcpyAsync(h_top, tot[top], c[top] * sizeof(fe), hipMemcpyDeviceToHost, s));
  STARK_HIP(ctx, hipStreamSynchronize(s));
  {
    const FieldHost& F = FieldHost::get();
    for (uint64_t i = 0; i < c[top]; ++i) {
      HostFp x;
      for (int k = 0; k < 4; ++k) x.v[k] = (uint64_t)h_top[i].w[2 * k] | ((uint64_t)h_top[i].w[2 * k + 1] << 32);
      h_top[i] = to_dev(F.inv(x));  // Montgomery in, Montgomery out; products are never zero
    }
  }
  STARK_HIP(ctx, hipMemcpyAsync(inv[top], h_top, c[top] * sizeof(fe), hipMemcpyHostToDevice, s));
  for (size_t i = top; i >= 1; --i)
    hipLaunchKernelGGL((inv_back_kernel<true, kInvChunkUp>), dim3(blocks(c[i])), dim3(256), 0, s,
                       (const fe*)tot[i - 1], c[i - 1], (const fe*)pref[i - 1], (const fe*)inv[i], inv[i - 1], mc);
  hipLaunchKernelGGL((inv_back_kernel<false, kInvChunk>), dim3(blocks(c[0])), dim3(256), 0, s, d_in, n,
                     (const fe*)pref0, (const fe*)inv[0], d_out, mc);
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
