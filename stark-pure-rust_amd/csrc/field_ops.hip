// Field-vector kernels: zero-preserving batch inverse (multi_inv,
// packages/fri/src/poly_utils.rs:38-70) and multi-point polynomial evaluation
// (eval_poly_at over every x, poly_utils.rs:93-102 as called at
// packages/r1cs-stark/src/prove.rs:216-220), plus expand_root_of_unity
// (packages/fri/src/fft.rs:5-14).
#include "internal.h"

namespace stark {

// Batch inverse kernels.  A canonical input x < p is read as the Montgomery
// image of x' = x R^-1, so no conversion is needed on the way in: the
// products and inverses live in the x' Montgomery domain, and inv(x') in
// Montgomery form is x^-1 R^2, so one montmul by R^-1 (canonical) gives the
// canonical x^-1 on the way out.
struct MontConsts {
  fe r2;    // R^2 mod p: montmul(x, r2) = Montgomery image of canonical x
  fe one;   // Montgomery image of 1 (= R mod p)
  fe rinv;  // R^-1 mod p as plain limbs
};

constexpr uint32_t kInvThreads = 256;

// Hillis-Steele inclusive product scans of the workgroup's 256 values, both
// directions at once; returns the product of every value but this thread's.
__device__ __forceinline__ fe wg_others_product(fe t, const fe& one, fe* q, fe* sfx, fe* total) {
  const uint32_t j = threadIdx.x;
  fe pq = t, ps = t;
  q[j] = pq;
  sfx[j] = ps;
  __syncthreads();
  for (uint32_t off = 1; off < kInvThreads; off <<= 1) {
    const fe a = j >= off ? q[j - off] : one;
    const fe b = j + off < kInvThreads ? sfx[j + off] : one;
    __syncthreads();
    pq = fe_mul(pq, a);
    ps = fe_mul(ps, b);
    q[j] = pq;
    sfx[j] = ps;
    __syncthreads();
  }
  *total = q[kInvThreads - 1];
  const fe before = j ? q[j - 1] : one;
  const fe after = j + 1 < kInvThreads ? sfx[j + 1] : one;
  return fe_mul(before, after);
}

// Up pass: thread g owns elements g, g + T, g + 2T, .. (T = all threads of the launch, so a wave's
// loads and stores are contiguous): exclusive prefix products of its non-zero elements into pref,
// then the workgroup scan gives others[g] (the product of the other threads' elements) and
// wg_tot[block].  Any partition gives the same inverses (each is exact; zeros map to zero).
__global__ __launch_bounds__(kInvThreads) void inv_up_kernel(const fe* __restrict__ v, uint64_t n, uint32_t chunk,
                                                             fe* __restrict__ pref, fe* __restrict__ others,
                                                             fe* __restrict__ wg_tot, MontConsts mc) {
  __shared__ fe q[kInvThreads], sfx[kInvThreads];
  (void)chunk;
  const uint64_t g = (uint64_t)blockIdx.x * kInvThreads + threadIdx.x;
  const uint64_t T = (uint64_t)gridDim.x * kInvThreads;
  fe acc = mc.one;
  for (uint64_t i = g; i < n; i += T) {
    fe_store(pref + i, acc);
    const fe x = fe_load(v + i);
    if (!fe_is_zero(x)) acc = fe_mul(acc, x);
  }
  fe total;
  others[g] = wg_others_product(acc, mc.one, q, sfx, &total);
  if (threadIdx.x == 0) wg_tot[blockIdx.x] = total;
}

// Down pass: wg_inv[block] = inverse of the workgroup total, so the inverse
// of this thread's product is wg_inv * others; then its elements are walked
// backwards (poly_utils.rs:55-67 order).  OUT_CANON: level 0, canonical out.
template <bool OUT_CANON>
__global__ __launch_bounds__(kInvThreads) void inv_down_kernel(const fe* __restrict__ v, uint64_t n, uint32_t chunk,
                                                               const fe* __restrict__ pref,
                                                               const fe* __restrict__ others,
                                                               const fe* __restrict__ wg_inv, fe* __restrict__ out,
                                                               MontConsts mc) {
  (void)chunk;
  const uint64_t g = (uint64_t)blockIdx.x * kInvThreads + threadIdx.x;
  if (g >= n) return;
  const uint64_t T = (uint64_t)gridDim.x * kInvThreads;
  fe inv = fe_mul(wg_inv[blockIdx.x], others[g]);
  for (uint64_t i = g + (n - 1 - g) / T * T;; i -= T) {  // this thread's elements, last first
    const fe x = fe_load(v + i);
    if (fe_is_zero(x)) {
      fe_store(out + i, fe_zero());
    } else {
      const fe r = fe_mul(pref[i], inv);
      fe_store(out + i, OUT_CANON ? fe_mul(r, mc.rinv) : r);
      inv = fe_mul(inv, x);
    }
    if (i < T) break;
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

// ---- multi_interp_4 / eval_quartic (poly_utils.rs:442-511) ----
// Row values are taken to Montgomery form on load (montmul by R^2), combined
// with Montgomery products and returned canonical (montmul by canonical 1).

// The four basis numerators eq_k (coefficients, Montgomery) of the cubic
// through x0..x3 (poly_utils.rs:458-486).
__device__ __forceinline__ void interp4_eqs(const fe x[4], const fe& one, fe eq[4][4]) {
  const fe x01 = fe_mul(x[0], x[1]), x02 = fe_mul(x[0], x[2]), x03 = fe_mul(x[0], x[3]);
  const fe x12 = fe_mul(x[1], x[2]), x13 = fe_mul(x[1], x[3]), x23 = fe_mul(x[2], x[3]);
  const fe z = fe_zero();
  eq[0][0] = fe_sub(z, fe_mul(x12, x[3]));
  eq[0][1] = fe_add(fe_add(x12, x13), x23);
  eq[0][2] = fe_sub(fe_sub(fe_sub(z, x[1]), x[2]), x[3]);
  eq[1][0] = fe_sub(z, fe_mul(x02, x[3]));
  eq[1][1] = fe_add(fe_add(x02, x03), x23);
  eq[1][2] = fe_sub(fe_sub(fe_sub(z, x[0]), x[2]), x[3]);
  eq[2][0] = fe_sub(z, fe_mul(x01, x[3]));
  eq[2][1] = fe_add(fe_add(x01, x03), x13);
  eq[2][2] = fe_sub(fe_sub(fe_sub(z, x[0]), x[1]), x[3]);
  eq[3][0] = fe_sub(z, fe_mul(x01, x[2]));
  eq[3][1] = fe_add(fe_add(x01, x02), x12);
  eq[3][2] = fe_sub(fe_sub(fe_sub(z, x[0]), x[1]), x[2]);
  for (int k = 0; k < 4; ++k) eq[k][3] = one;
}

// eval_quartic with Montgomery p and x: p0 + p1 x + p2 x^2 + p3 x^3.
__device__ __forceinline__ fe quartic_m(const fe p[4], const fe& x) {
  const fe xsq = fe_mul(x, x), xcb = fe_mul(xsq, x);
  return fe_add(fe_add(fe_add(p[0], fe_mul(p[1], x)), fe_mul(p[2], xsq)), fe_mul(p[3], xcb));
}

__device__ __forceinline__ fe canon_unit() {
  fe u = fe_zero();
  u.w[0] = 1;
  return u;
}

// den[4 i + k] = eq_k(x_k) of row i (canonical), the batch inverse's targets.
__global__ void interp4_den_kernel(const fe* __restrict__ xs, uint64_t rows, fe* __restrict__ den, MontConsts mc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  fe x[4], eq[4][4];
  for (int k = 0; k < 4; ++k) x[k] = fe_mul(fe_load(xs + 4 * i + k), mc.r2);
  interp4_eqs(x, mc.one, eq);
  const fe unit = canon_unit();
  for (int k = 0; k < 4; ++k) fe_store(den + 4 * i + k, fe_mul(quartic_m(eq[k], x[k]), unit));
}

// out[i][j] = sum_k eq_k[j] * y_k * inv(den_k) (poly_utils.rs:496-506).
__global__ void interp4_out_kernel(const fe* __restrict__ xs, const fe* __restrict__ ys, const fe* __restrict__ inv,
                                   uint64_t rows, fe* __restrict__ out, MontConsts mc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= rows) return;
  fe x[4], eq[4][4], iy[4];
  for (int k = 0; k < 4; ++k) x[k] = fe_mul(fe_load(xs + 4 * i + k), mc.r2);
  interp4_eqs(x, mc.one, eq);
  for (int k = 0; k < 4; ++k)  // canonical y times the Montgomery image of inv: canonical y inv
    iy[k] = fe_mul(fe_load(ys + 4 * i + k), fe_mul(fe_load(inv + 4 * i + k), mc.r2));
  for (int j = 0; j < 4; ++j) {  // Montgomery eq times canonical y inv: canonical
    fe acc = fe_mul(eq[0][j], iy[0]);
    for (int k = 1; k < 4; ++k) acc = fe_add(acc, fe_mul(eq[k][j], iy[k]));
    fe_store(out + 4 * i + j, acc);
  }
}

// out[i] = eval_quartic(polys[i], xs[i]) (poly_utils.rs:442-446), canonical.
__global__ void eval_quartic_kernel(const fe* __restrict__ polys, const fe* __restrict__ xs, uint64_t n,
                                    fe* __restrict__ out, MontConsts mc) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const fe x = fe_mul(fe_load(xs + i), mc.r2), xsq = fe_mul(x, x), xcb = fe_mul(xsq, x);
  const fe* p = polys + 4 * i;
  fe_store(out + i, fe_add(fe_add(fe_add(fe_load(p), fe_mul(fe_load(p + 1), x)), fe_mul(fe_load(p + 2), xsq)),
                           fe_mul(fe_load(p + 3), xcb)));
}

// out[i] = sum_c coef[c] * cols[c][i] (coef Montgomery, data canonical).
__global__ void lincomb_kernel(const fe* __restrict__ cols, uint32_t n_cols, uint64_t n, const fe* __restrict__ coef,
                               fe* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe acc = fe_zero();
  for (uint32_t c = 0; c < n_cols; ++c) acc = fe_add(acc, fe_mul(fe_load(cols + (uint64_t)c * n + i), coef[c]));
  fe_store(out + i, acc);
}

MontConsts mont_consts() {
  const FieldHost& F = FieldHost::get();
  MontConsts mc;
  mc.one = to_dev(F.one());
  uint64_t rmodp[4];
  const HostFp one = F.one();
  memcpy(rmodp, one.v, 32);
  mc.r2 = to_dev(F.from_canonical(rmodp));  // Montgomery image of R
  // R^-1 mod p: canonical form of inv(Montgomery image of R).
  uint64_t rinv[4];
  F.to_canonical(F.inv(F.from_canonical(rmodp)), rinv);
  HostFp t;
  memcpy(t.v, rinv, 32);
  mc.rinv = to_dev(t);
  return mc;
}

// Batch inverse (0 -> 0), the tree form of multi_inv (poly_utils.rs:38-70).
// Each level turns n_i values into one product per workgroup (chunks of
// `chunk` per thread, then a product scan over the 256 threads), until at
// most 16 remain; those are inverted on the host (one Fermat inversion there
// takes microseconds, on one GPU lane it is a ~250-product dependent chain),
// and the inverses flow back down.  Small levels use one element per thread
// so the dependent chain per level is ~10 products; large ones use up to 32
// per thread so the scan costs < 1 product per element.
constexpr uint64_t kInvTop = 16;
static_assert(kInvTop * 32 <= 512, "one top array per 512 B of pinned slot 1");

static uint32_t inv_chunk_for(uint64_t n) {
  uint32_t c = 1;
  while (c < 32 && n / c > ((uint64_t)1 << 17)) c <<= 1;
  return c;
}

// Phase 1: the up kernels (scratch from `buf`; the top level's <= 16 products land in h_top, a pinned
// coherent host array).  The caller synchronises, then multi_inv_top and multi_inv_down.
stark_status multi_inv_up(stark_ctx* ctx, const fe* d_in, fe* d_out, uint64_t n, hipStream_t s, DevBuf& buf,
                          fe* h_top, InvPlan& plan) {
  plan.lv.clear();
  plan.h_top = h_top;
  if (n == 0) return STARK_OK;
  std::vector<InvPlan::Level>& lv = plan.lv;
  uint64_t m = n;
  size_t total = 0;
  while (m > kInvTop || lv.empty()) {
    InvPlan::Level L{};
    L.n = m;
    L.chunk = inv_chunk_for(m);
    const uint64_t threads = (m + L.chunk - 1) / L.chunk;
    L.wgs = (uint32_t)((threads + kInvThreads - 1) / kInvThreads);
    total += m + (uint64_t)L.wgs * kInvThreads + 2 * (uint64_t)L.wgs;  // pref, others, tot, out of the next level
    lv.push_back(L);
    m = L.wgs;
  }
  stark_status st = ensure_buf(ctx, buf, total * sizeof(fe));
  if (st != STARK_OK) return st;
  fe* at = (fe*)buf.ptr;
  for (size_t i = 0; i < lv.size(); ++i) {
    InvPlan::Level& L = lv[i];
    L.in = i ? lv[i - 1].tot : d_in;
    L.out = i ? nullptr : d_out;
    L.pref = at;
    at += L.n;
    L.others = at;
    at += (uint64_t)L.wgs * kInvThreads;
    L.tot = at;
    at += L.wgs;
  }
  // out of level i (i >= 1) = inverses of the totals of level i - 1.
  for (size_t i = 1; i < lv.size(); ++i) {
    lv[i].out = at;
    at += lv[i].n;
  }
  // Top: at most 16 non-zero Montgomery products, written by the last up kernel straight into the
  // pinned (coherent) host array, inverted there on the host and read back by the first down kernel,
  // with no copies.
  lv.back().tot = h_top;
  const MontConsts mc = mont_consts();
  for (const InvPlan::Level& L : lv)
    hipLaunchKernelGGL(inv_up_kernel, dim3(L.wgs), dim3(kInvThreads), 0, s, L.in, L.n, L.chunk, L.pref, L.others,
                       L.tot, mc);
  STARK_HIP(ctx, hipGetLastError());
  return STARK_OK;
}

// Phase 2 (host, after the caller's synchronisation): the top level's inverses in place.
void multi_inv_top(const InvPlan& plan) {
  if (plan.lv.empty()) return;
  const FieldHost& F = FieldHost::get();
  for (uint32_t i = 0; i < plan.lv.back().wgs; ++i) {
    HostFp x;
    for (int k = 0; k < 4; ++k)
      x.v[k] = (uint64_t)plan.h_top[i].w[2 * k] | ((uint64_t)plan.h_top[i].w[2 * k + 1] << 32);
    plan.h_top[i] = to_dev(F.inv(x));  // Montgomery in, Montgomery out; products are never zero
  }
}

// Phase 3: the down kernels.
stark_status multi_inv_down(stark_ctx* ctx, const InvPlan& plan, hipStream_t s) {
  const std::vector<InvPlan::Level>& lv = plan.lv;
  if (lv.empty()) return STARK_OK;
  const MontConsts mc = mont_consts();
  for (size_t i = lv.size(); i-- > 0;) {
    const InvPlan::Level& L = lv[i];
    const fe* wg_inv = i + 1 < lv.size() ? lv[i + 1].out : plan.h_top;
    if (i == 0)
      hipLaunchKernelGGL(inv_down_kernel<true>, dim3(L.wgs), dim3(kInvThreads), 0, s, L.in, L.n, L.chunk,
                         (const fe*)L.pref, (const fe*)L.others, wg_inv, L.out, mc);
    else
      hipLaunchKernelGGL(inv_down_kernel<false>, dim3(L.wgs), dim3(kInvThreads), 0, s, L.in, L.n, L.chunk,
                         (const fe*)L.pref, (const fe*)L.others, wg_inv, L.out, mc);
  }
  STARK_HIP(ctx, hipGetLastError());
  return STARK_OK;
}

fe* multi_inv_h_top(stark_ctx* ctx, int k) {  // pinned slot 1: [2560 + 512 k, 3072 + 512 k), k < 2
  uint8_t* pinned = nullptr;
  if (ctx_pinned(ctx, 1, kPinned1Bytes, (void**)&pinned) != STARK_OK) return nullptr;
  return (fe*)(pinned + kPinned1InvTopOff + 512 * (size_t)k);
}

stark_status multi_inv_device(stark_ctx* ctx, const fe* d_in, fe* d_out, uint64_t n, hipStream_t s) {
  if (n == 0) return STARK_OK;
  fe* h_top = multi_inv_h_top(ctx, 0);
  if (!h_top) return STARK_ERR_OOM;
  InvPlan plan;
  // io2 and the pinned top array are the context's: a previous inverse on another stream may still
  // read them in its down kernels (the host rewrites the top array below, after s has waited for it).
  STARK_TRY(buf_acquire(ctx, ctx->io2, s));
  STARK_TRY(multi_inv_up(ctx, d_in, d_out, n, s, ctx->io2, h_top, plan));
  STARK_HIP(ctx, hipStreamSynchronize(s));
  multi_inv_top(plan);
  STARK_TRY(multi_inv_down(ctx, plan, s));
  return buf_release(ctx, ctx->io2, s);
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

stark_status stark_multi_interp_4(stark_ctx* ctx, const uint64_t* xsets, const uint64_t* ysets, size_t rows,
                                  uint64_t* out) {
  if (!ctx || (rows && (!xsets || !ysets || !out))) return STARK_ERR_BAD_ARG;
  if (rows == 0) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const size_t m = 4 * rows;
  stark_status st = ensure_buf(ctx, ctx->io, 5 * m * sizeof(fe));
  if (st != STARK_OK) return st;
  fe* d_x = (fe*)ctx->io.ptr;
  fe* d_y = d_x + m;
  fe* d_den = d_y + m;
  fe* d_inv = d_den + m;
  fe* d_out = d_inv + m;
  hipStream_t s = ctx->stream;
  STARK_HIP(ctx, hipMemcpyAsync(d_x, xsets, m * sizeof(fe), hipMemcpyHostToDevice, s));
  STARK_HIP(ctx, hipMemcpyAsync(d_y, ysets, m * sizeof(fe), hipMemcpyHostToDevice, s));
  const MontConsts mc = mont_consts();
  const unsigned grid = (unsigned)((rows + 255) / 256);
  hipLaunchKernelGGL(interp4_den_kernel, dim3(grid), dim3(256), 0, s, (const fe*)d_x, (uint64_t)rows, d_den, mc);
  STARK_HIP(ctx, hipGetLastError());
  st = multi_inv_device(ctx, d_den, d_inv, m, s);  // zero-preserving, like multi_inv (poly_utils.rs:38-70)
  if (st != STARK_OK) return st;
  hipLaunchKernelGGL(interp4_out_kernel, dim3(grid), dim3(256), 0, s, (const fe*)d_x, (const fe*)d_y,
                     (const fe*)d_inv, (uint64_t)rows, d_out, mc);
  STARK_HIP(ctx, hipGetLastError());
  STARK_HIP(ctx, hipMemcpyAsync(out, d_out, m * sizeof(fe), hipMemcpyDeviceToHost, s));
  STARK_HIP(ctx, hipStreamSynchronize(s));
  return STARK_OK;
}

stark_status stark_eval_quartic_multi(stark_ctx* ctx, const uint64_t* polys, const uint64_t* xs, size_t n,
                                      uint64_t* out) {
  if (!ctx || (n && (!polys || !xs || !out))) return STARK_ERR_BAD_ARG;
  if (n == 0) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  stark_status st = ensure_buf(ctx, ctx->io, 6 * n * sizeof(fe));
  if (st != STARK_OK) return st;
  fe* d_p = (fe*)ctx->io.ptr;
  fe* d_x = d_p + 4 * n;
  fe* d_o = d_x + n;
  hipStream_t s = ctx->stream;
  STARK_HIP(ctx, hipMemcpyAsync(d_p, polys, 4 * n * sizeof(fe), hipMemcpyHostToDevice, s));
  STARK_HIP(ctx, hipMemcpyAsync(d_x, xs, n * sizeof(fe), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(eval_quartic_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const fe*)d_p,
                     (const fe*)d_x, (uint64_t)n, d_o, mont_consts());
  STARK_HIP(ctx, hipGetLastError());
  STARK_HIP(ctx, hipMemcpyAsync(out, d_o, n * sizeof(fe), hipMemcpyDeviceToHost, s));
  STARK_HIP(ctx, hipStreamSynchronize(s));
  return STARK_OK;
}

stark_status stark_lincomb_dev(stark_ctx* ctx, const uint64_t* d_cols, uint32_t n_cols, size_t n,
                               const uint64_t* coeffs, uint64_t* d_out, void* stream) {
  if (!ctx || !d_out || (n_cols && (!d_cols || !coeffs))) return STARK_ERR_BAD_ARG;
  if (n == 0) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const FieldHost& F = FieldHost::get();
  std::vector<fe> h(n_cols ? n_cols : 1);
  for (uint32_t c = 0; c < n_cols; ++c) h[c] = to_dev(F.from_canonical(coeffs + 4 * c));  // Montgomery
  stark_status st = ensure_buf(ctx, ctx->io2, h.size() * sizeof(fe));
  if (st != STARK_OK) return st;
  hipStream_t s = pick_stream(ctx, stream);
  STARK_TRY(buf_acquire(ctx, ctx->io2, s));
  STARK_HIP(ctx, hipMemcpyAsync(ctx->io2.ptr, h.data(), h.size() * sizeof(fe), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(lincomb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, (const fe*)d_cols, n_cols,
                     (uint64_t)n, (const fe*)ctx->io2.ptr, (fe*)d_out);
  STARK_HIP(ctx, hipGetLastError());
  STARK_TRY(buf_release(ctx, ctx->io2, s));
  // h is pageable and goes out of scope: the copy must have consumed it.
  STARK_HIP(ctx, hipStreamSynchronize(s));
  return STARK_OK;
}

stark_status stark_lincomb(stark_ctx* ctx, const uint64_t* cols, uint32_t n_cols, size_t n, const uint64_t* coeffs,
                           uint64_t* out) {
  if (!ctx || (n && !out) || (n && n_cols && (!cols || !coeffs))) return STARK_ERR_BAD_ARG;
  if (n == 0) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  stark_status st = ensure_buf(ctx, ctx->io, ((size_t)n_cols + 1) * n * sizeof(fe));
  if (st != STARK_OK) return st;
  fe* d_cols = (fe*)ctx->io.ptr;
  fe* d_out = d_cols + (size_t)n_cols * n;
  if (n_cols)
    STARK_HIP(ctx, hipMemcpyAsync(d_cols, cols, (size_t)n_cols * n * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
  st = stark_lincomb_dev(ctx, (const uint64_t*)d_cols, n_cols, n, coeffs, (uint64_t*)d_out, nullptr);
  if (st != STARK_OK) return st;
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
