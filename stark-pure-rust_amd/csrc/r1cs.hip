// mk_r1cs_proof (packages/r1cs-stark/src/prove.rs:14-378) resident on one
// gfx950 GPU.
//
// Everything of size `steps` or `precision` lives in HBM from upload to
// proof; the host runs only the transcript (a_root -> r, m_root -> k,
// l_root -> positions, the FRI layer roots) and serialises the proof.
//
//   upload 6 step columns + permuted indices
//   index/accumulator kernel      IDX, PIDX, 40-B accumulator leaves
//   acc Merkle tree               -> a_root -> r (host, utils.rs:272-290)
//   batched iNTT(steps, g1) x 8 -> zero-pad -> batched NTT(precision, g2) x 8
//   A column: a_vals kernel, two product scans, multi_inv, iNTT/NTT
//   zb kernel + multi_inv         inverse Zb2 / Zb3 (0 -> 0)
//   constraint kernel             Q1..Q3 -> D1..D3, B2, B3 (with the
//                                 reference's divisibility asserts) written as
//                                 the 256-B main-tree rows P|A|S|D1|D2|D3|B2|B3
//   main Merkle tree (256-B leaves) -> m_root -> k (host, prove.rs:274-283)
//   linear-combination kernel     L, then its Merkle tree -> l_root
//   proof gathers + prove_low_degree on the resident L.
//
// Values are canonical in HBM; constants are Montgomery images so that
// fe_mul(data, const) is the canonical product (see fp_dev.h).
#include <string.h>

#include <string>
#include <vector>

#include "internal.h"
#include "blake2s.h"
#include "fe_db.h"

namespace stark {
void json_bytes(std::string& o, const uint8_t* p, size_t n);
void json_branches(std::string& o, const std::vector<uint8_t>& leaves, size_t leaf_len,
                   const std::vector<uint8_t>& nodes, size_t k, size_t depth);
void fri_proof_json_string(const stark_fri_proof* proof, std::string& o);
}  // namespace stark

namespace stark {

static inline fe fe_zero_host() {
  fe r;
  for (int i = 0; i < 8; ++i) r.w[i] = 0;
  return r;
}

constexpr int kExtensionFactor = 8;     // utils.rs:135
constexpr int kLogExtensionFactor = 3;  // utils.rs:134
constexpr int kSpotChecks = 80;         // utils.rs:136
constexpr uint32_t kScanBlock = 1024;   // elements per workgroup in the product scan

// Montgomery image of R (montmul(x, r2) = Montgomery image of x) and of 1.
struct Mont {
  fe r2, one, unit;  // unit = canonical 1 (montmul(x_m, unit) = canonical x)
  fe rinv;           // R^-1 as a canonical value (montmul(x_m, rinv) = x R^-1)
};

static Mont mont() {
  const FieldHost& F = FieldHost::get();
  Mont m;
  HostFp one = F.one();
  m.r2 = to_dev(F.from_canonical(one.v));
  m.one = to_dev(one);
  m.unit = fe_zero_host();
  m.unit.w[0] = 1;
  const HostFp rv = F.from_canonical(one.v);  // the value R
  m.rinv = to_dev(F.inv(F.mul(rv, rv)));      // the value R^-2, whose Montgomery image is R^-1
  return m;
}

__device__ __forceinline__ fe fe_from_u64(uint64_t v) {
  fe r = fe_zero();
  r.w[0] = (uint32_t)v;
  r.w[1] = (uint32_t)(v >> 32);
  return r;
}

// Fiat-Shamir values derived on the device from the tree roots, so the proof
// is enqueued end to end without waiting for the host.
constexpr int kLincombConsts = 29;
struct Transcript {
  fe r0;       // canonical r[0]
  fe r1_m;     // Montgomery r[1], r[2]
  fe r2_m;
  fe k_m[11];  // Montgomery k[0..10]
  fe kx_m[8][3];  // Montgomery k3 + k4 xs_t, k5 + k6 xs_t, k7 + k8 xs_t (t = i mod 8)
  uint32_t roots[3][8];  // a_root, m_root, l_root (LE words = the digest bytes)
  int err;
  // Digit-basis tables (fe_db.h) of L's constants: k0, k1, k2, k9, k10, then kx[t][c] at 5 + 3 t + c.
  uint32_t k_db[kLincombConsts][72];
  // The constraint kernel's constants as digit-basis tables: r[1], r[2] (r1cs_r_kernel), and from the
  // host (upload_constraint_tables) R^-1 (the x R^-1 scalings) and the partial-fraction coefficients a_k.
  uint32_t r_db[2][72];
  uint32_t c_db[33][72];  // R^-1 | a_0..a_7 | inv(Z) R^k at t = i mod 8, table 9 + 8 k + t (invz_m)
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Digest of a 32- or 33-byte message (words LE, zero padded).
__device__ __forceinline__ void b2s_short(const uint32_t* w, uint32_t extra_byte, uint32_t len, uint32_t out[8]) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) m[i] = w[i];
  m[8] = extra_byte;
#pragma unroll
  for (int i = 9; i < 16; ++i) m[i] = 0;
  b2s_init(out);
  b2s_compress(out, m, len, 0, true);
}

// The digit-basis table of a canonical constant c: limb j of c 2^(32 i) mod p at 9 i + j, each row one
// product by the Montgomery image of 2^(32 i) (Pow32), one row per thread.
__device__ __forceinline__ void db_limbs(const fe& c, uint32_t* __restrict__ out) {  // 9 x 29-bit limbs of c
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int bit = 29 * j, w = bit >> 5, sh = bit & 31;
    uint32_t v = c.w[w] >> sh;
    if (sh > 3 && w < 7) v |= c.w[w + 1] << (32 - sh);
    out[j] = v & STARK_DB_M29;
  }
}

// Montgomery images of 2^(32 i) mod p, i < 8: a digit-basis table's rows as independent products.
struct Pow32 {
  fe m[8];
};

// r = get_random_ff_values(a_root, precision, 3, 0) (utils.rs:272-290):
// get_pseudorandom_indices(seed, precision, 24, 0) (fri/src/utils.rs:82-109)
// expands seed || B(seed) || B(B(seed)), reads 24 big-endian words mod
// precision; each group of 8 is written as big-endian bytes and read back
// with from_bytes_le (mod p).
__global__ void r1cs_r_kernel(const uint32_t* __restrict__ a_root, uint32_t prec_mask, fe r2, Pow32 p32,
                              Transcript* __restrict__ tr) {
  __shared__ fe rs[2];
  if (threadIdx.x == 0) {
    uint32_t data[24];
#pragma unroll
    for (int i = 0; i < 8; ++i) data[i] = a_root[i];
    b2s_short(data, 0, 32, data + 8);
    b2s_short(data + 8, 0, 32, data + 16);
    fe r[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t v = bswap32(data[8 * c + i]) & prec_mask;  // BE word mod 2^k
        r[c].w[i] = bswap32(v);                                  // BE bytes read as LE words
      }
#pragma unroll
      for (int k = 0; k < 5; ++k) fe_reduce_once(r[c]);
    }
    tr->r0 = r[0];
    tr->r1_m = fe_mul(r[1], r2);
    tr->r2_m = fe_mul(r[2], r2);
    rs[0] = r[1];
    rs[1] = r[2];
#pragma unroll
    for (int i = 0; i < 8; ++i) tr->roots[0][i] = a_root[i];
  }
  __syncthreads();
  // The digit-basis tables of r[1], r[2] (the constraint kernel's): one row r 2^(32 i) per thread.
  const uint32_t t = threadIdx.x;
  if (t < 16) db_limbs(fe_mul(rs[t >> 3], p32.m[t & 7]), tr->r_db[t >> 3] + 9 * (t & 7));
}

// (g2^steps)^t, t < 8: the x^steps factor of L at the points i = t mod 8 (prove.rs:287-291).
struct XsPowers {
  fe v[8];
};

constexpr uint32_t kKThreads = 256;  // r1cs_k_kernel: kLincombConsts x 8 table rows
static_assert(kLincombConsts * 8 <= kKThreads, "r1cs_k_kernel rows");
// k_0 = 1, k_i = from_str(mk_seed([m_root, [i]])) = BE integer of
// Blake2s(m_root || i) mod p (prove.rs:274-283, utils.rs:25-27, 51-57); then the
// three per-residue coefficients of L, kx[t] = (k3 + k4 xs_t, k5 + k6 xs_t,
// k7 + k8 xs_t), so the L kernel needs 8 products per point instead of 14.
__global__ void r1cs_k_kernel(const uint32_t* __restrict__ m_root, fe r2, fe one_m, XsPowers xs, Pow32 p32,
                              Transcript* __restrict__ tr) {
  __shared__ fe ks[11];
  __shared__ fe kx[8][3];
  const uint32_t i = threadIdx.x;
  if (i == 0) {
    ks[0] = one_m;
    tr->k_m[0] = one_m;
#pragma unroll
    for (int j = 0; j < 8; ++j) tr->roots[1][j] = m_root[j];
  } else if (i <= 10) {
    uint32_t h[8];
    b2s_short(m_root, i, 33, h);
    fe k;
#pragma unroll
    for (int j = 0; j < 8; ++j) k.w[j] = bswap32(h[7 - j]);
#pragma unroll
    for (int t = 0; t < 5; ++t) fe_reduce_once(k);
    ks[i] = fe_mul(k, r2);
    tr->k_m[i] = ks[i];
  }
  __syncthreads();
  if (i < 8) {
    kx[i][0] = fe_add(ks[3], fe_mul(ks[4], xs.v[i]));
    kx[i][1] = fe_add(ks[5], fe_mul(ks[6], xs.v[i]));
    kx[i][2] = fe_add(ks[7], fe_mul(ks[8], xs.v[i]));
    tr->kx_m[i][0] = kx[i][0];
    tr->kx_m[i][1] = kx[i][1];
    tr->kx_m[i][2] = kx[i][2];
  }
  __syncthreads();
  // The constants' digit-basis tables, one row c 2^(32 r) mod p per thread (kKThreads threads)
  if (i < kLincombConsts * 8) {
    static constexpr int kIdx[5] = {0, 1, 2, 9, 10};
    const uint32_t c = i >> 3, r = i & 7;
    const fe m = c < 5 ? ks[kIdx[c]] : kx[(c - 5) / 3][(c - 5) % 3];
    fe unit = fe_zero();
    unit.w[0] = 1;
    const fe canon = fe_mul(m, unit);  // canonical constant (Montgomery image x R^-1)
    db_limbs(fe_mul(canon, p32.m[r]), tr->k_db[c] + 9 * r);
  }
}

__global__ void r1cs_l_root_kernel(const uint32_t* __restrict__ l_root, Transcript* __restrict__ tr) {
  if (threadIdx.x < 8) tr->roots[2][threadIdx.x] = l_root[threadIdx.x];
}

// Montgomery image of g^i from the two-level tables of g.
__device__ __forceinline__ fe pow_tab(const fe* __restrict__ lo, const fe* __restrict__ hi, uint32_t kb, uint64_t i) {
  return fe_mul(lo[i & (((uint64_t)1 << kb) - 1)], hi[i >> kb]);
}

// IDX / PIDX step columns (prove.rs:160-167 with the identity tail of
// prove.rs:55-56) and the accumulator leaves u64 LE index || to_bytes_le(w)
// (utils.rs:254-263).
// (IDX itself is not written: its extension is the context's shared ext_index_column.)
// (dig non-null: each 40-B leaf's Blake2s too, the accumulator tree's level 0 (merkle_level0), 8 words.)
__global__ void r1cs_index_kernel(const uint64_t* __restrict__ perm, uint64_t os, uint64_t steps,
                                  const fe* __restrict__ w, fe* __restrict__ pidx, uint64_t* __restrict__ acc_leaves,
                                  uint32_t* __restrict__ dig) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= steps) return;
  const uint64_t p = i < os ? perm[i] : i;
  fe_store(pidx + i, fe_from_u64(p));
  const fe x = fe_load(w + i);
  uint64_t* leaf = acc_leaves + 5 * i;
  leaf[0] = p;
#pragma unroll
  for (int k = 0; k < 4; ++k) leaf[1 + k] = (uint64_t)x.w[2 * k] | ((uint64_t)x.w[2 * k + 1] << 32);
  if (dig) {  // (uniform) one zero-padded block of the 40 leaf bytes
    uint32_t h[8], m[16];
    b2s_init(h);
    m[0] = (uint32_t)p;
    m[1] = (uint32_t)(p >> 32);
#pragma unroll
    for (int k = 0; k < 8; ++k) m[2 + k] = x.w[k];
#pragma unroll
    for (int k = 10; k < 16; ++k) m[k] = 0;
    b2s_compress(h, m, 40, 0, true);
    uint4* d = reinterpret_cast<uint4*>(dig + 8 * i);
    d[0] = make_uint4(h[0], h[1], h[2], h[3]);
    d[1] = make_uint4(h[4], h[5], h[6], h[7]);
  }
}

// Flag columns F0, F1, F2 (run.rs:283-308) from bytes: dst[f * steps + i] = fb[f * os + i].
__global__ void r1cs_flags_kernel(const uint8_t* __restrict__ fb, uint64_t os, uint64_t steps, fe* __restrict__ dst) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= 3 * os) return;
  const uint64_t f = g / os, i = g - f * os;
  fe_store(dst + f * steps + i, fe_from_u64(fb[g]));
}

// The proof's input columns from device-resident trace columns in one launch (the device trace builder's
// output, stark_prove_r1cs_bytes), in place of a dozen copies and fills: raw[c] (c < 6: K F0 F1 F2 S P) =
// the column zero-padded to `steps` (F0-F2 widened from their 0/1 bytes), wcopy = S, perm copied, and
// the transcript zeroed.
struct PackArgs {
  const fe* col[6];     // K, (F0, F1, F2 when given as elements), S, P
  const uint8_t* fb;    // F0-F2 as 3 x os bytes (or null)
  const uint64_t* perm_in;
  uint64_t os, steps;
  fe* raw;
  fe* wcopy;
  uint64_t* perm;
  uint32_t* tr;         // the transcript, tr_words u32
  uint32_t tr_words;
  uint32_t k_slot;      // K's raw slot: 0, or 1 when F0's extension is the shared one (F0 not written)
};
__global__ void r1cs_pack_kernel(PackArgs a) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.tr_words) a.tr[i] = 0;
  if (i >= a.steps) return;
  const bool in = i < a.os;
#pragma unroll
  for (int c = 0; c < 6; ++c) {
    if (c == 1 && a.k_slot) continue;  // (uniform)
    fe v = fe_zero();
    if (in) {
      if (a.fb && c >= 1 && c <= 3) v = fe_from_u64(a.fb[(uint64_t)(c - 1) * a.os + i]);
      else v = fe_load(a.col[c] + i);
    }
    fe_store(a.raw + (uint64_t)(c == 0 ? a.k_slot : c) * a.steps + i, v);
    if (c == 4) fe_store(a.wcopy + i, v);
  }
  if (in) a.perm[i] = a.perm_in[i];
}

// val_nmr / val_dnm of calc_a_mini_evaluations (utils.rs:317-318), written as
// Montgomery images for the product scans.
// ext_idx[8 j] = IDX[j] = j and ext_pidx[8 j] = PIDX[j] (the LDE interpolates the step
// values); with ext_idx == nullptr (distributed prover: the extended columns are
// sharded) they are taken from the step-domain permutation instead.
__global__ void r1cs_a_vals_kernel(const fe* __restrict__ ext_idx, const fe* __restrict__ ext_pidx,
                                   const uint64_t* __restrict__ perm, uint64_t os,
                                   const fe* __restrict__ w, uint64_t steps, const Transcript* __restrict__ tr, fe mr2,
                                   fe* __restrict__ nmr_m, fe* __restrict__ dnm_m) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= steps) return;
  const fe r0 = tr->r0, r1_m = tr->r1_m, r2_m = tr->r2_m;
  const fe rw = fe_mul(fe_load(w + j), r2_m);
  const fe xi = ext_idx ? fe_load(ext_idx + j * kExtensionFactor) : fe_from_u64(j);
  const fe xp = ext_idx ? fe_load(ext_pidx + j * kExtensionFactor) : fe_from_u64(j < os ? perm[j] : j);
  const fe vn = fe_add(fe_add(r0, fe_mul(xi, r1_m)), rw);
  const fe vd = fe_add(fe_add(r0, fe_mul(xp, r1_m)), rw);
  fe_store(nmr_m + j, fe_mul(vn, mr2));
  fe_store(dnm_m + j, fe_mul(vd, mr2));
}

// Inclusive product scan, phase 1: each workgroup scans kScanBlock Montgomery
// values in place (4 per thread, then a 256-entry scan of the thread
// products in LDS) and writes the block product to tot[blockIdx].
// The scans run over one or two arrays at once (blockIdx.y picks the array: the A column's numerators and
// denominators, one launch per phase for both).
struct ScanArrays {
  fe* v[2];
  fe* tot[2];
  fe* canon[2];
};

__global__ __launch_bounds__(256) void scan_block_kernel(ScanArrays a, uint64_t n, fe one_m) {
  __shared__ fe part[256];
  fe* __restrict__ v = a.v[blockIdx.y];
  fe* __restrict__ tot = a.tot[blockIdx.y];
  const uint64_t base = (uint64_t)blockIdx.x * kScanBlock + 4 * threadIdx.x;
  fe x[4];
  fe acc = one_m;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    x[k] = base + k < n ? fe_load(v + base + k) : one_m;
    acc = fe_mul(acc, x[k]);
    x[k] = acc;
  }
  part[threadIdx.x] = acc;
  __syncthreads();
  // Hillis-Steele over the 256 thread products.
  for (uint32_t off = 1; off < 256; off <<= 1) {
    fe t = part[threadIdx.x];
    if (threadIdx.x >= off) t = fe_mul(part[threadIdx.x - off], t);
    __syncthreads();
    part[threadIdx.x] = t;
    __syncthreads();
  }
  const fe pre = threadIdx.x ? part[threadIdx.x - 1] : one_m;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (base + k < n) fe_store(v + base + k, threadIdx.x ? fe_mul(pre, x[k]) : x[k]);
  if (threadIdx.x == 255) tot[blockIdx.x] = part[255];
}

// Phase 2: exclusive scan of the block products (one workgroup; each thread
// owns a contiguous run).
__global__ __launch_bounds__(256) void scan_tot_kernel(ScanArrays a, uint32_t nb, fe one_m) {
  __shared__ fe part[256];
  fe* __restrict__ tot = a.tot[blockIdx.y];
  const uint32_t per = (nb + 255) / 256;
  const uint32_t lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
  fe acc = one_m;
  for (uint32_t i = lo; i < hi; ++i) acc = fe_mul(acc, tot[i]);
  part[threadIdx.x] = acc;
  __syncthreads();
  // Inclusive Hillis-Steele scan of the 256 run products (8 dependent
  // products instead of a 256-long serial chain), then shift to exclusive.
  for (uint32_t off = 1; off < 256; off <<= 1) {
    fe t = part[threadIdx.x];
    if (threadIdx.x >= off) t = fe_mul(part[threadIdx.x - off], t);
    __syncthreads();
    part[threadIdx.x] = t;
    __syncthreads();
  }
  const fe excl = threadIdx.x ? part[threadIdx.x - 1] : one_m;
  __syncthreads();
  part[threadIdx.x] = excl;
  __syncthreads();
  acc = part[threadIdx.x];
  for (uint32_t i = lo; i < hi; ++i) {
    const fe t = tot[i];
    tot[i] = acc;
    acc = fe_mul(acc, t);
  }
}

// Phase 3: block b (> 0) times the product of blocks before it; also emits
// the canonical value into `canon` when given.
__global__ void scan_apply_kernel(ScanArrays a, uint64_t n, fe unit) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  fe* __restrict__ v = a.v[blockIdx.y];
  const fe* __restrict__ tot = a.tot[blockIdx.y];
  fe* __restrict__ canon = a.canon[blockIdx.y];
  fe x = fe_load(v + i);
  const uint64_t b = i / kScanBlock;
  if (b) x = fe_mul(x, tot[b]);
  fe_store(v + i, x);
  if (canon) fe_store(canon + i, fe_mul(x, unit));
}

// a_mini[j] = acc_nmr[j] * inv(acc_dnm[j]) (utils.rs:331-336); nmr Montgomery, inv canonical.
__global__ void r1cs_a_mini_kernel(const fe* __restrict__ nmr_m, const fe* __restrict__ inv_dnm, uint64_t steps,
                                   fe* __restrict__ out) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= steps) return;
  fe_store(out + j, fe_mul(fe_load(nmr_m + j), fe_load(inv_dnm + j)));
}

// Zb2(x) = prod_k (x - x_k) (utils.rs:438-455) and Zb3(x) = x - x_last
// (utils.rs:466-474) for the batch inverse, each as Zb R^-1 (unit = R^-1, Mont::rinv): their
// inverses are then the Montgomery images of 1 / Zb, which the constraint kernel multiplies exactly.
// Local point i is the global evaluation point g_add + (i << log_g) (a residue
// class of the precision domain on a distributed prover; g_add = log_g = 0 on one GPU).
__global__ void r1cs_zb_kernel(const fe* __restrict__ lo, const fe* __restrict__ hi, uint32_t kb, uint64_t prec,
                               uint64_t g_add, uint32_t log_g,
                               const fe* __restrict__ xpub_m, uint32_t npub, fe xlast_m, fe unit, fe one_m,
                               fe* __restrict__ zb2, fe* __restrict__ zb3) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= prec) return;
  const fe x_m = pow_tab(lo, hi, kb, g_add + (i << log_g));
  fe acc = one_m;
  for (uint32_t k = 0; k < npub; ++k) acc = fe_mul(acc, fe_sub(x_m, xpub_m[k]));
  fe_store(zb2 + i, fe_mul(acc, unit));
  if (zb3) fe_store(zb3 + i, fe_mul(fe_sub(x_m, xlast_m), unit));  // (null: 1 / Zb3 is the shared column)
}

struct ConstraintArgs {
  const fe* col[9];      // K F0 F1 F2 S P IDX PIDX A, precision (local points) each
  const fe* inv_zb;      // inv Zb2 (precision)
  const fe* inv_zb3;     // inv Zb3 (precision): inv_zb + precision, or the shared column
  // tinv != null: inv Zb2 by partial fractions instead of inv_zb, sum_k pf_coef[k] tinv[i - pf_shift[k]]
  // over the shared table tinv[m] = 1 / (x_m - 1) (kInvXm1; zb2_partial_fractions)
  const fe* tinv;
  uint32_t n_pf;
  uint64_t pf_shift[8];
  fe pf_coef[8];
  const fe* interp2;     // canonical coefficients, low degree first
  const fe* interp3;
  const fe* lo;          // g2 tables
  const fe* hi;
  fe* rows;              // precision x 8 elements: rows (plane = 0) or 8 columns of `plane` elements
  uint64_t plane;
  int* err;
  uint64_t prec;            // points on this GPU (a power of two)
  uint64_t shift1, shift2;  // original_steps/3*skips, original_steps/3*2*skips (mod precision), in local points
  uint64_t back;            // the -skips shift in local points
  uint64_t g_add;           // local point i is global point g_add + (i << log_g)
  uint32_t log_g;
  uint32_t log_prec, kb, n2, n3;
  const Transcript* tr;  // r0, r1, r2 (device transcript)
  // inv(Z) at the points t = i mod 8 (multi_inv of Z, prove.rs:203; 0 for t = 0) as the
  // Montgomery images of inv(Z) R^k, k = 0, 1, 2: the constraint kernel forms some Q's scaled by
  // R^-k (one product fewer per conversion it skips) and undoes the scale in D = Q inv(Z).
  fe invz_m[3][8];
  int mont_cols;         // K, F0-F2 are Montgomery images (prepared circuits); inv Zb2/Zb3 always are
  uint32_t* leaf = nullptr;  // non-null: each row's Blake2s (the main tree's level 0, merkle_level0), 8 words
};

// Q1/Q2/Q3 (utils.rs:181-248, 344-376) -> D1..D3 (utils.rs:379-418), I2/I3
// evaluations (prove.rs:216-220), B2/B3 (utils.rs:477-524); one main-tree row
// (prove.rs:235-258) per thread.
// (3 workgroups per CU: the digit-basis products need ~170 VGPRs; at 4 waves per SIMD they spill, at the
// compiler's free choice of 180-217 VGPRs two waves per SIMD leave the loads uncovered:
// 1.94 ms before the digit basis, 1.73 ms with it at this bound, 1.96-1.98 ms at the others,
// profiles/r05_constraint_db_ab.txt)
__global__ __launch_bounds__(256, 3) void r1cs_constraint_kernel(ConstraintArgs a) {
  // The 24 inv(Z) R^k tables in LDS (a lane's t = i mod 8 picks its table): 76 words apart, so the 8
  // tables a wave reads at once start on distinct 4-bank groups.
  __shared__ __attribute__((aligned(16))) uint32_t izt[24 * 76];
  {
    const uint4* src = reinterpret_cast<const uint4*>(&a.tr->c_db[9][0]);
    for (uint32_t k = threadIdx.x; k < 24 * 18; k += blockDim.x)
      reinterpret_cast<uint4*>(izt)[(k / 18) * 19 + k % 18] = src[k];
    __syncthreads();
  }
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.prec) return;
  const uint64_t n = a.prec, mask = n - 1;
  const fe* K = a.col[0];
  const fe* F0 = a.col[1];
  const fe* F1 = a.col[2];
  const fe* F2 = a.col[3];
  const fe* S = a.col[4];
  const fe* Pc = a.col[5];
  const fe* IDX = a.col[6];
  const fe* PIDX = a.col[7];
  const fe* A = a.col[8];
  const uint64_t prev = (i + n - a.back) & mask;
  const uint64_t gi = a.g_add + (i << a.log_g);  // global evaluation point
  const fe r0 = a.tr->r0;
  const fe p = fe_load(Pc + i), s = fe_load(S + i), av = fe_load(A + i);
  const fe p_prev = fe_load(Pc + prev), a_prev = fe_load(A + prev);
  const fe p2 = fe_load(Pc + ((i + a.shift1) & mask)), p3 = fe_load(Pc + ((i + a.shift2) & mask));
  // Data x data products: a Montgomery product of two canonical values is x y R^-1, so each Q is
  // formed at a scale R^-k and D = Q inv(Z) takes the inv(Z) R^k constant (zero tests are
  // scale-free).  Prepared circuits hold K, F0-F2 as Montgomery images: their products are exact.
  const bool mc = a.mont_cols != 0;
  // Products by the proof's constants (r1, r2, R^-1, the a_k below) by the digit basis from the
  // transcript's tables (wave-uniform: scalar loads), each reduced once to canonical: the same values
  // as the Montgomery products by their images, at about half the instructions.
  const uint32_t* __restrict__ db_r1 = a.tr->r_db[0];
  const uint32_t* __restrict__ db_r2 = a.tr->r_db[1];
  const uint32_t* __restrict__ db_rinv = a.tr->c_db[0];
  auto cmul = [](const fe& x, const uint32_t* __restrict__ w) {  // x w mod p, canonical (x < 4p)
    fe y = fe_mul_db(x, w);
    fe_reduce_once(y);
    return y;
  };
  const fe k_s = fe_mul(fe_load(K + i), s), f1_p = fe_mul(fe_load(F1 + i), p_prev);
  const fe q1 = fe_mul(fe_load(F0 + i), fe_sub(fe_sub(mc ? p : cmul(p, db_rinv), f1_p), k_s));  // R^-(mc ? 0 : 2)
  const fe q2 = fe_mul(fe_load(F2 + i), fe_sub(cmul(p3, db_rinv), fe_mul(p, p2)));            // R^-(mc ? 1 : 2)
  const fe rs = cmul(s, db_r2);
  const fe nmr = fe_add(fe_add(r0, cmul(fe_load(IDX + i), db_r1)), rs);
  const fe dnm = fe_add(fe_add(r0, cmul(fe_load(PIDX + i), db_r1)), rs);
  const fe q3 = fe_sub(fe_mul(av, dnm), fe_mul(a_prev, nmr));                                // R^-1
  const uint32_t t = (uint32_t)(gi & 7);
  if (t == 0 && !(fe_is_zero(q1) && fe_is_zero(q2) && fe_is_zero(q3))) atomicOr(a.err, 1);
  auto iz = [&](uint32_t k) {  // the table of inv(Z) R^k at this t
    return static_cast<const uint32_t*>(__builtin_assume_aligned(izt + 76 * (8 * k + t), 16));
  };
  const fe d1 = cmul(q1, iz(mc ? 0 : 2)), d2 = cmul(q2, iz(mc ? 1 : 2)), d3 = cmul(q3, iz(1));
  // I2 / I3 at x = g2^i (Horner; the interpolants are canonical).
  const fe x_m = pow_tab(a.lo, a.hi, a.kb, gi);
  // (Horner from the leading coefficient: the first step's 0 * x + c is c itself)
  fe i2 = a.n2 ? a.interp2[a.n2 - 1] : fe_zero();
  for (uint32_t k = a.n2 ? a.n2 - 1 : 0; k-- > 0;) i2 = fe_add(fe_mul(i2, x_m), a.interp2[k]);
  fe i3 = a.n3 ? a.interp3[a.n3 - 1] : fe_zero();
  for (uint32_t k = a.n3 ? a.n3 - 1 : 0; k-- > 0;) i3 = fe_add(fe_mul(i3, x_m), a.interp3[k]);
  fe izb2;
  if (a.tinv) {  // (uniform)
    izb2 = fe_zero();
    bool root = false;  // x = x_k: Zb2 = 0, whose batch inverse is 0
    for (uint32_t k = 0; k < a.n_pf; ++k) {
      const uint64_t m = (i + n - a.pf_shift[k]) & mask;
      root = root || (m == 0 && a.g_add == 0);
      // a_k tinv (a Montgomery image times a canonical a_k: the image of the product), sum in [0, 2p)
      izb2 = fe_add_raw(izb2, fe_mul_db(fe_load(a.tinv + m), a.tr->c_db[1 + k]));
      fe_csub2p(izb2);
    }
    fe_reduce_once(izb2);
    if (root) izb2 = fe_zero();
  } else {
    izb2 = fe_load(a.inv_zb + i);
  }
  const fe izb3 = fe_load(a.inv_zb3 + i);
  const fe e2 = fe_sub(s, i2), e3 = fe_sub(av, i3);
  if (fe_is_zero(izb2) && !fe_is_zero(e2)) atomicOr(a.err, 2);
  if (fe_is_zero(izb3) && !fe_is_zero(e3)) atomicOr(a.err, 4);
  const fe b2 = fe_mul(e2, izb2), b3 = fe_mul(e3, izb3);  // (Montgomery images of the inverses: exact)
  // Row i = P|A|S|D1|D2|D3|B2|B3: contiguous (256 B), or column c at rows + c * plane + i
  const uint64_t cs = a.plane ? a.plane : 1;
  fe* row = a.plane ? a.rows + i : a.rows + 8 * i;
  fe_store(row + 0 * cs, p);
  fe_store(row + 1 * cs, av);
  fe_store(row + 2 * cs, s);
  fe_store(row + 3 * cs, d1);
  fe_store(row + 4 * cs, d2);
  fe_store(row + 5 * cs, d3);
  fe_store(row + 6 * cs, b2);
  fe_store(row + 7 * cs, b3);
  if (a.leaf) {  // (uniform) the main tree's leaf: Blake2s of the 256-B row, 4 blocks of two values each
    uint32_t h[8], m[16];
    b2s_init(h);
    auto block = [&](const fe& x, const fe& y, uint32_t t_bytes, bool last) {
#pragma unroll
      for (int w = 0; w < 8; ++w) {
        m[w] = x.w[w];
        m[8 + w] = y.w[w];
      }
      b2s_compress(h, m, t_bytes, 0, last);
    };
    block(p, av, 64, false);
    block(s, d1, 128, false);
    block(d2, d3, 192, false);
    block(b2, b3, 256, true);
    uint4* q = reinterpret_cast<uint4*>(a.leaf + 8 * i);
    q[0] = make_uint4(h[0], h[1], h[2], h[3]);
    q[1] = make_uint4(h[4], h[5], h[6], h[7]);
  }
}

struct LincombArgs {
  const fe* rows;        // the constraint kernel's rows (plane = 0) or columns (plane elements apart)
  uint64_t plane;
  fe* out;
  uint64_t prec;
  uint64_t g_add;        // local point i is global point g_add + (i << log_g)
  uint32_t log_g;
  const Transcript* tr;  // k and kx (device transcript)
  uint32_t* leaf = nullptr;  // non-null: each value's Blake2s (the L tree's level 0, merkle_level0), 8 words
};

// L = k0 D1 + k1 D2 + k2 D3 + k3 P + k4 P x^steps + k5 B2 + k6 B2 x^steps +
//     k7 B3 + k8 B3 x^steps + k9 A + k10 S (prove.rs:293-322).
__global__ __launch_bounds__(256) void r1cs_lincomb_kernel(LincombArgs a) {
  // Every product is data x a constant of the proof: the digit-basis product (fe_db.h) from the
  // transcript's tables, staged in LDS; the sum stays in [0, 2p) and is reduced once at the end.
  __shared__ __attribute__((aligned(16))) uint32_t tab[kLincombConsts * 72];
  for (uint32_t k = threadIdx.x; k < kLincombConsts * 18; k += blockDim.x)
    reinterpret_cast<uint4*>(tab)[k] = reinterpret_cast<const uint4*>(&a.tr->k_db[0][0])[k];
  __syncthreads();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.prec) return;
  const uint64_t cs = a.plane ? a.plane : 1;
  const fe* row = a.plane ? a.rows + i : a.rows + 8 * i;
  const uint64_t gi = a.g_add + (i << a.log_g);
  const fe p = fe_load(row + 0 * cs), av = fe_load(row + 1 * cs), s = fe_load(row + 2 * cs),
           d1 = fe_load(row + 3 * cs), d2 = fe_load(row + 4 * cs), d3 = fe_load(row + 5 * cs),
           b2 = fe_load(row + 6 * cs), b3 = fe_load(row + 7 * cs);
  const uint32_t t = (uint32_t)(gi & 7);
  auto T = [&](uint32_t c) { return static_cast<const uint32_t*>(__builtin_assume_aligned(tab + 72 * c, 16)); };
  auto add = [](fe& acc, const fe& x) {  // acc, x in [0, 2p): acc + x < 4p < 2^256, back to [0, 2p)
    acc = fe_add_raw(acc, x);
    fe_csub2p(acc);
  };
  fe acc = fe_mul_db(d1, T(0));           // k0 D1
  add(acc, fe_mul_db(d2, T(1)));          // k1 D2
  add(acc, fe_mul_db(d3, T(2)));          // k2 D3
  add(acc, fe_mul_db(p, T(5 + 3 * t)));   // (k3 + k4 x^steps) P
  add(acc, fe_mul_db(b2, T(6 + 3 * t)));  // (k5 + k6 x^steps) B2
  add(acc, fe_mul_db(b3, T(7 + 3 * t)));  // (k7 + k8 x^steps) B3
  add(acc, fe_mul_db(av, T(3)));          // k9 A
  add(acc, fe_mul_db(s, T(4)));           // k10 S
  fe_reduce_once(acc);
  fe_store(a.out + i, acc);
  if (a.leaf) {  // (uniform) the L tree's leaf: Blake2s of the 32-B value
    uint32_t h[8], m[16];
    b2s_init(h);
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      m[w] = acc.w[w];
      m[8 + w] = 0;
    }
    b2s_compress(h, m, 32, 0, true);
    uint4* q = reinterpret_cast<uint4*>(a.leaf + 8 * i);
    q[0] = make_uint4(h[0], h[1], h[2], h[3]);
    q[1] = make_uint4(h[4], h[5], h[6], h[7]);
  }
}

// ---- host helpers -----------------------------------------------------------

// Z(g2^i) = (g2^steps)^(i mod 8) - 1; its inverse with 0 -> 0 (prove.rs:128-129, 203), times
// R^k for the kernel's R^-k-scaled Q's.
static void set_inv_z(ConstraintArgs& ca, const HostFp& g2, uint64_t steps) {
  const FieldHost& F = FieldHost::get();
  const HostFp rv = F.from_canonical(F.one().v);  // the field element R = 2^256 mod p
  const HostFp w8 = F.pow_u64(g2, steps);
  HostFp wt = F.one();
  for (int t = 0; t < 8; ++t) {
    const HostFp z = F.sub(wt, F.one());
    HostFp iz = FieldHost::eq(z, F.zero()) ? F.zero() : F.inv(z);
    for (int k = 0; k < 3; ++k) {
      ca.invz_m[k][t] = to_dev(iz);
      iz = F.mul(iz, rv);
    }
    wt = F.mul(wt, w8);
  }
}

// log2_ceil, utils.rs:14-23.
static uint32_t log2_ceil_ref(size_t v) {
  uint32_t l = 1;
  while (v > 1) {
    v /= 2;
    ++l;
  }
  return l;
}

static HostFp host_fe(const uint64_t* c) { return FieldHost::get().from_canonical(c); }

// c = a * b (coefficient lists, low degree first); the output coefficients are split over the
// host workers when the product is large.
static std::vector<HostFp> poly_mul(const std::vector<HostFp>& a, const std::vector<HostFp>& b) {
  const FieldHost& F = FieldHost::get();
  std::vector<HostFp> c(a.size() + b.size() - 1, F.zero());
  const size_t nc = c.size();
  const unsigned T = a.size() * b.size() > 20000 ? host_threads() : 1;
  host_parallel(T, [&](unsigned t) {
    for (size_t k = t; k < nc; k += T) {
      const size_t lo = k >= b.size() ? k - (b.size() - 1) : 0, hi = k < a.size() ? k : a.size() - 1;
      HostFp acc = F.zero();
      for (size_t i = lo; i <= hi; ++i) acc = F.add(acc, F.mul(a[i], b[k - i]));
      c[k] = acc;
    }
  });
  return c;
}

// lagrange_interp (fri/src/poly_utils.rs:409-439): the unique interpolant, n coefficients, Montgomery on
// the host.  The same polynomial as the reference's, by another O(n^2) route that parallelises:
//   root = prod (X - x_i) by a product tree (leaves on the host workers),
//   den_i = root'(x_i) = prod_{j != i} (x_i - x_j), one batch inverse (0 -> 0, as F.inv),
//   b = sum_i (y_i / den_i) root / (X - x_i), each worker summing its share of the i.
// (A public-input list of 1,062 wires, bits.r1cs, took 70 ms serially.)
std::vector<HostFp> lagrange_interp(const std::vector<HostFp>& xs, const std::vector<HostFp>& ys) {
  const FieldHost& F = FieldHost::get();
  const size_t n = xs.size();
  if (n == 0) return {};
  const unsigned T = n >= 64 ? host_threads() : 1;
  // Product tree: T leaf products, then pairwise merges.
  std::vector<std::vector<HostFp>> parts(T);
  host_parallel(T, [&](unsigned t) {
    const size_t i0 = n * t / T, i1 = n * (t + 1) / T;
    std::vector<HostFp> r(1, F.one());
    for (size_t i = i0; i < i1; ++i) {
      std::vector<HostFp> nxt(r.size() + 1, F.zero());
      for (size_t j = 0; j < r.size(); ++j) {
        nxt[j + 1] = F.add(nxt[j + 1], r[j]);
        nxt[j] = F.sub(nxt[j], F.mul(r[j], xs[i]));
      }
      r.swap(nxt);
    }
    parts[t] = std::move(r);
  });
  while (parts.size() > 1) {
    std::vector<std::vector<HostFp>> next;
    for (size_t i = 0; i + 1 < parts.size(); i += 2) next.push_back(poly_mul(parts[i], parts[i + 1]));
    if (parts.size() & 1) next.push_back(std::move(parts.back()));
    parts.swap(next);
  }
  const std::vector<HostFp>& root = parts[0];  // n + 1 coefficients, root[n] = 1
  std::vector<HostFp> droot(n);
  for (size_t d = 1; d <= n; ++d) droot[d - 1] = F.mul(root[d], F.from_u64(d));
  std::vector<HostFp> den(n);
  host_parallel(T, [&](unsigned t) {
    for (size_t i = t; i < n; i += T) {
      HostFp y = F.zero();
      for (size_t d = n; d-- > 0;) y = F.add(F.mul(y, xs[i]), droot[d]);
      den[i] = y;
    }
  });
  // Batch inverse with zeros kept (F.inv(0) = 0).
  std::vector<HostFp> pre(n);
  HostFp acc = F.one();
  for (size_t i = 0; i < n; ++i) {
    pre[i] = acc;
    if (!FieldHost::eq(den[i], F.zero())) acc = F.mul(acc, den[i]);
  }
  HostFp inv_acc = F.inv(acc);
  std::vector<HostFp> s(n);
  for (size_t i = n; i-- > 0;) {
    if (FieldHost::eq(den[i], F.zero())) {
      s[i] = F.zero();
      continue;
    }
    s[i] = F.mul(ys[i], F.mul(inv_acc, pre[i]));
    inv_acc = F.mul(inv_acc, den[i]);
  }
  std::vector<std::vector<HostFp>> partial(T, std::vector<HostFp>(n, F.zero()));
  host_parallel(T, [&](unsigned t) {
    std::vector<HostFp>& b = partial[t];
    std::vector<HostFp> num(n);
    for (size_t i = t; i < n; i += T) {
      HostFp carry = root[n];
      num[n - 1] = carry;
      for (size_t d = n - 1; d >= 1; --d) {  // root / (X - x_i), synthetic division
        carry = F.add(root[d], F.mul(carry, xs[i]));
        num[d - 1] = carry;
      }
      for (size_t j = 0; j < n; ++j) b[j] = F.add(b[j], F.mul(num[j], s[i]));
    }
  });
  std::vector<HostFp> b = std::move(partial[0]);
  for (unsigned t = 1; t < T; ++t)
    for (size_t j = 0; j < n; ++j) b[j] = F.add(b[j], partial[t][j]);
  return b;
}

// Carves the proof's buffers out of the context's grow-only arena (no
// hipMalloc/hipFree per proof).
struct Carve {
  size_t off = 0;
  std::vector<std::pair<void**, size_t>> req;
  template <class T>
  void add(T** p, size_t count) {
    req.push_back({(void**)p, off});
    off += ((count ? count : 1) * sizeof(T) + 255) & ~(size_t)255;
  }
  stark_status commit(stark_ctx* ctx, DevBuf& arena) {
    stark_status st = ensure_buf(ctx, arena, off);
    if (st != STARK_OK) return st;
    for (auto& r : req) *r.first = (uint8_t*)arena.ptr + r.second;
    return STARK_OK;
  }
};


static unsigned blocks_for(uint64_t n, unsigned t = 256) { return (unsigned)((n + t - 1) / t); }

// In-place inclusive product scan of n Montgomery values; canonical copy to `canon` if non-null.
// Inclusive product scans of the arrays a.v[0 .. count) (n elements each, in place, Montgomery images), their
// canonical values into a.canon[k] where given; a.tot[k] holds ceil(n / kScanBlock) block products.
static stark_status product_scan(stark_ctx* ctx, const ScanArrays& a, uint32_t count, uint64_t n, const Mont& mc,
                                 hipStream_t s) {
  const uint32_t nb = (uint32_t)((n + kScanBlock - 1) / kScanBlock);
  hipLaunchKernelGGL(scan_block_kernel, dim3(nb, count), dim3(256), 0, s, a, n, mc.one);
  hipLaunchKernelGGL(scan_tot_kernel, dim3(1, count), dim3(256), 0, s, a, nb, mc.one);
  hipLaunchKernelGGL(scan_apply_kernel, dim3(blocks_for(n), count), dim3(256), 0, s, a, n, mc.unit);
  STARK_HIP(ctx, hipGetLastError());
  return STARK_OK;
}

// LDE of `batch` step columns (in place in `coef`, destroyed) into `out`
// (batch x precision): inv_best_fft(., g1) then best_fft(., g2) (prove.rs:100-101).
// coef[c][k] *= g2^(r k) for the batch of step columns (coset shift of the LDE).
__global__ void coset_scale_kernel(fe* __restrict__ coef, uint32_t log_steps, uint64_t total, const fe* __restrict__ lo,
                                   const fe* __restrict__ hi, uint32_t kb, uint64_t r, uint64_t prec_mask) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total) return;
  const uint64_t k = g & (((uint64_t)1 << log_steps) - 1);
  fe_store(coef + g, fe_mul(fe_load(coef + g), pow_tab(lo, hi, kb, (r * k) & prec_mask)));
}

// The values of the step columns' polynomials at the points r + 2^log_g j of the precision
// domain (j < P = precision >> log_g): iNTT(steps, g1), coefficients scaled by g2^(r k), then a
// P-point NTT with root h = g2^(2^log_g) over the zero-padded coefficients (degree < steps <= P).
// log_g = r = 0 is the plain LDE of prove.rs:100-101.  coef is destroyed.
static stark_status coset_lde(stark_ctx* ctx, fe* coef, uint32_t batch, fe* out, uint32_t log_steps,
                              uint32_t log_prec, uint32_t log_g, uint32_t r, const Twiddles& tw_g1_inv,
                              const Twiddles& tw_g2, const Twiddles& tw_h, hipStream_t s) {
  STARK_TRY(ntt_device(ctx, coef, log_steps, batch, tw_g1_inv, true, s));
  if (r) {
    const uint64_t total = (uint64_t)batch << log_steps;
    hipLaunchKernelGGL(coset_scale_kernel, dim3(blocks_for(total)), dim3(256), 0, s, coef, log_steps, total,
                       tw_g2.d_lo, tw_g2.d_hi, tw_g2.kb, (uint64_t)r, ((uint64_t)1 << log_prec) - 1);
    STARK_HIP(ctx, hipGetLastError());
  }
  // best_fft's zero padding (fft.rs:327-357) is implicit: the first pass reads the steps coefficients only.
  const uint32_t log_p = log_prec - log_g;
  return ntt_device_from(ctx, coef, log_p - log_steps, out, log_p, batch, tw_h, false, s);
}

static stark_status lde(stark_ctx* ctx, fe* coef, uint32_t batch, fe* out, uint32_t log_steps, uint32_t log_prec,
                        const Twiddles& tw_g1_inv, const Twiddles& tw_g2, hipStream_t s) {
  return coset_lde(ctx, coef, batch, out, log_steps, log_prec, 0, 0, tw_g1_inv, tw_g2, tw_g2, s);
}

// tag 0: IDX[i] = i; tag > 0: F0[i] = 1 for i < tag (calc_flags' flag0, run.rs:283-308), 0 after.
__global__ void const_column_kernel(fe* __restrict__ out, uint64_t n, uint64_t tag) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) fe_store(out + i, fe_from_u64(tag ? (i < tag ? 1 : 0) : i));
}

// Columns of a proof that depend on its size only, over the rank's points r + 2^log_g j (the whole
// domain for log_g = r = 0); each is computed on a context's first proof of that size and shared by
// every later one:
//   kExtIdx: ext_indices (prove.rs:160-163), the extension of IDX[i] = i (coset_lde with log_g, r);
//   kExtF0:  the extension of F0, which calc_flags (run.rs:283-308) sets to 1 on each of the os trace
//            rows (zero-padded to steps);
//   kInvZb3: 1 / Zb3 = 1 / (x - x_last) (utils.rs:466-474; x_last = g2^((steps - 1) skips) depends on
//            the size alone), 0 at x_last as multi_inv gives it, as Montgomery images (r1cs_zb_kernel);
//   kInvXm1: 1 / (x - 1), the same way (0 at x = 1): the table of 1 / Zb2's partial fractions.
// Call before the proof enqueues work on `s`: a first call synchronises s.  An IDX extension larger
// than the cache cap lives in a per-context buffer for this proof only; the others are not built
// when they cannot be cached (*out = nullptr: the caller computes them as part of the proof).
//   kSpotF0 / kSpotIdx: F0's / IDX's first forward pass, transposed (ntt_first_pass_tmajor: the verifier's
//            cold build, circuit_spot_values; world 1), not built when it cannot be cached.
enum : uint32_t { kExtIdx = 0, kExtF0 = 1, kInvZb3 = 2, kInvXm1 = 3, kSpotF0 = 4, kSpotIdx = 5 };
static stark_status ext_const_column(stark_ctx* ctx, uint32_t kind, uint64_t os, uint32_t log_steps,
                                     uint32_t log_prec, uint32_t log_g, uint32_t r, const Twiddles& tw_g1_inv,
                                     const Twiddles& tw_g2, const Twiddles& tw_h, hipStream_t s, const fe** out) {
  const bool spot = kind == kSpotF0 || kind == kSpotIdx;
  if (spot && (log_g || r)) return STARK_ERR_BAD_ARG;
  const uint64_t tag = (kind == kExtF0 || kind == kSpotF0) ? os : 0;
  const auto key = std::make_tuple(kind, log_steps, log_prec, log_g, r, tag);
  auto it = ctx->ext_idx.find(key);
  if (it != ctx->ext_idx.end()) {
    it->second.used = ++ctx->cache_clock;
    *out = (const fe*)it->second.ptr;
    return STARK_OK;
  }
  const uint64_t steps = (uint64_t)1 << log_steps, P = (uint64_t)1 << (log_prec - log_g);
  // Counted in the context's capped cache (stark_ctx_set_cache_limit).
  const bool cached = cache_reserve(ctx, P * sizeof(fe), true);
  void *col = nullptr, *coef = nullptr;
  if (cached) {
    if (hipMalloc(&col, P * sizeof(fe)) != hipSuccess) {
      hipGetLastError();
      if (kind != kExtIdx) {
        *out = nullptr;
        return STARK_OK;
      }
      return STARK_ERR_OOM;
    }
    ctx->ext_idx[key] = CacheBuf{col, P * sizeof(fe), ++ctx->cache_clock};  // counted while it is built
  } else if (kind != kExtIdx) {
    *out = nullptr;
    return STARK_OK;
  } else {
    STARK_TRY(ensure_buf(ctx, ctx->ext_idx_tmp, P * sizeof(fe)));
    col = ctx->ext_idx_tmp.ptr;
  }
  auto drop = [&] {
    if (cached) {
      ctx->ext_idx.erase(key);
      hipFree(col);
    }
  };
  const bool inv = kind == kInvZb3 || kind == kInvXm1;
  const uint64_t tmp_n = inv ? 2 * P : steps;
  if (hipMalloc(&coef, tmp_n * sizeof(fe)) != hipSuccess) {
    hipGetLastError();
    drop();
    return STARK_ERR_OOM;
  }
  stark_status st = STARK_OK;
  if (inv) {  // r1cs_zb_kernel with no public points: Zb2 = 1 (unused), x - c in the second half
    const FieldHost& F = FieldHost::get();
    const Mont mc = mont();
    const uint64_t prec = (uint64_t)1 << log_prec, skips = prec >> log_steps;
    const fe c = kind == kInvZb3 ? to_dev(F.pow_u64(tw_g2.root, prec - skips)) : mc.one;
    fe* z = (fe*)coef;
    hipLaunchKernelGGL(r1cs_zb_kernel, dim3(blocks_for(P)), dim3(256), 0, s, tw_g2.d_lo, tw_g2.d_hi, tw_g2.kb, P,
                       (uint64_t)r, log_g, (const fe*)nullptr, 0u, c, mc.rinv, mc.one, z, z + P);
    st = hipGetLastError() == hipSuccess ? STARK_OK : STARK_ERR_HIP;
    if (st == STARK_OK) st = multi_inv_device(ctx, z + P, (fe*)col, P, s);
  } else {
    hipLaunchKernelGGL(const_column_kernel, dim3(blocks_for(steps)), dim3(256), 0, s, (fe*)coef, steps, tag);
    st = hipGetLastError() == hipSuccess ? STARK_OK : STARK_ERR_HIP;
    if (st == STARK_OK && spot) {
      uint32_t log_t = 0;
      st = ntt_device(ctx, (fe*)coef, log_steps, 1, tw_g1_inv, true, s);
      if (st == STARK_OK)
        st = ntt_first_pass_tmajor(ctx, (fe*)coef, log_prec - log_steps, (fe*)col, log_prec, 1, tw_g2, s, &log_t);
    } else if (st == STARK_OK) {
      st = coset_lde(ctx, (fe*)coef, 1, (fe*)col, log_steps, log_prec, log_g, r, tw_g1_inv, tw_g2, tw_h, s);
    }
  }
  if (hipStreamSynchronize(s) != hipSuccess && st == STARK_OK) st = STARK_ERR_HIP;
  hipFree(coef);
  if (st != STARK_OK) {
    drop();
    return st;
  }
  *out = (const fe*)col;
  return STARK_OK;
}

// The size-only columns of one proof (ext_const_column), taken in one place: every later reservation
// may evict an earlier column, so each is looked up again once all are taken (IDX last: its pointer is
// always valid).  want_f0: the flags are a trace builder's (F0 = 1 on the os rows).
struct SharedCols {
  const fe *idx = nullptr, *f0 = nullptr, *izb3 = nullptr, *tinv = nullptr;
};
static stark_status shared_columns(stark_ctx* ctx, bool want_f0, uint64_t os, uint32_t log_steps, uint32_t log_prec,
                                   uint32_t log_g, uint32_t r, const Twiddles& tw_g1_inv, const Twiddles& tw_g2,
                                   const Twiddles& tw_h, hipStream_t s, SharedCols& o) {
  STARK_TRY(ext_const_column(ctx, kInvZb3, 0, log_steps, log_prec, log_g, r, tw_g1_inv, tw_g2, tw_h, s, &o.izb3));
  STARK_TRY(ext_const_column(ctx, kInvXm1, 0, log_steps, log_prec, log_g, r, tw_g1_inv, tw_g2, tw_h, s, &o.tinv));
  if (want_f0)
    STARK_TRY(ext_const_column(ctx, kExtF0, os, log_steps, log_prec, log_g, r, tw_g1_inv, tw_g2, tw_h, s, &o.f0));
  STARK_TRY(ext_const_column(ctx, kExtIdx, 0, log_steps, log_prec, log_g, r, tw_g1_inv, tw_g2, tw_h, s, &o.idx));
  auto live = [&](uint32_t kind, uint64_t tag) {
    return ctx->ext_idx.count(std::make_tuple(kind, log_steps, log_prec, log_g, r, tag)) != 0;
  };
  if (o.izb3 && !live(kInvZb3, 0)) o.izb3 = nullptr;
  if (o.tinv && !live(kInvXm1, 0)) o.tinv = nullptr;
  if (o.f0 && !live(kExtF0, os)) o.f0 = nullptr;
  return STARK_OK;
}

// 1 / Zb2 = 1 / prod_k (x - x_k) (utils.rs:438-455) by partial fractions: sum_k c_k / (x - x_k) with
// c_k = 1 / prod_(j != k) (x_k - x_j), and 1 / (x - x_k) = x_k^-1 / (x / x_k - 1), where x / x_k is the
// domain point e_k = skips j_k places back, so the term is a_k tinv[i - e_k / 2^log_g] with
// a_k = c_k / x_k (Montgomery, like the table).  The same field value as the batch inverse, bit for
// bit (both canonical); at x = x_k the kernel gives 0 as the batch inverse does.  Up to 8 distinct
// points (false otherwise: the proof takes the batch inverse).
static bool zb2_partial_fractions(const HostFp& g2, uint64_t prec, uint64_t skips, uint32_t log_g,
                                  const size_t* public_first_indices, size_t n_pfi, ConstraintArgs& ca) {
  const FieldHost& F = FieldHost::get();
  constexpr size_t kMaxPf = sizeof(ca.pf_shift) / sizeof(ca.pf_shift[0]);
  if (n_pfi == 0 || n_pfi > kMaxPf) return false;
  std::vector<HostFp> xs(n_pfi);
  for (size_t k = 0; k < n_pfi; ++k) {
    const uint64_t e = (skips * (uint64_t)public_first_indices[2 * k + 1]) % prec;  // a multiple of skips
    xs[k] = F.pow_u64(g2, e);
    ca.pf_shift[k] = e >> log_g;
  }
  for (size_t k = 0; k < n_pfi; ++k) {
    HostFp c = xs[k];
    for (size_t j = 0; j < n_pfi; ++j) {
      if (j == k) continue;
      const HostFp d = F.sub(xs[k], xs[j]);
      if (FieldHost::eq(d, F.zero())) return false;  // a repeated point
      c = F.mul(c, d);
    }
    ca.pf_coef[k] = to_dev(F.inv(c));
  }
  ca.n_pf = (uint32_t)n_pfi;
  return true;
}

// The host part of the transcript's c_db: R^-1, the partial-fraction coefficients a_k and the 24 inv(Z) R^k
// constants (ca.pf_coef and ca.invz_m hold Montgomery images, which are the HostFp representation itself:
// the tables are of the values the Montgomery products multiply by).  A pageable copy: the
// runtime stages it before returning, so the table may live on this stack.
static Pow32 pow32() {
  const FieldHost& F = FieldHost::get();
  Pow32 p;
  HostFp x = F.one();
  const HostFp t = F.from_u64((uint64_t)1 << 32);
  for (int i = 0; i < 8; ++i) {
    p.m[i] = to_dev(x);
    x = F.mul(x, t);
  }
  return p;
}

static stark_status upload_constraint_tables(stark_ctx* ctx, Transcript* d_tr, const ConstraintArgs& ca,
                                             hipStream_t s) {
  const FieldHost& F = FieldHost::get();
  // built in pinned slot 4 (its first kPinned4ConstsOff bytes), so the copy is asynchronous
  static_assert(sizeof(uint32_t) * 33 * 72 <= kPinned4ConstsOff, "pinned slot 4 layout");
  void* pin = nullptr;
  STARK_TRY(ctx_pinned(ctx, 4, kPinned4ConstsOff, &pin));
  uint32_t(&t)[33][72] = *reinterpret_cast<uint32_t(*)[33][72]>(pin);
  db_table(F.inv(F.pow_u64(F.from_u64(2), 256)), t[0]);  // R^-1
  const uint32_t n = ca.tinv ? ca.n_pf : 0;
  for (uint32_t k = 0; k < 8; ++k) {
    HostFp c;
    if (k < n) memcpy(c.v, &ca.pf_coef[k], 32);
    else c = F.zero();
    db_table(c, t[1 + k]);
  }
  for (int k = 0; k < 3; ++k)
    for (int u = 0; u < 8; ++u) {
      HostFp c;
      memcpy(c.v, &ca.invz_m[k][u], 32);
      db_table(c, t[9 + 8 * k + u]);
    }
  STARK_HIP(ctx, hipMemcpyAsync(&d_tr->c_db[0][0], &t[0][0], sizeof t, hipMemcpyHostToDevice, s));
  return STARK_OK;
}

static stark_status ext_index_column(stark_ctx* ctx, uint32_t log_steps, uint32_t log_prec, uint32_t log_g,
                                     uint32_t r, const Twiddles& tw_g1_inv, const Twiddles& tw_g2,
                                     const Twiddles& tw_h, hipStream_t s, const fe** out) {
  return ext_const_column(ctx, kExtIdx, 0, log_steps, log_prec, log_g, r, tw_g1_inv, tw_g2, tw_h, s, out);
}

// The proof's roots (prove.rs:71-94): g2 = 7^((p-1)/precision), g1 = g2^skips = xs[skips], and
// h = g2^world (the generator of one rank's residue class of the domain), with the twiddle
// tables of g2, g1^-1 (the LDE's iNTT) and h.
struct ProofRoots {
  HostFp g2;
  uint64_t g2c[4];
  const Twiddles *tw2 = nullptr, *tw1i = nullptr, *twh = nullptr;
};

static stark_status proof_roots(stark_ctx* ctx, uint32_t log_steps, uint32_t log_prec, uint32_t world,
                                ProofRoots& R) {
  const FieldHost& F = FieldHost::get();
  uint64_t pm1[4];  // (p - 1) / precision
  memcpy(pm1, FieldHost::kP, 32);
  pm1[0] -= 1;
  for (uint32_t k = 0; k < log_prec; ++k)
    for (int l = 0; l < 4; ++l) pm1[l] = (pm1[l] >> 1) | (l < 3 ? pm1[l + 1] << 63 : 0);
  R.g2 = F.pow(F.from_u64(7), pm1, 4);
  uint32_t log_g = 0;
  while ((1u << log_g) < world) ++log_g;
  uint64_t g1ic[4], hc[4];
  F.to_canonical(R.g2, R.g2c);
  F.to_canonical(F.inv(F.pow_u64(R.g2, (uint64_t)1 << (log_prec - log_steps))), g1ic);
  F.to_canonical(F.pow_u64(R.g2, world), hc);
  STARK_TRY(get_twiddles(ctx, R.g2c, log_prec, &R.tw2));
  STARK_TRY(get_twiddles(ctx, g1ic, log_steps, &R.tw1i));
  STARK_TRY(get_twiddles(ctx, hc, log_prec - log_g, &R.twh));
  return STARK_OK;
}

// The proof's host-side constants (utils.rs:421-474): the boundary points x_k = g2^(skips w_k) of
// the public wires' first uses (Montgomery, for Zb2), the coefficients of the interpolant I2
// through (x_k, public value) and of I3 through (x_last, 1) (canonical): 2 n_pfi + 1 elements.
static std::vector<fe> boundary_consts(const HostFp& g2, uint64_t prec, uint64_t skips, const uint64_t* public_wires,
                                       const size_t* public_first_indices, size_t n_pfi, HostFp* x_last_out) {
  const FieldHost& F = FieldHost::get();
  const HostFp x_last = F.pow_u64(g2, prec - skips);
  std::vector<HostFp> xv(n_pfi), yv(n_pfi);
  for (size_t i = 0; i < n_pfi; ++i) {
    xv[i] = F.pow_u64(g2, skips * public_first_indices[2 * i + 1]);
    yv[i] = host_fe(public_wires + 4 * public_first_indices[2 * i]);
  }
  const std::vector<HostFp> interp2 = lagrange_interp(xv, yv);
  const std::vector<HostFp> interp3 = lagrange_interp({x_last}, {F.one()});
  auto canon_fe = [&](const HostFp& x) {
    uint64_t c[4];
    F.to_canonical(x, c);
    fe v;
    for (int k = 0; k < 4; ++k) {
      v.w[2 * k] = (uint32_t)c[k];
      v.w[2 * k + 1] = (uint32_t)(c[k] >> 32);
    }
    return v;
  };
  std::vector<fe> h(2 * n_pfi + 2);
  for (size_t i = 0; i < n_pfi; ++i) {
    h[i] = to_dev(xv[i]);
    h[n_pfi + i] = canon_fe(interp2[i]);
  }
  h[2 * n_pfi] = canon_fe(interp3[0]);
  *x_last_out = x_last;
  return h;
}

static stark_status prove_r1cs(stark_ctx* ctx, const uint64_t* witness_trace, const uint64_t* computational_trace,
                               size_t os, const uint64_t* public_wires, size_t n_public,
                               const size_t* public_first_indices, size_t n_pfi, const size_t* permuted_indices,
                               const uint64_t* coefficients, const uint64_t* flag0, const uint64_t* flag1,
                               const uint64_t* flag2, const uint8_t* flag_bytes, size_t n_constraints, size_t n_wires,
                               stark_r1cs_proof** out, const fe* pre = nullptr, bool dev_in = false) {
  // dev_in: every column, the flag bytes and the permutation are device pointers (one pack launch).
  // pre != nullptr: the circuit's LDE columns K F0 F1 F2 IDX PIDX (precision each) and the
  // inverses of Zb2, Zb3 (2 x precision), prepared once per circuit (stark_r1cs_circuit_new);
  // only S, P and A are extended here.
  PhaseClock clk("mk_r1cs_proof");
  const FieldHost& F = FieldHost::get();
  hipStream_t s = ctx->stream;
  // prove.rs:30-53
  if (os > 3 * n_constraints * n_wires || os % 3 != 0) return STARK_ERR_BAD_ARG;
  if (os < 5) return STARK_ERR_BAD_LENGTH;  // the reference's steps/log_steps disagree below 8 steps
  const uint32_t log_steps = log2_ceil_ref(os - 1);
  const uint32_t log_prec = log_steps + kLogExtensionFactor;
  // get_pseudorandom_indices(_, precision, ...) asserts precision < 2^24 (fri/src/utils.rs:88), first reached
  // when r is derived (utils.rs:279); the reference cannot prove larger traces.
  if (log_prec >= 24) return STARK_ERR_BAD_LENGTH;
  const uint64_t steps = (uint64_t)1 << log_steps, prec = (uint64_t)1 << log_prec;
  const uint64_t skips = prec / steps;
  for (size_t i = 0; i < n_pfi; ++i)
    if (public_first_indices[2 * i] >= n_public || public_first_indices[2 * i + 1] >= steps) return STARK_ERR_BAD_ARG;

  // Roots (prove.rs:71-94): g2 = 7^((p-1)/precision), g1 = g2^8.
  ProofRoots roots;
  STARK_TRY(proof_roots(ctx, log_steps, log_prec, 1, roots));
  const HostFp g2 = roots.g2;
  const uint64_t* g2c = roots.g2c;
  const Twiddles* tw2 = roots.tw2;
  const Twiddles* tw1i = roots.tw1i;
  const Mont mc = mont();
  // The shared size-only columns (prepared circuits carry their own): IDX's extension; F0's whenever
  // the flags are the trace builder's (flag bytes, calc_flags run.rs:283-308: 1 on the os rows), so only
  // K F1 F2 S P PIDX are extended here; 1 / Zb3; and the table that gives 1 / Zb2 by partial fractions,
  // so the proof has no batch inverse over the domain at all (zb2_partial_fractions).
  SharedCols sc;
  if (!pre)
    STARK_TRY(shared_columns(ctx, flag_bytes != nullptr, os, log_steps, log_prec, 0, 0, *tw1i, *tw2, *tw2, s, sc));
  const fe *idx_ext = sc.idx, *f0_ext = sc.f0, *izb3 = sc.izb3;
  ConstraintArgs ca;
  ca.tinv = nullptr;
  if (sc.tinv && izb3 && zb2_partial_fractions(g2, prec, skips, 0, public_first_indices, n_pfi, ca)) ca.tinv = sc.tinv;

  fe *raw, *wcopy, *cols, *nmr, *dnm, *tot, *dnm_c, *inv_dnm, *zb, *inv_zb, *consts, *rows, *lvals;
  uint64_t* perm;
  uint64_t* acc_leaves;
  Transcript* d_tr;
  const uint32_t nb = (uint32_t)((steps + kScanBlock - 1) / kScanBlock);
  Carve cv;
  cv.add(&raw, 7 * steps);  // K F0 F1 F2 S P PIDX (then A's coefficients reuse K's slot)
  cv.add(&wcopy, steps);
  cv.add(&perm, steps);
  cv.add(&acc_leaves, 5 * steps);
  cv.add(&cols, 8 * prec);  // the extensions of K F0 F1 F2 S P PIDX A (IDX's is shared: idx_ext)
  cv.add(&nmr, steps);
  cv.add(&dnm, steps);
  cv.add(&tot, 2 * (size_t)nb);
  cv.add(&dnm_c, steps);
  cv.add(&inv_dnm, steps);
  cv.add(&zb, 2 * prec);
  cv.add(&inv_zb, 2 * prec);
  cv.add(&consts, 2 * n_pfi + 2);
  cv.add(&rows, 8 * prec);
  cv.add(&lvals, prec);
  cv.add(&d_tr, 1);
  STARK_TRY(cv.commit(ctx, ctx->r1cs_arena));

  // Interpolants and boundary points (utils.rs:421-474), host side (#pub points).
  HostFp x_last;
  // alive until the proof's final synchronisation
  const std::vector<fe> h = boundary_consts(g2, prec, skips, public_wires, public_first_indices, n_pfi, &x_last);
  {  // through pinned slot 4 (an asynchronous copy; a pageable one blocks the host)
    uint8_t* pin = nullptr;
    STARK_TRY(ctx_pinned(ctx, 4, kPinned4ConstsOff + h.size() * sizeof(fe), (void**)&pin));
    memcpy(pin + kPinned4ConstsOff, h.data(), h.size() * sizeof(fe));
    STARK_HIP(ctx, hipMemcpyAsync(consts, pin + kPinned4ConstsOff, h.size() * sizeof(fe), hipMemcpyHostToDevice, s));
  }
  // Upload the six value columns, zero tails (prove.rs:59-69; inv_best_fft pads the flags).  The
  // inputs may be host or device pointers (the device trace builder's columns): hipMemcpyDefault.
  const uint64_t* src[6] = {coefficients, flag0, flag1, flag2, witness_trace, computational_trace};
  const bool pack = dev_in && !pre;
  if (pack) {
    if (!flag_bytes && (!flag0 || !flag1 || !flag2)) return STARK_ERR_BAD_ARG;
    PackArgs pa;
    for (int c = 0; c < 6; ++c) pa.col[c] = (const fe*)src[c];
    pa.fb = flag_bytes;
    pa.perm_in = (const uint64_t*)permuted_indices;
    pa.os = os;
    pa.steps = steps;
    pa.raw = raw;
    pa.wcopy = wcopy;
    pa.perm = perm;
    static_assert(sizeof(Transcript) % 4 == 0, "transcript words");
    pa.tr = (uint32_t*)d_tr;
    pa.tr_words = (uint32_t)(sizeof(Transcript) / 4);
    pa.k_slot = f0_ext ? 1 : 0;
    hipLaunchKernelGGL(r1cs_pack_kernel, dim3(blocks_for(std::max<uint64_t>(steps, pa.tr_words))), dim3(256), 0, s,
                       pa);
    STARK_HIP(ctx, hipGetLastError());
  }
  for (int c = pre ? 4 : 0; c < 6 && !pack; ++c) {
    if (!(flag_bytes && c >= 1 && c <= 3))
      STARK_HIP(ctx, hipMemcpyAsync(raw + c * steps, src[c], os * sizeof(fe), hipMemcpyDefault, s));
    if (steps > os) STARK_HIP(ctx, hipMemsetAsync(raw + c * steps + os, 0, (steps - os) * sizeof(fe), s));
  }
  if (flag_bytes && !pre && !pack) {  // 0/1 flags as bytes (the trace builder's compact form), widened on the GPU
    uint8_t* d_fb = (uint8_t*)zb;  // zb is free until the Zb kernel
    STARK_HIP(ctx, hipMemcpyAsync(d_fb, flag_bytes, 3 * os, hipMemcpyDefault, s));
    hipLaunchKernelGGL(r1cs_flags_kernel, dim3(blocks_for(3 * os)), dim3(256), 0, s, (const uint8_t*)d_fb,
                       (uint64_t)os, steps, raw + steps);
    STARK_HIP(ctx, hipGetLastError());
  }
  static_assert(sizeof(size_t) == sizeof(uint64_t), "size_t is 64-bit");
  if (!pack) {
    if (f0_ext)  // K into F0's slot: the six extended columns are contiguous from slot 1
      STARK_HIP(ctx, hipMemcpyAsync(raw + steps, raw, steps * sizeof(fe), hipMemcpyDeviceToDevice, s));
    STARK_HIP(ctx, hipMemcpyAsync(perm, permuted_indices, os * sizeof(uint64_t), hipMemcpyDefault, s));
    STARK_HIP(ctx, hipMemcpyAsync(wcopy, raw + 4 * steps, steps * sizeof(fe), hipMemcpyDeviceToDevice, s));
    STARK_HIP(ctx, hipMemsetAsync(d_tr, 0, sizeof(Transcript), s));
  }
  clk.mark("setup + uploads enqueued");
  auto proof = std::make_unique<stark_r1cs_proof>();
  // Accumulator tree -> a_root (utils.rs:250-270) -> r (utils.rs:272-290): the index kernel hashes each
  // 40-B leaf as it writes it (level 0).
  stark_merkle_tree *acc_tree, *m_tree, *l_tree;
  STARK_TRY(ctx_tree(ctx, 2, &acc_tree));
  STARK_TRY(ctx_tree(ctx, 3, &m_tree));
  STARK_TRY(ctx_tree(ctx, 4, &l_tree));
  uint32_t* acc_dig = nullptr;
  STARK_TRY(merkle_level0(ctx, acc_tree, steps, s, &acc_dig));
  // (IDX is not materialised: idx_ext is the shared extension.)
  hipLaunchKernelGGL(r1cs_index_kernel, dim3(blocks_for(steps)), dim3(256), 0, s, (const uint64_t*)perm,
                     (uint64_t)os, steps, (const fe*)wcopy, raw + 6 * steps, acc_leaves, acc_dig);
  STARK_HIP(ctx, hipGetLastError());
  STARK_TRY(merkle_build(ctx, acc_tree, (const uint8_t*)acc_leaves, steps, 40, s, 0, true));
  // A (utils.rs:293-339, prove.rs:183-184): r from a_root, the running products of the numerators and
  // denominators over the steps, their batch inverse (whose top level is the proof's one mid-pipeline host
  // round trip) and A = nmr / dnm.  It reads the trace and a_root only (IDX and PIDX at the step points
  // are i and the permutation), so when no Zb inverse shares its round trip it runs on the aux stream
  // beside the main LDE, which the host enqueues before it waits.
  const bool a_aside = pre || ca.tinv;
  if (!ctx->ev_aux) STARK_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_aux, hipEventDisableTiming));
  if (!ctx->aux) STARK_HIP(ctx, hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
  hipStream_t sa = s;
  if (a_aside) {
    sa = ctx->aux;
    STARK_HIP(ctx, hipEventRecord(ctx->ev_aux, s));  // the trace columns, the transcript's zero fill, a_root
    STARK_HIP(ctx, hipStreamWaitEvent(sa, ctx->ev_aux, 0));
  }
  hipLaunchKernelGGL(r1cs_r_kernel, dim3(1), dim3(64), 0, sa, (const uint32_t*)merkle_root_dev(acc_tree),
                     (uint32_t)(prec - 1), mc.r2, pow32(), d_tr);
  STARK_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(r1cs_a_vals_kernel, dim3(blocks_for(steps)), dim3(256), 0, sa, (const fe*)nullptr,
                     (const fe*)nullptr, (const uint64_t*)perm, (uint64_t)os, (const fe*)wcopy, steps,
                     (const Transcript*)d_tr, mc.r2, nmr, dnm);
  STARK_HIP(ctx, hipGetLastError());
  STARK_TRY(product_scan(ctx, ScanArrays{{nmr, dnm}, {tot, tot + nb}, {nullptr, dnm_c}}, 2, steps, mc, sa));
  // The cold proof's two batch inverses (the A denominators over the steps; Zb2, Zb3 over the precision
  // domain, which prepared circuits carry) share one host round trip: both up passes, one
  // synchronisation, both top levels on the host, then the down passes.
  InvPlan inv_d, inv_z;
  fe* const top_d = multi_inv_h_top(ctx, 0);
  fe* const top_z = multi_inv_h_top(ctx, 1);
  if (!top_d || !top_z) return STARK_ERR_OOM;
  // (io2's guard covers the pinned top arrays too: multi_inv_device on another stream uses both)
  STARK_TRY(buf_acquire(ctx, ctx->io2, sa));
  if (!pre && !ca.tinv) {
    hipLaunchKernelGGL(r1cs_zb_kernel, dim3(blocks_for(prec)), dim3(256), 0, s, tw2->d_lo, tw2->d_hi, tw2->kb, prec,
                       (uint64_t)0, (uint32_t)0, (const fe*)consts, (uint32_t)n_pfi, to_dev(x_last), mc.rinv, mc.one,
                       zb, izb3 ? nullptr : zb + prec);
    STARK_HIP(ctx, hipGetLastError());
    STARK_TRY(multi_inv_up(ctx, zb, inv_zb, izb3 ? prec : 2 * prec, s, ctx->io2, top_z, inv_z));
  }
  STARK_TRY(multi_inv_up(ctx, dnm_c, inv_dnm, steps, sa, ctx->inv_tmp, top_d, inv_d));
  if (pre)  // S and P only: K, the flags, IDX and PIDX are the circuit's
    STARK_TRY(lde(ctx, raw + 4 * steps, 2, cols + 4 * prec, log_steps, log_prec, *tw1i, *tw2, s));
  else if (f0_ext)  // K (in F0's slot) F1 F2 S P PIDX
    STARK_TRY(lde(ctx, raw + steps, 6, cols + prec, log_steps, log_prec, *tw1i, *tw2, s));
  else  // K F0 F1 F2 S P PIDX
    STARK_TRY(lde(ctx, raw, 7, cols, log_steps, log_prec, *tw1i, *tw2, s));
  STARK_HIP(ctx, hipStreamSynchronize(sa));
  multi_inv_top(inv_d);
  multi_inv_top(inv_z);
  STARK_TRY(multi_inv_down(ctx, inv_d, sa));
  // A = nmr / dnm into dnm (free after its scan's canonical copy)
  hipLaunchKernelGGL(r1cs_a_mini_kernel, dim3(blocks_for(steps)), dim3(256), 0, sa, (const fe*)nmr,
                     (const fe*)inv_dnm, steps, dnm);
  STARK_HIP(ctx, hipGetLastError());
  STARK_TRY(buf_release(ctx, ctx->io2, sa));
  if (a_aside) {
    STARK_HIP(ctx, hipEventRecord(ctx->ev_aux, sa));
    STARK_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_aux, 0));
  }
  STARK_TRY(lde(ctx, dnm, 1, cols + 7 * prec, log_steps, log_prec, *tw1i, *tw2, s));  // A in slot 7
  STARK_TRY(multi_inv_down(ctx, inv_z, s));  // (empty plan with a prepared circuit)
  const fe* ext_idx = pre ? pre + 4 * prec : idx_ext;
  const fe* ext_pidx = pre ? pre + 5 * prec : cols + 6 * prec;

  // Constraint kernel.
  for (int c = 0; c < 6; ++c) ca.col[c] = cols + (size_t)c * prec;
  ca.col[6] = ext_idx;
  ca.col[8] = cols + 7 * prec;  // A
  ca.col[7] = ext_pidx;
  if (f0_ext) {
    ca.col[0] = cols + prec;  // K
    ca.col[1] = f0_ext;
  }
  if (pre)
    for (int c = 0; c < 4; ++c) ca.col[c] = pre + (size_t)c * prec;
  ca.inv_zb = pre ? pre + 6 * prec : inv_zb;
  ca.inv_zb3 = izb3 ? izb3 : ca.inv_zb + prec;
  ca.interp2 = consts + n_pfi;
  ca.interp3 = consts + 2 * n_pfi;
  ca.lo = tw2->d_lo;
  ca.hi = tw2->d_hi;
  ca.rows = rows;
  ca.plane = prec;  // column-major: coalesced stores here and loads in the L kernel and the main tree
  ca.err = &d_tr->err;
  ca.prec = prec;
  ca.shift1 = (os / 3 * skips) % prec;
  ca.shift2 = (os / 3 * 2 * skips) % prec;
  ca.back = skips;
  ca.g_add = 0;
  ca.log_g = 0;
  ca.log_prec = log_prec;
  ca.kb = tw2->kb;
  ca.n2 = (uint32_t)n_pfi;
  ca.n3 = 1;
  ca.tr = d_tr;
  set_inv_z(ca, g2, steps);
  ca.mont_cols = pre ? 1 : 0;
  STARK_TRY(upload_constraint_tables(ctx, d_tr, ca, s));
  // Main tree over the 256-B rows (prove.rs:261-264): the constraint kernel hashes each row as it makes it
  // (level 0), the tree's levels above are built from those digests; the proofs open the rows as 8 planes.
  STARK_TRY(merkle_level0(ctx, m_tree, prec, s, &ca.leaf));
  hipLaunchKernelGGL(r1cs_constraint_kernel, dim3(blocks_for(prec)), dim3(256), 0, s, ca);
  STARK_HIP(ctx, hipGetLastError());
  STARK_TRY(merkle_build(ctx, m_tree, (const uint8_t*)rows, prec, 256, s, prec * sizeof(fe), true));
  {
    XsPowers xs;
    const HostFp w8 = F.pow_u64(g2, steps);
    HostFp wt = F.one();
    for (int t = 0; t < 8; ++t) {
      xs.v[t] = to_dev(wt);
      wt = F.mul(wt, w8);
    }
    hipLaunchKernelGGL(r1cs_k_kernel, dim3(1), dim3(kKThreads), 0, s, (const uint32_t*)merkle_root_dev(m_tree),
                       mc.r2, mc.one, xs, pow32(), d_tr);
    STARK_HIP(ctx, hipGetLastError());
  }
  LincombArgs la;
  la.rows = rows;
  la.plane = prec;
  la.out = lvals;
  la.prec = prec;
  la.g_add = 0;
  la.log_g = 0;
  la.tr = d_tr;
  // L tree (prove.rs:329-332): the linear-combination kernel hashes each value as it makes it (level 0).
  STARK_TRY(merkle_level0(ctx, l_tree, prec, s, &la.leaf));
  hipLaunchKernelGGL(r1cs_lincomb_kernel, dim3(blocks_for(prec)), dim3(256), 0, s, la);
  STARK_HIP(ctx, hipGetLastError());
  // Its root launch also copies the root into the transcript (l_root) and writes FRI layer 0's special_x
  // (fri.rs:135) into the FRI's slot 0 of fri_misc; where no tail launch makes the root, kernels do.
  STARK_TRY(ensure_buf(ctx, ctx->fri_misc, kFriMiscBytes));
  STARK_TRY(buf_acquire(ctx, ctx->fri_misc, s));
  RootFe l_rf{(fe*)ctx->fri_misc.ptr, mc.r2, &d_tr->roots[2][0], false};
  STARK_TRY(merkle_build(ctx, l_tree, (const uint8_t*)lvals, prec, 32, s, 0, true, &l_rf));
  if (!l_rf.made) {
    hipLaunchKernelGGL(r1cs_l_root_kernel, dim3(1), dim3(64), 0, s, (const uint32_t*)merkle_root_dev(l_tree), d_tr);
    STARK_HIP(ctx, hipGetLastError());
  }
  // The roots and the constraint flags come down behind the L tree; an event marks them.
  Transcript* h_tr = nullptr;
  // (slot 1 layout: internal.h kPinned1Bytes)
  // (only the head: the constants' digit-basis tables stay on the device)
  constexpr size_t kTrHead = offsetof(Transcript, k_db);
  static_assert(kTrHead <= 2048, "pinned slot 1 layout");
  STARK_TRY(ctx_pinned(ctx, 1, kPinned1Bytes, (void**)&h_tr));
  uint32_t* h_trace_err = reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(h_tr) + kPinned1TraceErrOff);
  STARK_HIP(ctx, hipMemcpyAsync(h_tr, d_tr, kTrHead, hipMemcpyDeviceToHost, s));
  if (ctx->trace_err) STARK_HIP(ctx, hipMemcpyAsync(h_trace_err, ctx->trace_err, 4, hipMemcpyDeviceToHost, s));
  if (!ctx->ev_aux) STARK_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_aux, hipEventDisableTiming));
  if (!ctx->aux) STARK_HIP(ctx, hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
  STARK_HIP(ctx, hipEventRecord(ctx->ev_aux, s));

  // prove_low_degree(L, g2, precision / 4, skips) on the resident L (prove.rs:367), enqueued behind the rest.
  FriPendingPtr fri_pending;
  clk.mark("prover kernels enqueued");
  STARK_TRY(fri_enqueue(ctx, (const fe*)lvals, prec, g2c, prec / 4, (uint32_t)skips, &fri_pending, l_tree,
                        l_rf.made));
  clk.mark("FRI kernels enqueued");
  // While the FRI layers run: the roots, the spot checks (prove.rs:337-362), their openings (gathered on
  // the second stream) and the StarkProof JSON up to fri_proof.
  STARK_HIP(ctx, hipEventSynchronize(ctx->ev_aux));
  clk.mark("wait for the L root");
  if (ctx->trace_err && *h_trace_err) {  // a wire id >= n_wires (reader.rs:4-89 bounds), found by the trace builder
    hipStreamSynchronize(s);
    ctx->last_error = "constraint record with a wire id >= n_wires";
    return STARK_ERR_BAD_ARG;
  }
  if (h_tr->err) {
    hipStreamSynchronize(s);  // (the enqueued FRI work finishes before the proof is dropped)
    ctx->last_error = (h_tr->err & 1) ? "invalid D: Q does not vanish where Z does (utils.rs:379-418)"
                                      : "invalid B: boundary value mismatch (utils.rs:477-524)";
    return STARK_ERR_CHECK;
  }
  memcpy(proof->a_root, h_tr->roots[0], 32);
  memcpy(proof->m_root, h_tr->roots[1], 32);
  memcpy(proof->l_root, h_tr->roots[2], 32);
  uint32_t pos32[kSpotChecks];
  STARK_TRY(stark_get_pseudorandom_indices(proof->l_root, 32, (uint32_t)prec, kSpotChecks, (uint32_t)skips, pos32));
  std::vector<size_t> positions(kSpotChecks), aug(4 * kSpotChecks);
  for (int i = 0; i < kSpotChecks; ++i) {
    const size_t j = pos32[i];
    positions[i] = j;
    aug[4 * i] = j;
    aug[4 * i + 1] = (j + prec - skips) % prec;
    aug[4 * i + 2] = (j + os / 3 * skips) % prec;
    aug[4 * i + 3] = (j + os / 3 * 2 * skips) % prec;
  }
  std::vector<uint8_t> l_leaves(32 * kSpotChecks), l_nodes(32 * kSpotChecks * log_prec);
  std::vector<uint8_t> m_leaves(256 * 4 * kSpotChecks), m_nodes(32 * 4 * kSpotChecks * log_prec);
  {
    // the trees are complete (behind the event); the gather runs beside the FRI kernels
    std::vector<GatherReq> spot = {{l_tree, positions.data(), (size_t)kSpotChecks, l_leaves.data(), l_nodes.data()},
                                   {m_tree, aug.data(), (size_t)4 * kSpotChecks, m_leaves.data(), m_nodes.data()}};
    STARK_TRY(merkle_gather_batch(ctx, spot, ctx->aux));
  }
  // StarkProof JSON (utils.rs:122-130; run.rs:549 serde_json::to_string), its head rendered now.
  JsonPieces j;
  j.text("{\"m_root\":");
  j.bytes(proof->m_root, 32);
  j.text(",\"l_root\":");
  j.bytes(proof->l_root, 32);
  j.text(",\"a_root\":");
  j.bytes(proof->a_root, 32);
  j.text(",\"main_branches\":");
  j.branches(m_leaves, 256, m_nodes, 4 * kSpotChecks, log_prec);
  j.text(",\"linear_comb_branches\":");
  j.branches(l_leaves, 32, l_nodes, kSpotChecks, log_prec);
  j.text(",\"fri_proof\":");
  clk.mark("spot-check openings");
  std::vector<GatherReq> extra;
  stark_fri_proof* fri = nullptr;
  {
    // The head renders on the side thread while this one waits for the FRI layers and gathers their
    // openings (for a small proof the FRI kernels finish before the head would be rendered).
    HostTask head([&] { j.prerender(16); });
    const stark_status st = fri_finish(ctx, fri_pending.get(), extra, &fri);
    clk.mark("FRI wait + indices + gather");
    head.wait();
    clk.mark("proof head JSON (beside them)");
    if (st != STARK_OK) return st;
  }
  proof->fri = fri;  // owned by the proof from here on
  fri_proof_json_pieces(fri, j);
  j.text("}");
  j.render(proof->json);
  clk.mark("proof JSON");
  proof->depth = log_prec;
  proof->m_leaves = std::move(m_leaves);
  proof->m_nodes = std::move(m_nodes);
  proof->l_leaves = std::move(l_leaves);
  proof->l_nodes = std::move(l_nodes);
  *out = proof.release();
  return STARK_OK;
}

// v[i] <- Montgomery image of v[i] (canonical in).
__global__ void to_mont_kernel(fe* __restrict__ v, uint64_t n, fe r2) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) fe_store(v + i, fe_mul(fe_load(v + i), r2));
}

// IDX / PIDX step columns only (the circuit's part of r1cs_index_kernel).
__global__ void r1cs_idx_kernel(const uint64_t* __restrict__ perm, uint64_t os, uint64_t steps, fe* __restrict__ idx,
                                fe* __restrict__ pidx) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= steps) return;
  fe_store(idx + i, fe_from_u64(i));
  fe_store(pidx + i, fe_from_u64(i < os ? perm[i] : i));
}

// The LDE columns of a circuit that no witness changes: K, F0, F1, F2, IDX, PIDX
// (prove.rs:100-124, 160-167), 6 x precision into `out`.  coef / flag bytes / perm
// are the device trace builder's circuit columns (os slots).
stark_status circuit_lde(stark_ctx* ctx, const fe* coef, const uint8_t* flag_bytes, const uint64_t* perm, size_t os,
                         const size_t* public_first_indices, size_t n_pfi, uint32_t world, uint32_t rank, DevBuf& out,
                         hipStream_t s, bool with_zb, const fe** colp, uint32_t* spot_log_t) {
  const FieldHost& F = FieldHost::get();
  // with_zb = false (the verifier's cold build, which needs six values per spot position): the columns
  // stay where they are made -- K's extension in slot 1, F0's and IDX's in their shared entries -- with
  // no slot copies and no Montgomery images (colp tells the caller where each one is).  With spot_log_t
  // no extension is made at all: out holds the six columns' first forward passes (circuit_spot_values).
  const bool verify_only = !with_zb;
  if (spot_log_t && (with_zb || world != 1)) return STARK_ERR_BAD_ARG;
  const fe* col[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  if (world == 0 || world > (uint32_t)kExtensionFactor || (world & (world - 1)) || rank >= world)
    return STARK_ERR_BAD_ARG;
  uint32_t log_g = 0;
  while ((1u << log_g) < world) ++log_g;
  if (os < 5 || os % 3 != 0) return STARK_ERR_BAD_LENGTH;
  const uint32_t log_steps = log2_ceil_ref(os - 1);
  const uint32_t log_prec = log_steps + kLogExtensionFactor;
  if (log_prec >= 24) return STARK_ERR_BAD_LENGTH;
  const uint64_t steps = (uint64_t)1 << log_steps, prec = (uint64_t)1 << log_prec;
  const uint64_t P = prec >> log_g;  // this rank's points r + world j
  ProofRoots roots;
  STARK_TRY(proof_roots(ctx, log_steps, log_prec, world, roots));
  const HostFp g2 = roots.g2;
  const Twiddles *tw2 = roots.tw2, *tw1i = roots.tw1i, *twh = roots.twh;
  for (size_t i = 0; i < n_pfi; ++i)
    if (public_first_indices[2 * i + 1] >= steps) return STARK_ERR_BAD_ARG;
  DevBuf& tmp = ctx->lde_tmp;  // 6 step columns, then Zb2 / Zb3 and the x_k (2 P + n_pfi)
  STARK_TRY(ensure_buf(ctx, tmp, (6 * steps + 2 * P + n_pfi + 1) * sizeof(fe)));
  stark_status st = ensure_buf(ctx, out, (with_zb ? 8 : 6) * P * sizeof(fe));
  if (st == STARK_OK) {
    fe* raw = (fe*)tmp.ptr;
    hipMemsetAsync(raw, 0, 6 * steps * sizeof(fe), s);
    hipMemcpyAsync(raw, coef, os * sizeof(fe), hipMemcpyDeviceToDevice, s);
    hipLaunchKernelGGL(r1cs_flags_kernel, dim3(blocks_for(3 * os)), dim3(256), 0, s, flag_bytes, (uint64_t)os, steps,
                       raw + steps);
    hipLaunchKernelGGL(r1cs_idx_kernel, dim3(blocks_for(steps)), dim3(256), 0, s, perm, (uint64_t)os, steps,
                       raw + 4 * steps, raw + 5 * steps);
    if (spot_log_t) {
      // The step columns' coefficients (inv_best_fft, one batch), then only the first pass of their
      // forward transforms over the precision domain, transposed (ntt_first_pass_tmajor).  F0's and
      // IDX's depend on the size alone: from the context's cache when it holds them (K moved over F0's
      // step column and PIDX over IDX's, K F1 F2 PIDX are then one batch of four), else in the batch.
      fe* const o = (fe*)out.ptr;
      const fe *yf0 = nullptr, *yidx = nullptr;
      st = ext_const_column(ctx, kSpotF0, os, log_steps, log_prec, 0, 0, *tw1i, *tw2, *twh, s, &yf0);
      if (st == STARK_OK) st = ext_const_column(ctx, kSpotIdx, 0, log_steps, log_prec, 0, 0, *tw1i, *tw2, *twh, s, &yidx);
      auto live = [&](uint32_t kind, uint64_t tag) {  // (a later reservation may evict an earlier column)
        return ctx->ext_idx.count(std::make_tuple(kind, log_steps, log_prec, 0u, 0u, tag)) != 0;
      };
      if (yf0 && !live(kSpotF0, os)) yf0 = nullptr;
      if (yidx && !live(kSpotIdx, 0)) yidx = nullptr;
      const bool shared = yf0 && yidx;
      if (st == STARK_OK && shared &&
          (hipMemcpyAsync(raw + steps, raw, steps * sizeof(fe), hipMemcpyDeviceToDevice, s) != hipSuccess ||
           hipMemcpyAsync(raw + 4 * steps, raw + 5 * steps, steps * sizeof(fe), hipMemcpyDeviceToDevice, s) !=
               hipSuccess))
        st = STARK_ERR_HIP;
      fe* const first = shared ? raw + steps : raw;
      const uint32_t batch = shared ? 4 : 6;
      if (st == STARK_OK) st = ntt_device(ctx, first, log_steps, batch, *tw1i, true, s);
      if (st == STARK_OK)
        st = ntt_first_pass_tmajor(ctx, first, log_prec - log_steps, o, log_prec, batch, *tw2, s, spot_log_t);
      if (shared) {
        const fe* c6[6] = {o, yf0, o + P, o + 2 * P, yidx, o + 3 * P};
        for (int k = 0; k < 6; ++k) col[k] = c6[k];
      } else {
        for (int k = 0; k < 6; ++k) col[k] = o + (uint64_t)k * P;
      }
      if (hipStreamSynchronize(s) != hipSuccess && st == STARK_OK) st = STARK_ERR_HIP;
      if (colp)
        for (int k = 0; k < 6; ++k) colp[k] = col[k];
      return st;
    }
    // K F0 F1 F2, then PIDX; IDX and F0 (1 on the os rows: the flags are circuit_build's calc_flags)
    // are the shared extensions (ext_const_column), copied into their slots.  With F0's: K is moved
    // over F0's step column, K F1 F2 are extended into slots 1-3, and K then copied to slot 0.
    const fe *idx_ext = nullptr, *f0_ext = nullptr;
    st = ext_const_column(ctx, kExtF0, os, log_steps, log_prec, log_g, rank, *tw1i, *tw2, *twh, s, &f0_ext);
    if (st == STARK_OK)
      st = ext_index_column(ctx, log_steps, log_prec, log_g, rank, *tw1i, *tw2, *twh, s, &idx_ext);
    if (f0_ext && !ctx->ext_idx.count(std::make_tuple(kExtF0, log_steps, log_prec, log_g, rank, (uint64_t)os)))
      f0_ext = nullptr;  // evicted by IDX's reservation
    fe* const o = (fe*)out.ptr;
    if (st == STARK_OK && f0_ext) {
      if (hipMemcpyAsync(raw + steps, raw, steps * sizeof(fe), hipMemcpyDeviceToDevice, s) != hipSuccess)
        st = STARK_ERR_HIP;
      if (st == STARK_OK)
        st = coset_lde(ctx, raw + steps, 3, o + P, log_steps, log_prec, log_g, rank, *tw1i, *tw2, *twh, s);
      if (st == STARK_OK && !verify_only &&
          (hipMemcpyAsync(o, o + P, P * sizeof(fe), hipMemcpyDeviceToDevice, s) != hipSuccess ||
           hipMemcpyAsync(o + P, f0_ext, P * sizeof(fe), hipMemcpyDeviceToDevice, s) != hipSuccess))
        st = STARK_ERR_HIP;
      col[0] = verify_only ? o + P : o;
      col[1] = verify_only ? f0_ext : o + P;
    } else if (st == STARK_OK) {
      st = coset_lde(ctx, raw, 4, o, log_steps, log_prec, log_g, rank, *tw1i, *tw2, *twh, s);
      col[0] = o;
      col[1] = o + P;
    }
    col[2] = o + 2 * P;
    col[3] = o + 3 * P;
    col[4] = verify_only ? idx_ext : o + 4 * P;
    col[5] = o + 5 * P;
    if (st == STARK_OK)
      st = coset_lde(ctx, raw + 5 * steps, 1, (fe*)out.ptr + 5 * P, log_steps, log_prec, log_g, rank, *tw1i, *tw2,
                     *twh, s);
    if (st == STARK_OK && !verify_only &&
        hipMemcpyAsync((fe*)out.ptr + 4 * P, idx_ext, P * sizeof(fe), hipMemcpyDeviceToDevice, s) != hipSuccess)
      st = STARK_ERR_HIP;
    // Zb2 = prod_k (x - x_k), Zb3 = x - x_last (utils.rs:438-474) and their inverses (0 -> 0).
    const uint64_t skips = prec / steps;
    std::vector<fe> xk(n_pfi + 1);
    for (size_t i = 0; i < n_pfi; ++i) xk[i] = to_dev(F.pow_u64(g2, skips * public_first_indices[2 * i + 1]));
    fe* zb = raw + 6 * steps;
    fe* d_xk = zb + 2 * P;
    const Mont mc = mont();
    if (st == STARK_OK && with_zb && n_pfi &&
        hipMemcpyAsync(d_xk, xk.data(), n_pfi * sizeof(fe), hipMemcpyHostToDevice, s) != hipSuccess)
      st = STARK_ERR_HIP;
    if (st == STARK_OK && with_zb) {
      hipLaunchKernelGGL(r1cs_zb_kernel, dim3(blocks_for(P)), dim3(256), 0, s, tw2->d_lo, tw2->d_hi, tw2->kb, P,
                         (uint64_t)rank, log_g, (const fe*)d_xk, (uint32_t)n_pfi,
                         to_dev(F.pow_u64(g2, prec - skips)), mc.rinv, mc.one, zb, zb + P);
      st = multi_inv_device(ctx, zb, (fe*)out.ptr + 6 * P, 2 * P, s);
    }
    if (st == STARK_OK && !verify_only) {  // K, F0-F2 as Montgomery images (ConstraintArgs::mont_cols; the Zb inverses are)
      hipLaunchKernelGGL(to_mont_kernel, dim3(blocks_for(4 * P)), dim3(256), 0, s, o, 4 * P, mc.r2);
      if (hipGetLastError() != hipSuccess) st = STARK_ERR_HIP;
    }
    if (st == STARK_OK && hipStreamSynchronize(s) != hipSuccess) st = STARK_ERR_HIP;
  }
  hipStreamSynchronize(s);  // tmp (a context buffer) is free for the next call
  if (colp)
    for (int k = 0; k < 6; ++k) colp[k] = col[k];
  return st;
}

// ---- the verifier's spot values (circuit_lde's spot mode) -------------------------------------------
//
// Y = the six step columns' first forward passes, T-major (column k at c.col[k], Y[t A + j], T = 2^log_t,
// A = P / T): column k at x = g2^e is sum_{j < A} x^j Y_k[(e mod T) A + j] (ntt_first_pass_tmajor), a
// contiguous run of A values per column and position instead of the two further passes of its extension.
// Workgroup (b, i) takes position i's j = g + S l (g = 256 b + thread < S, l < A / S): Horner over l with
// the constant x^S (its digit-basis table, spot_setup_kernel), then one product by x^g (the two-level
// table of g2), summed over the workgroup; spot_sum_kernel adds position i's workgroups.
constexpr uint32_t kSpotMax = 128;
struct SpotPos {
  uint64_t e[kSpotMax];
};

__global__ void spot_setup_kernel(SpotPos pos, uint32_t n, uint32_t log_s, uint64_t P, const fe* __restrict__ lo,
                                  const fe* __restrict__ hi, uint32_t kb, Pow32 p32, uint32_t* __restrict__ tabs) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, i = t >> 3, r = t & 7;  // row r of position i's table
  if (i >= n) return;
  fe unit = fe_zero();
  unit.w[0] = 1;
  const fe xs = fe_mul(pow_tab(lo, hi, kb, (pos.e[i] << log_s) & (P - 1)), unit);  // x^S, canonical
  db_limbs(fe_mul(xs, p32.m[r]), tabs + 72 * i + 9 * r);
}

struct SpotCols {
  const fe* c[6];
};

__global__ __launch_bounds__(256) void spot_eval_kernel(SpotCols y, uint64_t P, uint32_t log_t,
                                                        uint32_t log_s, SpotPos pos, const uint32_t* __restrict__ tabs,
                                                        const fe* __restrict__ lo, const fe* __restrict__ hi,
                                                        uint32_t kb, fe* __restrict__ partial) {
  __shared__ fe red[256];
  const uint32_t i = blockIdx.y;
  const uint64_t e = pos.e[i];
  const uint64_t T = (uint64_t)1 << log_t, A = P >> log_t, S = (uint64_t)1 << log_s, nl = A >> log_s;
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool on = g < S;
  const uint32_t* W = tabs + 72 * i;  // (uniform: scalar loads)
  const fe xg = on ? pow_tab(lo, hi, kb, (e * g) & (P - 1)) : fe_zero();  // Montgomery image of x^g
  const uint64_t off = (e & (T - 1)) * A + g;
  fe sum[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    fe acc = fe_zero();
    if (on) {
      const fe* c = y.c[k] + off;
      acc = fe_load(c + (nl - 1) * S);
#pragma unroll 4
      for (uint64_t l = nl - 1; l-- > 0;) {
        const fe v = fe_load(c + l * S);
        acc = fe_add_raw(fe_mul_db(acc, W), v);  // [0, 2p) + [0, p): below 3p, a digit-basis input
      }
      acc = fe_mul(acc, xg);  // canonical
    }
    sum[k] = acc;
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    red[threadIdx.x] = sum[k];
    __syncthreads();
    for (uint32_t w = blockDim.x / 2; w > 0; w >>= 1) {
      if (threadIdx.x < w) red[threadIdx.x] = fe_add(red[threadIdx.x], red[threadIdx.x + w]);
      __syncthreads();
    }
    if (threadIdx.x == 0) fe_store(partial + ((uint64_t)i * gridDim.x + blockIdx.x) * 6 + k, red[0]);
    __syncthreads();
  }
}

__global__ void spot_sum_kernel(const fe* __restrict__ partial, uint32_t bp, uint32_t n, fe* __restrict__ out) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;  // position q / 6, column q % 6
  if (q >= 6 * n) return;
  const uint32_t i = q / 6, k = q % 6;
  fe s = fe_zero();
  for (uint32_t b = 0; b < bp; ++b) s = fe_add(s, fe_load(partial + ((uint64_t)i * bp + b) * 6 + k));
  fe_store(out + (uint64_t)k * n + i, s);
}

stark_status circuit_spot_values(stark_ctx* ctx, const PreparedCircuit& c, const size_t* positions, size_t n,
                                 uint8_t* out, hipStream_t s) {
  if (!c.spot || !c.col[0] || n == 0 || n > kSpotMax || !positions || !out) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));  // (the verifier calls this from its side thread)
  const FieldHost& F = FieldHost::get();
  const uint32_t log_steps = log2_ceil_ref(c.os - 1), log_prec = log_steps + kLogExtensionFactor;
  const uint64_t P = (uint64_t)1 << log_prec;
  if (c.spot_log_t == 0 || c.spot_log_t > log_prec) return STARK_ERR_BAD_ARG;
  ProofRoots roots;
  STARK_TRY(proof_roots(ctx, log_steps, log_prec, 1, roots));
  const Twiddles& tw = *roots.tw2;
  // j's per thread: 16 where the positions' threads fill the chip (A = 2^16 at 2^20 steps: 80 x 16
  // workgroups), 4 below (a few hundred workgroups, each short)
  const uint32_t log_a = log_prec - c.spot_log_t;
  const uint32_t log_nl = std::min<uint32_t>(log_a, log_a >= 16 ? 4 : log_a >= 14 ? log_a - 12 : 2);
  const uint32_t log_s = log_a - log_nl;
  const uint32_t bp = log_s > 8 ? 1u << (log_s - 8) : 1u;
  SpotPos sp;
  for (size_t i = 0; i < n; ++i) {
    if (positions[i] >= P) return STARK_ERR_BAD_ARG;
    sp.e[i] = positions[i];
  }
  const size_t tab_bytes = (n * 72 * 4 + 255) & ~(size_t)255, part_bytes = n * bp * 6 * sizeof(fe);
  STARK_TRY(ensure_buf(ctx, ctx->spot, tab_bytes + part_bytes + 6 * n * sizeof(fe)));
  uint8_t* d = (uint8_t*)ctx->spot.ptr;
  uint32_t* tabs = (uint32_t*)d;
  fe* partial = (fe*)(d + tab_bytes);
  fe* vals = (fe*)(d + tab_bytes + part_bytes);
  uint8_t* host = nullptr;
  STARK_TRY(ctx_pinned(ctx, 0, 6 * n * sizeof(fe), (void**)&host));
  hipLaunchKernelGGL(spot_setup_kernel, dim3((unsigned)((8 * n + 255) / 256)), dim3(256), 0, s, sp, (uint32_t)n, log_s,
                     P, tw.d_lo, tw.d_hi, tw.kb, pow32(), tabs);
  SpotCols cols;
  for (int k = 0; k < 6; ++k) {
    if (!c.col[k]) return STARK_ERR_BAD_ARG;
    cols.c[k] = c.col[k];
  }
  hipLaunchKernelGGL(spot_eval_kernel, dim3(bp, (unsigned)n), dim3(256), 0, s, cols, P, c.spot_log_t,
                     log_s, sp, (const uint32_t*)tabs, tw.d_lo, tw.d_hi, tw.kb, partial);
  hipLaunchKernelGGL(spot_sum_kernel, dim3((unsigned)((6 * n + 255) / 256)), dim3(256), 0, s, (const fe*)partial, bp,
                     (uint32_t)n, vals);
  STARK_HIP(ctx, hipGetLastError());
  STARK_HIP(ctx, hipMemcpyAsync(host, vals, 6 * n * sizeof(fe), hipMemcpyDeviceToHost, s));
  STARK_HIP(ctx, hipStreamSynchronize(s));
  memcpy(out, host, 6 * n * sizeof(fe));
  return STARK_OK;
}

stark_status mk_r1cs_proof_prepared(stark_ctx* ctx, const uint64_t* witness_trace, const uint64_t* computational_trace,
                                    size_t os, const uint64_t* public_wires, size_t n_public,
                                    const size_t* public_first_indices, size_t n_pfi, const size_t* permuted_indices,
                                    const uint64_t* coefficients, const uint8_t* flag_bytes, size_t n_constraints,
                                    size_t n_wires, const fe* pre, stark_r1cs_proof** out) {
  if (!ctx || !out || !pre) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const stark_status st = prove_r1cs(ctx, witness_trace, computational_trace, os, public_wires, n_public,
                                     public_first_indices, n_pfi, permuted_indices, coefficients, nullptr, nullptr,
                                     nullptr, flag_bytes, n_constraints, n_wires, out, pre);
  hipStreamSynchronize(ctx->stream);
  return st;
}

stark_status mk_r1cs_proof_bytes_flags(stark_ctx* ctx, const uint64_t* witness_trace,
                                      const uint64_t* computational_trace, size_t os, const uint64_t* public_wires,
                                      size_t n_public, const size_t* public_first_indices, size_t n_pfi,
                                      const size_t* permuted_indices, const uint64_t* coefficients,
                                      const uint8_t* flag_bytes, size_t n_constraints, size_t n_wires,
                                      stark_r1cs_proof** out, bool dev_in) {
  if (!ctx || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const stark_status st = prove_r1cs(ctx, witness_trace, computational_trace, os, public_wires, n_public,
                                     public_first_indices, n_pfi, permuted_indices, coefficients, nullptr, nullptr,
                                     nullptr, flag_bytes, n_constraints, n_wires, out, nullptr, dev_in);
  hipStreamSynchronize(ctx->stream);
  return st;
}

// ---- distributed prover (one rank of `world` GPUs) -------------------------
//
// The precision domain is split by residue class: rank r owns the evaluation
// points i = r + G j (j < P = precision / G), G | 8.  Then
//  * the LDE of every column is a coset evaluation with no exchange: the
//    polynomial has degree < steps <= P, so f(g2^(r + G j)) =
//    sum_k (c_k g2^(r k)) (g2^G)^(j k) is a P-point NTT of the scaled
//    coefficients;
//  * every shifted read of the constraints (-skips, +k skips, +2k skips) is a
//    multiple of 8, hence of G, and stays inside the residue class;
//  * the FRI fold's four points i + t n/4 are in the same class while
//    n/4 >= G, so each layer's column is again residue-class distributed.
// Only the Merkle trees need other ranks' data; the caller exchanges leaf
// digests (stark_amd/dprove.py).  The small step-domain work (accumulator
// tree, transcript r, A's running products) is repeated on every rank.
struct DProveState {
  stark_ctx* ctx = nullptr;
  hipStream_t s = nullptr;
  uint32_t G = 1, r = 0, log_g = 0;
  uint64_t steps = 0, prec = 0, P = 0, skips = 0, os = 0;
  uint32_t log_steps = 0, log_prec = 0;
  uint64_t g2c[4];
  DevBuf arena;
  stark_merkle_tree* acc_tree = nullptr;
  fe *rows = nullptr, *lvals = nullptr;
  Transcript* d_tr = nullptr;
  fe xs_m[8];
};

}  // namespace stark

struct stark_dprove {
  stark::DProveState st;
  ~stark_dprove() {
    if (st.acc_tree) stark_merkle_free(st.acc_tree);
    if (st.arena.ptr) hipFree(st.arena.ptr);
  }
};

namespace stark {

// Coset LDE of `batch` step columns (coef, destroyed) into out (batch x P).
static stark_status lde_coset(DProveState& d, fe* coef, uint32_t batch, fe* out, const Twiddles& tw_g1_inv,
                              const Twiddles& tw_g2, const Twiddles& tw_h) {
  return coset_lde(d.ctx, coef, batch, out, d.log_steps, d.log_prec, d.log_g, d.r, tw_g1_inv, tw_g2, tw_h, d.s);
}

static stark_status dprove_begin(stark_ctx* ctx, uint32_t world, uint32_t rank, const uint64_t* witness_trace,
                                 const uint64_t* computational_trace, size_t os, const uint64_t* public_wires,
                                 size_t n_public, const size_t* public_first_indices, size_t n_pfi,
                                 const size_t* permuted_indices, const uint64_t* coefficients, const uint64_t* flag0,
                                 const uint64_t* flag1, const uint64_t* flag2, const uint8_t* flag_bytes,
                                 size_t n_constraints, size_t n_wires, hipStream_t s, stark_dprove* h,
                                 const fe* pre = nullptr) {
  // pre != nullptr: this rank's prepared circuit columns (circuit_lde with world, rank): the coset
  // LDEs of K F0 F1 F2 IDX PIDX and the Zb inverses; only S, P and A are extended here.
  const FieldHost& F = FieldHost::get();
  DProveState& d = h->st;
  if (world == 0 || world > (uint32_t)kExtensionFactor || (world & (world - 1)) || rank >= world)
    return STARK_ERR_BAD_ARG;
  // prove.rs:30-53 (as prove_r1cs)
  if (os > 3 * n_constraints * n_wires || os % 3 != 0) return STARK_ERR_BAD_ARG;
  if (os < 5) return STARK_ERR_BAD_LENGTH;
  const uint32_t log_steps = log2_ceil_ref(os - 1);
  const uint32_t log_prec = log_steps + kLogExtensionFactor;
  if (log_prec >= 24) return STARK_ERR_BAD_LENGTH;
  d.ctx = ctx;
  d.s = s;
  d.G = world;
  d.r = rank;
  while ((1u << d.log_g) < world) ++d.log_g;
  d.log_steps = log_steps;
  d.log_prec = log_prec;
  d.steps = (uint64_t)1 << log_steps;
  d.prec = (uint64_t)1 << log_prec;
  d.P = d.prec >> d.log_g;
  d.skips = d.prec / d.steps;
  d.os = os;
  const uint64_t steps = d.steps, prec = d.prec, P = d.P, skips = d.skips;
  for (size_t i = 0; i < n_pfi; ++i)
    if (public_first_indices[2 * i] >= n_public || public_first_indices[2 * i + 1] >= steps) return STARK_ERR_BAD_ARG;

  // Roots (prove.rs:71-94); h = g2^G generates this rank's coset of size P.
  ProofRoots roots;
  STARK_TRY(proof_roots(ctx, log_steps, log_prec, world, roots));
  const HostFp g2 = roots.g2;
  memcpy(d.g2c, roots.g2c, 32);
  const Twiddles *tw2 = roots.tw2, *tw1i = roots.tw1i, *twh = roots.twh;
  const Mont mc = mont();
  // This rank's share of the shared size-only columns, as in prove_r1cs.
  SharedCols sc;
  if (!pre)
    STARK_TRY(shared_columns(ctx, flag_bytes != nullptr, os, log_steps, log_prec, d.log_g, rank, *tw1i, *tw2, *twh, s,
                             sc));
  const fe *idx_ext = sc.idx, *f0_ext = sc.f0, *izb3 = sc.izb3;
  ConstraintArgs ca;
  ca.tinv = nullptr;
  if (sc.tinv && izb3 && zb2_partial_fractions(g2, prec, skips, d.log_g, public_first_indices, n_pfi, ca))
    ca.tinv = sc.tinv;

  fe *raw, *wcopy, *cols, *nmr, *dnm, *tot, *dnm_c, *inv_dnm, *zb, *inv_zb, *consts;
  uint64_t* perm;
  uint64_t* acc_leaves;
  const uint32_t nb = (uint32_t)((steps + kScanBlock - 1) / kScanBlock);
  Carve cv;
  cv.add(&raw, 7 * steps);  // K F0 F1 F2 S P PIDX
  cv.add(&wcopy, steps);
  cv.add(&perm, steps);
  cv.add(&acc_leaves, 5 * steps);
  cv.add(&cols, 8 * P);  // K F0 F1 F2 S P PIDX A (IDX's extension is shared: idx_ext)
  cv.add(&nmr, steps);
  cv.add(&dnm, steps);
  cv.add(&tot, 2 * (size_t)nb);
  cv.add(&dnm_c, steps);
  cv.add(&inv_dnm, steps);
  cv.add(&zb, 2 * P > 3 * os / 32 + 1 ? 2 * P : 3 * os / 32 + 1);
  cv.add(&inv_zb, 2 * P);
  cv.add(&consts, 2 * n_pfi + 2);
  cv.add(&d.rows, 8 * P);
  cv.add(&d.lvals, P);
  cv.add(&d.d_tr, 1);
  STARK_TRY(cv.commit(ctx, d.arena));

  // Interpolants and boundary points (utils.rs:421-474).
  HostFp x_last;
  const std::vector<fe> hc2 = boundary_consts(g2, prec, skips, public_wires, public_first_indices, n_pfi, &x_last);
  STARK_HIP(ctx, hipMemcpyAsync(consts, hc2.data(), hc2.size() * sizeof(fe), hipMemcpyHostToDevice, s));
  // Step columns (prove.rs:59-69), host or device sources.
  const uint64_t* src[6] = {coefficients, flag0, flag1, flag2, witness_trace, computational_trace};
  for (int c = pre ? 4 : 0; c < 6; ++c) {
    if (!(flag_bytes && c >= 1 && c <= 3))
      STARK_HIP(ctx, hipMemcpyAsync(raw + c * steps, src[c], os * sizeof(fe), hipMemcpyDefault, s));
    if (steps > os) STARK_HIP(ctx, hipMemsetAsync(raw + c * steps + os, 0, (steps - os) * sizeof(fe), s));
  }
  if (flag_bytes && !pre) {
    uint8_t* d_fb = (uint8_t*)zb;  // zb is free until the Zb kernel (sized for the 3 os flag bytes)
    STARK_HIP(ctx, hipMemcpyAsync(d_fb, flag_bytes, 3 * os, hipMemcpyDefault, s));
    hipLaunchKernelGGL(r1cs_flags_kernel, dim3(blocks_for(3 * os)), dim3(256), 0, s, (const uint8_t*)d_fb,
                       (uint64_t)os, steps, raw + steps);
    STARK_HIP(ctx, hipGetLastError());
  }
  if (f0_ext)  // K into F0's slot: the six extended columns are contiguous from slot 1
    STARK_HIP(ctx, hipMemcpyAsync(raw + steps, raw, steps * sizeof(fe), hipMemcpyDeviceToDevice, s));
  STARK_HIP(ctx, hipMemcpyAsync(perm, permuted_indices, os * sizeof(uint64_t), hipMemcpyDefault, s));
  STARK_HIP(ctx, hipMemcpyAsync(wcopy, raw + 4 * steps, steps * sizeof(fe), hipMemcpyDeviceToDevice, s));
  STARK_HIP(ctx, hipMemsetAsync(d.d_tr, 0, sizeof(Transcript), s));
  // (PIDX in slot 6; IDX is not materialised: idx_ext)
  hipLaunchKernelGGL(r1cs_index_kernel, dim3(blocks_for(steps)), dim3(256), 0, s, (const uint64_t*)perm,
                     (uint64_t)os, steps, (const fe*)wcopy, raw + 6 * steps, acc_leaves, (uint32_t*)nullptr);
  STARK_HIP(ctx, hipGetLastError());
  // Accumulator tree -> a_root -> r (utils.rs:250-290), on every rank.
  STARK_TRY(stark_merkle_new(ctx, &d.acc_tree));
  STARK_TRY(merkle_build(ctx, d.acc_tree, (const uint8_t*)acc_leaves, steps, 40, s));
  // A (utils.rs:293-339): step-domain scans on every rank, then this rank's coset.  As on one GPU, the
  // chain (r, the scans, their batch inverse with its host round trip, A = nmr / dnm) runs on the
  // context's aux stream beside the coset LDE, which the host enqueues before it waits.
  if (!ctx->ev_aux) STARK_HIP(ctx, hipEventCreateWithFlags(&ctx->ev_aux, hipEventDisableTiming));
  if (!ctx->aux) STARK_HIP(ctx, hipStreamCreateWithFlags(&ctx->aux, hipStreamNonBlocking));
  hipStream_t sa = ctx->aux;
  STARK_HIP(ctx, hipEventRecord(ctx->ev_aux, s));  // the trace columns, the transcript's zero fill, a_root
  STARK_HIP(ctx, hipStreamWaitEvent(sa, ctx->ev_aux, 0));
  hipLaunchKernelGGL(r1cs_r_kernel, dim3(1), dim3(64), 0, sa, (const uint32_t*)merkle_root_dev(d.acc_tree),
                     (uint32_t)(prec - 1), mc.r2, pow32(), d.d_tr);
  STARK_HIP(ctx, hipGetLastError());
  hipLaunchKernelGGL(r1cs_a_vals_kernel, dim3(blocks_for(steps)), dim3(256), 0, sa, (const fe*)nullptr,
                     (const fe*)nullptr, (const uint64_t*)perm, (uint64_t)os, (const fe*)wcopy, steps,
                     (const Transcript*)d.d_tr, mc.r2, nmr, dnm);
  STARK_HIP(ctx, hipGetLastError());
  STARK_TRY(product_scan(ctx, ScanArrays{{nmr, dnm}, {tot, tot + nb}, {nullptr, dnm_c}}, 2, steps, mc, sa));
  InvPlan inv_d;
  fe* const top_d = multi_inv_h_top(ctx, 0);
  if (!top_d) return STARK_ERR_OOM;
  STARK_TRY(buf_acquire(ctx, ctx->io2, sa));  // (io2's guard covers the pinned top arrays too)
  STARK_TRY(multi_inv_up(ctx, dnm_c, inv_dnm, steps, sa, ctx->io2, top_d, inv_d));
  if (pre)
    STARK_TRY(lde_coset(d, raw + 4 * steps, 2, cols + 4 * P, *tw1i, *tw2, *twh));
  else if (f0_ext)  // K (in F0's slot) F1 F2 S P PIDX
    STARK_TRY(lde_coset(d, raw + steps, 6, cols + P, *tw1i, *tw2, *twh));
  else  // K F0 F1 F2 S P PIDX
    STARK_TRY(lde_coset(d, raw, 7, cols, *tw1i, *tw2, *twh));
  STARK_HIP(ctx, hipStreamSynchronize(sa));
  multi_inv_top(inv_d);
  STARK_TRY(multi_inv_down(ctx, inv_d, sa));
  // A = nmr / dnm into dnm (free after its scan's canonical copy; raw may still be read by the LDE)
  hipLaunchKernelGGL(r1cs_a_mini_kernel, dim3(blocks_for(steps)), dim3(256), 0, sa, (const fe*)nmr,
                     (const fe*)inv_dnm, steps, dnm);
  STARK_HIP(ctx, hipGetLastError());
  STARK_TRY(buf_release(ctx, ctx->io2, sa));
  STARK_HIP(ctx, hipEventRecord(ctx->ev_aux, sa));
  STARK_HIP(ctx, hipStreamWaitEvent(s, ctx->ev_aux, 0));
  STARK_TRY(lde_coset(d, dnm, 1, cols + 7 * P, *tw1i, *tw2, *twh));  // A in slot 7
  if (!pre && !ca.tinv) {  // Zb2 / Zb3 at this rank's points and their inverses
    hipLaunchKernelGGL(r1cs_zb_kernel, dim3(blocks_for(P)), dim3(256), 0, s, tw2->d_lo, tw2->d_hi, tw2->kb, P,
                       (uint64_t)rank, d.log_g, (const fe*)consts, (uint32_t)n_pfi, to_dev(x_last), mc.rinv, mc.one,
                       zb, izb3 ? nullptr : zb + P);
    STARK_HIP(ctx, hipGetLastError());
    STARK_TRY(multi_inv_device(ctx, zb, inv_zb, izb3 ? P : 2 * P, s));
  }
  for (int c = 0; c < 6; ++c) ca.col[c] = cols + (size_t)c * P;
  ca.col[8] = cols + 7 * P;  // A
  ca.inv_zb = pre ? pre + 6 * P : inv_zb;
  ca.inv_zb3 = izb3 ? izb3 : ca.inv_zb + P;
  ca.col[6] = pre ? pre + 4 * P : idx_ext;
  ca.col[7] = pre ? pre + 5 * P : cols + 6 * P;
  if (f0_ext) {
    ca.col[0] = cols + P;  // K
    ca.col[1] = f0_ext;
  }
  if (pre)
    for (int c = 0; c < 4; ++c) ca.col[c] = pre + (size_t)c * P;
  ca.interp2 = consts + n_pfi;
  ca.interp3 = consts + 2 * n_pfi;
  ca.lo = tw2->d_lo;
  ca.hi = tw2->d_hi;
  ca.rows = d.rows;
  ca.plane = 0;  // the distributed prover exports its rows (stark_dprove_rows)
  ca.err = &d.d_tr->err;
  ca.prec = P;
  ca.shift1 = ((os / 3 * skips) % prec) >> d.log_g;  // multiples of 8, hence of G
  ca.shift2 = ((os / 3 * 2 * skips) % prec) >> d.log_g;
  ca.back = skips >> d.log_g;
  ca.g_add = rank;
  ca.log_g = d.log_g;
  ca.log_prec = log_prec;
  ca.kb = tw2->kb;
  ca.n2 = (uint32_t)n_pfi;
  ca.n3 = 1;
  ca.tr = d.d_tr;
  set_inv_z(ca, g2, steps);
  ca.mont_cols = pre ? 1 : 0;
  {
    const HostFp w8 = F.pow_u64(g2, steps);
    HostFp wt = F.one();
    for (int t = 0; t < 8; ++t) {
      d.xs_m[t] = to_dev(wt);
      wt = F.mul(wt, w8);
    }
  }
  STARK_TRY(upload_constraint_tables(ctx, d.d_tr, ca, s));
  hipLaunchKernelGGL(r1cs_constraint_kernel, dim3(blocks_for(P)), dim3(256), 0, s, ca);
  STARK_HIP(ctx, hipGetLastError());
  // hc2 and the uploads above must outlive the copies: wait here (the caller
  // reads a_root and the constraint flags next anyway).
  STARK_HIP(ctx, hipStreamSynchronize(s));
  return STARK_OK;
}

}  // namespace stark

using namespace stark;

extern "C" {

stark_status stark_mk_r1cs_proof(stark_ctx* ctx, const uint64_t* witness_trace, const uint64_t* computational_trace,
                                 size_t original_steps, const uint64_t* public_wires, size_t n_public,
                                 const size_t* public_first_indices, size_t n_public_first,
                                 const size_t* permuted_indices, const uint64_t* coefficients, const uint64_t* flag0,
                                 const uint64_t* flag1, const uint64_t* flag2, size_t n_constraints, size_t n_wires,
                                 stark_r1cs_proof** out) {
  if (!ctx || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  if (original_steps && (!witness_trace || !computational_trace || !permuted_indices || !coefficients || !flag0 ||
                         !flag1 || !flag2))
    return STARK_ERR_BAD_ARG;
  if ((n_public && !public_wires) || (n_public_first && !public_first_indices)) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const stark_status st = prove_r1cs(ctx, witness_trace, computational_trace, original_steps, public_wires, n_public,
                                     public_first_indices, n_public_first, permuted_indices, coefficients, flag0,
                                     flag1, flag2, nullptr, n_constraints, n_wires, out);
  hipStreamSynchronize(ctx->stream);
  return st;
}

stark_status stark_r1cs_proof_json(const stark_r1cs_proof* proof, char* buf, size_t cap, size_t* len) {
  if (!proof || !len) return STARK_ERR_BAD_ARG;
  *len = proof->json.size();
  if (buf && cap) {
    const size_t k = proof->json.size() < cap ? proof->json.size() : cap;
    host_memcpy(buf, proof->json.data(), k);
    if (k < cap) buf[k] = 0;
  }
  return STARK_OK;
}

stark_status stark_r1cs_proof_json_view(const stark_r1cs_proof* proof, const char** data, size_t* len) {
  if (!proof || !data || !len) return STARK_ERR_BAD_ARG;
  *data = proof->json.data();
  *len = proof->json.size();
  return STARK_OK;
}

stark_status stark_r1cs_proof_roots(const stark_r1cs_proof* proof, uint8_t m_root[32], uint8_t l_root[32],
                                    uint8_t a_root[32]) {
  if (!proof) return STARK_ERR_BAD_ARG;
  if (m_root) memcpy(m_root, proof->m_root, 32);
  if (l_root) memcpy(l_root, proof->l_root, 32);
  if (a_root) memcpy(a_root, proof->a_root, 32);
  return STARK_OK;
}

stark_status stark_r1cs_proof_branches(const stark_r1cs_proof* proof, int which, size_t* k, size_t* leaf_len,
                                       size_t* depth, uint8_t* leaves, size_t leaves_cap, uint8_t* nodes,
                                       size_t nodes_cap) {
  if (!proof || (which != 0 && which != 1)) return STARK_ERR_BAD_ARG;
  const size_t ll = which == 0 ? 256 : 32;
  const std::vector<uint8_t>& lv = which == 0 ? proof->m_leaves : proof->l_leaves;
  const std::vector<uint8_t>& nd = which == 0 ? proof->m_nodes : proof->l_nodes;
  if (k) *k = lv.size() / ll;
  if (leaf_len) *leaf_len = ll;
  if (depth) *depth = proof->depth;
  // capacities checked before either buffer is written
  if ((leaves && leaves_cap < lv.size()) || (nodes && nodes_cap < nd.size())) return STARK_ERR_BAD_LENGTH;
  if (leaves) memcpy(leaves, lv.data(), lv.size());
  if (nodes) memcpy(nodes, nd.data(), nd.size());
  return STARK_OK;
}

const stark_fri_proof* stark_r1cs_proof_fri(const stark_r1cs_proof* proof) { return proof ? proof->fri : nullptr; }

void stark_r1cs_proof_free(stark_r1cs_proof* proof) { delete proof; }

stark_status stark_dprove_begin(stark_ctx* ctx, uint32_t world, uint32_t rank, const uint64_t* witness_trace,
                                const uint64_t* computational_trace, size_t original_steps,
                                const uint64_t* public_wires, size_t n_public, const size_t* public_first_indices,
                                size_t n_public_first, const size_t* permuted_indices, const uint64_t* coefficients,
                                const uint64_t* flag0, const uint64_t* flag1, const uint64_t* flag2,
                                size_t n_constraints, size_t n_wires, void* stream, stark_dprove** out) {
  if (!ctx || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  if (original_steps && (!witness_trace || !computational_trace || !permuted_indices || !coefficients || !flag0 ||
                         !flag1 || !flag2))
    return STARK_ERR_BAD_ARG;
  if ((n_public && !public_wires) || (n_public_first && !public_first_indices)) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  auto h = std::make_unique<stark_dprove>();
  hipStream_t s = pick_stream(ctx, stream);
  const stark_status st = dprove_begin(ctx, world, rank, witness_trace, computational_trace, original_steps,
                                       public_wires, n_public, public_first_indices, n_public_first, permuted_indices,
                                       coefficients, flag0, flag1, flag2, nullptr, n_constraints, n_wires, s, h.get());
  if (st != STARK_OK) {
    hipStreamSynchronize(s);
    return st;
  }
  *out = h.release();
  return STARK_OK;
}

}  // extern "C"

stark_status stark::dprove_begin_prepared(stark_ctx* ctx, uint32_t world, uint32_t rank, const uint64_t* witness_trace,
                                          const uint64_t* computational_trace, size_t os, const uint64_t* public_wires,
                                          size_t n_public, const size_t* public_first_indices, size_t n_pfi,
                                          const size_t* permuted_indices, const uint64_t* coefficients,
                                          const uint8_t* flag_bytes, size_t n_constraints, size_t n_wires,
                                          const fe* pre, void* stream, stark_dprove** out) {
  if (!ctx || !out || !pre) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  auto h = std::make_unique<stark_dprove>();
  hipStream_t s = pick_stream(ctx, stream);
  const stark_status st = dprove_begin(ctx, world, rank, witness_trace, computational_trace, os, public_wires,
                                       n_public, public_first_indices, n_pfi, permuted_indices, coefficients, nullptr,
                                       nullptr, nullptr, flag_bytes, n_constraints, n_wires, s, h.get(), pre);
  if (st != STARK_OK) {
    hipStreamSynchronize(s);
    return st;
  }
  *out = h.release();
  return STARK_OK;
}

extern "C" {

stark_status stark_dprove_begin_bytes(stark_ctx* ctx, uint32_t world, uint32_t rank, const uint8_t* r1cs,
                                      size_t r1cs_len, const uint8_t* wtns, size_t wtns_len, void* stream,
                                      stark_dprove** out) {
  if (!ctx || !r1cs || !wtns || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  DevTrace dt;
  stark_status st = r1cs_trace_device(ctx, r1cs, r1cs_len, wtns, wtns_len, &dt);
  if (st != STARK_OK) return st;
  return dprove_begin_trace(ctx, world, rank, dt, stream, out);
}

}  // extern "C"

stark_status stark::dprove_begin_trace(stark_ctx* ctx, uint32_t world, uint32_t rank, const DevTrace& dt, void* stream,
                                       stark_dprove** out) {
  if (!ctx || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  STARK_HIP(ctx, hipStreamSynchronize(ctx->stream));  // the trace builder runs on the context stream
  auto h = std::make_unique<stark_dprove>();
  hipStream_t s = pick_stream(ctx, stream);
  const stark_status st = dprove_begin(ctx, world, rank, (const uint64_t*)dt.wit, (const uint64_t*)dt.comp, dt.os,
                                       dt.public_wires.data(), dt.public_wires.size() / 4,
                                       dt.public_first_indices.data(), dt.public_first_indices.size() / 2,
                                       (const size_t*)dt.perm, (const uint64_t*)dt.coef, nullptr, nullptr, nullptr,
                                       dt.flags, dt.n_constraints, dt.n_wires, s, h.get());
  if (st != STARK_OK) {
    hipStreamSynchronize(s);
    return st;
  }
  *out = h.release();
  return STARK_OK;
}

extern "C" {

stark_status stark_dprove_info(stark_dprove* h, size_t* precision, size_t* n_local, size_t* original_steps,
                               uint64_t g2[4], uint8_t a_root[32]) {
  if (!h) return STARK_ERR_BAD_ARG;
  DProveState& d = h->st;
  if (precision) *precision = d.prec;
  if (n_local) *n_local = d.P;
  if (original_steps) *original_steps = d.os;
  if (g2) memcpy(g2, d.g2c, 32);
  Transcript t;
  STARK_HIP(d.ctx, hipMemcpyAsync(&t, d.d_tr, sizeof(Transcript), hipMemcpyDeviceToHost, d.s));
  STARK_HIP(d.ctx, hipStreamSynchronize(d.s));
  if (a_root) memcpy(a_root, t.roots[0], 32);
  if (t.err) {
    d.ctx->last_error = (t.err & 1) ? "invalid D: Q does not vanish where Z does (utils.rs:379-418)"
                                    : "invalid B: boundary value mismatch (utils.rs:477-524)";
    return STARK_ERR_CHECK;
  }
  return STARK_OK;
}

stark_status stark_dprove_rows(stark_dprove* h, uint8_t** rows_dev) {
  if (!h || !rows_dev) return STARK_ERR_BAD_ARG;
  *rows_dev = (uint8_t*)h->st.rows;
  return STARK_OK;
}

// k from the main tree's root (prove.rs:274-283) on the device, then L at this rank's points; the root
// is host memory (m_root) or device memory (d_m_root, no host round trip).
static stark_status dprove_lincomb(stark_dprove* h, const uint8_t* m_root, const uint8_t* d_m_root, uint64_t** l_dev) {
  DProveState& d = h->st;
  const Mont mc = mont();
  STARK_HIP(d.ctx, hipSetDevice(d.ctx->device));
  const uint32_t* d_root = (const uint32_t*)d_m_root;
  if (m_root) {
    STARK_HIP(d.ctx, hipMemcpyAsync(d.d_tr->roots[1], m_root, 32, hipMemcpyHostToDevice, d.s));
    d_root = d.d_tr->roots[1];
  }
  XsPowers xs;
  for (int t = 0; t < 8; ++t) xs.v[t] = d.xs_m[t];
  hipLaunchKernelGGL(r1cs_k_kernel, dim3(1), dim3(kKThreads), 0, d.s, (const uint32_t*)d_root, mc.r2, mc.one, xs,
                     pow32(), d.d_tr);
  STARK_HIP(d.ctx, hipGetLastError());
  LincombArgs la;
  la.rows = d.rows;
  la.plane = 0;
  la.out = d.lvals;
  la.prec = d.P;
  la.g_add = d.r;
  la.log_g = d.log_g;
  la.tr = d.d_tr;
  hipLaunchKernelGGL(r1cs_lincomb_kernel, dim3(blocks_for(d.P)), dim3(256), 0, d.s, la);
  STARK_HIP(d.ctx, hipGetLastError());
  if (m_root) STARK_HIP(d.ctx, hipStreamSynchronize(d.s));  // m_root is the caller's (pageable) buffer
  *l_dev = (uint64_t*)d.lvals;
  return STARK_OK;
}

stark_status stark_dprove_lincomb(stark_dprove* h, const uint8_t m_root[32], uint64_t** l_dev) {
  if (!h || !m_root || !l_dev) return STARK_ERR_BAD_ARG;
  return dprove_lincomb(h, m_root, nullptr, l_dev);
}

stark_status stark_dprove_lincomb_dev(stark_dprove* h, const uint8_t* d_m_root, uint64_t** l_dev) {
  if (!h || !d_m_root || !l_dev || (((uintptr_t)d_m_root) & 3)) return STARK_ERR_BAD_ARG;
  return dprove_lincomb(h, nullptr, d_m_root, l_dev);
}

void stark_dprove_free(stark_dprove* h) { delete h; }

}  // extern "C"
