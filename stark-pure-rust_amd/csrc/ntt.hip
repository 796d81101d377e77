// NTT over BN254 Fr on gfx950: natural order in, natural order out, exactly
// best_fft / inv_best_fft's output (packages/fri/src/fft.rs:150-379):
//   out[i] = sum_j c_j w^(i j)           (forward)
//   out[i] = n^-1 sum_j c_j w^-(i j)     (inverse)
//
// Algorithm: mixed-radix Stockham decomposition n = R_0 * R_1 * ... .  Pass p
// (radix R = 2^LOG_R, Ns = R_0 * ... * R_{p-1}) reads column j as
// in[j + r n/R], applies the column twiddle w_{Ns R}^{(j mod Ns) r}, performs
// an R-point DFT in LDS (radix-2 DIT over a bit-reversed LDS image) and
// writes out[(j / Ns) Ns R + (j mod Ns) + r Ns].  A workgroup owns B adjacent
// columns so every global access is a run of B*32 contiguous bytes, and the
// LDS image is [r][b] so adjacent lanes touch adjacent 32-B slots.
//
// Data stays canonical, twiddles are Montgomery (see fp_dev.h), so no
// to/from-Montgomery passes are needed; the inverse's n^-1 is folded into
// the last pass's store.
#include <stdlib.h>

#include "fe_db.h"
#include "internal.h"

namespace stark {

// Twiddle of column exponent e (< n): direct table when the pass's
// w_{Ns R} powers fit the 2^16-entry table, else the two-level lo * hi form.
struct ColTw {
  const fe* t16;    // Shoup pairs of t16[i] = w^(i * n / 2^l16), i < 2^l16 (t16[2i], t16[2i + 1])
  const fe* lo;     // lo[i]  = w^i,                i < 2^kb
  const fe* hi;     // hi[i]  = w^(i 2^kb),         i < 2^(log_n - kb)
  const fe* full;   // last pass only: full[c R + r] = w^(c r) (or null)
  uint32_t l16, kb;
  const fe* post;   // last pass only: output k is multiplied by post[k] (Montgomery), or null
};

// One Stockham pass (see the file comment): each workgroup transforms one tile of B adjacent
// columns x R points.  T = B*R/4 threads, each owning exactly 4 elements in every phase.

// Two independent Montgomery products interleaved in one asm block (the full-table and two-level
// column twiddles).  Shoup products stay one chain per block: the interleaved pair measured 1.867 vs
// 1.843 ms per 2^24 transform.
__device__ __forceinline__ void shoup2(fe& r, fe& s, const fe& a, const fe& w, const fe& wq, const fe& c,
                                       const fe& x, const fe& xq) {
  r = fe_mul_shoup(a, w, wq);
  s = fe_mul_shoup(c, x, xq);
}
__device__ __forceinline__ void mul2(fe& r, fe& s, const fe& a, const fe& b, const fe& c, const fe& d) {
  fe_mul_lazy2(r, s, a, b, c, d);
}

// fe_bfly_lazy for an X input already below 2p (a product or a canonical load): no reduction of X.
__device__ __forceinline__ void bfly_lt2p(fe& x, fe& y, const fe& t) {
  fe_bfly_lazy_reduced(x, y, t);
}

// The pass's lazy range is [0, 4p + 2^224) (4p + 2^224 < 2^256: top word 0xc19139cb).
// csub2p_top: x <- x - 2p when x's top word is above 2p's (so x > 2p), a branch over the 8-word
// subtraction (exec-masked: 1 compare + 8 VALU instead of the 8 + 8 of a select); the result is
// below 2p + 2^224 (an x not subtracted has a top word <= 2p's).
__device__ __forceinline__ void sub2p(fe& t) {
  const P2Limbs q = p2_vgprs();  // (a literal and VCC would both take gfx950's one constant-bus read)
  asm("v_sub_co_u32 %0, vcc, %0, %8\n\t"
      "v_subb_co_u32 %1, vcc, %1, %9, vcc\n\t"
      "v_subb_co_u32 %2, vcc, %2, %10, vcc\n\t"
      "v_subb_co_u32 %3, vcc, %3, %11, vcc\n\t"
      "v_subb_co_u32 %4, vcc, %4, %12, vcc\n\t"
      "v_subb_co_u32 %5, vcc, %5, %13, vcc\n\t"
      "v_subb_co_u32 %6, vcc, %6, %14, vcc\n\t"
      "v_subb_co_u32 %7, vcc, %7, %15, vcc"
      : "+v"(t.w[0]), "+v"(t.w[1]), "+v"(t.w[2]), "+v"(t.w[3]), "+v"(t.w[4]), "+v"(t.w[5]), "+v"(t.w[6]),
        "+v"(t.w[7])
      : "v"(q.l[0]), "v"(q.l[1]), "v"(q.l[2]), "v"(q.l[3]), "v"(q.l[4]), "v"(q.l[5]), "v"(q.l[6]), "v"(q.l[7])
      : "vcc");
}
__device__ __forceinline__ void csub2p_top(fe& t) {
  if (t.w[7] > STARK_2P7) sub2p(t);
}
// X in [0, 4p + 2^224), T in [0, 2p): x <- X' + T, y <- X' + 2p - T, both in [0, 4p + 2^224).
template <bool FAST>
__device__ __forceinline__ void bfly(fe& x, fe& y, const fe& t) {
  if (FAST) {
    csub2p_top(x);
    fe_bfly_lazy_reduced(x, y, t);
  } else {
    fe_bfly_lazy(x, y, t);
  }
}
// [0, 4p + 2^224) -> [0, 2p) (an unmultiplied value taking a butterfly's T role).
template <bool FAST>
__device__ __forceinline__ void csub2p_t(fe& t) {
  if (FAST) csub2p_top(t);
  fe_csub2p(t);
}
// [0, 4p + 2^224) -> canonical.
template <bool FAST>
__device__ __forceinline__ void reduce_full(fe& t) {
  csub2p_t<FAST>(t);
  fe_reduce_once(t);
}

// The digit-basis table of constant k in LDS: 72 u32 per constant, 16-B aligned.  Constants 8 apart
// would share banks (72 * 8 = 0 mod 64 banks) and a radix-4 step reads k, k + 8, k + 16, k + 24 in
// one ds_read_b128 lane group, so each group of 8 constants starts 4 banks after the previous one.
__device__ __forceinline__ const uint32_t* dbt(const uint32_t* sdb, uint32_t k) {
  return static_cast<const uint32_t*>(__builtin_assume_aligned(sdb + 72 * k + 4 * (k >> 3), 16));
}

// COL: the pass's column-twiddle source, fixed per launch so each instance carries one product
// form (kColNone: first pass; kColFull: last-pass full table, Montgomery; kColT16: Shoup pairs;
// kColTwoLevel: lo * hi, Montgomery).
enum : int { kColNone = 0, kColFull = 1, kColT16 = 2, kColTwoLevel = 3, kColSparse = 4 };
// (kColSparse: a first pass over a zero-padded input (Sparse::skip > 0); no column twiddle either.)

// Elements per workgroup tile: 2^10 (B = 1024 / R columns, 256 threads).  4096- and 2048-element
// tiles measured slower (one or two workgroups per CU leave the barriers uncovered).
constexpr uint32_t kTileLog = 10;
constexpr uint32_t kPassThreads = (1u << kTileLog) / 4;

// Which radix-4 steps multiply by the digit-basis product (fe_db.h), radices 2^4..2^8:
//   * every step before the pass's last one: constants w_R^(4k), k < R/8 (32 for R = 256, 9 KB of
//     LDS, staged once per workgroup).  Where a wave's constant is uniform (the first step's w_4 and
//     the jj-major first twiddled step) its table is read from the global one into SGPRs instead
//     (scalar loads; the column sums take it as the SGPR operand of v_mad_u64_u32): no LDS reads;
//   * the last step too for radices 2^4..2^7 (2^7 outside sparse passes): once the step has read its inputs, all R/2 constants
//     (L2-resident, <= 18 KB) are staged over the data image (two more barriers per tile).
// (Measured and dropped, DESIGN.md section 5: no digit basis, the R/2-constant table resident (2
// workgroups per CU), the m <= 4 steps only with global Shoup pairs, the tables read through L1.)
// Radix 2^8, and radix 2^7 in a sparse first pass, run as T x 16 inside the tile (`four`, T = R/16): after the first stages (a
// T-point DFT over each group of T image rows) every element is multiplied by its twiddle w_R^(r1 k1),
// and the last two radix-4 steps are a 16-point DFT across the groups, whose constants (w_4, and
// w_16^a for the wave's a) are wave-uniform.  Every digit-basis constant of the pass then comes from
// SGPRs; the only per-lane constants are the twiddles, Shoup pairs of w_R^e, e < R, staged in LDS
// (16 / 8 KB).  The LDE's sparse first pass (radix 2^7, three copy stages) enters at the twiddles.
template <int LOG_R, int COL>
struct DbPlan {
  static constexpr bool on = LOG_R >= 4 && LOG_R <= 8;
  static constexpr bool four = LOG_R == 8 || (LOG_R == 7 && COL == kColSparse);
  static constexpr int s_end = on ? LOG_R - 2 : 0;  // DB for steps s < s_end
  static constexpr uint32_t stride = 4;             // the table holds w_R^(4 k), k < R / 8
  static constexpr uint32_t entries = (on && !four) ? (1u << LOG_R) / (2 * stride) : 0;
  // 72 u32 per constant, plus 4 u32 of bank rotation per 8 constants (dbt)
  static constexpr uint32_t lds_fe = entries * 9 + entries / 16;
  static constexpr bool last = on && !four && LOG_R <= 7;
  static constexpr uint32_t full_entries = last ? (1u << LOG_R) / 2 : 0;
  static constexpr uint32_t full_fe = full_entries * 9 + full_entries / 16;
  // staged Shoup pairs: the last step's w_R^k, k < R/2, or the twiddles' w_R^e, e < R (four)
  static constexpr uint32_t shoup_fe = last ? 0 : four ? 2 * (1u << LOG_R) : (1u << LOG_R);
  static constexpr int occupancy = on ? 3 : 4;                     // workgroups per CU the LDS allows
};

// Streaming (non-temporal) forms of fe_load / fe_store: one use per transform, nothing to keep in L2.
// The passes store through fe_store_nt and the last pass reads its full twiddle table through
// fe_load_nt (2^20 -3.5 %, 2^22 -1.9 %, 2^26 -1.4 %, 2^24 within noise; tools/ab_libs.py,
// profiles/r05_nt_ab.txt).  Non-temporal tile loads measured +3.6 % at 2^24 and are not used.
typedef unsigned int u32x4_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ fe fe_load_nt(const fe* p) {
  const u32x4_nt* q = reinterpret_cast<const u32x4_nt*>(p);
  const u32x4_nt lo = __builtin_nontemporal_load(q), hi = __builtin_nontemporal_load(q + 1);
  fe r;
  r.w[0] = lo.x; r.w[1] = lo.y; r.w[2] = lo.z; r.w[3] = lo.w;
  r.w[4] = hi.x; r.w[5] = hi.y; r.w[6] = hi.z; r.w[7] = hi.w;
  return r;
}
__device__ __forceinline__ void fe_store_nt(fe* p, const fe& v) {
  u32x4_nt* q = reinterpret_cast<u32x4_nt*>(p);
  __builtin_nontemporal_store(u32x4_nt{v.w[0], v.w[1], v.w[2], v.w[3]}, q);
  __builtin_nontemporal_store(u32x4_nt{v.w[4], v.w[5], v.w[6], v.w[7]}, q + 1);
}

// LDS data image of a pass, element index i = (row << log_b) + column.  The two 16-B halves of each
// element sit in separate planes (lo at v[i], hi at v[n + i]), so the 16 lanes of a ds_read_b128 group
// read 16 adjacent 16-B slots instead of every other one.
struct XImage {
  fe* base;
  uint32_t n;  // elements
  __device__ __forceinline__ fe ld(uint32_t i) const {
    const uint4* v = reinterpret_cast<const uint4*>(base);
    const uint4 lo = v[i], hi = v[n + i];
    fe r;
    r.w[0] = lo.x; r.w[1] = lo.y; r.w[2] = lo.z; r.w[3] = lo.w;
    r.w[4] = hi.x; r.w[5] = hi.y; r.w[6] = hi.z; r.w[7] = hi.w;
    return r;
  }
  __device__ __forceinline__ void st(uint32_t i, const fe& x) const {
    uint4* v = reinterpret_cast<uint4*>(base);
    v[i] = make_uint4(x.w[0], x.w[1], x.w[2], x.w[3]);
    v[n + i] = make_uint4(x.w[4], x.w[5], x.w[6], x.w[7]);
  }
};

template <int LOG_R, int COL>
__global__ __launch_bounds__(kPassThreads, (DbPlan<LOG_R, COL>::occupancy)) void ntt_pass_kernel(
    const fe* __restrict__ in, fe* __restrict__ out, uint32_t log_n, uint32_t log_ns, uint32_t log_b, ColTw ct,
    const fe* __restrict__ small, const uint32_t* __restrict__ db, fe scale, int do_scale, uint32_t log_tiles,
    uint32_t total_tiles, Sparse sp) {
  constexpr uint32_t R = 1u << LOG_R;
  using DB = DbPlan<LOG_R, COL>;
  // The top-word reduction (csub2p_top) in the radix-2^6 passes only: there it measured 1.2 % faster at
  // 2^26 (6, 6, 6, 8); in the 16 x 16 radix-2^8 passes it was 1.1 % slower at 2^24, and 2 % slower in the
  // radix-2^4 pass of 2^20 (profiles/r05_csub_top_ab.txt).
  constexpr bool FAST = LOG_R == 6;
  extern __shared__ __attribute__((aligned(16))) fe lds[];
  fe* sm = lds;          // R/2 small roots w_R^k as Shoup pairs: sm[2k] = w_R^k, sm[2k + 1] = its quotient
  uint32_t* sdb = reinterpret_cast<uint32_t*>(lds + DB::shoup_fe);  // digit-basis tables (DbPlan)
  fe* X = lds + DB::shoup_fe + DB::lds_fe;  // [R][B] data image
  const uint32_t B = 1u << log_b;
  const XImage XI{X, B << LOG_R};
  const uint32_t nthr = (B << LOG_R) >> 2;  // active threads
  const uint32_t tid = threadIdx.x;
  const bool active = tid < nthr;
  const uint32_t log_cols = log_n - LOG_R;
  const size_t ns_mask = ((size_t)1 << log_ns) - 1;
  const uint32_t tile_mask = (1u << log_tiles) - 1;
  const uint32_t tile = blockIdx.x;
  if (tile >= total_tiles) return;  // (uniform per workgroup)

  // This thread's 4 elements of a tile: (eb[t], er[t]) = (column, row) as stored and loaded.
  uint32_t eb[4], er[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t e = tid + (uint32_t)t * nthr;
    eb[t] = e & (B - 1);
    er[t] = e >> log_b;
  }
  const uint32_t b = tid & (B - 1);
  const uint32_t q = tid >> log_b;  // radix-4 group within the column

  // Sparse first pass (sp.skip > 0): only rows < R >> sp.zero_log are
  // non-zero (read from a compact input of batch stride 2^sp.log_in), and the
  // first sp.skip radix-2 stages are copies; rows < R >> sp.skip are loaded.
  const uint32_t live_rows = R >> sp.skip, nz_rows = R >> sp.zero_log;
  const uint32_t log_in = sp.zero_log ? sp.log_in : log_n;
  fe v[4];
  if (active) {
    const fe* src = in + ((size_t)(tile >> log_tiles) << log_in) + ((size_t)(tile & tile_mask) << log_b);
#pragma unroll
    for (int t = 0; t < 4; ++t)
      v[t] = er[t] < nz_rows ? fe_load(src + eb[t] + ((size_t)er[t] << log_cols)) : fe_zero();
  }

  // Stage the pass's LDS tables once the tile's loads are in flight, every staging load before any
  // store, so a wave waits for one memory latency instead of one per staging round.  (The global
  // digit-basis table holds every w_R^k, k < R/2; the LDS copy every stride-th one.)
  {
    constexpr uint32_t kSm = 2 * DB::shoup_fe, kDb = DB::on ? DB::entries * 18 : 0;  // 16-B units
    const uint4* db4 = reinterpret_cast<const uint4*>(db);
    const uint4* small4 = reinterpret_cast<const uint4*>(small);
    uint4* sm4 = reinterpret_cast<uint4*>(sm);
    uint4* sdb4 = reinterpret_cast<uint4*>(sdb);
    auto db_src = [&](uint32_t k) { const uint32_t e = k / 18; return (e * DB::stride) * 18 + (k - e * 18); };
    auto db_dst = [&](uint32_t k) { return k + ((k / 18) >> 3); };
    if (blockDim.x == kPassThreads) {
      constexpr uint32_t nSm = (kSm + kPassThreads - 1) / kPassThreads, nDb = (kDb + kPassThreads - 1) / kPassThreads;
      // (full rounds need no bounds test: tid < kPassThreads here)
      auto in_sm = [&](uint32_t i) { return (i + 1) * kPassThreads <= kSm || tid + i * kPassThreads < kSm; };
      auto in_db = [&](uint32_t i) { return (i + 1) * kPassThreads <= kDb || tid + i * kPassThreads < kDb; };
      uint4 ts[nSm ? nSm : 1], td[nDb ? nDb : 1];
#pragma unroll
      for (uint32_t i = 0; i < nSm; ++i)
        if (in_sm(i)) ts[i] = small4[tid + i * kPassThreads];
#pragma unroll
      for (uint32_t i = 0; i < nDb; ++i)
        if (in_db(i)) td[i] = db4[db_src(tid + i * kPassThreads)];
#pragma unroll
      for (uint32_t i = 0; i < nSm; ++i)
        if (in_sm(i)) sm4[tid + i * kPassThreads] = ts[i];
#pragma unroll
      for (uint32_t i = 0; i < nDb; ++i)
        if (in_db(i)) sdb4[db_dst(tid + i * kPassThreads)] = td[i];
    } else {
      for (uint32_t k = tid; k < kSm; k += blockDim.x) sm4[k] = small4[k];
      for (uint32_t k = tid; k < kDb; k += blockDim.x) sdb4[db_dst(k)] = db4[db_src(k)];
    }
  }
  const size_t boff = (size_t)(tile >> log_tiles) << log_n;
  const size_t j0 = (size_t)(tile & tile_mask) << log_b;

  // ---- column twiddle, scatter into the bit-reversed LDS image ----
  if (active) {
    if (COL != kColNone && COL != kColSparse) {
      const uint32_t lnr = log_ns + LOG_R;  // w_{Ns R} powers
      fe tw[4];
      if (COL == kColFull) {  // the transform's last pass (lnr == log_n) with a full table
#pragma unroll
        for (int t = 0; t < 4; ++t) tw[t] = fe_load_nt(ct.full + ((((j0 + eb[t]) & ns_mask) << LOG_R) + er[t]));
        // Montgomery images (the table streams from HBM once per transform, so it stays 32 B per
        // entry): v < 4p, tw < p -> [0, 2p); two interleaved products per block
        mul2(v[0], v[1], v[0], tw[0], v[1], tw[1]);
        mul2(v[2], v[3], v[2], tw[2], v[3], tw[3]);
      } else if (COL == kColT16) {
        // Shoup pairs from the L2-resident t16 table: v < 2^256 -> [0, 2p)
        const fe* e[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint64_t k = ((uint64_t)((j0 + eb[t]) & ns_mask) * er[t]) & (((uint64_t)1 << lnr) - 1);
          e[t] = ct.t16 + 2 * (k << (ct.l16 - lnr));
        }
        shoup2(v[0], v[1], v[0], e[0][0], e[0][1], v[1], e[1][0], e[1][1]);
        shoup2(v[2], v[3], v[2], e[2][0], e[2][1], v[3], e[3][0], e[3][1]);
      } else {
        const uint32_t unit = log_n - lnr;
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const uint64_t ex = ((uint64_t)((j0 + eb[t]) & ns_mask) * er[t]) << unit;
          tw[t] = fe_mul(ct.lo[ex & (((uint64_t)1 << ct.kb) - 1)], ct.hi[ex >> ct.kb]);
        }
        mul2(v[0], v[1], v[0], tw[0], v[1], tw[1]);
        mul2(v[2], v[3], v[2], tw[2], v[3], tw[3]);
      }
    }
    if (sp.skip == 0) {
      // The first stage in registers: the thread holds rows r0 + t R/4 of column eb, whose image rows
      // are 4 rev(r0) + {0, 2, 1, 3}[t], i.e. exactly one group of the first radix-4 step (w_4 only)
      // or two pairs of the odd radices' radix-2 stage 0.  No LDS round trip, one barrier less.
      // Its inputs are below 2p (canonical loads, or column-twiddle products in [0, 2p)), so the first
      // butterflies need no reductions.
      if ((LOG_R & 1) == 0) {  // x0..x3 = v[0], v[2], v[1], v[3]
        bfly_lt2p(v[0], v[2], v[2]);
        bfly_lt2p(v[1], v[3], v[3]);
        fe t3;
        if (DB::on) {
          t3 = fe_mul_db(v[3], db + 72u * (1u << (LOG_R - 2)));  // w_4^1 = w_R^(R/4), wave-uniform: SGPRs
        } else {
          const uint32_t ic = 2 * (1u << (LOG_R - 2));  // w_4^1 (sm is not staged yet: the global table)
          t3 = fe_mul_shoup(v[3], small[ic], small[ic + 1]);
        }
        fe_csub2p(v[1]);
        bfly<FAST>(v[0], v[1], v[1]);
        bfly<FAST>(v[2], v[3], t3);
      } else {
        bfly_lt2p(v[0], v[2], v[2]);
        bfly_lt2p(v[1], v[3], v[3]);
      }
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t rr = __builtin_bitreverse32(er[t]) >> (32 - LOG_R);
        XI.st((rr << log_b) + eb[t], v[t]);
      }
    } else {
      // Rows >= live_rows are zero, so after sp.skip DIT stages every
      // position of a group of 2^skip holds the group's one live input.
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (er[t] >= live_rows) continue;
        const uint32_t rr = __builtin_bitreverse32(er[t]) >> (32 - LOG_R);
        for (uint32_t k = 0; k < (1u << sp.skip); ++k) XI.st(((rr + k) << log_b) + eb[t], v[t]);
      }
    }
  }
  __syncthreads();

  // ---- R-point DIT over the bit-reversed image ----
  // Lazy representation: every value in LDS is in [0, 4p); products are
  // left in [0, 2p) and each radix-2 butterfly reduces only its X input
  // (fe_bfly_lazy).  The pass's last store reduces to canonical only when
  // it is the transform's last pass.
  // A dense pass did its first stage in registers before the scatter (radix-4 step s = 0 for an
  // even radix, the radix-2 stage 0 for an odd one); a sparse pass starts after its copy stages.
  int s = sp.skip ? (int)sp.skip : (LOG_R & 1) ? 1 : 2;
  // The first radix-4 step with twiddles (s0 = 2, m = 4 for an even radix; s0 = 1, m = 2 after the
  // radix-2 stage of an odd one) with a jj-major thread mapping: each 1/m of the threads takes one
  // jj, so with B R >= 1024 every wave has a single jj and the jj = 0 waves skip the products by
  // w_{2m}^0 = w_{4m}^0 = 1 (3 of 4; branch uniform per wave; lane masking was measured slower,
  // DESIGN section 5): 3n/16 products per even pass, 3n/8 per odd one.
  constexpr int kS0 = (LOG_R & 1) ? 1 : 2;
  if (LOG_R >= 5 && s == kS0) {
    if (active) {
      const uint32_t lq = LOG_R + log_b - 2 - kS0;  // log2(threads per jj)
      const uint32_t jj = tid >> lq;
      const uint32_t rest = tid & ((1u << lq) - 1);
      const uint32_t i0 = ((((rest >> log_b) << (kS0 + 2)) + jj) << log_b) + (rest & (B - 1));
      const uint32_t st = (1u << kS0) << log_b;  // m rows
      fe x0 = XI.ld(i0), x1 = XI.ld(i0 + st), x2 = XI.ld(i0 + 2 * st), x3 = XI.ld(i0 + 3 * st);
      if (jj == 0) {
        csub2p_t<FAST>(x1);
        csub2p_t<FAST>(x3);
        bfly<FAST>(x0, x1, x1);
        bfly<FAST>(x2, x3, x3);
        fe t3;
        if (DB::on) {
          t3 = fe_mul_db(x3, db + 72u * (1u << (LOG_R - 2)));  // w_{4m}^m = w_4^1
        } else {
          const uint32_t ic = 2 * (1u << (LOG_R - 2));
          t3 = fe_mul_shoup(x3, sm[ic], sm[ic + 1]);
        }
        csub2p_t<FAST>(x2);
        bfly<FAST>(x0, x2, x2);
        bfly<FAST>(x1, x3, t3);
      } else if (DB::on && DB::s_end > kS0 && lq >= 6) {
        // every wave has one jj: the constants come from the global table into SGPRs (no LDS reads)
        const uint32_t ju = __builtin_amdgcn_readfirstlane(jj);
        const uint32_t* wa = db + 72u * (ju << (LOG_R - 1 - kS0));  // w_{2m}^jj
        const fe t1 = fe_mul_db(x1, wa);
        fe t3 = fe_mul_db(x3, wa);
        bfly<FAST>(x0, x1, t1);
        bfly<FAST>(x2, x3, t3);
        const fe t2 = fe_mul_db(x2, db + 72u * (ju << (LOG_R - 2 - kS0)));                // w_{4m}^jj
        t3 = fe_mul_db(x3, db + 72u * ((ju + (1u << kS0)) << (LOG_R - 2 - kS0)));  // w_{4m}^(jj+m)
        bfly<FAST>(x0, x2, t2);
        bfly<FAST>(x1, x3, t3);
      } else if (DB::on && DB::s_end > kS0) {
        constexpr uint32_t S = DB::stride;
        // (four: no LDS table; small tiles read the global one per lane)
        auto tab = [&](uint32_t e) { return DB::four ? db + 72u * e : dbt(sdb, e / S); };
        const uint32_t* wa = tab(jj << (LOG_R - 1 - kS0));  // w_{2m}^jj
        const fe t1 = fe_mul_db(x1, wa);
        fe t3 = fe_mul_db(x3, wa);
        bfly<FAST>(x0, x1, t1);
        bfly<FAST>(x2, x3, t3);
        const fe t2 = fe_mul_db(x2, tab(jj << (LOG_R - 2 - kS0)));                // w_{4m}^jj
        t3 = fe_mul_db(x3, tab((jj + (1u << kS0)) << (LOG_R - 2 - kS0)));  // w_{4m}^(jj+m)
        bfly<FAST>(x0, x2, t2);
        bfly<FAST>(x1, x3, t3);
      } else {
        fe t1, t3;
        const uint32_t ia = 2 * (jj << (LOG_R - 1 - kS0));
        const fe ta = sm[ia], taq = sm[ia + 1];
        shoup2(t1, t3, x1, ta, taq, x3, ta, taq);
        bfly<FAST>(x0, x1, t1);
        bfly<FAST>(x2, x3, t3);
        const uint32_t ic = 2 * ((jj + (1u << kS0)) << (LOG_R - 2 - kS0));
        const fe tc = sm[ic], tcq = sm[ic + 1];
        const uint32_t ib = 2 * (jj << (LOG_R - 2 - kS0));
        const fe t2 = fe_mul_shoup(x2, sm[ib], sm[ib + 1]);
        t3 = fe_mul_shoup(x3, tc, tcq);
        bfly<FAST>(x0, x2, t2);
        bfly<FAST>(x1, x3, t3);
      }
      XI.st(i0, x0);
      XI.st(i0 + 2 * st, x2);
      XI.st(i0 + st, x1);
      XI.st(i0 + 3 * st, x3);
    }
    __syncthreads();
    s = kS0 + 2;
  }
  // ---- radix 2^8 / 2^7 as T x 16 (DbPlan::four): twiddles, then a 16-point DFT across the groups ----
  // Image row T g + t now holds Z[r1][k1 = t], the T-point DFT of the natural inputs r1 + 16 r2
  // with r1 = rev4(g); Y[k1 + T k2] = sum_r1 w_16^(r1 k2) (w_R^(r1 k1) Z[r1][k1]).  Both steps below
  // keep the generic steps' thread mapping (s = LT: rows 4 T a + t + T k; then rows q + (R/4) k), so
  // the last one still ends in the store's registers.  (A sparse pass that skips more than the first
  // LT stages arrives here with s > LT and runs the generic last steps: its copies span the twiddles.)
  bool kept = false;  // the pass's last step left its outputs in yl (the store's mapping)
  fe yl[4];
  constexpr uint32_t LT = LOG_R >= 4 ? LOG_R - 4 : 0;  // log2 of T = R / 16, the rows of a group
  if (DB::four && s == (int)LT) {
    if (active) {
      const uint32_t t = q & ((1u << LT) - 1), a = q >> LT;
      const uint32_t i0 = (((a << (LT + 2)) + t) << log_b) + b, st = (1u << LT) << log_b;
      fe x[4];
      // (group g = 0's twiddle is w^0: with one a per wave the a = 0 waves skip that product)
      const bool unit0 = ((64u >> log_b) <= (1u << LT) ? __builtin_amdgcn_readfirstlane(a) : a) == 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const fe v = XI.ld(i0 + k * st);
        if (k == 0 && unit0) {
          x[0] = v;
          fe_csub2p(x[0]);  // [0, 4p) -> [0, 2p)
          continue;
        }
        const uint32_t e = (__builtin_bitreverse32((a << 2) + k) >> 28) * t;  // rev4(g) k1, < R
        x[k] = fe_mul_shoup(v, sm[2 * e], sm[2 * e + 1]);                      // [0, 2p)
      }
      // 16-point DFT across the groups, first radix-4 step (stride 16 rows): only w_4 (SGPRs); the
      // twiddled inputs are below 2p
      bfly_lt2p(x[0], x[1], x[1]);
      bfly_lt2p(x[2], x[3], x[3]);
      const fe t3 = fe_mul_db(x[3], db + 72u * (1u << (LOG_R - 2)));
      fe_csub2p(x[2]);
      bfly<FAST>(x[0], x[2], x[2]);
      bfly<FAST>(x[1], x[3], t3);
#pragma unroll
      for (int k = 0; k < 4; ++k) XI.st(i0 + k * st, x[k]);
    }
    __syncthreads();
    if (active) {
      // second radix-4 step (stride R/4 rows, jj = a = q >> LT): w_8^a, w_16^a, w_16^(a + 4)
      const uint32_t i0 = (q << log_b) + b, st = (R / 4) << log_b;
      fe x0 = XI.ld(i0), x1 = XI.ld(i0 + st), x2 = XI.ld(i0 + 2 * st), x3 = XI.ld(i0 + 3 * st);
      auto step = [&](const uint32_t a) {
        if (a == 0) {
          csub2p_t<FAST>(x1);
          csub2p_t<FAST>(x3);
          bfly<FAST>(x0, x1, x1);
          bfly<FAST>(x2, x3, x3);
          const fe t3 = fe_mul_db(x3, db + 72u * (1u << (LOG_R - 2)));  // w_4
          csub2p_t<FAST>(x2);
          bfly<FAST>(x0, x2, x2);
          bfly<FAST>(x1, x3, t3);
        } else {
          const uint32_t* wa = db + 72u * (a << (LOG_R - 3));  // w_8^a = w_R^(a R/8)
          const fe t1 = fe_mul_db(x1, wa);
          fe t3 = fe_mul_db(x3, wa);
          bfly<FAST>(x0, x1, t1);
          bfly<FAST>(x2, x3, t3);
          const fe t2 = fe_mul_db(x2, db + 72u * (a << LT));  // w_16^a = w_R^(a R/16)
          t3 = fe_mul_db(x3, db + 72u * ((a + 4) << LT));     // w_16^(a + 4)
          bfly<FAST>(x0, x2, t2);
          bfly<FAST>(x1, x3, t3);
        }
      };
      // a wave holds 64 / B consecutive q, all with one a when 64 / B <= T (the 1024-element tile): a is
      // uniform, its constants come from SGPRs; smaller tiles read them per lane
      if ((64u >> log_b) <= (1u << LT))
        step(__builtin_amdgcn_readfirstlane(q >> LT));
      else
        step(q >> LT);
      yl[0] = x0;
      yl[1] = x1;
      yl[2] = x2;
      yl[3] = x3;
    }
    kept = true;
    s = LOG_R;
  }
  if (DB::on && !DB::four) {
#pragma unroll 1
    for (; s < DB::s_end; s += 2) {
      if (active) {
        const uint32_t m = 1u << s;
        const uint32_t jj = q & (m - 1);
        const uint32_t base = ((q >> s) << (s + 2)) + jj;
        fe x0 = XI.ld((base << log_b) + b);
        fe x1 = XI.ld(((base + m) << log_b) + b);
        fe x2 = XI.ld(((base + 2 * m) << log_b) + b);
        fe x3 = XI.ld(((base + 3 * m) << log_b) + b);
        // exponents (in w_R units) jj R/2m, jj R/4m, (jj + m) R/4m: multiples of 4 before the last step
        constexpr uint32_t S = DB::stride;
        const uint32_t* wa = dbt(sdb, (jj << (LOG_R - 1 - s)) / S);  // w_{2m}^jj
        const fe t1 = fe_mul_db(x1, wa);
        fe t3 = fe_mul_db(x3, wa);
        bfly<FAST>(x0, x1, t1);  // (y0, y1)
        bfly<FAST>(x2, x3, t3);  // (y2, y3)
        const fe t2 = fe_mul_db(x2, dbt(sdb, (jj << (LOG_R - 2 - s)) / S));  // w_{4m}^jj
        t3 = fe_mul_db(x3, dbt(sdb, ((jj + m) << (LOG_R - 2 - s)) / S));   // w_{4m}^(jj+m)
        bfly<FAST>(x0, x2, t2);
        bfly<FAST>(x1, x3, t3);
        XI.st((base << log_b) + b, x0);
        XI.st(((base + 2 * m) << log_b) + b, x2);
        XI.st(((base + m) << log_b) + b, x1);
        XI.st(((base + 3 * m) << log_b) + b, x3);
      }
      __syncthreads();
    }
  }
  // The last radix-4 step (m = R/4) leaves thread tid the rows q + k R/4 of column b: exactly the
  // elements (er[k], eb[k]) it stores, so it keeps them in registers (no LDS round trip and one
  // barrier less per tile; radix 2^9 spills at its 128-register budget).
  constexpr bool fuse = LOG_R <= 8;
#pragma unroll 1
  for (; s < (DB::last ? LOG_R - 2 : LOG_R); s += 2) {
    const bool keep = fuse && s == LOG_R - 2;  // uniform
    if (active) {
      const uint32_t m = 1u << s;
      const uint32_t jj = q & (m - 1);
      const uint32_t base = ((q >> s) << (s + 2)) + jj;
      fe x0 = XI.ld((base << log_b) + b);
      fe x1 = XI.ld(((base + m) << log_b) + b);
      fe x2 = XI.ld(((base + 2 * m) << log_b) + b);
      fe x3 = XI.ld(((base + 3 * m) << log_b) + b);
      fe t1, t3;
      const uint32_t ia = 2 * (jj << (LOG_R - 1 - s));  // w_{2m}^jj, Shoup pairs staged in LDS
      const fe ta = sm[ia], taq = sm[ia + 1];
      shoup2(t1, t3, x1, ta, taq, x3, ta, taq);
      bfly<FAST>(x0, x1, t1);  // (y0, y1)
      bfly<FAST>(x2, x3, t3);  // (y2, y3)
      const uint32_t ic = 2 * ((jj + m) << (LOG_R - 2 - s));  // w_{4m}^(jj+m)
      const fe tc = sm[ic], tcq = sm[ic + 1];
      const uint32_t ib = 2 * (jj << (LOG_R - 2 - s));  // w_{4m}^jj
      const fe t2 = fe_mul_shoup(x2, sm[ib], sm[ib + 1]);
      t3 = fe_mul_shoup(x3, tc, tcq);
      bfly<FAST>(x0, x2, t2);
      bfly<FAST>(x1, x3, t3);
      if (keep) {
        yl[0] = x0;
        yl[1] = x1;
        yl[2] = x2;
        yl[3] = x3;
      } else {
        XI.st((base << log_b) + b, x0);
        XI.st(((base + 2 * m) << log_b) + b, x2);
        XI.st(((base + m) << log_b) + b, x1);
        XI.st(((base + 3 * m) << log_b) + b, x3);
      }
    }
    kept = keep;
    if (!keep) __syncthreads();
  }
  if (DB::last && s == LOG_R - 2) {  // (a sparse first pass whose copy stages cover all of R has none)
    // Last step (s = LOG_R - 2, m = R/4: thread q owns rows q + k m of column b) by the digit basis:
    // read the inputs, then stage the R/2 constants over the data image (L2-resident table).
    const uint32_t m = 1u << (LOG_R - 2);
    const uint32_t i0 = (q << log_b) + b, st = m << log_b;
    fe x0, x1, x2, x3;
    if (active) {
      x0 = XI.ld(i0);
      x1 = XI.ld(i0 + st);
      x2 = XI.ld(i0 + 2 * st);
      x3 = XI.ld(i0 + 3 * st);
    }
    __syncthreads();
    uint32_t* ft = reinterpret_cast<uint32_t*>(X);
    for (uint32_t k = tid; k < DB::full_entries * 18; k += blockDim.x) {
      const uint32_t e = k / 18;
      reinterpret_cast<uint4*>(ft)[k + (e >> 3)] = reinterpret_cast<const uint4*>(db)[k];
    }
    __syncthreads();
    if (active) {
      const uint32_t jj = q;
      const uint32_t* wa = dbt(ft, 2 * jj);  // w_{2m}^jj = w_R^(2 jj)
      const fe t1 = fe_mul_db(x1, wa);
      fe t3 = fe_mul_db(x3, wa);
      bfly<FAST>(x0, x1, t1);
      bfly<FAST>(x2, x3, t3);
      const fe t2 = fe_mul_db(x2, dbt(ft, jj));  // w_{4m}^jj
      t3 = fe_mul_db(x3, dbt(ft, jj + m));       // w_{4m}^(jj+m)
      bfly<FAST>(x0, x2, t2);
      bfly<FAST>(x1, x3, t3);
      yl[0] = x0;
      yl[1] = x1;
      yl[2] = x2;
      yl[3] = x3;
    }
    kept = fuse;
    if (!fuse) {  // the store reads the image: write it back once the table is no longer read
      __syncthreads();
      if (active) {
        XI.st(i0, yl[0]);
        XI.st(i0 + st, yl[1]);
        XI.st(i0 + 2 * st, yl[2]);
        XI.st(i0 + 3 * st, yl[3]);
      }
      __syncthreads();
    }
  }

  // ---- store: out[(j / Ns) Ns R + (j mod Ns) + r Ns] ----
  const bool last = log_ns + LOG_R == log_n;  // the transform's last pass stores canonical values
  if (active) {
    fe* dst = out + boff;
    if (kept || ((size_t)1 << log_ns) >= B) {
      // (Ns < B from registers, the first pass: each wave stores B runs of 16 adjacent outputs.)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const size_t j = j0 + eb[t];
        const size_t o = ((j >> log_ns) << (log_ns + LOG_R)) + (j & ns_mask) + ((size_t)er[t] << log_ns);
        fe val = kept ? yl[t] : XI.ld((er[t] << log_b) + eb[t]);
        if (last && ct.post) {  // (uniform branch) the products take [0, 4p) inputs and reduce fully
          if (do_scale) val = fe_mul(val, scale);
          val = fe_mul(val, ct.post[o]);
        } else {
          if (last) reduce_full<FAST>(val);
          if (do_scale) val = fe_mul(val, scale);
        }
        fe_store_nt(dst + o, val);
      }
    } else {
      // Ns < B: the tile's output is the contiguous run [j0 R, (j0 + B) R).
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t o = tid + (uint32_t)t * nthr;
        const uint32_t qq = o >> (log_ns + LOG_R);
        const uint32_t rem = o & ((1u << (log_ns + LOG_R)) - 1);
        const uint32_t r = rem >> log_ns;
        const uint32_t bb = (qq << log_ns) + (rem & (uint32_t)ns_mask);
        fe val = XI.ld((r << log_b) + bb);
        if (last) reduce_full<FAST>(val);
        if (do_scale) val = fe_mul(val, scale);
        if (last && ct.post) val = fe_mul(val, ct.post[(j0 << LOG_R) + o]);
        fe_store_nt(dst + (j0 << LOG_R) + o, val);
      }
    }
  }
}

// dst[c][i] = i < 2^log_m ? src[c][i] : 0 (best_fft's zero padding, fft.rs:327-357).
__global__ void pad_kernel(const fe* __restrict__ src, fe* __restrict__ dst, uint32_t log_m, uint32_t log_n,
                           uint64_t total) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= total) return;
  const uint64_t c = g >> log_n, i = g & (((uint64_t)1 << log_n) - 1);
  fe v = fe_zero();
  if ((i >> log_m) == 0) v = fe_load(src + (c << log_m) + i);
  fe_store(dst + g, v);
}

// n = 2 (best_fft with log_order_of_root = 1): out = (a + b, a - b) [* 1/2].
__global__ void ntt2_kernel(fe* d, fe scale, int do_scale) {
  const size_t off = (size_t)blockIdx.x * 2;
  const fe a = fe_load(d + off), c = fe_load(d + off + 1);
  fe x = fe_add(a, c), y = fe_sub(a, c);
  if (do_scale) {
    x = fe_mul(x, scale);
    y = fe_mul(y, scale);
  }
  fe_store(d + off, x);
  fe_store(d + off + 1, y);
}

namespace {

struct PassPlan {
  int n_pass = 0;
  uint32_t log_r[8] = {0};
};

constexpr uint32_t kMaxLogR = 9;  // largest radix with a kernel instance and small-root table
// Radix cap of a size: 2^8 (three passes of 256 at the headline 2^24).  Radix 2^9 passes (three
// passes instead of four) at 2^25 and from 2^27 on.  At 2^25 (8, 8, 9) beats (6, 6, 6, 7): 3.49-3.51 vs
// 3.55-3.56 ms, and (9, 8, 8) measured within 0.7 % of it (profiles/r04_plan_2_25_26_ab.txt); 2^26 has its
// own plan (plan_passes).
inline uint32_t max_log_r(uint32_t log_n) { return (log_n == 25 || log_n >= 27) ? 9 : 8; }

// The smaller radices lead: a sparse first pass of odd radix can skip 3 copy
// stages, an even one only 2.  (Every plan of a size has the same last radix,
// which the cached full last-pass twiddle table depends on.)
PassPlan plan_passes(uint32_t log_n) {
  PassPlan p;
  if (log_n == 20) {
    // 2^20 (config 2): the two radix-2^8 passes run 16 x 16 (ntt.hip DbPlan::four), the radix-4 pass
    // is short; 0.104-0.105 vs 0.107-0.108 ms for (6, 7, 7), and the 2^17 -> 2^20 LDE 0.768-0.777 vs
    // 0.786-0.790 ms (profiles/r04_plan_2_20_22_ab.txt).  (8, 8, 4) measured the same, (8, 6, 6) slower.
    p.n_pass = 3;
    p.log_r[0] = 8;
    p.log_r[1] = 4;
    p.log_r[2] = 8;
    return p;
  }
  if (log_n == 26) {
    // 2^26: the last pass radix 2^8 (16 x 16, full table) after three digit-basis radix-2^6 passes:
    // 6.76-6.77 / 6.98-7.00 vs 7.22 / 7.52-7.54 ms for (6, 6, 7, 7) on two boxes (profiles/r04_plan_2_25_26_ab.txt;
    // (6, 4, 8, 8) 7.00-7.04, (5, 5, 8, 8) 6.88-6.89, (8, 4, 6, 8) 7.06-7.09, (8, 9, 9) 7.22-7.28)
    p.n_pass = 4;
    p.log_r[0] = 6;
    p.log_r[1] = 6;
    p.log_r[2] = 6;
    p.log_r[3] = 8;
    return p;
  }
  const uint32_t cap = max_log_r(log_n);
  p.n_pass = (int)((log_n + cap - 1) / cap);
  const uint32_t base = log_n / p.n_pass, extra = log_n % p.n_pass;
  for (int i = 0; i < p.n_pass; ++i)
    p.log_r[i] = base + ((uint32_t)(p.n_pass - 1 - i) < extra ? 1 : 0);
  return p;
}

// Columns per workgroup (log2): 1024 elements (256 threads x 4) when the
// transform has that many columns, so every global access is a run of
// B*32 >= 128 contiguous bytes for R <= 256.
uint32_t choose_log_b_impl(uint32_t log_n, uint32_t log_r, uint32_t tile_log) {
  uint32_t lb = log_r >= tile_log ? 0 : tile_log - log_r;
  if (lb > log_n - log_r) lb = log_n - log_r;
  return lb;
}

typedef void (*pass_fn)(const fe*, fe*, uint32_t, uint32_t, uint32_t, ColTw, const fe*, const uint32_t*, fe, int,
                        uint32_t, uint32_t, Sparse);

// Minimum data-image size of a pass instance (in fe): the last-step table is staged over it.
template <int COL>
size_t db_full_fe_c(uint32_t log_r) {
  switch (log_r) {
    case 4: return DbPlan<4, COL>::full_fe;
    case 5: return DbPlan<5, COL>::full_fe;
    case 6: return DbPlan<6, COL>::full_fe;
    case 7: return DbPlan<7, COL>::full_fe;
    case 8: return DbPlan<8, COL>::full_fe;
    default: return 0;
  }
}
size_t db_full_fe(uint32_t log_r, int col) {
  switch (col) {
    case kColNone: return db_full_fe_c<kColNone>(log_r);
    case kColSparse: return db_full_fe_c<kColSparse>(log_r);
    case kColFull: return db_full_fe_c<kColFull>(log_r);
    case kColT16: return db_full_fe_c<kColT16>(log_r);
    default: return db_full_fe_c<kColTwoLevel>(log_r);
  }
}

// LDS of a pass instance beyond its data image: staged Shoup pairs + digit-basis tables (in fe).
template <int COL>
size_t db_lds_fe_c(uint32_t log_r) {
  switch (log_r) {
    case 4: return DbPlan<4, COL>::lds_fe + DbPlan<4, COL>::shoup_fe;
    case 5: return DbPlan<5, COL>::lds_fe + DbPlan<5, COL>::shoup_fe;
    case 6: return DbPlan<6, COL>::lds_fe + DbPlan<6, COL>::shoup_fe;
    case 7: return DbPlan<7, COL>::lds_fe + DbPlan<7, COL>::shoup_fe;
    case 8: return DbPlan<8, COL>::lds_fe + DbPlan<8, COL>::shoup_fe;
    case 9: return DbPlan<9, COL>::lds_fe + DbPlan<9, COL>::shoup_fe;
    default: return (size_t)1 << log_r;
  }
}
size_t db_lds_fe(uint32_t log_r, int col) {
  switch (col) {
    case kColNone: return db_lds_fe_c<kColNone>(log_r);
    case kColSparse: return db_lds_fe_c<kColSparse>(log_r);
    case kColFull: return db_lds_fe_c<kColFull>(log_r);
    case kColT16: return db_lds_fe_c<kColT16>(log_r);
    default: return db_lds_fe_c<kColTwoLevel>(log_r);
  }
}

template <int LOG_R>
pass_fn pass_kernel_r(int col) {
  switch (col) {
    case kColNone: return ntt_pass_kernel<LOG_R, kColNone>;
    case kColSparse: return ntt_pass_kernel<LOG_R, kColSparse>;
    case kColFull: return ntt_pass_kernel<LOG_R, kColFull>;
    case kColT16: return ntt_pass_kernel<LOG_R, kColT16>;
    default: return ntt_pass_kernel<LOG_R, kColTwoLevel>;
  }
}

pass_fn pass_kernel(uint32_t log_r, int col) {
  switch (log_r) {
    case 2: return pass_kernel_r<2>(col);
    case 3: return pass_kernel_r<3>(col);
    case 4: return pass_kernel_r<4>(col);
    case 5: return pass_kernel_r<5>(col);
    case 6: return pass_kernel_r<6>(col);
    case 7: return pass_kernel_r<7>(col);
    case 8: return pass_kernel_r<8>(col);
    case 9: return pass_kernel_r<9>(col);
    default: return nullptr;
  }
}

}  // namespace

stark_status get_twiddles(stark_ctx* ctx, const uint64_t root[4], uint32_t log_n, const Twiddles** out) {
  const FieldHost& F = FieldHost::get();
  if (log_n > 28) return STARK_ERR_BAD_LENGTH;  // 2-adicity of BN254 Fr
  auto key = std::make_tuple(root[0], root[1], root[2], root[3], log_n);
  auto it = ctx->tw.find(key);
  if (it != ctx->tw.end()) {
    *out = it->second.get();
    return STARK_OK;
  }
  const HostFp w = F.from_canonical(root);
  // Primitive 2^log_n-th root: w^(2^(log_n-1)) == -1 (or w == 1 when n == 1).
  HostFp t = w;
  if (log_n == 0) {
    if (!FieldHost::eq(w, F.one())) return STARK_ERR_BAD_ROOT;
  } else {
    for (uint32_t i = 1; i < log_n; ++i) t = F.mul(t, t);
    const HostFp minus_one = F.sub(F.zero(), F.one());
    if (!FieldHost::eq(t, minus_one)) return STARK_ERR_BAD_ROOT;
  }
  auto tw = std::make_unique<Twiddles>();
  tw->log_n = log_n;
  tw->kb = (log_n + 1) / 2;
  tw->root = w;
  tw->inv_n = F.inv(F.from_u64((uint64_t)1 << log_n));
  const size_t n_lo = (size_t)1 << tw->kb, n_hi = (size_t)1 << (log_n - tw->kb);
  std::vector<fe> h_lo(n_lo), h_hi(n_hi);
  HostFp acc = F.one();
  for (size_t i = 0; i < n_lo; ++i) {
    h_lo[i] = to_dev(acc);
    acc = F.mul(acc, w);
  }
  const HostFp step = acc;  // w^(2^kb)
  acc = F.one();
  for (size_t i = 0; i < n_hi; ++i) {
    h_hi[i] = to_dev(acc);
    acc = F.mul(acc, step);
  }
  // Small-root tables for every radix 2^l (l <= min(log_n, 9)): w^(k n / R), k < R/2 (k < R for
  // R = 2^8: the 16 x 16 passes' twiddles, DbPlan::four).
  std::vector<fe> h_small;
  for (uint32_t l = 1; l <= kMaxLogR && l <= log_n; ++l) {
    tw->small_off[l] = (uint32_t)h_small.size();
    const HostFp wr = F.pow_u64(w, (uint64_t)1 << (log_n - l));
    HostFp a = F.one();
    for (uint32_t k = 0; k < ((l == 7 || l == 8) ? (1u << l) : (1u << (l - 1))); ++k) {
      fe pr[2];
      shoup_pair(a, pr);
      h_small.push_back(pr[0]);
      h_small.push_back(pr[1]);
      a = F.mul(a, wr);
    }
  }
  if (h_small.empty()) {
    fe pr[2];
    shoup_pair(F.one(), pr);
    h_small.push_back(pr[0]);
    h_small.push_back(pr[1]);
  }
  // t16[i] = w^(i n / 2^l16): the w_{Ns R} powers of every pass with Ns R <= 2^l16
  // (2^16 entries; 2^18 from 2^25 on, where the middle pass of radix 2^9 has Ns R = 2^17 / 2^18).
  tw->l16 = log_n >= 25 ? 18 : (log_n < 16 ? log_n : 16);
  const size_t n16 = (size_t)1 << tw->l16;
  std::vector<fe> h_t16(2 * n16);
  {
    const HostFp w16 = F.pow_u64(w, (uint64_t)1 << (log_n - tw->l16));
    HostFp a = F.one();
    for (size_t i = 0; i < n16; ++i) {
      shoup_pair(a, &h_t16[2 * i]);
      a = F.mul(a, w16);
    }
  }
  // Copies scaled by n^-1: the inverse's last pass multiplies every element by
  // a column twiddle anyway, so folding n^-1 into it makes the scale free.
  std::vector<fe> h_hi_s(n_hi), h_t16_s(2 * n16);
  {
    HostFp a = F.one();
    const HostFp step_hi = F.pow_u64(w, (uint64_t)1 << tw->kb);
    for (size_t i = 0; i < n_hi; ++i) {
      h_hi_s[i] = to_dev(F.mul(a, tw->inv_n));
      a = F.mul(a, step_hi);
    }
    const HostFp w16 = F.pow_u64(w, (uint64_t)1 << (log_n - tw->l16));
    a = F.one();
    for (size_t i = 0; i < n16; ++i) {
      shoup_pair(F.mul(a, tw->inv_n), &h_t16_s[2 * i]);
      a = F.mul(a, w16);
    }
  }
  tw->n_small_pairs = h_small.size() / 2;
  // Digit-basis tables: w_R^k, k < R/2, for R = 2^l, 1 <= l <= min(log_n, 9) (a pass stages every
  // stride-th one, DbPlan; the distributed NTT's cross-rank DFTs use l <= 3, dist.hip).
  std::vector<uint32_t> h_db;
  for (uint32_t l = 1; l <= kMaxLogR && l <= log_n; ++l) {
    tw->db_off[l] = (uint32_t)h_db.size();
    const HostFp wr = F.pow_u64(w, (uint64_t)1 << (log_n - l));
    HostFp a = F.one();
    for (uint32_t k = 0; k < (1u << (l - 1)); ++k) {
      uint32_t t[72];
      db_table(a, t);
      h_db.insert(h_db.end(), t, t + 72);
      a = F.mul(a, wr);
    }
  }
  if (h_db.empty()) h_db.resize(72, 0);
  const size_t db_fe = h_db.size() / 8;  // 72 u32 = 9 fe per constant
  const size_t bytes = (n_lo + 2 * n_hi + h_small.size() + 4 * n16 + db_fe) * sizeof(fe);
  void* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) return STARK_ERR_OOM;
  tw->d_lo = (fe*)d;
  tw->d_hi = tw->d_lo + n_lo;
  tw->d_small = tw->d_hi + n_hi;
  tw->d_t16 = tw->d_small + h_small.size();
  tw->d_hi_s = tw->d_t16 + 2 * n16;
  tw->d_t16_s = tw->d_hi_s + n_hi;
  tw->d_db = reinterpret_cast<uint32_t*>(tw->d_t16_s + 2 * n16);
  tw->base_bytes = bytes;
  STARK_HIP(ctx, hipMemcpy(tw->d_lo, h_lo.data(), n_lo * sizeof(fe), hipMemcpyHostToDevice));
  STARK_HIP(ctx, hipMemcpy(tw->d_hi, h_hi.data(), n_hi * sizeof(fe), hipMemcpyHostToDevice));
  STARK_HIP(ctx, hipMemcpy(tw->d_small, h_small.data(), h_small.size() * sizeof(fe), hipMemcpyHostToDevice));
  STARK_HIP(ctx, hipMemcpy(tw->d_t16, h_t16.data(), 2 * n16 * sizeof(fe), hipMemcpyHostToDevice));
  STARK_HIP(ctx, hipMemcpy(tw->d_hi_s, h_hi_s.data(), n_hi * sizeof(fe), hipMemcpyHostToDevice));
  STARK_HIP(ctx, hipMemcpy(tw->d_t16_s, h_t16_s.data(), 2 * n16 * sizeof(fe), hipMemcpyHostToDevice));
  STARK_HIP(ctx, hipMemcpy(tw->d_db, h_db.data(), h_db.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
  *out = tw.get();
  ctx->tw.emplace(key, std::move(tw));
  return STARK_OK;
}

// full[g] = w^(c r) (Montgomery), g = c R + r; times `scale` when given.
__global__ void full_tw_kernel(const fe* __restrict__ lo, const fe* __restrict__ hi, uint32_t kb, uint32_t log_r,
                               uint64_t n, fe scale, int do_scale, fe* __restrict__ out) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const uint64_t e = (g >> log_r) * (g & (((uint64_t)1 << log_r) - 1));  // c r < n
  fe t = fe_mul(lo[e & (((uint64_t)1 << kb) - 1)], hi[e >> kb]);
  if (do_scale) t = fe_mul(t, scale);
  fe_store(out + g, t);
}

// The last pass's full twiddle table, built once per (root, n, direction) and kept in the context's
// size-capped cache (cache_reserve: least recently used tables go first).  When it cannot be cached
// (larger than the cap, or no device memory) *out is null and the pass takes the two-level form.
static stark_status full_table(stark_ctx* ctx, const Twiddles& tw_c, uint32_t log_r, bool scaled, hipStream_t stream,
                               const fe** out) {
  Twiddles& tw = const_cast<Twiddles&>(tw_c);  // lazily filled cache entry
  fe*& slot = scaled ? tw.d_full_s : tw.d_full;
  const int d = scaled ? 1 : 0;
  (scaled ? tw.full_s_used : tw.full_used) = ++ctx->cache_clock;
  if (!slot) {
    const uint64_t n = (uint64_t)1 << tw.log_n;
    void* p = nullptr;
    if (!cache_reserve(ctx, n * sizeof(fe), false) || hipMalloc(&p, n * sizeof(fe)) != hipSuccess) {
      hipGetLastError();  // (a failed allocation is not an error here)
      *out = nullptr;     // no room: fall back to the two-level form
      return STARK_OK;
    }
    hipLaunchKernelGGL(full_tw_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, tw.d_lo, tw.d_hi,
                       tw.kb, log_r, n, to_dev(tw.inv_n), scaled ? 1 : 0, (fe*)p);
    STARK_HIP(ctx, hipGetLastError());
    // Published now, complete only when the fill has run on `stream`: a call on another stream
    // waits for this event (fill_wait below) instead of reading a table still being written.
    STARK_TRY(fill_mark(ctx, tw.full_ev[d], tw.full_fill[d], stream));
    slot = (fe*)p;
  } else {
    STARK_TRY(fill_wait(ctx, tw.full_ev[d], tw.full_fill[d], stream));
  }
  *out = slot;
  return STARK_OK;
}

}  // namespace stark

extern "C" uint32_t stark_ntt_plan(uint32_t log_n, uint32_t* log_r, uint32_t cap) {
  if (log_n < 2 || log_n > 28) return 0;
  const stark::PassPlan p = stark::plan_passes(log_n);
  for (int i = 0; i < p.n_pass && (uint32_t)i < cap; ++i) log_r[i] = p.log_r[i];
  return (uint32_t)p.n_pass;
}

namespace stark {

uint32_t ntt_first_log_r(uint32_t log_n) { return log_n < 2 ? log_n : plan_passes(log_n).log_r[0]; }

stark_status ntt_device(stark_ctx* ctx, fe* d_data, uint32_t log_n, uint32_t batch, const Twiddles& tw,
                        bool inverse, hipStream_t stream, const fe* post) {
  return ntt_device_from(ctx, nullptr, 0, d_data, log_n, batch, tw, inverse, stream, post);
}

// src != nullptr: the input is src (batch columns of 2^(log_n - zero_log)
// elements, the rest of each column implicitly zero) and the output goes to
// d_data; the zero tail is never written or read (forward LDE of best_fft's
// padded coefficients).
stark_status ntt_device_from(stark_ctx* ctx, const fe* src, uint32_t zero_log, fe* d_data, uint32_t log_n,
                             uint32_t batch, const Twiddles& tw, bool inverse, hipStream_t stream, const fe* post) {
  if (batch == 0) return STARK_OK;
  if (src && zero_log > log_n) return STARK_ERR_BAD_ARG;
  if (src && (zero_log == 0 || log_n < 2 || zero_log > plan_passes(log_n).log_r[0])) {
    // Not expressible as a sparse first pass: materialise the padded columns.
    const uint64_t total = (uint64_t)batch << log_n;
    hipLaunchKernelGGL(pad_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, src, d_data,
                       log_n - zero_log, log_n, total);
    STARK_HIP(ctx, hipGetLastError());
    src = nullptr;
  }
  if (((uint64_t)batch << log_n) > ((uint64_t)1 << 34)) return STARK_ERR_BAD_ARG;
  const size_t n = (size_t)1 << log_n;
  const fe scale = to_dev(tw.inv_n);
  if (log_n == 0) return STARK_OK;  // 1-point DFT is the identity (n^-1 = 1)
  if (log_n == 1) {
    if (post) return STARK_ERR_BAD_ARG;  // (the distributed callers have M >= 4)
    hipLaunchKernelGGL(ntt2_kernel, dim3(batch), dim3(1), 0, stream, d_data, scale, inverse ? 1 : 0);
    STARK_HIP(ctx, hipGetLastError());
    return STARK_OK;
  }
  const PassPlan plan = plan_passes(log_n);
  // The ping-pong buffer is the context's, shared by every stream that calls in: this stream waits
  // for the last use on another one (buf_acquire) and marks its own after the passes (buf_release).
  // (A single-pass transform never touches it.)
  fe* scratch = nullptr;
  stark_status st = STARK_OK;
  if (plan.n_pass > 1) {
    st = ensure_buf(ctx, ctx->scratch, n * batch * sizeof(fe));
    if (st != STARK_OK) return st;
    STARK_TRY(buf_acquire(ctx, ctx->scratch, stream));
    scratch = (fe*)ctx->scratch.ptr;
  }
  const fe* cur = src ? src : d_data;
  uint32_t log_ns = 0;
  for (int p = 0; p < plan.n_pass; ++p) {
    const uint32_t lr = plan.log_r[p];
    const bool last = p == plan.n_pass - 1;
    // Passes before the last ping-pong; the last pass (Ns R = n) reads and
    // writes the same positions, so it always lands in d_data.
    fe* dst = last ? d_data : (cur == d_data ? scratch : d_data);
    Sparse sp{0, 0, log_n};
    if (p == 0 && src) {
      // Copy stages the pass's stage pairing can skip: odd radices run a
      // radix-2 stage 0 then pairs (1,2), (3,4)..; even ones pairs (0,1)..
      uint32_t k = zero_log < lr ? zero_log : lr;
      if ((k & 1) != (lr & 1)) --k;
      sp = Sparse{k, zero_log, log_n - zero_log};
    }
    const uint32_t lb = choose_log_b_impl(log_n, lr, kTileLog);
    const uint32_t elems = 1u << (lr + lb);
    const uint32_t threads = elems / 4 < 64 ? 64 : elems / 4;
    const uint32_t log_tiles = log_n - lr - lb;
    const uint64_t total = (uint64_t)batch << log_tiles;
    // Inverse: n^-1 rides on the last pass's column twiddles (scaled tables)
    // when that pass has them (log_ns > 0), else it is an explicit product.
    const bool fold = inverse && last && log_ns > 0;
    const fe* full = nullptr;
    if (last && log_ns > 0 && log_n > tw.l16 && log_n >= 17 && log_n <= 26) {
      st = full_table(ctx, tw, lr, fold, stream, &full);
      if (st != STARK_OK) return st;
    }
    ColTw ct{fold ? tw.d_t16_s : tw.d_t16, tw.d_lo, fold ? tw.d_hi_s : tw.d_hi, full, tw.l16, tw.kb,
             last ? post : nullptr};
    const int col = log_ns == 0 ? (sp.skip ? kColSparse : kColNone)
                    : full ? kColFull : log_ns + lr <= tw.l16 ? kColT16 : kColTwoLevel;
    // data image + staged Shoup pairs + digit-basis tables (DbPlan of this instance)
    const size_t image = std::max((size_t)elems, db_full_fe(lr, col));
    const size_t lds = (image + db_lds_fe(lr, col)) * sizeof(fe);
    hipLaunchKernelGGL(pass_kernel(lr, col), dim3((unsigned)total), dim3(threads), lds, stream, cur, dst, log_n,
                       log_ns, lb, ct, tw.d_small + tw.small_off[lr], tw.d_db + tw.db_off[lr], scale,
                       (inverse && last && !fold) ? 1 : 0, log_tiles, (uint32_t)total, sp);
    STARK_HIP(ctx, hipGetLastError());
    cur = dst;
    log_ns += lr;
  }
  if (scratch) buf_release(ctx, ctx->scratch, stream);
  return STARK_OK;
}

// Pass 0 launched as if it were the transform's last pass (Ns = A = n / T): the store's
// out[(j / Ns) Ns R + (j mod Ns) + r Ns] is then out[j + r A] (every column j < A), reduced to canonical,
// and the pass has no column twiddle whatever its Ns (kColNone / kColSparse read none).
stark_status ntt_first_pass_tmajor(stark_ctx* ctx, const fe* src, uint32_t zero_log, fe* out, uint32_t log_n,
                                   uint32_t batch, const Twiddles& tw, hipStream_t stream, uint32_t* log_t) {
  if (!src || log_n < 2 || zero_log == 0 || batch == 0 || tw.log_n != log_n) return STARK_ERR_BAD_ARG;
  if (((uint64_t)batch << log_n) > ((uint64_t)1 << 34)) return STARK_ERR_BAD_ARG;
  const uint32_t lr = plan_passes(log_n).log_r[0];
  if (zero_log > lr) return STARK_ERR_BAD_ARG;  // (the LDEs here: zero_log 3 <= every plan's first radix)
  uint32_t k = zero_log;
  if ((k & 1) != (lr & 1)) --k;
  const Sparse sp{k, zero_log, log_n - zero_log};
  const uint32_t lb = choose_log_b_impl(log_n, lr, kTileLog);
  const uint32_t elems = 1u << (lr + lb);
  const uint32_t threads = elems / 4 < 64 ? 64 : elems / 4;
  const uint32_t log_tiles = log_n - lr - lb;
  const uint64_t total = (uint64_t)batch << log_tiles;
  const int col = sp.skip ? kColSparse : kColNone;
  const ColTw ct{tw.d_t16, tw.d_lo, tw.d_hi, nullptr, tw.l16, tw.kb, nullptr};
  const size_t image = std::max((size_t)elems, db_full_fe(lr, col));
  const size_t lds = (image + db_lds_fe(lr, col)) * sizeof(fe);
  hipLaunchKernelGGL(pass_kernel(lr, col), dim3((unsigned)total), dim3(threads), lds, stream, src, out, log_n,
                     log_n - lr, lb, ct, tw.d_small + tw.small_off[lr], tw.d_db + tw.db_off[lr], to_dev(tw.inv_n), 0,
                     log_tiles, (uint32_t)total, sp);
  STARK_HIP(ctx, hipGetLastError());
  *log_t = lr;
  return STARK_OK;
}

}  // namespace stark
