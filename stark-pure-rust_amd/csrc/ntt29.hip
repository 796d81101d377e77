// NTT pass kernels in radix 2^29 (fp29_dev.h): the same Stockham decomposition, thread mapping and
// results as ntt.hip's pass kernel (best_fft / inv_best_fft, packages/fri/src/fft.rs:150-379), with
// the working representation changed so that the arithmetic is cheaper on gfx950:
//   * products by twiddles are carry-free Shoup products (143 v_mad_u64_u32, no carry counting);
//   * butterflies are 9 + 18 full-rate v_add_u32 / v_sub_u32 (x + t, x - t + 4p), no carry chains and
//     no conditional subtractions;
//   * limbs grow by < 2^30 per level; the radix-4 step normalises the two of its four inputs that are
//     not multiplied first (x0, x2), which keeps every product input below 2^31.6 per limb.
// Between passes elements live in HBM as three planes (limbs 0-3, 4-7, 8: 36 B per element); the first
// pass reads the caller's canonical 32-B elements and the last pass writes canonical 32-B elements.
// Twiddles are fe29p Shoup pairs (80 B) read from global memory (L1/L2-resident small tables, or the
// last pass's streamed full table), so the LDS holds only the 36-B-per-element data image (36 KB at
// R = 256, B = 4: four workgroups per CU).
#include <stdlib.h>

#include "fp29_dev.h"
#include "internal.h"

namespace stark {

// From Shoup pairs (w, q32) at src[2i], src[2i + 1].
__global__ void pair29_from_shoup_kernel(const fe* __restrict__ src, fe29p* __restrict__ dst, uint64_t n) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const fe w = src[2 * g], q = src[2 * g + 1];
  uint32_t m[8];
  uint32_t pl[8];
  for (int i = 0; i < 8; ++i) pl[i] = p_limb(i);
  mul_lo256(q.w, pl, m);  // w 2^256 - q p = m  ->  m = -(q p) mod 2^256
  neg256(m);
  dst[g] = pair29(w, q.w, m);
}

__global__ void pair29_from_mont_kernel(const fe* __restrict__ src, fe29p* __restrict__ dst, uint64_t n, fe scale,
                                        int do_scale) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  fe m = src[g];
  if (do_scale) {  // Montgomery(m * s) = m s 2^-256 with both Montgomery images: the image of w * scale
    m = fe_mul(m, scale);
  }
  dst[g] = pair29_from_mont(m);
}
// full[g] = w^(c r) (and * n^-1), g = c R + r, straight to fe29p pairs.
__global__ void full29_kernel(const fe* __restrict__ lo, const fe* __restrict__ hi, uint32_t kb, uint32_t log_r,
                              uint64_t n, fe scale, int do_scale, fe29p* __restrict__ out) {
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  const uint64_t e = (g >> log_r) * (g & (((uint64_t)1 << log_r) - 1));
  fe t = fe_mul(lo[e & (((uint64_t)1 << kb) - 1)], hi[e >> kb]);
  if (do_scale) t = fe_mul(t, scale);
  out[g] = pair29_from_mont(t);
}

struct ColTw29 {
  const fe29p* t16;   // w^(i n / 2^l16), i < 2^l16
  const fe29p* lo;    // w^i, i < 2^kb
  const fe29p* hi;    // w^(i 2^kb)
  const fe29p* full;  // last pass: full[c R + r] = w^(c r)
  uint32_t l16, kb;
};

// 8p with every limb but the top one borrowed up to >= 2^29 - 1 (the s = 0 step's unmultiplied
// second operand is a sum of two inputs: normalised, value < 8p).
__device__ __forceinline__ uint32_t k8p29(int i) {
  switch (i) {
    case 0: return 0x20000008u; case 1: return 0x387d64fbu; case 2: return 0x32e12286u; case 3: return 0x3e84879au;
    case 4: return 0x2c2e9418u; case 5: return 0x36da0604u; case 6: return 0x25370a07u; case 7: return 0x32e1319fu;
    default: return 0x01832272u;
  }
}
__device__ __forceinline__ fe29 fe29_subk8(const fe29& x, const fe29& t) {
  fe29 y;
#pragma unroll
  for (int i = 0; i < 9; ++i) y.l[i] = x.l[i] + k8p29(i) - t.l[i];
  return y;
}

// Workgroups per CU the pass kernel is compiled for (4: 128 VGPRs; 3: 168).
#ifndef STARK_NTT29_WG_PER_CU
#define STARK_NTT29_WG_PER_CU 4
#endif

enum : int { kCol29None = 0, kCol29Full = 1, kCol29T16 = 2, kCol29TwoLevel = 3 };

// One Stockham pass (ntt.hip's thread mapping: B adjacent columns per workgroup, 4 elements per
// thread).  IN29: the input is plane-format fe29 (else canonical fe); OUT29: plane-format output
// (else canonical fe: the transform's last pass).  ps_in / ps_out: plane strides in elements.
template <int LOG_R, int COL, bool IN29, bool OUT29>
__global__ __launch_bounds__(256, STARK_NTT29_WG_PER_CU) void ntt29_pass_kernel(const void* __restrict__ in, void* __restrict__ out,
                                                            uint64_t ps_in, uint64_t ps_out, uint32_t log_n,
                                                            uint32_t log_ns, uint32_t log_b, ColTw29 ct,
                                                            const fe29p* __restrict__ small,
                                                            const fe29p* __restrict__ scale, uint32_t log_tiles,
                                                            uint32_t total_tiles, Sparse sp) {
  constexpr uint32_t R = 1u << LOG_R;
  extern __shared__ __attribute__((aligned(16))) uint32_t lds29[];
  const uint32_t B = 1u << log_b;
  const uint32_t ps_l = R << log_b;  // LDS plane stride
  const uint32_t nthr = (B << LOG_R) >> 2;
  const uint32_t tid = threadIdx.x;
  const bool active = tid < nthr;
  const uint32_t log_cols = log_n - LOG_R;
  const size_t ns_mask = ((size_t)1 << log_ns) - 1;
  const uint32_t tile_mask = (1u << log_tiles) - 1;
  const uint32_t tile = blockIdx.x;
  if (tile >= total_tiles) return;

  uint32_t eb[4], er[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const uint32_t e = tid + (uint32_t)t * nthr;
    eb[t] = e & (B - 1);
    er[t] = e >> log_b;
  }
  const uint32_t b = tid & (B - 1);
  const uint32_t q = tid >> log_b;

  const uint32_t live_rows = R >> sp.skip, nz_rows = R >> sp.zero_log;
  const uint32_t log_in = sp.zero_log ? sp.log_in : log_n;
  const size_t j0 = (size_t)(tile & tile_mask) << log_b;

  // ---- load, column twiddle, scatter into the bit-reversed LDS image ----
  if (active) {
    fe29 v[4];
    const size_t ibase = ((size_t)(tile >> log_tiles) << log_in) + j0;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const size_t idx = ibase + eb[t] + ((size_t)er[t] << log_cols);
      if (IN29) {
        v[t] = fe29_load_planes(static_cast<const uint32_t*>(in), idx, ps_in);
      } else if (er[t] < nz_rows) {
        v[t] = fe29_from32(fe_load(static_cast<const fe*>(in) + idx));
      } else {
#pragma unroll
        for (int i = 0; i < 9; ++i) v[t].l[i] = 0;
      }
    }
    if (COL == kCol29TwoLevel) {
      const uint32_t lnr = log_ns + LOG_R;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const size_t jc = (j0 + eb[t]) & ns_mask;
        const uint64_t ex = ((uint64_t)jc * er[t]) << (log_n - lnr);
        v[t] = fe29_mul_pair(v[t], ct.lo + (ex & (((uint64_t)1 << ct.kb) - 1)));
        v[t] = fe29_mul_pair(v[t], ct.hi + (ex >> ct.kb));
      }
    } else if (COL != kCol29None) {
      // One pair per element from the t16 table or the last pass's full table; the next element's
      // pair is loaded while this one's product runs (two pair buffers).
      const uint32_t lnr = log_ns + LOG_R;
      const fe29p* tp[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const size_t jc = (j0 + eb[t]) & ns_mask;
        if (COL == kCol29Full) {
          tp[t] = ct.full + ((jc << LOG_R) + er[t]);
        } else {
          const uint64_t k = ((uint64_t)jc * er[t]) & (((uint64_t)1 << lnr) - 1);
          tp[t] = ct.t16 + (k << (ct.l16 - lnr));
        }
      }
      fe29 w[2], wq[2];
      fe29p_load(tp[0], w[0], wq[0]);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (t + 1 < 4) fe29p_load(tp[t + 1], w[(t + 1) & 1], wq[(t + 1) & 1]);
        v[t] = fe29_mul_shoup(v[t], w[t & 1], wq[t & 1]);
      }
    }
    if (sp.skip == 0) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const uint32_t rr = __builtin_bitreverse32(er[t]) >> (32 - LOG_R);
        fe29_store_planes(lds29, (rr << log_b) + eb[t], ps_l, v[t]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if (er[t] >= live_rows) continue;
        const uint32_t rr = __builtin_bitreverse32(er[t]) >> (32 - LOG_R);
        for (uint32_t k = 0; k < (1u << sp.skip); ++k) fe29_store_planes(lds29, ((rr + k) << log_b) + eb[t], ps_l, v[t]);
      }
    }
  }
  __syncthreads();

  // ---- R-point DIT over the bit-reversed image ----
  int s = (int)sp.skip;
  if ((LOG_R & 1) && sp.skip == 0) {
    if (active) {  // radix-2 stage 0: twiddles 1; inputs normalised with value < 4p
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint32_t g = q * 2 + h;
        const uint32_t ia = ((2 * g) << log_b) + b, ib = ((2 * g + 1) << log_b) + b;
        fe29 a = fe29_load_planes(lds29, ia, ps_l), c = fe29_load_planes(lds29, ib, ps_l);
        const fe29 y = fe29_subk(a, c);
        fe29_add(a, c);
        fe29_store_planes(lds29, ia, ps_l, a);
        fe29_store_planes(lds29, ib, ps_l, y);
      }
    }
    __syncthreads();
    s = 1;
  }
  if (s == 0) {
    // Radix-4 step s = 0: twiddles 1 except w_4^1 (small[R/4]).
    if (active) {
      const uint32_t base = q << 2;
      fe29 x0 = fe29_load_planes(lds29, (base << log_b) + b, ps_l);
      fe29 x1 = fe29_load_planes(lds29, ((base + 1) << log_b) + b, ps_l);
      fe29 x2 = fe29_load_planes(lds29, ((base + 2) << log_b) + b, ps_l);
      fe29 x3 = fe29_load_planes(lds29, ((base + 3) << log_b) + b, ps_l);
      fe29_bfly(x0, x1, x1);
      fe29_bfly(x2, x3, x3);
      const fe29 t3 = fe29_mul_pair(x3, small + (R >> 2));
      fe29_normalize(x2);  // the unmultiplied operand: x2 + x3 < 8p
      const fe29 y2 = fe29_subk8(x0, x2);
      fe29_add(x0, x2);
      fe29_bfly(x1, x3, t3);
      fe29_store_planes(lds29, (base << log_b) + b, ps_l, x0);
      fe29_store_planes(lds29, ((base + 2) << log_b) + b, ps_l, y2);
      fe29_store_planes(lds29, ((base + 1) << log_b) + b, ps_l, x1);
      fe29_store_planes(lds29, ((base + 3) << log_b) + b, ps_l, x3);
    }
    __syncthreads();
    s = 2;
  }
#pragma unroll 1
  for (; s < LOG_R; s += 2) {
    if (active) {
      const uint32_t m = 1u << s;
      const uint32_t jj = q & (m - 1);
      const uint32_t base = ((q >> s) << (s + 2)) + jj;
      // The step's three twiddle pairs (global, L1-resident) are requested before the LDS reads.
      fe29 taw, taq, tbw, tbq;
      fe29p_load(small + (jj << (LOG_R - 1 - s)), taw, taq);  // w_{2m}^jj
      fe29p_load(small + (jj << (LOG_R - 2 - s)), tbw, tbq);  // w_{4m}^jj
      fe29 x0 = fe29_load_planes(lds29, (base << log_b) + b, ps_l);
      fe29 x1 = fe29_load_planes(lds29, ((base + m) << log_b) + b, ps_l);
      fe29 x2 = fe29_load_planes(lds29, ((base + 2 * m) << log_b) + b, ps_l);
      fe29 x3 = fe29_load_planes(lds29, ((base + 3 * m) << log_b) + b, ps_l);
      fe29_normalize(x0);
      fe29_normalize(x2);
      const fe29 t1 = fe29_mul_shoup(x1, taw, taq);
      fe29 t3 = fe29_mul_shoup(x3, taw, taq);
      fe29 tcw, tcq;
      fe29p_load(small + ((jj + m) << (LOG_R - 2 - s)), tcw, tcq);  // w_{4m}^(jj+m)
      fe29_bfly(x0, x1, t1);
      fe29_bfly(x2, x3, t3);
      const fe29 t2 = fe29_mul_shoup(x2, tbw, tbq);
      t3 = fe29_mul_shoup(x3, tcw, tcq);
      fe29_bfly(x0, x2, t2);
      fe29_bfly(x1, x3, t3);
      fe29_store_planes(lds29, (base << log_b) + b, ps_l, x0);
      fe29_store_planes(lds29, ((base + 2 * m) << log_b) + b, ps_l, x2);
      fe29_store_planes(lds29, ((base + m) << log_b) + b, ps_l, x1);
      fe29_store_planes(lds29, ((base + 3 * m) << log_b) + b, ps_l, x3);
    }
    __syncthreads();
  }

  // ---- store: out[(j / Ns) Ns R + (j mod Ns) + r Ns] ----
  if (active) {
    const size_t boff = (size_t)(tile >> log_tiles) << log_n;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      size_t o;
      uint32_t li;
      if (((size_t)1 << log_ns) >= B) {
        const size_t j = j0 + eb[t];
        o = ((j >> log_ns) << (log_ns + LOG_R)) + (j & ns_mask) + ((size_t)er[t] << log_ns);
        li = (er[t] << log_b) + eb[t];
      } else {
        // Ns < B: the tile's output is the contiguous run [j0 R, (j0 + B) R).
        const uint32_t oo = tid + (uint32_t)t * nthr;
        const uint32_t qq = oo >> (log_ns + LOG_R);
        const uint32_t rem = oo & ((1u << (log_ns + LOG_R)) - 1);
        const uint32_t r = rem >> log_ns;
        const uint32_t bb = (qq << log_ns) + (rem & (uint32_t)ns_mask);
        o = (j0 << LOG_R) + oo;
        li = (r << log_b) + bb;
      }
      fe29 val = fe29_load_planes(lds29, li, ps_l);
      if (OUT29) {
        fe29_store_planes(static_cast<uint32_t*>(out), boff + o, ps_out, val);
      } else {
        if (scale) val = fe29_mul_pair(val, scale);
        fe_store(static_cast<fe*>(out) + boff + o, fe29_canonical(val));
      }
    }
  }
}

namespace {

typedef void (*pass29_fn)(const void*, void*, uint64_t, uint64_t, uint32_t, uint32_t, uint32_t, ColTw29,
                          const fe29p*, const fe29p*, uint32_t, uint32_t, Sparse);

template <int LOG_R, int COL>
pass29_fn pick_io(bool in29, bool out29) {
  if (in29) return out29 ? ntt29_pass_kernel<LOG_R, COL, true, true> : ntt29_pass_kernel<LOG_R, COL, true, false>;
  return out29 ? ntt29_pass_kernel<LOG_R, COL, false, true> : ntt29_pass_kernel<LOG_R, COL, false, false>;
}
template <int LOG_R>
pass29_fn pick_col(int col, bool in29, bool out29) {
  // The first pass (no column twiddle) reads canonical input; every later pass reads fe29 planes.
  if (col == kCol29None) return in29 ? nullptr : pick_io<LOG_R, kCol29None>(false, out29);
  if (!in29) return nullptr;
  switch (col) {
    case kCol29Full: return pick_io<LOG_R, kCol29Full>(true, out29);
    case kCol29T16: return pick_io<LOG_R, kCol29T16>(true, out29);
    default: return pick_io<LOG_R, kCol29TwoLevel>(true, out29);
  }
}
pass29_fn pass29_kernel(uint32_t log_r, int col, bool in29, bool out29) {
  switch (log_r) {
    case 2: return pick_col<2>(col, in29, out29);
    case 3: return pick_col<3>(col, in29, out29);
    case 4: return pick_col<4>(col, in29, out29);
    case 5: return pick_col<5>(col, in29, out29);
    case 6: return pick_col<6>(col, in29, out29);
    case 7: return pick_col<7>(col, in29, out29);
    case 8: return pick_col<8>(col, in29, out29);
    case 9: return pick_col<9>(col, in29, out29);
    default: return nullptr;
  }
}

stark_status alloc29(stark_ctx* ctx, size_t count, fe29p** out) {
  void* d = nullptr;
  STARK_HIP(ctx, hipMalloc(&d, count * sizeof(fe29p)));
  *out = (fe29p*)d;
  return STARK_OK;
}

stark_status conv_shoup(stark_ctx* ctx, const fe* src, size_t n, hipStream_t s, fe29p** out) {
  stark_status st = alloc29(ctx, n, out);
  if (st != STARK_OK) return st;
  hipLaunchKernelGGL(pair29_from_shoup_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, *out,
                     (uint64_t)n);
  STARK_HIP(ctx, hipGetLastError());
  return STARK_OK;
}
stark_status conv_mont(stark_ctx* ctx, const fe* src, size_t n, const fe* scale, hipStream_t s, fe29p** out) {
  stark_status st = alloc29(ctx, n, out);
  if (st != STARK_OK) return st;
  hipLaunchKernelGGL(pair29_from_mont_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, *out,
                     (uint64_t)n, scale ? *scale : fe{}, scale ? 1 : 0);
  STARK_HIP(ctx, hipGetLastError());
  return STARK_OK;
}

}  // namespace

// The radix-2^29 twiddle tables of a Twiddles entry, converted on the device from its 32-bit tables
// on first use (same values, Shoup pairs with wq = floor(w 2^261 / p)).
struct Tw29 {
  fe29p *small = nullptr, *t16 = nullptr, *t16s = nullptr, *lo = nullptr, *hi = nullptr, *his = nullptr;
  fe29p *full = nullptr, *fulls = nullptr, *invn = nullptr;
  size_t n_small = 0;
  ~Tw29() {
    for (fe29p* p : {small, t16, t16s, lo, hi, his, full, fulls, invn})
      if (p) hipFree(p);
  }
};

void tw29_free(Tw29* t) { delete t; }

static stark_status tw29_get(stark_ctx* ctx, const Twiddles& tw_c, hipStream_t s, Tw29** out) {
  Twiddles& tw = const_cast<Twiddles&>(tw_c);
  if (tw.t29) {
    *out = tw.t29;
    return STARK_OK;
  }
  std::unique_ptr<Tw29> t(new Tw29());
  const uint32_t log_n = tw.log_n;
  const size_t n_lo = (size_t)1 << tw.kb, n_hi = (size_t)1 << (log_n - tw.kb), n16 = (size_t)1 << tw.l16;
  t->n_small = tw.n_small_pairs;
  stark_status st = conv_shoup(ctx, tw.d_small, tw.n_small_pairs, s, &t->small);
  if (st == STARK_OK) st = conv_shoup(ctx, tw.d_t16, n16, s, &t->t16);
  if (st == STARK_OK) st = conv_shoup(ctx, tw.d_t16_s, n16, s, &t->t16s);
  if (st == STARK_OK) st = conv_mont(ctx, tw.d_lo, n_lo, nullptr, s, &t->lo);
  if (st == STARK_OK) st = conv_mont(ctx, tw.d_hi, n_hi, nullptr, s, &t->hi);
  if (st == STARK_OK) st = conv_mont(ctx, tw.d_hi_s, n_hi, nullptr, s, &t->his);
  if (st == STARK_OK) {
    // n^-1 as a pair: the Montgomery image of n^-1 is the first entry of hi_s (hi[0] = 1).
    st = conv_mont(ctx, tw.d_hi_s, 1, nullptr, s, &t->invn);
  }
  if (st != STARK_OK) return st;
  tw.t29 = t.release();
  *out = tw.t29;
  return STARK_OK;
}

static stark_status full29_table(stark_ctx* ctx, const Twiddles& tw, Tw29& t, uint32_t log_r, bool scaled,
                                 hipStream_t s, const fe29p** out) {
  fe29p*& slot = scaled ? t.fulls : t.full;
  if (!slot) {
    const uint64_t n = (uint64_t)1 << tw.log_n;
    void* d = nullptr;
    if (hipMalloc(&d, n * sizeof(fe29p)) != hipSuccess) {
      (void)hipGetLastError();
      *out = nullptr;  // no room: the two-level form
      return STARK_OK;
    }
    hipLaunchKernelGGL(full29_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, tw.d_lo, tw.d_hi, tw.kb,
                       log_r, n, to_dev(tw.inv_n), scaled ? 1 : 0, (fe29p*)d);
    STARK_HIP(ctx, hipGetLastError());
    slot = (fe29p*)d;
  }
  *out = slot;
  return STARK_OK;
}

// Opt-in (STARK_NTT29=1): on gfx950 the radix-2^32 kernels are as fast (this
// form issues 21-24 % fewer VALU instructions per pass, but its denser v_mad_u64_u32 stream runs at a
// ~13 % lower clock under the power limit).
bool ntt29_enabled() {
  static const bool on = [] {
    const char* e = getenv("STARK_NTT29");
    return e && e[0] == '1';
  }();
  return on;
}

// ntt_device_from (ntt.hip) in radix 2^29: same arguments, same results.
stark_status ntt29_device_from(stark_ctx* ctx, const fe* src, uint32_t zero_log, fe* d_data, uint32_t log_n,
                               uint32_t batch, const Twiddles& tw, bool inverse, hipStream_t stream,
                               const uint32_t* plan_log_r, int n_pass) {
  Tw29* t = nullptr;
  stark_status st = tw29_get(ctx, tw, stream, &t);
  if (st != STARK_OK) return st;
  const size_t n_all = (size_t)batch << log_n;
  // Two plane-format buffers (36 B per element each): the passes ping-pong between them, the first
  // reads the caller's data and the last writes it (never in place: a plane image and the canonical
  // image of one element sit at different offsets).
  if (n_pass > 1) {
    st = ensure_buf(ctx, ctx->scratch, n_all * 36);
    if (st == STARK_OK) st = ensure_buf(ctx, ctx->scratch2, n_all * 36);
    if (st != STARK_OK) return st;
  }
  uint32_t* bufs[2] = {(uint32_t*)ctx->scratch.ptr, (uint32_t*)ctx->scratch2.ptr};
  const void* cur = src ? (const void*)src : (const void*)d_data;
  uint32_t log_ns = 0;
  for (int p = 0; p < n_pass; ++p) {
    const uint32_t lr = plan_log_r[p];
    const bool last = p == n_pass - 1;
    void* dst = last ? (void*)d_data : (void*)bufs[p & 1];
    Sparse sp{0, 0, log_n};
    if (p == 0 && src) {
      uint32_t k = zero_log < lr ? zero_log : lr;
      if ((k & 1) != (lr & 1)) --k;
      sp = Sparse{k, zero_log, log_n - zero_log};
    }
    const uint32_t lb = ntt_choose_log_b(log_n, lr);
    const uint32_t elems = 1u << (lr + lb);
    const uint32_t threads = elems / 4 < 64 ? 64 : elems / 4;
    const size_t lds = (size_t)elems * 36;
    const uint32_t log_tiles = log_n - lr - lb;
    const uint64_t total = (uint64_t)batch << log_tiles;
    const bool fold = inverse && last && log_ns > 0;
    const fe29p* full = nullptr;
    if (last && log_ns > 0 && log_n > tw.l16 && log_n >= 17 && log_n <= 26 && ntt_full_table_enabled()) {
      st = full29_table(ctx, tw, *t, lr, fold, stream, &full);
      if (st != STARK_OK) return st;
    }
    ColTw29 ct{fold ? t->t16s : t->t16, t->lo, fold ? t->his : t->hi, full, tw.l16, tw.kb};
    const int col = log_ns == 0 ? kCol29None : full ? kCol29Full : log_ns + lr <= tw.l16 ? kCol29T16 : kCol29TwoLevel;
    const pass29_fn fn = pass29_kernel(lr, col, p > 0, !last);
    if (!fn) return STARK_ERR_BAD_ARG;
    const fe29p* scale = (inverse && last && !fold) ? t->invn : nullptr;
    hipLaunchKernelGGL(fn, dim3((unsigned)total), dim3(threads), lds, stream, cur, dst, (uint64_t)n_all,
                       (uint64_t)n_all, log_n, log_ns, lb, ct, t->small + tw.small_off[lr] / 2, scale, log_tiles,
                       (uint32_t)total, sp);
    STARK_HIP(ctx, hipGetLastError());
    cur = dst;
    log_ns += lr;
  }
  return STARK_OK;
}

}  // namespace stark
