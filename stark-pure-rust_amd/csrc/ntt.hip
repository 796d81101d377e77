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
#include "internal.h"

namespace stark {

template <int LOG_R>
__global__ __launch_bounds__(256) void ntt_pass_kernel(const fe* __restrict__ in, fe* __restrict__ out,
                                                       uint32_t log_n, uint32_t log_ns, uint32_t log_b,
                                                       const fe* __restrict__ tw_lo, const fe* __restrict__ tw_hi,
                                                       uint32_t kb, const fe* __restrict__ small, fe scale,
                                                       int do_scale) {
  constexpr uint32_t R = 1u << LOG_R;
  extern __shared__ __attribute__((aligned(16))) fe lds[];
  const uint32_t B = 1u << log_b;
  const uint32_t E = B << LOG_R;
  const uint32_t T = blockDim.x;
  const size_t boff = (size_t)blockIdx.y << log_n;
  in += boff;
  out += boff;
  const size_t j0 = (size_t)blockIdx.x << log_b;
  const uint32_t log_cols = log_n - LOG_R;  // n / R columns
  const size_t ns_mask = ((size_t)1 << log_ns) - 1;
  const uint32_t tw_shift = log_n - log_ns - LOG_R;  // exponent unit n / (Ns R)
  const uint64_t lo_mask = ((uint64_t)1 << kb) - 1;

  // Load + column twiddle, scattered into the bit-reversed LDS image [r][b].
  for (uint32_t e = threadIdx.x; e < E; e += T) {
    const uint32_t b = e & (B - 1), r = e >> log_b;
    const size_t j = j0 + b;
    fe v = fe_load(in + j + ((size_t)r << log_cols));
    if (log_ns != 0 && r != 0) {
      const uint64_t ex = ((uint64_t)(j & ns_mask) * r) << tw_shift;
      const fe t = fe_mul(tw_lo[ex & lo_mask], tw_hi[ex >> kb]);
      v = fe_mul(v, t);
    }
    const uint32_t rr = __builtin_bitreverse32(r) >> (32 - LOG_R);
    lds[(rr << log_b) + b] = v;
  }
  __syncthreads();

  // R-point radix-2 DIT, in place in LDS.
#pragma unroll 1
  for (int s = 0; s < LOG_R; ++s) {
    const uint32_t m = 1u << s;
    for (uint32_t g = threadIdx.x; g < E / 2; g += T) {
      const uint32_t b = g & (B - 1), q = g >> log_b;
      const uint32_t jj = q & (m - 1);
      const uint32_t pa = ((q >> s) << (s + 1)) + jj;
      fe* xa = &lds[(pa << log_b) + b];
      fe* xb = &lds[((pa + m) << log_b) + b];
      fe a = *xa, c = *xb;
      if (s != 0) c = fe_mul(c, small[jj << (LOG_R - 1 - s)]);
      *xa = fe_add(a, c);
      *xb = fe_sub(a, c);
    }
    __syncthreads();
  }

  // Store: out[(j / Ns) Ns R + (j mod Ns) + r Ns].
  if (((size_t)1 << log_ns) >= B) {
    for (uint32_t e = threadIdx.x; e < E; e += T) {
      const uint32_t b = e & (B - 1), r = e >> log_b;
      const size_t j = j0 + b;
      const size_t dst = ((j >> log_ns) << (log_ns + LOG_R)) + (j & ns_mask) + ((size_t)r << log_ns);
      fe v = lds[(r << log_b) + b];
      if (do_scale) v = fe_mul(v, scale);
      fe_store(out + dst, v);
    }
  } else {
    // Ns < B: the workgroup's output is the contiguous run [j0 R, (j0 + B) R).
    for (uint32_t o = threadIdx.x; o < E; o += T) {
      const uint32_t q = o >> (log_ns + LOG_R);
      const uint32_t rem = o & ((1u << (log_ns + LOG_R)) - 1);
      const uint32_t r = rem >> log_ns;
      const uint32_t b = (q << log_ns) + (rem & (uint32_t)ns_mask);
      fe v = lds[(r << log_b) + b];
      if (do_scale) v = fe_mul(v, scale);
      fe_store(out + (j0 << LOG_R) + o, v);
    }
  }
}

namespace {

struct PassPlan {
  int n_pass = 0;
  uint32_t log_r[8] = {0};
};

constexpr uint32_t kMaxLogR = 8;

PassPlan plan_passes(uint32_t log_n) {
  PassPlan p;
  p.n_pass = (int)((log_n + kMaxLogR - 1) / kMaxLogR);
  const uint32_t base = log_n / p.n_pass, extra = log_n % p.n_pass;
  for (int i = 0; i < p.n_pass; ++i) p.log_r[i] = base + ((uint32_t)i < extra ? 1 : 0);
  return p;
}

// Columns per workgroup (log2): >= 4 columns (128-B runs) when possible,
// enough elements to give 256 butterflies, never more than n / R columns.
uint32_t choose_log_b(uint32_t log_n, uint32_t log_r) {
  uint32_t lb = 2;
  while (log_r + lb < 9) ++lb;
  if (lb > log_n - log_r) lb = log_n - log_r;
  return lb;
}

typedef void (*pass_fn)(const fe*, fe*, uint32_t, uint32_t, uint32_t, const fe*, const fe*, uint32_t, const fe*,
                        fe, int);

pass_fn pass_kernel(uint32_t log_r) {
  switch (log_r) {
    case 1: return ntt_pass_kernel<1>;
    case 2: return ntt_pass_kernel<2>;
    case 3: return ntt_pass_kernel<3>;
    case 4: return ntt_pass_kernel<4>;
    case 5: return ntt_pass_kernel<5>;
    case 6: return ntt_pass_kernel<6>;
    case 7: return ntt_pass_kernel<7>;
    case 8: return ntt_pass_kernel<8>;
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
  // Small-root tables for every radix 2^l (l <= min(log_n, 8)): w^(k n / R), k < R/2.
  std::vector<fe> h_small;
  for (uint32_t l = 1; l <= kMaxLogR && l <= log_n; ++l) {
    tw->small_off[l] = (uint32_t)h_small.size();
    const HostFp wr = F.pow_u64(w, (uint64_t)1 << (log_n - l));
    HostFp a = F.one();
    for (uint32_t k = 0; k < (1u << (l - 1)); ++k) {
      h_small.push_back(to_dev(a));
      a = F.mul(a, wr);
    }
  }
  if (h_small.empty()) h_small.push_back(to_dev(F.one()));
  const size_t bytes = (n_lo + n_hi + h_small.size()) * sizeof(fe);
  void* d = nullptr;
  if (hipMalloc(&d, bytes) != hipSuccess) return STARK_ERR_OOM;
  tw->d_lo = (fe*)d;
  tw->d_hi = tw->d_lo + n_lo;
  tw->d_small = tw->d_hi + n_hi;
  STARK_HIP(ctx, hipMemcpy(tw->d_lo, h_lo.data(), n_lo * sizeof(fe), hipMemcpyHostToDevice));
  STARK_HIP(ctx, hipMemcpy(tw->d_hi, h_hi.data(), n_hi * sizeof(fe), hipMemcpyHostToDevice));
  STARK_HIP(ctx, hipMemcpy(tw->d_small, h_small.data(), h_small.size() * sizeof(fe), hipMemcpyHostToDevice));
  *out = tw.get();
  ctx->tw.emplace(key, std::move(tw));
  return STARK_OK;
}

stark_status ntt_device(stark_ctx* ctx, fe* d_data, uint32_t log_n, uint32_t batch, const Twiddles& tw,
                        bool inverse, hipStream_t stream) {
  if (batch == 0) return STARK_OK;
  if (batch > 65535) return STARK_ERR_BAD_ARG;
  const size_t n = (size_t)1 << log_n;
  const fe scale = to_dev(tw.inv_n);
  if (log_n == 0) return STARK_OK;  // 1-point DFT is the identity (n^-1 = 1)
  const PassPlan plan = plan_passes(log_n);
  stark_status st = ensure_buf(ctx, ctx->scratch, n * batch * sizeof(fe));
  if (st != STARK_OK) return st;
  fe* scratch = (fe*)ctx->scratch.ptr;
  fe* cur = d_data;
  uint32_t log_ns = 0;
  for (int p = 0; p < plan.n_pass; ++p) {
    const uint32_t lr = plan.log_r[p];
    const bool last = p == plan.n_pass - 1;
    // Passes before the last ping-pong; the last pass (Ns R = n) reads and
    // writes the same positions, so it always lands in d_data.
    fe* dst = last ? d_data : (cur == d_data ? scratch : d_data);
    const uint32_t lb = choose_log_b(log_n, lr);
    const uint32_t elems = 1u << (lr + lb);
    const uint32_t threads = elems / 2 < 256 ? (elems / 2 < 64 ? 64 : elems / 2) : 256;
    dim3 grid((unsigned)(n >> (lr + lb)), batch);
    hipLaunchKernelGGL(pass_kernel(lr), grid, dim3(threads), elems * sizeof(fe), stream, cur, dst, log_n, log_ns,
                       lb, tw.d_lo, tw.d_hi, tw.kb, tw.d_small + tw.small_off[lr], scale, (inverse && last) ? 1 : 0);
    STARK_HIP(ctx, hipGetLastError());
    cur = dst;
    log_ns += lr;
  }
  return STARK_OK;
}

}  // namespace stark
