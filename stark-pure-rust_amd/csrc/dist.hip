// Local building blocks of the multi-GPU four-step NTT (stark_amd/distributed.py):
// a tiled transpose of 32-B field elements and the four-step twiddle
// data[i][j] *= w^((row_base + i) * (col_base + j)).  The exchange steps are
// RCCL all-to-alls issued by the caller (torch.distributed, backend "nccl").
#include "fe_db.h"
#include "internal.h"

namespace stark {

constexpr int kTT = 32;  // transpose tile (elements)

// dst[c][r] = src[r][c] for a rows x cols matrix, batch matrices back to back.
__global__ __launch_bounds__(256) void transpose_kernel(const fe* __restrict__ src, fe* __restrict__ dst,
                                                        uint64_t rows, uint64_t cols) {
  __shared__ fe tile[kTT][kTT + 1];
  const uint64_t mat = (uint64_t)blockIdx.z * rows * cols;
  const uint64_t r0 = (uint64_t)blockIdx.y * kTT, c0 = (uint64_t)blockIdx.x * kTT;
  const uint32_t tx = threadIdx.x & (kTT - 1), ty = threadIdx.x / kTT;  // 32 x 8
  for (uint32_t y = ty; y < kTT; y += 8) {
    const uint64_t r = r0 + y, c = c0 + tx;
    if (r < rows && c < cols) tile[y][tx] = src[mat + r * cols + c];
  }
  __syncthreads();
  for (uint32_t y = ty; y < kTT; y += 8) {
    const uint64_t c = c0 + y, r = r0 + tx;
    if (r < rows && c < cols) dst[mat + c * rows + r] = tile[tx][y];
  }
}

// data[i * cols + j] *= w^(((row_base + i) * (col_base + j)) mod order), w's
// powers from the two-level tables (exponents < 2^log_order).
__global__ void twiddle2d_kernel(fe* __restrict__ data, uint64_t rows, uint64_t cols, uint64_t row_base,
                                 uint64_t col_base, const fe* __restrict__ lo, const fe* __restrict__ hi, uint32_t kb,
                                 uint32_t log_order) {
  const uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * cols) return;
  const uint64_t i = idx / cols, j = idx % cols;
  const uint64_t mask = ((uint64_t)1 << log_order) - 1;
  const uint64_t e = ((row_base + i) & mask) * ((col_base + j) & mask) & mask;
  const fe t = fe_mul(lo[e & (((uint64_t)1 << kb) - 1)], hi[e >> kb]);
  fe_store(data + idx, fe_mul(fe_load(data + idx), t));
}

// post[k] = w^(rank k mod n), k < m (Montgomery images of the two-level tables' product): the
// one-exchange distributed NTT's twiddle, multiplied into the rank's local transform's last store.
__global__ void post_tw_kernel(fe* __restrict__ out, uint64_t m, uint64_t rank, uint32_t log_n,
                               const fe* __restrict__ lo, const fe* __restrict__ hi, uint32_t kb) {
  const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= m) return;
  const uint64_t e = (rank * k) & (((uint64_t)1 << log_n) - 1);
  fe_store(out + k, fe_mul(lo[e & (((uint64_t)1 << kb) - 1)], hi[e >> kb]));
}

// Small DFTs across a stride: for each i < stride, the G = 2^LOG_G points
// d[i + stride j], j < G, are replaced by their DFT (root w_G), in place:
//   out[i + stride k] = sum_j d[i + stride j] w_G^(j k)   [* G^-1 when scaling].
// One thread per i, the G values in registers; adjacent threads touch
// adjacent elements, so every access is coalesced.  This is the cross-rank
// DFT of the one-exchange distributed NTT (stark_amd/distributed.py).
struct SmallRoots {
  fe w[8];  // w_G^k, k < G/2 (Montgomery)
};

// Optional input twiddle, applied before the DFT: d[i + stride j] *=
// w^(j (base + i)) (w from the two-level tables) -- the one-exchange
// distributed NTT's w^(r k2) factor applied at the receiver, fused here so the
// sender does not spend a separate pass over HBM on it.
struct StridedTw {
  const fe* lo;
  const fe* hi;
  uint32_t kb;
  uint64_t base, mask;  // exponent (base + i) & mask, mask = order - 1
};

// db != nullptr: the DFT's constants w_G^k (k < G/2) as digit-basis tables (fe_db.h, 72 words each):
// uniform across the grid, so the product takes them from SGPRs (140 VALU instead of a Montgomery
// product's ~300); the result is reduced to canonical for the full-reduction butterflies.
template <int LOG_G, bool TW>
__global__ __launch_bounds__(256) void strided_ntt_kernel(fe* __restrict__ d, uint64_t stride, SmallRoots rt,
                                                          fe scale, int do_scale, StridedTw tw,
                                                          const uint32_t* __restrict__ db) {
  constexpr int G = 1 << LOG_G;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= stride) return;
  fe x[G];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    int br = 0;
#pragma unroll
    for (int b = 0; b < LOG_G; ++b) br |= ((j >> b) & 1) << (LOG_G - 1 - b);
    x[br] = fe_load(d + i + stride * (uint64_t)j);  // bit-reversed order for the in-place DIT
  }
  if (TW) {
    const uint64_t e = (tw.base + i) & tw.mask;
    const fe step = fe_mul(tw.lo[e & (((uint64_t)1 << tw.kb) - 1)], tw.hi[e >> tw.kb]);  // w^e, Montgomery
    fe t = step;
#pragma unroll
    for (int j = 1; j < G; ++j) {
      int br = 0;
#pragma unroll
      for (int b = 0; b < LOG_G; ++b) br |= ((j >> b) & 1) << (LOG_G - 1 - b);
      x[br] = fe_mul(x[br], t);  // canonical * Montgomery -> canonical
      if (j + 1 < G) t = fe_mul(t, step);
    }
  }
#pragma unroll
  for (int s = 0; s < LOG_G; ++s) {
    const int m = 1 << s;
#pragma unroll
    for (int k = 0; k < G; k += 2 * m)
#pragma unroll
      for (int jj = 0; jj < m; ++jj) {
        fe t = x[k + jj + m];
        if (jj) {  // w_{2m}^jj
          if (db) {
            t = fe_mul_db(t, db + 72u * (jj << (LOG_G - 1 - s)));
            fe_reduce_once(t);
          } else {
            t = fe_mul(t, rt.w[jj << (LOG_G - 1 - s)]);
          }
        }
        const fe u = x[k + jj];
        x[k + jj] = fe_add(u, t);
        x[k + jj + m] = fe_sub(u, t);
      }
  }
#pragma unroll
  for (int k = 0; k < G; ++k) fe_store(d + i + stride * (uint64_t)k, do_scale ? fe_mul(x[k], scale) : x[k]);
}

}  // namespace stark

using namespace stark;

extern "C" {

stark_status stark_transpose_dev(stark_ctx* ctx, const uint64_t* d_src, uint64_t* d_dst, size_t rows, size_t cols,
                                 uint32_t batch, void* stream) {
  if (!ctx || !d_src || !d_dst || d_src == d_dst) return STARK_ERR_BAD_ARG;
  if (rows == 0 || cols == 0 || batch == 0) return STARK_OK;
  if ((rows + kTT - 1) / kTT > 65535 || batch > 65535) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  dim3 grid((unsigned)((cols + kTT - 1) / kTT), (unsigned)((rows + kTT - 1) / kTT), batch);
  hipLaunchKernelGGL(transpose_kernel, grid, dim3(256), 0, pick_stream(ctx, stream), (const fe*)d_src, (fe*)d_dst,
                     (uint64_t)rows, (uint64_t)cols);
  STARK_HIP(ctx, hipGetLastError());
  return STARK_OK;
}

static stark_status strided(stark_ctx* ctx, uint64_t* d_data, uint32_t log_g, size_t stride, const uint64_t root[4],
                            int inverse, const uint64_t* tw_root, uint32_t log_order, uint64_t tw_base, void* stream) {
  if (!ctx || !d_data || !root) return STARK_ERR_BAD_ARG;
  if (log_g > 4) return STARK_ERR_BAD_LENGTH;
  if (stride == 0 || log_g == 0) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const FieldHost& F = FieldHost::get();
  HostFp w = F.from_canonical(root);
  // root must be a primitive 2^log_g-th root: w^(G/2) = -1.
  const HostFp half = F.pow_u64(w, (uint64_t)1 << (log_g - 1));
  if (!FieldHost::eq(F.add(half, F.one()), F.zero())) return STARK_ERR_BAD_ROOT;
  if (inverse) w = F.inv(w);
  SmallRoots rt;
  HostFp p = F.one();
  for (int k = 0; k < 8; ++k) {
    rt.w[k] = to_dev(p);
    p = F.mul(p, w);
  }
  StridedTw tw{nullptr, nullptr, 0, tw_base, 0};
  if (tw_root) {
    const Twiddles* t = nullptr;
    const stark_status st = get_twiddles(ctx, tw_root, log_order, &t);
    if (st != STARK_OK) return st;
    tw = StridedTw{t->d_lo, t->d_hi, t->kb, tw_base, ((uint64_t)1 << log_order) - 1};
  }
  const fe scale = to_dev(F.inv(F.from_u64((uint64_t)1 << log_g)));
  // the DFT's constants as digit-basis tables (the tables of the root w (or w^-1) of order G)
  const uint32_t* db = nullptr;
  {
    uint64_t wc[4];
    F.to_canonical(w, wc);
    const Twiddles* tg = nullptr;
    const stark_status st = get_twiddles(ctx, wc, log_g, &tg);
    if (st != STARK_OK) return st;
    db = tg->d_db + tg->db_off[log_g];
  }
  const unsigned grid = (unsigned)((stride + 255) / 256);
  hipStream_t s = pick_stream(ctx, stream);
  fe* d = (fe*)d_data;
  const int sc = inverse ? 1 : 0;
  const uint64_t st = stride;
#define STARK_STRIDED(LG)                                                                                      \
  do {                                                                                                        \
    if (tw_root)                                                                                              \
      hipLaunchKernelGGL((strided_ntt_kernel<LG, true>), dim3(grid), dim3(256), 0, s, d, st, rt, scale, sc, tw,   \
                         db);                                                                                 \
    else                                                                                                      \
      hipLaunchKernelGGL((strided_ntt_kernel<LG, false>), dim3(grid), dim3(256), 0, s, d, st, rt, scale, sc, tw,  \
                         db);                                                                                 \
  } while (0)
  switch (log_g) {
    case 1: STARK_STRIDED(1); break;
    case 2: STARK_STRIDED(2); break;
    case 3: STARK_STRIDED(3); break;
    default: STARK_STRIDED(4); break;
  }
#undef STARK_STRIDED
  STARK_HIP(ctx, hipGetLastError());
  return STARK_OK;
}

stark_status stark_ntt_strided_dev(stark_ctx* ctx, uint64_t* d_data, uint32_t log_g, size_t stride,
                                   const uint64_t root[4], int inverse, void* stream) {
  return strided(ctx, d_data, log_g, stride, root, inverse, nullptr, 0, 0, stream);
}

stark_status stark_ntt_strided_tw_dev(stark_ctx* ctx, uint64_t* d_data, uint32_t log_g, size_t stride,
                                      const uint64_t root[4], int inverse, const uint64_t tw_root[4],
                                      uint32_t log_order, uint64_t tw_base, void* stream) {
  if (!tw_root) return STARK_ERR_BAD_ARG;
  return strided(ctx, d_data, log_g, stride, root, inverse, tw_root, log_order, tw_base, stream);
}

stark_status stark_cyclic_ntt_local_dev(stark_ctx* ctx, uint64_t* d_data, uint32_t log_n, uint32_t log_g,
                                       uint32_t rank, const uint64_t root[4], int inverse, void* stream) {
  if (!ctx || !d_data || !root) return STARK_ERR_BAD_ARG;
  // M = 2^(log_n - log_g) >= 4 points per rank, and G | M (the exchange's chunks)
  if (log_n > 28 || log_g > 4 || log_n < log_g + 2 || log_n < 2 * log_g || rank >= (1u << log_g))
    return STARK_ERR_BAD_LENGTH;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const FieldHost& F = FieldHost::get();
  const uint32_t log_m = log_n - log_g;
  HostFp w = F.from_canonical(root);
  {  // a primitive 2^log_n-th root: w^(n/2) = -1
    const HostFp half = F.pow_u64(w, (uint64_t)1 << (log_n - 1));
    if (!FieldHost::eq(F.add(half, F.one()), F.zero())) return STARK_ERR_BAD_ROOT;
  }
  if (inverse) w = F.inv(w);
  // the local M-point transform's root w^G (its inverse tables for the inverse direction)
  uint64_t wl[4];
  F.to_canonical(F.pow_u64(w, (uint64_t)1 << log_g), wl);
  const Twiddles* tl = nullptr;
  STARK_TRY(get_twiddles(ctx, wl, log_m, &tl));
  // post[k] = w^(rank k), k < M (cached per root, size and rank, in the capped table cache)
  uint64_t wc[4];
  F.to_canonical(w, wc);
  const auto key = std::make_tuple(wc[0], wc[1], wc[2], wc[3], log_n, rank);
  hipStream_t s = pick_stream(ctx, stream);
  auto it = ctx->post_tw.find(key);
  if (it == ctx->post_tw.end()) {
    const Twiddles* tn = nullptr;
    STARK_TRY(get_twiddles(ctx, wc, log_n, &tn));
    const uint64_t M = (uint64_t)1 << log_m;
    void* p = nullptr;
    const bool cached = cache_reserve(ctx, M * sizeof(fe), false);
    if (!cached) {
      // Larger than the cache cap: this call's own table, allocated and freed in the stream's order (no
      // host synchronisation: the call stays asynchronous on s).
      STARK_HIP(ctx, hipMallocAsync(&p, M * sizeof(fe), s));
      hipLaunchKernelGGL(post_tw_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, (fe*)p, M,
                         (uint64_t)rank, log_n, tn->d_lo, tn->d_hi, tn->kb);
      const hipError_t ke = hipGetLastError();
      stark_status st = ke == hipSuccess ? STARK_OK : hip_fail(ctx, ke, "post_tw_kernel");
      if (st == STARK_OK) st = ntt_device(ctx, (fe*)d_data, log_m, 1, *tl, inverse != 0, s, (const fe*)p);
      const hipError_t fe_ = hipFreeAsync(p, s);
      if (st == STARK_OK && fe_ != hipSuccess) st = hip_fail(ctx, fe_, "hipFreeAsync");
      return st;
    }
    if (hipMalloc(&p, M * sizeof(fe)) != hipSuccess) {
      hipGetLastError();
      return STARK_ERR_OOM;
    }
    hipLaunchKernelGGL(post_tw_kernel, dim3((unsigned)((M + 255) / 256)), dim3(256), 0, s, (fe*)p, M, (uint64_t)rank,
                       log_n, tn->d_lo, tn->d_hi, tn->kb);
    {
      const hipError_t e_ = hipGetLastError();
      if (e_ != hipSuccess) {
        hipFree(p);
        return hip_fail(ctx, e_, "post_tw_kernel");
      }
    }
    CacheBuf cb{p, M * sizeof(fe), 0};
    {
      const stark_status st = fill_mark(ctx, cb.ev, cb.fill, s);  // complete once the fill has run on s
      if (st != STARK_OK) {
        hipStreamSynchronize(s);  // (the fill may still run)
        hipFree(p);
        if (cb.ev) hipEventDestroy(cb.ev);
        return st;
      }
    }
    it = ctx->post_tw.emplace(key, cb).first;
  }
  CacheBuf& e = it->second;
  e.used = ++ctx->cache_clock;
  STARK_TRY(fill_wait(ctx, e.ev, e.fill, s));  // (filled by a call on another stream)
  // Held while the transform is enqueued: its last pass's full table (ntt_device -> cache_reserve)
  // must not evict this entry and launch with a freed pointer.
  e.in_use = true;
  const stark_status st = ntt_device(ctx, (fe*)d_data, log_m, 1, *tl, inverse != 0, s, (const fe*)e.ptr);
  e.in_use = false;
  return st;
}

stark_status stark_twiddle2d_dev(stark_ctx* ctx, uint64_t* d_data, size_t rows, size_t cols, uint64_t row_base,
                                 uint64_t col_base, const uint64_t root[4], uint32_t log_order, void* stream) {
  if (!ctx || !d_data || !root) return STARK_ERR_BAD_ARG;
  if (rows == 0 || cols == 0) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const Twiddles* tw = nullptr;
  stark_status st = get_twiddles(ctx, root, log_order, &tw);
  if (st != STARK_OK) return st;
  const uint64_t total = (uint64_t)rows * cols;
  hipLaunchKernelGGL(twiddle2d_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, pick_stream(ctx, stream),
                     (fe*)d_data, (uint64_t)rows, (uint64_t)cols, row_base, col_base, tw->d_lo, tw->d_hi, tw->kb,
                     log_order);
  STARK_HIP(ctx, hipGetLastError());
  return STARK_OK;
}

}  // extern "C"
