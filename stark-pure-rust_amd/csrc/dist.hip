// Local building blocks of the multi-GPU four-step NTT (stark_amd/distributed.py):
// a tiled transpose of 32-B field elements and the four-step twiddle
// data[i][j] *= w^((row_base + i) * (col_base + j)).  The exchange steps are
// RCCL all-to-alls issued by the caller (torch.distributed, backend "nccl").
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
