# Variant E4 (round 6, timing only; measured and dropped): a persistent dense first pass (radix 2^8 as
# 16 x 16, B = 4) whose next tile lands in a second LDS image by LDS-DMA (global_load_lds_dwordx4, issued
# by inline asm so the compiler's own LDS-DMA tracking does not drain it with a vmcnt(0) at the next
# ds_read) while the workgroup computes the current tile; raw s_barrier after lgkmcnt(0), and a counted
# vmcnt(8) (the previous tile's 8 stores are younger) retires the DMA.  80 KB of LDS per workgroup, so 2
# workgroups per CU.  Digests equal; 2^24 +3 %: the pass's VALU issue fell from 0.88 to 0.63 at 2 waves per
# SIMD (profiles/r06_ntt_first_pass_dma_ab.txt).
# Build: tools/build_variant.sh out.so @tools/ntt_variants/e4_first_pass_dma.py
KERNEL = r'''
// Persistent dense first pass with the next tile's loads in flight (variant E4, see tools/ntt_variants).
typedef __attribute__((address_space(3))) void glds_lvoid;
__device__ __forceinline__ void raw_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__global__ __launch_bounds__(kPassThreads, 2) void ntt_first_dma_kernel(const fe* __restrict__ in, fe* __restrict__ out,
                                                                       uint32_t log_n, const fe* __restrict__ small,
                                                                       const uint32_t* __restrict__ db,
                                                                       uint32_t log_tiles, uint32_t total_tiles) {
  constexpr uint32_t LOG_R = 8, R = 1u << LOG_R, LT = 4, log_b = 2, kImg = 1024;
  extern __shared__ __attribute__((aligned(16))) fe lds[];
  fe* sm = lds;  // R Shoup pairs w_R^e
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const uint32_t log_cols = log_n - LOG_R, tile_mask = (1u << log_tiles) - 1;
  const uint32_t b = tid & 3, q = tid >> 2;
  uint32_t tile = blockIdx.x;
  if (tile >= total_tiles) return;  // (uniform)
  auto dma = [&](uint32_t t, uint32_t buf) {
    const fe* src = in + ((size_t)(t >> log_tiles) << log_n) + ((size_t)(t & tile_mask) << log_b);
    uint4* img = reinterpret_cast<uint4*>(lds + 2 * R + buf * kImg);
#pragma unroll
    for (uint32_t u = 0; u < 8; ++u) {
      const uint32_t blk = wave * 4 + (u >> 1), plane = u & 1;
      const uint32_t slot = blk * 64 + lane;
      const uint32_t r = __builtin_bitreverse32(slot >> 2) >> 24;  // natural row of image row slot / 4
      const uint4* g = reinterpret_cast<const uint4*>(src + (slot & 3) + ((size_t)r << log_cols)) + plane;
      const uint32_t m0 = __builtin_amdgcn_readfirstlane(
          (uint32_t)(size_t)(glds_lvoid*)(img + plane * kImg + blk * 64));
      asm volatile("s_mov_b32 m0, %0\n\tglobal_load_lds_dwordx4 %1, off" ::"s"(m0), "v"(g) : "memory", "m0");
    }
  };
  dma(tile, 0);
  {  // the twiddle pairs, once per workgroup
    const uint4* small4 = reinterpret_cast<const uint4*>(small);
    uint4* sm4 = reinterpret_cast<uint4*>(sm);
    uint4 ts[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) ts[i] = small4[tid + i * kPassThreads];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) sm4[tid + i * kPassThreads] = ts[i];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  for (uint32_t it = 0;; ++it) {
    if (it) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this tile's DMA (the previous stores are younger)
    raw_barrier();
    const uint32_t next = tile + gridDim.x;
    if (next < total_tiles) dma(next, (it + 1) & 1);
    const XImage XI{lds + 2 * R + (it & 1) * kImg, kImg};
    const size_t boff = (size_t)(tile >> log_tiles) << log_n;
    const size_t j0 = (size_t)(tile & tile_mask) << log_b;
    {  // first radix-4 step: image rows 4q .. 4q + 3 of column b (canonical inputs, < p)
      const uint32_t i0 = (q << 4) + b;
      fe x0 = XI.ld(i0), x1 = XI.ld(i0 + 4), x2 = XI.ld(i0 + 8), x3 = XI.ld(i0 + 12);
      bfly_lt2p(x0, x1, x1);
      bfly_lt2p(x2, x3, x3);
      const fe t3 = fe_mul_db(x3, db + 72u * (1u << (LOG_R - 2)));
      fe_csub2p(x2);
      bfly<false>(x0, x2, x2);
      bfly<false>(x1, x3, t3);
      XI.st(i0, x0);
      XI.st(i0 + 4, x1);
      XI.st(i0 + 8, x2);
      XI.st(i0 + 12, x3);
    }
    raw_barrier();
    {  // radix-4 step s = 2 (m = 4), jj-major: one jj per wave
      const uint32_t jj = wave, rest = lane;
      const uint32_t i0 = ((((rest >> log_b) << 4) + jj) << log_b) + (rest & 3), st = 4u << log_b;
      fe x0 = XI.ld(i0), x1 = XI.ld(i0 + st), x2 = XI.ld(i0 + 2 * st), x3 = XI.ld(i0 + 3 * st);
      if (jj == 0) {
        csub2p_t<false>(x1);
        csub2p_t<false>(x3);
        bfly<false>(x0, x1, x1);
        bfly<false>(x2, x3, x3);
        const fe t3 = fe_mul_db(x3, db + 72u * (1u << (LOG_R - 2)));
        csub2p_t<false>(x2);
        bfly<false>(x0, x2, x2);
        bfly<false>(x1, x3, t3);
      } else {
        const uint32_t ju = __builtin_amdgcn_readfirstlane(jj);
        const uint32_t* wa = db + 72u * (ju << (LOG_R - 3));  // w_8^jj
        const fe t1 = fe_mul_db(x1, wa);
        fe t3 = fe_mul_db(x3, wa);
        bfly<false>(x0, x1, t1);
        bfly<false>(x2, x3, t3);
        const fe t2 = fe_mul_db(x2, db + 72u * (ju << (LOG_R - 4)));  // w_16^jj
        t3 = fe_mul_db(x3, db + 72u * ((ju + 4) << (LOG_R - 4)));     // w_16^(jj + 4)
        bfly<false>(x0, x2, t2);
        bfly<false>(x1, x3, t3);
      }
      XI.st(i0, x0);
      XI.st(i0 + 2 * st, x2);
      XI.st(i0 + st, x1);
      XI.st(i0 + 3 * st, x3);
    }
    raw_barrier();
    {  // twiddles w_R^(rev4(g) t), then the first radix-4 step of the 16-point DFT across the groups
      const uint32_t t = q & 15, a = q >> LT;
      const uint32_t i0 = (((a << (LT + 2)) + t) << log_b) + b, st = (1u << LT) << log_b;
      const bool unit0 = __builtin_amdgcn_readfirstlane(a) == 0;
      fe x[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const fe v = XI.ld(i0 + k * st);
        if (k == 0 && unit0) {
          x[0] = v;
          fe_csub2p(x[0]);
          continue;
        }
        const uint32_t e = (__builtin_bitreverse32((a << 2) + k) >> 28) * t;
        x[k] = fe_mul_shoup(v, sm[2 * e], sm[2 * e + 1]);
      }
      bfly_lt2p(x[0], x[1], x[1]);
      bfly_lt2p(x[2], x[3], x[3]);
      const fe t3 = fe_mul_db(x[3], db + 72u * (1u << (LOG_R - 2)));
      fe_csub2p(x[2]);
      bfly<false>(x[0], x[2], x[2]);
      bfly<false>(x[1], x[3], t3);
#pragma unroll
      for (int k = 0; k < 4; ++k) XI.st(i0 + k * st, x[k]);
    }
    raw_barrier();
    fe yl[4];
    {  // second radix-4 step (stride R/4 rows), a = q >> 4 uniform per wave
      const uint32_t i0 = (q << log_b) + b, st = (R / 4) << log_b;
      fe x0 = XI.ld(i0), x1 = XI.ld(i0 + st), x2 = XI.ld(i0 + 2 * st), x3 = XI.ld(i0 + 3 * st);
      const uint32_t a = __builtin_amdgcn_readfirstlane(q >> LT);
      if (a == 0) {
        csub2p_t<false>(x1);
        csub2p_t<false>(x3);
        bfly<false>(x0, x1, x1);
        bfly<false>(x2, x3, x3);
        const fe t3 = fe_mul_db(x3, db + 72u * (1u << (LOG_R - 2)));
        csub2p_t<false>(x2);
        bfly<false>(x0, x2, x2);
        bfly<false>(x1, x3, t3);
      } else {
        const uint32_t* wa = db + 72u * (a << (LOG_R - 3));
        const fe t1 = fe_mul_db(x1, wa);
        fe t3 = fe_mul_db(x3, wa);
        bfly<false>(x0, x1, t1);
        bfly<false>(x2, x3, t3);
        const fe t2 = fe_mul_db(x2, db + 72u * (a << LT));
        t3 = fe_mul_db(x3, db + 72u * ((a + 4) << LT));
        bfly<false>(x0, x2, t2);
        bfly<false>(x1, x3, t3);
      }
      yl[0] = x0;
      yl[1] = x1;
      yl[2] = x2;
      yl[3] = x3;
    }
    // store: out[j R + r], rows q + 64 k of column j = j0 + b
    fe* dst = out + boff + ((j0 + b) << LOG_R) + q;
#pragma unroll
    for (int k = 0; k < 4; ++k) fe_store_nt(dst + 64 * k, yl[k]);
    tile = next;
    if (tile >= total_tiles) break;
  }
}
'''
LAUNCH = r'''    int cus = 0;
    if (col == kColNone && lr == 8 && lb == 2 && !last &&
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ctx->device) == hipSuccess &&
        total >= (uint64_t)8 * cus) {
      const unsigned grid = (unsigned)std::min<uint64_t>(total, (uint64_t)2 * cus);
      const size_t lds_dma = (2 * 256 + 2 * 1024) * sizeof(fe);
      static const hipError_t attr = hipFuncSetAttribute((const void*)ntt_first_dma_kernel,
                                                         hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_dma);
      (void)attr;
      hipLaunchKernelGGL(ntt_first_dma_kernel, dim3(grid), dim3(kPassThreads), lds_dma, stream, cur, dst, log_n,
                         tw.d_small + tw.small_off[lr], tw.d_db + tw.db_off[lr], log_tiles, (uint32_t)total);
    } else
'''
ANCHOR_K = "// dst[c][i] = i < 2^log_m ? src[c][i] : 0 (best_fft's zero padding, fft.rs:327-357)."
ANCHOR_L = """    hipLaunchKernelGGL(pass_kernel(lr, col), dim3((unsigned)total), dim3(threads), lds, stream, cur, dst, log_n,
                       log_ns, lb, ct, tw.d_small + tw.small_off[lr], tw.d_db + tw.db_off[lr], scale,"""


def apply(s):
    assert s.count(ANCHOR_K) == 1 and s.count(ANCHOR_L) == 1
    s = s.replace(ANCHOR_K, KERNEL + "\n" + ANCHOR_K)
    return s.replace(ANCHOR_L, LAUNCH + ANCHOR_L)
