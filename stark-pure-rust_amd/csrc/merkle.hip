// Blake2s Merkle commitment on gfx950: the tree of
// gen_multi_proofs_multi_core (packages/commitment/src/merkle_proof_in_place.rs:106-206):
// leaf node = Blake2s(leaf bytes), parent = Blake2s(left || right), root =
// the single node of the top level.  The reference splits the tree into
// 2^log2(cpus) subtrees and a top tree; every split yields this same tree.
//
// HBM layout: all 2n-1 digests, level-major (level 0 = leaf digests, then
// n/2 parents, ... , root), each 32 B.  gen_proofs only gathers siblings from
// this resident tree.
//
// Build: one workgroup owns a block of 1024 nodes of its input level: it
// hashes them (leaf mode: one leaf per node; pair mode: two child digests per
// node read from the level below), then reduces the block in LDS for the
// next levels, writing every level to HBM.  Only the levels with >= 256
// nodes per block (one per thread) are reduced in LDS, so no lane idles
// through the narrow levels; the top of the tree (< 64K nodes per level) is
// finished by merkle_tail_kernel, which spreads each compression over a quad
// of lanes to cut the per-level latency.
#include "internal.h"
#include "blake2s.h"
#include "merkle_dev.h"

struct stark_merkle_tree {
  stark_ctx* ctx = nullptr;
  size_t n = 0, leaf_len = 0;
  uint32_t depth = 0;                // log2(n)
  stark::DevBuf nodes;               // (2n - 1) * 32 B
  stark::DevBuf own_leaves;          // leaves copied from the host
  const uint8_t* d_leaves = nullptr; // leaves the proofs are read from
  uint64_t plane_stride = 0;         // 0: contiguous leaves; else 32-B planes (merkle_build)
  bool built = false;
  bool has_root = false;             // set by gen_proofs (reference: root = H::default() before)
  uint8_t root[32];
  stark::DevBuf gather;              // scratch for proof gathers
};

namespace stark {

constexpr uint32_t kMerkleBlock = 1024;   // nodes per workgroup at its input level
constexpr uint32_t kMerkleThreads = 256;


// Digest of a leaf stored as len / 32 planes: its bytes [32 c, 32 c + 32) sit at
// base + c * stride + 32 * node (a column-major table whose rows are the leaves).  Every
// lane of a wave reads 32 adjacent bytes of each plane, so the loads coalesce.
__device__ __forceinline__ Digest hash_leaf_planes(const uint8_t* __restrict__ base, uint64_t node,
                                                   uint64_t stride, uint32_t len) {
  Digest d;
  b2s_init(d.h);
  const uint32_t planes = len / 32;
  uint32_t m[16];
  for (uint32_t c = 0; c < planes; c += 2) {
    const uint4* q0 = reinterpret_cast<const uint4*>(base + c * stride + 32 * node);
    uint4 x[4] = {q0[0], q0[1], make_uint4(0, 0, 0, 0), make_uint4(0, 0, 0, 0)};
    if (c + 1 < planes) {
      const uint4* q1 = reinterpret_cast<const uint4*>(base + (c + 1) * stride + 32 * node);
      x[2] = q1[0];
      x[3] = q1[1];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      m[4 * i] = x[i].x; m[4 * i + 1] = x[i].y; m[4 * i + 2] = x[i].z; m[4 * i + 3] = x[i].w;
    }
    const bool last = c + 2 >= planes;
    b2s_compress(d.h, m, last ? len : 32 * (c + 2), 0, last);
  }
  return d;
}

// One launch: input level `lvl_in` nodes [0, count) are produced by this
// workgroup's block (leaf mode: from leaves; pair mode: from level lvl_in-1
// at `below`), then `extra` more levels are reduced in LDS.
//   out_level[k] = pointer to level (lvl_in + k) in the node buffer.
struct LevelPtrs {
  Digest* lv[12];
};

template <bool LEAF32>
__global__ __launch_bounds__(kMerkleThreads) void merkle_build_kernel(const uint8_t* __restrict__ leaves,
                                                                      uint32_t leaf_len,
                                                                      const Digest* __restrict__ below,
                                                                      uint64_t count, uint32_t block,
                                                                      uint32_t extra, LevelPtrs out,
                                                                      uint64_t plane_stride) {
  __shared__ __attribute__((aligned(16))) Digest lds[kMerkleBlock];
  const uint64_t base = (uint64_t)blockIdx.x * block;
  const uint32_t here = (uint32_t)((count - base) < block ? (count - base) : block);
  if (leaves && !LEAF32) {
    for (uint32_t i = threadIdx.x; i < here; i += blockDim.x) {
      const uint64_t node = base + i;
      const Digest d = plane_stride ? hash_leaf_planes(leaves, node, plane_stride, leaf_len)
                                    : hash_leaf(leaves + node * leaf_len, leaf_len);
      store_digest(out.lv[0] + node, d);
      lds[i] = d;
    }
  } else {
    // 32-byte leaves or child pairs: the next node's message words are
    // loaded while the current one is hashed, so HBM latency hides behind
    // the compression instead of stalling every iteration.
    constexpr int kWords = LEAF32 ? 2 : 4;  // uint4 per node input
    const uint4* src = LEAF32 ? reinterpret_cast<const uint4*>(leaves + base * 32)
                              : reinterpret_cast<const uint4*>(below + 2 * base);
    uint4 nxt[kWords];
    uint32_t i = threadIdx.x;
    if (i < here) {
#pragma unroll
      for (int w = 0; w < kWords; ++w) nxt[w] = src[(size_t)i * kWords + w];
    }
    for (; i < here; i += blockDim.x) {
      uint4 cur[kWords];
#pragma unroll
      for (int w = 0; w < kWords; ++w) cur[w] = nxt[w];
      if (i + blockDim.x < here) {
#pragma unroll
        for (int w = 0; w < kWords; ++w) nxt[w] = src[(size_t)(i + blockDim.x) * kWords + w];
      }
      uint32_t m[16];
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        const uint4 x = w < kWords ? cur[w < kWords ? w : 0] : make_uint4(0, 0, 0, 0);
        m[4 * w] = x.x; m[4 * w + 1] = x.y; m[4 * w + 2] = x.z; m[4 * w + 3] = x.w;
      }
      Digest d;
      b2s_init(d.h);
      b2s_compress(d.h, m, LEAF32 ? 32 : 64, 0, true);
      store_digest(out.lv[0] + base + i, d);
      lds[i] = d;
    }
  }
  __syncthreads();
  uint32_t width = here;
  for (uint32_t k = 1; k <= extra; ++k) {
    width >>= 1;  // <= kMerkleBlock / 2 = 2 nodes per thread, held in registers (no scratch array)
    static_assert(kMerkleBlock / 2 <= 2 * kMerkleThreads, "two pair hashes per thread per level");
    const uint32_t i0 = threadIdx.x, i1 = threadIdx.x + blockDim.x;
    Digest r0, r1;
    if (i0 < width) r0 = hash_pair(lds[2 * i0], lds[2 * i0 + 1]);
    if (i1 < width) r1 = hash_pair(lds[2 * i1], lds[2 * i1 + 1]);
    __syncthreads();
    if (i0 < width) {
      lds[i0] = r0;
      store_digest(out.lv[k] + (base >> k) + i0, r0);
    }
    if (i1 < width) {
      lds[i1] = r1;
      store_digest(out.lv[k] + (base >> k) + i1, r1);
    }
    __syncthreads();
  }
}

// ---- Narrow top of the tree: one compression per quad of lanes (hash_pair_quad, merkle_dev.h) ----

constexpr uint32_t kTailThreads = 1024;
constexpr uint32_t kTailBlock = kTailThreads / 4;  // input-level nodes per workgroup
constexpr uint64_t kTailFrom = 65536;              // pair levels narrower than this take the quad kernel

// The levels of one workgroup's block: `here` nodes of the input level from the pairs in msg (LDS, already
// loaded), then `extra` more levels; level k's nodes go to out.lv[k] + (base >> k).  With `coherent`, the
// block's last node is written by agent-scope stores (write-through to the chip's coherence point), so
// another workgroup can read it in the same launch.
__device__ __forceinline__ void tail_levels(uint32_t* msg, uint64_t base, uint32_t here, uint32_t extra,
                                            const LevelPtrs& out, bool coherent) {
  const uint32_t node = threadIdx.x >> 2, q = threadIdx.x & 3;
  uint32_t width = here;
  for (uint32_t k = 0; k <= extra; ++k) {
    const bool active = node < width;
    uint32_t lo = 0, hi = 0;
    if (active) hash_pair_quad(msg + node * 16, q, lo, hi);
    __syncthreads();
    if (active) {
      msg[node * 8 + q] = lo;
      msg[node * 8 + 4 + q] = hi;
      uint32_t* g = reinterpret_cast<uint32_t*>(out.lv[k] + (base >> k) + node);
      if (coherent && k == extra) {
        __hip_atomic_store(g + q, lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(g + 4 + q, hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        g[q] = lo;
        g[4 + q] = hi;
      }
    }
    __syncthreads();
    width >>= 1;
  }
}

// Pair mode only: input level (count nodes) from `below`, then `extra` more levels in LDS; same LevelPtrs
// convention as merkle_build_kernel.  extra2 > 0 (grid > 1): the launch also does the next launch's work,
// i.e. the levels above its workgroups' top nodes (gridDim.x / 2 nodes, then extra2 - 1 more levels, into
// out2), in the workgroup that finishes last.  Each workgroup publishes its top node with agent-scope
// stores, waits for them, and counts itself in *done (agent scope); the workgroup that counts last reads
// the gridDim.x top nodes with agent-scope loads and resets *done for the tree's next build.  (No release
// fence: it would write back the XCD's whole L2, and only these nodes are read in this launch.)
// The root as a field element (RootFe, internal.h): its LE words reduced mod p, times r2, from the root in
// msg[0..7] (the workgroup's last level, node 0).
__device__ __forceinline__ void root_fe_out(const uint32_t* msg, const RootFe& rf) {
  fe x;
#pragma unroll
  for (int i = 0; i < 8; ++i) x.w[i] = msg[i];
  if (rf.copy) {
#pragma unroll
    for (int i = 0; i < 8; ++i) rf.copy[i] = x.w[i];
  }
  if (rf.out) {
#pragma unroll
    for (int k = 0; k < 5; ++k) fe_reduce_once(x);  // x < 2^256 < 6p
    *rf.out = fe_mul(x, rf.r2);
  }
}

// rf.made: this launch reaches the root (one workgroup, or the fused top), which the workgroup that made it
// also writes out as a field element (the FRI fold's special_x, fri.rs:135) and / or copies (RootFe).
__global__ __launch_bounds__(kTailThreads) void merkle_tail_kernel(const Digest* __restrict__ below, uint64_t count,
                                                                   uint32_t extra, LevelPtrs out, uint32_t extra2,
                                                                   LevelPtrs out2, uint32_t* done, RootFe rf) {
  __shared__ __attribute__((aligned(16))) uint32_t msg[2 * kTailBlock * 8];
  __shared__ uint32_t last;
  const uint64_t base = (uint64_t)blockIdx.x * kTailBlock;
  const uint32_t here = (uint32_t)((count - base) < kTailBlock ? (count - base) : kTailBlock);
  const uint4* src = reinterpret_cast<const uint4*>(below + 2 * base);
  for (uint32_t i = threadIdx.x; i < here * 4; i += blockDim.x) reinterpret_cast<uint4*>(msg)[i] = src[i];
  __syncthreads();
  tail_levels(msg, base, here, extra, out, extra2 > 0);
  if (extra2 == 0) {  // (uniform)
    if (rf.made && gridDim.x == 1 && threadIdx.x == 0) root_fe_out(msg, rf);
    return;
  }
  if (threadIdx.x < 4) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the top node's stores have landed
  __syncthreads();
  if (threadIdx.x == 0)
    last = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  if (!last) return;  // (uniform)
  const uint32_t n_top = gridDim.x;  // one top node per workgroup, at out.lv[extra]
  const uint32_t* top = reinterpret_cast<const uint32_t*>(out.lv[extra]);
  for (uint32_t i = threadIdx.x; i < n_top * 8; i += blockDim.x)
    msg[i] = __hip_atomic_load(top + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x == 0) __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  tail_levels(msg, 0, n_top / 2, extra2 - 1, out2, false);
  if (rf.made && threadIdx.x == 0) root_fe_out(msg, rf);
}

// Proof gather: for proof i (index idx[i]): the leaf bytes and the depth
// siblings ((idx >> d) ^ 1 at level d), leaf -> root.
// Byte b of leaf id: contiguous leaves, or 32-B planes plane_stride apart (merkle_build).
__device__ __forceinline__ const uint8_t* leaf_byte(const uint8_t* leaves, uint64_t id, uint32_t leaf_len,
                                                    uint64_t plane_stride, uint32_t b) {
  return plane_stride ? leaves + (b >> 5) * plane_stride + 32 * id + (b & 31) : leaves + id * leaf_len + b;
}

__global__ void merkle_gather_kernel(const uint8_t* __restrict__ leaves, uint32_t leaf_len, uint64_t plane_stride,
                                     const Digest* __restrict__ nodes, uint64_t n, uint32_t depth,
                                     const uint64_t* __restrict__ idx, uint32_t k, uint8_t* __restrict__ leaf_out,
                                     Digest* __restrict__ node_out) {
  const uint32_t i = blockIdx.x;
  if (i >= k) return;
  const uint64_t id = idx[i];
  for (uint32_t b = threadIdx.x; b < leaf_len; b += blockDim.x)
    leaf_out[(uint64_t)i * leaf_len + b] = *leaf_byte(leaves, id, leaf_len, plane_stride, b);
  uint64_t off = 0, width = n;
  for (uint32_t d = 0; d < depth; ++d) {
    if (threadIdx.x == d % blockDim.x) node_out[(uint64_t)i * depth + d] = nodes[off + ((id >> d) ^ 1)];
    off += width;
    width >>= 1;
  }
}

static uint64_t level_offset(uint64_t n, uint32_t level) {
  uint64_t off = 0, w = n;
  for (uint32_t l = 0; l < level; ++l) {
    off += w;
    w >>= 1;
  }
  return off;
}

// Leaf digests only: out[i] = Blake2s(leaf i) (the level-0 nodes of a tree
// whose parents another GPU may build, distributed prover).
__global__ void merkle_leaf_digest_kernel(const uint8_t* __restrict__ leaves, uint32_t leaf_len, uint64_t n,
                                          Digest* __restrict__ out) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const bool l32 = leaf_len == 32 && (((uintptr_t)leaves) & 15) == 0;
  store_digest(out + i, l32 ? hash_leaf32(leaves + i * 32) : hash_leaf(leaves + i * leaf_len, leaf_len));
}

// level0[G m + r] = chunks[r][m]: the digests of G ranks' residue classes,
// received as G contiguous chunks of n/G (one per sender), in leaf order.
__global__ void merkle_interleave_kernel(const Digest* __restrict__ chunks, uint64_t n, uint32_t log_g,
                                         Digest* __restrict__ level0) {
  const uint64_t o = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= n) return;
  const uint64_t r = o & ((1u << log_g) - 1), m = o >> log_g;
  store_digest(level0 + o, load_digest(chunks + r * (n >> log_g) + m));
}

// The top of a tree split into g subtrees (merkle_proof_in_place.rs:176-180): the g subtree roots
// hashed pairwise level by level in LDS by one workgroup; out = the g - 1 digests above them, level
// by level (the root last).
constexpr uint32_t kTopMax = 1024;
__global__ __launch_bounds__(kTopMax / 2) void merkle_top_kernel(const Digest* __restrict__ roots, uint32_t g,
                                                                 Digest* __restrict__ out) {
  __shared__ Digest lv[kTopMax];
  const uint32_t t = threadIdx.x;
  for (uint32_t i = t; i < g; i += blockDim.x) lv[i] = load_digest(roots + i);
  __syncthreads();
  uint32_t off = 0;
  for (uint32_t w = g >> 1; w >= 1; w >>= 1) {
    Digest d;
    if (t < w) d = hash_pair(lv[2 * t], lv[2 * t + 1]);
    __syncthreads();
    if (t < w) {
      lv[t] = d;
      store_digest(out + off + t, d);
    }
    __syncthreads();
    off += w;
  }
}

// The node buffer holds the 2n - 1 digests and, in its last 32 bytes, the fused tail's workgroup counter
// (merkle_tail_kernel), zeroed when the buffer is allocated and reset by every launch that uses it.
static uint32_t* tail_counter(stark_merkle_tree* t) {
  return reinterpret_cast<uint32_t*>((uint8_t*)t->nodes.ptr + t->nodes.bytes - 32);
}
static stark_status ensure_nodes(stark_ctx* ctx, stark_merkle_tree* t, size_t n, hipStream_t stream) {
  const void* before = t->nodes.ptr;
  const size_t before_bytes = t->nodes.bytes;
  STARK_TRY(ensure_buf(ctx, t->nodes, (2 * n - 1) * sizeof(Digest) + 32));
  // (a reallocation can return the old address, so the size tells it too)
  if (t->nodes.ptr != before || t->nodes.bytes != before_bytes)
    STARK_HIP(ctx, hipMemsetAsync(tail_counter(t), 0, 32, stream));
  return STARK_OK;
}

// Level 0 of the tree over n leaves (the leaf digests, 8 words each), for a kernel that hashes the leaves as
// it makes them (the constraint kernel: the main tree's rows); merkle_build(..., level0_ready) then builds the
// levels above.
stark_status merkle_level0(stark_ctx* ctx, stark_merkle_tree* t, size_t n, hipStream_t stream, uint32_t** level0) {
  if (n == 0 || (n & (n - 1)) != 0) return STARK_ERR_BAD_LENGTH;
  STARK_TRY(ensure_nodes(ctx, t, n, stream));
  *level0 = reinterpret_cast<uint32_t*>(t->nodes.ptr);  // (level_offset(n, 0) = 0)
  return STARK_OK;
}

// Builds every level of the tree over d_leaves (n leaves of leaf_len bytes);
// with d_leaves == nullptr or level0_ready level 0 (the leaf digests) is already in place (with
// level0_ready the proofs still open d_leaves).
// plane_stride != 0: leaf i's bytes [32 c, 32 c + 32) are at d_leaves + c * plane_stride + 32 i
// (leaf_len a multiple of 32, 16-B aligned planes).
stark_status merkle_build(stark_ctx* ctx, stark_merkle_tree* t, const uint8_t* d_leaves, size_t n, size_t leaf_len,
                          hipStream_t stream, size_t plane_stride, bool level0_ready, RootFe* root_fe) {
  // (root_fe: made by the tail launch that makes the root; root_fe->made false where no tail launch does,
  // and the caller makes it itself)
  const RootFe rf_none{};
  if (root_fe) root_fe->made = false;
  if (n == 0 || (n & (n - 1)) != 0) return STARK_ERR_BAD_LENGTH;
  if (leaf_len > 0xFFFFFFFFull) return STARK_ERR_BAD_ARG;
  if (plane_stride && (!d_leaves || leaf_len == 0 || leaf_len % 32 || plane_stride % 16 || plane_stride < 32 * n ||
                       (((uintptr_t)d_leaves) & 15)))
    return STARK_ERR_BAD_ARG;
  uint32_t depth = 0;
  while (((size_t)1 << depth) < n) ++depth;
  stark_status st = ensure_nodes(ctx, t, n, stream);
  if (st != STARK_OK) return st;
  Digest* nodes = (Digest*)t->nodes.ptr;
  uint32_t* done = tail_counter(t);
  const bool have_level0 = d_leaves == nullptr || level0_ready;
  uint32_t level = have_level0 ? 1 : 0;
  uint64_t count = have_level0 ? n / 2 : n;
  bool leaf_mode = !have_level0;
  while (depth > 0 || !have_level0) {
    if (!leaf_mode && count < kTailFrom) {
      // Narrow pair levels: quad kernel, up to 8 levels per launch; with more than one workgroup, the
      // levels above the workgroups' top nodes (the next launch's) run in the last workgroup to finish.
      const uint64_t blk = count < kTailBlock ? count : kTailBlock;
      uint32_t extra = 0;
      while ((blk >> (extra + 1)) >= 1 && level + extra + 1 <= depth) ++extra;
      LevelPtrs lp;
      for (uint32_t k = 0; k <= extra; ++k) lp.lv[k] = nodes + level_offset(n, level + k);
      const unsigned grid = (unsigned)((count + kTailBlock - 1) / kTailBlock);
      uint32_t extra2 = 0;
      LevelPtrs lp2{};
      const bool fuse = grid > 1 && (count >> extra) == grid && level + extra < depth;
      if (fuse) {  // the next launch: count2 = grid / 2 nodes at level + extra + 1 (grid <= kTailBlock)
        const uint32_t level2 = level + extra + 1;
        const uint64_t blk2 = grid / 2;
        while ((blk2 >> (extra2 + 1)) >= 1 && level2 + extra2 + 1 <= depth) ++extra2;
        for (uint32_t k = 0; k <= extra2; ++k) lp2.lv[k] = nodes + level_offset(n, level2 + k);
      }
      const bool to_root = fuse ? level + extra + 1 + extra2 == depth : (grid == 1 && level + extra == depth);
      RootFe rf = rf_none;
      if (root_fe && to_root) {
        root_fe->made = true;
        rf = *root_fe;
      }
      hipLaunchKernelGGL(merkle_tail_kernel, dim3(grid), dim3(kTailThreads), 0, stream,
                         (const Digest*)(nodes + level_offset(n, level - 1)), count, extra, lp,
                         fuse ? extra2 + 1 : 0u, lp2, done, rf);
      STARK_HIP(ctx, hipGetLastError());
      level += extra;
      count >>= extra;
      if (fuse) {
        ++level;
        count >>= 1;
        level += extra2;
        count >>= extra2;
      }
    } else {
      // Wide levels: one lane per node, blocks of 1024 nodes reduced by 2
      // more levels in LDS (1024 -> 512 -> 256, one node per thread).  A
      // narrow leaf level is hashed alone, one node per thread.
      const bool narrow_leaf = count < kTailFrom;
      const uint32_t block = narrow_leaf ? kMerkleThreads : kMerkleBlock;
      const uint64_t blk = count < block ? count : block;
      const uint32_t max_extra = narrow_leaf ? 0 : 2;
      uint32_t extra = 0;
      while ((blk >> (extra + 1)) >= 1 && extra + 1 <= max_extra && level + extra + 1 <= depth) ++extra;
      LevelPtrs lp;
      for (uint32_t k = 0; k <= extra; ++k) lp.lv[k] = nodes + level_offset(n, level + k);
      const unsigned grid = (unsigned)((count + block - 1) / block);
      const Digest* below = leaf_mode ? nullptr : nodes + level_offset(n, level - 1);
      const bool leaf32 = leaf_mode && leaf_len == 32 && (((uintptr_t)d_leaves) & 15) == 0;
      hipLaunchKernelGGL(leaf32 ? merkle_build_kernel<true> : merkle_build_kernel<false>, dim3(grid),
                         dim3(kMerkleThreads), 0, stream, leaf_mode ? d_leaves : nullptr, (uint32_t)leaf_len, below,
                         count, block, extra, lp, (uint64_t)plane_stride);
      STARK_HIP(ctx, hipGetLastError());
      level += extra;
      count >>= extra;
    }
    if (level == depth) break;
    // Next launch starts by hashing pairs of the current top level.
    ++level;
    count >>= 1;
    leaf_mode = false;
  }
  t->n = n;
  t->leaf_len = leaf_len;
  t->depth = depth;
  t->d_leaves = d_leaves ? d_leaves : (const uint8_t*)nodes;
  t->plane_stride = d_leaves ? plane_stride : 0;
  t->built = true;
  return STARK_OK;
}

size_t merkle_device_bytes(const stark_merkle_tree* t) {
  if (!t) return 0;
  size_t b = 0;
  for (const DevBuf* d : {&t->nodes, &t->own_leaves, &t->gather}) b += d->ptr ? d->bytes : 0;
  return b;
}

// Device address of the root digest (valid after merkle_build).
const uint8_t* merkle_root_dev(const stark_merkle_tree* t) {
  return (const uint8_t*)t->nodes.ptr + (2 * t->n - 2) * sizeof(Digest);
}

stark_status merkle_root_d2h(stark_ctx* ctx, stark_merkle_tree* t, hipStream_t stream, uint8_t out[32]) {
  const Digest* nodes = (const Digest*)t->nodes.ptr;
  STARK_HIP(ctx, hipMemcpyAsync(out, nodes + (2 * t->n - 2), 32, hipMemcpyDeviceToHost, stream));
  STARK_HIP(ctx, hipStreamSynchronize(stream));
  return STARK_OK;
}

// Gathers k proofs (leaf bytes + siblings) to host buffers.  sync = false
// leaves the copies in flight: `indices` and the outputs must stay alive until
// the caller synchronises the stream.
stark_status merkle_gather(stark_ctx* ctx, stark_merkle_tree* t, const size_t* indices, size_t k,
                           uint8_t* leaves_out, uint8_t* nodes_out, hipStream_t stream, bool sync) {
  if (k == 0) return STARK_OK;
  for (size_t i = 0; i < k; ++i)
    if (indices[i] >= t->n) return STARK_ERR_BAD_ARG;
  const size_t idx_bytes = k * sizeof(uint64_t);
  const size_t leaf_bytes = k * t->leaf_len;
  const size_t node_bytes = k * t->depth * sizeof(Digest);
  const size_t total = idx_bytes + ((leaf_bytes + 15) & ~(size_t)15) + node_bytes;
  stark_status st = ensure_buf(ctx, t->gather, total);
  if (st != STARK_OK) return st;
  uint8_t* base = (uint8_t*)t->gather.ptr;
  uint64_t* d_idx = (uint64_t*)base;
  uint8_t* d_leaf = base + idx_bytes;
  Digest* d_node = (Digest*)(base + idx_bytes + ((leaf_bytes + 15) & ~(size_t)15));
  static_assert(sizeof(size_t) == sizeof(uint64_t), "size_t indices are uploaded as u64");
  STARK_HIP(ctx, hipMemcpyAsync(d_idx, indices, idx_bytes, hipMemcpyHostToDevice, stream));
  hipLaunchKernelGGL(merkle_gather_kernel, dim3((unsigned)k), dim3(64), 0, stream, t->d_leaves,
                     (uint32_t)t->leaf_len, (uint64_t)t->plane_stride, (const Digest*)t->nodes.ptr, (uint64_t)t->n, t->depth, d_idx,
                     (uint32_t)k, d_leaf, d_node);
  STARK_HIP(ctx, hipGetLastError());
  if (leaves_out) STARK_HIP(ctx, hipMemcpyAsync(leaves_out, d_leaf, leaf_bytes, hipMemcpyDeviceToHost, stream));
  if (nodes_out && node_bytes)
    STARK_HIP(ctx, hipMemcpyAsync(nodes_out, d_node, node_bytes, hipMemcpyDeviceToHost, stream));
  if (sync) STARK_HIP(ctx, hipStreamSynchronize(stream));
  return STARK_OK;
}

// Many gathers in one launch, zero-copy: the kernel reads the indices from
// and writes every request's leaves and siblings straight into the context's
// pinned (coherent) host scratch, so the whole opening phase is one launch
// and one synchronisation (per-request launches and a separate D2H copy cost
// ~7 us and ~70 us of engine latency each).
constexpr uint32_t kGatherMaxReq = 64;  // requests per launch (descriptors travel as kernel arguments)

struct GatherDesc {
  const uint8_t* leaves;
  const Digest* nodes;
  uint64_t n;        // leaves
  uint64_t out_off;  // byte offset of this request's region in the output
  uint64_t plane_stride;
  uint32_t first;    // first proof (block) of this request
  uint32_t k, leaf_len, depth;
};
struct GatherDescs {
  GatherDesc d[kGatherMaxReq];
};

// Block p = one proof: leaf bytes then the depth siblings ((idx >> d) ^ 1 at
// level d, leaf -> root).  Region layout per request: k leaves (padded to 16
// bytes), then k * depth digests.
__global__ __launch_bounds__(64) void merkle_gather_multi_kernel(GatherDescs g, uint32_t n_req,
                                                                  const uint64_t* __restrict__ idx,
                                                                  uint8_t* __restrict__ out,
                                                                  uint32_t* __restrict__ err) {
  const uint32_t p = blockIdx.x;
  uint32_t r = 0;
  while (r + 1 < n_req && g.d[r + 1].first <= p) ++r;
  const GatherDesc& q = g.d[r];
  const uint32_t i = p - q.first;
  const uint64_t id = idx[p];
  if (id >= q.n) {  // an index written on the device (fri_indices_kernel) out of range: no read, flagged
    if (threadIdx.x == 0) *err = 1u;
    return;
  }
  uint8_t* region = out + q.out_off;
  uint8_t* leaf_out = region + (uint64_t)i * q.leaf_len;
  const uint8_t* leaf_in = q.leaves + id * q.leaf_len;
  if (q.plane_stride) {  // 32-B planes (4-B aligned: leaf_len and the planes are multiples of 16)
    for (uint32_t w = threadIdx.x; w < q.leaf_len / 4; w += blockDim.x)
      reinterpret_cast<uint32_t*>(leaf_out)[w] =
          *reinterpret_cast<const uint32_t*>(leaf_byte(q.leaves, id, q.leaf_len, q.plane_stride, 4 * w));
  } else if ((q.leaf_len & 3) == 0 && (((uintptr_t)leaf_in | (uintptr_t)leaf_out) & 3) == 0) {
    for (uint32_t w = threadIdx.x; w < q.leaf_len / 4; w += blockDim.x)
      reinterpret_cast<uint32_t*>(leaf_out)[w] = reinterpret_cast<const uint32_t*>(leaf_in)[w];
  } else {
    for (uint32_t b = threadIdx.x; b < q.leaf_len; b += blockDim.x) leaf_out[b] = leaf_in[b];
  }
  Digest* node_out = reinterpret_cast<Digest*>(region + ((q.k * (uint64_t)q.leaf_len + 15) & ~(uint64_t)15)) +
                     (uint64_t)i * q.depth;
  for (uint32_t d = threadIdx.x; d < q.depth; d += blockDim.x) {
    const uint64_t off = 2 * q.n - 2 * (q.n >> d);  // first node of level d (n a power of two)
    const uint4* src = reinterpret_cast<const uint4*>(q.nodes + off + ((id >> d) ^ 1));
    uint4* dst = reinterpret_cast<uint4*>(node_out + d);
    dst[0] = src[0];
    dst[1] = src[1];
  }
}

stark_status merkle_gather_batch(stark_ctx* ctx, const std::vector<GatherReq>& reqs, hipStream_t stream,
                                 const GatherHook& before_launch) {
  size_t n_idx = 0, out_bytes = 0;
  std::vector<size_t> off(reqs.size()), first(reqs.size());
  for (size_t r = 0; r < reqs.size(); ++r) {
    const GatherReq& q = reqs[r];
    if (!q.idx && q.k && !before_launch) return STARK_ERR_BAD_ARG;
    if (q.idx)
      for (size_t i = 0; i < q.k; ++i)
        if (q.idx[i] >= q.t->n) return STARK_ERR_BAD_ARG;
    first[r] = n_idx;
    n_idx += q.k;
    off[r] = out_bytes;
    out_bytes += ((q.k * q.t->leaf_len + 15) & ~(size_t)15) + q.k * q.t->depth * sizeof(Digest);
  }
  if (n_idx == 0) return STARK_OK;
  if (n_idx > 0xFFFFFFFFull) return STARK_ERR_BAD_ARG;
  const size_t idx_bytes = n_idx * sizeof(uint64_t);
  uint8_t* host = nullptr;
  stark_status st = ctx_pinned(ctx, 0, idx_bytes + out_bytes + 16, (void**)&host);
  if (st != STARK_OK) return st;
  uint64_t* h_idx = (uint64_t*)host;
  uint8_t* h_out = host + idx_bytes;
  uint32_t* h_err = (uint32_t*)(h_out + out_bytes);  // (out_bytes is a multiple of 16)
  *h_err = 0;
  for (size_t r = 0; r < reqs.size(); ++r)
    if (reqs[r].idx)
      for (size_t i = 0; i < reqs[r].k; ++i) h_idx[first[r] + i] = reqs[r].idx[i];
  if (before_launch) STARK_TRY(before_launch(h_idx, first));
  // Launches of up to kGatherMaxReq requests; proofs are numbered across the batch.
  size_t r0 = 0, p0 = 0;
  while (r0 < reqs.size()) {
    GatherDescs g;
    uint32_t m = 0, proofs = 0;
    size_t r = r0;
    for (; r < reqs.size() && m < kGatherMaxReq; ++r) {
      const GatherReq& q = reqs[r];
      if (q.k == 0) continue;
      GatherDesc& d = g.d[m++];
      d.leaves = q.t->d_leaves;
      d.nodes = (const Digest*)q.t->nodes.ptr;
      d.n = q.t->n;
      d.out_off = off[r];
      d.plane_stride = q.t->plane_stride;
      d.first = proofs;
      d.k = (uint32_t)q.k;
      d.leaf_len = (uint32_t)q.t->leaf_len;
      d.depth = q.t->depth;
      proofs += (uint32_t)q.k;
    }
    if (m) {
      hipLaunchKernelGGL(merkle_gather_multi_kernel, dim3(proofs), dim3(64), 0, stream, g, m,
                         (const uint64_t*)(h_idx + p0), h_out, h_err);
      STARK_HIP(ctx, hipGetLastError());
    }
    p0 += proofs;
    r0 = r;
  }
  STARK_HIP(ctx, hipStreamSynchronize(stream));
  if (*(volatile uint32_t*)h_err) {
    ctx->last_error = "gather index out of range (device-written indices)";
    return STARK_ERR_BAD_ARG;
  }
  for (size_t r = 0; r < reqs.size(); ++r) {
    const GatherReq& q = reqs[r];
    const uint8_t* leaf = h_out + off[r];
    const uint8_t* node = leaf + ((q.k * q.t->leaf_len + 15) & ~(size_t)15);
    if (q.leaves_out) memcpy(q.leaves_out, leaf, q.k * q.t->leaf_len);
    if (q.nodes_out) memcpy(q.nodes_out, node, q.k * q.t->depth * sizeof(Digest));
  }
  return STARK_OK;
}

}  // namespace stark

using namespace stark;

extern "C" {

stark_status stark_merkle_new(stark_ctx* ctx, stark_merkle_tree** out) {
  if (!ctx || !out) return STARK_ERR_BAD_ARG;
  stark_merkle_tree* t = new (std::nothrow) stark_merkle_tree();
  if (!t) return STARK_ERR_OOM;
  t->ctx = ctx;
  *out = t;
  return STARK_OK;
}

void stark_merkle_free(stark_merkle_tree* t) {
  if (!t) return;
  hipSetDevice(t->ctx->device);
  if (t->nodes.ptr) hipFree(t->nodes.ptr);
  if (t->own_leaves.ptr) hipFree(t->own_leaves.ptr);
  if (t->gather.ptr) hipFree(t->gather.ptr);
  delete t;
}

stark_status stark_merkle_update(stark_merkle_tree* t, const uint8_t* leaves, size_t n, size_t leaf_len) {
  if (!t || (!leaves && n * leaf_len)) return STARK_ERR_BAD_ARG;
  if (n == 0 || (n & (n - 1))) return STARK_ERR_BAD_LENGTH;
  stark_ctx* ctx = t->ctx;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  stark_status st = ensure_buf(ctx, t->own_leaves, n * leaf_len ? n * leaf_len : 16);
  if (st != STARK_OK) return st;
  if (n * leaf_len)
    STARK_HIP(ctx, hipMemcpyAsync(t->own_leaves.ptr, leaves, n * leaf_len, hipMemcpyHostToDevice, ctx->stream));
  st = merkle_build(ctx, t, (const uint8_t*)t->own_leaves.ptr, n, leaf_len, ctx->stream);
  if (st != STARK_OK) return st;
  STARK_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return STARK_OK;
}

stark_status stark_merkle_update_dev(stark_merkle_tree* t, const uint8_t* d_leaves, size_t n, size_t leaf_len,
                                     void* stream) {
  if (!t || (!d_leaves && n * leaf_len)) return STARK_ERR_BAD_ARG;
  stark_ctx* ctx = t->ctx;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  return merkle_build(ctx, t, d_leaves, n, leaf_len, pick_stream(ctx, stream));
}

stark_status stark_merkle_leaf_digests_dev(stark_ctx* ctx, const uint8_t* d_leaves, size_t n, size_t leaf_len,
                                           uint8_t* d_digests, void* stream) {
  if (!ctx || (n && (!d_leaves || !d_digests)) || leaf_len > 0xFFFFFFFFull) return STARK_ERR_BAD_ARG;
  if (n == 0) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  hipLaunchKernelGGL(merkle_leaf_digest_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                     pick_stream(ctx, stream), d_leaves, (uint32_t)leaf_len, (uint64_t)n, (Digest*)d_digests);
  STARK_HIP(ctx, hipGetLastError());
  return STARK_OK;
}

stark_status stark_merkle_update_digests_dev(stark_merkle_tree* t, const uint8_t* d_digests, size_t n,
                                            uint32_t interleave, void* stream) {
  if (!t || !d_digests || interleave == 0 || (interleave & (interleave - 1))) return STARK_ERR_BAD_ARG;
  if (n == 0 || (n & (n - 1)) || n % interleave) return STARK_ERR_BAD_LENGTH;
  stark_ctx* ctx = t->ctx;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  hipStream_t s = pick_stream(ctx, stream);
  stark_status st = ensure_nodes(ctx, t, n, s);
  if (st != STARK_OK) return st;
  uint32_t log_g = 0;
  while ((1u << log_g) < interleave) ++log_g;
  hipLaunchKernelGGL(merkle_interleave_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s,
                     (const Digest*)d_digests, (uint64_t)n, log_g, (Digest*)t->nodes.ptr);
  STARK_HIP(ctx, hipGetLastError());
  return merkle_build(ctx, t, nullptr, n, 32, s);
}

stark_status stark_merkle_root_dev(const stark_merkle_tree* t, uint8_t* d_out, void* stream) {
  if (!t || !d_out) return STARK_ERR_BAD_ARG;
  if (!t->built) return STARK_ERR_STATE;
  stark_ctx* ctx = t->ctx;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  STARK_HIP(ctx, hipMemcpyAsync(d_out, merkle_root_dev(t), 32, hipMemcpyDeviceToDevice, pick_stream(ctx, stream)));
  return STARK_OK;
}

stark_status stark_merkle_top_dev(stark_ctx* ctx, const uint8_t* d_roots, size_t g, uint8_t* d_levels, void* stream) {
  if (!ctx || (g > 1 && (!d_roots || !d_levels))) return STARK_ERR_BAD_ARG;
  if (g == 0 || (g & (g - 1)) || g > kTopMax) return STARK_ERR_BAD_LENGTH;
  if ((((uintptr_t)d_roots) | ((uintptr_t)d_levels)) & 15) return STARK_ERR_BAD_ARG;  // 16-B digest loads
  if (g == 1) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  hipLaunchKernelGGL(merkle_top_kernel, dim3(1), dim3((unsigned)(g / 2)), 0, pick_stream(ctx, stream),
                     (const Digest*)d_roots, (uint32_t)g, (Digest*)d_levels);
  STARK_HIP(ctx, hipGetLastError());
  return STARK_OK;
}

// Every opening of a distributed proof on this rank in one zero-copy gather launch:
// request i reads paths (and leaf digests) from reqs[i].tree, or, with tree == NULL,
// leaf bytes from a row buffer.
stark_status stark_open_batch(stark_ctx* ctx, const stark_open_req* reqs, size_t n_req, void* stream) {
  if (!ctx || (n_req && !reqs)) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  std::vector<stark_merkle_tree> views(n_req);  // row buffers seen as depth-0 trees
  std::vector<GatherReq> g;
  for (size_t i = 0; i < n_req; ++i) {
    const stark_open_req& q = reqs[i];
    if (q.k && (!q.idx || (!q.leaves_out && !q.nodes_out))) return STARK_ERR_BAD_ARG;
    stark_merkle_tree* t = q.tree;
    if (!t) {
      if (!q.d_rows || q.row_bytes > 0xFFFFFFFFull) return STARK_ERR_BAD_ARG;
      stark_merkle_tree& v = views[i];
      v.ctx = ctx;
      v.n = q.n_rows;
      v.leaf_len = q.row_bytes;
      v.depth = 0;
      v.d_leaves = q.d_rows;
      v.built = true;
      t = &v;
    } else if (!t->built) {
      return STARK_ERR_STATE;
    }
    g.push_back({t, q.idx, q.k, q.leaves_out, q.nodes_out});
  }
  return merkle_gather_batch(ctx, g, pick_stream(ctx, stream));
}

size_t stark_merkle_width(const stark_merkle_tree* t) { return t ? t->n : 0; }
size_t stark_merkle_leaf_len(const stark_merkle_tree* t) { return t ? t->leaf_len : 0; }

stark_status stark_merkle_get_root(const stark_merkle_tree* t, uint8_t root[32], size_t* root_len) {
  if (!t || !root_len) return STARK_ERR_BAD_ARG;
  if (!t->has_root) {
    *root_len = 0;
    return STARK_OK;
  }
  if (root) memcpy(root, t->root, 32);
  *root_len = 32;
  return STARK_OK;
}

stark_status stark_merkle_gen_proofs(stark_merkle_tree* t, const size_t* indices, size_t k, uint8_t* leaves_out,
                                     uint8_t* nodes_out) {
  if (!t || (k && !indices)) return STARK_ERR_BAD_ARG;
  if (!t->built) return STARK_ERR_STATE;
  stark_ctx* ctx = t->ctx;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  stark_status st = merkle_root_d2h(ctx, t, ctx->stream, t->root);
  if (st != STARK_OK) return st;
  t->has_root = true;
  return merkle_gather(ctx, t, indices, k, leaves_out, nodes_out, ctx->stream, true);
}

stark_status stark_merkle_verify(const uint8_t root[32], const size_t* indices, size_t k, const uint8_t* leaves,
                                 size_t leaf_len, const uint8_t* nodes, size_t depth) {
  if (!root || (k && (!indices || !leaves || (depth && !nodes)))) return STARK_ERR_BAD_ARG;
  for (size_t i = 0; i < k; ++i) {
    uint8_t cur[32], msg[64];
    b2s_host(leaves + i * leaf_len, leaf_len, cur);
    size_t pos = indices[i];
    for (size_t d = 0; d < depth; ++d) {
      const uint8_t* sib = nodes + (i * depth + d) * 32;
      if (pos % 2 == 0) {
        memcpy(msg, cur, 32);
        memcpy(msg + 32, sib, 32);
      } else {
        memcpy(msg, sib, 32);
        memcpy(msg + 32, cur, 32);
      }
      b2s_host(msg, 64, cur);
      pos /= 2;
    }
    if (memcmp(cur, root, 32) != 0) return STARK_ERR_BAD_ARG;
  }
  return STARK_OK;
}

}  // extern "C"
