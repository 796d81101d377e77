// FRI prover (prove_low_degree, packages/fri/src/fri.rs:46-224) on gfx950.
//
// Per layer, everything large stays in HBM: the Merkle tree of the layer's
// values, the 4->1 fold, the Merkle tree of the folded column and the
// proof-path gathers.  The host only runs the transcript (root -> special_x,
// Blake2s index sampling) and assembles the proof.
//
// Fold (fri.rs:141-164 with multi_interp_4 poly_utils.rs:449-511 and
// eval_quartic :442-446): row i interpolates the cubic through
// (w^(i + j n/4), v[i + j n/4]), j = 0..3, and evaluates it at special_x.
// The four x's are x0 * zeta^j with zeta = w^(n/4) (zeta^2 = -1), so with
// u = special_x / x0 the cubic's value is sum_k d_k u^k where d = the inverse
// 4-point DFT of the y's:
//   d0 = (y0+y1+y2+y3)/4         d2 = (y0-y1+y2-y3)/4
//   d1 = ((y0-y2) - zeta(y1-y3))/4  d3 = ((y0-y2) + zeta(y1-y3))/4
// It is the same unique cubic, so the column is bit-identical to the
// reference's, with 7 modular products per row and no batch inverse.
#include <string.h>

#include <algorithm>
#include <iterator>
#include <array>
#include <string>

#include <atomic>
#include <thread>

#include "internal.h"
#include "blake2s.h"
#include "host_json.h"
#include "merkle_dev.h"


namespace stark {

// special_x = T::from_bytes_le(m_root) (fri.rs:135) computed on the device from
// the tree's root digest (LE bytes = LE words), reduced mod p, as a Montgomery
// image for the fold.  The transcript never leaves the GPU between layers.
__global__ void fri_special_x_kernel(const uint32_t* __restrict__ root, fe* __restrict__ s_m, fe r2) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  fe x;
#pragma unroll
  for (int i = 0; i < 8; ++i) x.w[i] = root[i];
#pragma unroll
  for (int k = 0; k < 5; ++k) fe_reduce_once(x);  // x < 2^256 < 6p
  *s_m = fe_mul(x, r2);
}

// Row i of q (local rows; global row g_add + (i << log_g) on a distributed
// prover whose values are the residue class g_add mod 2^log_g, where the four
// points of a row are local too since n/4 is a multiple of 2^log_g).
__device__ __forceinline__ fe fri_fold_row(const fe* __restrict__ v, fe* __restrict__ col, uint64_t i, uint64_t q,
                                             uint32_t shift, uint64_t g_add, uint32_t log_g,
                                             const fe* __restrict__ lo, const fe* __restrict__ hi, uint32_t kb,
                                             const fe& s_m, const fe& zeta_m, const fe& inv4_m) {
  const fe y0 = fe_load(v + i), y1 = fe_load(v + i + q), y2 = fe_load(v + i + 2 * q), y3 = fe_load(v + i + 3 * q);
  const uint64_t e = (g_add + (i << log_g)) << shift;
  const fe winv = fe_mul(lo[e & (((uint64_t)1 << kb) - 1)], hi[e >> kb]);  // Montgomery w^-i
  const fe u_m = fe_mul(s_m, winv);                                         // Montgomery special_x * w^-i
  const fe s02 = fe_add(y0, y2), s13 = fe_add(y1, y3);
  const fe e02 = fe_sub(y0, y2);
  const fe z = fe_mul(fe_sub(y1, y3), zeta_m);
  const fe d0 = fe_add(s02, s13), d2 = fe_sub(s02, s13);
  const fe d1 = fe_sub(e02, z), d3 = fe_add(e02, z);
  fe acc = fe_add(fe_mul(d3, u_m), d2);
  acc = fe_add(fe_mul(acc, u_m), d1);
  acc = fe_add(fe_mul(acc, u_m), d0);
  const fe out = fe_mul(acc, inv4_m);
  fe_store(col + i, out);
  return out;
}

// leaf non-null: each output's Blake2s too (the next layer tree's level 0, merkle_level0), 8 words.
__global__ void fri_fold_kernel(const fe* __restrict__ v, fe* __restrict__ col, uint64_t q, uint32_t shift,
                                uint64_t g_add, uint32_t log_g,
                                const fe* __restrict__ lo, const fe* __restrict__ hi, uint32_t kb,
                                const fe* __restrict__ s_ptr, fe zeta_m, fe inv4_m, uint32_t* __restrict__ leaf) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= q) return;
  const fe x = fri_fold_row(v, col, i, q, shift, g_add, log_g, lo, hi, kb, *s_ptr, zeta_m, inv4_m);
  if (leaf) {  // (uniform)
    uint32_t h[8], m[16];
    b2s_init(h);
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      m[w] = x.w[w];
      m[8 + w] = 0;
    }
    b2s_compress(h, m, 32, 0, true);
    uint4* d = reinterpret_cast<uint4*>(leaf + 8 * i);
    d[0] = make_uint4(h[0], h[1], h[2], h[3]);
    d[1] = make_uint4(h[4], h[5], h[6], h[7]);
  }
}

// Roots of up to 16 trees gathered into one buffer (one D2H for the transcript).
struct RootPtrs {
  const uint32_t* p[16];
};
__global__ void collect_roots_kernel(RootPtrs r, uint32_t count, uint32_t* __restrict__ out) {
  const uint32_t t = threadIdx.x;
  if (t < 8 * count) out[t] = r.p[t / 8][t % 8];
}

// get_pseudorandom_indices(root2_l, q_l, 40, excl) (fri/src/utils.rs:84-111; stark_get_pseudorandom_indices)
// for every layer on the device, so the openings' gather follows the last layer in stream order with no
// host round trip: thread l extends layer l's root by four chained Blake2s hashes (160 bytes), reads the
// 40 big-endian words and writes the column indices ys and the poly indices ys + j q (fri.rs:181-204)
// into the gather's index array.  (fri_enqueue checked q < 2^24 and the exclusion's divisor up front.)
struct FriIdxArgs {
  const uint32_t* root[16];  // root2 of layer l: the root of the layer's column tree
  uint32_t q[16];
  uint64_t col_at[16], poly_at[16];  // first slots in the index array
};
// One 64-lane workgroup per layer: a quad of lanes hashes the chain (hash_pair_quad, merkle_dev.h; one
// compression's latency is about a quarter of a lane's), then 40 lanes write one index each.
__global__ __launch_bounds__(64) void fri_indices_kernel(FriIdxArgs a, uint32_t excl, uint64_t* __restrict__ idx) {
  __shared__ uint32_t data[40];   // 160 bytes, little-endian words
  __shared__ uint32_t msg[16];
  const uint32_t l = blockIdx.x, t = threadIdx.x;
  if (t < 8) {
    data[t] = a.root[l][t];
    msg[t] = data[t];
  } else if (t < 16) {
    msg[t] = 0;
  }
  __syncthreads();
#pragma unroll 1
  for (int b = 1; b < 5; ++b) {
    uint32_t lo = 0, hi = 0;
    if (t < 4) hash_pair_quad(msg, t, lo, hi, 32);
    __syncthreads();
    if (t < 4) {
      data[8 * b + t] = lo;
      data[8 * b + 4 + t] = hi;
      msg[t] = lo;
      msg[4 + t] = hi;
    }
    __syncthreads();
  }
  if (t >= 40) return;
  const uint32_t q = a.q[l];
  const uint32_t real_mod = excl ? (uint32_t)((uint64_t)q * (excl - 1) / excl) : q;
  const uint32_t w = __builtin_bswap32(data[t]);
  const uint32_t v = w % real_mod;
  const uint64_t y = excl ? v + 1 + v / (excl - 1) : v;
  idx[a.col_at[l] + t] = y;
#pragma unroll
  for (int j = 0; j < 4; ++j) idx[a.poly_at[l] + 4 * t + j] = y + (uint64_t)q * j;
}

// Pinned slot 1 layout: [0, 2048) mk_r1cs_proof's transcript, [2048, 2560) FRI roots.
constexpr size_t kFriRootsOff = 2048;

struct FriPending {
  std::unique_ptr<stark_fri_proof> proof;
  size_t layers = 0, last_len = 0;
  uint32_t excl = 0;
  std::vector<size_t> qs;
  const fe* last_dev = nullptr;  // the last layer's values (device)
  std::vector<stark_merkle_tree*> trees;  // trees[l] commits layer l's values
  const uint8_t* h_roots = nullptr;  // pinned: roots of trees[0..layers]
};

// prove_low_degree on device values, phase 1.  Per layer everything is
// enqueued on the context stream with no host round trip: build the values'
// tree, derive special_x from its root on the device, fold, build the
// column's tree; finally the roots are queued for download.
void FriPendingDeleter::operator()(FriPending* p) const { delete p; }

stark_status fri_enqueue(stark_ctx* ctx, const fe* d_values, size_t n, const uint64_t root[4], size_t max_deg_plus_1,
                         uint32_t excl, FriPendingPtr* out, stark_merkle_tree* tree0, bool sx0_made) {
  const FieldHost& F = FieldHost::get();
  hipStream_t s = ctx->stream;
  FriPendingPtr p(new FriPending());
  p->proof = std::make_unique<stark_fri_proof>();
  p->excl = excl;
  // Layer sizes and checks up front (the reference panics on these).
  size_t layers = 0;
  {
    size_t m = n, deg = max_deg_plus_1;
    while (deg > 16) {
      if (m < 8 || (m & (m - 1))) return STARK_ERR_BAD_LENGTH;
      if (excl != 0 && (excl == 1 || (uint64_t)(m / 4) * (excl - 1) / excl == 0)) return STARK_ERR_BAD_ARG;
      if (m / 4 >= (1u << 24)) return STARK_ERR_BAD_ARG;  // get_pseudorandom_indices assert
      m /= 4;
      deg /= 4;
      ++layers;
    }
  }
  if (layers + 1 > 16) return STARK_ERR_BAD_LENGTH;
  p->layers = layers;
  const Twiddles* tw = nullptr;
  uint32_t log_n0 = 0;
  while (((size_t)1 << log_n0) < n) ++log_n0;
  if (layers > 0) {
    // values.len() must equal the order of root (xs = expand_root_of_unity, fri.rs:84).
    uint64_t inv_root[4];
    F.to_canonical(F.inv(F.from_canonical(root)), inv_root);
    stark_status st = get_twiddles(ctx, inv_root, log_n0, &tw);
    if (st != STARK_OK) return st;
  }
  // Column buffers: n/4 + n/16 + ... elements; special_x per layer; the roots.
  size_t col_total = 0;
  {
    size_t m = n;
    for (size_t l = 0; l < layers; ++l) {
      m /= 4;
      col_total += m;
    }
  }
  stark_status st = ensure_buf(ctx, ctx->fri_cols, (col_total ? col_total : 1) * sizeof(fe));
  if (st != STARK_OK) return st;
  st = ensure_buf(ctx, ctx->fri_misc, kFriMiscBytes);
  if (st != STARK_OK) return st;
  STARK_TRY(buf_acquire(ctx, ctx->fri_misc, s));  // (the distributed fold's slot 15 is on the caller's stream)
  uint8_t* pinned = nullptr;
  st = ctx_pinned(ctx, 1, kPinned1Bytes, (void**)&pinned);
  if (st != STARK_OK) return st;
  p->h_roots = pinned + kFriRootsOff;
  fe* d_sx = (fe*)ctx->fri_misc.ptr;
  while (ctx->fri_trees.size() < layers + 1) {
    stark_merkle_tree* t = nullptr;
    st = stark_merkle_new(ctx, &t);
    if (st != STARK_OK) return st;
    ctx->fri_trees.push_back(t);
  }
  // trees[l] commits layer l's values; tree0, when given, is the caller's tree of d_values (the
  // prover's L tree: the same leaves, so layer 0's tree is not built twice).
  p->trees.assign(ctx->fri_trees.begin(), ctx->fri_trees.begin() + layers + 1);
  if (tree0) p->trees[0] = tree0;
  std::vector<stark_merkle_tree*>& trees = p->trees;

  const fe* cur = d_values;
  fe* next = (fe*)ctx->fri_cols.ptr;
  size_t m = n;
  HostFp w = F.from_canonical(root);
  const HostFp inv4 = F.inv(F.from_u64(4));
  const fe r2 = to_dev(F.from_canonical(F.one().v));  // Montgomery image of R
  // special_x of this layer already made by its tree's root launch (layer 0: by the caller's tree0 build,
  // into slot 0 of fri_misc)
  bool sx_made = tree0 && sx0_made;
  for (size_t layer = 0; layer < layers; ++layer) {
    if (layer == 0 && !tree0) {
      st = merkle_build(ctx, trees[0], (const uint8_t*)cur, m, 32, s);
      if (st != STARK_OK) return st;
    }
    if (!sx_made)
      hipLaunchKernelGGL(fri_special_x_kernel, dim3(1), dim3(64), 0, s,
                         (const uint32_t*)merkle_root_dev(trees[layer]), d_sx + layer, r2);
    const size_t q = m / 4;
    const HostFp zeta = F.pow_u64(w, q);  // w^(n/4)
    const unsigned blocks = (unsigned)((q + 255) / 256);
    // The next layer's tree: the fold hashes each value it makes (level 0: no leaf pass of its own).
    uint32_t* leaf = nullptr;
    STARK_TRY(merkle_level0(ctx, trees[layer + 1], q, s, &leaf));
    hipLaunchKernelGGL(fri_fold_kernel, dim3(blocks), dim3(256), 0, s, cur, next, (uint64_t)q, (uint32_t)(2 * layer),
                       (uint64_t)0, (uint32_t)0,
                       tw->d_lo, tw->d_hi, tw->kb, (const fe*)(d_sx + layer), to_dev(zeta), to_dev(inv4), leaf);
    STARK_HIP(ctx, hipGetLastError());
    // (the next layer's special_x from its tree's root launch where that is the tail kernel)
    RootFe rf{d_sx + layer + 1, r2, nullptr, false};
    st = merkle_build(ctx, trees[layer + 1], (const uint8_t*)next, q, 32, s, 0, leaf != nullptr,
                      layer + 1 < layers ? &rf : nullptr);
    if (st != STARK_OK) return st;
    sx_made = rf.made;
    p->qs.push_back(q);
    // Recurse on the column with w^4 (fri.rs:215-223).
    cur = next;
    next += q;
    m = q;
    w = F.pow_u64(w, 4);
  }
  p->last_dev = cur;
  p->last_len = m;
  if (layers) {
    RootPtrs rp;
    for (size_t l = 0; l <= layers; ++l) rp.p[l] = (const uint32_t*)merkle_root_dev(trees[l]);
    // Straight into the pinned (coherent) host slot: no copy behind it.
    hipLaunchKernelGGL(collect_roots_kernel, dim3(1), dim3(128), 0, s, rp, (uint32_t)(layers + 1),
                       (uint32_t*)p->h_roots);
    STARK_HIP(ctx, hipGetLastError());
  }
  STARK_TRY(buf_release(ctx, ctx->fri_misc, s));
  *out = std::move(p);
  return STARK_OK;
}

// Phase 2: every opening in one gather batch together with the caller's `extra` requests, and the Last
// layer (fri.rs:108-110).  The layers' indices (the transcript, fri.rs:181-204) are derived on the device
// behind the last layer, so the gather needs no host round trip: one synchronisation in all.  The host
// then takes the indices from the index array and checks them against its own derivation.
stark_status fri_finish(stark_ctx* ctx, FriPending* p, std::vector<GatherReq>& extra, stark_fri_proof** out) {
  hipStream_t s = ctx->stream;
  std::vector<stark_merkle_tree*>& trees = p->trees;
  stark_fri_proof* proof = p->proof.get();
  proof->layers.resize(p->layers);
  std::vector<GatherReq> reqs = extra;
  const size_t n_extra = reqs.size();
  for (size_t layer = 0; layer < p->layers; ++layer) {
    stark_fri_layer& L = proof->layers[layer];
    const size_t q = p->qs[layer];
    L.col_idx.resize(40);
    L.poly_idx.resize(160);
    L.col_depth = 0;
    while (((size_t)1 << L.col_depth) < q) ++L.col_depth;
    L.poly_depth = L.col_depth + 2;
    L.col_leaves.resize(40 * 32);
    L.col_nodes.resize(40 * L.col_depth * 32);
    L.poly_leaves.resize(160 * 32);
    L.poly_nodes.resize(160 * L.poly_depth * 32);
    reqs.push_back({trees[layer + 1], nullptr, 40, L.col_leaves.data(), L.col_nodes.data()});
    reqs.push_back({trees[layer], nullptr, 160, L.poly_leaves.data(), L.poly_nodes.data()});
  }
  uint64_t* h_idx = nullptr;
  std::vector<size_t> first;
  auto indices = [&](uint64_t* hi, const std::vector<size_t>& f) -> stark_status {
    h_idx = hi;
    first = f;
    FriIdxArgs a;
    for (size_t l = 0; l < p->layers; ++l) {
      a.root[l] = (const uint32_t*)merkle_root_dev(trees[l + 1]);
      a.q[l] = (uint32_t)p->qs[l];
      a.col_at[l] = f[n_extra + 2 * l];
      a.poly_at[l] = f[n_extra + 2 * l + 1];
    }
    if (p->layers) {
      hipLaunchKernelGGL(fri_indices_kernel, dim3((unsigned)p->layers), dim3(64), 0, s, a, p->excl, hi);
      STARK_HIP(ctx, hipGetLastError());
    }
    return STARK_OK;
  };
  // The last layer's values come down with the gather (one synchronisation) when they fit the pinned slot.
  const size_t last_bytes = p->last_len * 32;
  uint8_t* h_last = const_cast<uint8_t*>(p->h_roots) - kFriRootsOff + kPinned1LastOff;
  const bool last_pinned = last_bytes && last_bytes <= kPinned1Bytes - kPinned1LastOff;
  if (last_pinned) STARK_HIP(ctx, hipMemcpyAsync(h_last, p->last_dev, last_bytes, hipMemcpyDeviceToHost, s));
  stark_status st = merkle_gather_batch(ctx, reqs, s, indices);
  if (st != STARK_OK) return st;
  size_t gathered = 0;
  for (const GatherReq& q : reqs) gathered += q.k;
  if (gathered == 0) STARK_HIP(ctx, hipStreamSynchronize(s));  // (no gather: no synchronisation)
  for (size_t layer = 0; layer < p->layers; ++layer) {
    stark_fri_layer& L = proof->layers[layer];
    const size_t q = p->qs[layer];
    memcpy(L.root2, p->h_roots + 32 * (layer + 1), 32);
    // ys = get_pseudorandom_indices(m2_root, column.len(), 40, exclude) (fri.rs:181-189)
    uint32_t ys[40];
    st = stark_get_pseudorandom_indices(L.root2, 32, (uint32_t)q, 40, p->excl, ys);
    if (st != STARK_OK) return st;
    for (int i = 0; i < 40; ++i) {
      L.col_idx[i] = (size_t)h_idx[first[n_extra + 2 * layer] + i];
      for (int j = 0; j < 4; ++j) L.poly_idx[4 * i + j] = (size_t)h_idx[first[n_extra + 2 * layer + 1] + 4 * i + j];
      if (L.col_idx[i] != ys[i]) {
        ctx->last_error = "FRI indices derived on the device differ from the host's";
        return STARK_ERR_HIP;
      }
    }
  }
  stark_fri_layer last;
  last.last = true;
  last.last_values.resize(last_bytes);
  if (last_pinned)
    memcpy(last.last_values.data(), h_last, last_bytes);
  else if (last_bytes)
    STARK_HIP(ctx, hipMemcpy(last.last_values.data(), p->last_dev, last_bytes, hipMemcpyDeviceToHost));
  proof->layers.push_back(std::move(last));
  *out = p->proof.release();
  return STARK_OK;
}

stark_status fri_prove_device(stark_ctx* ctx, const fe* d_values, size_t n, const uint64_t root[4],
                              size_t max_deg_plus_1, uint32_t excl, stark_fri_proof** out) {
  FriPendingPtr p;
  stark_status st = fri_enqueue(ctx, d_values, n, root, max_deg_plus_1, excl, &p);
  if (st != STARK_OK) return st;
  std::vector<GatherReq> none;
  return fri_finish(ctx, p.get(), none, out);
}

// "[b0,b1,...]" for a byte string (serde_json of Vec<u8>), table driven: each byte is one 4-byte store
// of its digits and a comma and an advance by their count (no branch); the last comma becomes ']'.
struct ByteText {
  uint32_t s[256];  // the decimal digits of i then ',' (little-endian bytes)
  uint8_t len[256];
  ByteText() {
    for (int i = 0; i < 256; ++i) {
      char t[8] = {0};
      len[i] = (uint8_t)snprintf(t, sizeof t, "%d,", i);
      memcpy(&s[i], t, 4);  // (4 bytes: the padding past the comma is overwritten by the next byte)
    }
  }
};

// Writes "[b0,...]" at w and returns the end; nothing past the end is written (the last byte's digits
// are stored exactly, every earlier 4-byte store is overwritten by the bytes after it).
static char* json_bytes_at(char* w, const uint8_t* p, size_t n) {
  static const ByteText T;
  *w++ = '[';
  if (n) {
    size_t i = 0;
    if (n >= 16 && json_simd_width() == 64) {
      // 16 items at a time, each with its comma; when they cover every byte the last comma is the ']'
      const size_t k = n / 16;
      w = json_items16_v512(w, p, k);
      i = 16 * k;
      if (i == n) {
        w[-1] = ']';
        return w;
      }
    }
    for (; i + 1 < n; ++i) {
      const uint8_t b = p[i];
      memcpy(w, &T.s[b], 4);
      w += T.len[b];
    }
    const uint8_t b = p[n - 1];
    const char* d = reinterpret_cast<const char*>(&T.s[b]);
    for (uint32_t k = 0; k + 1 < T.len[b]; ++k) *w++ = d[k];
  }
  *w++ = ']';
  return w;
}

// Its exact length: 2 + the digits + n - 1 commas.
static size_t json_bytes_len(const uint8_t* p, size_t n) {
  size_t d = 0;
  if (json_simd_width() == 64) d = json_digits_v512(p, n);
  else
    for (size_t i = 0; i < n; ++i) d += 1 + (p[i] >= 10) + (p[i] >= 100);
  return 2 + d + (n ? n - 1 : 0);
}

void json_bytes(std::string& o, const uint8_t* p, size_t n) {
  const size_t at = o.size();
  o.resize(at + json_bytes_len(p, n));
  json_bytes_at(&o[at], p, n);
}

// Proofs [i0, i1) of a serde_json Vec<Proof<Vec<u8>, BlakeDigest>>
// (commitment/src/merkle_tree.rs:14-18), each preceded by a comma unless it is
// proof 0; the caller writes the brackets.
static const char kLeafKey[] = "{\"leaf\":", kNodesKey[] = ",\"nodes\":[";
static char* json_branch_range_at(char* w, const uint8_t* leaves, size_t leaf_len, const uint8_t* nodes, size_t i0,
                                  size_t i1, size_t depth) {
  for (size_t i = i0; i < i1; ++i) {
    if (i) *w++ = ',';
    memcpy(w, kLeafKey, sizeof kLeafKey - 1);
    w += sizeof kLeafKey - 1;
    w = json_bytes_at(w, leaves + leaf_len * i, leaf_len);
    memcpy(w, kNodesKey, sizeof kNodesKey - 1);
    w += sizeof kNodesKey - 1;
    for (size_t d = 0; d < depth; ++d) {
      if (d) *w++ = ',';
      w = json_bytes_at(w, nodes + (i * depth + d) * 32, 32);
    }
    *w++ = ']';
    *w++ = '}';
  }
  return w;
}
static size_t json_branch_range_len(const uint8_t* leaves, size_t leaf_len, const uint8_t* nodes, size_t i0,
                                    size_t i1, size_t depth) {
  size_t t = 0;
  for (size_t i = i0; i < i1; ++i) {
    t += (i ? 1 : 0) + (sizeof kLeafKey - 1) + json_bytes_len(leaves + leaf_len * i, leaf_len) +
         (sizeof kNodesKey - 1) + (depth ? depth - 1 : 0) + 2;
    for (size_t d = 0; d < depth; ++d) t += json_bytes_len(nodes + (i * depth + d) * 32, 32);
  }
  return t;
}

void json_branches(std::string& o, const std::vector<uint8_t>& leaves, size_t leaf_len,
                   const std::vector<uint8_t>& nodes, size_t k, size_t depth) {
  const size_t at = o.size();
  o.resize(at + 2 + json_branch_range_len(leaves.data(), leaf_len, nodes.data(), 0, k, depth));
  char* w = &o[at];
  *w++ = '[';
  w = json_branch_range_at(w, leaves.data(), leaf_len, nodes.data(), 0, k, depth);
  *w = ']';
}

void JsonPieces::text(const std::string& s) {
  if (!pieces.empty() && !pieces.back().size && pieces.back().text.size() < 4096) {
    pieces.back().text += s;  // adjacent short fixed texts are one piece (a prerendered one is not grown)
    return;
  }
  pieces.push_back(Piece{s, nullptr, nullptr});
}

void JsonPieces::bytes(const uint8_t* p, size_t n) {
  pieces.push_back(Piece{std::string(), [p, n] { return json_bytes_len(p, n); },
                         [p, n](char* w) { return json_bytes_at(w, p, n); }});
}

void JsonPieces::byte_rows(const uint8_t* p, size_t rows, size_t row_len) {
  constexpr size_t per = 256;  // rows per piece
  for (size_t r0 = 0; r0 < rows; r0 += per) {
    const size_t r1 = r0 + per < rows ? r0 + per : rows;
    pieces.push_back(Piece{std::string(),
                           [=] {
                             size_t t = 0;
                             for (size_t r = r0; r < r1; ++r) t += (r ? 1 : 0) + json_bytes_len(p + r * row_len, row_len);
                             return t;
                           },
                           [=](char* w) {
                             for (size_t r = r0; r < r1; ++r) {
                               if (r) *w++ = ',';
                               w = json_bytes_at(w, p + r * row_len, row_len);
                             }
                             return w;
                           }});
  }
}

void JsonPieces::branches(const std::vector<uint8_t>& leaves, size_t leaf_len, const std::vector<uint8_t>& nodes,
                          size_t k, size_t depth) {
  text("[");
  const size_t per = 40;  // proofs per piece
  for (size_t i0 = 0; i0 < k; i0 += per) {
    const size_t i1 = i0 + per < k ? i0 + per : k;
    const uint8_t* lp = leaves.data();
    const uint8_t* np = nodes.data();
    pieces.push_back(Piece{std::string(), [=] { return json_branch_range_len(lp, leaf_len, np, i0, i1, depth); },
                           [=](char* w) { return json_branch_range_at(w, lp, leaf_len, np, i0, i1, depth); }});
  }
  text("]");
}

// The pieces' lengths (computed ones on the host workers) and their offsets in the text.
static std::vector<size_t> piece_offsets(std::vector<JsonPieces::Piece>& pieces, unsigned max_threads) {
  const size_t k = pieces.size();
  std::vector<size_t> len(k, 0);
  std::atomic<size_t> next{0};
  unsigned nt = host_threads();
  if (nt > max_threads) nt = max_threads;
  if (k < 8) nt = 1;
  host_parallel(nt, [&](unsigned) {
    for (size_t i; (i = next.fetch_add(1)) < k;) len[i] = pieces[i].size ? pieces[i].size() : pieces[i].text.size();
  });
  std::vector<size_t> off(k + 1, 0);
  for (size_t i = 0; i < k; ++i) off[i + 1] = off[i] + len[i];
  return off;
}

// Every piece written at its offset in dst (the host workers take pieces in order of claim).
static void write_pieces(std::vector<JsonPieces::Piece>& pieces, const std::vector<size_t>& off, char* dst,
                         unsigned max_threads) {
  std::atomic<size_t> next{0};
  unsigned nt = host_threads();
  if (nt > max_threads) nt = max_threads;
  if (pieces.size() < 8 || off.back() < ((size_t)1 << 16)) nt = 1;
  host_parallel(nt, [&](unsigned) {
    for (size_t i; (i = next.fetch_add(1)) < pieces.size();) {
      const JsonPieces::Piece& q = pieces[i];
      if (q.size) q.write(dst + off[i]);
      else memcpy(dst + off[i], q.text.data(), q.text.size());
    }
  });
}

void JsonPieces::prerender(unsigned max_threads) {
  std::vector<size_t> off = piece_offsets(pieces, max_threads);
  std::string all(off.back(), '\0');
  write_pieces(pieces, off, &all[0], max_threads);
  pieces.clear();
  pieces.push_back(Piece{std::move(all), nullptr, nullptr});
}

void JsonPieces::render(std::string& o) {
  std::vector<size_t> off = piece_offsets(pieces, 16);
  const size_t at = o.size();
  o.resize(at + off.back());
  write_pieces(pieces, off, &o[at], 16);
  pieces.clear();
}

void JsonPieces::render(JsonText& o) {
  std::vector<size_t> off = piece_offsets(pieces, 16);
  o.n = off.back();
  o.p.reset(new char[o.n + 1]);  // uninitialised; its pages fault in on the threads that write them
  o.p[o.n] = 0;
  write_pieces(pieces, off, o.p.get(), 16);
  pieces.clear();
}

// serde_json of Vec<FriProof<BlakeDigest>> (fri.rs:16-26) as pieces.
void fri_proof_json_pieces(const stark_fri_proof* proof, JsonPieces& j) {
  j.text("[");
  for (size_t l = 0; l < proof->layers.size(); ++l) {
    const stark_fri_layer& L = proof->layers[l];
    if (l) j.text(",");
    if (L.last) {
      j.text("{\"Last\":{\"last\":[");
      j.byte_rows(L.last_values.data(), L.last_values.size() / 32, 32);
      j.text("]}}");
    } else {
      j.text("{\"Middle\":{\"root2\":");
      j.bytes(L.root2, 32);
      j.text(",\"column_branches\":");
      j.branches(L.col_leaves, 32, L.col_nodes, L.col_idx.size(), L.col_depth);
      j.text(",\"poly_branches\":");
      j.branches(L.poly_leaves, 32, L.poly_nodes, L.poly_idx.size(), L.poly_depth);
      j.text("}}");
    }
  }
  j.text("]");
}

void fri_proof_json_string(const stark_fri_proof* proof, std::string& o) {
  JsonPieces j;
  fri_proof_json_pieces(proof, j);
  j.render(o);
}

}  // namespace stark

using namespace stark;

extern "C" {

stark_status stark_prove_low_degree_dev(stark_ctx* ctx, const uint64_t* d_values, size_t n, const uint64_t root[4],
                                        size_t max_deg_plus_1, uint32_t exclude_multiples_of, stark_fri_proof** out) {
  if (!ctx || !root || !out || (n && !d_values)) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  return fri_prove_device(ctx, (const fe*)d_values, n, root, max_deg_plus_1, exclude_multiples_of, out);
}

stark_status stark_prove_low_degree(stark_ctx* ctx, const uint64_t* values, size_t n, const uint64_t root[4],
                                    size_t max_deg_plus_1, uint32_t exclude_multiples_of, stark_fri_proof** out) {
  if (!ctx || !root || !out || (n && !values)) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  stark_status st = ensure_buf(ctx, ctx->io, (n ? n : 1) * sizeof(fe));
  if (st != STARK_OK) return st;
  if (n) STARK_HIP(ctx, hipMemcpyAsync(ctx->io.ptr, values, n * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
  st = fri_prove_device(ctx, (const fe*)ctx->io.ptr, n, root, max_deg_plus_1, exclude_multiples_of, out);
  hipStreamSynchronize(ctx->stream);
  return st;
}

void stark_fri_proof_free(stark_fri_proof* proof) { delete proof; }

// One FRI fold on this GPU's residue class (distributed prover, fri.rs:135-164):
// `values` holds the layer's values at the points rank + world*j (n/world of
// them), `column` receives the folded column at the same residue class of the
// n/4 rows; special_x = from_bytes_le(m_root) (fri.rs:135).
// special_x from a host root (m_root) or a device-resident one (d_m_root: the fold reads it on the stream,
// no host round trip).
static stark_status fri_fold(stark_ctx* ctx, const uint64_t* values, uint64_t* column, size_t n,
                             const uint64_t root[4], const uint8_t* m_root, const uint8_t* d_m_root, uint32_t world,
                             uint32_t rank, void* stream) {
  if (!ctx || !values || !column || !root || (!m_root && !d_m_root)) return STARK_ERR_BAD_ARG;
  if (world == 0 || (world & (world - 1)) || rank >= world) return STARK_ERR_BAD_ARG;
  if (n < 4 || (n & (n - 1)) || (n / 4) % world != 0) return STARK_ERR_BAD_LENGTH;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const FieldHost& F = FieldHost::get();
  hipStream_t s = pick_stream(ctx, stream);
  uint32_t log_n = 0, log_g = 0;
  while (((size_t)1 << log_n) < n) ++log_n;
  while ((1u << log_g) < world) ++log_g;
  uint64_t inv_root[4];
  F.to_canonical(F.inv(F.from_canonical(root)), inv_root);
  const Twiddles* tw = nullptr;
  stark_status st = get_twiddles(ctx, inv_root, log_n, &tw);
  if (st != STARK_OK) return st;
  st = ensure_buf(ctx, ctx->fri_misc, kFriMiscBytes);
  if (st != STARK_OK) return st;
  STARK_TRY(buf_acquire(ctx, ctx->fri_misc, s));  // (prove_low_degree writes slots 0-14 on the context stream)
  fe* d_sx = (fe*)ctx->fri_misc.ptr + 15;  // slot 15: unused by prove_low_degree's <= 15 layers
  fe sx;
  if (m_root) {
    sx = to_dev(F.from_bytes_le(m_root, 32));
    STARK_HIP(ctx, hipMemcpyAsync(d_sx, &sx, sizeof(fe), hipMemcpyHostToDevice, s));
  } else {  // fri.rs:135 on the device: the root read as LE words, reduced mod p, Montgomery image
    hipLaunchKernelGGL(fri_special_x_kernel, dim3(1), dim3(64), 0, s, (const uint32_t*)d_m_root, d_sx,
                       to_dev(F.from_canonical(F.one().v)));
    STARK_HIP(ctx, hipGetLastError());
  }
  const HostFp zeta = F.pow_u64(F.from_canonical(root), n / 4);
  const size_t q = n / 4 / world;
  hipLaunchKernelGGL(fri_fold_kernel, dim3((unsigned)((q + 255) / 256)), dim3(256), 0, s, (const fe*)values,
                     (fe*)column, (uint64_t)q, (uint32_t)0, (uint64_t)rank, log_g, tw->d_lo, tw->d_hi, tw->kb,
                     (const fe*)d_sx, to_dev(zeta), to_dev(F.inv(F.from_u64(4))), (uint32_t*)nullptr);
  STARK_HIP(ctx, hipGetLastError());
  STARK_TRY(buf_release(ctx, ctx->fri_misc, s));
  if (m_root) STARK_HIP(ctx, hipStreamSynchronize(s));  // sx lives on this stack frame
  return STARK_OK;
}

stark_status stark_fri_fold_dev(stark_ctx* ctx, const uint64_t* values, uint64_t* column, size_t n,
                                const uint64_t root[4], const uint8_t m_root[32], uint32_t world, uint32_t rank,
                                void* stream) {
  if (!m_root) return STARK_ERR_BAD_ARG;
  return fri_fold(ctx, values, column, n, root, m_root, nullptr, world, rank, stream);
}

stark_status stark_fri_fold_dev_root(stark_ctx* ctx, const uint64_t* values, uint64_t* column, size_t n,
                                     const uint64_t root[4], const uint8_t* d_m_root, uint32_t world, uint32_t rank,
                                     void* stream) {
  if (!d_m_root || (((uintptr_t)d_m_root) & 3)) return STARK_ERR_BAD_ARG;
  return fri_fold(ctx, values, column, n, root, nullptr, d_m_root, world, rank, stream);
}

// serde_json of a StarkProof (r1cs-stark/src/utils.rs:122-130) from its parts
// (the distributed prover's rank 0 assembles the openings of every rank).
stark_status stark_r1cs_proof_json_from_parts(const uint8_t m_root[32], const uint8_t l_root[32],
                                              const uint8_t a_root[32], const stark_branches* main_branches,
                                              const stark_branches* linear_comb_branches,
                                              const stark_fri_layer_parts* layers, size_t n_layers,
                                              const uint8_t* last_values, size_t n_last, char* buf, size_t cap,
                                              size_t* len) {
  if (!m_root || !l_root || !a_root || !main_branches || !linear_comb_branches || !len) return STARK_ERR_BAD_ARG;
  if ((n_layers && !layers) || (n_last && !last_values)) return STARK_ERR_BAD_ARG;
  auto vec = [](const uint8_t* p, size_t n) { return std::vector<uint8_t>(p, p + n); };
  const stark_branches& mb = *main_branches;
  const stark_branches& lb = *linear_comb_branches;
  const std::vector<uint8_t> ml = vec(mb.leaves, mb.k * mb.leaf_len), mn = vec(mb.nodes, mb.k * mb.depth * 32);
  const std::vector<uint8_t> ll = vec(lb.leaves, lb.k * lb.leaf_len), ln = vec(lb.nodes, lb.k * lb.depth * 32);
  stark_fri_proof fri;
  for (size_t l = 0; l < n_layers; ++l)  // FRI leaves are field elements (fri.rs:16-26): 32 B each
    if (layers[l].column.leaf_len != 32 || layers[l].poly.leaf_len != 32) return STARK_ERR_BAD_ARG;
  for (size_t l = 0; l < n_layers; ++l) {
    const stark_fri_layer_parts& P = layers[l];
    stark_fri_layer L;
    memcpy(L.root2, P.root2, 32);
    L.col_idx.resize(P.column.k);
    L.poly_idx.resize(P.poly.k);
    L.col_depth = P.column.depth;
    L.poly_depth = P.poly.depth;
    L.col_leaves = vec(P.column.leaves, P.column.k * 32);
    L.col_nodes = vec(P.column.nodes, P.column.k * P.column.depth * 32);
    L.poly_leaves = vec(P.poly.leaves, P.poly.k * 32);
    L.poly_nodes = vec(P.poly.nodes, P.poly.k * P.poly.depth * 32);
    fri.layers.push_back(std::move(L));
  }
  stark_fri_layer last;
  last.last = true;
  last.last_values = vec(last_values, 32 * n_last);
  fri.layers.push_back(std::move(last));
  JsonPieces j;
  j.text("{\"m_root\":");
  j.bytes(m_root, 32);
  j.text(",\"l_root\":");
  j.bytes(l_root, 32);
  j.text(",\"a_root\":");
  j.bytes(a_root, 32);
  j.text(",\"main_branches\":");
  j.branches(ml, mb.leaf_len, mn, mb.k, mb.depth);
  j.text(",\"linear_comb_branches\":");
  j.branches(ll, lb.leaf_len, ln, lb.k, lb.depth);
  j.text(",\"fri_proof\":");
  fri_proof_json_pieces(&fri, j);
  j.text("}");
  std::string o;
  j.render(o);
  *len = o.size();
  if (buf && cap) {
    const size_t k = o.size() < cap ? o.size() : cap;
    memcpy(buf, o.data(), k);
    if (k < cap) buf[k] = 0;
  }
  return STARK_OK;
}


stark_status stark_fri_proof_json(const stark_fri_proof* proof, char* buf, size_t cap, size_t* len) {
  if (!proof || !len) return STARK_ERR_BAD_ARG;
  std::string o;
  fri_proof_json_string(proof, o);
  *len = o.size();
  if (buf && cap) {
    const size_t k = o.size() < cap ? o.size() : cap;
    memcpy(buf, o.data(), k);
    if (k < cap) buf[k] = 0;
  }
  return STARK_OK;
}

size_t stark_fri_proof_num_layers(const stark_fri_proof* proof) { return proof ? proof->layers.size() : 0; }

stark_status stark_fri_proof_layer_info(const stark_fri_proof* proof, size_t i, int* is_last, uint8_t root2[32],
                                        size_t* n_column, size_t* column_depth, size_t* n_poly, size_t* poly_depth,
                                        size_t* n_last) {
  if (!proof || i >= proof->layers.size()) return STARK_ERR_BAD_ARG;
  const stark_fri_layer& L = proof->layers[i];
  if (is_last) *is_last = L.last ? 1 : 0;
  if (root2) memcpy(root2, L.root2, 32);
  if (n_column) *n_column = L.col_idx.size();
  if (column_depth) *column_depth = L.col_depth;
  if (n_poly) *n_poly = L.poly_idx.size();
  if (poly_depth) *poly_depth = L.poly_depth;
  if (n_last) *n_last = L.last_values.size() / 32;
  return STARK_OK;
}

stark_status stark_fri_proof_layer_data(const stark_fri_proof* proof, size_t i, uint8_t* column_leaves,
                                        size_t column_leaves_cap, uint8_t* column_nodes, size_t column_nodes_cap,
                                        uint8_t* poly_leaves, size_t poly_leaves_cap, uint8_t* poly_nodes,
                                        size_t poly_nodes_cap, uint8_t* last_values, size_t last_values_cap) {
  if (!proof || i >= proof->layers.size()) return STARK_ERR_BAD_ARG;
  const stark_fri_layer& L = proof->layers[i];
  // Every capacity is checked before anything is written: a short buffer is STARK_ERR_BAD_LENGTH
  // and leaves all five outputs untouched.
  const std::pair<const std::vector<uint8_t>*, std::pair<uint8_t*, size_t>> outs[5] = {
      {&L.col_leaves, {column_leaves, column_leaves_cap}},
      {&L.col_nodes, {column_nodes, column_nodes_cap}},
      {&L.poly_leaves, {poly_leaves, poly_leaves_cap}},
      {&L.poly_nodes, {poly_nodes, poly_nodes_cap}},
      {&L.last_values, {last_values, last_values_cap}}};
  for (const auto& o : outs)
    if (o.second.first && o.second.second < o.first->size()) return STARK_ERR_BAD_LENGTH;
  for (const auto& o : outs)
    if (o.second.first && !o.first->empty()) memcpy(o.second.first, o.first->data(), o.first->size());
  return STARK_OK;
}

}  // extern "C"
