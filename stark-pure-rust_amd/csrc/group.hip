// Device groups: one transform, one tree or one proof over G contexts ("Multi-GPU is a
// ctx group created once"; 8(e)).  The reference's only parallelism is the thread pool a call builds
// for itself (Worker::new inside best_fft, fri/src/fft.rs:332; commitment/src/multicore.rs:43-45); a
// group is that pool with GPUs as its workers, created once by the caller and handed to the group
// entry points, which keep the reference's signatures (best_fft / inv_best_fft, MerkleTree, and
// prove_with_witness).
//
// Transport: peer copies.  Every exchange is pulled by the receiving member on its own stream, after an
// event wait on each sender's stream (hipMemcpyPeerAsync between devices over xGMI, a device-to-device
// copy when two members share a GPU), so one code path runs G contexts on one device and G devices.
// After the copies each member waits for every other member's "copied" event, so no sender reuses a
// buffer a peer still reads.  Nothing waits for the host between the steps of a transform or of a
// proof's commit phase; RCCL is not used here because it refuses two ranks on one GPU, and the
// library needs no collective beyond these all-to-alls and gathers.
//
// The algorithms are the torch.distributed ones, moved into the library:
//  - NTT: the one-exchange cyclic form of stark_amd/distributed.py cyclic_ntt (member r transforms
//    x[r + G j], one all-to-all, G-point DFTs across the received chunks);
//  - Merkle: contiguous leaf blocks per member, subtree roots gathered to member 0, the top log2 G
//    levels hashed there -- the reference's own subtree + top-tree split
//    (commitment/src/merkle_proof_in_place.rs:106-206);
//  - prover: the residue-class layout of stark_amd/dprove.py: coset LDEs, constraints
//    and FRI folds local, Merkle trees by one digest all-to-all each.
#include <string.h>

#include <algorithm>
#include <array>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>

#include "internal.h"

// One host thread per member after the first, created with the group and parked between calls: a call's
// per-member steps (a member's synchronous library calls) run on all GPUs at once without spawning
// threads per call (≈ 0.15 ms per 7 threads).
struct GroupWorkers {
  std::mutex mu;
  std::condition_variable wake, done_cv;
  uint64_t gen = 0;
  size_t done = 0;
  bool stop = false;
  const std::function<void(size_t)>* job = nullptr;
  std::vector<std::thread> th;
  void start(size_t G) {
    for (size_t r = 1; r < G; ++r)
      th.emplace_back([this, r, G] {
        uint64_t seen = 0;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
          wake.wait(lk, [&] { return stop || gen != seen; });
          if (stop) return;
          seen = gen;
          const std::function<void(size_t)>* f = job;
          lk.unlock();
          (*f)(r);
          lk.lock();
          if (++done == G - 1) done_cv.notify_one();
        }
      });
  }
  // fn(0) on the caller's thread, fn(r) on worker r; returns when all have finished.
  void run(const std::function<void(size_t)>& fn) {
    const size_t others = th.size();
    {
      std::lock_guard<std::mutex> lk(mu);
      job = &fn;
      done = 0;
      ++gen;
    }
    wake.notify_all();
    fn(0);
    std::unique_lock<std::mutex> lk(mu);
    done_cv.wait(lk, [&] { return done == others; });
  }
  ~GroupWorkers() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    wake.notify_all();
    for (auto& t : th) t.join();
  }
};

struct stark_group {
  std::vector<stark_ctx*> m;             // member contexts (owned)
  GroupWorkers workers;
  std::vector<hipEvent_t> ready, copied;  // per member, created on its device
  std::string last_error;
  // Per-member buffers and trees reused across calls: a call takes them in a fixed order (slot cursor),
  // so calls of one shape reuse the same allocations.
  std::vector<std::vector<stark::DevBuf>> slots;
  std::vector<std::vector<stark_merkle_tree*>> trees;
  std::vector<size_t> slot_at, tree_at;
  std::vector<void*> pinned;  // per member host staging (best_fft)
  std::vector<size_t> pinned_bytes;
};

struct stark_group_tree {
  stark_group* g = nullptr;
  size_t n = 0, leaf_len = 0, m = 0;  // m leaves per member (split), else n on member 0
  bool split = false, built = false, has_root = false;
  uint32_t depth = 0, log_g = 0;
  std::vector<stark_merkle_tree*> sub;  // per member subtree
  stark::DevBuf roots;                   // member 0: G subtree roots, then the G - 1 digests above them
  std::vector<uint8_t> levels;           // the same on the host ((2G - 1) x 32 B)
  uint8_t root[32];
};

namespace stark {
namespace {

uint32_t log2_exact(size_t v) {
  uint32_t l = 0;
  while (((size_t)1 << l) < v) ++l;
  return l;
}

stark_status gfail(stark_group* g, size_t r, stark_status st) {
  if (st != STARK_OK && g->last_error.empty()) {
    g->last_error = "member " + std::to_string(r) + ": " + g->m[r]->last_error;
  }
  return st;
}

stark_status ghip(stark_group* g, hipError_t e, const char* what) {
  if (e == hipSuccess) return STARK_OK;
  g->last_error = std::string(what) + ": " + hipGetErrorString(e);
  return e == hipErrorOutOfMemory ? STARK_ERR_OOM : STARK_ERR_HIP;
}
#define G_HIP(g, call)                                   \
  do {                                                   \
    const stark_status s_ = ghip(g, (call), #call);      \
    if (s_ != STARK_OK) return s_;                       \
  } while (0)

// fn(r) for every member, member 0 on the calling thread and the others on the group's worker threads (a
// synchronous library call then runs on all GPUs at once).  The first failing member's status.
template <class Fn>
stark_status for_members(stark_group* g, Fn&& fn) {
  const size_t G = g->m.size();
  std::vector<stark_status> st(G, STARK_OK);
  const std::function<void(size_t)> job = [&](size_t r) {
    try {
      st[r] = fn(r);
    } catch (...) {  // (std::bad_alloc from a member's host containers)
      st[r] = STARK_ERR_OOM;
    }
  };
  g->workers.run(job);
  for (size_t r = 0; r < G; ++r)
    if (st[r] != STARK_OK) return gfail(g, r, st[r]);
  return STARK_OK;
}

void reset_cursors(stark_group* g) {
  std::fill(g->slot_at.begin(), g->slot_at.end(), 0);
  std::fill(g->tree_at.begin(), g->tree_at.end(), 0);
}

// The next per-call device buffer of member r (at least `bytes`).
stark_status take(stark_group* g, size_t r, size_t bytes, void** out) {
  auto& v = g->slots[r];
  const size_t i = g->slot_at[r]++;
  if (i == v.size()) v.emplace_back();
  STARK_TRY(gfail(g, r, ensure_buf(g->m[r], v[i], bytes)));
  *out = v[i].ptr;
  return STARK_OK;
}

stark_status take_tree(stark_group* g, size_t r, stark_merkle_tree** out) {
  auto& v = g->trees[r];
  const size_t i = g->tree_at[r]++;
  if (i == v.size()) {
    stark_merkle_tree* t = nullptr;
    STARK_TRY(gfail(g, r, stark_merkle_new(g->m[r], &t)));
    v.push_back(t);
  }
  *out = v[i];
  return STARK_OK;
}

hipStream_t stream_of(stark_group* g, size_t r) { return g->m[r]->stream; }

stark_status copy_from(stark_group* g, size_t dst_m, void* dst, size_t src_m, const void* src, size_t bytes) {
  const int dd = g->m[dst_m]->device, sd = g->m[src_m]->device;
  if (!bytes) return STARK_OK;
  if (dd == sd) {
    G_HIP(g, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, stream_of(g, dst_m)));
  } else {
    G_HIP(g, hipMemcpyPeerAsync(dst, dd, src, sd, bytes, stream_of(g, dst_m)));
  }
  return STARK_OK;
}

// Every member's stream marks what it has enqueued so far (the senders' buffers are then complete).
stark_status mark_ready(stark_group* g) {
  for (size_t r = 0; r < g->m.size(); ++r) {
    G_HIP(g, hipSetDevice(g->m[r]->device));
    G_HIP(g, hipEventRecord(g->ready[r], stream_of(g, r)));
  }
  return STARK_OK;
}

// After a member's pulls: every member waits for every other member's pulls, so nothing overwrites (or a
// later call frees) a send buffer that a peer's copy may still read.
stark_status mark_copied(stark_group* g) {
  const size_t G = g->m.size();
  for (size_t r = 0; r < G; ++r) {
    G_HIP(g, hipSetDevice(g->m[r]->device));
    G_HIP(g, hipEventRecord(g->copied[r], stream_of(g, r)));
  }
  for (size_t r = 0; r < G; ++r) {
    G_HIP(g, hipSetDevice(g->m[r]->device));
    for (size_t s = 0; s < G; ++s)
      if (s != r) G_HIP(g, hipStreamWaitEvent(stream_of(g, r), g->copied[s], 0));
  }
  return STARK_OK;
}

// The all-to-all of equal chunks: member r's recv[r] + s chunk <- member s's send[s] + r chunk (with
// gather: send[s] + 0, i.e. every member receives every member's first `chunk` bytes in member order).
stark_status exchange(stark_group* g, const uint8_t* const* send, uint8_t* const* recv, size_t chunk, bool gather) {
  const size_t G = g->m.size();
  STARK_TRY(mark_ready(g));
  for (size_t r = 0; r < G; ++r) {
    G_HIP(g, hipSetDevice(g->m[r]->device));
    for (size_t s = 0; s < G; ++s) {
      if (s != r) G_HIP(g, hipStreamWaitEvent(stream_of(g, r), g->ready[s], 0));
      STARK_TRY(copy_from(g, r, recv[r] + s * chunk, s, send[s] + (gather ? 0 : r * chunk), chunk));
    }
  }
  return mark_copied(g);
}

// Member 0 receives every member's first `chunk` bytes (member order) at dst0.
stark_status gather_to0(stark_group* g, const uint8_t* const* send, uint8_t* dst0, size_t chunk) {
  const size_t G = g->m.size();
  STARK_TRY(mark_ready(g));
  G_HIP(g, hipSetDevice(g->m[0]->device));
  for (size_t s = 0; s < G; ++s) {
    if (s) G_HIP(g, hipStreamWaitEvent(stream_of(g, 0), g->ready[s], 0));
    STARK_TRY(copy_from(g, 0, dst0 + s * chunk, s, send[s], chunk));
  }
  return mark_copied(g);
}

stark_status sync_all(stark_group* g) {
  for (size_t r = 0; r < g->m.size(); ++r) {
    G_HIP(g, hipSetDevice(g->m[r]->device));
    G_HIP(g, hipStreamSynchronize(stream_of(g, r)));
  }
  return STARK_OK;
}

void canon(const HostFp& x, uint64_t out[4]) { FieldHost::get().to_canonical(x, out); }

// ---- NTT ----------------------------------------------------------------------------------------
// One transform of n = 2^log_n points over the G members (stark_amd/distributed.py cyclic_ntt):
// member r's shard[r] holds x[r + G j], j < M = n / G, and is destroyed; out[r] receives
// X[r c + i + M k1] at k1 c + i (c = M / G).  Asynchronous on the member streams.
stark_status group_ntt(stark_group* g, uint64_t* const* shard, uint64_t* const* out, uint32_t log_n,
                       const uint64_t root[4], bool inverse) {
  const size_t G = g->m.size();
  const uint32_t log_g = log2_exact(G);
  if (log_n < 2 * log_g || log_n > 30) return STARK_ERR_BAD_LENGTH;
  const FieldHost& F = FieldHost::get();
  const size_t n = (size_t)1 << log_n, M = n / G, c = M / G;
  const uint32_t log_m = log_n - log_g;
  const HostFp w = F.from_canonical(root);
  uint64_t wg[4], wm[4], wtw[4];
  canon(F.pow_u64(w, G), wg);
  canon(F.pow_u64(w, M), wm);
  canon(inverse ? F.inv(w) : w, wtw);
  // The twiddle w^(r k2) goes into the sender's last local pass from G = 8 on, and into the receiver's
  // strided DFT below that (cheaper there: profiles/r04_distributed_local_step.txt).
  const bool fused = G >= 8;
  for (size_t r = 0; r < G; ++r) {
    stark_ctx* cx = g->m[r];
    if (fused) {
      STARK_TRY(gfail(g, r, stark_cyclic_ntt_local_dev(cx, shard[r], log_n, log_g, (uint32_t)r, root,
                                                       inverse ? 1 : 0, nullptr)));
    } else {
      STARK_TRY(gfail(g, r, stark_ntt_dev(cx, shard[r], log_m, 1, wg, inverse ? 1 : 0, nullptr)));
    }
  }
  std::vector<const uint8_t*> send(G);
  std::vector<uint8_t*> recv(G);
  for (size_t r = 0; r < G; ++r) {
    send[r] = (const uint8_t*)shard[r];
    recv[r] = (uint8_t*)out[r];
  }
  STARK_TRY(exchange(g, send.data(), recv.data(), c * sizeof(fe), false));
  for (size_t r = 0; r < G; ++r) {
    stark_ctx* cx = g->m[r];
    if (fused) {
      STARK_TRY(gfail(g, r, stark_ntt_strided_dev(cx, out[r], log_g, c, wm, inverse ? 1 : 0, nullptr)));
    } else {
      STARK_TRY(gfail(g, r, stark_ntt_strided_tw_dev(cx, out[r], log_g, c, wm, inverse ? 1 : 0, wtw, log_n,
                                                     (uint64_t)(r * c), nullptr)));
    }
  }
  return STARK_OK;
}

stark_status group_pinned(stark_group* g, size_t r, size_t bytes, void** out) {
  if (g->pinned_bytes[r] < bytes) {
    if (g->pinned[r]) hipHostFree(g->pinned[r]);
    g->pinned[r] = nullptr;
    g->pinned_bytes[r] = 0;
    G_HIP(g, hipSetDevice(g->m[r]->device));
    G_HIP(g, hipHostMalloc(&g->pinned[r], bytes));
    g->pinned_bytes[r] = bytes;
  }
  *out = g->pinned[r];
  return STARK_OK;
}

// best_fft / inv_best_fft (fft.rs:327-379) on the group: the host input is zero-padded and dealt out
// cyclically, the results are collected back into natural order.
stark_status group_fft_host(stark_group* g, const uint64_t* in, size_t len, const uint64_t root[4], uint32_t log_n,
                            uint64_t* out, bool inverse) {
  if (!g || !root || !out || (len && !in)) return STARK_ERR_BAD_ARG;
  if (log_n > 28) return STARK_ERR_BAD_LENGTH;
  const size_t n = (size_t)1 << log_n;
  if (len > n) return STARK_ERR_BAD_LENGTH;  // fft.rs:162
  const size_t G = g->m.size();
  const uint32_t log_g = log2_exact(G);
  g->last_error.clear();
  if (G == 1 || log_n < 2 * log_g) {  // too small to split: member 0 alone
    const stark_status st = inverse ? stark_inv_best_fft(g->m[0], in, len, root, log_n, out)
                                    : stark_best_fft(g->m[0], in, len, root, log_n, out);
    return gfail(g, 0, st);
  }
  reset_cursors(g);
  const size_t M = n / G, c = M / G;
  std::vector<uint64_t*> shard(G), res(G), host(G);
  for (size_t r = 0; r < G; ++r) {
    void* p = nullptr;
    STARK_TRY(take(g, r, M * sizeof(fe), &p));
    shard[r] = (uint64_t*)p;
    STARK_TRY(take(g, r, M * sizeof(fe), &p));
    res[r] = (uint64_t*)p;
    STARK_TRY(group_pinned(g, r, M * sizeof(fe), &p));
    host[r] = (uint64_t*)p;
  }
  // shard r = x[r + G j]: one pass over the input, each host worker a range of j
  const unsigned nt = (unsigned)std::min<size_t>(host_threads(), std::max<size_t>(M >> 12, 1));
  host_parallel(nt, [&](unsigned t) {
    const size_t j0 = M * t / nt, j1 = M * (t + 1) / nt;
    for (size_t j = j0; j < j1; ++j)
      for (size_t r = 0; r < G; ++r) {
        const size_t i = r + G * j;
        uint64_t* d = host[r] + 4 * j;
        if (i < len) {
          memcpy(d, in + 4 * i, 32);
        } else {
          memset(d, 0, 32);
        }
      }
  });
  for (size_t r = 0; r < G; ++r) {
    G_HIP(g, hipSetDevice(g->m[r]->device));
    G_HIP(g, hipMemcpyAsync(shard[r], host[r], M * sizeof(fe), hipMemcpyHostToDevice, stream_of(g, r)));
  }
  STARK_TRY(group_ntt(g, shard.data(), res.data(), log_n, root, inverse));
  for (size_t r = 0; r < G; ++r) {
    G_HIP(g, hipSetDevice(g->m[r]->device));
    G_HIP(g, hipMemcpyAsync(host[r], res[r], M * sizeof(fe), hipMemcpyDeviceToHost, stream_of(g, r)));
  }
  STARK_TRY(sync_all(g));
  // member r's run k1 (c values) is X[r c + M k1 ..]
  const size_t runs = G * G;
  host_parallel((unsigned)std::min<size_t>(host_threads(), runs), [&](unsigned t) {
    const unsigned nt2 = (unsigned)std::min<size_t>(host_threads(), runs);
    for (size_t q = t; q < runs; q += nt2) {
      const size_t r = q / G, k1 = q % G;
      memcpy(out + 4 * (r * c + M * k1), host[r] + 4 * (k1 * c), c * sizeof(fe));
    }
  });
  return STARK_OK;
}

// ---- Merkle --------------------------------------------------------------------------------------
// Subtrees built: gather their roots to member 0, hash the top levels there, bring them to the host.
stark_status tree_top(stark_group_tree* t) {
  stark_group* g = t->g;
  const size_t G = g->m.size();
  if (!t->split) {
    STARK_TRY(sync_all(g));
    G_HIP(g, hipSetDevice(g->m[0]->device));
    STARK_TRY(gfail(g, 0, merkle_root_d2h(g->m[0], t->sub[0], stream_of(g, 0), t->root)));
    t->levels.assign(t->root, t->root + 32);
    return STARK_OK;
  }
  STARK_TRY(gfail(g, 0, ensure_buf(g->m[0], t->roots, (2 * G - 1) * 32)));
  std::vector<const uint8_t*> send(G);
  for (size_t r = 0; r < G; ++r) send[r] = merkle_root_dev(t->sub[r]);
  uint8_t* lv = (uint8_t*)t->roots.ptr;
  STARK_TRY(gather_to0(g, send.data(), lv, 32));
  STARK_TRY(gfail(g, 0, stark_merkle_top_dev(g->m[0], lv, G, lv + 32 * G, nullptr)));
  t->levels.resize((2 * G - 1) * 32);
  G_HIP(g, hipSetDevice(g->m[0]->device));
  G_HIP(g, hipMemcpyAsync(t->levels.data(), lv, t->levels.size(), hipMemcpyDeviceToHost, stream_of(g, 0)));
  STARK_TRY(sync_all(g));
  memcpy(t->root, t->levels.data() + t->levels.size() - 32, 32);
  return STARK_OK;
}

stark_status tree_prepare(stark_group_tree* t, size_t n, size_t leaf_len) {
  stark_group* g = t->g;
  const size_t G = g->m.size();
  if (n == 0 || (n & (n - 1))) return STARK_ERR_BAD_LENGTH;  // merkle_proof_in_place.rs:113
  g->last_error.clear();
  t->n = n;
  t->leaf_len = leaf_len;
  t->depth = log2_exact(n);
  t->split = G > 1 && n >= G;
  t->m = t->split ? n / G : n;
  t->built = t->has_root = false;
  return STARK_OK;
}

// ---- prover --------------------------------------------------------------------------------------
// A Merkle tree over n leaves held by residue class (member r: leaves r + G j), stark_amd/dprove.py
// DistTree: digests hashed where the leaves are, one all-to-all of digests, member s builds the subtree of
// leaves [s P, (s+1) P), the subtree roots gathered to every member, and the top levels hashed on each
// (every member's next step reads the root on its own stream).
struct DTree {
  bool blocked = false;
  size_t n = 0, nl = 0, leaf_len = 0;
  std::vector<const uint8_t*> leaves;
  std::vector<stark_merkle_tree*> t;
  std::vector<uint8_t*> levels;  // blocked: G roots then the G - 1 above (root last); else the root
  std::vector<uint8_t> host;
  const uint8_t* d_root(size_t r, size_t G) const { return levels[r] + (blocked ? (2 * G - 2) * 32 : 0); }
  const uint8_t* root() const { return host.data() + host.size() - 32; }
  size_t level_width(size_t G, uint32_t lvl) const { return G >> lvl; }
  const uint8_t* level_node(size_t G, uint32_t lvl, size_t i) const {
    size_t at = 0;
    for (uint32_t l = 0; l < lvl; ++l) at += G >> l;
    return host.data() + 32 * (at + i);
  }
};

stark_status dtree_commit(stark_group* g, DTree& d, const std::vector<const uint8_t*>& leaves, size_t nl,
                          size_t leaf_len) {
  const size_t G = g->m.size();
  d.leaves = leaves;
  d.nl = nl;
  d.n = nl * G;
  d.leaf_len = leaf_len;
  d.blocked = nl % G == 0;
  d.t.assign(G, nullptr);
  d.levels.assign(G, nullptr);
  std::vector<uint8_t*> dig(G), recv(G), mine(G);
  for (size_t r = 0; r < G; ++r) {
    void* p;
    STARK_TRY(take(g, r, nl * 32, &p));
    dig[r] = (uint8_t*)p;
    STARK_TRY(take(g, r, d.blocked ? nl * 32 : d.n * 32, &p));
    recv[r] = (uint8_t*)p;
    STARK_TRY(take(g, r, (2 * G - 1) * 32, &p));
    d.levels[r] = (uint8_t*)p;
    STARK_TRY(take_tree(g, r, &d.t[r]));
    STARK_TRY(gfail(g, r, stark_merkle_leaf_digests_dev(g->m[r], leaves[r], nl, leaf_len, dig[r], nullptr)));
  }
  std::vector<const uint8_t*> send(dig.begin(), dig.end());
  if (!d.blocked) {
    // few leaves: every member builds the whole tree from all the digests
    STARK_TRY(exchange(g, send.data(), recv.data(), nl * 32, true));
    for (size_t r = 0; r < G; ++r) {
      STARK_TRY(gfail(g, r, stark_merkle_update_digests_dev(d.t[r], recv[r], d.n, (uint32_t)G, nullptr)));
      STARK_TRY(gfail(g, r, stark_merkle_root_dev(d.t[r], d.levels[r], nullptr)));
    }
    return STARK_OK;
  }
  STARK_TRY(exchange(g, send.data(), recv.data(), nl / G * 32, false));
  for (size_t r = 0; r < G; ++r)
    STARK_TRY(gfail(g, r, stark_merkle_update_digests_dev(d.t[r], recv[r], nl, (uint32_t)G, nullptr)));
  for (size_t r = 0; r < G; ++r) send[r] = merkle_root_dev(d.t[r]);
  STARK_TRY(exchange(g, send.data(), d.levels.data(), 32, true));
  for (size_t r = 0; r < G; ++r)
    STARK_TRY(gfail(g, r, stark_merkle_top_dev(g->m[r], d.levels[r], G, d.levels[r] + 32 * G, nullptr)));
  return STARK_OK;
}

// Openings of `idx` from a DTree: member (i mod G) holds leaf i, member (i / P) its lower path (member 0
// the whole path of an unblocked tree), the top levels come from the downloaded roots.
struct DOpen {
  const DTree* d = nullptr;
  std::vector<size_t> idx;
  std::vector<std::vector<size_t>> leaf_local, path_local;  // per member
  std::vector<std::vector<uint8_t>> leaf_out, path_out;     // per member
  std::vector<uint8_t> leaves, nodes;                        // assembled, k x leaf_len / k x depth x 32
};

void dopen_plan(DOpen& o, const DTree& d, std::vector<size_t> idx, size_t G) {
  o.d = &d;
  o.idx = std::move(idx);
  o.leaf_local.assign(G, {});
  o.path_local.assign(G, {});
  for (size_t i : o.idx) {
    o.leaf_local[i % G].push_back(i / G);
    if (d.blocked) {
      o.path_local[i / d.nl].push_back(i % d.nl);
    } else {
      o.path_local[0].push_back(i);
    }
  }
  o.leaf_out.assign(G, {});
  o.path_out.assign(G, {});
  const uint32_t low = d.blocked ? log2_exact(d.nl) : log2_exact(d.n);
  for (size_t r = 0; r < G; ++r) {
    o.leaf_out[r].resize(o.leaf_local[r].size() * d.leaf_len);
    o.path_out[r].resize(o.path_local[r].size() * low * 32);
  }
}

void dopen_assemble(DOpen& o, size_t G) {
  const DTree& d = *o.d;
  const size_t k = o.idx.size();
  const uint32_t depth = log2_exact(d.n), low = d.blocked ? log2_exact(d.nl) : depth;
  o.leaves.resize(k * d.leaf_len);
  o.nodes.resize(k * depth * 32);
  std::vector<size_t> at_leaf(G, 0), at_path(G, 0);
  for (size_t q = 0; q < k; ++q) {
    const size_t i = o.idx[q];
    const size_t lr = i % G;
    memcpy(o.leaves.data() + q * d.leaf_len, o.leaf_out[lr].data() + (at_leaf[lr]++) * d.leaf_len, d.leaf_len);
    const size_t pr = d.blocked ? i / d.nl : 0;
    uint8_t* nd = o.nodes.data() + q * depth * 32;
    memcpy(nd, o.path_out[pr].data() + (at_path[pr]++) * low * 32, low * 32);
    if (d.blocked) {
      size_t pos = i / d.nl;
      for (uint32_t l = 0; low + l < depth; ++l, pos >>= 1) memcpy(nd + (low + l) * 32, d.level_node(G, l, pos ^ 1), 32);
    }
  }
}

// serde_json of the StarkProof (utils.rs:122-130, run.rs:549) from the proof's fields.
void render_proof(stark_r1cs_proof* p, size_t k_main, size_t k_l) {
  JsonPieces j;
  j.text("{\"m_root\":");
  j.bytes(p->m_root, 32);
  j.text(",\"l_root\":");
  j.bytes(p->l_root, 32);
  j.text(",\"a_root\":");
  j.bytes(p->a_root, 32);
  j.text(",\"main_branches\":");
  j.branches(p->m_leaves, 256, p->m_nodes, k_main, p->depth);
  j.text(",\"linear_comb_branches\":");
  j.branches(p->l_leaves, 32, p->l_nodes, k_l, p->depth);
  j.text(",\"fri_proof\":");
  fri_proof_json_pieces(p->fri, j);
  j.text("}");
  j.render(p->json);
}

constexpr size_t kExt = 8;         // r1cs-stark/src/utils.rs:135 (extension factor; FRI excludes its multiples)
constexpr size_t kSpot = 80;       // utils.rs:136
constexpr uint32_t kFriTailLog = 16;  // layers of <= 2^16 values: member 0 proves the rest alone

struct DProveHandles {
  std::vector<stark_dprove*> h;
  ~DProveHandles() {
    for (stark_dprove* x : h) stark_dprove_free(x);
  }
};

stark_status indices(const uint8_t* seed, size_t modulus, size_t count, uint32_t excl, std::vector<size_t>& out) {
  std::vector<uint32_t> v(count);
  STARK_TRY(stark_get_pseudorandom_indices(seed, 32, (uint32_t)modulus, count, excl, v.data()));
  out.assign(v.begin(), v.end());
  return STARK_OK;
}

// prove_with_witness (run.rs:310-452) = mk_r1cs_proof (prove.rs:14-378) over the group; begin(r) starts
// member r's share (trace, coset LDEs, constraints; stark_dprove_begin_*).
template <class Begin>
stark_status group_prove(stark_group* g, Begin&& begin, stark_r1cs_proof** out) {
  const size_t G = g->m.size();
  const FieldHost& F = FieldHost::get();
  reset_cursors(g);
  DProveHandles hs;
  hs.h.assign(G, nullptr);
  std::vector<size_t> prec(G), nl(G), os(G);
  std::vector<std::array<uint64_t, 4>> g2(G);
  std::vector<std::array<uint8_t, 32>> a_root(G);
  // trace, LDE and constraints on every member at once (each call ends with its stream synchronised)
  STARK_TRY(for_members(g, [&](size_t r) {
    STARK_TRY(begin(r, &hs.h[r]));
    return stark_dprove_info(hs.h[r], &prec[r], &nl[r], &os[r], g2[r].data(), a_root[r].data());
  }));
  const size_t P = prec[0], n_local = nl[0], osteps = os[0];
  const uint32_t log_prec = log2_exact(P);
  std::vector<const uint8_t*> rows(G), lv(G);
  for (size_t r = 0; r < G; ++r) {
    uint8_t* p = nullptr;
    STARK_TRY(gfail(g, r, stark_dprove_rows(hs.h[r], &p)));
    rows[r] = p;
  }
  // main tree over the 256-B rows (prove.rs:235-264) -> k -> L (prove.rs:274-322) -> L tree; each
  // root is read on the device by the next step
  DTree main, ltree;
  STARK_TRY(dtree_commit(g, main, rows, n_local, 256));
  for (size_t r = 0; r < G; ++r) {
    uint64_t* l = nullptr;
    STARK_TRY(gfail(g, r, stark_dprove_lincomb_dev(hs.h[r], main.d_root(r, G), &l)));
    lv[r] = (const uint8_t*)l;
  }
  STARK_TRY(dtree_commit(g, ltree, lv, n_local, 32));
  // prove_low_degree(L, g2, precision / 4, 8) (prove.rs:367, fri.rs:46-224), layer by layer while the
  // layers are large; the fold's special_x comes from the previous tree's root on the device
  struct Layer {
    DTree t2;
    const DTree* mt;
    size_t q;
  };
  std::vector<std::unique_ptr<Layer>> layers;
  std::vector<const uint8_t*> vals = lv;
  size_t n = P, deg = P / 4;
  HostFp w = F.from_canonical(g2[0].data());
  const DTree* mtree = &ltree;
  while (deg > 16 && n > ((size_t)1 << kFriTailLog)) {
    const size_t q = n / 4;
    uint64_t wc[4];
    canon(w, wc);
    std::vector<const uint8_t*> col(G);
    for (size_t r = 0; r < G; ++r) {
      void* p;
      STARK_TRY(take(g, r, q / G * 32, &p));
      col[r] = (const uint8_t*)p;
      STARK_TRY(gfail(g, r, stark_fri_fold_dev_root(g->m[r], (const uint64_t*)vals[r], (uint64_t*)p, n, wc,
                                                     mtree->d_root(r, G), (uint32_t)G, (uint32_t)r, nullptr)));
    }
    auto L = std::make_unique<Layer>();
    STARK_TRY(dtree_commit(g, L->t2, col, q / G, 32));
    L->mt = mtree;
    L->q = q;
    mtree = &L->t2;
    layers.push_back(std::move(L));
    vals = col;
    n = q;
    w = F.pow_u64(w, 4);
    deg /= 4;
  }
  // every tree's top levels (member 0) and the last layer's values (every member), one download each
  std::vector<DTree*> trees = {&main, &ltree};
  for (auto& L : layers) trees.push_back(&L->t2);
  for (DTree* t : trees) t->host.resize(t->blocked ? (2 * G - 1) * 32 : 32);
  const size_t nv = n / G;
  std::vector<uint8_t> last_local(G * nv * 32);
  G_HIP(g, hipSetDevice(g->m[0]->device));
  for (DTree* t : trees)
    G_HIP(g, hipMemcpyAsync(t->host.data(), t->levels[0], t->host.size(), hipMemcpyDeviceToHost, stream_of(g, 0)));
  for (size_t r = 0; r < G; ++r) {
    G_HIP(g, hipSetDevice(g->m[r]->device));
    G_HIP(g, hipMemcpyAsync(last_local.data() + r * nv * 32, vals[r], nv * 32, hipMemcpyDeviceToHost,
                            stream_of(g, r)));
  }
  STARK_TRY(sync_all(g));
  // the transcript: spot-check positions from l_root (prove.rs:337-362), each layer's ys from its root2
  const size_t skips = kExt;
  std::vector<size_t> positions, aug;
  STARK_TRY(indices(ltree.root(), P, kSpot, (uint32_t)skips, positions));
  for (size_t j : positions) {
    aug.push_back(j);
    aug.push_back((j + P - skips) % P);
    aug.push_back((j + osteps / 3 * skips) % P);
    aug.push_back((j + osteps / 3 * 2 * skips) % P);
  }
  std::vector<DOpen> opens(2 + 2 * layers.size());
  dopen_plan(opens[0], main, aug, G);
  dopen_plan(opens[1], ltree, positions, G);
  for (size_t li = 0; li < layers.size(); ++li) {
    const Layer& L = *layers[li];
    std::vector<size_t> ys, poly;
    STARK_TRY(indices(L.t2.root(), L.q, 40, (uint32_t)skips, ys));  // fri.rs:181-189
    for (size_t y : ys)
      for (size_t j = 0; j < 4; ++j) poly.push_back(y + L.q * j);   // fri.rs:193-204
    dopen_plan(opens[2 + 2 * li], L.t2, ys, G);
    dopen_plan(opens[3 + 2 * li], *L.mt, poly, G);
  }
  // every member gathers what it holds in one zero-copy launch
  STARK_TRY(for_members(g, [&](size_t r) {
    std::vector<stark_open_req> reqs;
    for (DOpen& o : opens) {
      const DTree& d = *o.d;
      stark_open_req a{};
      a.d_rows = d.leaves[r];
      a.row_bytes = d.leaf_len;
      a.n_rows = d.nl;
      a.idx = o.leaf_local[r].data();
      a.k = o.leaf_local[r].size();
      a.leaves_out = o.leaf_out[r].data();
      reqs.push_back(a);
      stark_open_req b{};
      b.tree = d.t[r];
      b.idx = o.path_local[r].data();
      b.k = o.path_local[r].size();
      b.nodes_out = o.path_out[r].data();
      reqs.push_back(b);
    }
    return stark_open_batch(g->m[r], reqs.data(), reqs.size(), nullptr);
  }));
  for (DOpen& o : opens) dopen_assemble(o, G);
  // the proof
  auto proof = std::make_unique<stark_r1cs_proof>();
  memcpy(proof->a_root, a_root[0].data(), 32);
  memcpy(proof->m_root, main.root(), 32);
  memcpy(proof->l_root, ltree.root(), 32);
  proof->depth = log_prec;
  proof->m_leaves = std::move(opens[0].leaves);
  proof->m_nodes = std::move(opens[0].nodes);
  proof->l_leaves = std::move(opens[1].leaves);
  proof->l_nodes = std::move(opens[1].nodes);
  auto fri = std::make_unique<stark_fri_proof>();
  for (size_t li = 0; li < layers.size(); ++li) {
    stark_fri_layer L;
    memcpy(L.root2, layers[li]->t2.root(), 32);
    DOpen& c = opens[2 + 2 * li];
    DOpen& p = opens[3 + 2 * li];
    L.col_idx = c.idx;
    L.poly_idx = p.idx;
    L.col_depth = log2_exact(layers[li]->t2.n);
    L.poly_depth = log2_exact(layers[li]->mt->n);
    L.col_leaves = std::move(c.leaves);
    L.col_nodes = std::move(c.nodes);
    L.poly_leaves = std::move(p.leaves);
    L.poly_nodes = std::move(p.nodes);
    fri->layers.push_back(std::move(L));
  }
  // the last distributed layer's values in natural order (value r + G j is member r's j-th)
  std::vector<uint8_t> values(n * 32);
  for (size_t r = 0; r < G; ++r)
    for (size_t j = 0; j < nv; ++j) memcpy(values.data() + (r + G * j) * 32, last_local.data() + (r * nv + j) * 32, 32);
  if (deg <= 16) {  // fri.rs:65-77: Last
    stark_fri_layer L;
    L.last = true;
    L.last_values = std::move(values);
    fri->layers.push_back(std::move(L));
  } else {  // the rest of prove_low_degree_rec on member 0
    uint64_t wc[4];
    canon(w, wc);
    stark_fri_proof* tail = nullptr;
    STARK_TRY(gfail(g, 0, stark_prove_low_degree(g->m[0], (const uint64_t*)values.data(), n, wc, deg,
                                                 (uint32_t)skips, &tail)));
    for (auto& L : tail->layers) fri->layers.push_back(std::move(L));
    stark_fri_proof_free(tail);
  }
  proof->fri = fri.release();
  render_proof(proof.get(), aug.size(), positions.size());
  *out = proof.release();
  return STARK_OK;
}

}  // namespace
}  // namespace stark

using namespace stark;

extern "C" {

stark_status stark_group_create(const int* devices, uint32_t g, stark_group** out) {
  if (!devices || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  if (g == 0 || (g & (g - 1)) || g > 8) return STARK_ERR_BAD_ARG;
  auto grp = std::make_unique<stark_group>();
  for (uint32_t r = 0; r < g; ++r) {
    stark_ctx* c = nullptr;
    const stark_status st = stark_ctx_create(devices[r], &c);
    if (st != STARK_OK) {
      for (stark_ctx* x : grp->m) stark_ctx_destroy(x);
      return st;
    }
    grp->m.push_back(c);
  }
  // peer access between distinct devices (xGMI); the copies also work without it (staged by the runtime)
  for (uint32_t a = 0; a < g; ++a)
    for (uint32_t b = 0; b < g; ++b) {
      const int da = devices[a], db = devices[b];
      if (da == db) continue;
      int can = 0;
      if (hipDeviceCanAccessPeer(&can, da, db) == hipSuccess && can) {
        hipSetDevice(da);
        const hipError_t e = hipDeviceEnablePeerAccess(db, 0);
        if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled) {
          for (stark_ctx* x : grp->m) stark_ctx_destroy(x);
          return STARK_ERR_HIP;
        }
        hipGetLastError();  // (an already-enabled pair leaves a sticky-looking status)
      }
    }
  grp->ready.assign(g, nullptr);
  grp->copied.assign(g, nullptr);
  for (uint32_t r = 0; r < g; ++r) {
    hipSetDevice(devices[r]);
    if (hipEventCreateWithFlags(&grp->ready[r], hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&grp->copied[r], hipEventDisableTiming) != hipSuccess) {
      stark_group_destroy(grp.release());
      return STARK_ERR_HIP;
    }
  }
  grp->slots.assign(g, {});
  grp->trees.assign(g, {});
  grp->slot_at.assign(g, 0);
  grp->tree_at.assign(g, 0);
  grp->pinned.assign(g, nullptr);
  grp->pinned_bytes.assign(g, 0);
  grp->workers.start(g);
  *out = grp.release();
  return STARK_OK;
}

void stark_group_destroy(stark_group* g) {
  if (!g) return;
  for (size_t r = 0; r < g->m.size(); ++r) {
    hipSetDevice(g->m[r]->device);
    hipStreamSynchronize(g->m[r]->stream);
    if (r < g->slots.size())
      for (DevBuf& b : g->slots[r])
        if (b.ptr) hipFree(b.ptr);
    if (r < g->trees.size())
      for (stark_merkle_tree* t : g->trees[r]) stark_merkle_free(t);
    if (r < g->ready.size() && g->ready[r]) hipEventDestroy(g->ready[r]);
    if (r < g->copied.size() && g->copied[r]) hipEventDestroy(g->copied[r]);
    if (r < g->pinned.size() && g->pinned[r]) hipHostFree(g->pinned[r]);
  }
  for (stark_ctx* c : g->m) stark_ctx_destroy(c);
  delete g;
}

uint32_t stark_group_size(const stark_group* g) { return g ? (uint32_t)g->m.size() : 0; }

stark_ctx* stark_group_ctx(stark_group* g, uint32_t i) { return g && i < g->m.size() ? g->m[i] : nullptr; }

const char* stark_group_last_error(const stark_group* g) { return g ? g->last_error.c_str() : ""; }

stark_status stark_group_synchronize(stark_group* g) {
  if (!g) return STARK_ERR_BAD_ARG;
  return sync_all(g);
}

stark_status stark_group_best_fft(stark_group* g, const uint64_t* coeffs, size_t len, const uint64_t root[4],
                                  uint32_t log_n, uint64_t* out) {
  return group_fft_host(g, coeffs, len, root, log_n, out, false);
}

stark_status stark_group_inv_best_fft(stark_group* g, const uint64_t* evals, size_t len, const uint64_t root[4],
                                      uint32_t log_n, uint64_t* out) {
  return group_fft_host(g, evals, len, root, log_n, out, true);
}

stark_status stark_group_ntt_dev(stark_group* g, uint64_t* const* d_shards, uint64_t* const* d_out, uint32_t log_n,
                                 const uint64_t root[4], int inverse) {
  if (!g || !d_shards || !d_out || !root) return STARK_ERR_BAD_ARG;
  for (size_t r = 0; r < g->m.size(); ++r)
    if (!d_shards[r] || !d_out[r] || d_shards[r] == d_out[r]) return STARK_ERR_BAD_ARG;
  g->last_error.clear();
  if (g->m.size() == 1) {
    STARK_TRY(gfail(g, 0, stark_ntt_dev(g->m[0], d_shards[0], log_n, 1, root, inverse, nullptr)));
    G_HIP(g, hipSetDevice(g->m[0]->device));
    G_HIP(g, hipMemcpyAsync(d_out[0], d_shards[0], ((size_t)1 << log_n) * sizeof(fe), hipMemcpyDeviceToDevice,
                            g->m[0]->stream));
    return STARK_OK;
  }
  return group_ntt(g, d_shards, d_out, log_n, root, inverse != 0);
}

stark_status stark_group_merkle_new(stark_group* g, stark_group_tree** out) {
  if (!g || !out) return STARK_ERR_BAD_ARG;
  auto t = std::make_unique<stark_group_tree>();
  t->g = g;
  t->log_g = log2_exact(g->m.size());
  for (size_t r = 0; r < g->m.size(); ++r) {
    stark_merkle_tree* s = nullptr;
    const stark_status st = stark_merkle_new(g->m[r], &s);
    if (st != STARK_OK) {
      stark_group_merkle_free(t.release());
      return st;
    }
    t->sub.push_back(s);
  }
  *out = t.release();
  return STARK_OK;
}

void stark_group_merkle_free(stark_group_tree* t) {
  if (!t) return;
  for (stark_merkle_tree* s : t->sub) stark_merkle_free(s);
  if (t->roots.ptr) {
    hipSetDevice(t->g->m[0]->device);
    hipFree(t->roots.ptr);
  }
  delete t;
}

stark_status stark_group_merkle_update(stark_group_tree* t, const uint8_t* leaves, size_t n, size_t leaf_len) {
  if (!t || (!leaves && n * leaf_len)) return STARK_ERR_BAD_ARG;
  STARK_TRY(tree_prepare(t, n, leaf_len));
  stark_group* g = t->g;
  if (!t->split) {
    STARK_TRY(gfail(g, 0, stark_merkle_update(t->sub[0], leaves, n, leaf_len)));
  } else {
    const size_t blk = t->m * leaf_len;
    STARK_TRY(for_members(g, [&](size_t r) { return stark_merkle_update(t->sub[r], leaves + r * blk, t->m, leaf_len); }));
  }
  STARK_TRY(tree_top(t));
  t->built = true;
  return STARK_OK;
}

stark_status stark_group_merkle_update_dev(stark_group_tree* t, const uint8_t* const* d_blocks, size_t n,
                                           size_t leaf_len) {
  if (!t || !d_blocks) return STARK_ERR_BAD_ARG;
  STARK_TRY(tree_prepare(t, n, leaf_len));
  stark_group* g = t->g;
  const size_t members = t->split ? g->m.size() : 1;
  for (size_t r = 0; r < members; ++r) {
    if (!d_blocks[r] && leaf_len) return STARK_ERR_BAD_ARG;
    STARK_TRY(gfail(g, r, stark_merkle_update_dev(t->sub[r], d_blocks[r], t->m, leaf_len, nullptr)));
  }
  STARK_TRY(tree_top(t));
  t->built = true;
  return STARK_OK;
}

size_t stark_group_merkle_width(const stark_group_tree* t) { return t ? t->n : 0; }

stark_status stark_group_merkle_get_root(const stark_group_tree* t, uint8_t root[32], size_t* root_len) {
  if (!t || !root_len) return STARK_ERR_BAD_ARG;
  if (!t->has_root) {
    *root_len = 0;
    return STARK_OK;
  }
  if (root) memcpy(root, t->root, 32);
  *root_len = 32;
  return STARK_OK;
}

stark_status stark_group_merkle_gen_proofs(stark_group_tree* t, const size_t* indices, size_t k, uint8_t* leaves_out,
                                           uint8_t* nodes_out) {
  if (!t || (k && (!indices || !leaves_out || !nodes_out))) return STARK_ERR_BAD_ARG;
  if (!t->built) return STARK_ERR_STATE;
  stark_group* g = t->g;
  const size_t G = t->split ? g->m.size() : 1;
  for (size_t q = 0; q < k; ++q)
    if (indices[q] >= t->n) return STARK_ERR_BAD_ARG;
  const uint32_t low = log2_exact(t->m);
  std::vector<std::vector<size_t>> local(G);
  for (size_t q = 0; q < k; ++q) local[indices[q] / t->m].push_back(indices[q] % t->m);
  std::vector<std::vector<uint8_t>> lv(G), nd(G);
  for (size_t r = 0; r < G; ++r) {
    lv[r].resize(local[r].size() * t->leaf_len + 1);
    nd[r].resize(local[r].size() * low * 32 + 1);
  }
  STARK_TRY(for_members(g, [&](size_t r) {
    if (r >= G || local[r].empty()) return STARK_OK;
    return stark_merkle_gen_proofs(t->sub[r], local[r].data(), local[r].size(), lv[r].data(), nd[r].data());
  }));
  std::vector<size_t> at(G, 0);
  for (size_t q = 0; q < k; ++q) {
    const size_t r = indices[q] / t->m, a = at[r]++;
    memcpy(leaves_out + q * t->leaf_len, lv[r].data() + a * t->leaf_len, t->leaf_len);
    uint8_t* o = nodes_out + q * t->depth * 32;
    memcpy(o, nd[r].data() + a * low * 32, low * 32);
    size_t pos = r, at_lvl = 0;
    for (uint32_t l = 0; low + l < t->depth; ++l) {  // siblings of the subtree root up to the top
      memcpy(o + (low + l) * 32, t->levels.data() + 32 * (at_lvl + (pos ^ 1)), 32);
      at_lvl += G >> l;
      pos >>= 1;
    }
  }
  t->has_root = true;
  return STARK_OK;
}

stark_status stark_group_prove_r1cs_bytes(stark_group* g, const uint8_t* r1cs, size_t r1cs_len, const uint8_t* wtns,
                                          size_t wtns_len, stark_r1cs_proof** out) {
  if (!g || !r1cs || !wtns || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  g->last_error.clear();
  if (g->m.size() == 1) return gfail(g, 0, stark_prove_r1cs_bytes(g->m[0], r1cs, r1cs_len, wtns, wtns_len, out));
  const uint32_t G = (uint32_t)g->m.size();
  // The host stage of the trace build (headers, record walk, uploads) runs once, on member 0; the others
  // copy its raw bytes and walk tables device to device and build their own traces from them
  // (r1cs_trace_device's producer / consumer modes), instead of G walks queued on the one host pool.
  TraceShare share;
  const stark_status st = group_prove(
      g,
      [&](size_t r, stark_dprove** h) {
        stark_ctx* c = g->m[r];
        if (hipSetDevice(c->device) != hipSuccess) {
          if (r == 0) {  // (the consumers wait for member 0's publication)
            share.status = STARK_ERR_HIP;
            share.ready_p.set_value();
          }
          return STARK_ERR_HIP;
        }
        DevTrace dt;
        STARK_TRY(r1cs_trace_device(c, r1cs, r1cs_len, wtns, wtns_len, &dt, false, &share, r == 0));
        return dprove_begin_trace(c, G, (uint32_t)r, dt, nullptr, h);
      },
      out);
  if (share.ev) hipEventDestroy(share.ev);
  return st;
}

stark_status stark_group_circuit_new(stark_group* g, const uint8_t* r1cs, size_t r1cs_len,
                                     stark_r1cs_circuit** circuits) {
  if (!g || !r1cs || !circuits) return STARK_ERR_BAD_ARG;
  const uint32_t G = (uint32_t)g->m.size();
  for (uint32_t r = 0; r < G; ++r) circuits[r] = nullptr;
  g->last_error.clear();
  const stark_status st = for_members(g, [&](size_t r) {
    return G == 1 ? stark_r1cs_circuit_new(g->m[0], r1cs, r1cs_len, &circuits[0])
                  : stark_dprove_circuit_new(g->m[r], G, (uint32_t)r, r1cs, r1cs_len, &circuits[r]);
  });
  if (st != STARK_OK)
    for (uint32_t r = 0; r < G; ++r) {
      stark_r1cs_circuit_free(circuits[r]);
      circuits[r] = nullptr;
    }
  return st;
}

stark_status stark_group_prove_r1cs_circuit(stark_group* g, stark_r1cs_circuit* const* circuits, const uint8_t* wtns,
                                            size_t wtns_len, stark_r1cs_proof** out) {
  if (!g || !circuits || !wtns || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  g->last_error.clear();
  const size_t G = g->m.size();
  for (size_t r = 0; r < G; ++r)
    if (!circuits[r] || circuits[r]->ctx != g->m[r] || circuits[r]->c.world != G || circuits[r]->c.rank != r)
      return STARK_ERR_BAD_ARG;
  if (G == 1) return gfail(g, 0, stark_prove_r1cs_circuit(g->m[0], circuits[0], wtns, wtns_len, out));
  return group_prove(
      g,
      [&](size_t r, stark_dprove** h) {
        return stark_dprove_begin_circuit(g->m[r], circuits[r], wtns, wtns_len, nullptr, h);
      },
      out);
}

}  // extern "C"
