// Internal declarations shared by the HIP translation units of libstark_hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>

#include <functional>
#include <future>
#include <map>
#include <memory>
#include <string>
#include <tuple>
#include <vector>

#include "stark_hip.h"
#include "fp_dev.h"
#include "fp_host.h"
#include "host_pool.h"

namespace stark {

// STARK_PROFILE=1: host-side phase timings of a call on stderr (what the
// host waits on between the device phases; the kernels themselves are timed
// with rocprofv3).
struct PhaseClock {
  bool on;
  std::chrono::steady_clock::time_point t0, last;
  explicit PhaseClock(const char* what) : on(enabled()) {
    if (on) {
      t0 = last = std::chrono::steady_clock::now();
      fprintf(stderr, "[stark] %s\n", what);
    }
  }
  static bool enabled() {
    static const bool e = [] {
      const char* v = getenv("STARK_PROFILE");
      return v && v[0] && v[0] != '0';
    }();
    return e;
  }
  void mark(const char* phase) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    fprintf(stderr, "[stark]   %-28s %8.1f us (at %8.1f)\n", phase,
            std::chrono::duration<double, std::micro>(now - last).count(),
            std::chrono::duration<double, std::micro>(now - t0).count());
    last = now;
  }
};

// Device buffer owned by a context.  A context buffer that calls on different streams share (the NTT
// ping-pong, the batch inverse's scratch, the fold's special_x slot, ...) also carries the stream of
// its last enqueued use: buf_acquire makes a call on another stream wait for everything enqueued on
// that one (an event recorded there at that moment), buf_release notes the stream (api.hip).
struct DevBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  hipEvent_t ev = nullptr;
  hipStream_t last = nullptr;
};

// Twiddle set for one (root, log_n): everything in Montgomery form.
//   lo[i] = w^i                   i < 2^kb
//   hi[i] = w^(i * 2^kb)          i < 2^(log_n - kb)
//   small_off[l] = offset (in fe) into `small` of the Shoup pairs of w_R^k = w^(k * n / R), k < R/2, R = 2^l
//     (k < R for R = 2^8)
struct Twiddles {
  uint32_t log_n = 0, kb = 0;
  fe* d_lo = nullptr;
  fe* d_hi = nullptr;
  fe* d_small = nullptr; // Shoup pairs (shoup_pair), 2 fe per root
  fe* d_t16 = nullptr;   // Shoup pairs of t16[i] = w^(i n / 2^l16), l16 = min(16, log_n) (18 from 2^25 on)
  fe* d_hi_s = nullptr;  // hi[i] * n^-1   (last pass of an inverse transform)
  fe* d_t16_s = nullptr; // Shoup pairs of t16[i] * n^-1
  uint32_t l16 = 0;
  uint32_t small_off[16] = {0};
  // Full column-twiddle table of the last pass (built on first use when that
  // pass's twiddles do not fit t16): full[c R + r] = w^(c r), c < n/R, r < R;
  // full_s = full * n^-1 for the inverse.  One product per element instead of
  // the two of lo * hi, for one 32-B coalesced read.
  fe* d_full = nullptr;
  fe* d_full_s = nullptr;
  uint64_t full_used = 0, full_s_used = 0;  // cache clock of their last use (LRU eviction, cache_reserve)
  // The fill of d_full / d_full_s ([1]) is enqueued on the stream of the call that first needs it;
  // a call on another stream waits for this event until the fill is known to be complete (fill = null).
  hipEvent_t full_ev[2] = {nullptr, nullptr};
  hipStream_t full_fill[2] = {nullptr, nullptr};
  size_t base_bytes = 0;         // device bytes of the tables above d_full (one allocation at d_lo)
  size_t n_small_pairs = 0;      // Shoup pairs in d_small
  // Digit-basis tables (fe_db.h) of w_R^k, k < R/2, for every radix R = 2^l >= 16: the constants of the
  // radix-4 steps (ntt.hip DbPlan).  db_off[l] = offset in u32 into d_db (72 u32 per root).
  uint32_t* d_db = nullptr;
  uint32_t db_off[16] = {0};
  HostFp root;      // the root these tables were built for (Montgomery)
  HostFp inv_n;     // n^-1 (Montgomery)
};

// A cached device buffer with the cache clock of its last use.
struct CacheBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
  uint64_t used = 0;
  bool in_use = false;          // held by a call in progress: never evicted (cache_reserve)
  hipEvent_t ev = nullptr;      // the fill's event while it may still run (stream `fill`), as Twiddles::full_ev
  hipStream_t fill = nullptr;
};

// Default cap on a context's cached tables (the last-pass full twiddle tables, 2^log_n x 32 B per
// direction, and the shared IDX extensions): both directions of a 2^26 transform.
constexpr size_t kDefaultCacheLimit = (size_t)4 << 30;

}  // namespace stark

struct stark_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  std::string last_error;
  stark::DevBuf scratch;   // NTT ping-pong partner
  stark::DevBuf io;        // staging for host-buffer entry points
  stark::DevBuf io2;
  stark::DevBuf fri_cols;    // folded FRI columns (prove_low_degree)
  stark::DevBuf r1cs_arena;  // mk_r1cs_proof working set
  stark::DevBuf trace_arena;  // device trace builder working set (r1cs_trace_dev.hip)
  stark::DevBuf trace_raw;    // the raw constraint section and witness bytes it reads
  stark::DevBuf lde_tmp;      // circuit_lde's step columns and Zb values
  stark::DevBuf verify_arena, verify_lde;  // the verifier's circuit, kept for the next call
  stark::DevBuf ext_idx_tmp;  // an IDX extension too large for the cache cap (this proof only)
  stark::DevBuf inv_tmp;      // the scratch of a second batch inverse sharing a host round trip (r1cs.hip)
  stark::DevBuf spot;         // circuit_spot_values' tables and sums (r1cs.hip)
  // Merkle trees reused across calls: [0, 1] FRI layer ping-pong, [2..4] the
  // accumulator, main and linear-combination trees of mk_r1cs_proof.
  stark_merkle_tree* trees[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  std::vector<stark_merkle_tree*> fri_trees;  // one per FRI layer (+ the input's), reused across proofs
  stark::DevBuf fri_misc;                     // per-layer special_x (device transcript)
  void* pinned[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};  // pinned host scratch (ctx_pinned)
  size_t pinned_bytes[5] = {0, 0, 0, 0, 0};
  hipEvent_t staged = nullptr;  // the last DMA out of pinned slot 3 (r1cs_trace_dev.hip staged_upload)
  // A second stream and an event for work the host overlaps with the main stream (the prover's spot-check
  // openings gathered while its FRI layers still run, r1cs.hip); created on first use.
  hipStream_t aux = nullptr;
  hipEvent_t ev_aux = nullptr;
  // The device trace builder's deferred wire-id flag for the proof being built (stark_prove_r1cs_bytes).
  const uint32_t* trace_err = nullptr;
  // (root canonical limbs, log_n) -> tables
  std::map<std::tuple<uint64_t, uint64_t, uint64_t, uint64_t, uint32_t>, std::unique_ptr<stark::Twiddles>> tw;
  // (log_steps, log_prec, log_world, rank) -> the extension of the index column IDX[i] = i
  // (prove.rs:160-163) at that rank's points: it depends on the trace length only, so every
  // proof of that size shares it (r1cs.hip ext_index_column).
  // Size-only columns of the r1cs prover (r1cs.hip ext_const_column), key (kind, log_steps, log_prec,
  // log_g, rank, os): kind 0 = IDX's extension, 1 = F0's (1 on the first os rows), 2 = 1 / Zb3.
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t, uint32_t, uint64_t>, stark::CacheBuf> ext_idx;
  // (root canonical limbs, log_n, rank) -> post[k] = root^(rank k), k < n / world: the one-exchange
  // distributed NTT's twiddle, applied in the rank's last local pass (dist.hip).
  std::map<std::tuple<uint64_t, uint64_t, uint64_t, uint64_t, uint32_t, uint32_t>, stark::CacheBuf> post_tw;
  // Cached tables (full twiddle tables + ext_idx) stay under cache_limit bytes: least recently used
  // ones are freed first (stark::cache_reserve).  stark_ctx_set_cache_limit changes it.
  size_t cache_limit = stark::kDefaultCacheLimit;
  uint64_t cache_clock = 0;
};

namespace stark {

stark_status hip_fail(stark_ctx* ctx, hipError_t e, const char* what);
#define STARK_HIP(ctx, call)                                  \
  do {                                                        \
    hipError_t e_ = (call);                                   \
    if (e_ != hipSuccess) return ::stark::hip_fail(ctx, e_, #call); \
  } while (0)

#define STARK_TRY(expr)              \
  do {                               \
    stark_status st_ = (expr);       \
    if (st_ != STARK_OK) return st_; \
  } while (0)

// STARK_POISON=1: fill new device allocations with 0xA5 (api.hip; diagnostics only).
bool poison_on();
void poison_dev(void* p, size_t bytes);
stark_status ensure_buf(stark_ctx* ctx, DevBuf& b, size_t bytes);
// Cross-stream use of a context buffer (DevBuf::last): acquire before the first enqueued use on s (s
// waits for what the previous user's stream has enqueued so far), release after the last one.  A
// cached table filled on one stream and read on another: fill_mark records the fill's event, fill_wait
// makes another stream wait for it until it is known to be complete.
stark_status buf_acquire(stark_ctx* ctx, DevBuf& b, hipStream_t s);
stark_status buf_release(stark_ctx* ctx, DevBuf& b, hipStream_t s);
stark_status buf_drain(stark_ctx* ctx, DevBuf& b);  // host-waits for the last use's stream, forgets it
stark_status fill_wait(stark_ctx* ctx, hipEvent_t ev, hipStream_t& fill, hipStream_t s);
stark_status fill_mark(stark_ctx* ctx, hipEvent_t& ev, hipStream_t& fill, hipStream_t s);
// Bytes held by the context's cached tables (full twiddle tables and IDX extensions).
size_t cache_bytes(const stark_ctx* ctx);
// Makes room for `need` more cached bytes under ctx->cache_limit by freeing least recently used
// entries (after a device synchronisation: a kernel of any stream may still read them).  Full
// twiddle tables are always candidates; IDX extensions only with evict_ext (a proof's start, where
// no pointer into one is held).  False when the bytes cannot fit (the caller then does not cache).
bool cache_reserve(stark_ctx* ctx, size_t need, bool evict_ext);
// Context-owned pinned host scratch of at least `bytes` (async copy target).
// Slot 0: gather batches; slot 1: transcript values and roots; slot 2: the device trace builder's
// record-walk tables; slot 3: its upload staging (the raw .r1cs constraint section and witness); slot 4:
// the prover's small host-made uploads (constraint tables at 0, boundary constants from kPinned4ConstsOff),
// so they are asynchronous copies (a pageable copy blocks the host).
constexpr size_t kPinned4ConstsOff = 16384;
stark_status ctx_pinned(stark_ctx* ctx, int slot, size_t bytes, void** out);
// Pinned slot 1 (always this size, so no caller's pointer into it moves): [0, 2048) the prover's
// transcript head, [2048, 2560) FRI roots, [2560, 3584) two batch inverses' top levels, [3584, 3588) the
// trace builder's deferred flag, [4096, 16384) the last FRI layer's values.
constexpr size_t kPinned1Bytes = 16384;
constexpr size_t kPinned1InvTopOff = 2560;
constexpr size_t kPinned1TraceErrOff = 3584;
constexpr size_t kPinned1LastOff = 4096;

// Batch inverse (0 -> 0) in phases (field_ops.hip), so that one host round trip can serve two of them:
// multi_inv_up enqueues the up kernels, the caller synchronises its stream, multi_inv_top inverts the
// top level on the host, multi_inv_down enqueues the down kernels.  multi_inv_device does all four.
struct InvPlan {
  struct Level {
    uint64_t n;
    uint32_t chunk, wgs;
    const fe* in;
    fe *out, *pref, *others, *tot;
  };
  std::vector<Level> lv;
  fe* h_top = nullptr;
};
stark_status multi_inv_up(stark_ctx* ctx, const fe* d_in, fe* d_out, uint64_t n, hipStream_t s, DevBuf& buf,
                          fe* h_top, InvPlan& plan);
void multi_inv_top(const InvPlan& plan);
stark_status multi_inv_down(stark_ctx* ctx, const InvPlan& plan, hipStream_t s);
fe* multi_inv_h_top(stark_ctx* ctx, int k);  // top array k < 2 in pinned slot 1 (null: no pinned memory)
stark_status multi_inv_device(stark_ctx* ctx, const fe* d_in, fe* d_out, uint64_t n, hipStream_t s);

// Context-owned Merkle tree slot (created on first use).
stark_status ctx_tree(stark_ctx* ctx, int slot, stark_merkle_tree** out);
hipStream_t pick_stream(stark_ctx* ctx, void* stream);

// Returns tables for `root` (canonical limbs) of order exactly 2^log_n, or
// STARK_ERR_BAD_ROOT.  Cached per context.
stark_status get_twiddles(stark_ctx* ctx, const uint64_t root[4], uint32_t log_n, const Twiddles** out);

// Device NTT over `batch` contiguous transforms (in place, canonical values).
// post != nullptr: output k of each transform is multiplied by post[k] (Montgomery images, n entries)
// in the last pass's store (the one-exchange distributed NTT's twiddle, dist.hip).
stark_status ntt_device(stark_ctx* ctx, fe* d_data, uint32_t log_n, uint32_t batch, const Twiddles& tw,
                        bool inverse, hipStream_t stream, const fe* post = nullptr);
// Forward/inverse transform of src's batch columns of 2^(log_n - zero_log)
// elements, zero-extended to 2^log_n, into d_data (zero_log <= the plan's
// first radix); the zero tail is neither stored nor read.
uint32_t ntt_first_log_r(uint32_t log_n);  // log2 of the first pass's radix
stark_status ntt_device_from(stark_ctx* ctx, const fe* src, uint32_t zero_log, fe* d_data, uint32_t log_n,
                             uint32_t batch, const Twiddles& tw, bool inverse, hipStream_t stream,
                             const fe* post = nullptr);
// The forward transform's first pass alone over src's zero-extended columns (as ntt_device_from), stored
// transposed and canonical: out[c][t A + j] = sum_r src[c][j + r A] w_T^(r t), T = 2^*log_t (the plan's
// first radix), A = n / T, w_T = w^A.  Then X[c][i] = sum_j w^(i j) out[c][(i mod T) A + j]: one output of
// the whole transform is a dot product of length A over a contiguous run (the verifier's spot values).
stark_status ntt_first_pass_tmajor(stark_ctx* ctx, const fe* src, uint32_t zero_log, fe* out, uint32_t log_n,
                                   uint32_t batch, const Twiddles& tw, hipStream_t stream, uint32_t* log_t);

// First pass of a transform whose input is zero beyond its first n >> zero_log elements (best_fft's
// zero padding): skip = the number of leading radix-2 stages that are plain copies (<= zero_log,
// matching the pass's stage pairing); log_in = log2 of the compact input's batch stride.
struct Sparse {
  uint32_t skip, zero_log, log_in;
};

// Merkle internals (merkle.hip).
// Made by the kernel that makes a tree's root (merkle_build's root_fe, where that is the tail kernel; made
// tells whether it was): the root as a field element (fri.rs:135's special_x: the root's LE words reduced
// mod p, times r2) into *out, and the root's words into copy[0..8) (each when non-null).
struct RootFe {
  fe* out;
  fe r2;
  uint32_t* copy;
  bool made;
};
stark_status merkle_build(stark_ctx* ctx, stark_merkle_tree* t, const uint8_t* d_leaves, size_t n, size_t leaf_len,
                          hipStream_t stream, size_t plane_stride = 0, bool level0_ready = false,
                          RootFe* root_fe = nullptr);
stark_status merkle_level0(stark_ctx* ctx, stark_merkle_tree* t, size_t n, hipStream_t stream, uint32_t** level0);
stark_status merkle_root_d2h(stark_ctx* ctx, stark_merkle_tree* t, hipStream_t stream, uint8_t out[32]);
const uint8_t* merkle_root_dev(const stark_merkle_tree* t);
size_t merkle_device_bytes(const stark_merkle_tree* t);  // device memory the tree owns (0 for null)
stark_status merkle_gather(stark_ctx* ctx, stark_merkle_tree* t, const size_t* indices, size_t k,
                           uint8_t* leaves_out, uint8_t* nodes_out, hipStream_t stream, bool sync = true);

struct GatherReq {
  stark_merkle_tree* t;
  const size_t* idx;    // null: the indices are written on the device by `before_launch` (below)
  size_t k;
  uint8_t* leaves_out;  // k * leaf_len bytes
  uint8_t* nodes_out;   // k * depth * 32 bytes
};
// All requests in one pinned upload, one download, one synchronisation.  before_launch (optional) is
// called once the host's indices are in the pinned index array h_idx and before the gather is enqueued,
// with h_idx and each request's first slot in it; it enqueues on `stream` what writes the indices of
// the requests whose idx is null (they must be below the tree's leaf count).
using GatherHook = std::function<stark_status(uint64_t* h_idx, const std::vector<size_t>& first)>;
stark_status merkle_gather_batch(stark_ctx* ctx, const std::vector<GatherReq>& reqs, hipStream_t stream,
                                 const GatherHook& before_launch = GatherHook());

// A rendered JSON text: one uninitialised allocation written once (a std::string would be
// zero-filled first), so a multi-MB proof is assembled by several threads in parallel.
struct JsonText {
  std::unique_ptr<char[]> p;
  size_t n = 0;
  const char* data() const { return p.get(); }
  size_t size() const { return n; }
};

// serde_json text in pieces: fixed text, or a piece whose exact length is known before it is rendered
// (size) and which renders straight into its place (write: returns the end, writes nothing past it), so
// the whole text is sized once and its pieces written in parallel at their offsets (fri.hip).
struct JsonPieces {
  struct Piece {
    std::string text;                    // fixed (or prerendered) text when size is empty
    std::function<size_t()> size;
    std::function<char*(char*)> write;
  };
  std::vector<Piece> pieces;
  void text(const std::string& s);
  void bytes(const uint8_t* p, size_t n);  // p must outlive render()
  // rows of row_len bytes, "[..],[..]" (the caller writes the brackets)
  void byte_rows(const uint8_t* p, size_t rows, size_t row_len);
  void branches(const std::vector<uint8_t>& leaves, size_t leaf_len, const std::vector<uint8_t>& nodes, size_t k,
                size_t depth);
  void render(std::string& o);
  void render(JsonText& o);  // sized, then every piece written at its offset on the host workers
  // renders the pieces added so far into fixed text now (e.g. while the GPU still works)
  void prerender(unsigned max_threads = 16);
};
void fri_proof_json_pieces(const stark_fri_proof* proof, JsonPieces& j);

}  // namespace stark

// FRI and StarkProof values held by the library (fri.hip, r1cs.hip, group.hip).
struct stark_fri_layer {
  bool last = false;
  uint8_t root2[32];
  size_t col_depth = 0, poly_depth = 0;
  std::vector<size_t> col_idx, poly_idx;
  std::vector<uint8_t> col_leaves, col_nodes;    // 32 B leaves, depth*32 B paths
  std::vector<uint8_t> poly_leaves, poly_nodes;
  std::vector<uint8_t> last_values;              // n * 32 B
};

struct stark_fri_proof {
  std::vector<stark_fri_layer> layers;
};

struct stark_r1cs_proof {
  uint8_t m_root[32], l_root[32], a_root[32];
  stark::JsonText json;
  // The parts, for callers that build their own StarkProof value (stark_r1cs_proof_branches / _fri):
  // main and linear-combination openings (leaves, then depth siblings per opening, leaf to root).
  size_t depth = 0;
  std::vector<uint8_t> m_leaves, m_nodes, l_leaves, l_nodes;
  stark_fri_proof* fri = nullptr;
  ~stark_r1cs_proof() { stark_fri_proof_free(fri); }
};

namespace stark {

// R1CS v1 / wtns v2 headers (circom2bellman_core/src/reader.rs:4-89,
// r1cs-stark/src/reader.rs:7-42), r1cs_trace.hip.
struct R1csHeader {
  uint32_t n_wires, n_pub_out, n_pub_in, n_constraints;
  size_t cons_off;  // byte offset of the first constraint
};
struct WtnsHeader {
  uint32_t field_size, n_wit;
  size_t values_off;  // byte offset of witness value 0
};
stark_status parse_r1cs_header(const uint8_t* r1cs, size_t len, R1csHeader* h);
stark_status parse_wtns_header(const uint8_t* wtns, size_t len, WtnsHeader* h);

// The R1CS trace built on the device (r1cs_trace_dev.hip): the host
// builder's columns (coefficients, witness, computational as canonical
// elements; flags as bytes; permutation as u64 slots) in ctx->trace_arena,
// plus the small host-side public inputs.
struct DevTrace {
  size_t os = 0, n_constraints = 0, n_wires = 0;
  fe *coef = nullptr, *wit = nullptr, *comp = nullptr;
  uint8_t* flags = nullptr;
  uint64_t* perm = nullptr;
  std::vector<uint64_t> public_wires;       // canonical limbs, 4 per wire
  std::vector<size_t> public_first_indices;  // (wire, slot) pairs
  const uint32_t* d_err = nullptr;           // defer_err: the device's wire-id flag, not yet read
};
// A device trace build whose host part (headers, public wires, record walk, the upload of the raw bytes)
// runs once for several contexts: the producer (a group's member 0) does it all and publishes its
// results and its device copies of the raw bytes and walk tables; each consumer waits for `ready`, copies
// those from the producer's device (peer copies, stream-ordered behind `ev`) and builds its own columns.
struct TraceShare {
  R1csHeader hd{};
  WtnsHeader wh{};
  size_t n_public = 0, cons_len = 0, o_raw_w = 0, wbytes = 0, fac_n = 0, base_n = 0;
  uint64_t a_len = 0;
  std::vector<uint64_t> public_wires;
  bool pf_ok = false;
  std::vector<uint64_t> pf_host;
  stark_ctx* src = nullptr;             // the producer's context
  const uint8_t* raw = nullptr;         // its raw bytes (constraint section, then the witness at o_raw_w)
  const uint32_t *fac = nullptr, *base = nullptr;  // its walk tables (device)
  hipEvent_t ev = nullptr;              // recorded on the producer's stream behind those copies
  stark_status status = STARK_OK;       // the producer's host stage (consumers stop on an error)
  std::promise<void> ready_p;           // set once the fields above are final
  std::shared_future<void> ready = ready_p.get_future().share();
};
// defer_err: no read-back when the host finds the public wires' first uses itself; the caller then
// reads d_err (non-zero: a wire id >= n_wires, STARK_ERR_BAD_ARG) at its own first synchronisation.
// share: null (a build of its own), or the group's shared host stage; producer: this call runs it.
stark_status r1cs_trace_device(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len, const uint8_t* wtns,
                               size_t wtns_len, DevTrace* out, bool defer_err = false, TraceShare* share = nullptr,
                               bool producer = false);
// mk_r1cs_proof for rank `rank` of `world` on a device trace (r1cs.hip; stark_dprove_begin_bytes' second half).
stark_status dprove_begin_trace(stark_ctx* ctx, uint32_t world, uint32_t rank, const DevTrace& dt, void* stream,
                                stark_dprove** out);
// mk_r1cs_proof on trace columns given as host or device pointers, flags as
// bytes (r1cs.hip).
// The witness-independent columns of a circuit: the LDEs of K F0 F1 F2 IDX PIDX and the
// inverses of Zb2, Zb3 at the points rank + world j (8 x precision/world; K, F0-F2 and the
// inverses as Montgomery images).  world = 1: the whole domain.  with_zb = false (the verifier,
// which reads only the first six and evaluates Zb2 / Zb3 at its spot positions): 6 x P, no inverses.
stark_status circuit_lde(stark_ctx* ctx, const fe* coef, const uint8_t* flag_bytes, const uint64_t* perm, size_t os,
                         const size_t* public_first_indices, size_t n_pfi, uint32_t world, uint32_t rank, DevBuf& out,
                         hipStream_t s, bool with_zb = true, const fe** colp = nullptr,
                         uint32_t* spot_log_t = nullptr);
// mk_r1cs_proof with those columns given (only S, P and A are extended).
stark_status mk_r1cs_proof_prepared(stark_ctx* ctx, const uint64_t* witness_trace, const uint64_t* computational_trace,
                                    size_t os, const uint64_t* public_wires, size_t n_public,
                                    const size_t* public_first_indices, size_t n_pfi, const size_t* permuted_indices,
                                    const uint64_t* coefficients, const uint8_t* flag_bytes, size_t n_constraints,
                                    size_t n_wires, const fe* pre, stark_r1cs_proof** out);
// dprove_begin (r1cs.hip) with a prepared circuit's columns for this rank.
stark_status dprove_begin_prepared(stark_ctx* ctx, uint32_t world, uint32_t rank, const uint64_t* witness_trace,
                                   const uint64_t* computational_trace, size_t os, const uint64_t* public_wires,
                                   size_t n_public, const size_t* public_first_indices, size_t n_pfi,
                                   const size_t* permuted_indices, const uint64_t* coefficients,
                                   const uint8_t* flag_bytes, size_t n_constraints, size_t n_wires, const fe* pre,
                                   void* stream, stark_dprove** out);
// A circuit prepared for many proofs (r1cs_trace_dev.hip): everything of a proof that depends on
// the .r1cs alone.  lde = circuit_lde's columns for (world, rank).
struct PreparedCircuit;
// The six circuit columns K F0 F1 F2 IDX PIDX at n positions of the precision domain (a spot build):
// out[(k n + i) 32 ..] = column k at g2^positions[i], canonical little-endian.
stark_status circuit_spot_values(stark_ctx* ctx, const PreparedCircuit& c, const size_t* positions, size_t n,
                                 uint8_t* out, hipStream_t s);
struct PreparedCircuit {
  DevBuf arena, lde;
  size_t os = 0, n_wires = 0, n_public = 0;
  uint32_t n_c = 0;
  uint32_t world = 1, rank = 0;  // the points rank + world j of the precision domain (distributed prover)
  bool with_zb = true;           // false: lde holds K F0 F1 F2 IDX PIDX only (the verifier's cold build)
  // Where the six columns K F0 F1 F2 IDX PIDX are (slots of lde, or for the verifier's cold build
  // K's slot 1 and the shared F0 / IDX extensions); K F0-F2 are Montgomery images iff with_zb.
  const fe* col[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  // spot: the verifier's cold build holds no extensions, only the columns' first forward passes
  // (circuit_spot_values; first radix 2^spot_log_t).
  bool spot = false;
  uint32_t spot_log_t = 0;
  uint64_t a_len = 0;
  std::vector<size_t> pfi;
  const uint32_t* base = nullptr;
  const fe* coef = nullptr;
  const uint8_t* flags = nullptr;
  const uint64_t* perm = nullptr;
  const uint32_t* slot_wire = nullptr;
};
stark_status circuit_build(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len, PreparedCircuit& c);
// lagrange_interp (fri/src/poly_utils.rs:409-439): coefficients, low degree first (r1cs.hip).
std::vector<HostFp> lagrange_interp(const std::vector<HostFp>& xs, const std::vector<HostFp>& ys);
// mk_r1cs_proof with the flags as 3 x os bytes from a trace builder (calc_flags, run.rs:283-308):
// flag0 must be 1 on every row (the prover then takes F0's shared extension instead of extending it).
stark_status mk_r1cs_proof_bytes_flags(stark_ctx* ctx, const uint64_t* witness_trace,
                                      const uint64_t* computational_trace, size_t os, const uint64_t* public_wires,
                                      size_t n_public, const size_t* public_first_indices, size_t n_pfi,
                                      const size_t* permuted_indices, const uint64_t* coefficients,
                                      const uint8_t* flag_bytes, size_t n_constraints, size_t n_wires,
                                      stark_r1cs_proof** out, bool dev_in = false);

// FRI prover on device values (fri.hip).  fri_enqueue puts every layer on the
// context stream with a device-side transcript and queues the roots' download;
// after the caller's stream synchronisation, fri_finish samples the indices
// and gathers all openings (with the caller's extra requests) in one batch.
struct FriPending;
struct FriPendingDeleter {
  void operator()(FriPending* p) const;
};
using FriPendingPtr = std::unique_ptr<FriPending, FriPendingDeleter>;
// ctx->fri_misc: 16 special_x slots (one per FRI layer; 15 is the distributed fold's) and 16 roots.
constexpr size_t kFriMiscBytes = 16 * sizeof(fe) + 16 * 32;
stark_status fri_enqueue(stark_ctx* ctx, const fe* d_values, size_t n, const uint64_t root[4], size_t max_deg_plus_1,
                         uint32_t excl, FriPendingPtr* out, stark_merkle_tree* tree0 = nullptr,
                         bool sx0_made = false);
stark_status fri_finish(stark_ctx* ctx, FriPending* p, std::vector<GatherReq>& extra, stark_fri_proof** out);
stark_status fri_prove_device(stark_ctx* ctx, const fe* d_values, size_t n, const uint64_t root[4],
                              size_t max_deg_plus_1, uint32_t excl, stark_fri_proof** out);

// Montgomery image of a host value as a device fe (same bytes).
inline fe to_dev(const HostFp& x) {
  fe r;
  for (int i = 0; i < 4; ++i) {
    r.w[2 * i] = (uint32_t)x.v[i];
    r.w[2 * i + 1] = (uint32_t)(x.v[i] >> 32);
  }
  return r;
}

// Shoup pair of a constant w (tools/gen_fe_mul_asm.py shoup_stream): out[0] = w canonical,
// out[1] = wq = floor(w 2^256 / p).  With m = w R mod p (the Montgomery image, R = 2^256),
// w 2^256 = wq p + m exactly, so wq = (2^256 - m) p^-1 mod 2^256 (m = 0 <=> w = 0 <=> wq = 0).
inline void shoup_pair(const HostFp& x, fe out[2]) {
  static constexpr uint64_t kPinv256[4] = {0x3d1e0a6c10000001ull, 0x9a7979b4b396ee4cull, 0x1c6567d766f9dc6eull,
                                           0x8c07d0e2f27cbe4dull};
  uint64_t c[4];
  FieldHost::get().to_canonical(x, c);
  uint64_t neg[4], q[4] = {0, 0, 0, 0};
  unsigned __int128 borrow = 0;
  for (int i = 0; i < 4; ++i) {  // neg = 2^256 - m (mod 2^256)
    const unsigned __int128 d = (unsigned __int128)0 - x.v[i] - borrow;
    neg[i] = (uint64_t)d;
    borrow = (d >> 64) ? 1 : 0;
  }
  for (int i = 0; i < 4; ++i) {  // q = neg * pinv mod 2^256
    unsigned __int128 carry = 0;
    for (int j = 0; i + j < 4; ++j) {
      const unsigned __int128 t = (unsigned __int128)neg[i] * kPinv256[j] + q[i + j] + carry;
      q[i + j] = (uint64_t)t;
      carry = t >> 64;
    }
  }
  memcpy(out[0].w, c, 32);
  memcpy(out[1].w, q, 32);
}

// Digit-basis table of a constant w (fe_db.h): out[9 i + j] = 29-bit limb j of w 2^(32 i) mod p.
inline void db_table(const HostFp& x, uint32_t out[72]) {
  const FieldHost& F = FieldHost::get();
  const HostFp two32 = F.from_u64((uint64_t)1 << 32);
  HostFp cur = x;
  for (int i = 0; i < 8; ++i) {
    uint64_t c[4];
    F.to_canonical(cur, c);
    for (int j = 0; j < 9; ++j) {
      const int bit = 29 * j, word = bit >> 6, sh = bit & 63;
      uint64_t v = c[word] >> sh;
      if (sh > 35 && word < 3) v |= c[word + 1] << (64 - sh);
      out[9 * i + j] = (uint32_t)v & 0x1fffffffu;
    }
    cur = F.mul(cur, two32);
  }
}

}  // namespace stark

// A prepared circuit handle (stark_r1cs_circuit_new, r1cs_trace_dev.hip).
struct stark_r1cs_circuit {
  stark_ctx* ctx = nullptr;
  stark::PreparedCircuit c;
  ~stark_r1cs_circuit() {
    if (c.arena.ptr) hipFree(c.arena.ptr);
    if (c.lde.ptr) hipFree(c.lde.ptr);
  }
};
