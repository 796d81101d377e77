// R1CS trace construction on the GPU: the same trace as the host builder
// (r1cs_trace.hip, restating run.rs:109-308 and :388-419), built in HBM from
// the raw .r1cs / .wtns bytes so the prover reads it without a host round trip.
//
//   host   header parse + one walk over the constraint records' counts
//          (factor offsets, the per-constraint slot bases)
//   GPU    witness decode (from_bytes_le: reduce mod p; canonical + Montgomery)
//          slot fill: one thread per (constraint, factor) writes its slots'
//            coefficient, witness and running-sum (computational) values and
//            the (wire, slot) pair of every use in push order
//          flags (calc_flags, run.rs:283-308)
//          stable radix sort of the uses by wire (hipCUB), then the cyclic
//            permutation of each wire's uses (run.rs:388-401) and the first
//            use of every public wire (run.rs:411-419)
//
// Malformed input (a wire id >= n_wires inside a record) is flagged on the
// device and reported as STARK_ERR_BAD_ARG, like the host builder.
#include <string.h>

#include <algorithm>
#include <atomic>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

#include "host_walk.h"
#include "internal.h"

namespace stark {

namespace {

__device__ __forceinline__ fe reduce_any(fe v) {  // any 256-bit value < 5.3 p -> canonical
#pragma unroll
  for (int t = 0; t < 5; ++t) fe_reduce_once(v);
  return v;
}

// from_bytes_le of witness values of `words` 32-bit words (run.rs:354-357).
// (err, when given: the trace's wire-id flag, cleared here for slot_fill_kernel's atomicOr.)
__global__ void wit_decode_kernel(const uint32_t* __restrict__ w, uint32_t words, uint64_t n, fe r2,
                                  fe* __restrict__ wcan, fe* __restrict__ wmont, uint32_t* __restrict__ err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0 && err) *err = 0;
  if (i >= n) return;
  fe v = fe_zero();
  for (uint32_t k = 0; k < words; ++k) v.w[k] = w[i * words + k];
  v = reduce_any(v);
  fe_store(wcan + i, v);
  fe_store(wmont + i, fe_mul(v, r2));
}

struct FillArgs {
  const uint8_t* cons;      // constraint section (first constraint at offset 0)
  const uint32_t* fac_rec;  // byte offset of factor k's first record
  const uint32_t* fac_cnt;  // records of factor k
  const uint32_t* base;     // first slot of constraint ci (n_constraints + 1 entries)
  uint32_t n_constraints, n_wires;
  uint64_t a_len;
  const fe* wcan;
  const fe* wmont;
  fe *coef, *wit, *comp;
  uint32_t *keys, *vals;
  uint32_t* slot_wire;  // optional: the wire of every slot (prepared circuits)
  uint32_t* err;
  // initialised here for the kernels behind (flags_kernel, perm_kernel): flag0 = flag1 = 1, flag2 = 0 on
  // the 3 a_len trace rows, and the public wires' first uses "not found"
  uint8_t* flags;
  uint64_t* pf;
  uint32_t n_public;
  uint32_t* long_count;  // running_sum_kernel's long-factor counter, cleared here (or null)
};

// The constraint whose slots contain slot j of a third: the last ci with base[ci] <= j (empty
// constraints share their base with the next one, so the last is the owner).
__device__ __forceinline__ uint32_t owner_of(const uint32_t* __restrict__ base, uint32_t n_constraints, uint32_t j) {
  uint32_t lo = 0, hi = n_constraints;  // base[lo] <= j < base[hi]
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (base[mid] <= j) lo = mid;
    else hi = mid;
  }
  return lo;
}

// calc_coefficients_and_witness (run.rs:109-281), one thread per slot: factor f of constraint ci
// owns slots base[ci] .. base[ci+1]-1 of third f; a slot past the factor's records is padding
// (last wire, coefficient 0).  The slot's term coefficient * witness goes to comp; running_sum_kernel
// then forms the running sums, so the products run in parallel and only additions are serial
// (a factor may hold a thousand terms: bits.r1cs).
__global__ void slot_fill_kernel(FillArgs a) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < a.n_public) a.pf[t] = ~0ull;
  if (t == 0 && a.long_count) *a.long_count = 0;
  if (t >= 3 * a.a_len) return;
  {
    const uint64_t os = 3 * a.a_len;
    a.flags[t] = 1;
    a.flags[os + t] = 1;
    a.flags[2 * os + t] = 0;
  }
  const uint32_t f = (uint32_t)(t / a.a_len), j = (uint32_t)(t - (uint64_t)f * a.a_len);
  const uint32_t ci = owner_of(a.base, a.n_constraints, j);
  const uint32_t b0 = a.base[ci], n_coeff = a.base[ci + 1] - b0, i = j - b0;
  const uint64_t fi = 3 * (uint64_t)ci + f;
  const uint32_t cnt = a.fac_cnt[fi];
  const uint64_t slot = t;  // f a_len + b0 + i
  uint32_t wire = a.n_wires - 1;
  fe cf = fe_zero();
  if (i < cnt) {
    const uint32_t* r = reinterpret_cast<const uint32_t*>(a.cons + a.fac_rec[fi] + 36 * (uint64_t)i);
    wire = r[0];
    if (wire >= a.n_wires) {
      atomicOr(a.err, 1u);
      wire = a.n_wires - 1;
    }
    fe v;
#pragma unroll
    for (int k = 0; k < 8; ++k) v.w[k] = r[1 + k];
    cf = reduce_any(v);  // canonical from_bytes_le
  }
  fe_store(a.coef + slot, cf);
  if (a.wmont) {  // no witness: circuit columns only
    fe_store(a.wit + slot, fe_load(a.wcan + wire));
    fe_store(a.comp + slot, i < cnt ? fe_mul(cf, fe_load(a.wmont + wire)) : fe_zero());  // canonical * Montgomery
  }
  if (a.slot_wire) a.slot_wire[slot] = wire;
  const uint64_t push = 3 * (uint64_t)b0 + (uint64_t)f * n_coeff + i;
  a.keys[push] = wire;
  a.vals[push] = (uint32_t)slot;
}

// comp[slot] <- the factor's running sum up to slot (its terms were written by the fill kernels), one
// thread per factor for factors of up to kLongFactor slots.  The terms are loaded sixteen at a time ahead
// of their additions.  A longer factor (hundreds of terms in pedersen_test, a thousand in bits.r1cs) is
// listed instead (list / count, the order of no consequence) for running_sum_long_kernel.
constexpr uint32_t kLongFactor = 32;
__global__ void running_sum_kernel(const uint32_t* __restrict__ base, uint32_t n_constraints, uint64_t a_len,
                                   fe* __restrict__ comp, uint32_t* __restrict__ list, uint32_t* __restrict__ count) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= 3 * (uint64_t)n_constraints) return;
  const uint32_t ci = (uint32_t)(t / 3), f = (uint32_t)(t - 3 * (uint64_t)ci);
  const uint32_t b0 = base[ci], n_coeff = base[ci + 1] - b0;
  if (n_coeff > kLongFactor) {
    if (f == 0) list[atomicAdd(count, 1u)] = ci;
    return;
  }
  fe* c = comp + (uint64_t)f * a_len + b0;
  fe acc = fe_zero();
  constexpr uint32_t kAhead = 16;
  for (uint32_t i = 0; i < n_coeff; i += kAhead) {
    fe v[kAhead];
#pragma unroll
    for (uint32_t k = 0; k < kAhead; ++k)
      if (i + k < n_coeff) v[k] = fe_load(c + i + k);
#pragma unroll
    for (uint32_t k = 0; k < kAhead; ++k)
      if (i + k < n_coeff) {
        acc = fe_add(acc, v[k]);
        fe_store(c + i + k, acc);
      }
  }
}

// The listed long factors, one wave per factor (the grid's waves stride over the 3 count factors): 64
// slots at a time, an inclusive scan across the wave (six shifted additions), plus the running total of
// the slots before.  Field addition is associative, so the sums are the sequential ones.
__global__ __launch_bounds__(256) void running_sum_long_kernel(const uint32_t* __restrict__ base,
                                                               const uint32_t* __restrict__ list,
                                                               const uint32_t* __restrict__ count, uint64_t a_len,
                                                               fe* __restrict__ comp) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nw = (gridDim.x * blockDim.x) >> 6;
  const uint32_t items = 3 * *count;
  for (uint32_t it = (blockIdx.x * blockDim.x + threadIdx.x) >> 6; it < items; it += nw) {
    const uint32_t ci = list[it / 3], f = it % 3;
    const uint32_t b0 = base[ci], n = base[ci + 1] - b0;
    fe* c = comp + (uint64_t)f * a_len + b0;
    fe carry = fe_zero();
    for (uint32_t o = 0; o < n; o += 64) {
      const uint32_t i = o + lane;
      fe x = i < n ? fe_load(c + i) : fe_zero();
#pragma unroll
      for (uint32_t d = 1; d < 64; d <<= 1) {
        fe y;
#pragma unroll
        for (int k = 0; k < 8; ++k) y.w[k] = (uint32_t)__shfl_up((int)x.w[k], d, 64);
        if (lane >= d) x = fe_add(x, y);
      }
      x = fe_add(x, carry);
      if (i < n) fe_store(c + i, x);
#pragma unroll
      for (int k = 0; k < 8; ++k) carry.w[k] = (uint32_t)__shfl((int)x.w[k], 63, 64);
    }
  }
}
constexpr unsigned kLongSumBlocks = 256;

// calc_flags (run.rs:283-308): flag1 = 0 at (last slot + 1) mod a_len in every
// third, flag2 = 1 at each constraint's last slot (first third).
__global__ void flags_kernel(const uint32_t* __restrict__ base, uint32_t n_constraints, uint64_t a_len,
                             uint8_t* __restrict__ f1, uint8_t* __restrict__ f2) {
  const uint64_t ci = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (ci >= n_constraints) return;
  const uint64_t e = base[ci + 1];
  const uint64_t k = e % a_len;
  f1[k] = 0;
  f1[k + a_len] = 0;
  f1[k + 2 * a_len] = 0;
  f2[e - 1] = 1;
}

__global__ void group_last_kernel(const uint32_t* __restrict__ keys, uint64_t n, uint32_t* __restrict__ last) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t k = keys[j];
  if (j + 1 == n || keys[j + 1] != k) last[k] = (uint32_t)j;
}

// Each wire's uses, in push order, form one cycle (run.rs:388-401): a use
// points at the previous use, the first at the last.  pf[w] = first use of
// public wire w (run.rs:411-419).
__global__ void perm_kernel(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ vals, uint64_t n,
                            const uint32_t* __restrict__ last, uint32_t n_public, uint64_t* __restrict__ perm,
                            uint64_t* __restrict__ pf) {
  const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= n) return;
  const uint32_t k = keys[j];
  const bool start = j == 0 || keys[j - 1] != k;
  perm[vals[j]] = start ? vals[last[k]] : vals[j - 1];
  if (start && k < n_public) pf[k] = vals[j];
}

// The witness columns of a prepared circuit: the slot fill's witness / term part (run.rs:109-281) from
// the stored slot wires and coefficients, one thread per slot (running_sum_kernel follows).
__global__ void wit_fill_kernel(uint64_t n_slots, const uint32_t* __restrict__ slot_wire, const fe* __restrict__ coef,
                                const fe* __restrict__ wcan, const fe* __restrict__ wmont, fe* __restrict__ wit,
                                fe* __restrict__ comp) {
  const uint64_t slot = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (slot >= n_slots) return;
  const uint32_t wire = slot_wire[slot];
  fe_store(comp + slot, fe_mul(fe_load(coef + slot), fe_load(wmont + wire)));  // padding slots: coefficient 0
  fe_store(wit + slot, fe_load(wcan + wire));
}

unsigned blocks(uint64_t n) { return (unsigned)((n + 255) / 256); }

// The slots' (wire, slot) pairs sorted by wire (stable: both algorithms below are).  rocPRIM's default
// dispatch takes its merge sort for 4-byte keys up to 2^20 items: about 20 launches of ~5 us at 2^19 slots;
// from 2^18 slots its onesweep radix sort (a histogram, a scan and one pass per 8 key bits) is used instead
// (profiles/r06_slot_sort_ab.txt: 0.1 ms off the 2^20-step proof; below, on pedersen, the merge sort is faster).
constexpr int kOnesweepFrom = 1 << 18;
using OnesweepConfig =
    rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>;
hipError_t sort_slots(void* tmp, size_t& tmp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                      const uint32_t* vals_in, uint32_t* vals_out, int n, int begin_bit, int end_bit, hipStream_t s) {
  if (n >= kOnesweepFrom)
    return rocprim::radix_sort_pairs<OnesweepConfig>(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out,
                                                     (unsigned)n, (unsigned)begin_bit, (unsigned)end_bit, s);
  return rocprim::radix_sort_pairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, vals_out, (unsigned)n,
                                   (unsigned)begin_bit, (unsigned)end_bit, s);
}

// The first use of every public wire (run.rs:411-419) read from the records on the host, in push order
// (constraint, factor, slot; a factor's padding slots use the last wire), as perm_kernel finds it after
// the sort.  Stops once every public wire is found; false (undecided) past `budget` slots or at a wire
// id >= n_wires (the device flags that one and the caller reports it).
bool host_first_uses(const uint8_t* cons, const uint32_t* fac, const uint32_t* base, uint32_t n_c, uint64_t a_len,
                     size_t n_public, uint32_t n_wires, uint64_t budget, std::vector<uint64_t>& pf) {
  pf.assign(n_public, ~0ull);
  size_t found = 0;
  uint64_t seen = 0;
  const uint32_t* fac_rec = fac;
  const uint32_t* fac_cnt = fac + (size_t)3 * n_c;
  for (uint32_t ci = 0; ci < n_c && found < n_public; ++ci) {
    const uint32_t b0 = base[ci], n_coeff = base[ci + 1] - b0;
    for (uint32_t f = 0; f < 3 && found < n_public; ++f) {
      const uint32_t cnt = fac_cnt[3 * (size_t)ci + f];
      const uint8_t* r = cons + fac_rec[3 * (size_t)ci + f];
      for (uint32_t i = 0; i < n_coeff; ++i) {
        uint32_t wire = n_wires - 1;
        if (i < cnt) {
          memcpy(&wire, r + 36 * (size_t)i, 4);
          if (wire >= n_wires) return false;
        }
        if (wire < n_public && pf[wire] == ~0ull) {
          pf[wire] = (uint64_t)f * a_len + b0 + i;
          if (++found == n_public) break;
        }
      }
      seen += n_coeff;
      if (seen > budget) return false;
    }
  }
  return true;
}

}  // namespace

// The host threads of an upload with the record walk beside it: the walk's parts (each a share of the
// section, so as many as can run at once; a part's task stages chunks once its part is walked) and the tasks
// that only stage, together no more tasks than threads.
static void split_host_threads(unsigned* walkers, unsigned* stagers) {
  const unsigned t = host_threads();
  *walkers = std::max(1u, std::min(8u, t / 2));
  *stagers = std::max(1u, t > *walkers ? t - *walkers : 1u);
}

// Host-to-device copies of caller (pageable) memory through the context's pinned staging buffer:
// the copy is split in 2 MB chunks that `workers` host threads memcpy into the staging buffer, each
// thread enqueueing the DMA of a chunk as soon as it is staged, so the DMAs overlap the memcpys.  A
// pageable hipMemcpyAsync blocks the caller and stages through the runtime's own small buffers.
// Returns once every DMA is enqueued on s; ctx->staged marks their completion, which the next call
// waits for before it writes the staging buffer again.
struct Upload {
  void* dst;
  const void* src;
  size_t len;
};
constexpr size_t kStageAlone = (size_t)1 << 20;  // smaller uploads: one thread, no pool
static stark_status staged_upload(stark_ctx* ctx, const std::vector<Upload>& ups, hipStream_t s, unsigned workers,
                                  unsigned sides, const std::function<void(unsigned)>& side) {
  constexpr size_t kChunk = (size_t)2 << 20;
  size_t total = 0;
  for (const Upload& u : ups) total += u.len;
  if (!ctx->staged) STARK_HIP(ctx, hipEventCreateWithFlags(&ctx->staged, hipEventDisableTiming));
  STARK_HIP(ctx, hipEventSynchronize(ctx->staged));  // the previous call's DMAs have left the buffer
  uint8_t* stage = nullptr;
  stark_status st = ctx_pinned(ctx, 3, total, (void**)&stage);
  if (st != STARK_OK) return st;
  if (total < kStageAlone) {
    // A small circuit: the side tasks and the copies on this thread (waking the pool costs more than they do)
    for (unsigned k = 0; k < sides; ++k) side(k);
    size_t at = 0;
    hipError_t e = hipSuccess;
    for (const Upload& u : ups) {
      memcpy(stage + at, u.src, u.len);
      if (e == hipSuccess && u.len) e = hipMemcpyAsync(u.dst, stage + at, u.len, hipMemcpyHostToDevice, s);
      at += u.len;
    }
    const hipError_t rec = hipEventRecord(ctx->staged, s);  // (also on the error path: see below)
    if (e != hipSuccess) {
      if (rec != hipSuccess) hipStreamSynchronize(s);
      return hip_fail(ctx, e, "r1cs/wtns upload");
    }
    if (rec != hipSuccess) return hip_fail(ctx, rec, "hipEventRecord(staged)");
    return STARK_OK;
  }
  struct Piece {
    uint8_t* dst;
    const uint8_t* src;
    uint8_t* stage;
    size_t len;
  };
  // The first pieces are small (256 KB, doubling up to kChunk) so the first DMA starts after a short
  // memcpy instead of a 2 MB one; the rest stay at kChunk (each DMA costs ~9 us of engine overhead).
  std::vector<Piece> pieces;
  size_t at = 0, piece = kChunk / 8;
  for (const Upload& u : ups)
    for (size_t o = 0; o < u.len;) {
      const size_t len = std::min(piece, u.len - o);
      pieces.push_back({(uint8_t*)u.dst + o, (const uint8_t*)u.src + o, stage + at, len});
      at += len;
      o += len;
      piece = std::min(kChunk, 2 * piece);
    }
  std::atomic<size_t> next{0};
  // The first failing copy's error, recorded by the worker that saw it (HIP's last-error state is
  // per thread, so the caller could not read it back with hipGetLastError).
  std::atomic<int> failed{(int)hipSuccess};
  // tasks 1 .. sides run side(0 .. sides - 1) (the record walk's parts) and then stage too; the caller and the
  // other `workers - 1` tasks stage chunks in order of claim from the start
  host_parallel(workers + sides, [&](unsigned t) {
    if (t >= 1 && t <= sides) side(t - 1);
    // (a worker's current device is whatever it last ran for: the context's, for its copies)
    if (t > 0 && hipSetDevice(ctx->device) != hipSuccess) {
      int ok = (int)hipSuccess;
      failed.compare_exchange_strong(ok, (int)hipErrorInvalidDevice);
      return;
    }
    for (size_t i; (i = next.fetch_add(1)) < pieces.size();) {
      if (failed.load(std::memory_order_relaxed) != (int)hipSuccess) break;
      const Piece& p = pieces[i];
      memcpy(p.stage, p.src, p.len);
      const hipError_t e = hipMemcpyAsync(p.dst, p.stage, p.len, hipMemcpyHostToDevice, s);
      int ok = (int)hipSuccess;
      if (e != hipSuccess) failed.compare_exchange_strong(ok, (int)e);
    }
  });
  // Recorded on the error path too: DMAs already enqueued from the staging buffer must be covered by
  // the event the next call waits on before it writes that buffer again.
  const hipError_t rec = hipEventRecord(ctx->staged, s);
  if (failed.load() != (int)hipSuccess) {
    if (rec != hipSuccess) hipStreamSynchronize(s);  // no event: drain the stream instead
    return hip_fail(ctx, (hipError_t)failed.load(), "r1cs/wtns upload");
  }
  if (rec != hipSuccess) return hip_fail(ctx, rec, "hipEventRecord(staged)");
  return STARK_OK;
}

// The producer's half of a shared build (TraceShare): publishes what the consumers read, and releases them
// (also on an error, with its status).
struct ShareGuard {
  TraceShare* sh;
  bool done = false;
  void publish(stark_status st) {
    if (!sh || done) return;
    sh->status = st;
    done = true;
    sh->ready_p.set_value();
  }
  ~ShareGuard() { publish(STARK_ERR_STATE); }
};

static stark_status peer_copy(stark_ctx* dst_ctx, void* dst, const stark_ctx* src_ctx, const void* src, size_t bytes,
                              hipStream_t s) {
  if (!bytes) return STARK_OK;
  if (dst_ctx->device == src_ctx->device) {
    STARK_HIP(dst_ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, s));
  } else {
    STARK_HIP(dst_ctx, hipMemcpyPeerAsync(dst, dst_ctx->device, src, src_ctx->device, bytes, s));
  }
  return STARK_OK;
}

stark_status r1cs_trace_device(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len, const uint8_t* wtns,
                               size_t wtns_len, DevTrace* out, bool defer_err, TraceShare* share, bool producer) {
  PhaseClock clk("r1cs trace build (device)");
  const FieldHost& F = FieldHost::get();
  ShareGuard guard{producer ? share : nullptr};
  const bool consumer = share && !producer;
  R1csHeader hd;
  WtnsHeader wh;
  size_t n_public, cons_len, wbytes, fac_n, base_n, o_raw_w;
  uint64_t a_len;
  stark_status st;
  uint8_t* RAW;
  hipStream_t s = ctx->stream;
  std::vector<uint64_t> pf_host;
  bool pf_ok = false;
  const uint32_t* fac_src = nullptr;   // the walk tables to upload (host pinned) or copy (a producer's device)
  const uint32_t* base_src = nullptr;
  if (consumer) {
    // The producer's host stage: headers, public wires and walk, raw bytes already on its device.
    share->ready.wait();
    if (share->status != STARK_OK) return share->status;
    hd = share->hd;
    wh = share->wh;
    n_public = share->n_public;
    cons_len = share->cons_len;
    wbytes = share->wbytes;
    fac_n = share->fac_n;
    base_n = share->base_n;
    o_raw_w = share->o_raw_w;
    a_len = share->a_len;
    out->public_wires = share->public_wires;
    pf_ok = share->pf_ok;
    pf_host = share->pf_host;
    st = ensure_buf(ctx, ctx->trace_raw, o_raw_w + wbytes);
    if (st != STARK_OK) return st;
    RAW = (uint8_t*)ctx->trace_raw.ptr;
    STARK_HIP(ctx, hipStreamWaitEvent(s, share->ev, 0));
    STARK_TRY(peer_copy(ctx, RAW, share->src, share->raw, o_raw_w + wbytes, s));
    clk.mark("raw bytes from the producer (peer copy)");
  } else {
    st = parse_r1cs_header(r1cs, r1cs_len, &hd);
    if (st != STARK_OK) return st;
    st = parse_wtns_header(wtns, wtns_len, &wh);
    if (st != STARK_OK) return st;
  }
  const uint32_t n_c = hd.n_constraints, n_wires = hd.n_wires, n_wit = wh.n_wit;
  if (!consumer) {
    n_public = 1 + (size_t)hd.n_pub_in + hd.n_pub_out;  // run.rs:359-360
    if (n_wit < n_wires || n_public > n_wit) return STARK_ERR_BAD_ARG;
    // witness[0] must be 1 (run.rs:358); the public wires are the first n_public values.
    const uint8_t* wv = wtns + wh.values_off;
    {
      const HostFp w0 = F.reduce_bytes_le(wv, wh.field_size);
      if (!(w0.v[0] == 1 && w0.v[1] == 0 && w0.v[2] == 0 && w0.v[3] == 0)) return STARK_ERR_BAD_ARG;
    }
    out->public_wires.resize(4 * n_public);
    for (size_t i = 0; i < n_public; ++i) {
      const HostFp v = F.reduce_bytes_le(wv + i * wh.field_size, wh.field_size);
      memcpy(&out->public_wires[4 * i], v.v, 32);
    }

    // Host walk: record counts only (the records themselves are read on the GPU).  It runs on a host
    // worker while this thread uploads the raw constraint section and witness (pageable memory: the
    // copies block), and it writes straight into pinned memory, so its tables go up asynchronously.
    const uint8_t* cons = r1cs + hd.cons_off;
    cons_len = r1cs_len - hd.cons_off;
    wbytes = (size_t)n_wit * wh.field_size;
    fac_n = (size_t)6 * n_c + 1;
    base_n = (size_t)n_c + 1;
    uint32_t* walk = nullptr;
    st = ctx_pinned(ctx, 2, (fac_n + base_n) * 4, (void**)&walk);
    if (st != STARK_OK) return st;
    uint32_t* fac = walk;
    uint32_t* base = walk + fac_n;
    fac_src = fac;
    base_src = base;
    o_raw_w = (cons_len + 255) & ~(size_t)255;
    st = ensure_buf(ctx, ctx->trace_raw, o_raw_w + wbytes);
    if (st != STARK_OK) return st;
    RAW = (uint8_t*)ctx->trace_raw.ptr;
    // The walk's parts run beside the stagers (RecordWalk, host_walk.h), then link on this thread.
    // defer_err: the public wires' first uses are also read on the host (a bounded scan that usually ends
    // in the first constraints), so the build needs no read-back and the caller checks the device's
    // wire-id flag at its own first synchronisation (d_err).
    unsigned walkers, stagers;
    split_host_threads(&walkers, &stagers);
    RecordWalk rw(cons, cons_len, n_c, n_wires, walkers);
    st = staged_upload(ctx, {{RAW, cons, cons_len}, {RAW + o_raw_w, wv, wbytes}}, s, stagers, rw.parts(),
                       [&](unsigned k) { rw.part(k); });
    if (st != STARK_OK) return st;
    const stark_status walk_st = rw.finish(fac, base);
    if (walk_st != STARK_OK) return walk_st;
    if (defer_err && n_wires > 0)
      pf_ok = host_first_uses(cons, fac, base, n_c, base[n_c], n_public, n_wires, (uint64_t)1 << 18, pf_host);
    a_len = base[n_c];
    clk.mark("headers + record walk || uploads");
  }
  const uint64_t os = 3 * a_len;
  if (a_len == 0) return STARK_ERR_BAD_ARG;

  // Device buffers (context-owned arena).
  uint32_t key_bits = 1;
  while (key_bits < 32 && (1ull << key_bits) < n_wires) ++key_bits;
  size_t sort_tmp = 0;
  STARK_HIP(ctx, sort_slots(nullptr, sort_tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                   (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)os, 0,
                                                   (int)key_bits, ctx->stream));
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  const size_t o_fac = take(fac_n * 4), o_base = take(base_n * 4), o_wcan = take((size_t)n_wit * 32),
               o_wmont = take((size_t)n_wit * 32), o_coef = take(os * 32), o_wit = take(os * 32),
               o_comp = take(os * 32), o_flags = take(3 * os), o_perm = take(os * 8), o_k = take(os * 4),
               o_v = take(os * 4), o_k2 = take(os * 4), o_v2 = take(os * 4), o_last = take((size_t)n_wires * 4),
               o_pf = take(n_public * 8), o_err = take(4), o_tmp = take(sort_tmp), o_long = take((size_t)n_c * 4),
               o_cnt = take(4);
  st = ensure_buf(ctx, ctx->trace_arena, off);
  if (st != STARK_OK) return st;
  uint8_t* A = (uint8_t*)ctx->trace_arena.ptr;
  if (consumer) {
    STARK_TRY(peer_copy(ctx, A + o_fac, share->src, share->fac, fac_n * 4, s));
    STARK_TRY(peer_copy(ctx, A + o_base, share->src, share->base, base_n * 4, s));
  } else {
    STARK_HIP(ctx, hipMemcpyAsync(A + o_fac, fac_src, fac_n * 4, hipMemcpyHostToDevice, s));
    STARK_HIP(ctx, hipMemcpyAsync(A + o_base, base_src, base_n * 4, hipMemcpyHostToDevice, s));
  }
  if (producer) {
    // the consumers copy the raw bytes and walk tables from here, behind this event
    if (!share->ev) STARK_HIP(ctx, hipEventCreateWithFlags(&share->ev, hipEventDisableTiming));
    STARK_HIP(ctx, hipEventRecord(share->ev, s));
    share->hd = hd;
    share->wh = wh;
    share->n_public = n_public;
    share->cons_len = cons_len;
    share->wbytes = wbytes;
    share->fac_n = fac_n;
    share->base_n = base_n;
    share->o_raw_w = o_raw_w;
    share->a_len = a_len;
    share->public_wires = out->public_wires;
    share->pf_ok = pf_ok;
    share->pf_host = pf_host;
    share->src = ctx;
    share->raw = RAW;
    share->fac = (const uint32_t*)(A + o_fac);
    share->base = (const uint32_t*)(A + o_base);
    guard.publish(STARK_OK);
  }
  fe* wcan = (fe*)(A + o_wcan);
  fe* wmont = (fe*)(A + o_wmont);
  uint32_t* err = (uint32_t*)(A + o_err);
  {
    uint64_t one_r[4];  // Montgomery image of R = R^2 mod p
    memcpy(one_r, F.one().v, 32);
    hipLaunchKernelGGL(wit_decode_kernel, dim3(blocks(std::max<uint64_t>(n_wit, 1))), dim3(256), 0, s,
                       (const uint32_t*)(RAW + o_raw_w), wh.field_size / 4, (uint64_t)n_wit,
                       to_dev(F.from_canonical(one_r)), wcan, wmont, err);
  }
  FillArgs fa;
  fa.cons = RAW;
  fa.fac_rec = (const uint32_t*)(A + o_fac);
  fa.fac_cnt = (const uint32_t*)(A + o_fac) + (size_t)3 * n_c;
  fa.base = (const uint32_t*)(A + o_base);
  fa.n_constraints = n_c;
  fa.n_wires = n_wires;
  fa.a_len = a_len;
  fa.wcan = wcan;
  fa.wmont = wmont;
  fa.coef = (fe*)(A + o_coef);
  fa.wit = (fe*)(A + o_wit);
  fa.comp = (fe*)(A + o_comp);
  fa.keys = (uint32_t*)(A + o_k);
  fa.vals = (uint32_t*)(A + o_v);
  fa.slot_wire = nullptr;
  fa.err = err;
  uint8_t* flags = A + o_flags;
  fa.flags = flags;
  fa.pf = (uint64_t*)(A + o_pf);
  fa.n_public = (uint32_t)n_public;
  uint32_t* long_list = (uint32_t*)(A + o_long);
  uint32_t* long_cnt = (uint32_t*)(A + o_cnt);
  fa.long_count = long_cnt;
  hipLaunchKernelGGL(slot_fill_kernel, dim3(blocks(std::max<uint64_t>(3 * a_len, n_public))), dim3(256), 0, s, fa);
  hipLaunchKernelGGL(running_sum_kernel, dim3(blocks(3 * (uint64_t)n_c)), dim3(256), 0, s, fa.base, n_c, a_len,
                     fa.comp, long_list, long_cnt);
  hipLaunchKernelGGL(running_sum_long_kernel, dim3(kLongSumBlocks), dim3(256), 0, s, fa.base,
                     (const uint32_t*)long_list, (const uint32_t*)long_cnt, a_len, fa.comp);
  hipLaunchKernelGGL(flags_kernel, dim3(blocks(n_c)), dim3(256), 0, s, (const uint32_t*)(A + o_base), n_c, a_len,
                     flags + os, flags + 2 * os);
  STARK_HIP(ctx, hipGetLastError());
  size_t tmp_bytes = sort_tmp;
  STARK_HIP(ctx, sort_slots(A + o_tmp, tmp_bytes, (const uint32_t*)(A + o_k),
                                                   (uint32_t*)(A + o_k2), (const uint32_t*)(A + o_v),
                                                   (uint32_t*)(A + o_v2), (int)os, 0, (int)key_bits, s));
  const uint32_t* keys = (const uint32_t*)(A + o_k2);
  const uint32_t* vals = (const uint32_t*)(A + o_v2);
  uint32_t* last = (uint32_t*)(A + o_last);
  hipLaunchKernelGGL(group_last_kernel, dim3(blocks(os)), dim3(256), 0, s, keys, os, last);
  hipLaunchKernelGGL(perm_kernel, dim3(blocks(os)), dim3(256), 0, s, keys, vals, os, (const uint32_t*)last,
                     (uint32_t)n_public, (uint64_t*)(A + o_perm), (uint64_t*)(A + o_pf));
  STARK_HIP(ctx, hipGetLastError());
  clk.mark("kernels enqueued");
  std::vector<uint64_t> pf(n_public);
  out->d_err = nullptr;
  if (pf_ok) {  // the host scan found them: no read-back, the caller checks err later
    pf = pf_host;
    out->d_err = err;
  } else {
    // First uses of the public wires and the error flag: the one host read-back.
    uint32_t h_err = 0;
    STARK_HIP(ctx, hipMemcpyAsync(pf.data(), A + o_pf, n_public * 8, hipMemcpyDeviceToHost, s));
    STARK_HIP(ctx, hipMemcpyAsync(&h_err, err, 4, hipMemcpyDeviceToHost, s));
    STARK_HIP(ctx, hipStreamSynchronize(s));
    if (h_err) return STARK_ERR_BAD_ARG;  // a wire id >= n_wires (reader.rs:4-89 bounds)
  }
  out->public_first_indices.clear();
  for (size_t wi = 0; wi < n_public && wi < n_wires; ++wi)
    if (pf[wi] != ~0ull) {
      out->public_first_indices.push_back(wi);
      out->public_first_indices.push_back((size_t)pf[wi]);
    }
  out->os = os;
  out->n_constraints = n_c;
  out->n_wires = n_wires;
  out->coef = fa.coef;
  out->wit = fa.wit;
  out->comp = fa.comp;
  out->flags = flags;
  out->perm = (uint64_t*)(A + o_perm);
  clk.mark("device build + read-back");
  return STARK_OK;
}

// ---- prepared circuits --------------------------------------------------------
//
// Everything of a proof that depends on the .r1cs alone, built once: the slot
// layout (and each slot's wire), the coefficient and flag columns, the
// permutation, the public wires' first uses, and the LDEs of K, F0, F1, F2, IDX
// and PIDX.  A proof for a new witness then builds S and P (wit_fill_kernel) and
// extends only S, P and A: 3 of the 9 LDE columns.

stark_status circuit_build(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len, PreparedCircuit& c) {
  PhaseClock clk("circuit_build");
  R1csHeader hd;
  stark_status st = parse_r1cs_header(r1cs, r1cs_len, &hd);
  if (st != STARK_OK) return st;
  const uint32_t n_c = hd.n_constraints, n_wires = hd.n_wires;
  const size_t n_public = 1 + (size_t)hd.n_pub_in + hd.n_pub_out;  // run.rs:359-360
  if (n_wires == 0 || n_public > n_wires) return STARK_ERR_BAD_ARG;
  const uint8_t* cons = r1cs + hd.cons_off;
  const size_t cons_len = r1cs_len - hd.cons_off;
  hipStream_t s = ctx->stream;
  // As in r1cs_trace_device: the raw constraint section goes up through the staging buffer (into the
  // context's trace_raw, scratch here) while a host worker walks the records into pinned memory and
  // looks for the public wires' first uses, so the build needs no read-back before its LDE.
  const size_t fac_n = (size_t)6 * n_c + 1, base_n = (size_t)n_c + 1;
  uint32_t* walk = nullptr;
  STARK_TRY(ctx_pinned(ctx, 2, (fac_n + base_n + 1) * 4, (void**)&walk));
  uint32_t* const fac = walk;
  uint32_t* const base = walk + fac_n;
  uint32_t* const h_err = base + base_n;  // the wire-id flag's read-back (pinned: an async copy)
  STARK_TRY(ensure_buf(ctx, ctx->trace_raw, cons_len));
  uint8_t* const RAW = (uint8_t*)ctx->trace_raw.ptr;
  unsigned walkers, stagers;
  split_host_threads(&walkers, &stagers);
  RecordWalk rw(cons, cons_len, n_c, n_wires, walkers);
  st = staged_upload(ctx, {{RAW, cons, cons_len}}, s, stagers, rw.parts(), [&](unsigned k) { rw.part(k); });
  if (st != STARK_OK) return st;
  const stark_status walk_st = rw.finish(fac, base);
  if (walk_st != STARK_OK) return walk_st;
  std::vector<uint64_t> pf_host;
  const bool pf_ok =
      host_first_uses(cons, fac, base, n_c, base[n_c], n_public, n_wires, (uint64_t)1 << 18, pf_host);
  clk.mark("record walk || upload");
  const uint64_t a_len = base[n_c];
  const uint64_t os = 3 * a_len;
  if (a_len == 0) return STARK_ERR_BAD_ARG;
  uint32_t key_bits = 1;
  while (key_bits < 32 && (1ull << key_bits) < n_wires) ++key_bits;
  size_t sort_tmp = 0;
  STARK_HIP(ctx, sort_slots(nullptr, sort_tmp, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                                   (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)os, 0,
                                                   (int)key_bits, s));
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  // Kept: base, coef, flags, perm, slot wires.  Scratch (the circuit's own arena, so a
  // prepared circuit never aliases the context's trace arena): walk tables, sort buffers.
  const size_t o_base = take(base_n * 4), o_coef = take(os * 32), o_flags = take(3 * os), o_perm = take(os * 8),
               o_sw = take(os * 4), o_fac = take(fac_n * 4), o_k = take(os * 4), o_v = take(os * 4),
               o_k2 = take(os * 4), o_v2 = take(os * 4), o_last = take((size_t)n_wires * 4),
               o_pf = take(n_public * 8), o_err = take(4), o_tmp = take(sort_tmp);
  st = ensure_buf(ctx, c.arena, off);
  if (st != STARK_OK) return st;
  uint8_t* A = (uint8_t*)c.arena.ptr;
  STARK_HIP(ctx, hipMemcpyAsync(A + o_fac, fac, fac_n * 4, hipMemcpyHostToDevice, s));
  STARK_HIP(ctx, hipMemcpyAsync(A + o_base, base, base_n * 4, hipMemcpyHostToDevice, s));
  STARK_HIP(ctx, hipMemsetAsync(A + o_err, 0, 4, s));
  FillArgs fa;
  fa.cons = RAW;
  fa.fac_rec = (const uint32_t*)(A + o_fac);
  fa.fac_cnt = (const uint32_t*)(A + o_fac) + (size_t)3 * n_c;
  fa.base = (const uint32_t*)(A + o_base);
  fa.n_constraints = n_c;
  fa.n_wires = n_wires;
  fa.a_len = a_len;
  fa.wcan = nullptr;
  fa.wmont = nullptr;  // circuit columns only
  fa.coef = (fe*)(A + o_coef);
  fa.wit = nullptr;
  fa.comp = nullptr;
  fa.keys = (uint32_t*)(A + o_k);
  fa.vals = (uint32_t*)(A + o_v);
  fa.slot_wire = (uint32_t*)(A + o_sw);
  fa.err = (uint32_t*)(A + o_err);
  fa.flags = A + o_flags;
  fa.pf = (uint64_t*)(A + o_pf);
  fa.n_public = (uint32_t)n_public;
  fa.long_count = nullptr;  // (circuit columns only: no running sums here)
  hipLaunchKernelGGL(slot_fill_kernel, dim3(blocks(std::max<uint64_t>(3 * a_len, n_public))), dim3(256), 0, s, fa);
  uint8_t* flags = A + o_flags;
  hipLaunchKernelGGL(flags_kernel, dim3(blocks(n_c)), dim3(256), 0, s, (const uint32_t*)(A + o_base), n_c, a_len,
                     flags + os, flags + 2 * os);
  STARK_HIP(ctx, hipGetLastError());
  size_t tmp_bytes = sort_tmp;
  STARK_HIP(ctx, sort_slots(A + o_tmp, tmp_bytes, (const uint32_t*)(A + o_k),
                                                   (uint32_t*)(A + o_k2), (const uint32_t*)(A + o_v),
                                                   (uint32_t*)(A + o_v2), (int)os, 0, (int)key_bits, s));
  hipLaunchKernelGGL(group_last_kernel, dim3(blocks(os)), dim3(256), 0, s, (const uint32_t*)(A + o_k2), os,
                     (uint32_t*)(A + o_last));
  hipLaunchKernelGGL(perm_kernel, dim3(blocks(os)), dim3(256), 0, s, (const uint32_t*)(A + o_k2),
                     (const uint32_t*)(A + o_v2), os, (const uint32_t*)(A + o_last), (uint32_t)n_public,
                     (uint64_t*)(A + o_perm), (uint64_t*)(A + o_pf));
  STARK_HIP(ctx, hipGetLastError());
  // The wire-id flag comes back behind the LDE (circuit_lde ends in a synchronisation; the slot kernels
  // clamp a bad wire id, so what runs before the check stays in bounds).  The first uses come from the
  // host scan, or, where it gave up, from the device with the one read-back.
  *h_err = 0;
  STARK_HIP(ctx, hipMemcpyAsync(h_err, A + o_err, 4, hipMemcpyDeviceToHost, s));
  std::vector<uint64_t> pf(n_public);
  if (pf_ok) {
    pf = pf_host;
  } else {
    STARK_HIP(ctx, hipMemcpyAsync(pf.data(), A + o_pf, n_public * 8, hipMemcpyDeviceToHost, s));
    STARK_HIP(ctx, hipStreamSynchronize(s));
    if (*h_err) return STARK_ERR_BAD_ARG;
  }
  clk.mark("slots, sort, perm enqueued");
  c.pfi.clear();
  for (size_t wi = 0; wi < n_public; ++wi)
    if (pf[wi] != ~0ull) {
      c.pfi.push_back(wi);
      c.pfi.push_back((size_t)pf[wi]);
    }
  c.os = os;
  c.n_c = n_c;
  c.n_wires = n_wires;
  c.n_public = n_public;
  c.a_len = a_len;
  c.base = (const uint32_t*)(A + o_base);
  c.coef = (const fe*)(A + o_coef);
  c.flags = flags;
  c.perm = (const uint64_t*)(A + o_perm);
  c.slot_wire = (const uint32_t*)(A + o_sw);
  st = circuit_lde(ctx, c.coef, c.flags, c.perm, os, c.pfi.data(), c.pfi.size() / 2, c.world, c.rank, c.lde, s,
                   c.with_zb, c.col, c.spot ? &c.spot_log_t : nullptr);
  clk.mark("circuit LDE (synced)");
  if (hipStreamSynchronize(s) != hipSuccess && st == STARK_OK) st = STARK_ERR_HIP;
  if (*h_err) return STARK_ERR_BAD_ARG;  // a wire id >= n_wires (reader.rs:4-89 bounds)
  return st;
}

// The witness of one proof: decode, then S and P from the circuit's slot wires.
static stark_status circuit_witness(stark_ctx* ctx, const PreparedCircuit& c, const uint8_t* wtns, size_t wtns_len,
                                    DevTrace* out) {
  const FieldHost& F = FieldHost::get();
  WtnsHeader wh;
  stark_status st = parse_wtns_header(wtns, wtns_len, &wh);
  if (st != STARK_OK) return st;
  const uint32_t n_wit = wh.n_wit;
  if (n_wit < c.n_wires || c.n_public > n_wit) return STARK_ERR_BAD_ARG;
  const uint8_t* wv = wtns + wh.values_off;
  {
    const HostFp w0 = F.reduce_bytes_le(wv, wh.field_size);  // witness[0] == 1 (run.rs:358)
    if (!(w0.v[0] == 1 && w0.v[1] == 0 && w0.v[2] == 0 && w0.v[3] == 0)) return STARK_ERR_BAD_ARG;
  }
  out->public_wires.resize(4 * c.n_public);
  for (size_t i = 0; i < c.n_public; ++i) {
    const HostFp v = F.reduce_bytes_le(wv + i * wh.field_size, wh.field_size);
    memcpy(&out->public_wires[4 * i], v.v, 32);
  }
  const size_t wbytes = (size_t)n_wit * wh.field_size;
  size_t off = 0;
  auto take = [&](size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  };
  const size_t o_w = take(wbytes), o_wcan = take((size_t)n_wit * 32), o_wmont = take((size_t)n_wit * 32),
               o_wit = take(c.os * 32), o_comp = take(c.os * 32), o_long = take((size_t)c.n_c * 4), o_cnt = take(4);
  st = ensure_buf(ctx, ctx->trace_arena, off);
  if (st != STARK_OK) return st;
  uint8_t* A = (uint8_t*)ctx->trace_arena.ptr;
  hipStream_t s = ctx->stream;
  STARK_HIP(ctx, hipMemcpyAsync(A + o_w, wv, wbytes, hipMemcpyHostToDevice, s));
  uint64_t one_r[4];
  memcpy(one_r, F.one().v, 32);
  hipLaunchKernelGGL(wit_decode_kernel, dim3(blocks(n_wit)), dim3(256), 0, s, (const uint32_t*)(A + o_w),
                     wh.field_size / 4, (uint64_t)n_wit, to_dev(F.from_canonical(one_r)), (fe*)(A + o_wcan),
                     (fe*)(A + o_wmont), (uint32_t*)(A + o_cnt));  // (clears the long-factor counter)
  hipLaunchKernelGGL(wit_fill_kernel, dim3(blocks(3 * c.a_len)), dim3(256), 0, s, 3 * c.a_len, c.slot_wire, c.coef,
                     (const fe*)(A + o_wcan), (const fe*)(A + o_wmont), (fe*)(A + o_wit), (fe*)(A + o_comp));
  hipLaunchKernelGGL(running_sum_kernel, dim3(blocks(3 * (uint64_t)c.n_c)), dim3(256), 0, s, c.base, c.n_c, c.a_len,
                     (fe*)(A + o_comp), (uint32_t*)(A + o_long), (uint32_t*)(A + o_cnt));
  hipLaunchKernelGGL(running_sum_long_kernel, dim3(kLongSumBlocks), dim3(256), 0, s, c.base,
                     (const uint32_t*)(A + o_long), (const uint32_t*)(A + o_cnt), c.a_len, (fe*)(A + o_comp));
  STARK_HIP(ctx, hipGetLastError());
  out->os = c.os;
  out->n_constraints = c.n_c;
  out->n_wires = c.n_wires;
  out->wit = (fe*)(A + o_wit);
  out->comp = (fe*)(A + o_comp);
  out->public_first_indices = c.pfi;
  return STARK_OK;
}

}  // namespace stark

using namespace stark;

extern "C" {

stark_status stark_prove_r1cs_bytes(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len, const uint8_t* wtns,
                                    size_t wtns_len, stark_r1cs_proof** out) {
  if (!ctx || !r1cs || !wtns || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  DevTrace dt;
  stark_status st = r1cs_trace_device(ctx, r1cs, r1cs_len, wtns, wtns_len, &dt, true);
  if (st != STARK_OK) return st;
  // (a deferred wire-id flag is read with the prover's first download and reported as STARK_ERR_BAD_ARG)
  ctx->trace_err = dt.d_err;
  st = mk_r1cs_proof_bytes_flags(ctx, (const uint64_t*)dt.wit, (const uint64_t*)dt.comp, dt.os,
                                 dt.public_wires.data(), dt.public_wires.size() / 4,
                                 dt.public_first_indices.data(), dt.public_first_indices.size() / 2,
                                 (const size_t*)dt.perm, (const uint64_t*)dt.coef, dt.flags, dt.n_constraints,
                                 dt.n_wires, out, true);  // (device columns: one pack launch)
  ctx->trace_err = nullptr;
  return st;
}


stark_status stark_r1cs_circuit_new(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len, stark_r1cs_circuit** out) {
  if (!ctx || !r1cs || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  auto h = std::make_unique<stark_r1cs_circuit>();
  h->ctx = ctx;
  const stark_status st = circuit_build(ctx, r1cs, r1cs_len, h->c);
  hipStreamSynchronize(ctx->stream);
  if (st != STARK_OK) return st;
  *out = h.release();
  return STARK_OK;
}

void stark_r1cs_circuit_free(stark_r1cs_circuit* c) { delete c; }

stark_status stark_prove_r1cs_circuit(stark_ctx* ctx, const stark_r1cs_circuit* circuit, const uint8_t* wtns,
                                      size_t wtns_len, stark_r1cs_proof** out) {
  if (!ctx || !circuit || !wtns || !out || circuit->ctx != ctx || circuit->c.world != 1) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const PreparedCircuit& c = circuit->c;
  DevTrace dt;
  const stark_status st = circuit_witness(ctx, c, wtns, wtns_len, &dt);
  if (st != STARK_OK) return st;
  return mk_r1cs_proof_prepared(ctx, (const uint64_t*)dt.wit, (const uint64_t*)dt.comp, c.os, dt.public_wires.data(),
                                dt.public_wires.size() / 4, c.pfi.data(), c.pfi.size() / 2, (const size_t*)c.perm,
                                (const uint64_t*)c.coef, c.flags, c.n_c, c.n_wires, (const fe*)c.lde.ptr, out);
}

stark_status stark_dprove_circuit_new(stark_ctx* ctx, uint32_t world, uint32_t rank, const uint8_t* r1cs,
                                      size_t r1cs_len, stark_r1cs_circuit** out) {
  if (!ctx || !r1cs || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  if (world == 0 || world > 8 || (world & (world - 1)) || rank >= world) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  auto h = std::make_unique<stark_r1cs_circuit>();
  h->ctx = ctx;
  h->c.world = world;
  h->c.rank = rank;
  const stark_status st = circuit_build(ctx, r1cs, r1cs_len, h->c);
  hipStreamSynchronize(ctx->stream);
  if (st != STARK_OK) return st;
  *out = h.release();
  return STARK_OK;
}

stark_status stark_dprove_begin_circuit(stark_ctx* ctx, const stark_r1cs_circuit* circuit, const uint8_t* wtns,
                                        size_t wtns_len, void* stream, stark_dprove** out) {
  if (!ctx || !circuit || !wtns || !out || circuit->ctx != ctx) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const PreparedCircuit& c = circuit->c;
  DevTrace dt;
  stark_status st = circuit_witness(ctx, c, wtns, wtns_len, &dt);
  if (st != STARK_OK) return st;
  STARK_HIP(ctx, hipStreamSynchronize(ctx->stream));  // the witness columns are built on the context stream
  return dprove_begin_prepared(ctx, c.world, c.rank, (const uint64_t*)dt.wit, (const uint64_t*)dt.comp, c.os,
                               dt.public_wires.data(), dt.public_wires.size() / 4, c.pfi.data(), c.pfi.size() / 2,
                               (const size_t*)c.perm, (const uint64_t*)c.coef, c.flags, c.n_c, c.n_wires,
                               (const fe*)c.lde.ptr, stream, out);
}

}  // extern "C"
