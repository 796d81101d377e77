// C ABI: contexts, buffers, NTT entry points, Blake2s and the index sampler.
// Each extern "C" function cites the reference item it replaces in
// include/stark_hip.h.
#include <new>
#include <string.h>

#include "internal.h"
#include "host_b2s.h"
#include "host_json.h"
#include "blake2s.h"

namespace stark {

stark_status hip_fail(stark_ctx* ctx, hipError_t e, const char* what) {
  if (ctx) {
    ctx->last_error = std::string(what) + ": " + hipGetErrorString(e);
  }
  return e == hipErrorOutOfMemory ? STARK_ERR_OOM : STARK_ERR_HIP;
}

// STARK_POISON=1 (diagnostics): every device allocation of the library and every pinned staging buffer
// is filled with 0xA5 bytes when it is made, so a kernel that reads memory nobody wrote gives a
// reproducible wrong result instead of one that depends on what the memory held before.
bool poison_on() {
  static const bool on = [] {
    const char* v = getenv("STARK_POISON");
    return v && v[0] == '1';
  }();
  return on;
}
void poison_dev(void* p, size_t bytes) {
  if (poison_on() && p && bytes) {
    hipMemset(p, 0xA5, bytes);
    hipDeviceSynchronize();
  }
}

stark_status ensure_buf(stark_ctx* ctx, DevBuf& b, size_t bytes) {
  if (b.bytes >= bytes && b.ptr) return STARK_OK;
  if (b.ptr) {
    STARK_TRY(buf_drain(ctx, b));  // the last enqueued use (any stream) has finished before the buffer goes
    hipError_t e = hipFree(b.ptr);
    b.ptr = nullptr;
    b.bytes = 0;
    if (e != hipSuccess) return hip_fail(ctx, e, "hipFree");
  }
  // (on the context's device whatever the calling thread's current one is: group members run on
  // threads of their own)
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  hipError_t e = hipMalloc(&b.ptr, bytes ? bytes : 16);
  if (e != hipSuccess) {
    b.ptr = nullptr;
    return hip_fail(ctx, e, "hipMalloc");
  }
  poison_dev(b.ptr, bytes);
  b.bytes = bytes;
  return STARK_OK;
}

// Lazy ordering: a use only notes its stream (buf_release, no GPU work); when a call on another
// stream comes, an event recorded on the previous stream at that moment covers every use enqueued
// there, and the new stream waits for it.  (An event recorded after every use cost ~4 us of GPU time
// per NTT, tools/ab_libs.py; this costs one marker per change of stream.)  Hence the ABI rule that a
// stream handed to a call stays valid until the context's next call on another stream.
// The stream of a last use is kept as a non-null handle: the HIP null stream (stream 0) as kNullStream.
static const hipStream_t kNullStream = hipStreamLegacy;
static hipStream_t tag(hipStream_t s) { return s ? s : kNullStream; }
static hipStream_t untag(hipStream_t s) { return s == kNullStream ? nullptr : s; }

stark_status buf_acquire(stark_ctx* ctx, DevBuf& b, hipStream_t s) {
  if (b.last && b.last != tag(s)) {
    if (!b.ev) STARK_HIP(ctx, hipEventCreateWithFlags(&b.ev, hipEventDisableTiming));
    STARK_HIP(ctx, hipEventRecord(b.ev, untag(b.last)));
    STARK_HIP(ctx, hipStreamWaitEvent(s, b.ev, 0));
  }
  b.last = tag(s);
  return STARK_OK;
}

stark_status buf_release(stark_ctx* ctx, DevBuf& b, hipStream_t s) {
  (void)ctx;
  b.last = tag(s);
  return STARK_OK;
}

stark_status buf_drain(stark_ctx* ctx, DevBuf& b) {
  if (b.last) {
    STARK_HIP(ctx, hipStreamSynchronize(untag(b.last)));
    b.last = nullptr;
  }
  return STARK_OK;
}

stark_status fill_wait(stark_ctx* ctx, hipEvent_t ev, hipStream_t& fill, hipStream_t s) {
  if (!fill || fill == tag(s)) return STARK_OK;
  const hipError_t q = hipEventQuery(ev);
  if (q == hipSuccess) {
    fill = nullptr;  // the table is complete for every later reader
    return STARK_OK;
  }
  if (q != hipErrorNotReady) return hip_fail(ctx, q, "hipEventQuery(table fill)");
  STARK_HIP(ctx, hipStreamWaitEvent(s, ev, 0));
  return STARK_OK;
}

stark_status fill_mark(stark_ctx* ctx, hipEvent_t& ev, hipStream_t& fill, hipStream_t s) {
  if (!ev) STARK_HIP(ctx, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  STARK_HIP(ctx, hipEventRecord(ev, s));
  fill = tag(s);
  return STARK_OK;
}

size_t cache_bytes(const stark_ctx* ctx) {
  size_t b = 0;
  for (const auto& kv : ctx->tw) {
    const size_t full = ((size_t)1 << kv.second->log_n) * sizeof(fe);
    if (kv.second->d_full) b += full;
    if (kv.second->d_full_s) b += full;
  }
  for (const auto& kv : ctx->ext_idx) b += kv.second.bytes;
  for (const auto& kv : ctx->post_tw) b += kv.second.bytes;
  return b;
}

bool cache_reserve(stark_ctx* ctx, size_t need, bool evict_ext) {
  if (need > ctx->cache_limit) return false;
  bool synced = false;
  for (size_t have = cache_bytes(ctx); have + need > ctx->cache_limit;) {
    // the least recently used candidate
    fe** full_slot = nullptr;
    size_t full_bytes = 0;
    auto ext_it = ctx->ext_idx.end();
    uint64_t oldest = UINT64_MAX;
    for (auto& kv : ctx->tw) {
      Twiddles& t = *kv.second;
      const size_t bytes = ((size_t)1 << t.log_n) * sizeof(fe);
      if (t.d_full && t.full_used < oldest) {
        oldest = t.full_used;
        full_slot = &t.d_full;
        full_bytes = bytes;
      }
      if (t.d_full_s && t.full_s_used < oldest) {
        oldest = t.full_s_used;
        full_slot = &t.d_full_s;
        full_bytes = bytes;
      }
    }
    if (evict_ext)
      for (auto it = ctx->ext_idx.begin(); it != ctx->ext_idx.end(); ++it)
        if (it->second.used < oldest) {
          oldest = it->second.used;
          ext_it = it;
          full_slot = nullptr;
        }
    auto post_it = ctx->post_tw.end();  // (a candidate unless a call in progress holds it)
    for (auto it = ctx->post_tw.begin(); it != ctx->post_tw.end(); ++it)
      if (!it->second.in_use && it->second.used < oldest) {
        oldest = it->second.used;
        post_it = it;
        full_slot = nullptr;
        ext_it = ctx->ext_idx.end();
      }
    if (!full_slot && ext_it == ctx->ext_idx.end() && post_it == ctx->post_tw.end()) return false;
    if (!synced) {
      // A kernel of any stream may still read the victim.  After a failed synchronisation (a sticky
      // device error) nothing is freed: the caller does not cache, and the error surfaces at its
      // own next HIP call.
      if (hipDeviceSynchronize() != hipSuccess) return false;
      synced = true;
    }
    if (full_slot) {
      hipFree(*full_slot);
      *full_slot = nullptr;
      have -= full_bytes;
      for (auto& kv : ctx->tw)  // the victim's fill is complete (synchronised above)
        for (int d = 0; d < 2; ++d)
          if (full_slot == (d ? &kv.second->d_full_s : &kv.second->d_full)) kv.second->full_fill[d] = nullptr;
    } else if (post_it != ctx->post_tw.end()) {
      hipFree(post_it->second.ptr);
      if (post_it->second.ev) hipEventDestroy(post_it->second.ev);
      have -= post_it->second.bytes;
      ctx->post_tw.erase(post_it);
    } else {
      hipFree(ext_it->second.ptr);
      have -= ext_it->second.bytes;
      ctx->ext_idx.erase(ext_it);
    }
  }
  return true;
}

stark_status ctx_pinned(stark_ctx* ctx, int slot, size_t bytes, void** out) {
  if (ctx->pinned_bytes[slot] < bytes) {
    if (ctx->pinned[slot]) {
      // no copy or zero-copy kernel of any stream may still use the old buffer (it only ever grows)
      STARK_HIP(ctx, hipDeviceSynchronize());
      hipHostFree(ctx->pinned[slot]);
    }
    ctx->pinned[slot] = nullptr;
    ctx->pinned_bytes[slot] = 0;
    const size_t want = bytes < 4096 ? 4096 : bytes;
    // Coherent: kernels read and write this memory directly (zero-copy gathers).
    STARK_HIP(ctx, hipHostMalloc(&ctx->pinned[slot], want, hipHostMallocCoherent));
    if (poison_on()) memset(ctx->pinned[slot], 0xA5, want);
    ctx->pinned_bytes[slot] = want;
  }
  *out = ctx->pinned[slot];
  return STARK_OK;
}

stark_status ctx_tree(stark_ctx* ctx, int slot, stark_merkle_tree** out) {
  if (!ctx->trees[slot]) {
    stark_status st = stark_merkle_new(ctx, &ctx->trees[slot]);
    if (st != STARK_OK) return st;
  }
  *out = ctx->trees[slot];
  return STARK_OK;
}

// NULL = the context's stream; hipStreamLegacy (the legacy default stream as a handle: how a caller on
// torch's default stream names it, stark_amd.torch_stream) = the HIP null stream itself, which every HIP
// call takes as 0 (not every one accepts the handle value: hipStreamWaitEvent faults on it).
hipStream_t pick_stream(stark_ctx* ctx, void* stream) {
  if (!stream) return ctx->stream;
  return (hipStream_t)stream == hipStreamLegacy ? nullptr : (hipStream_t)stream;
}

// Host-buffer NTT: copy in (zero-padded), transform on the GPU, copy out.
static stark_status fft_host(stark_ctx* ctx, const uint64_t* in, size_t len, const uint64_t root[4], uint32_t log_n,
                             uint64_t* out, bool inverse) {
  if (!ctx || !root || !out || (len && !in)) return STARK_ERR_BAD_ARG;
  if (log_n > 28) return STARK_ERR_BAD_LENGTH;
  const size_t n = (size_t)1 << log_n;
  if (len > n) return STARK_ERR_BAD_LENGTH;  // fft.rs:162 assert_eq!(values.len(), order)
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const FieldHost& F = FieldHost::get();
  uint64_t use_root[4];
  memcpy(use_root, root, 32);
  if (inverse) {  // inv_serial_fft uses root^-1 (fft.rs:288)
    HostFp w = F.from_canonical(root);
    F.to_canonical(F.inv(w), use_root);
  }
  const Twiddles* tw = nullptr;
  stark_status st = get_twiddles(ctx, use_root, log_n, &tw);
  if (st != STARK_OK) return st;
  st = ensure_buf(ctx, ctx->io, n * sizeof(fe));
  if (st != STARK_OK) return st;
  fe* d = (fe*)ctx->io.ptr;
  // A power-of-two input padded by at most the first pass's radix: the pass
  // reads the len coefficients only (ntt_device_from), no zero fill.
  uint32_t log_len = 0;
  while (((size_t)1 << log_len) < len) ++log_len;
  const bool sparse = len && len < n && ((size_t)1 << log_len) == len && log_n >= 2 &&
                      log_n - log_len <= ntt_first_log_r(log_n);  // else zero fill (cheaper than a pad pass)
  if (sparse) {
    st = ensure_buf(ctx, ctx->io2, len * sizeof(fe));
    if (st != STARK_OK) return st;
    fe* src = (fe*)ctx->io2.ptr;
    STARK_HIP(ctx, hipMemcpyAsync(src, in, len * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    st = ntt_device_from(ctx, src, log_n - log_len, d, log_n, 1, *tw, inverse, ctx->stream);
  } else {
    if (len) STARK_HIP(ctx, hipMemcpyAsync(d, in, len * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
    if (len < n) STARK_HIP(ctx, hipMemsetAsync(d + len, 0, (n - len) * sizeof(fe), ctx->stream));
    st = ntt_device(ctx, d, log_n, 1, *tw, inverse, ctx->stream);
  }
  if (st != STARK_OK) return st;
  STARK_HIP(ctx, hipMemcpyAsync(out, d, n * sizeof(fe), hipMemcpyDeviceToHost, ctx->stream));
  STARK_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return STARK_OK;
}

}  // namespace stark

using namespace stark;

extern "C" {

const char* stark_status_str(stark_status s) {
  switch (s) {
    case STARK_OK: return "ok";
    case STARK_ERR_BAD_LENGTH: return "bad length";
    case STARK_ERR_BAD_ROOT: return "root is not a primitive 2^k-th root of unity";
    case STARK_ERR_BAD_ARG: return "bad argument";
    case STARK_ERR_OOM: return "out of memory";
    case STARK_ERR_HIP: return "HIP runtime error";
    case STARK_ERR_NO_DEVICE: return "no gfx950 device";
    case STARK_ERR_STATE: return "bad call order";
    case STARK_ERR_CHECK: return "constraint check failed";
  }
  return "unknown";
}

uint32_t stark_abi_version(void) { return STARK_ABI_VERSION; }
uint32_t stark_verify_simd_width(void) { return (uint32_t)b2s_paths_width(); }
uint32_t stark_json_simd_width(void) { return (uint32_t)json_simd_width(); }

stark_status stark_ctx_create(int device, stark_ctx** out) {
  if (!out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return STARK_ERR_NO_DEVICE;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return STARK_ERR_NO_DEVICE;
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return STARK_ERR_NO_DEVICE;
  stark_ctx* ctx = new (std::nothrow) stark_ctx();
  if (!ctx) return STARK_ERR_OOM;
  ctx->device = device;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking) != hipSuccess) {
    delete ctx;
    return STARK_ERR_HIP;
  }
  *out = ctx;
  return STARK_OK;
}

void stark_ctx_destroy(stark_ctx* ctx) {
  if (!ctx) return;
  hipSetDevice(ctx->device);
  hipStreamSynchronize(ctx->stream);
  hipDeviceSynchronize();  // (work the caller enqueued on its own streams may still read context buffers)
  for (auto& kv : ctx->tw) {
    if (kv.second->d_lo) hipFree(kv.second->d_lo);
    if (kv.second->d_full) hipFree(kv.second->d_full);
    if (kv.second->d_full_s) hipFree(kv.second->d_full_s);
    for (hipEvent_t e : kv.second->full_ev)
      if (e) hipEventDestroy(e);
  }
  for (stark_merkle_tree*& t : ctx->trees) {
    stark_merkle_free(t);
    t = nullptr;
  }
  for (stark_merkle_tree* t : ctx->fri_trees) stark_merkle_free(t);
  for (void* p : ctx->pinned)
    if (p) hipHostFree(p);
  for (auto& kv : ctx->ext_idx)
    if (kv.second.ptr) hipFree(kv.second.ptr);
  for (auto& kv : ctx->post_tw) {
    if (kv.second.ptr) hipFree(kv.second.ptr);
    if (kv.second.ev) hipEventDestroy(kv.second.ev);
  }
  if (ctx->staged) hipEventDestroy(ctx->staged);
  if (ctx->ev_aux) hipEventDestroy(ctx->ev_aux);
  if (ctx->aux) hipStreamDestroy(ctx->aux);
  ctx->fri_trees.clear();
  for (DevBuf* b : {&ctx->scratch, &ctx->io, &ctx->io2, &ctx->inv_tmp, &ctx->fri_cols, &ctx->r1cs_arena, &ctx->trace_arena, &ctx->trace_raw, &ctx->fri_misc,
                     &ctx->lde_tmp, &ctx->verify_arena, &ctx->verify_lde, &ctx->ext_idx_tmp, &ctx->spot}) {
    if (b->ptr) hipFree(b->ptr);
    if (b->ev) hipEventDestroy(b->ev);
  }
  hipStreamDestroy(ctx->stream);
  delete ctx;
}

const char* stark_ctx_last_error(const stark_ctx* ctx) { return ctx ? ctx->last_error.c_str() : ""; }

stark_status stark_ctx_set_cache_limit(stark_ctx* ctx, size_t bytes) {
  if (!ctx) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  ctx->cache_limit = bytes;
  cache_reserve(ctx, 0, true);  // down to the new cap at once (every cached entry is a candidate here)
  return STARK_OK;
}

stark_status stark_ctx_memory(const stark_ctx* ctx, size_t* cached_bytes, size_t* cache_limit,
                              size_t* resident_bytes) {
  if (!ctx) return STARK_ERR_BAD_ARG;
  const size_t cached = cache_bytes(ctx);
  size_t total = cached;
  for (const auto& kv : ctx->tw) total += kv.second->base_bytes;
  for (const DevBuf* b : {&ctx->scratch, &ctx->io, &ctx->io2, &ctx->inv_tmp, &ctx->fri_cols, &ctx->r1cs_arena, &ctx->trace_arena,
                          &ctx->trace_raw, &ctx->fri_misc, &ctx->lde_tmp, &ctx->verify_arena, &ctx->verify_lde,
                          &ctx->ext_idx_tmp, &ctx->spot})
    total += b->ptr ? b->bytes : 0;
  for (const stark_merkle_tree* t : ctx->trees) total += merkle_device_bytes(t);
  for (const stark_merkle_tree* t : ctx->fri_trees) total += merkle_device_bytes(t);
  if (cached_bytes) *cached_bytes = cached;
  if (cache_limit) *cache_limit = ctx->cache_limit;
  if (resident_bytes) *resident_bytes = total;
  return STARK_OK;
}
void* stark_ctx_stream(stark_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

stark_status stark_best_fft(stark_ctx* ctx, const uint64_t* coeffs, size_t len, const uint64_t root[4], uint32_t log_n,
                            uint64_t* out) {
  return fft_host(ctx, coeffs, len, root, log_n, out, false);
}

stark_status stark_inv_best_fft(stark_ctx* ctx, const uint64_t* evals, size_t len, const uint64_t root[4],
                                uint32_t log_n, uint64_t* out) {
  return fft_host(ctx, evals, len, root, log_n, out, true);
}

stark_status stark_fft_in_place(stark_ctx* ctx, uint64_t* values, const uint64_t root[4], uint32_t log_n,
                                int inverse) {
  if (log_n > 28) return STARK_ERR_BAD_LENGTH;
  return fft_host(ctx, values, (size_t)1 << log_n, root, log_n, values, inverse != 0);
}

stark_status stark_ntt_dev(stark_ctx* ctx, uint64_t* d_data, uint32_t log_n, uint32_t batch, const uint64_t root[4],
                           int inverse, void* stream) {
  if (!ctx || !d_data || !root) return STARK_ERR_BAD_ARG;
  if (log_n > 28) return STARK_ERR_BAD_LENGTH;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const FieldHost& F = FieldHost::get();
  uint64_t use_root[4];
  memcpy(use_root, root, 32);
  if (inverse) F.to_canonical(F.inv(F.from_canonical(root)), use_root);
  const Twiddles* tw = nullptr;
  stark_status st = get_twiddles(ctx, use_root, log_n, &tw);
  if (st != STARK_OK) return st;
  return ntt_device(ctx, (fe*)d_data, log_n, batch, *tw, inverse != 0, pick_stream(ctx, stream));
}

stark_status stark_lde_dev(stark_ctx* ctx, uint64_t* d_values, uint64_t* d_out, uint32_t log_steps,
                           uint32_t log_blowup, uint32_t batch, const uint64_t g1[4], const uint64_t g2[4],
                           void* stream) {
  if (!ctx || !d_values || !d_out || !g1 || !g2 || d_values == d_out) return STARK_ERR_BAD_ARG;
  if (log_steps + log_blowup > 28) return STARK_ERR_BAD_LENGTH;
  if (batch == 0) return STARK_OK;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const FieldHost& F = FieldHost::get();
  // g1 must be g2^(2^log_blowup) (prove.rs:71-94: g1 = g2^extension_factor).
  const HostFp w2 = F.from_canonical(g2);
  if (!FieldHost::eq(F.pow_u64(w2, (uint64_t)1 << log_blowup), F.from_canonical(g1))) return STARK_ERR_BAD_ROOT;
  uint64_t g1_inv[4];
  F.to_canonical(F.inv(F.from_canonical(g1)), g1_inv);
  const Twiddles *t1 = nullptr, *t2 = nullptr;
  stark_status st = get_twiddles(ctx, g1_inv, log_steps, &t1);
  if (st != STARK_OK) return st;
  st = get_twiddles(ctx, g2, log_steps + log_blowup, &t2);
  if (st != STARK_OK) return st;
  hipStream_t s = pick_stream(ctx, stream);
  st = ntt_device(ctx, (fe*)d_values, log_steps, batch, *t1, true, s);  // inv_best_fft(values, g1)
  if (st != STARK_OK) return st;
  // best_fft(coefficients zero-padded to 2^(log_steps + log_blowup), g2)
  return ntt_device_from(ctx, (const fe*)d_values, log_blowup, (fe*)d_out, log_steps + log_blowup, batch, *t2, false,
                         s);
}

stark_status stark_lde(stark_ctx* ctx, const uint64_t* values, size_t steps, const uint64_t g1[4],
                       uint32_t log_blowup, const uint64_t g2[4], uint64_t* out) {
  if (!ctx || !values || !out || !g1 || !g2 || steps == 0 || (steps & (steps - 1))) return STARK_ERR_BAD_ARG;
  uint32_t log_steps = 0;
  while (((size_t)1 << log_steps) < steps) ++log_steps;
  if (log_steps + log_blowup > 28) return STARK_ERR_BAD_LENGTH;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  const size_t prec = steps << log_blowup;
  stark_status st = ensure_buf(ctx, ctx->io, prec * sizeof(fe));
  if (st != STARK_OK) return st;
  st = ensure_buf(ctx, ctx->io2, steps * sizeof(fe));
  if (st != STARK_OK) return st;
  fe* d_in = (fe*)ctx->io2.ptr;
  fe* d_out = (fe*)ctx->io.ptr;
  STARK_HIP(ctx, hipMemcpyAsync(d_in, values, steps * sizeof(fe), hipMemcpyHostToDevice, ctx->stream));
  st = stark_lde_dev(ctx, (uint64_t*)d_in, (uint64_t*)d_out, log_steps, log_blowup, 1, g1, g2, nullptr);
  if (st != STARK_OK) return st;
  STARK_HIP(ctx, hipMemcpyAsync(out, d_out, prec * sizeof(fe), hipMemcpyDeviceToHost, ctx->stream));
  STARK_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return STARK_OK;
}

void stark_blake(const uint8_t* msg, size_t len, uint8_t out[32]) { b2s_host(msg, len, out); }

stark_status stark_get_pseudorandom_indices(const uint8_t* seed, size_t seed_len, uint32_t modulus, size_t count,
                                            uint32_t exclude_multiples_of, uint32_t* out) {
  if ((count && !out) || (seed_len && !seed)) return STARK_ERR_BAD_ARG;
  if (modulus >= (1u << 24)) return STARK_ERR_BAD_ARG;  // fri/src/utils.rs:88
  // data[len-32..] must exist when the seed is extended (utils.rs:91).
  if (seed_len < 4 * count && seed_len < 32) return STARK_ERR_BAD_ARG;
  uint32_t real_mod = modulus;
  if (exclude_multiples_of != 0) {
    if (exclude_multiples_of == 1) return STARK_ERR_BAD_ARG;  // division by zero in the reference
    // The reference computes modulus * (e - 1) in u32 (utils.rs:101); refuse inputs where that overflows.
    if ((uint64_t)modulus * (exclude_multiples_of - 1) > 0xFFFFFFFFull) return STARK_ERR_BAD_ARG;
    real_mod = (uint32_t)((uint64_t)modulus * (exclude_multiples_of - 1) / exclude_multiples_of);
  }
  if (count && real_mod == 0) return STARK_ERR_BAD_ARG;  // % 0 panics in the reference
  std::vector<uint8_t> data(seed, seed + seed_len);
  while (data.size() < 4 * count) {
    uint8_t d[32];
    b2s_host(data.data() + data.size() - 32, 32, d);
    data.insert(data.end(), d, d + 32);
  }
  for (size_t i = 0; i < count; ++i) {
    const uint32_t w = ((uint32_t)data[4 * i] << 24) | ((uint32_t)data[4 * i + 1] << 16) |
                       ((uint32_t)data[4 * i + 2] << 8) | (uint32_t)data[4 * i + 3];
    const uint32_t v = w % real_mod;
    out[i] = exclude_multiples_of ? v + 1 + v / (exclude_multiples_of - 1) : v;
  }
  return STARK_OK;
}

stark_status stark_dev_alloc(stark_ctx* ctx, size_t bytes, void** d_ptr) {
  if (!ctx || !d_ptr) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  STARK_HIP(ctx, hipMalloc(d_ptr, bytes ? bytes : 16));
  poison_dev(*d_ptr, bytes);
  return STARK_OK;
}
stark_status stark_dev_free(stark_ctx* ctx, void* d_ptr) {
  if (!ctx) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  STARK_HIP(ctx, hipFree(d_ptr));
  return STARK_OK;
}
stark_status stark_memcpy_h2d(stark_ctx* ctx, void* d_dst, const void* h_src, size_t bytes) {
  if (!ctx) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  STARK_HIP(ctx, hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, ctx->stream));
  STARK_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return STARK_OK;
}
stark_status stark_memcpy_d2h(stark_ctx* ctx, void* h_dst, const void* d_src, size_t bytes) {
  if (!ctx) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  STARK_HIP(ctx, hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  STARK_HIP(ctx, hipStreamSynchronize(ctx->stream));
  return STARK_OK;
}
stark_status stark_ctx_synchronize(stark_ctx* ctx) {
  if (!ctx) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  STARK_HIP(ctx, hipStreamSynchronize(ctx->stream));
  // Every stream the context's buffers were last used on is drained, and no longer referenced.
  for (DevBuf* b : {&ctx->scratch, &ctx->io2, &ctx->fri_misc}) STARK_TRY(buf_drain(ctx, *b));
  return STARK_OK;
}

}  // extern "C"
