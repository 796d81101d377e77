// R1CS front end (host C++): the binary readers and the trace construction
// that feed mk_r1cs_proof.
//
//   read_r1cs     packages/circom2bellman_core/src/reader.rs:4-89
//   read_witness  packages/r1cs-stark/src/reader.rs:7-42
//   prove_with_witness up to the prover call, run.rs:310-437:
//     calc_coefficients_and_witness run.rs:109-281, calc_flags :283-308,
//     permuted indices :388-401, public_first_indices :411-419.
//
// The reference panics on malformed input (bytes::Buf underflow, assert_eq!);
// this returns STARK_ERR_BAD_ARG instead.
#include <string.h>

#include <memory>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

#include "internal.h"

namespace stark {
namespace {

// Large host buffers of freed traces are kept for the next build (a few, at
// most 1 GiB): a fresh multi-MB allocation is mmapped and first-touch page
// faults cost as much as filling it (milliseconds at 2^20 steps, serialised
// on the address-space lock across the fill threads).
class HostPool {
 public:
  static HostPool& get() {
    static HostPool p;
    return p;
  }
  void* take(size_t bytes, size_t* cap) {
    {
      std::lock_guard<std::mutex> g(m_);
      size_t best = free_.size();
      for (size_t i = 0; i < free_.size(); ++i)
        if (free_[i].second >= bytes && free_[i].second <= 2 * bytes + (1u << 20) &&
            (best == free_.size() || free_[i].second < free_[best].second))
          best = i;
      if (best != free_.size()) {
        void* q = free_[best].first;
        *cap = free_[best].second;
        cached_ -= *cap;
        free_.erase(free_.begin() + (long)best);
        return q;
      }
    }
    *cap = bytes;
    return malloc(bytes ? bytes : 8);
  }
  void give(void* q, size_t cap) {
    if (!q) return;
    if (cap < ((size_t)1 << 20)) {
      free(q);
      return;
    }
    std::lock_guard<std::mutex> g(m_);
    free_.emplace_back(q, cap);
    cached_ += cap;
    while (free_.size() > kMaxBuffers || cached_ > kMaxBytes) {
      cached_ -= free_.front().second;
      free(free_.front().first);
      free_.erase(free_.begin());
    }
  }

 private:
  static constexpr size_t kMaxBuffers = 8;
  static constexpr size_t kMaxBytes = (size_t)1 << 30;
  std::mutex m_;
  std::vector<std::pair<void*, size_t>> free_;
  size_t cached_ = 0;
};

// Runs fn(lo, hi) over [0, n) in contiguous ranges on the host workers
// (inline when n < min_per_thread * 2).
template <class Fn>
void parallel_ranges(size_t n, size_t min_per_thread, Fn&& fn) {
  size_t nt = host_threads();
  const size_t by_size = n / (min_per_thread ? min_per_thread : 1);
  if (by_size < nt) nt = by_size;
  if (nt <= 1) {
    fn((size_t)0, n);
    return;
  }
  host_parallel((unsigned)nt, [&](unsigned k) { fn(n * k / nt, n * (k + 1) / nt); });
}

}  // namespace
}  // namespace stark

// Uninitialised u64 array (every element is written by the builder), from the pool.
struct U64Array {
  uint64_t* p = nullptr;
  size_t n = 0, cap = 0;
  U64Array() = default;
  U64Array(const U64Array&) = delete;
  U64Array& operator=(const U64Array&) = delete;
  ~U64Array() { stark::HostPool::get().give(p, cap); }
  bool alloc(size_t count) {
    stark::HostPool::get().give(p, cap);
    p = (uint64_t*)stark::HostPool::get().take(count * sizeof(uint64_t), &cap);
    n = p ? count : 0;
    return p != nullptr;
  }
  uint64_t* data() const { return p; }
  uint64_t& operator[](size_t i) { return p[i]; }
  size_t size() const { return n; }
};

struct stark_r1cs_trace {
  size_t n_constraints = 0, n_wires = 0;
  U64Array witness_trace, computational_trace, coefficients;  // 4 limbs per element
  std::vector<uint8_t> flags;                                // flag0 | flag1 | flag2, one byte per slot
  U64Array permuted_indices;
  std::vector<uint64_t> public_wires;
  std::vector<size_t> public_first_indices;  // (k, w) pairs
};

namespace stark {
stark_status mk_r1cs_proof_bytes_flags(stark_ctx* ctx, const uint64_t* witness_trace,
                                      const uint64_t* computational_trace, size_t os, const uint64_t* public_wires,
                                      size_t n_public, const size_t* public_first_indices, size_t n_pfi,
                                      const size_t* permuted_indices, const uint64_t* coefficients,
                                      const uint8_t* flag_bytes, size_t n_constraints, size_t n_wires,
                                      stark_r1cs_proof** out, bool dev_in);
}

namespace stark {
namespace {

struct Cursor {
  const uint8_t* p;
  size_t left;
  bool ok = true;
  uint32_t u32() {
    if (left < 4) return fail();
    uint32_t v;
    memcpy(&v, p, 4);
    p += 4;
    left -= 4;
    return v;
  }
  uint64_t u64() {
    if (left < 8) return fail();
    uint64_t v;
    memcpy(&v, p, 8);
    p += 8;
    left -= 8;
    return v;
  }
  const uint8_t* raw(size_t n) {
    if (left < n) {
      fail();
      return nullptr;
    }
    const uint8_t* r = p;
    p += n;
    left -= n;
    return r;
  }
  uint32_t fail() {
    ok = false;
    left = 0;
    return 0;
  }
};

struct Coefficient {
  uint32_t wire_id;
  const uint8_t* value;  // 32 B little endian
};

const uint8_t kBn254R[32] = {1,   0,  0,   240, 147, 245, 225, 67,  145, 112, 185, 121, 72,  232, 51, 40,
                             93,  88, 129, 129, 182, 69,  80,  184, 41,  160, 49,  225, 114, 78,  100, 48};

void push_canon(std::vector<uint64_t>& v, const HostFp& x) {
  uint64_t c[4];
  FieldHost::get().to_canonical(x, c);
  v.insert(v.end(), c, c + 4);
}

}  // namespace

stark_status parse_r1cs_header(const uint8_t* r1cs, size_t len, R1csHeader* h) {
  if (!r1cs || !h) return STARK_ERR_BAD_ARG;
  Cursor c{r1cs, len};
  if (c.u32() != 0x73633172u /* "r1cs" */ || c.u32() != 1 || c.u32() != 3 || c.u32() != 1) return STARK_ERR_BAD_ARG;
  c.u64();
  c.u32();  // field_size
  const uint8_t* prime = c.raw(32);
  h->n_wires = c.u32();
  h->n_pub_out = c.u32();
  h->n_pub_in = c.u32();
  c.u32();  // n_private_inputs
  c.u64();  // n_labels
  h->n_constraints = c.u32();
  if (!c.ok || memcmp(prime, kBn254R, 32) != 0) return STARK_ERR_BAD_ARG;  // run.rs:344-350
  if (c.u32() != 2) return STARK_ERR_BAD_ARG;                               // ConstraintSection
  c.u64();
  if (!c.ok || h->n_wires == 0) return STARK_ERR_BAD_ARG;
  h->cons_off = len - c.left;
  return STARK_OK;
}

stark_status parse_wtns_header(const uint8_t* wtns, size_t len, WtnsHeader* h) {
  if (!wtns || !h) return STARK_ERR_BAD_ARG;
  Cursor w{wtns, len};
  if (w.u32() != 1936618615u) return STARK_ERR_BAD_ARG;  // "wtns"
  for (int i = 0; i < 5; ++i) w.u32();
  h->field_size = w.u32();
  if (h->field_size == 0 || h->field_size > 32 || h->field_size % 4) return STARK_ERR_BAD_ARG;
  w.raw(h->field_size);
  h->n_wit = w.u32();
  w.u32();
  w.u32();
  w.u32();
  if (!w.ok || (uint64_t)h->n_wit * h->field_size > w.left) return STARK_ERR_BAD_ARG;
  h->values_off = len - w.left;
  return STARK_OK;
}

}  // namespace stark

using namespace stark;

extern "C" {

stark_status stark_r1cs_trace_build(const uint8_t* r1cs, size_t r1cs_len, const uint8_t* wtns, size_t wtns_len,
                                    stark_r1cs_trace** out) {
  if (!r1cs || !wtns || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  PhaseClock clk("r1cs trace build");
  const FieldHost& F = FieldHost::get();
  // ---- read_r1cs (reader.rs:4-89): header section, then constraints, in that order.
  R1csHeader hd;
  stark_status hst = parse_r1cs_header(r1cs, r1cs_len, &hd);
  if (hst != STARK_OK) return hst;
  const uint32_t n_wires = hd.n_wires, n_pub_out = hd.n_pub_out, n_pub_in = hd.n_pub_in;
  const uint32_t n_constraints = hd.n_constraints;
  Cursor c{r1cs + hd.cons_off, r1cs_len - hd.cons_off};
  // All coefficients in file order (wire id + pointer to the 32-B value in
  // the file); factor k = coefs[fac_off[k], fac_off[k+1]).  Pooled buffers:
  // every entry read is written first.
  U64Array coef_buf, fac_buf;
  if (!coef_buf.alloc(2 * (r1cs_len / 36 + 1)) || !fac_buf.alloc((size_t)3 * n_constraints + 1)) return STARK_ERR_OOM;
  static_assert(sizeof(Coefficient) == 16, "two u64 per coefficient");
  Coefficient* coefs = reinterpret_cast<Coefficient*>(coef_buf.data());
  uint64_t* fac_off = fac_buf.data();
  fac_off[0] = 0;
  size_t n_coefs = 0;
  for (uint32_t i = 0; i < n_constraints && c.ok; ++i)
    for (int f = 0; f < 3; ++f) {
      const uint32_t nc = c.u32();
      if (nc > c.left / 36) return STARK_ERR_BAD_ARG;
      const uint8_t* rec = c.raw((size_t)nc * 36);
      for (uint32_t k = 0; k < nc; ++k, rec += 36) {
        uint32_t wire;
        memcpy(&wire, rec, 4);
        if (wire >= n_wires) return STARK_ERR_BAD_ARG;
        coefs[n_coefs].wire_id = wire;
        coefs[n_coefs].value = rec + 4;
        ++n_coefs;
      }
      fac_off[(size_t)3 * i + f + 1] = n_coefs;
    }
  if (!c.ok || n_wires == 0) return STARK_ERR_BAD_ARG;

  clk.mark("read_r1cs");
  // ---- read_witness (r1cs-stark/src/reader.rs:7-42)
  WtnsHeader wh;
  hst = parse_wtns_header(wtns, wtns_len, &wh);
  if (hst != STARK_OK) return hst;
  const uint32_t field_size = wh.field_size, n_wit = wh.n_wit;
  // from_bytes_le reduces mod p (run.rs:354-357): wcan holds the canonical
  // values (the trace's witness column), witness their Montgomery images (the
  // products' right operand).
  const uint8_t* wbytes = wtns + wh.values_off;
  U64Array wbuf;
  if (!wbuf.alloc((size_t)8 * n_wit + 8)) return STARK_ERR_OOM;
  HostFp* witness = reinterpret_cast<HostFp*>(wbuf.data());
  HostFp* wcan = witness + n_wit;
  parallel_ranges(n_wit, 1u << 12, [&](size_t lo, size_t hi) {
    for (size_t i = lo; i < hi; ++i) {
      wcan[i] = F.reduce_bytes_le(wbytes + i * field_size, field_size);
      witness[i] = F.from_canonical(wcan[i].v);
    }
  });
  if (n_wit < n_wires || !FieldHost::eq(witness[0], F.one())) return STARK_ERR_BAD_ARG;  // run.rs:358

  clk.mark("read_witness");
  auto t = std::make_unique<stark_r1cs_trace>();
  t->n_constraints = n_constraints;
  t->n_wires = n_wires;
  const size_t n_public = 1 + (size_t)n_pub_in + n_pub_out;  // run.rs:359-360
  if (n_public > n_wit) return STARK_ERR_BAD_ARG;
  for (size_t i = 0; i < n_public; ++i) push_canon(t->public_wires, witness[i]);  // run.rs:359-360

  // ---- calc_coefficients_and_witness (run.rs:109-281)
  // Constraint ci owns n_coeff = max(|A|, |B|, |C|) slots starting at base[ci]
  // in each of the three factor thirds of the trace.
  U64Array base_buf;
  if (!base_buf.alloc((size_t)n_constraints + 1)) return STARK_ERR_OOM;
  uint64_t* base = base_buf.data();
  base[0] = 0;
  for (uint32_t ci = 0; ci < n_constraints; ++ci) {
    uint64_t n_coeff = 0;
    for (int f = 0; f < 3; ++f) {
      const uint64_t k = fac_off[(size_t)3 * ci + f + 1] - fac_off[(size_t)3 * ci + f];
      if (k > n_coeff) n_coeff = k;
    }
    base[ci + 1] = base[ci] + n_coeff;
  }
  const size_t a_len = base[n_constraints];
  const size_t os = 3 * a_len;
  if (a_len == 0) return STARK_ERR_BAD_ARG;
  // Canonical arithmetic: montmul(c_canonical, w_montgomery) = c * w canonical,
  // so each slot costs one modular product and no conversions.
  clk.mark("slot bases");
  if (!t->witness_trace.alloc(4 * os) || !t->computational_trace.alloc(4 * os) || !t->coefficients.alloc(4 * os))
    return STARK_ERR_OOM;
  // Slot filling is independent per constraint: split the constraints over threads.
  auto fill = [&](uint32_t c0, uint32_t c1) {
    for (uint32_t ci = c0; ci < c1; ++ci) {
      const uint64_t n_coeff = base[ci + 1] - base[ci];
      for (int f = 0; f < 3; ++f) {
        const uint64_t lo = fac_off[(size_t)3 * ci + f], hi = fac_off[(size_t)3 * ci + f + 1];
        HostFp tacc = F.zero();
        for (uint64_t i = 0; i < n_coeff; ++i) {
          const size_t slot = (size_t)f * a_len + base[ci] + i;
          size_t wire = n_wires - 1;  // padding slot: last wire, coefficient 0, trace unchanged
          HostFp coef = F.zero();
          if (lo + i < hi) {
            wire = coefs[lo + i].wire_id;
            coef = F.reduce_bytes_le(coefs[lo + i].value, 32);  // canonical from_bytes_le
            tacc = F.add(tacc, F.mul(coef, witness[wire]));
          }
          memcpy(&t->witness_trace[4 * slot], wcan[wire].v, 32);
          memcpy(&t->computational_trace[4 * slot], tacc.v, 32);
          memcpy(&t->coefficients[4 * slot], coef.v, 32);
        }
      }
    }
  };
  parallel_ranges(n_constraints, os < (1u << 16) ? n_constraints + 1 : 1u << 12,
                  [&](size_t lo, size_t hi) { fill((uint32_t)lo, (uint32_t)hi); });
  clk.mark("slot fill (threads)");
  // ---- calc_flags (run.rs:283-308): flag0 = 1, flag1 = 0 at each constraint's
  // first slot (in all three thirds), flag2 = 1 at its last slot.
  t->flags.assign(3 * os, 0);
  uint8_t* f0 = t->flags.data();
  uint8_t* f1 = f0 + os;
  uint8_t* f2 = f1 + os;
  memset(f0, 1, os);
  memset(f1, 1, os);
  for (uint32_t ci = 0; ci < n_constraints; ++ci) {
    const size_t k = base[ci + 1] % a_len;  // (last_coeff + 1) % a_trace_len
    f1[k] = f1[k + a_len] = f1[k + 2 * a_len] = 0;
  }
  for (uint32_t ci = 0; ci < n_constraints; ++ci) f2[base[ci + 1] - 1] = 1;
  clk.mark("flags");
  // ---- wire uses in push order (run.rs:160, 195, 230: factor A's slots, then B's, then C's per
  // constraint), as trace positions a_len * factor + slot; counting sort by wire.
  // Uses of constraints [c0, c1) in push order.
  auto for_each_use = [&](uint32_t c0, uint32_t c1, auto&& fn) {
    for (uint32_t ci = c0; ci < c1; ++ci) {
      const uint64_t n_coeff = base[ci + 1] - base[ci];
      for (int f = 0; f < 3; ++f) {
        const uint64_t lo = fac_off[(size_t)3 * ci + f], hi = fac_off[(size_t)3 * ci + f + 1];
        for (uint64_t i = 0; i < n_coeff; ++i)
          fn(lo + i < hi ? coefs[lo + i].wire_id : n_wires - 1, (size_t)f * a_len + base[ci] + i);
      }
    }
  };
  // Stable parallel counting sort: thread k owns a contiguous constraint range
  // (so its uses are contiguous in push order), counts its uses per wire, and
  // scatters them after wire-major, thread-minor offsets are known.
  unsigned nt = host_threads();
  while (nt > 1 && ((uint64_t)n_wires * nt > 4 * (uint64_t)os + (1u << 16) || n_constraints < 1024u * nt)) --nt;
  std::vector<uint32_t> cut(nt + 1);
  for (unsigned k = 0; k <= nt; ++k) cut[k] = (uint32_t)((uint64_t)n_constraints * k / nt);
  U64Array cnt_buf;  // cnt[k * n_wires + wire], zeroed by thread k
  if (!cnt_buf.alloc((size_t)nt * n_wires + 1)) return STARK_ERR_OOM;
  uint64_t* cnt = cnt_buf.data();
  auto run = [&](auto&& body) { host_parallel(nt, [&](unsigned k) { body(k); }); };
  run([&](unsigned k) {
    uint64_t* c = cnt + (size_t)k * n_wires;
    memset(c, 0, (size_t)n_wires * sizeof(uint64_t));
    for_each_use(cut[k], cut[k + 1], [&](size_t wire, size_t) { ++c[wire]; });
  });
  std::vector<uint64_t> use_off((size_t)n_wires + 1, 0);
  {
    uint64_t at = 0;
    for (size_t wi = 0; wi < n_wires; ++wi) {
      use_off[wi] = at;
      for (unsigned k = 0; k < nt; ++k) {
        const uint64_t c = cnt[(size_t)k * n_wires + wi];
        cnt[(size_t)k * n_wires + wi] = at;  // becomes thread k's cursor for this wire
        at += c;
      }
    }
    use_off[n_wires] = at;
  }
  U64Array uses_buf;
  if (!uses_buf.alloc(os)) return STARK_ERR_OOM;
  uint64_t* uses = uses_buf.data();
  run([&](unsigned k) {
    uint64_t* cur = cnt + (size_t)k * n_wires;
    for_each_use(cut[k], cut[k + 1], [&](size_t wire, size_t pos) { uses[cur[wire]++] = pos; });
  });
  clk.mark("wire uses (counting sort)");
  // ---- permuted indices (run.rs:388-401): a cycle through every wire's uses.
  if (!t->permuted_indices.alloc(os)) return STARK_ERR_OOM;
  parallel_ranges(n_wires, 1u << 12, [&](size_t w0, size_t w1) {
    for (size_t wi = w0; wi < w1; ++wi) {
      const uint64_t lo = use_off[wi], hi = use_off[wi + 1];
      if (lo == hi) continue;
      uint64_t old_w = uses[hi - 1];
      for (uint64_t j = lo; j < hi; ++j) {
        t->permuted_indices[uses[j]] = old_w;
        old_w = uses[j];
      }
    }
  });
  // ---- public_first_indices (run.rs:411-419)
  for (size_t wi = 0; wi < n_public && wi < n_wires; ++wi)
    if (use_off[wi] != use_off[wi + 1]) {
      t->public_first_indices.push_back(wi);
      t->public_first_indices.push_back(uses[use_off[wi]]);
    }
  clk.mark("permutation + public firsts");
  *out = t.release();
  return STARK_OK;
}

stark_status stark_r1cs_trace_dims(const stark_r1cs_trace* t, size_t* original_steps, size_t* n_public,
                                   size_t* n_public_first, size_t* n_constraints, size_t* n_wires) {
  if (!t) return STARK_ERR_BAD_ARG;
  if (original_steps) *original_steps = t->coefficients.size() / 4;
  if (n_public) *n_public = t->public_wires.size() / 4;
  if (n_public_first) *n_public_first = t->public_first_indices.size() / 2;
  if (n_constraints) *n_constraints = t->n_constraints;
  if (n_wires) *n_wires = t->n_wires;
  return STARK_OK;
}

stark_status stark_r1cs_trace_export(const stark_r1cs_trace* t, uint64_t* witness_trace, uint64_t* computational_trace,
                                     uint64_t* coefficients, uint64_t* flag0, uint64_t* flag1, uint64_t* flag2,
                                     size_t* permuted_indices, uint64_t* public_wires, size_t* public_first_indices) {
  if (!t) return STARK_ERR_BAD_ARG;
  auto cp = [](void* dst, const void* src, size_t bytes) {
    if (dst && bytes) memcpy(dst, src, bytes);
  };
  cp(witness_trace, t->witness_trace.data(), t->witness_trace.size() * 8);
  cp(computational_trace, t->computational_trace.data(), t->computational_trace.size() * 8);
  cp(coefficients, t->coefficients.data(), t->coefficients.size() * 8);
  const size_t os = t->coefficients.size() / 4;
  uint64_t* fl[3] = {flag0, flag1, flag2};
  for (int f = 0; f < 3; ++f)
    if (fl[f])
      for (size_t i = 0; i < os; ++i) {
        fl[f][4 * i] = t->flags[f * os + i];
        fl[f][4 * i + 1] = fl[f][4 * i + 2] = fl[f][4 * i + 3] = 0;
      }
  cp(permuted_indices, t->permuted_indices.data(), t->permuted_indices.size() * sizeof(size_t));
  cp(public_wires, t->public_wires.data(), t->public_wires.size() * 8);
  cp(public_first_indices, t->public_first_indices.data(), t->public_first_indices.size() * sizeof(size_t));
  return STARK_OK;
}

void stark_r1cs_trace_free(stark_r1cs_trace* t) { delete t; }

stark_status stark_prove_r1cs_trace(stark_ctx* ctx, const stark_r1cs_trace* t, stark_r1cs_proof** out) {
  if (!t) return STARK_ERR_BAD_ARG;
  return mk_r1cs_proof_bytes_flags(ctx, t->witness_trace.data(), t->computational_trace.data(),
                                   t->coefficients.size() / 4, t->public_wires.data(), t->public_wires.size() / 4,
                                   t->public_first_indices.data(), t->public_first_indices.size() / 2,
                                   (const size_t*)t->permuted_indices.data(), t->coefficients.data(),
                                   t->flags.data(), t->n_constraints, t->n_wires, out);
}

}  // extern "C"
