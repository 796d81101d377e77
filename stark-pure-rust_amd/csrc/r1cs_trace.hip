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

#include <vector>

#include "internal.h"

struct stark_r1cs_trace {
  size_t n_constraints = 0, n_wires = 0;
  std::vector<uint64_t> witness_trace, computational_trace, coefficients, flag0, flag1, flag2;  // 4 limbs each
  std::vector<size_t> permuted_indices;
  std::vector<uint64_t> public_wires;
  std::vector<size_t> public_first_indices;  // (k, w) pairs
};

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
}  // namespace stark

using namespace stark;

extern "C" {

stark_status stark_r1cs_trace_build(const uint8_t* r1cs, size_t r1cs_len, const uint8_t* wtns, size_t wtns_len,
                                    stark_r1cs_trace** out) {
  if (!r1cs || !wtns || !out) return STARK_ERR_BAD_ARG;
  *out = nullptr;
  const FieldHost& F = FieldHost::get();
  // ---- read_r1cs (reader.rs:4-89): header section, then constraints, in that order.
  Cursor c{r1cs, r1cs_len};
  if (c.u32() != 0x73633172u /* "r1cs" */ || c.u32() != 1 || c.u32() != 3 || c.u32() != 1) return STARK_ERR_BAD_ARG;
  c.u64();
  c.u32();  // field_size
  const uint8_t* prime = c.raw(32);
  const uint32_t n_wires = c.u32();
  const uint32_t n_pub_out = c.u32();
  const uint32_t n_pub_in = c.u32();
  c.u32();  // n_private_inputs
  c.u64();  // n_labels
  const uint32_t n_constraints = c.u32();
  if (!c.ok || memcmp(prime, kBn254R, 32) != 0) return STARK_ERR_BAD_ARG;  // run.rs:344-350
  if (c.u32() != 2) return STARK_ERR_BAD_ARG;                               // ConstraintSection
  c.u64();
  std::vector<std::vector<Coefficient>> factors;  // 3 per constraint
  factors.reserve((size_t)3 * n_constraints);
  for (uint32_t i = 0; i < n_constraints && c.ok; ++i)
    for (int f = 0; f < 3; ++f) {
      const uint32_t nc = c.u32();
      if (nc > c.left / 36) return STARK_ERR_BAD_ARG;
      std::vector<Coefficient> v(nc);
      for (uint32_t k = 0; k < nc; ++k) {
        v[k].wire_id = c.u32();
        v[k].value = c.raw(32);
        if (v[k].wire_id >= n_wires) return STARK_ERR_BAD_ARG;
      }
      factors.push_back(std::move(v));
    }
  if (!c.ok || n_wires == 0) return STARK_ERR_BAD_ARG;

  // ---- read_witness (r1cs-stark/src/reader.rs:7-42)
  Cursor w{wtns, wtns_len};
  if (w.u32() != 1936618615u) return STARK_ERR_BAD_ARG;  // "wtns"
  for (int i = 0; i < 5; ++i) w.u32();
  const uint32_t field_size = w.u32();
  if (field_size == 0 || field_size > 32 || field_size % 4) return STARK_ERR_BAD_ARG;
  w.raw(field_size);
  const uint32_t n_wit = w.u32();
  w.u32();
  w.u32();
  w.u32();
  if (!w.ok || (uint64_t)n_wit * field_size > w.left) return STARK_ERR_BAD_ARG;
  std::vector<HostFp> witness(n_wit);  // Montgomery; from_bytes_le reduces mod p (run.rs:354-357)
  for (uint32_t i = 0; i < n_wit; ++i) witness[i] = F.from_bytes_le(w.raw(field_size), field_size);
  if (n_wit < n_wires || !FieldHost::eq(witness[0], F.one())) return STARK_ERR_BAD_ARG;  // run.rs:358

  auto t = std::make_unique<stark_r1cs_trace>();
  t->n_constraints = n_constraints;
  t->n_wires = n_wires;
  const size_t n_public = 1 + (size_t)n_pub_in + n_pub_out;  // run.rs:359-360
  if (n_public > n_wit) return STARK_ERR_BAD_ARG;
  for (size_t i = 0; i < n_public; ++i) push_canon(t->public_wires, witness[i]);  // run.rs:359-360

  // ---- calc_coefficients_and_witness (run.rs:109-281)
  // Canonical arithmetic: montmul(c_canonical, w_montgomery) = c * w canonical,
  // so each slot costs one modular product and no conversions.
  std::vector<HostFp> wcan(n_wit);
  for (uint32_t i = 0; i < n_wit; ++i) {
    uint64_t cc[4];
    F.to_canonical(witness[i], cc);
    memcpy(wcan[i].v, cc, 32);
  }
  std::vector<HostFp> wit_l[3], tr_l[3], co_l[3];
  std::vector<std::vector<std::pair<uint8_t, size_t>>> wire_using(n_wires);
  std::vector<size_t> last_coeff;
  size_t acc_n = 0;
  for (uint32_t ci = 0; ci < n_constraints; ++ci) {
    const std::vector<Coefficient>* fac = &factors[(size_t)3 * ci];
    size_t n_coeff = fac[0].size();
    if (fac[1].size() > n_coeff) n_coeff = fac[1].size();
    if (fac[2].size() > n_coeff) n_coeff = fac[2].size();
    for (int f = 0; f < 3; ++f) {
      HostFp tacc = F.zero();
      for (size_t i = 0; i < n_coeff; ++i) {
        size_t wire;
        HostFp coef = F.zero();
        if (i < fac[f].size()) {
          wire = fac[f][i].wire_id;
          coef = F.reduce_bytes_le(fac[f][i].value, 32);  // canonical from_bytes_le
          tacc = F.add(tacc, F.mul(coef, witness[wire]));
        } else {
          wire = n_wires - 1;  // padding slot uses the last wire with coefficient 0
        }
        wire_using[wire].push_back({(uint8_t)f, co_l[f].size()});
        wit_l[f].push_back(wcan[wire]);
        co_l[f].push_back(coef);
        tr_l[f].push_back(tacc);
      }
    }
    acc_n += n_coeff;
    last_coeff.push_back(acc_n - 1);
  }
  const size_t a_len = co_l[0].size();
  const size_t os = 3 * a_len;
  if (a_len == 0) return STARK_ERR_BAD_ARG;
  t->witness_trace.reserve(4 * os);
  t->computational_trace.reserve(4 * os);
  t->coefficients.reserve(4 * os);
  for (int f = 0; f < 3; ++f)
    for (size_t i = 0; i < a_len; ++i) {
      t->witness_trace.insert(t->witness_trace.end(), wit_l[f][i].v, wit_l[f][i].v + 4);
      t->computational_trace.insert(t->computational_trace.end(), tr_l[f][i].v, tr_l[f][i].v + 4);
      t->coefficients.insert(t->coefficients.end(), co_l[f][i].v, co_l[f][i].v + 4);
    }
  // ---- calc_flags (run.rs:283-308)
  std::vector<uint8_t> f1(os, 1), f2(os, 0);
  for (size_t v : last_coeff) {
    const size_t k = (v + 1) % a_len;
    f1[k] = f1[k + a_len] = f1[k + 2 * a_len] = 0;
  }
  for (size_t k : last_coeff) f2[k] = 1;
  t->flag0.assign(4 * os, 0);
  t->flag1.assign(4 * os, 0);
  t->flag2.assign(4 * os, 0);
  for (size_t i = 0; i < os; ++i) {
    t->flag0[4 * i] = 1;
    t->flag1[4 * i] = f1[i];
    t->flag2[4 * i] = f2[i];
  }
  // ---- permuted indices (run.rs:388-401): a cycle through every wire's uses.
  t->permuted_indices.assign(os, 0);
  for (const auto& vs : wire_using) {
    if (vs.empty()) continue;
    size_t old_w = a_len * vs.back().first + vs.back().second;
    for (const auto& kv : vs) {
      const size_t wpos = a_len * kv.first + kv.second;
      t->permuted_indices[wpos] = old_w;
      old_w = wpos;
    }
  }
  // ---- public_first_indices (run.rs:411-419)
  for (size_t wi = 0; wi < n_public && wi < n_wires; ++wi)
    if (!wire_using[wi].empty()) {
      t->public_first_indices.push_back(wi);
      t->public_first_indices.push_back(a_len * wire_using[wi][0].first + wire_using[wi][0].second);
    }
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
  cp(flag0, t->flag0.data(), t->flag0.size() * 8);
  cp(flag1, t->flag1.data(), t->flag1.size() * 8);
  cp(flag2, t->flag2.data(), t->flag2.size() * 8);
  cp(permuted_indices, t->permuted_indices.data(), t->permuted_indices.size() * sizeof(size_t));
  cp(public_wires, t->public_wires.data(), t->public_wires.size() * 8);
  cp(public_first_indices, t->public_first_indices.data(), t->public_first_indices.size() * sizeof(size_t));
  return STARK_OK;
}

void stark_r1cs_trace_free(stark_r1cs_trace* t) { delete t; }

stark_status stark_prove_r1cs_trace(stark_ctx* ctx, const stark_r1cs_trace* t, stark_r1cs_proof** out) {
  if (!t) return STARK_ERR_BAD_ARG;
  return stark_mk_r1cs_proof(ctx, t->witness_trace.data(), t->computational_trace.data(), t->coefficients.size() / 4,
                             t->public_wires.data(), t->public_wires.size() / 4, t->public_first_indices.data(),
                             t->public_first_indices.size() / 2, t->permuted_indices.data(), t->coefficients.data(),
                             t->flag0.data(), t->flag1.data(), t->flag2.data(), t->n_constraints, t->n_wires, out);
}

}  // extern "C"
