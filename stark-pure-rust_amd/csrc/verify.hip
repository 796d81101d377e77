// Verifier: verify_low_degree_proof (packages/fri/src/fri.rs:226-404) and
// verify_with_witness + verify_r1cs_proof (packages/r1cs-stark/src/run.rs:454-526,
// verify.rs:13-258).
//
// The verifier's data-parallel part is the same as the prover's: the
// extensions of K, F0-F2, IDX and PIDX over the precision domain (read at the
// 80 spot-check positions).  It is taken from a prepared circuit
// (circuit_build: slot layout, flags, permutation and those LDEs on the GPU);
// the rest -- Merkle paths, the FRI layer checks and the 80 spot checks -- is
// a few thousand hashes and products on the host (a one-launch GPU path check
// measured slower than the host pass), and the cold entry
// points read the proof on a side thread while the circuit is built.
//
// Status: STARK_OK for a valid proof, STARK_ERR_CHECK where the reference
// would fail an assert (an invalid proof), STARK_ERR_BAD_ARG for malformed
// input (including the reference's Err results).
#include <string.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <string>
#include <vector>

#include "internal.h"
#include "host_json.h"
#include "blake2s.h"
#include "host_b2s.h"

namespace stark {
namespace {

// ---- the proof, as serde_json writes it (utils.rs:122-130, merkle_tree.rs:14-18, fri.rs:16-26) ----

// Bytes held elsewhere: the proof text's arena (ProofIn::arena) or the caller's arrays.  A parsed proof
// makes no allocation per opening (freeing ~3,600 small vectors written by 16 threads took ~0.27 ms of a
// 1.35 ms pedersen verify, profiles/r05_verify_phases.txt).
struct Bytes {
  const uint8_t* p = nullptr;
  size_t n = 0;
  const uint8_t* data() const { return p; }
  size_t size() const { return n; }
  const uint8_t* begin() const { return p; }
  const uint8_t* end() const { return p + n; }
};

struct Branch {  // commitment::merkle_tree::Proof
  Bytes leaf;
  Bytes nodes;  // 32 B each, leaf -> root
};

struct FriIn {  // FriProof::Middle { root2, column_branches, poly_branches } | Last { last }
  bool last = false;
  uint8_t root2[32] = {0};
  std::vector<Branch> col, poly;
  std::vector<std::vector<uint8_t>> last_vals;
};

struct ProofIn {
  uint8_t m_root[32], l_root[32], a_root[32];
  std::vector<Branch> main, lcomb;
  std::vector<FriIn> fri;
  // The openings' bytes: the opening whose text starts at offset t is written from arena + t / 2 (a
  // number takes two characters at least, so an opening's bytes end before its text's end / 2 and
  // openings side by side never overlap; pre_parse_branches bounds each parallel parse by the next
  // candidate's start, so a candidate nested inside another opening cannot write into it).
  std::unique_ptr<uint8_t[]> arena;
};

class Json;

// Merkle openings parsed ahead of the sequential reader, in parallel: every `{"leaf":` of the text
// starts a candidate Branch object (in serde_json's own output the key occurs nowhere else), and
// serde_json writes no whitespace.  Candidate i writes its bytes only inside [off_i / 2, off_{i+1} / 2) of
// the arena, which a Branch that contains no other candidate always fits; one that does not fit (it has
// an object with a `{"leaf":` key nested in it, which serde accepts as an unknown member) is left to
// the reader.  The reader takes a pre-parsed Branch only when it reaches that exact offset itself and the
// parse succeeded, and parses every other Branch itself after the parallel phase, so the result is the
// sequential parse and no two threads write the same bytes.
struct PreBranches {
  std::vector<size_t> off, end;
  std::vector<Branch> br;
  std::vector<uint8_t> good;
  size_t next = 0;
};

// A reader for exactly this schema: objects with string keys, arrays, u8 numbers.
class Json {
  static constexpr int kBranchDepth = 6;  // a Proof object's nesting in a StarkProof (at most; FRI branches)

 public:
  Json(const char* s, size_t n, PreBranches* pre = nullptr, uint8_t* arena = nullptr, uint8_t* lim = nullptr)
      : p_(s), e_(s + n), base_(s), pre_(pre), arena_(arena), lim_(lim) {}
  Json(const char* base, size_t n, size_t at, uint8_t* arena, uint8_t* lim)
      : p_(base + at), e_(base + n), base_(base), arena_(arena), lim_(lim) {}
  bool ok = true;
  size_t pos() const { return (size_t)(p_ - base_); }

  bool accept(char c) {
    ws();
    if (p_ < e_ && *p_ == c) {
      ++p_;
      return true;
    }
    return false;
  }
  void expect(char c) {
    if (!accept(c)) ok = false;
  }
  // A member name, unescaped (serde_json matches field names after decoding "\u0061" and the like).
  std::string key() {
    std::string k;
    ws();
    if (!str(&k)) ok = false;
    expect(':');
    return k;
  }
  // A JSON string at p_ (serde_json's rules: escapes \" \\ \/ \b \f \n \r \t \uXXXX with surrogate pairs,
  // no raw control characters, valid UTF-8), decoded into out when given.
  bool str(std::string* out) {
    if (p_ >= e_ || *p_ != '"') return false;
    ++p_;
    for (;;) {
      if (p_ >= e_) return false;
      const unsigned char c = (unsigned char)*p_++;
      if (c == '"') return true;
      if (c < 0x20) return false;
      if (c == '\\') {
        if (p_ >= e_) return false;
        const char x = *p_++;
        uint32_t cp;
        switch (x) {
          case '"': cp = '"'; break;
          case '\\': cp = '\\'; break;
          case '/': cp = '/'; break;
          case 'b': cp = 8; break;
          case 'f': cp = 12; break;
          case 'n': cp = 10; break;
          case 'r': cp = 13; break;
          case 't': cp = 9; break;
          case 'u': {
            if (!hex4(&cp)) return false;
            if (cp >= 0xDC00 && cp <= 0xDFFF) return false;  // a lone trailing surrogate
            if (cp >= 0xD800 && cp <= 0xDBFF) {                // a leading one: its pair must follow
              uint32_t lo;
              if (e_ - p_ < 2 || p_[0] != '\\' || p_[1] != 'u') return false;
              p_ += 2;
              if (!hex4(&lo) || lo < 0xDC00 || lo > 0xDFFF) return false;
              cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
            }
            break;
          }
          default:
            return false;
        }
        if (out) utf8(cp, *out);
        continue;
      }
      if (c < 0x80) {
        if (out) out->push_back((char)c);
        continue;
      }
      // a multi-byte UTF-8 sequence: lead byte, continuation bytes, no overlong / surrogate / > U+10FFFF forms
      const int n = c >= 0xF0 ? 3 : c >= 0xE0 ? 2 : c >= 0xC2 ? 1 : -1;
      if (n < 0 || c > 0xF4 || e_ - p_ < n) return false;
      uint32_t cp = c & (0x3F >> n);
      for (int i = 0; i < n; ++i) {
        const unsigned char d = (unsigned char)p_[i];
        if ((d & 0xC0) != 0x80) return false;
        cp = (cp << 6) | (d & 0x3F);
      }
      if ((n == 2 && (cp < 0x800 || (cp >= 0xD800 && cp <= 0xDFFF))) || (n == 3 && (cp < 0x10000 || cp > 0x10FFFF)))
        return false;
      if (out) out->append(p_ - 1, (size_t)n + 1);
      p_ += n;
    }
  }
  // Any JSON value, skipped: serde_json ignores the members of a struct that it does not know (no
  // deny_unknown_fields on StarkProof, Proof or FriProof's variants).  depth: containers already open.
  bool skip_value(int depth) {
    ws();
    if (p_ >= e_ || depth > 128) return false;  // (serde_json's recursion limit)
    const char c = *p_;
    if (c == '{' || c == '[') {
      const char close = c == '{' ? '}' : ']';
      ++p_;
      if (accept(close)) return true;
      do {
        if (c == '{') {
          ws();
          if (!str(nullptr) || !accept(':')) return false;
        }
        if (!skip_value(depth + 1)) return false;
      } while (accept(','));
      return accept(close);
    }
    if (c == '"') return str(nullptr);
    for (const char* lit : {"true", "false", "null"}) {
      const size_t n = strlen(lit);
      if ((size_t)(e_ - p_) >= n && memcmp(p_, lit, n) == 0) {
        p_ += n;
        return true;
      }
    }
    // a number: -?(0|[1-9][0-9]*)(.[0-9]+)?([eE][+-]?[0-9]+)?
    auto digit = [&] { return p_ < e_ && (unsigned)(*p_ - '0') < 10u; };
    if (p_ < e_ && *p_ == '-') ++p_;
    if (!digit()) return false;
    if (*p_ == '0') ++p_;
    else
      while (digit()) ++p_;
    if (p_ < e_ && *p_ == '.') {
      ++p_;
      if (!digit()) return false;
      while (digit()) ++p_;
    }
    if (p_ < e_ && (*p_ == 'e' || *p_ == 'E')) {
      ++p_;
      if (p_ < e_ && (*p_ == '+' || *p_ == '-')) ++p_;
      if (!digit()) return false;
      while (digit()) ++p_;
    }
    return true;
  }
  // A u8 array, each value handed to put (false: stop, malformed).  Tight loop: serde_json writes no
  // whitespace, so the separator is checked before falling back to the general whitespace skip.  A number
  // is read from its first four bytes without branching on its length (1-3 digits); like serde_json the
  // reader refuses a leading zero ("05"), four or more digits and values above 255.
  template <class Put>
  void u8_array(Put put) {
    expect('[');
    if (!ok || accept(']')) return;
    ws();
    for (;;) {
      unsigned v = 0;
      bool bad;
      if (e_ - p_ >= 4) {
        const unsigned b0 = (unsigned)(unsigned char)p_[0] - '0', b1 = (unsigned)(unsigned char)p_[1] - '0',
                       b2 = (unsigned)(unsigned char)p_[2] - '0', b3 = (unsigned)(unsigned char)p_[3] - '0';
        const unsigned d1 = b1 < 10u, d2 = d1 & (b2 < 10u), d3 = d2 & (b3 < 10u);
        bad = b0 >= 10u || d3 || (b0 == 0 && d1);
        v = b0;
        v = d1 ? 10 * v + b1 : v;
        v = d2 ? 10 * v + b2 : v;
        p_ += 1 + d1 + d2;
      } else {
        int nd = 0;
        unsigned first = 0;
        while (p_ < e_ && (unsigned)(*p_ - '0') < 10u && nd < 4) {
          if (nd == 0) first = (unsigned)(*p_ - '0');
          v = 10 * v + (unsigned)(*p_++ - '0');
          ++nd;
        }
        bad = nd == 0 || nd > 3 || (first == 0 && nd > 1);
      }
      if (bad || v > 255 || !put((uint8_t)v)) {
        ok = false;
        return;
      }
      if (p_ < e_ && *p_ == ',') {
        ++p_;
        if (p_ < e_ && (unsigned)(*p_ - '0') >= 10u) ws();
        continue;
      }
      if (p_ < e_ && *p_ == ']') {
        ++p_;
        return;
      }
      ws();
      if (p_ < e_ && *p_ == ',') {
        ++p_;
        ws();
        continue;
      }
      expect(']');
      return;
    }
  }
  void bytes(std::vector<uint8_t>& out) {
    out.clear();
    u8_array([&](uint8_t v) {
      out.push_back(v);
      return true;
    });
  }
  // Into out[0..max): the count (a longer array is malformed).
  size_t bytes_to(uint8_t* out, size_t max) {
    if (p_ < e_ && *p_ == '[' && json_simd_width() == 64) {
      // the compact form in AVX-512 registers; any other text is re-read by the scalar loop below
      size_t n = 0;
      if (const char* r = json_u8s_v512(p_ + 1, e_, out, max, &n)) {
        p_ = r;
        return n;
      }
    }
    size_t k = 0;
    u8_array([&](uint8_t v) {
      if (k == max) return false;
      out[k++] = v;
      return true;
    });
    return k;
  }
  void digest(uint8_t out[32]) {
    if (bytes_to(out, 32) != 32) ok = false;
  }
  void branch(Branch& b) {
    if (!arena_) {
      ok = false;
      return;
    }
    uint8_t* w = arena_ + pos() / 2;  // this opening's part of the arena (ProofIn::arena), up to lim_
    if (w > lim_) {
      ok = false;
      return;
    }
    expect('{');
    bool has_leaf = false, has_nodes = false;
    do {
      const std::string k = key();
      if ((k == "leaf" && has_leaf) || (k == "nodes" && has_nodes)) {
        ok = false;  // serde_json: duplicate field
      } else if (k == "leaf") {
        const size_t n = bytes_to(w, std::min((size_t)(e_ - p_) / 2 + 1, (size_t)(lim_ - w)));
        b.leaf = Bytes{w, n};
        w += n;
        has_leaf = true;
      } else if (k == "nodes") {
        uint8_t* const n0 = w;
        expect('[');
        if (!accept(']')) {
          do {
            if (lim_ - w < 32) {
              ok = false;
              break;
            }
            digest(w);
            w += 32;
          } while (ok && accept(','));
          expect(']');
        }
        b.nodes = Bytes{n0, (size_t)(w - n0)};
        has_nodes = true;
      } else if (ok && !skip_value(kBranchDepth)) {
        ok = false;
      }
    } while (ok && accept(','));
    expect('}');
    if (!has_leaf || !has_nodes) ok = false;
  }
  void branches(std::vector<Branch>& v) {
    expect('[');
    if (!ok || accept(']')) return;
    do {
      v.emplace_back();
      if (!take_pre(v.back())) branch(v.back());
    } while (ok && accept(','));
    expect(']');
  }
  void fri_layer(FriIn& f) {
    expect('{');
    const std::string tag = key();
    expect('{');
    if (tag == "Middle") {
      bool r = false, c = false, q = false;
      do {
        const std::string k = key();
        if ((k == "root2" && r) || (k == "column_branches" && c) || (k == "poly_branches" && q)) {
          ok = false;  // duplicate field
        } else if (k == "root2") {
          digest(f.root2);
          r = true;
        } else if (k == "column_branches") {
          branches(f.col);
          c = true;
        } else if (k == "poly_branches") {
          branches(f.poly);
          q = true;
        } else if (ok && !skip_value(4)) {
          ok = false;
        }
      } while (ok && accept(','));
      if (!(r && c && q)) ok = false;
    } else if (tag == "Last") {
      f.last = true;
      bool l = false;
      do {
        const std::string k = key();
        if (k == "last" && l) {
          ok = false;  // duplicate field
        } else if (k == "last") {
          l = true;
          expect('[');
          if (ok && !accept(']')) {
            do {
              f.last_vals.emplace_back();
              bytes(f.last_vals.back());
            } while (ok && accept(','));
            expect(']');
          }
        } else if (ok && !skip_value(4)) {
          ok = false;
        }
      } while (ok && accept(','));
      if (!l) ok = false;
    } else {
      ok = false;
    }
    expect('}');
    expect('}');
  }
  void stark_proof(ProofIn& pr) {
    expect('{');
    int seen = 0;
    do {
      const std::string k = key();
      if (k == "m_root" && !(seen & 1)) digest(pr.m_root), seen |= 1;
      else if (k == "l_root" && !(seen & 2)) digest(pr.l_root), seen |= 2;
      else if (k == "a_root" && !(seen & 4)) digest(pr.a_root), seen |= 4;
      else if (k == "main_branches" && !(seen & 8)) branches(pr.main), seen |= 8;
      else if (k == "linear_comb_branches" && !(seen & 16)) branches(pr.lcomb), seen |= 16;
      else if (k == "fri_proof" && !(seen & 32)) {
        expect('[');
        if (!accept(']')) {
          do {
            pr.fri.emplace_back();
            fri_layer(pr.fri.back());
          } while (ok && accept(','));
          expect(']');
        }
        seen |= 32;
      } else if (k == "m_root" || k == "l_root" || k == "a_root" || k == "main_branches" ||
                 k == "linear_comb_branches" || k == "fri_proof" || !skip_value(1)) {
        ok = false;  // a duplicate field (the first five arms above take only a first occurrence), or no value
      }
    } while (ok && accept(','));
    expect('}');
    ws();
    if (seen != 63 || p_ != e_) ok = false;
  }

 private:
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
  }
  bool hex4(uint32_t* v) {
    if (e_ - p_ < 4) return false;
    uint32_t x = 0;
    for (int i = 0; i < 4; ++i) {
      const char c = *p_++;
      const int d = c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c >= 'A' && c <= 'F' ? c - 'A' + 10 : -1;
      if (d < 0) return false;
      x = 16 * x + (uint32_t)d;
    }
    *v = x;
    return true;
  }
  static void utf8(uint32_t cp, std::string& o) {
    if (cp < 0x80) {
      o.push_back((char)cp);
    } else if (cp < 0x800) {
      o.push_back((char)(0xC0 | (cp >> 6)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      o.push_back((char)(0xE0 | (cp >> 12)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      o.push_back((char)(0xF0 | (cp >> 18)));
      o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  // The pre-parsed Branch starting exactly here, if any (offsets ascend with the reader).
  bool take_pre(Branch& b) {
    if (!pre_) return false;
    ws();
    const size_t at = pos();
    PreBranches& P = *pre_;
    while (P.next < P.off.size() && P.off[P.next] < at) ++P.next;
    if (P.next == P.off.size() || P.off[P.next] != at) return false;
    const size_t i = P.next++;
    if (!P.good[i]) return false;  // (parsed here instead: the sequential parse decides)
    b = std::move(P.br[i]);
    p_ = base_ + P.end[i];
    return true;
  }
  const char* p_;
  const char* e_;
  const char* base_;
  PreBranches* pre_ = nullptr;
  uint8_t* arena_ = nullptr;
  uint8_t* lim_ = nullptr;  // arena_'s write bound for this parse
};

// Finds every Branch start and parses each from its offset on the host workers.
void pre_parse_branches(const char* s, size_t n, PreBranches& P, uint8_t* arena, uint8_t* arena_end) {
  static const char kKey[] = "{\"leaf\":";
  const size_t klen = sizeof(kKey) - 1;
  const unsigned parts = n < ((size_t)1 << 18) ? 1u : host_threads();
  std::vector<std::vector<size_t>> found(parts);
  host_parallel(parts, [&](unsigned t) {
    const size_t lo = n * t / parts, hi = n * (t + 1) / parts;  // starts in [lo, hi)
    const char* p = s + lo;
    // every '{' by memchr (vectorised; in serde's text '{' opens objects only, most of them branches),
    // then the key compared in place
    const char* const stop = s + std::min(n, hi);  // (a match starting before hi may end past it)
    while (p < stop) {
      const char* q = (const char*)memchr(p, '{', (size_t)(stop - p));
      if (!q) break;
      if ((size_t)(s + n - q) >= klen && memcmp(q, kKey, klen) == 0) found[t].push_back((size_t)(q - s));
      p = q + 1;
    }
  });
  for (auto& f : found) P.off.insert(P.off.end(), f.begin(), f.end());
  const size_t k = P.off.size();
  P.end.assign(k, 0);
  P.good.assign(k, 0);
  P.br.assign(k, Branch());
  std::atomic<size_t> next{0};
  host_parallel(std::min<unsigned>(host_threads(), (unsigned)((k + 15) / 16)), [&](unsigned) {
    for (size_t c; (c = next.fetch_add(16)) < k;)
      for (size_t i = c; i < std::min(k, c + 16); ++i) {
        Json j(s, n, P.off[i], arena, i + 1 < k ? arena + P.off[i + 1] / 2 : arena_end);
        j.branch(P.br[i]);
        P.good[i] = j.ok;
        P.end[i] = j.pos();
      }
  });
}

// ---- field helpers ----

// T::from_bytes_le (ff_utils/src/fp.rs:70-77): the little-endian integer of the bytes mod p.
HostFp fe_from_bytes(const uint8_t* b, size_t n) {
  const FieldHost& F = FieldHost::get();
  if (n <= 32) return F.from_bytes_le(b, n);
  HostFp acc = F.zero();
  const HostFp base = F.from_u64(256);
  for (size_t i = n; i-- > 0;) acc = F.add(F.mul(acc, base), F.from_u64(b[i]));
  return acc;
}
HostFp fe_from_bytes(const std::vector<uint8_t>& b) { return fe_from_bytes(b.data(), b.size()); }
HostFp fe_from_bytes(const Bytes& b) { return fe_from_bytes(b.data(), b.size()); }

HostFp eval_poly(const std::vector<HostFp>& poly, const HostFp& x) {  // eval_poly_at, poly_utils.rs:93-102
  const FieldHost& F = FieldHost::get();
  HostFp acc = F.zero();
  for (size_t k = poly.size(); k-- > 0;) acc = F.add(F.mul(acc, x), poly[k]);
  return acc;
}

// Proof::validate (merkle_tree.rs:25-43) for many (root, index, opening) triples of different trees
// in one pass over the host workers, split by node count (verify_multi_branch, :46-58, zips indices
// and openings: the callers check that every index has one).
struct PathCheck {
  const uint8_t* root;
  size_t index;
  const Branch* b;
};
// ok[i] = check i's path leads to its root: b2s_paths (host_b2s.h), a SIMD register of paths of one
// shape per compression (the checks come in runs of equal leaf length and depth), split by compression
// count over the host workers.
void paths_check(const std::vector<PathCheck>& v, std::vector<uint8_t>& ok) {
  ok.assign(v.size(), 0);
  std::vector<PathJob> jobs(v.size());
  std::vector<size_t> cost(v.size() + 1, 0);
  for (size_t i = 0; i < v.size(); ++i) {
    const Branch& b = *v[i].b;
    jobs[i] = PathJob{v[i].root, (uint64_t)v[i].index, b.leaf.data(), b.nodes.data(), (uint32_t)b.leaf.size(),
                      (uint32_t)(b.nodes.size() / 32)};
    cost[i + 1] = cost[i] + (b.leaf.size() + 63) / 64 + jobs[i].depth + 1;
  }
  const size_t per_part = 48 * (size_t)b2s_paths_width();  // compressions per part at least
  const unsigned parts =
      std::max(1u, (unsigned)std::min<size_t>(host_threads(), cost.back() / per_part));
  host_parallel(parts, [&](unsigned t) {
    const size_t lo = std::lower_bound(cost.begin(), cost.end(), cost.back() * t / parts) - cost.begin();
    const size_t hi = std::lower_bound(cost.begin(), cost.end(), cost.back() * (t + 1) / parts) - cost.begin();
    if (lo < hi && lo < v.size()) b2s_paths(jobs.data() + lo, std::min(hi, v.size()) - lo, ok.data() + lo);
  });
}
bool sampler(const uint8_t seed[32], size_t modulus, uint32_t count, uint32_t excl, std::vector<size_t>& out) {
  if (modulus > 0xFFFFFFFFull) return false;
  std::vector<uint32_t> v(count);
  if (stark_get_pseudorandom_indices(seed, 32, (uint32_t)modulus, count, excl, v.data()) != STARK_OK) return false;
  out.assign(v.begin(), v.end());
  return true;
}

// verify_low_degree_proof_rec (fri.rs:244-404).
// `extra` (optional): more path checks to run in the same parallel pass as the layers' (the verifier's
// main and L openings); *extra_ok tells whether they all hold, whatever this function returns.
stark_status verify_fri(const uint8_t merkle_root_in[32], HostFp root, const std::vector<FriIn>& proof,
                        size_t max_deg_plus_1, uint32_t excl, const std::vector<PathCheck>* extra = nullptr,
                        bool* extra_ok = nullptr) {
  const FieldHost& F = FieldHost::get();
  if (proof.empty()) return STARK_ERR_BAD_ARG;
  uint64_t rou_deg = 1;
  for (HostFp t = root; !FieldHost::eq(t, F.one()); t = F.mul(t, t)) {
    rou_deg *= 2;
    if (rou_deg > ((uint64_t)1 << 28)) return STARK_ERR_BAD_ARG;  // not a root of unity of 2-power order
  }
  if (rou_deg < 4 && proof.size() > 1) return STARK_ERR_BAD_ARG;
  uint8_t m_root[32];
  memcpy(m_root, merkle_root_in, 32);
  HostFp quartic[4] = {F.one(), F.one(), F.one(), F.one()};
  if (rou_deg >= 4)
    for (int j = 1; j < 4; ++j) quartic[j] = F.pow_u64(root, rou_deg / 4 * (uint64_t)j);
  const HostFp inv4 = F.inv(F.from_u64(4));
  // Every layer's indices follow from the proof's own roots, so all the layers' Merkle paths are
  // checked first, in one parallel pass (the reference checks them layer by layer, fri.rs:288-316;
  // the accept/reject outcome is the same).  A layer whose shape the reference would reject before
  // its paths keeps that order: the pass stops at it.
  std::vector<std::vector<size_t>> ys_l, pos_l;
  {
    std::vector<PathCheck> checks;
    const uint8_t* root_l = merkle_root_in;
    uint64_t deg = rou_deg;
    for (size_t l = 0; l + 1 < proof.size(); ++l) {
      const FriIn& L = proof[l];
      if (L.last || deg < 4) break;  // reported in order below
      std::vector<size_t> ys, poly_pos;
      if (!sampler(L.root2, deg / 4, 40, excl, ys)) break;
      for (size_t y : ys)
        for (size_t j = 0; j < 4; ++j) poly_pos.push_back(j * (deg / 4) + y);
      if (L.col.size() < ys.size() || L.poly.size() < poly_pos.size()) return STARK_ERR_CHECK;  // zip (:46-58)
      ys_l.push_back(std::move(ys));
      pos_l.push_back(std::move(poly_pos));
      deg /= 4;
      root_l = L.root2;
    }
    root_l = merkle_root_in;
    for (size_t l = 0; l < ys_l.size(); ++l) {
      const FriIn& L = proof[l];
      for (size_t i = 0; i < ys_l[l].size(); ++i) checks.push_back({L.root2, ys_l[l][i], &L.col[i]});
      for (size_t i = 0; i < pos_l[l].size(); ++i) checks.push_back({root_l, pos_l[l][i], &L.poly[i]});
      root_l = L.root2;
    }
    const size_t n_fri = checks.size();
    if (extra) checks.insert(checks.end(), extra->begin(), extra->end());
    std::vector<uint8_t> ok;
    paths_check(checks, ok);
    if (extra_ok) *extra_ok = std::find(ok.begin() + n_fri, ok.end(), 0) == ok.end();
    if (std::find(ok.begin(), ok.begin() + n_fri, 0) != ok.begin() + n_fri) return STARK_ERR_CHECK;
  }
  // Every row of every layer is independent once the roots are known: the cubic checks run on the host
  // workers, and the layer loop below reports the first failure in the reference's order
  // (fri.rs:318-345).  x1 = root_l^y has order dividing rou_deg_l, so 1 / x1^3 = root_l^(-3y mod rou_deg_l)
  // needs no inversion.
  std::vector<uint8_t> row_ok(ys_l.size(), 1);
  {
    struct Row {
      size_t l, i;
    };
    std::vector<Row> rows;
    std::vector<HostFp> root_at(ys_l.size()), sx_at(ys_l.size());
    std::vector<uint64_t> deg_at(ys_l.size());
    HostFp rt = root;
    uint64_t dg = rou_deg;
    const uint8_t* mr = merkle_root_in;
    for (size_t l = 0; l < ys_l.size(); ++l) {
      root_at[l] = rt;
      deg_at[l] = dg;
      sx_at[l] = F.from_bytes_le(mr, 32);
      for (size_t i = 0; i < ys_l[l].size(); ++i) rows.push_back({l, i});
      mr = proof[l].root2;
      rt = F.pow_u64(rt, 4);
      dg /= 4;
    }
    std::vector<uint8_t> good(rows.size(), 0);
    std::atomic<size_t> next{0};
    host_parallel(std::max(1u, std::min<unsigned>(host_threads(), (unsigned)((rows.size() + 7) / 8))), [&](unsigned) {
      for (size_t k; (k = next.fetch_add(4)) < rows.size();)
        for (size_t q = k; q < std::min(rows.size(), k + 4); ++q) {
          const size_t l = rows[q].l, i = rows[q].i;
          const FriIn& L = proof[l];
          const uint64_t y = ys_l[l][i], dl = deg_at[l];
          // The cubic through (x1 zeta^j, row_j) at special_x (multi_interp_4 + eval_quartic,
          // poly_utils.rs:442-511): Lagrange weights prod_{k != j}(sx - x_k) / (4 x1^3 zeta^(3j)).
          const HostFp x1 = F.pow_u64(root_at[l], y);
          const HostFp inv_x13 = F.pow_u64(root_at[l], (dl - (3 * y) % dl) % dl);
          const HostFp& sx = sx_at[l];
          HostFp xs[4], num[4];
          for (int j = 0; j < 4; ++j) xs[j] = F.mul(quartic[j], x1);
          for (int j = 0; j < 4; ++j) {
            num[j] = F.one();
            for (int t = 0; t < 4; ++t)
              if (t != j) num[j] = F.mul(num[j], F.sub(sx, xs[t]));
          }
          const HostFp inv_den = F.mul(inv4, inv_x13);  // 1 / (4 x1^3); zeta^(-3j) = zeta^j
          HostFp val = F.zero();
          for (int j = 0; j < 4; ++j)
            val = F.add(val, F.mul(F.mul(fe_from_bytes(L.poly[i * 4 + j].leaf), num[j]), F.mul(inv_den, quartic[j])));
          good[q] = FieldHost::eq(val, fe_from_bytes(L.col[i].leaf));  // assert_eq (fri.rs:337)
        }
    });
    for (size_t q = 0; q < rows.size(); ++q)
      if (!good[q]) row_ok[rows[q].l] = 0;
  }
  for (size_t l = 0; l + 1 < proof.size(); ++l) {
    const FriIn& L = proof[l];
    if (L.last) return STARK_ERR_BAD_ARG;  // "FRI proofs must consist of FriProof::Middle except the last element."
    if (l >= ys_l.size()) return STARK_ERR_CHECK;  // get_pseudorandom_indices panics
    if (!row_ok[l]) return STARK_ERR_CHECK;          // a row's cubic disagrees with its column value
    memcpy(m_root, L.root2, 32);
    root = F.pow_u64(root, 4);
    max_deg_plus_1 /= 4;
    rou_deg /= 4;
    if (rou_deg < 4 && l + 2 < proof.size()) return STARK_ERR_BAD_ARG;
  }
  const FriIn& last = proof.back();
  if (!last.last) return STARK_ERR_BAD_ARG;  // "The last element of FRI proofs must be FriProof::Last."
  if (max_deg_plus_1 < 16 / 2) return STARK_ERR_CHECK;           // MIN_DEG_DIRECT_CHECKING / 2 (fri.rs:348-351)
  const size_t n = last.last_vals.size();
  if (n <= max_deg_plus_1) return STARK_ERR_CHECK;               // fri.rs:359
  if (n & (n - 1)) return STARK_ERR_CHECK;                       // MerkleProofInPlace::update (merkle_proof_in_place.rs:113)
  {
    // m_tree over the raw last values (fri.rs:367-372).
    std::vector<std::vector<uint8_t>> lv;
    std::vector<uint8_t> cur(32 * n);
    for (size_t i = 0; i < n; ++i) b2s_host(last.last_vals[i].data(), last.last_vals[i].size(), &cur[32 * i]);
    for (size_t w = n; w > 1; w /= 2) {
      std::vector<uint8_t> up(32 * (w / 2));
      for (size_t i = 0; i < w / 2; ++i) b2s_host(&cur[64 * i], 64, &up[32 * i]);
      cur.swap(up);
    }
    if (memcmp(cur.data(), m_root, 32) != 0) return STARK_ERR_CHECK;
  }
  // Degree of the last values (fri.rs:377-401): xs = expand_root_of_unity(root).
  std::vector<HostFp> xs(1, F.one());
  for (HostFp t = root; !FieldHost::eq(t, F.one()); t = F.mul(t, root)) xs.push_back(t);
  std::vector<size_t> pts;
  for (size_t pos = 0; pos < n; ++pos)
    if (excl == 0 || pos % excl != 0) pts.push_back(pos);
  if (pts.size() < max_deg_plus_1) return STARK_ERR_CHECK;  // split_off panics
  for (size_t pos : pts)
    if (pos >= xs.size()) return STARK_ERR_CHECK;  // xs[pos] out of bounds
  std::vector<HostFp> xv, yv;
  for (size_t i = 0; i < max_deg_plus_1; ++i) {
    xv.push_back(xs[pts[i]]);
    yv.push_back(fe_from_bytes(last.last_vals[pts[i]]));
  }
  const std::vector<HostFp> poly = lagrange_interp(xv, yv);
  for (size_t i = max_deg_plus_1; i < pts.size(); ++i)
    if (!FieldHost::eq(eval_poly(poly, xs[pts[i]]), fe_from_bytes(last.last_vals[pts[i]]))) return STARK_ERR_CHECK;
  return STARK_OK;
}

uint32_t log2_ceil_ref(size_t v) {  // log2_ceil (r1cs-stark/src/utils.rs:14-23)
  uint32_t l = 1;
  for (size_t t = v; t > 1; t /= 2) ++l;
  return l;
}

}  // namespace

// verify_r1cs_proof (verify.rs:13-258) for a prepared circuit; `pub_bytes` holds the public
// wires as 32-byte little-endian integers (from_bytes_le, run.rs:477-480).
static stark_status verify_r1cs(stark_ctx* ctx, const PreparedCircuit& c, const uint8_t* pub_bytes, size_t n_public,
                                const ProofIn& pr) {
  const FieldHost& F = FieldHost::get();
  PhaseClock clk("verify_r1cs_proof");
  if (c.world != 1) return STARK_ERR_BAD_ARG;
  // The reference builds its boundary points from every supplied wire (run.rs:503-509); a prepared
  // circuit holds the first uses of the header's 1 + n_pub_in + n_pub_out wires only, so any other
  // count is refused rather than silently truncated.
  if (n_public != c.n_public) return STARK_ERR_BAD_ARG;
  std::vector<HostFp> pub(c.n_public);
  for (size_t i = 0; i < c.n_public; ++i) pub[i] = F.from_bytes_le(pub_bytes + 32 * i, 32);
  if (!FieldHost::eq(pub[0], F.one())) return STARK_ERR_CHECK;  // run.rs:480
  const size_t os = c.os;
  const uint32_t log_steps = log2_ceil_ref(os - 1);
  const uint64_t steps = std::max<uint64_t>((uint64_t)1 << log_steps, 8), prec = 8 * steps, skips = 8;
  uint64_t pm1[4];  // g2 = 7^((p-1)/precision) (verify.rs:55-63)
  memcpy(pm1, FieldHost::kP, 32);
  pm1[0] -= 1;
  for (uint64_t t = prec; t > 1; t /= 2)
    for (int l = 0; l < 4; ++l) pm1[l] = (pm1[l] >> 1) | (l < 3 ? pm1[l + 1] << 63 : 0);
  const HostFp g2 = F.pow(F.from_u64(7), pm1, 4);
  // FRI on the linear combination (verify.rs:80-84), then the spot checks' openings (verify.rs:86-118).
  // Every Merkle path of both -- the FRI layers', the 320 main and 80 L openings -- is checked in one
  // parallel pass inside verify_fri; the outcomes are reported in the reference's order.
  std::vector<size_t> positions, aug;
  const bool sampled = sampler(pr.l_root, prec, 80, (uint32_t)skips, positions);
  if (sampled)
    for (size_t j : positions) {
      aug.push_back(j);
      aug.push_back((j + prec - skips) % prec);
      aug.push_back((j + os / 3 * skips) % prec);
      aug.push_back((j + os / 3 * 2 * skips) % prec);
    }
  // (zip: every index needs its opening)
  const bool sized = sampled && pr.main.size() >= aug.size() && pr.lcomb.size() >= positions.size();
  std::vector<PathCheck> checks;
  if (sized) {
    for (size_t i = 0; i < aug.size(); ++i) checks.push_back({pr.m_root, aug[i], &pr.main[i]});
    for (size_t i = 0; i < positions.size(); ++i) checks.push_back({pr.l_root, positions[i], &pr.lcomb[i]});
  }
  // K, F0-F2, IDX, PIDX at the positions: the circuit's extensions (K, F0-F2 as Montgomery images in a
  // prover's prepared circuit, canonical in the verifier's cold build; IDX and PIDX canonical), gathered
  // in one launch on the side thread while this one checks the paths and the FRI layers (the positions
  // depend on l_root alone).
  const size_t n_pos = positions.size();
  std::vector<uint8_t> got(6 * n_pos * 32);
  stark_status st_got = STARK_OK;
  bool paths_ok = false;
  stark_status st;
  {
    HostTask gather([&] {
      if (!sized) return;
      if (c.spot) {  // the cold build's first passes: the six values per position evaluated from them
        st_got = circuit_spot_values(ctx, c, positions.data(), n_pos, got.data(), ctx->stream);
        return;
      }
      stark_open_req req[6];
      for (int k = 0; k < 6; ++k)
        req[k] = stark_open_req{nullptr, (const uint8_t*)c.col[k], 32, prec, positions.data(), n_pos,
                              got.data() + (size_t)k * n_pos * 32, nullptr};
      st_got = stark_open_batch(ctx, req, 6, nullptr);
    });
    st = verify_fri(pr.l_root, g2, pr.fri, prec / 4, (uint32_t)skips, sized ? &checks : nullptr, &paths_ok);
  }
  if (st != STARK_OK) return st;
  clk.mark("FRI layers + main/L paths || gather");
  if (!sized || !paths_ok) return STARK_ERR_CHECK;
  for (size_t i = 0; i < aug.size(); ++i)
    if (pr.main[i].leaf.size() < 256) return STARK_ERR_CHECK;  // m_branch[k] chunks (verify.rs:185-200)
  if (st_got != STARK_OK) return st_got;
  auto col_val = [&](int k, size_t i) {
    HostFp v;
    memcpy(v.v, got.data() + ((size_t)k * n_pos + i) * 32, 32);
    while (FieldHost::ge_p(v.v)) FieldHost::sub_p_in_place(v.v);
    return k < 4 && c.with_zb ? v : F.from_canonical(v.v);  // a Montgomery image's bits are the HostFp itself
  };
  // Boundary interpolants (verify.rs:151-155, utils.rs:421-474) and Zb2's points.
  std::vector<HostFp> bx, by;
  for (size_t i = 0; i + 1 < c.pfi.size(); i += 2) {
    bx.push_back(F.pow_u64(g2, skips * c.pfi[i + 1]));
    by.push_back(pub[c.pfi[i]]);
  }
  const std::vector<HostFp> interp2 = lagrange_interp(bx, by);
  const HostFp x_last = F.pow_u64(g2, (steps - 1) * skips);
  const std::vector<HostFp> interp3 = lagrange_interp({x_last}, {F.one()});
  // r (utils.rs:272-290) and k (verify.rs:164-173).
  HostFp r[3];
  {
    std::vector<size_t> rnd;
    if (!sampler(pr.a_root, prec, 24, 0, rnd)) return STARK_ERR_CHECK;
    for (int k = 0; k < 3; ++k) {
      uint8_t be[32];
      for (int i = 0; i < 8; ++i) {
        const uint32_t v = (uint32_t)rnd[8 * k + i];
        be[4 * i] = (uint8_t)(v >> 24);
        be[4 * i + 1] = (uint8_t)(v >> 16);
        be[4 * i + 2] = (uint8_t)(v >> 8);
        be[4 * i + 3] = (uint8_t)v;
      }
      r[k] = F.from_bytes_le(be, 32);
    }
  }
  HostFp kk[11];
  kk[0] = F.one();
  for (int i = 1; i < 11; ++i) {
    uint8_t msg[33], h[32], le[32];
    memcpy(msg, pr.m_root, 32);
    msg[32] = (uint8_t)i;
    b2s_host(msg, 33, h);
    for (int b = 0; b < 32; ++b) le[b] = h[31 - b];  // from_str of the big-endian integer
    kk[i] = F.from_bytes_le(le, 32);
  }
  // The 80 spot checks are independent: checked on the host workers.
  auto spot = [&](size_t i) -> bool {
    const HostFp x = F.pow_u64(g2, positions[i]);
    auto leaf = [&](int b, int chunk) {
      return fe_from_bytes(pr.main[4 * i + b].leaf.data() + 32 * chunk, 32);
    };
    const HostFp p_x = leaf(0, 0), p_prev = leaf(1, 0), p_w = leaf(2, 0), p_2w = leaf(3, 0);
    const HostFp a_x = leaf(0, 1), a_prev = leaf(1, 1), s_x = leaf(0, 2), d1 = leaf(0, 3), d2 = leaf(0, 4),
                 d3 = leaf(0, 5), b2 = leaf(0, 6), b3 = leaf(0, 7);
    const HostFp z = F.sub(F.pow_u64(x, steps), F.one());  // best_fft of X^steps - 1 at x
    const HostFp k_x = col_val(0, i), f0 = col_val(1, i), f1 = col_val(2, i), f2 = col_val(3, i);
    const HostFp ext_idx = col_val(4, i), ext_pidx = col_val(5, i);
    // Q1 = Z D1, Q2 = Z D2 (verify.rs:208-219)
    if (!FieldHost::eq(F.mul(f0, F.sub(F.sub(p_x, F.mul(f1, p_prev)), F.mul(k_x, s_x))), F.mul(z, d1)))
      return false;
    if (!FieldHost::eq(F.mul(f2, F.sub(p_2w, F.mul(p_x, p_w))), F.mul(z, d2))) return false;
    // Q3 = Z D3 (verify.rs:221-225)
    const HostFp rs = F.mul(r[2], s_x);
    const HostFp nmr = F.add(F.add(r[0], F.mul(r[1], ext_idx)), rs);
    const HostFp dnm = F.add(F.add(r[0], F.mul(r[1], ext_pidx)), rs);
    if (!FieldHost::eq(F.sub(F.mul(a_x, dnm), F.mul(a_prev, nmr)), F.mul(z, d3))) return false;
    // Boundary constraints (verify.rs:227-238)
    HostFp zb2 = F.one();
    for (const HostFp& xk : bx) zb2 = F.mul(zb2, F.sub(x, xk));
    if (!FieldHost::eq(F.sub(s_x, eval_poly(interp2, x)), F.mul(zb2, b2))) return false;
    if (!FieldHost::eq(F.sub(a_x, eval_poly(interp3, x)), F.mul(F.sub(x, x_last), b3))) return false;
    // The linear combination (verify.rs:240-254)
    const HostFp xs = F.pow_u64(x, steps);
    HostFp l = F.mul(kk[0], d1);
    l = F.add(l, F.mul(kk[1], d2));
    l = F.add(l, F.mul(kk[2], d3));
    l = F.add(l, F.mul(kk[3], p_x));
    l = F.add(l, F.mul(F.mul(kk[4], p_x), xs));
    l = F.add(l, F.mul(kk[5], b2));
    l = F.add(l, F.mul(F.mul(kk[6], b2), xs));
    l = F.add(l, F.mul(kk[7], b3));
    l = F.add(l, F.mul(F.mul(kk[8], b3), xs));
    l = F.add(l, F.mul(kk[9], a_x));
    l = F.add(l, F.mul(kk[10], s_x));
    if (!FieldHost::eq(fe_from_bytes(pr.lcomb[i].leaf), l)) return false;
    return true;
  };
  std::vector<uint8_t> spot_ok(positions.size(), 0);
  std::atomic<size_t> next_spot{0};
  host_parallel(std::min<unsigned>(host_threads(), (unsigned)((positions.size() + 4) / 5)), [&](unsigned) {
    for (size_t i; (i = next_spot.fetch_add(1)) < positions.size();) spot_ok[i] = spot(i);
  });
  for (uint8_t g : spot_ok)
    if (!g) return STARK_ERR_CHECK;
  clk.mark("spot checks");
  return STARK_OK;
}

}  // namespace stark

using namespace stark;

extern "C" {

stark_status stark_verify_low_degree_proof(const uint8_t merkle_root[32], const uint64_t root_of_unity[4],
                                           const stark_fri_layer_parts* layers, size_t n_layers,
                                           const uint8_t* const* last_values, const size_t* last_lens, size_t n_last,
                                           size_t max_deg_plus_1, uint32_t exclude_multiples_of) {
  if (!merkle_root || !root_of_unity || (n_layers && !layers) || (n_last && (!last_values || !last_lens)))
    return STARK_ERR_BAD_ARG;
  std::vector<FriIn> proof(n_layers + 1);
  for (size_t l = 0; l < n_layers; ++l) {
    const stark_fri_layer_parts& P = layers[l];
    if (!P.root2) return STARK_ERR_BAD_ARG;
    memcpy(proof[l].root2, P.root2, 32);
    for (int which = 0; which < 2; ++which) {
      const stark_branches& B = which ? P.poly : P.column;
      std::vector<Branch>& out = which ? proof[l].poly : proof[l].col;
      if (B.k && (!B.leaves || (B.depth && !B.nodes))) return STARK_ERR_BAD_ARG;
      for (size_t i = 0; i < B.k; ++i) {
        Branch b;  // (views into the caller's arrays, which outlive the call)
        b.leaf = Bytes{B.leaves + i * B.leaf_len, B.leaf_len};
        b.nodes = Bytes{B.depth ? B.nodes + i * B.depth * 32 : nullptr, B.depth * 32};
        out.push_back(std::move(b));
      }
    }
  }
  proof[n_layers].last = true;
  for (size_t i = 0; i < n_last; ++i) proof[n_layers].last_vals.emplace_back(last_values[i], last_values[i] + last_lens[i]);
  const FieldHost& F = FieldHost::get();
  return verify_fri(merkle_root, F.from_canonical(root_of_unity), proof, max_deg_plus_1, exclude_multiples_of);
}

}  // extern "C"

namespace stark {
// The StarkProof JSON into pr; false where serde_json::from_reader fails (run.rs:579).
static bool read_proof(const char* proof_json, size_t json_len, ProofIn& pr) {
  PhaseClock clk("verify: read proof");
  PreBranches pre;
  pr.arena.reset(new uint8_t[json_len / 2 + 64]);
  uint8_t* const arena_end = pr.arena.get() + json_len / 2 + 64;
  pre_parse_branches(proof_json, json_len, pre, pr.arena.get(), arena_end);
  clk.mark("openings parsed (parallel)");
  Json j(proof_json, json_len, &pre, pr.arena.get(), arena_end);
  j.stark_proof(pr);
  clk.mark("StarkProof JSON parsed");
  return j.ok;
}
}  // namespace stark

extern "C" {

stark_status stark_verify_r1cs_circuit(stark_ctx* ctx, const stark_r1cs_circuit* circuit,
                                       const uint8_t* public_wires, size_t n_public, const char* proof_json,
                                       size_t json_len) {
  if (!ctx || !circuit || circuit->ctx != ctx || !public_wires || !proof_json || n_public == 0)
    return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  ProofIn pr;
  if (!read_proof(proof_json, json_len, pr)) return STARK_ERR_BAD_ARG;
  return verify_r1cs(ctx, circuit->c, public_wires, n_public, pr);
}

stark_status stark_verify_r1cs_bytes(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len,
                                     const uint8_t* public_wires, size_t n_public, const char* proof_json,
                                     size_t json_len) {
  if (!ctx || !r1cs || !public_wires || !proof_json || n_public == 0) return STARK_ERR_BAD_ARG;
  STARK_HIP(ctx, hipSetDevice(ctx->device));
  // The circuit's buffers are the context's, grown as needed and kept for the next call
  // (hipMalloc / hipFree of the extensions would otherwise dominate a small circuit's check).
  stark_r1cs_circuit circ;
  circ.ctx = ctx;
  std::swap(circ.c.arena, ctx->verify_arena);
  std::swap(circ.c.lde, ctx->verify_lde);
  circ.c.with_zb = false;  // verify_r1cs evaluates Zb2 / Zb3 at its spot positions on the host
  circ.c.spot = true;      // and the six circuit columns there from their first forward passes
  PhaseClock clk("verify: circuit");
  // The proof is read on the side thread while this one builds the circuit (mostly device work and
  // its synchronisations): the two do not depend on each other.
  auto pr = std::make_unique<ProofIn>();
  bool parsed = false;
  stark_status st;
  {
    HostTask read([&] { parsed = read_proof(proof_json, json_len, *pr); });
    st = circuit_build(ctx, r1cs, r1cs_len, circ.c);
    clk.mark("circuit build (proof read beside it)");
  }
  clk.mark("proof read joined");
  if (st == STARK_OK && !parsed) st = STARK_ERR_BAD_ARG;  // serde_json::from_reader fails (run.rs:579)
  if (st == STARK_OK) st = verify_r1cs(ctx, circ.c, public_wires, n_public, *pr);
  clk.mark("verify_r1cs returned");
  pr.reset();
  clk.mark("proof freed");
  std::swap(circ.c.arena, ctx->verify_arena);
  std::swap(circ.c.lde, ctx->verify_lde);
  return st;
}

stark_status stark_verify_with_witness(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len, const uint8_t* wtns,
                                       size_t wtns_len, const char* proof_json, size_t json_len) {
  if (!ctx || !r1cs || !wtns || !proof_json) return STARK_ERR_BAD_ARG;
  R1csHeader hd;
  WtnsHeader wh;
  stark_status st = parse_r1cs_header(r1cs, r1cs_len, &hd);
  if (st == STARK_OK) st = parse_wtns_header(wtns, wtns_len, &wh);
  if (st != STARK_OK) return st;
  // public_wires = witness[..1 + n_public_inputs + n_public_outputs] (run.rs:582-585)
  const size_t n_public = 1 + (size_t)hd.n_pub_in + hd.n_pub_out;
  if (n_public > wh.n_wit) return STARK_ERR_BAD_ARG;
  std::vector<uint8_t> pub(32 * n_public, 0);
  for (size_t i = 0; i < n_public; ++i) memcpy(&pub[32 * i], wtns + wh.values_off + i * wh.field_size, wh.field_size);
  return stark_verify_r1cs_bytes(ctx, r1cs, r1cs_len, pub.data(), n_public, proof_json, json_len);
}

}  // extern "C"
