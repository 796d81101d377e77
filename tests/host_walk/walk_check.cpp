// The split record walk (csrc/host_walk.cpp, RecordWalk) against the serial walk (walk_records_into) on
// generated constraint sections: the same status, and on success the same fac / base words.
//   walk_check check N   N seeds of each case (exit 1 on the first difference)
//   walk_check bench     serial vs split on a 20 MB section (timing only)
// Cases: canonical random coefficients, small-integer ones (the hard case for a part's guess: their zero
// words read as empty factors), -1, zero; factor counts 0..k; trailing bytes after the section (the file's
// later sections); truncations and corrupted counts at random places; n_c larger than the section holds.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <random>
#include <vector>

#include "host_pool.h"
#include "host_walk.h"

using namespace stark;

namespace {

struct Section {
  std::vector<uint8_t> bytes;
  uint32_t n_c, n_wires;
};

void put32(std::vector<uint8_t>& b, uint32_t v) {
  uint8_t t[4];
  memcpy(t, &v, 4);
  b.insert(b.end(), t, t + 4);
}

// mode 0 canonical random, 1 small integers, 2 p - 1, 3 a mix, 4 zero
Section make(std::mt19937_64& rng, uint32_t n_c, uint32_t n_wires, int mode, uint32_t max_count, size_t trailing) {
  static const uint32_t pm1[8] = {0xF0000000u, 0x43E1F593u, 0x79B97091u, 0x2833E848u,
                                  0x8181585Du, 0xB85045B6u, 0xE131A029u, 0x30644E72u};
  Section s;
  s.n_c = n_c;
  s.n_wires = n_wires;
  s.bytes.reserve((size_t)n_c * 3 * (4 + 36 * (max_count + 1) / 2) + trailing + 64);
  for (uint32_t ci = 0; ci < n_c; ++ci)
    for (int f = 0; f < 3; ++f) {
      uint32_t nc = (uint32_t)(rng() % (max_count + 1));
      if (f == 2 && rng() % 3 == 0) nc = 0;
      put32(s.bytes, nc);
      for (uint32_t i = 0; i < nc; ++i) {
        put32(s.bytes, (uint32_t)(rng() % n_wires));
        const int m = mode == 3 ? (int)(rng() % 3) : mode;
        uint32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (m == 0) {
          for (int w = 0; w < 8; ++w) c[w] = (uint32_t)rng();
          c[7] %= 0x30644E72u;
        } else if (m == 1) {
          c[0] = 1 + (uint32_t)(rng() % 7);
        } else if (m == 2) {
          memcpy(c, pm1, 32);
        }
        for (int w = 0; w < 8; ++w) put32(s.bytes, c[w]);
      }
    }
  for (size_t t = 0; t < trailing; ++t) s.bytes.push_back((uint8_t)rng());
  return s;
}

struct Result {
  stark_status st;
  std::vector<uint32_t> fac, base;
};

Result serial(const uint8_t* b, size_t len, uint32_t n_c) {
  Result r;
  r.fac.assign((size_t)6 * n_c + 1, 0xDEADBEEFu);
  r.base.assign((size_t)n_c + 1, 0xDEADBEEFu);
  r.st = walk_records_into(b, len, n_c, r.fac.data(), r.base.data());
  return r;
}

Result split(const uint8_t* b, size_t len, uint32_t n_c, uint32_t n_wires, unsigned parts, bool reverse, int* path,
             double* serial_frac = nullptr) {
  Result r;
  r.fac.assign((size_t)6 * n_c + 1, 0xDEADBEEFu);
  r.base.assign((size_t)n_c + 1, 0xDEADBEEFu);
  RecordWalk w(b, len, n_c, n_wires, parts);
  if (reverse) {
    for (unsigned k = w.parts(); k-- > 0;) w.part(k);
  } else {
    host_parallel(w.parts(), [&](unsigned k) { w.part(k); });
  }
  r.st = w.finish(r.fac.data(), r.base.data());
  *path = w.path();
  if (serial_frac) *serial_frac = n_c ? (double)w.serial_factors() / (3.0 * n_c) : 0.0;
  return r;
}

bool same(const Result& a, const Result& b) {
  if (a.st != b.st) return false;
  if (a.st != STARK_OK) return true;
  return a.fac == b.fac && a.base == b.base;
}

int check(int seeds) {
  const unsigned parts_list[] = {2, 3, 4, 7, 8, 16};
  int paths[5][3] = {};
  double serial_sum[5] = {};
  size_t cases = 0;
  for (int seed = 0; seed < seeds; ++seed)
    for (int mode = 0; mode < 5; ++mode) {
      std::mt19937_64 rng(0x5EED5A1Cull * (seed + 1) + mode);
      const uint32_t n_c = 4000 + (uint32_t)(rng() % 12000);
      const uint32_t n_wires = 50 + (uint32_t)(rng() % 100000);
      const uint32_t max_count = 1 + (uint32_t)(rng() % 6);
      const Section s = make(rng, n_c, n_wires, mode, max_count, (size_t)(rng() % 200000));
      // the intact section, then damaged copies: truncated, a count made too large, n_c over-claimed
      struct Variant {
        size_t len;
        uint32_t n_c;
        std::vector<uint8_t> bytes;
      };
      std::vector<Variant> vs;
      vs.push_back({s.bytes.size(), n_c, s.bytes});
      vs.push_back({(size_t)(rng() % s.bytes.size()), n_c, s.bytes});
      {
        Variant v{s.bytes.size(), n_c, s.bytes};
        const Result r = serial(v.bytes.data(), v.len, n_c);
        if (r.st == STARK_OK) {  // corrupt the count of a random factor
          const size_t k = (size_t)(rng() % (3ull * n_c));
          const uint32_t pos = r.fac[k] - 4;
          const uint32_t huge = 0x7FFFFFF0u;
          memcpy(v.bytes.data() + pos, &huge, 4);
        }
        vs.push_back(std::move(v));
      }
      vs.push_back({s.bytes.size(), n_c + 1 + (uint32_t)(rng() % 50000), s.bytes});
      for (size_t vi = 0; vi < vs.size(); ++vi) {
        const Variant& v = vs[vi];
        const Result want = serial(v.bytes.data(), v.len, v.n_c);
        for (unsigned parts : parts_list)
          for (int rev = 0; rev < 2; ++rev) {
            int path = -1;
            double frac = 0;
            const Result got = split(v.bytes.data(), v.len, v.n_c, n_wires, parts, rev != 0, &path, &frac);
            ++cases;
            if (!same(got, want)) {
              fprintf(stderr, "MISMATCH seed %d mode %d variant %zu parts %u rev %d: status %d vs %d\n", seed, mode,
                      vi, parts, rev, (int)got.st, (int)want.st);
              return 1;
            }
            if (vi == 0 && v.len >= ((size_t)1 << 20)) {
              ++paths[mode][path];
              serial_sum[mode] += frac;
            }
          }
      }
    }
  printf("cases %zu, all equal\n", cases);
  for (int m = 0; m < 5; ++m)
    printf("mode %d intact (>= 1 MB): path0 %d path1 %d path2 %d, factors walked while linking %.2f %%\n", m,
           paths[m][0], paths[m][1], paths[m][2],
           100.0 * serial_sum[m] / std::max(1, paths[m][0] + paths[m][1] + paths[m][2]));
  // The split must be the rule on canonical coefficients (mode 0): no more than 1 in 20 runs serial.
  const int m0 = paths[0][0] + paths[0][1] + paths[0][2];
  if (paths[0][2] * 20 > m0) {
    fprintf(stderr, "mode 0 fell back to the serial walk in %d of %d runs\n", paths[0][2], m0);
    return 2;
  }
  return 0;
}

int bench() {
  std::mt19937_64 rng(42);
  const Section s = make(rng, 58255, 58258, 3, 5, 500000);
  printf("section %zu bytes, n_c %u, host threads %u\n", s.bytes.size(), s.n_c, host_threads());
  for (int rep = 0; rep < 5; ++rep) {
    auto t0 = std::chrono::steady_clock::now();
    const Result a = serial(s.bytes.data(), s.bytes.size(), s.n_c);
    auto t1 = std::chrono::steady_clock::now();
    Result b;
    b.fac.assign((size_t)6 * s.n_c + 1, 0);
    b.base.assign((size_t)s.n_c + 1, 0);
    auto t2 = std::chrono::steady_clock::now();
    RecordWalk w(s.bytes.data(), s.bytes.size(), s.n_c, s.n_wires, host_threads());
    host_parallel(w.parts(), [&](unsigned k) { w.part(k); });
    auto t3 = std::chrono::steady_clock::now();
    b.st = w.finish(b.fac.data(), b.base.data());
    auto t4 = std::chrono::steady_clock::now();
    auto us = [](auto x, auto y) { return std::chrono::duration<double, std::micro>(y - x).count(); };
    printf("serial %.1f us (with its output's allocation), split: parts %.1f us + finish %.1f us (path %d, equal %d)\n",
           us(t0, t1), us(t2, t3), us(t3, t4), w.path(), (int)same(a, b));
  }
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "check";
  if (!strcmp(mode, "bench")) return bench();
  return check(argc > 2 ? atoi(argv[2]) : 4);
}
