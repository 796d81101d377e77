// Host-only timing of the proof JSON renderer (JsonPieces, csrc/fri.hip) on a pedersen-sized proof shape:
// 160 + 40 spot-check branches and 10 FRI layers of 2 x 40 branches.  No GPU call.
//   hipcc -O3 -std=c++17 -I../../include -I../../stark-pure-rust_amd/csrc json_render_bench.cpp \
//     -L../../stark-pure-rust_amd -lstark_hip -Wl,-rpath,$PWD/../../stark-pure-rust_amd -o /tmp/jrb
#include <chrono>
#include <cstdio>
#include <random>
#include "internal.h"

namespace stark {
void json_bytes(std::string& o, const uint8_t* p, size_t n);
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  std::mt19937 rng(1);
  auto fill = [&](size_t n) {
    std::vector<uint8_t> v(n);
    for (auto& b : v) b = (uint8_t)rng();
    return v;
  };
  const size_t depth = 20;
  std::vector<std::vector<uint8_t>> keep;
  auto add_branches = [&](stark::JsonPieces& j, size_t k, size_t leaf_len, size_t d) {
    keep.push_back(fill(k * leaf_len));
    keep.push_back(fill(k * d * 32));
    j.branches(keep[keep.size() - 2], leaf_len, keep.back(), k, d);
  };
  double best = 1e9, sum = 0;
  size_t n = 0;
  for (int r = 0; r < reps; ++r) {
    keep.clear();
    keep.reserve(64);
    stark::JsonPieces j;
    j.text("{\"main_branches\":");
    add_branches(j, 160, 256, depth);
    j.text(",\"linear_comb_branches\":");
    add_branches(j, 40, 32, depth);
    j.text(",\"fri_proof\":[");
    for (int l = 0; l < 10; ++l) {
      if (l) j.text(",");
      j.text("{\"Middle\":{\"column_branches\":");
      add_branches(j, 40, 32, depth - 2 * l > 2 ? depth - 2 * l : 2);
      j.text(",\"poly_branches\":");
      add_branches(j, 160, 32, depth - 2 * l > 2 ? depth - 2 * l : 2);
      j.text("}}");
    }
    j.text("]}");
    stark::JsonText t;
    const auto t0 = std::chrono::steady_clock::now();
    j.render(t);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    n = t.size();
    if (r) {
      best = us < best ? us : best;
      sum += us;
    }
  }
  printf("json %zu B  render best %.1f us  mean %.1f us  (%u host threads)\n", n, best, sum / (reps - 1),
         stark::host_threads());
  // one thread: json_bytes over 40960 digests of 32 B (1.3 MB, the size of a pedersen proof's bytes)
  const std::vector<uint8_t> d = fill((size_t)40960 * 32);
  std::string o;
  o.reserve((size_t)6 << 20);
  double b1 = 1e9;
  for (int r = 0; r < reps; ++r) {
    o.clear();
    const auto t0 = std::chrono::steady_clock::now();
    for (size_t i = 0; i < 40960; ++i) stark::json_bytes(o, d.data() + 32 * i, 32);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    b1 = us < b1 ? us : b1;
  }
  printf("one thread: %zu B of text from 1.3 MB in best %.1f us (%.2f ns per byte)\n", o.size(), b1,
         b1 * 1e3 / (40960.0 * 32));
  return 0;
}
