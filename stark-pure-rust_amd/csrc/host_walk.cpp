// The constraint section's record walk (host_walk.h): the serial walk and its split over host threads.
#include "host_walk.h"

#include <string.h>

#include <algorithm>

#include "host_pool.h"

namespace stark {

stark_status walk_records_into(const uint8_t* cons, size_t cons_len, uint32_t n_c, uint32_t* fac, uint32_t* base) {
  if (cons_len > 0xFFFFFFFFull) return STARK_ERR_BAD_ARG;
  uint32_t* fac_rec = fac;
  uint32_t* fac_cnt = fac + (size_t)3 * n_c;
  fac[(size_t)6 * n_c] = 0;
  base[0] = 0;
  size_t pos = 0;
  uint64_t b = 0;
  for (uint32_t ci = 0; ci < n_c; ++ci) {
    uint32_t n_coeff = 0;
    for (int f = 0; f < 3; ++f) {
      if (cons_len - pos < 4) return STARK_ERR_BAD_ARG;
      uint32_t nc;
      memcpy(&nc, cons + pos, 4);
      pos += 4;
      if (nc > (cons_len - pos) / 36) return STARK_ERR_BAD_ARG;
      fac_rec[3 * (size_t)ci + f] = (uint32_t)pos;
      fac_cnt[3 * (size_t)ci + f] = nc;
      pos += (size_t)nc * 36;
      if (nc > n_coeff) n_coeff = nc;
    }
    b += n_coeff;
    if (b > 0xFFFFFFFFull / 3) return STARK_ERR_BAD_LENGTH;
    base[ci + 1] = (uint32_t)b;
  }
  return STARK_OK;
}

namespace {
constexpr uint64_t kSplitFrom = (uint64_t)1 << 20;  // smaller sections: the serial walk
constexpr uint64_t kWindow = (uint64_t)1 << 18;     // a part's guess lies within this many bytes of its share
constexpr int kCheckHeaders = 16;                   // headers read by a guess
constexpr uint32_t kCoefTop = 0x30644E72u;          // BN254 r's top word: a canonical coefficient's is <= this
constexpr uint32_t kGuessCount = 1024;              // larger counts do not start a guess (a wire id read as a
                                                    // count would send the guess's walk far past its share)
}  // namespace

RecordWalk::RecordWalk(const uint8_t* cons, size_t cons_len, uint32_t n_c, uint32_t n_wires, unsigned parts)
    : cons_(cons), len_(cons_len), n_c_(n_c), n_wires_(n_wires) {
  if (len_ < kSplitFrom || len_ > 0xFFFFFFFFull || n_c == 0 || n_wires == 0) parts = 1;
  chains_.resize(parts ? parts : 1);
}

// kCheckHeaders factor headers in a row from p whose counts fit the section (and kGuessCount), whose records (up to 8 per
// factor) carry wire ids below n_wires and canonical-looking coefficients, at least half of them non-empty
// and never three empty in a row (a run of zero words, e.g. inside small coefficients, reads as empty
// factors; a real constraint has at most two).
bool RecordWalk::plausible(uint64_t p) const {
  uint64_t q = p;
  int nonempty = 0, empty_run = 0;
  for (int h = 0; h < kCheckHeaders; ++h) {
    if (len_ - q < 4) return false;
    uint32_t nc;
    memcpy(&nc, cons_ + q, 4);
    if (nc > kGuessCount || nc > (len_ - q - 4) / 36) return false;
    empty_run = nc ? 0 : empty_run + 1;
    if (empty_run == 3) return false;
    const uint32_t check = nc < 8 ? nc : 8;
    for (uint32_t i = 0; i < check; ++i) {
      const uint8_t* r = cons_ + q + 4 + 36 * (uint64_t)i;
      uint32_t wire, top;
      memcpy(&wire, r, 4);
      memcpy(&top, r + 32, 4);
      if (wire >= n_wires_ || top > kCoefTop) return false;
    }
    nonempty += nc != 0;
    q += 4 + 36 * (uint64_t)nc;
  }
  return 2 * nonempty >= kCheckHeaders;
}

// Headers sit at multiples of 4 from the section's start (4 + 36 nc bytes per factor).
uint64_t RecordWalk::guess(unsigned k) const {
  if (k == 0) return 0;
  const uint64_t s = (len_ * k / chains_.size() + 3) & ~(uint64_t)3;
  const uint64_t e = std::min(len_, s + kWindow);
  for (uint64_t p = s; p + 4 <= e; p += 4)
    if (plausible(p)) return p;
  return kNone;
}

void RecordWalk::part(unsigned k) {
  if (chains_.size() < 2 || k >= chains_.size()) return;
  Chain& ch = chains_[k];
  ch.hdr.clear();
  ch.cnt.clear();
  ch.end = 0;
  ch.stop = 3;  // (no start)
  const uint64_t start = guess(k);
  if (start == kNone) return;
  uint64_t target = len_;  // the next part's start
  for (unsigned j = k + 1; j < chains_.size(); ++j) {
    const uint64_t g = guess(j);
    if (g != kNone) {
      target = g;
      break;
    }
  }
  const size_t expect = (size_t)((target > start ? target - start : 0) / 96) + 16;
  ch.hdr.reserve(expect);
  ch.cnt.reserve(expect);
  uint64_t p = start;
  ch.stop = 0;
  while (p < target) {
    if (len_ - p < 4) {
      ch.stop = 1;
      break;
    }
    uint32_t nc;
    memcpy(&nc, cons_ + p, 4);
    if (nc > (len_ - p - 4) / 36) {
      ch.stop = 2;
      break;
    }
    ch.hdr.push_back((uint32_t)p);
    ch.cnt.push_back(nc);
    p += 4 + 36 * (uint64_t)nc;
  }
  ch.end = p;
}

stark_status RecordWalk::finish(uint32_t* fac, uint32_t* base) {
  serial_ = 0;
  auto serial = [&] {
    path_ = 2;
    return walk_records_into(cons_, len_, n_c_, fac, base);
  };
  if (chains_.size() < 2) return serial();
  const uint64_t total = 3ull * n_c_;
  // The true walk's factors in order, as runs of parts (chain >= 0) or of its own linking steps (-1).
  struct Seg {
    int chain;
    size_t from, n;
    uint64_t f0;  // factor index of the run's first factor
  };
  std::vector<Seg> segs;
  std::vector<uint32_t> xh, xc;
  uint64_t F = 0;
  size_t k = 0, i = 0;  // the true walk is at part k's header i (part 0 starts at the section's start)
  if (chains_[0].stop == 3) return serial();
  for (;;) {
    const Chain& ch = chains_[k];
    const size_t n = (size_t)std::min<uint64_t>(ch.hdr.size() - i, total - F);
    if (n) segs.push_back({(int)k, i, n, F});
    F += n;
    if (F == total) break;
    if (ch.stop != 0) return serial();  // the true walk stops here: the serial walk's own status
    // Link: from the true walk's next header, step on until a later part has the same header.
    uint64_t p = ch.end;
    const size_t x0 = xh.size();
    const uint64_t xf0 = F;
    // (one serial step of the true walk; false where the serial walk would stop)
    auto step = [&]() {
      if (len_ - p < 4) return false;
      uint32_t nc;
      memcpy(&nc, cons_ + p, 4);
      if (nc > (len_ - p - 4) / 36) return false;
      xh.push_back((uint32_t)p);
      xc.push_back(nc);
      ++F;
      p += 4 + 36 * (uint64_t)nc;
      return true;
    };
    // The part to link with is the latest one starting at or before p (a wrong guess's walk may run on
    // far past the next part's start, so the parts' ranges can overlap).
    size_t cur = chains_.size(), m = 0, nxt = k + 1;
    while (F < total) {
      for (; nxt < chains_.size(); ++nxt) {
        const Chain& c = chains_[nxt];
        if (c.hdr.empty()) continue;
        if (c.hdr[0] > p) break;
        cur = nxt;
        m = (size_t)(std::lower_bound(c.hdr.begin(), c.hdr.end(), (uint32_t)p) - c.hdr.begin());
      }
      if (cur < chains_.size()) {
        const Chain& c = chains_[cur];
        while (m < c.hdr.size() && c.hdr[m] < p) ++m;
        if (m < c.hdr.size() && c.hdr[m] == p) {
          k = cur;
          i = m;
          break;
        }
      }
      if (!step()) return serial();
    }
    if (xh.size() > x0) segs.push_back({-1, x0, xh.size() - x0, xf0});
    serial_ += xh.size() - x0;
    if (F == total) break;
  }
  path_ = serial_ ? 1 : 0;
  // fac: each run into its place (one task per run); the records start 4 bytes after their header.
  host_parallel((unsigned)segs.size(), [&](unsigned s) {
    const Seg& g = segs[s];
    const uint32_t* h = g.chain < 0 ? xh.data() : chains_[g.chain].hdr.data();
    const uint32_t* c = g.chain < 0 ? xc.data() : chains_[g.chain].cnt.data();
    for (size_t t = 0; t < g.n; ++t) {
      fac[g.f0 + t] = h[g.from + t] + 4;
      fac[total + g.f0 + t] = c[g.from + t];
    }
  });
  fac[2 * total] = 0;
  // base: the prefix sums of each constraint's largest count, over ranges of constraints.
  const uint32_t* cnt = fac + total;
  const unsigned R = std::max(1u, std::min<unsigned>(host_threads(), n_c_ / 4096));
  std::vector<uint64_t> sums(R + 1, 0);
  auto widest = [&](uint64_t ci) {
    return std::max(cnt[3 * ci], std::max(cnt[3 * ci + 1], cnt[3 * ci + 2]));
  };
  host_parallel(R, [&](unsigned r) {
    uint64_t b = 0;
    for (uint64_t ci = (uint64_t)n_c_ * r / R, hi = (uint64_t)n_c_ * (r + 1) / R; ci < hi; ++ci) b += widest(ci);
    sums[r + 1] = b;
  });
  for (unsigned r = 0; r < R; ++r) sums[r + 1] += sums[r];
  // (the running sum only grows: it passes the bound iff the total does, as the serial walk finds)
  if (sums[R] > 0xFFFFFFFFull / 3) return STARK_ERR_BAD_LENGTH;
  base[0] = 0;
  host_parallel(R, [&](unsigned r) {
    uint64_t b = sums[r];
    for (uint64_t ci = (uint64_t)n_c_ * r / R, hi = (uint64_t)n_c_ * (r + 1) / R; ci < hi; ++ci) {
      b += widest(ci);
      base[ci + 1] = (uint32_t)b;
    }
  });
  return STARK_OK;
}

}  // namespace stark
