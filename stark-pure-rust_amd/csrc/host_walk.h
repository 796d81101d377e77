// The walk over an .r1cs constraint section's record counts (host_walk.cpp): host-only C++, no HIP, so it
// is built and checked on its own on the CPU (tests/host_walk: the parallel walk against the serial one).
//
// The section is n_c constraints of three factors each, a factor being a u32 count nc followed by nc
// 36-byte records (u32 wire id, 32-byte LE coefficient; circom2bellman_core reader.rs:4-89 reads them one
// by one, run.rs:109-137 counts the slots).  The walk yields, per factor k = 3 ci + f, the byte offset of
// its first record (fac[k]) and its count (fac[3 n_c + k]), a pad word fac[6 n_c] = 0, and base[ci], the
// first slot of constraint ci (n_c + 1 entries: the prefix sums of each constraint's largest count).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

#include "stark_hip.h"

namespace stark {

// The serial walk: its results, and its status on malformed input, define the walk.
stark_status walk_records_into(const uint8_t* cons, size_t cons_len, uint32_t n_c, uint32_t* fac, uint32_t* base);

// The same walk split over `parts` host threads.  The next factor's position depends on the previous
// count, so part k (k > 0) starts at a guessed factor header near k / parts of the section (a position
// from which several headers in a row read as plausible counts, wire ids and coefficients) and walks to the
// next part's guess.  finish() then links the parts in order: a part is taken from the first position the
// true walk (part 0 onwards) shares with it -- from there the two walks are the same walk, the next
// position being a function of the current one -- and where a guess was wrong the true walk goes on
// serially until it meets a later part.  Only positions the true walk reaches are used, so the results
// equal walk_records_into's; whenever the true walk would stop early (a count past the end, too few
// bytes), finish() runs walk_records_into itself for its exact status.
class RecordWalk {
 public:
  RecordWalk(const uint8_t* cons, size_t cons_len, uint32_t n_c, uint32_t n_wires, unsigned parts);
  unsigned parts() const { return (unsigned)chains_.size(); }
  // The walk of part k (0 <= k < parts): any thread, any order, the parts do not wait for one another.
  void part(unsigned k);
  // Links the parts and writes fac / base (host_parallel over the parts); after every part() has run.
  stark_status finish(uint32_t* fac, uint32_t* base);
  // How the last finish() got there: 0 every guess was right, 1 some factors were walked serially while
  // linking, 2 the serial walk (input too small to split, or the true walk stops early).
  int path() const { return path_; }
  // Factors walked serially while linking (path 1).
  size_t serial_factors() const { return serial_; }

 private:
  struct Chain {
    std::vector<uint32_t> hdr;  // header positions, ascending
    std::vector<uint32_t> cnt;  // their counts
    uint64_t end = 0;           // the position after the last header (or where the walk stopped)
    int stop = 0;               // 0 reached the next part's guess, 1 fewer than 4 bytes left, 2 count past the end
  };
  uint64_t guess(unsigned k) const;  // part k's start (0 for k = 0); kNone when no plausible header is near
  bool plausible(uint64_t p) const;
  static constexpr uint64_t kNone = ~0ull;
  const uint8_t* cons_;
  uint64_t len_;
  uint32_t n_c_, n_wires_;
  std::vector<Chain> chains_;
  int path_ = 2;
  size_t serial_ = 0;
};

}  // namespace stark
