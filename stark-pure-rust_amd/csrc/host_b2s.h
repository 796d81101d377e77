// Host Merkle path checks (Proof::validate, packages/commitment/src/merkle_tree.rs:25-43) with Blake2s
// compressions of W paths per SIMD register: the verifier's ~2.6e4 path compressions per proof
// (verify.hip paths_check).  Plain C++ (host_b2s*.cpp, built by g++): one translation unit per vector
// width, picked at run time from the CPU's features.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace stark {

struct PathJob {
  const uint8_t* root;   // 32 B
  uint64_t index;        // leaf index: bit d picks the side at level d
  const uint8_t* leaf;   // leaf bytes (hashed whole: Blake2s(leaf))
  const uint8_t* nodes;  // depth siblings of 32 B, leaf -> root
  uint32_t leaf_len, depth;
};

// ok[i] = 1 iff job i's path leads to its root.  Consecutive jobs with equal (leaf_len, depth) share
// registers; any mix is accepted.
void b2s_paths(const PathJob* jobs, size_t n, uint8_t* ok);

// The vector width b2s_paths uses on this CPU (16: AVX-512, 8: AVX2, 4: SSE2; STARK_B2S_WIDTH may
// narrow it).
int b2s_paths_width();

}  // namespace stark
