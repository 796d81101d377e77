// Blake2s Merkle node hashing (merkle.hip's kernels): leaf node =
// Blake2s(leaf bytes), parent = Blake2s(left || right) (merkle_proof_in_place.rs:106-206).
#pragma once
#include "blake2s.h"
#include "internal.h"

namespace stark {

struct Digest {
  uint32_t h[8];
};

// Digest of one leaf of `len` bytes at p.
__device__ __forceinline__ Digest hash_leaf(const uint8_t* __restrict__ p, uint32_t len) {
  Digest d;
  b2s_init(d.h);
  uint32_t m[16];
  const bool vec = ((((uintptr_t)p) & 15) == 0) && ((len & 15) == 0);
  uint32_t off = 0;
  // Full blocks that are not the last one.
  while (len - off > 64) {
    if (vec) {
      const uint4* q = reinterpret_cast<const uint4*>(p + off);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint4 x = q[i];
        m[4 * i] = x.x; m[4 * i + 1] = x.y; m[4 * i + 2] = x.z; m[4 * i + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i)
        m[i] = (uint32_t)p[off + 4 * i] | ((uint32_t)p[off + 4 * i + 1] << 8) |
               ((uint32_t)p[off + 4 * i + 2] << 16) | ((uint32_t)p[off + 4 * i + 3] << 24);
    }
    off += 64;
    b2s_compress(d.h, m, off, 0, false);
  }
  // Final (possibly partial or empty) block, zero padded.
  const uint32_t rem = len - off;
  if (vec) {
    const uint4* q = reinterpret_cast<const uint4*>(p + off);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint4 x = (uint32_t)(16 * i) < rem ? q[i] : make_uint4(0, 0, 0, 0);
      m[4 * i] = x.x; m[4 * i + 1] = x.y; m[4 * i + 2] = x.z; m[4 * i + 3] = x.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      uint32_t w = 0;
      for (int k = 0; k < 4; ++k) {
        const uint32_t b = 4 * i + k;
        if (b < rem) w |= (uint32_t)p[off + b] << (8 * k);
      }
      m[i] = w;
    }
  }
  b2s_compress(d.h, m, len, 0, true);
  return d;
}

// A 32-byte leaf (one canonical field element): one final block whose words
// 8..15 are compile-time zeros, so their message additions fold away.
__device__ __forceinline__ Digest hash_leaf32(const uint8_t* __restrict__ p) {
  Digest d;
  b2s_init(d.h);
  uint32_t m[16];
  const uint4* q = reinterpret_cast<const uint4*>(p);
  const uint4 x = q[0], y = q[1];
  m[0] = x.x; m[1] = x.y; m[2] = x.z; m[3] = x.w;
  m[4] = y.x; m[5] = y.y; m[6] = y.z; m[7] = y.w;
#pragma unroll
  for (int i = 8; i < 16; ++i) m[i] = 0;
  b2s_compress(d.h, m, 32, 0, true);
  return d;
}

__device__ __forceinline__ Digest hash_pair(const Digest& l, const Digest& r) {
  uint32_t m[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[i] = l.h[i];
    m[i + 8] = r.h[i];
  }
  Digest d;
  b2s_init(d.h);
  b2s_compress(d.h, m, 64, 0, true);
  return d;
}

__device__ __forceinline__ Digest load_digest(const Digest* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 a = q[0], b = q[1];
  Digest d;
  d.h[0] = a.x; d.h[1] = a.y; d.h[2] = a.z; d.h[3] = a.w;
  d.h[4] = b.x; d.h[5] = b.y; d.h[6] = b.z; d.h[7] = b.w;
  return d;
}
__device__ __forceinline__ void store_digest(Digest* p, const Digest& d) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(d.h[0], d.h[1], d.h[2], d.h[3]);
  q[1] = make_uint4(d.h[4], d.h[5], d.h[6], d.h[7]);
}


}  // namespace stark
