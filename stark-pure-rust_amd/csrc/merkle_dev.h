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



// ---- One compression per quad of lanes (merkle.hip's tail kernel, fri.hip's index kernel) ----
//
// Once a level has fewer nodes than the chip has lanes, a level costs one
// full compression's latency (a single lane issues ~1100 dependent-ish
// VALU ops: about 2 us).  Here the 4x4 Blake2s state is spread over the 4
// lanes of a quad, lane q holding column q (v[q], v[4+q], v[8+q], v[12+q]):
// the column step is one G per lane, the diagonal step is one G per lane
// after rotating b, c, d by 1, 2, 3 lanes with quad_perm DPP moves.  Each
// lane fetches its two message words per step from the message in LDS with a
// lane-dependent SIGMA index.

// SIGMA row r packed as 16 nibbles (entry i at bits 4i..4i+3).
__host__ __device__ constexpr uint64_t b2s_sigma_packed(int r) {
  uint64_t x = 0;
  for (int i = 0; i < 16; ++i) x |= (uint64_t)b2s_sigma(r, i) << (4 * i);
  return x;
}

template <int CTRL>
__device__ __forceinline__ uint32_t quad_perm(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)x, CTRL, 0xF, 0xF, false);
}
// quad_perm controls: lane i reads lane (i + k) & 3.
constexpr int kQuadRot1 = 1 | (2 << 2) | (3 << 4) | (0 << 6);
constexpr int kQuadRot2 = 2 | (3 << 2) | (0 << 4) | (1 << 6);
constexpr int kQuadRot3 = 3 | (0 << 2) | (1 << 4) | (2 << 6);

__device__ __forceinline__ void b2s_g(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t x, uint32_t y) {
  a = a + b + x;
  d = __builtin_amdgcn_alignbit(d ^ a, d ^ a, 16);
  c = c + d;
  b = __builtin_amdgcn_alignbit(b ^ c, b ^ c, 12);
  a = a + b + y;
  d = __builtin_amdgcn_alignbit(d ^ a, d ^ a, 8);
  c = c + d;
  b = __builtin_amdgcn_alignbit(b ^ c, b ^ c, 7);
}

__device__ __forceinline__ uint32_t sel4(uint32_t q, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3) {
  return q == 0 ? c0 : q == 1 ? c1 : q == 2 ? c2 : c3;
}

// Blake2s of the one-block message at msg (LDS, 16 words, zero padded past t_bytes <= 64) on the quad;
// lane q returns digest words q (lo) and 4 + q (hi).  All 4 lanes must be active.
__device__ __forceinline__ void hash_pair_quad(const uint32_t* msg, uint32_t q, uint32_t& lo, uint32_t& hi,
                                               uint32_t t_bytes = 64) {
  const uint32_t h_a = sel4(q, STARK_B2S_H0, STARK_B2S_IV1, STARK_B2S_IV2, STARK_B2S_IV3);
  const uint32_t h_b = sel4(q, STARK_B2S_IV4, STARK_B2S_IV5, STARK_B2S_IV6, STARK_B2S_IV7);
  uint32_t a = h_a, b = h_b;
  uint32_t c = sel4(q, STARK_B2S_IV0, STARK_B2S_IV1, STARK_B2S_IV2, STARK_B2S_IV3);
  // t = t_bytes (one final block) into v[12]; final flag into v[14].
  uint32_t d = h_b ^ sel4(q, t_bytes, 0u, 0xFFFFFFFFu, 0u);
  const uint32_t sh = 8 * q;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t sg = b2s_sigma_packed(r);
    const uint32_t col = (uint32_t)sg, dia = (uint32_t)(sg >> 32);
    const uint32_t x0 = msg[(col >> sh) & 15], y0 = msg[(col >> (sh + 4)) & 15];
    const uint32_t x1 = msg[(dia >> sh) & 15], y1 = msg[(dia >> (sh + 4)) & 15];
    b2s_g(a, b, c, d, x0, y0);
    b = quad_perm<kQuadRot1>(b);
    c = quad_perm<kQuadRot2>(c);
    d = quad_perm<kQuadRot3>(d);
    b2s_g(a, b, c, d, x1, y1);
    b = quad_perm<kQuadRot3>(b);
    c = quad_perm<kQuadRot2>(c);
    d = quad_perm<kQuadRot1>(d);
  }
  lo = h_a ^ a ^ c;
  hi = h_b ^ b ^ d;
}

}  // namespace stark
