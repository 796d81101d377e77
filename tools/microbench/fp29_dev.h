// EXPERIMENT (not used by libstark_hip): BN254 Fr in radix 2^29.
// Result: the product alone is ~1.3x faster than the radix-2^32 asm fe_mul
// (modmul29.hip, modmul29b.hip), but a full radix-4 NTT pass built on it ran
// 2.54 ms vs 2.13 ms per 2^24 transform (147 VGPRs -> 3 waves/SIMD, 9-limb
// LDS traffic), so the product path stays radix 2^32.  See DESIGN.md 9.
//
// BN254 Fr in radix 2^29: 9 x u32 limbs, each < 2^29 when normalised.
//
// Why: on gfx950 v_mad_u64_u32 and every carry op (v_add_co/v_addc) issue at
// half rate (tools/microbench/isa_lat.hip).  With 32-bit limbs a Montgomery
// product needs 128 mads + 128 carry counts; with 29-bit limbs 18 products of
// < 2^58 plus a carry-in never overflow a 64-bit accumulator, so the product
// is 162 mads and no carry instructions, and add/sub are full-rate limb adds.
// Montgomery radix R = 2^261.  Values are kept "lazily" in [0, 2^260):
// fe29_mul(a, b) < 2p whenever a < 2^260 and b < 2p (a*b < R p), so sums and
// differences need no modular reduction, only limb normalisation.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../stark-pure-rust_amd/csrc/fp_dev.h"

namespace stark {

constexpr uint32_t kM29 = (1u << 29) - 1;

struct fe29 {
  uint32_t l[9];
};

// Table entry: a normalised fe29 padded to 48 B so it loads as 3 x 16 B.
struct alignas(16) fe29t {
  uint32_t l[12];
};

// p in radix 2^29 (limb 8 holds bits 232..253).
__device__ __forceinline__ uint32_t p29(int i) {
  switch (i) {
    case 0: return 0x10000001u; case 1: return 0x1f0fac9fu; case 2: return 0x0e5c2450u; case 3: return 0x07d090f3u;
    case 4: return 0x1585d283u; case 5: return 0x02db40c0u; case 6: return 0x00a6e141u; case 7: return 0x0e5c2634u;
    default: return 0x0030644eu;
  }
}

// Montgomery product, R = 2^261.  -p^-1 mod 2^29 = 2^28 - 1, so the quotient
// digit is ((t << 28) - t) mod 2^29 (two full-rate ops instead of a multiply).
__device__ __forceinline__ fe29 fe29_mul(const fe29& a, const fe29& b) {
  uint32_t m[9];
  fe29 r;
  uint64_t acc = 0;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
#pragma unroll
    for (int j = 0; j < k; ++j) {
      acc += (uint64_t)a.l[j] * b.l[k - j];
      acc += (uint64_t)m[j] * p29(k - j);
    }
    acc += (uint64_t)a.l[k] * b.l[0];
    const uint32_t t = (uint32_t)acc;
    m[k] = ((t << 28) - t) & kM29;
    acc += (uint64_t)m[k] * p29(0);  // low 29 bits become 0
    acc >>= 29;
  }
#pragma unroll
  for (int k = 9; k < 17; ++k) {
#pragma unroll
    for (int j = k - 8; j < 9; ++j) {
      acc += (uint64_t)a.l[j] * b.l[k - j];
      acc += (uint64_t)m[j] * p29(k - j);
    }
    r.l[k - 9] = (uint32_t)acc & kM29;
    acc >>= 29;
  }
  r.l[8] = (uint32_t)acc;
  return r;
}

// Carry-propagate signed limbs into [0, 2^29) (top limb takes the rest).
__device__ __forceinline__ void fe29_normalize(fe29& x) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int32_t c = (int32_t)x.l[i] >> 29;
    x.l[i] &= kM29;
    x.l[i + 1] += (uint32_t)c;
  }
}

__device__ __forceinline__ fe29 fe29_add(const fe29& a, const fe29& b) {
  fe29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = a.l[i] + b.l[i];
  fe29_normalize(r);
  return r;
}

// Limb i of K p in radix 2^29 (compile-time; K < 32), built from p's
// 32-bit words so the offsets below are instruction literals, not registers.
__host__ __device__ constexpr uint32_t kp29_limb(uint32_t K, int i) {
  constexpr uint32_t P32[8] = {0xf0000001u, 0x43e1f593u, 0x79b97091u, 0x2833e848u,
                               0x8181585du, 0xb85045b6u, 0xe131a029u, 0x30644e72u};
  // bits [29 i, 29 i + 29) of K p, computed word by word with carries
  uint32_t w[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  uint64_t c = 0;
  for (int k = 0; k < 8; ++k) {
    const uint64_t t = (uint64_t)P32[k] * K + c;
    w[k] = (uint32_t)t;
    c = t >> 32;
  }
  w[8] = (uint32_t)c;
  const int bit = 29 * i, wi = bit / 32, sh = bit % 32;
  uint64_t v = w[wi] >> sh;
  if (wi + 1 < 9) v |= (uint64_t)w[wi + 1] << (32 - sh);
  return (uint32_t)v & ((1u << 29) - 1);
}

// a - b + K p (K chosen by the caller so that b < K p, hence the result >= 0).
template <uint32_t K>
__device__ __forceinline__ fe29 fe29_sub(const fe29& a, const fe29& b) {
  fe29 r;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.l[i] = a.l[i] - b.l[i] + kp29_limb(K, i);
  fe29_normalize(r);
  return r;
}

// 8 x u32 canonical (or any value < 2^256) -> radix 2^29.
__device__ __forceinline__ fe29 fe29_from_fe(const fe& x) {
  fe29 r;
  r.l[0] = x.w[0] & kM29;
  r.l[1] = __builtin_amdgcn_alignbit(x.w[1], x.w[0], 29) & kM29;
  r.l[2] = __builtin_amdgcn_alignbit(x.w[2], x.w[1], 26) & kM29;
  r.l[3] = __builtin_amdgcn_alignbit(x.w[3], x.w[2], 23) & kM29;
  r.l[4] = __builtin_amdgcn_alignbit(x.w[4], x.w[3], 20) & kM29;
  r.l[5] = __builtin_amdgcn_alignbit(x.w[5], x.w[4], 17) & kM29;
  r.l[6] = __builtin_amdgcn_alignbit(x.w[6], x.w[5], 14) & kM29;
  r.l[7] = __builtin_amdgcn_alignbit(x.w[7], x.w[6], 11) & kM29;
  r.l[8] = x.w[7] >> 8;
  return r;
}

// Normalised radix 2^29 value < 2^256 -> 8 x u32.
__device__ __forceinline__ fe fe_from_fe29(const fe29& x) {
  fe r;
  r.w[0] = x.l[0] | (x.l[1] << 29);
  r.w[1] = (x.l[1] >> 3) | (x.l[2] << 26);
  r.w[2] = (x.l[2] >> 6) | (x.l[3] << 23);
  r.w[3] = (x.l[3] >> 9) | (x.l[4] << 20);
  r.w[4] = (x.l[4] >> 12) | (x.l[5] << 17);
  r.w[5] = (x.l[5] >> 15) | (x.l[6] << 14);
  r.w[6] = (x.l[6] >> 18) | (x.l[7] << 11);
  r.w[7] = (x.l[7] >> 21) | (x.l[8] << 8);
  return r;
}

// Multiples q p (q < 32) in normalised radix 2^29, for fe29_canonical.
struct Kp29Table {
  uint32_t l[32][9];
};

// x (normalised, x < 32 p) -> x mod p as canonical 8 x u32.  The quotient
// estimate q = (x_hi * floor(2^264 / p)) >> 32 from the top limb satisfies
// floor(x/p) - 1 <= q <= floor(x/p), so x - q p < 2p and one conditional
// subtraction of p finishes.
__device__ __forceinline__ fe fe29_canonical(fe29 x, const Kp29Table* __restrict__ kp) {
  const uint32_t q = __umulhi(x.l[8], 1354u);
#pragma unroll
  for (int i = 0; i < 9; ++i) x.l[i] -= kp->l[q][i];
  fe29_normalize(x);
  fe29 y;
#pragma unroll
  for (int i = 0; i < 9; ++i) y.l[i] = x.l[i] - p29(i);
  fe29_normalize(y);
  const bool neg = (int32_t)y.l[8] < 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) x.l[i] = neg ? x.l[i] : y.l[i];
  return fe_from_fe29(x);
}

}  // namespace stark
