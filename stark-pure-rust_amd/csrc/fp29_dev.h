// BN254 Fr in radix 2^29 on the gfx950 VALU: the NTT pass kernel's working representation.
//
// fe29 = 9 x u32 limbs, value sum l_i 2^(29 i).  Limbs are NOT kept normalised: a sum or a difference
// is 9 independent v_add_u32 / v_sub_u32 (full-rate instructions, no carry chain), and the Shoup
// product (fe29_asm.inc) accepts limbs below 2^31.6 because its 64-bit column accumulators hold
// 18 products of < 2^60.6 without overflow, so it needs no carry instructions either.  Measured on
// gfx950 (tools/microbench/pair_rates.hip): v_mad_u64_u32 and every carry op cost ~4.4 issue cycles,
// v_add_u32 / v_and_b32 ~2.4 and v_mov_b32 ~0.5, which is what this representation trades on.
//
// Bounds (checked by tests/test_fe29.py on an exact emulation):
//   normalised: l_i < 2^29 (i < 8);  a product's output is normalised with value < 3p;
//   fe29_add(x, t) = x + t,  fe29_subk(x, t) = x - t + 4p  (t normalised with value < 3p, so every
//   limb of 4p's borrowed image kK29 is >= t's: no limb underflows);  each grows a limb by < 2^30;
//   product inputs: limbs < 2^31.6 (normalised + two levels of growth) and value < 2^261.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fp_dev.h"

namespace stark {

constexpr uint32_t kM29 = (1u << 29) - 1;

struct fe29 {
  uint32_t l[9];
};

// A Shoup pair (w, wq = floor(w 2^261 / p)) as stored in the twiddle tables: 20 dwords, 16-B aligned.
struct alignas(16) fe29p {
  uint32_t w[9], wq[9], pad[2];
};

#include "fe29_asm.inc"

// 4p with every limb but the top one borrowed up to >= 2^29 - 1 (>= any normalised limb) and the top
// limb 0xc19138 >= the top limb of any value below 3p.
__device__ __forceinline__ uint32_t k4p29(int i) {
  switch (i) {
    case 0: return 0x20000004u; case 1: return 0x3c3eb27du; case 2: return 0x39709142u; case 3: return 0x3f4243ccu;
    case 4: return 0x36174a0bu; case 5: return 0x2b6d0301u; case 6: return 0x229b8503u; case 7: return 0x397098cfu;
    default: return 0x00c19138u;
  }
}

// 2^261 - p, normalised (the modular reduction's addend).
__device__ __forceinline__ uint32_t np29(int i) {
  switch (i) {
    case 0: return 0x0fffffffu; case 1: return 0x00f05360u; case 2: return 0x11a3dbafu; case 3: return 0x182f6f0cu;
    case 4: return 0x0a7a2d7cu; case 5: return 0x1d24bf3fu; case 6: return 0x1f591ebeu; case 7: return 0x11a3d9cbu;
    default: return 0x1fcf9bb1u;
  }
}

__device__ __forceinline__ void fe29_add(fe29& x, const fe29& t) {
#pragma unroll
  for (int i = 0; i < 9; ++i) x.l[i] += t.l[i];
}

// y = x - t + 4p
__device__ __forceinline__ fe29 fe29_subk(const fe29& x, const fe29& t) {
  fe29 y;
#pragma unroll
  for (int i = 0; i < 9; ++i) y.l[i] = x.l[i] + k4p29(i) - t.l[i];
  return y;
}

// Radix-2 butterfly: (x, y) <- (x + t, x - t + 4p); t may alias y.
__device__ __forceinline__ void fe29_bfly(fe29& x, fe29& y, const fe29& t) {
  const fe29 d = fe29_subk(x, t);
  fe29_add(x, t);
  y = d;
}

// Carry-propagate limbs 0..7 into 29-bit limbs (limb 8 takes the rest).
__device__ __forceinline__ void fe29_normalize(fe29& x) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    x.l[i + 1] += x.l[i] >> 29;
    x.l[i] &= kM29;
  }
}

// Canonical u32x8 (any value < 2^256) -> normalised fe29.
__device__ __forceinline__ fe29 fe29_from32(const fe& a) {
  fe29 x;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int bit = 29 * i, j = bit >> 5, s = bit & 31;
    const uint32_t lo = a.w[j], hi = j + 1 < 8 ? a.w[j + 1] : 0u;
    x.l[i] = __builtin_amdgcn_alignbit(hi, lo, s) & kM29;
  }
  x.l[8] = a.w[7] >> 8;
  return x;
}

// Normalised fe29 of value < 2^256 -> u32x8.
__device__ __forceinline__ fe fe29_to32(const fe29& x) {
  fe a;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int bit = 32 * j, i = bit / 29, s = bit % 29;
    uint32_t v = x.l[i] >> s;
    v |= x.l[i + 1] << (29 - s);
    if (29 * (i + 2) < 32 * (j + 1)) v |= x.l[i + 2] << (58 - s);
    a.w[j] = v;
  }
  return a;
}

// Any fe29 with value < 2^261 and limbs < 2^32 -> canonical u32x8 (the transform's last store).
// q = floor(l_8 / (p_8 + 1)) underestimates floor(x / p) by at most one (the float quotient is
// scaled down by 2^-20 so it never rounds up), so x - q p = x + q (2^261 - p) mod 2^261 < 3p.
__device__ __forceinline__ fe fe29_canonical(fe29 x) {
  fe29_normalize(x);
  const uint32_t q = (uint32_t)((float)x.l[8] * (float)(1.0 / 3171407.0 * (1.0 - 1.0 / (1 << 20))));
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint64_t t = (uint64_t)q * np29(i) + x.l[i] + c;
    x.l[i] = (uint32_t)t & kM29;
    c = t >> 29;
  }
  fe r = fe29_to32(x);  // < 3p < 2^256
  fe_reduce_lazy(r);    // [0, 4p) -> [0, p)
  return r;
}

// Global / LDS image of an element as three planes (limbs 0-3, 4-7, 8), so every access is an
// aligned 16-B or 4-B vector access: plane stride `ps` elements between A, B and C.
__device__ __forceinline__ fe29 fe29_load_planes(const uint32_t* base, size_t idx, size_t ps) {
  const uint4 a = reinterpret_cast<const uint4*>(base)[idx];
  const uint4 b = reinterpret_cast<const uint4*>(base)[ps + idx];
  const uint32_t c = base[8 * ps + idx];
  fe29 x;
  x.l[0] = a.x; x.l[1] = a.y; x.l[2] = a.z; x.l[3] = a.w;
  x.l[4] = b.x; x.l[5] = b.y; x.l[6] = b.z; x.l[7] = b.w;
  x.l[8] = c;
  return x;
}
__device__ __forceinline__ void fe29_store_planes(uint32_t* base, size_t idx, size_t ps, const fe29& x) {
  reinterpret_cast<uint4*>(base)[idx] = make_uint4(x.l[0], x.l[1], x.l[2], x.l[3]);
  reinterpret_cast<uint4*>(base)[ps + idx] = make_uint4(x.l[4], x.l[5], x.l[6], x.l[7]);
  base[8 * ps + idx] = x.l[8];
}

__device__ __forceinline__ void fe29p_load(const fe29p* t, fe29& w, fe29& wq) {
  const uint4* q = reinterpret_cast<const uint4*>(t);
  const uint4 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4];
  w.l[0] = a.x; w.l[1] = a.y; w.l[2] = a.z; w.l[3] = a.w;
  w.l[4] = b.x; w.l[5] = b.y; w.l[6] = b.z; w.l[7] = b.w;
  w.l[8] = c.x; wq.l[0] = c.y; wq.l[1] = c.z; wq.l[2] = c.w;
  wq.l[3] = d.x; wq.l[4] = d.y; wq.l[5] = d.z; wq.l[6] = d.w;
  wq.l[7] = e.x; wq.l[8] = e.y;
}

__device__ __forceinline__ fe29 fe29_mul_pair(const fe29& a, const fe29p* t) {
  fe29 w, wq;
  fe29p_load(t, w, wq);
  return fe29_mul_shoup(a, w, wq);
}

// ---- 256-bit helpers for the table conversion (one-time, per table entry) ----
__device__ __forceinline__ void mul_lo256(const uint32_t* a, const uint32_t* b, uint32_t* r) {
  uint32_t t[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
    for (int j = 0; i + j < 8; ++j) {
      const uint64_t v = (uint64_t)a[i] * b[j] + t[i + j] + c;
      t[i + j] = (uint32_t)v;
      c = v >> 32;
    }
  }
  for (int i = 0; i < 8; ++i) r[i] = t[i];
}
__device__ __forceinline__ void neg256(uint32_t* x) {  // x <- 2^256 - x (mod 2^256)
  uint64_t borrow = 0;
  for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)0 - x[i] - borrow;
    x[i] = (uint32_t)d;
    borrow = (d >> 32) & 1;
  }
}
__device__ __forceinline__ bool ge_p(const uint32_t* x) {
  for (int i = 7; i >= 0; --i) {
    const uint32_t pi = p_limb(i);
    if (x[i] != pi) return x[i] > pi;
  }
  return true;
}
__device__ __forceinline__ void sub_p(uint32_t* x) {
  uint64_t borrow = 0;
  for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)x[i] - p_limb(i) - borrow;
    x[i] = (uint32_t)d;
    borrow = (d >> 32) & 1;
  }
}

// p^-1 mod 2^256 (u32 limbs)
__device__ __forceinline__ uint32_t pinv32(int i) {
  switch (i) {
    case 0: return 0x10000001u; case 1: return 0x3d1e0a6cu; case 2: return 0xb396ee4cu; case 3: return 0x9a7979b4u;
    case 4: return 0x66f9dc6eu; case 5: return 0x1c6567d7u; case 6: return 0xf27cbe4du; default: return 0x8c07d0e2u;
  }
}

// The radix-2^29 Shoup pair of w from (w canonical, q32 = floor(w 2^256 / p), m = w 2^256 mod p):
// wq = floor(w 2^261 / p) = 32 q32 + floor(32 m / p).
__device__ inline fe29p pair29(const fe& w, const uint32_t* q32, const uint32_t* m) {
  uint32_t t[8];
  for (int i = 0; i < 8; ++i) t[i] = m[i];
  uint32_t d = 0;
  for (int k = 0; k < 5; ++k) {  // t < p < 2^254: doubling never overflows
    uint32_t c = 0;
    for (int i = 0; i < 8; ++i) {
      const uint32_t v = t[i];
      t[i] = (v << 1) | c;
      c = v >> 31;
    }
    d <<= 1;
    if (ge_p(t)) {
      sub_p(t);
      d |= 1;
    }
  }
  uint32_t v[9];  // 32 q32 + d, 261 bits
  v[0] = (q32[0] << 5) | d;
  for (int i = 1; i < 8; ++i) v[i] = (q32[i] << 5) | (q32[i - 1] >> 27);
  v[8] = q32[7] >> 27;
  fe29p out;
  for (int i = 0; i < 9; ++i) {
    const int bit = 29 * i, j = bit >> 5, s = bit & 31;
    const uint64_t two = (uint64_t)v[j] | ((uint64_t)(j + 1 < 9 ? v[j + 1] : 0u) << 32);
    out.wq[i] = (uint32_t)(two >> s) & kM29;
  }
  const fe29 w29 = fe29_from32(w);
  for (int i = 0; i < 9; ++i) out.w[i] = w29.l[i];
  out.pad[0] = out.pad[1] = 0;
  return out;
}

// From a Montgomery image m = w 2^256 mod p.
__device__ inline fe29p pair29_from_mont(fe mm) {
  fe one = fe_zero();
  one.w[0] = 1;
  const fe w = fe_mul(mm, one);  // m 2^-256 = w, canonical
  uint32_t q[8];
  uint32_t m[8];
  for (int i = 0; i < 8; ++i) m[i] = mm.w[i];
  uint32_t nm[8];
  for (int i = 0; i < 8; ++i) nm[i] = m[i];
  neg256(nm);
  uint32_t pv[8];
  for (int i = 0; i < 8; ++i) pv[i] = pinv32(i);
  mul_lo256(nm, pv, q);  // q = -m p^-1 mod 2^256 = floor(w 2^256 / p)
  return pair29(w, q, m);
}
}  // namespace stark
