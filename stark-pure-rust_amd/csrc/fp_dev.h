// BN254 scalar-field arithmetic on gfx950 VALU.
//
// Element = 8 x u32 little-endian limbs.  Multiplication is Montgomery with
// R = 2^256 (ff_derive 0.10's representation for Fp, ff_utils/src/fp.rs:7-12),
// so a limb image is byte-identical to the reference's [u64; 4].
//
// Convention used by every kernel in this library: DATA stays canonical
// (the to_bytes_le image), CONSTANTS (twiddles, scales) are stored in
// Montgomery form.  montmul(data, const_mont) = data * const (canonical), so
// linear transforms never need to_mont/from_mont passes.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace stark {

struct fe {
  uint32_t w[8];
};

// p = 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001
#define STARK_P0 0xf0000001u
#define STARK_P1 0x43e1f593u
#define STARK_P2 0x79b97091u
#define STARK_P3 0x2833e848u
#define STARK_P4 0x8181585du
#define STARK_P5 0xb85045b6u
#define STARK_P6 0xe131a029u
#define STARK_P7 0x30644e72u
// -p^{-1} mod 2^32
#define STARK_PINV32 0xefffffffu

__device__ __forceinline__ uint32_t p_limb(int i) {
  switch (i) {
    case 0: return STARK_P0; case 1: return STARK_P1; case 2: return STARK_P2; case 3: return STARK_P3;
    case 4: return STARK_P4; case 5: return STARK_P5; case 6: return STARK_P6; default: return STARK_P7;
  }
}

// r = t - p if t >= p (t < 2p on entry).
__device__ __forceinline__ void fe_reduce_once(fe& t) {
  uint32_t d[8];
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t x = (uint64_t)t.w[i] - p_limb(i) - borrow;
    d[i] = (uint32_t)x;
    borrow = (x >> 32) & 1;
  }
  const bool keep = borrow != 0;  // t < p
#pragma unroll
  for (int i = 0; i < 8; i++) t.w[i] = keep ? t.w[i] : d[i];
}

__device__ __forceinline__ fe fe_add(const fe& a, const fe& b) {
  fe r;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += (uint64_t)a.w[i] + b.w[i];
    r.w[i] = (uint32_t)c;
    c >>= 32;
  }
  fe_reduce_once(r);  // a + b < 2p < 2^255: no carry out of limb 7
  return r;
}

__device__ __forceinline__ fe fe_sub(const fe& a, const fe& b) {
  fe r;
  uint64_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t x = (uint64_t)a.w[i] - b.w[i] - borrow;
    r.w[i] = (uint32_t)x;
    borrow = (x >> 32) & 1;
  }
  const uint32_t mask = 0u - (uint32_t)borrow;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    c += (uint64_t)r.w[i] + (p_limb(i) & mask);
    r.w[i] = (uint32_t)c;
    c >>= 32;
  }
  return r;
}

__device__ __forceinline__ fe fe_neg(const fe& a) {
  fe z;
#pragma unroll
  for (int i = 0; i < 8; i++) z.w[i] = 0;
  return fe_sub(z, a);
}

// acc(64) + carry word c += a * b: one v_mad_u64_u32 whose carry-out is
// counted into c by v_addc_co_u32 (gfx950: ~5 + ~2 cycles per wave64).
__device__ __forceinline__ void fe_mac(uint64_t& acc, uint32_t& c, uint32_t a, uint32_t b) {
  uint64_t cy;
  asm("v_mad_u64_u32 %0, %1, %3, %4, %0\n\t"
      "v_addc_co_u32 %2, %1, %2, 0, %1"
      : "+v"(acc), "=&s"(cy), "+v"(c)
      : "v"(a), "v"(b));
}

// Montgomery product a*b*2^-256 mod p, product scanning with the reduction
// interleaved per column (FIPS order): 64 a*b + 64 m*p word products, each a
// single mad_u64_u32 into a 96-bit column accumulator; no partial-product
// arrays, no carry-propagation chains.  Inputs < p, output < p.
__device__ __forceinline__ fe fe_mul(const fe& a, const fe& b) {
  uint32_t m[8];
  fe r;
  uint64_t acc = 0;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int j = 0; j < k; ++j) {
      fe_mac(acc, c, a.w[j], b.w[k - j]);
      fe_mac(acc, c, m[j], p_limb(k - j));
    }
    fe_mac(acc, c, a.w[k], b.w[0]);
    m[k] = (uint32_t)acc * STARK_PINV32;
    fe_mac(acc, c, m[k], STARK_P0);  // clears the low word
    acc = (acc >> 32) | ((uint64_t)c << 32);
    c = 0;
  }
#pragma unroll
  for (int k = 8; k < 15; ++k) {
#pragma unroll
    for (int j = k - 7; j < 8; ++j) {
      fe_mac(acc, c, a.w[j], b.w[k - j]);
      fe_mac(acc, c, m[j], p_limb(k - j));
    }
    r.w[k - 8] = (uint32_t)acc;
    acc = (acc >> 32) | ((uint64_t)c << 32);
    c = 0;
  }
  r.w[7] = (uint32_t)acc;  // result < 2p < 2^255
  fe_reduce_once(r);
  return r;
}

__device__ __forceinline__ fe fe_zero() {
  fe z;
#pragma unroll
  for (int i = 0; i < 8; i++) z.w[i] = 0;
  return z;
}

__device__ __forceinline__ bool fe_is_zero(const fe& a) {
  uint32_t x = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) x |= a.w[i];
  return x == 0;
}

// Global memory I/O: one element = 32 B = two 16-B vector accesses.
__device__ __forceinline__ fe fe_load(const fe* p) {
  const uint4* q = reinterpret_cast<const uint4*>(p);
  uint4 lo = q[0], hi = q[1];
  fe r;
  r.w[0] = lo.x; r.w[1] = lo.y; r.w[2] = lo.z; r.w[3] = lo.w;
  r.w[4] = hi.x; r.w[5] = hi.y; r.w[6] = hi.z; r.w[7] = hi.w;
  return r;
}
__device__ __forceinline__ void fe_store(fe* p, const fe& v) {
  uint4* q = reinterpret_cast<uint4*>(p);
  q[0] = make_uint4(v.w[0], v.w[1], v.w[2], v.w[3]);
  q[1] = make_uint4(v.w[4], v.w[5], v.w[6], v.w[7]);
}

}  // namespace stark
