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

// p's limbs as loop-invariant VGPR operands: gfx950's VOP2/VOP3 carry chains
// cannot take a literal or a second SGPR next to the carry (constant-bus
// limit 1), so the modulus lives in VGPRs that the compiler hoists.
struct PLimbs {
  uint32_t l[8];
};
__device__ __forceinline__ PLimbs p_vgprs() {
  PLimbs q;
  q.l[0] = STARK_P0; q.l[1] = STARK_P1; q.l[2] = STARK_P2; q.l[3] = STARK_P3;
  q.l[4] = STARK_P4; q.l[5] = STARK_P5; q.l[6] = STARK_P6; q.l[7] = STARK_P7;
  return q;
}

// t <- t - p if t >= p (t < 2p on entry): one borrow chain + 8 selects.
__device__ __forceinline__ void fe_reduce_once(fe& t) {
  const PLimbs q = p_vgprs();
  uint32_t d0, d1, d2, d3, d4, d5, d6, d7;
  asm("v_sub_co_u32 %8, vcc, %0, %16\n\t"
      "v_subb_co_u32 %9, vcc, %1, %17, vcc\n\t"
      "v_subb_co_u32 %10, vcc, %2, %18, vcc\n\t"
      "v_subb_co_u32 %11, vcc, %3, %19, vcc\n\t"
      "v_subb_co_u32 %12, vcc, %4, %20, vcc\n\t"
      "v_subb_co_u32 %13, vcc, %5, %21, vcc\n\t"
      "v_subb_co_u32 %14, vcc, %6, %22, vcc\n\t"
      "v_subb_co_u32 %15, vcc, %7, %23, vcc\n\t"
      "v_cndmask_b32 %0, %8, %0, vcc\n\t"
      "v_cndmask_b32 %1, %9, %1, vcc\n\t"
      "v_cndmask_b32 %2, %10, %2, vcc\n\t"
      "v_cndmask_b32 %3, %11, %3, vcc\n\t"
      "v_cndmask_b32 %4, %12, %4, vcc\n\t"
      "v_cndmask_b32 %5, %13, %5, vcc\n\t"
      "v_cndmask_b32 %6, %14, %6, vcc\n\t"
      "v_cndmask_b32 %7, %15, %7, vcc"
      : "+v"(t.w[0]), "+v"(t.w[1]), "+v"(t.w[2]), "+v"(t.w[3]), "+v"(t.w[4]), "+v"(t.w[5]), "+v"(t.w[6]),
        "+v"(t.w[7]), "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "=&v"(d4), "=&v"(d5), "=&v"(d6), "=&v"(d7)
      : "v"(q.l[0]), "v"(q.l[1]), "v"(q.l[2]), "v"(q.l[3]), "v"(q.l[4]), "v"(q.l[5]), "v"(q.l[6]), "v"(q.l[7])
      : "vcc");
}

__device__ __forceinline__ fe fe_add(const fe& a, const fe& b) {
  fe r = a;
  asm("v_add_co_u32 %0, vcc, %0, %8\n\t"
      "v_addc_co_u32 %1, vcc, %1, %9, vcc\n\t"
      "v_addc_co_u32 %2, vcc, %2, %10, vcc\n\t"
      "v_addc_co_u32 %3, vcc, %3, %11, vcc\n\t"
      "v_addc_co_u32 %4, vcc, %4, %12, vcc\n\t"
      "v_addc_co_u32 %5, vcc, %5, %13, vcc\n\t"
      "v_addc_co_u32 %6, vcc, %6, %14, vcc\n\t"
      "v_addc_co_u32 %7, vcc, %7, %15, vcc"
      : "+v"(r.w[0]), "+v"(r.w[1]), "+v"(r.w[2]), "+v"(r.w[3]), "+v"(r.w[4]), "+v"(r.w[5]), "+v"(r.w[6]),
        "+v"(r.w[7])
      : "v"(b.w[0]), "v"(b.w[1]), "v"(b.w[2]), "v"(b.w[3]), "v"(b.w[4]), "v"(b.w[5]), "v"(b.w[6]), "v"(b.w[7])
      : "vcc");
  fe_reduce_once(r);  // a + b < 2p < 2^255: no carry out of limb 7
  return r;
}

// a + b without reduction (the caller bounds the sum below 2^256).
__device__ __forceinline__ fe fe_add_raw(const fe& a, const fe& b) {
  fe r = a;
  asm("v_add_co_u32 %0, vcc, %0, %8\n\t"
      "v_addc_co_u32 %1, vcc, %1, %9, vcc\n\t"
      "v_addc_co_u32 %2, vcc, %2, %10, vcc\n\t"
      "v_addc_co_u32 %3, vcc, %3, %11, vcc\n\t"
      "v_addc_co_u32 %4, vcc, %4, %12, vcc\n\t"
      "v_addc_co_u32 %5, vcc, %5, %13, vcc\n\t"
      "v_addc_co_u32 %6, vcc, %6, %14, vcc\n\t"
      "v_addc_co_u32 %7, vcc, %7, %15, vcc"
      : "+v"(r.w[0]), "+v"(r.w[1]), "+v"(r.w[2]), "+v"(r.w[3]), "+v"(r.w[4]), "+v"(r.w[5]), "+v"(r.w[6]),
        "+v"(r.w[7])
      : "v"(b.w[0]), "v"(b.w[1]), "v"(b.w[2]), "v"(b.w[3]), "v"(b.w[4]), "v"(b.w[5]), "v"(b.w[6]), "v"(b.w[7])
      : "vcc");
  return r;
}

__device__ __forceinline__ fe fe_sub(const fe& a, const fe& b) {
  fe r = a;
  uint64_t borrow;
  asm("v_sub_co_u32 %0, vcc, %0, %9\n\t"
      "v_subb_co_u32 %1, vcc, %1, %10, vcc\n\t"
      "v_subb_co_u32 %2, vcc, %2, %11, vcc\n\t"
      "v_subb_co_u32 %3, vcc, %3, %12, vcc\n\t"
      "v_subb_co_u32 %4, vcc, %4, %13, vcc\n\t"
      "v_subb_co_u32 %5, vcc, %5, %14, vcc\n\t"
      "v_subb_co_u32 %6, vcc, %6, %15, vcc\n\t"
      "v_subb_co_u32 %7, %8, %7, %16, vcc"
      : "+v"(r.w[0]), "+v"(r.w[1]), "+v"(r.w[2]), "+v"(r.w[3]), "+v"(r.w[4]), "+v"(r.w[5]), "+v"(r.w[6]),
        "+v"(r.w[7]), "=s"(borrow)
      : "v"(b.w[0]), "v"(b.w[1]), "v"(b.w[2]), "v"(b.w[3]), "v"(b.w[4]), "v"(b.w[5]), "v"(b.w[6]), "v"(b.w[7])
      : "vcc");
  // r += p where the subtraction borrowed.
  const PLimbs q = p_vgprs();
  uint32_t e0, e1, e2, e3, e4, e5, e6, e7;
  asm("v_add_co_u32 %8, vcc, %0, %17\n\t"
      "v_addc_co_u32 %9, vcc, %1, %18, vcc\n\t"
      "v_addc_co_u32 %10, vcc, %2, %19, vcc\n\t"
      "v_addc_co_u32 %11, vcc, %3, %20, vcc\n\t"
      "v_addc_co_u32 %12, vcc, %4, %21, vcc\n\t"
      "v_addc_co_u32 %13, vcc, %5, %22, vcc\n\t"
      "v_addc_co_u32 %14, vcc, %6, %23, vcc\n\t"
      "v_addc_co_u32 %15, vcc, %7, %24, vcc\n\t"
      "v_cndmask_b32_e64 %0, %0, %8, %16\n\t"
      "v_cndmask_b32_e64 %1, %1, %9, %16\n\t"
      "v_cndmask_b32_e64 %2, %2, %10, %16\n\t"
      "v_cndmask_b32_e64 %3, %3, %11, %16\n\t"
      "v_cndmask_b32_e64 %4, %4, %12, %16\n\t"
      "v_cndmask_b32_e64 %5, %5, %13, %16\n\t"
      "v_cndmask_b32_e64 %6, %6, %14, %16\n\t"
      "v_cndmask_b32_e64 %7, %7, %15, %16"
      : "+v"(r.w[0]), "+v"(r.w[1]), "+v"(r.w[2]), "+v"(r.w[3]), "+v"(r.w[4]), "+v"(r.w[5]), "+v"(r.w[6]),
        "+v"(r.w[7]), "=&v"(e0), "=&v"(e1), "=&v"(e2), "=&v"(e3), "=&v"(e4), "=&v"(e5), "=&v"(e6), "=&v"(e7)
      : "s"(borrow), "v"(q.l[0]), "v"(q.l[1]), "v"(q.l[2]), "v"(q.l[3]), "v"(q.l[4]), "v"(q.l[5]), "v"(q.l[6]),
        "v"(q.l[7])
      : "vcc");
  return r;
}

// The Montgomery product as one inline-asm block (fe_mul_lazy, generated by
// tools/gen_fe_mul_asm.py): FIPS product scanning, 64 a*b + 64 m*p word
// products, each one v_mad_u64_u32 into a 96-bit column accumulator whose
// carry-outs v_addc_co_u32 counts.  One block instead of one per product
// removes hipcc's boundary wait state after every block.
#include "fe_mul_asm.inc"

// Montgomery product, canonical result: inputs < p (or a < 4p, b < p).
__device__ __forceinline__ fe fe_mul(const fe& a, const fe& b) {
  fe r = fe_mul_lazy(a, b);
  fe_reduce_once(r);
  return r;
}

// ---- lazy ("Harvey") representation: values in [0, 4p) -------------------
// 4p < 2^256 < 5p for BN254 r, so sums of two values below 2p never carry
// out of limb 7.  The NTT butterflies keep data in [0, 4p) and only the last
// pass reduces to canonical.
#define STARK_2P0 0xe0000002u
#define STARK_2P1 0x87c3eb27u
#define STARK_2P2 0xf372e122u
#define STARK_2P3 0x5067d090u
#define STARK_2P4 0x0302b0bau
#define STARK_2P5 0x70a08b6du
#define STARK_2P6 0xc2634053u
#define STARK_2P7 0x60c89ce5u

struct P2Limbs {
  uint32_t l[8];
};
__device__ __forceinline__ P2Limbs p2_vgprs() {
  P2Limbs q;
  q.l[0] = STARK_2P0; q.l[1] = STARK_2P1; q.l[2] = STARK_2P2; q.l[3] = STARK_2P3;
  q.l[4] = STARK_2P4; q.l[5] = STARK_2P5; q.l[6] = STARK_2P6; q.l[7] = STARK_2P7;
  return q;
}

// x <- x - 2p if x >= 2p (x < 4p on entry, < 2p on exit).
__device__ __forceinline__ void fe_csub2p(fe& t) {
  const P2Limbs q = p2_vgprs();
  uint32_t d0, d1, d2, d3, d4, d5, d6, d7;
  asm("v_sub_co_u32 %8, vcc, %0, %16\n\t"
      "v_subb_co_u32 %9, vcc, %1, %17, vcc\n\t"
      "v_subb_co_u32 %10, vcc, %2, %18, vcc\n\t"
      "v_subb_co_u32 %11, vcc, %3, %19, vcc\n\t"
      "v_subb_co_u32 %12, vcc, %4, %20, vcc\n\t"
      "v_subb_co_u32 %13, vcc, %5, %21, vcc\n\t"
      "v_subb_co_u32 %14, vcc, %6, %22, vcc\n\t"
      "v_subb_co_u32 %15, vcc, %7, %23, vcc\n\t"
      "v_cndmask_b32 %0, %8, %0, vcc\n\t"
      "v_cndmask_b32 %1, %9, %1, vcc\n\t"
      "v_cndmask_b32 %2, %10, %2, vcc\n\t"
      "v_cndmask_b32 %3, %11, %3, vcc\n\t"
      "v_cndmask_b32 %4, %12, %4, vcc\n\t"
      "v_cndmask_b32 %5, %13, %5, vcc\n\t"
      "v_cndmask_b32 %6, %14, %6, vcc\n\t"
      "v_cndmask_b32 %7, %15, %7, vcc"
      : "+v"(t.w[0]), "+v"(t.w[1]), "+v"(t.w[2]), "+v"(t.w[3]), "+v"(t.w[4]), "+v"(t.w[5]), "+v"(t.w[6]),
        "+v"(t.w[7]), "=&v"(d0), "=&v"(d1), "=&v"(d2), "=&v"(d3), "=&v"(d4), "=&v"(d5), "=&v"(d6), "=&v"(d7)
      : "v"(q.l[0]), "v"(q.l[1]), "v"(q.l[2]), "v"(q.l[3]), "v"(q.l[4]), "v"(q.l[5]), "v"(q.l[6]), "v"(q.l[7])
      : "vcc");
}

// Radix-2 butterfly in the lazy representation (Harvey):
//   X in [0, 4p), T in [0, 2p)  ->  X' = X mod 2p in [0, 2p),
//   x <- X' + T in [0, 4p),  y <- X' - T + 2p in (0, 4p).
__device__ __forceinline__ void fe_bfly_lazy_reduced(fe& x, fe& y, const fe& t);
__device__ __forceinline__ void fe_bfly_lazy(fe& x, fe& y, const fe& t) {
  fe_csub2p(x);
  fe_bfly_lazy_reduced(x, y, t);
}
// The same for X already in [0, 2p).
__device__ __forceinline__ void fe_bfly_lazy_reduced(fe& x, fe& y, const fe& t) {
  const P2Limbs q = p2_vgprs();
  // s = X' + T and d = (X' + 2p) - T written to fresh registers (an in-place form would copy X'
  // into both first: 16 v_mov_b32 per butterfly).  X' + 2p < 4p < 2^256 and >= T, so neither
  // chain carries out.
  fe s, d;
  asm("v_add_co_u32 %0, vcc, %16, %24\n\t"
      "v_addc_co_u32 %1, vcc, %17, %25, vcc\n\t"
      "v_addc_co_u32 %2, vcc, %18, %26, vcc\n\t"
      "v_addc_co_u32 %3, vcc, %19, %27, vcc\n\t"
      "v_addc_co_u32 %4, vcc, %20, %28, vcc\n\t"
      "v_addc_co_u32 %5, vcc, %21, %29, vcc\n\t"
      "v_addc_co_u32 %6, vcc, %22, %30, vcc\n\t"
      "v_addc_co_u32 %7, vcc, %23, %31, vcc\n\t"
      "v_add_co_u32 %8, vcc, %16, %32\n\t"
      "v_addc_co_u32 %9, vcc, %17, %33, vcc\n\t"
      "v_addc_co_u32 %10, vcc, %18, %34, vcc\n\t"
      "v_addc_co_u32 %11, vcc, %19, %35, vcc\n\t"
      "v_addc_co_u32 %12, vcc, %20, %36, vcc\n\t"
      "v_addc_co_u32 %13, vcc, %21, %37, vcc\n\t"
      "v_addc_co_u32 %14, vcc, %22, %38, vcc\n\t"
      "v_addc_co_u32 %15, vcc, %23, %39, vcc\n\t"
      "v_sub_co_u32 %8, vcc, %8, %24\n\t"
      "v_subb_co_u32 %9, vcc, %9, %25, vcc\n\t"
      "v_subb_co_u32 %10, vcc, %10, %26, vcc\n\t"
      "v_subb_co_u32 %11, vcc, %11, %27, vcc\n\t"
      "v_subb_co_u32 %12, vcc, %12, %28, vcc\n\t"
      "v_subb_co_u32 %13, vcc, %13, %29, vcc\n\t"
      "v_subb_co_u32 %14, vcc, %14, %30, vcc\n\t"
      "v_subb_co_u32 %15, vcc, %15, %31, vcc"
      : "=&v"(s.w[0]), "=&v"(s.w[1]), "=&v"(s.w[2]), "=&v"(s.w[3]), "=&v"(s.w[4]), "=&v"(s.w[5]), "=&v"(s.w[6]),
        "=&v"(s.w[7]), "=&v"(d.w[0]), "=&v"(d.w[1]), "=&v"(d.w[2]), "=&v"(d.w[3]), "=&v"(d.w[4]), "=&v"(d.w[5]),
        "=&v"(d.w[6]), "=&v"(d.w[7])
      : "v"(x.w[0]), "v"(x.w[1]), "v"(x.w[2]), "v"(x.w[3]), "v"(x.w[4]), "v"(x.w[5]), "v"(x.w[6]), "v"(x.w[7]),
        "v"(t.w[0]), "v"(t.w[1]), "v"(t.w[2]), "v"(t.w[3]), "v"(t.w[4]), "v"(t.w[5]), "v"(t.w[6]), "v"(t.w[7]),
        "v"(q.l[0]), "v"(q.l[1]), "v"(q.l[2]), "v"(q.l[3]), "v"(q.l[4]), "v"(q.l[5]), "v"(q.l[6]), "v"(q.l[7])
      : "vcc");
  x = s;
  y = d;
}

// [0, 4p) -> canonical [0, p).
__device__ __forceinline__ void fe_reduce_lazy(fe& t) {
  fe_csub2p(t);
  fe_reduce_once(t);
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
