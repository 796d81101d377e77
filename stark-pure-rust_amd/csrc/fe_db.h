// Digit-basis constant product for BN254 Fr on gfx950 VALU.
//
// a * w mod p for a constant w without a quotient product: the constant is
// stored as its eight "digit images" W_i = w * 2^(32 i) mod p, each in nine
// 29-bit limbs, so for a = sum a_i 2^(32 i) (a < 4p + 2^224)
//   S = sum_i a_i W_i = sum_j acc_j 2^(29 j),   acc_j = sum_i a_i W_i[j]
// is congruent to a w and every column sum acc_j fits 64 bits with no carry
// out (8 (2^32 - 1)(2^29 - 1) < 2^64): 72 v_mad_u64_u32, no carry counting.
// S < 8 * 2^32 * p, so q = floor(S / p) < 2^36 comes from the top two columns
// in double precision (underestimated by a margin, so q is exact or one short)
// and r = S - q p = (S + q (2^261 - p)) mod 2^261 lies in [0, 2p): 18 more
// v_mad_u64_u32 and one carry pass over the nine columns.  The Shoup product
// needs 115 word products and ~99 carry counts for the same result range.
//
// Table layout (per constant): 72 u32, W[9 i + j] = limb j of W_i.
#pragma once
#include "fp_dev.h"

namespace stark {

#define STARK_DB_M29 0x1fffffffu
// N = 2^261 - p in 29-bit limbs.
#define STARK_DB_N0 0x0fffffffu
#define STARK_DB_N1 0x00f05360u
#define STARK_DB_N2 0x11a3dbafu
#define STARK_DB_N3 0x182f6f0cu
#define STARK_DB_N4 0x0a7a2d7cu
#define STARK_DB_N5 0x1d24bf3fu
#define STARK_DB_N6 0x1f591ebeu
#define STARK_DB_N7 0x11a3d9cbu
#define STARK_DB_N8 0x1fcf9bb1u

__device__ __forceinline__ uint32_t db_n(int j) {
  switch (j) {
    case 0: return STARK_DB_N0; case 1: return STARK_DB_N1; case 2: return STARK_DB_N2;
    case 3: return STARK_DB_N3; case 4: return STARK_DB_N4; case 5: return STARK_DB_N5;
    case 6: return STARK_DB_N6; case 7: return STARK_DB_N7; default: return STARK_DB_N8;
  }
}

// 2^232 / p and 2^235 / p (nearest doubles) and the quotient margin 2^-12
// (tests/test_fe_db.py checks every constant).
#define STARK_DB_C8 3.153175148504101e-07
#define STARK_DB_C7 2.5225401188032808e-06
#define STARK_DB_MARGIN 2.44140625e-4

// r = a * w mod p in [0, 2p) for a < 4p + 2^224 (the NTT's lazy range: [0, 4p) in the radix-2^8 passes,
// [0, 4p + 2^224) in the radix-2^6 ones, csrc/ntt.hip), W the constant's digit-basis table.
//   acc_j = sum_i a_i W_i[j]: 72 v_mad_u64_u32 into nine 64-bit columns;
//   q: f = acc_8 2^232 / p + hi(acc_7) 2^235 / p - 2^-12 in doubles (the dropped terms are < 2^-15,
//      the rounding < 2^-15, so floor(f) is floor(S / p) or one less), q = qh 2^29 + ql;
//   acc_j += ql N_j + qh N_{j-1} (17 mads; a < 4p + 2^224 bounds a_7 < 2^31.6 + 1, so every column stays below
//      7 2^61 + 2^60.6 + 2^58 < 2^64 with the carry added);
//   one carry pass to 29-bit limbs (mod 2^261) and the repack to 32-bit words.
__device__ __forceinline__ fe fe_mul_db(const fe& a, const uint32_t* __restrict__ W) {
  uint64_t acc[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) acc[j] = (uint64_t)a.w[0] * W[j];
#pragma unroll
  for (int i = 1; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[j] += (uint64_t)a.w[i] * W[9 * i + j];
  const double d8 = fma((double)(uint32_t)(acc[8] >> 32), 0x1p32, (double)(uint32_t)acc[8]);
  const double d7 = (double)(uint32_t)(acc[7] >> 32);
  const double f = fmax(fma(d8, STARK_DB_C8, fma(d7, STARK_DB_C7, -STARK_DB_MARGIN)), 0.0);
  const uint32_t qh = (uint32_t)(f * 0x1p-29);
  const uint32_t ql = (uint32_t)fma((double)qh, -0x1p29, f);
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    acc[j] += (uint64_t)ql * db_n(j);
    if (j) acc[j] += (uint64_t)qh * db_n(j - 1);
  }
  // Carry pass: t_j = acc_j + (t_{j-1} >> 29); limb j is t_j mod 2^29 (the result mod 2^261).  Each output
  // word is one bit-field extract of a limb and one shift-or of the next limb's low word, whose bits
  // above the word are shifted out, so the limbs are never masked separately.
  uint32_t lo[9];
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const uint64_t t = acc[j] + c;
    lo[j] = (uint32_t)t;
    c = t >> 29;
  }
  // (asm: the compiler turns a constant bit-field extract back into a shift and a mask)
  fe o;
  asm("v_bfe_u32 %0, %8, 0, 29\n\t"
      "v_lshl_or_b32 %0, %9, 29, %0\n\t"
      "v_bfe_u32 %1, %9, 3, 26\n\t"
      "v_lshl_or_b32 %1, %10, 26, %1\n\t"
      "v_bfe_u32 %2, %10, 6, 23\n\t"
      "v_lshl_or_b32 %2, %11, 23, %2\n\t"
      "v_bfe_u32 %3, %11, 9, 20\n\t"
      "v_lshl_or_b32 %3, %12, 20, %3\n\t"
      "v_bfe_u32 %4, %12, 12, 17\n\t"
      "v_lshl_or_b32 %4, %13, 17, %4\n\t"
      "v_bfe_u32 %5, %13, 15, 14\n\t"
      "v_lshl_or_b32 %5, %14, 14, %5\n\t"
      "v_bfe_u32 %6, %14, 18, 11\n\t"
      "v_lshl_or_b32 %6, %15, 11, %6\n\t"
      "v_bfe_u32 %7, %15, 21, 8\n\t"
      "v_lshl_or_b32 %7, %16, 8, %7"  // r < 2p < 2^255: limb 8 < 2^23
      : "=&v"(o.w[0]), "=&v"(o.w[1]), "=&v"(o.w[2]), "=&v"(o.w[3]), "=&v"(o.w[4]), "=&v"(o.w[5]), "=&v"(o.w[6]),
        "=&v"(o.w[7])
      : "v"(lo[0]), "v"(lo[1]), "v"(lo[2]), "v"(lo[3]), "v"(lo[4]), "v"(lo[5]), "v"(lo[6]), "v"(lo[7]), "v"(lo[8]));
  return o;
}

}  // namespace stark
