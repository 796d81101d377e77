// Blake2s-256 (RFC 7693), unkeyed, 32-byte digest: the `blake2` 0.9.1 crate's
// Blake2s as used by blake() (packages/fri/src/utils.rs:5-10,
// packages/commitment/src/utils.rs:5-10).  One compression function shared by
// host (transcript, verification) and device (Merkle kernels).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace stark {

#define STARK_B2S_IV0 0x6A09E667u
#define STARK_B2S_IV1 0xBB67AE85u
#define STARK_B2S_IV2 0x3C6EF372u
#define STARK_B2S_IV3 0xA54FF53Au
#define STARK_B2S_IV4 0x510E527Fu
#define STARK_B2S_IV5 0x9B05688Cu
#define STARK_B2S_IV6 0x1F83D9ABu
#define STARK_B2S_IV7 0x5BE0CD19u
// h0 of the parameter block: digest 32, key 0, fanout 1, depth 1.
#define STARK_B2S_H0 (STARK_B2S_IV0 ^ 0x01010020u)

__host__ __device__ __forceinline__ uint32_t b2s_rotr(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }

// Message-word schedule of round r, position i (RFC 7693 SIGMA).
__host__ __device__ constexpr int b2s_sigma(int r, int i) {
  constexpr int kSigma[10][16] = {
      {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15},
      {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
      {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4},
      {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
      {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13},
      {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
      {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11},
      {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
      {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5},
      {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};
  return kSigma[r][i];
}

#define STARK_B2S_G(a, b, c, d, x, y)        \
  do {                                       \
    v[a] = v[a] + v[b] + (x);                \
    v[d] = b2s_rotr(v[d] ^ v[a], 16);        \
    v[c] = v[c] + v[d];                      \
    v[b] = b2s_rotr(v[b] ^ v[c], 12);        \
    v[a] = v[a] + v[b] + (y);                \
    v[d] = b2s_rotr(v[d] ^ v[a], 8);         \
    v[c] = v[c] + v[d];                      \
    v[b] = b2s_rotr(v[b] ^ v[c], 7);         \
  } while (0)

// h <- F(h, m, t, last).  m holds 16 little-endian message words.  Fully
// unrolled so the SIGMA schedule becomes static register selection.
__host__ __device__ __forceinline__ void b2s_compress(uint32_t h[8], const uint32_t m[16], uint32_t t_lo,
                                                      uint32_t t_hi, bool last) {
  uint32_t v[16];
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = h[i];
  v[8] = STARK_B2S_IV0; v[9] = STARK_B2S_IV1; v[10] = STARK_B2S_IV2; v[11] = STARK_B2S_IV3;
  v[12] = STARK_B2S_IV4 ^ t_lo;
  v[13] = STARK_B2S_IV5 ^ t_hi;
  v[14] = last ? ~STARK_B2S_IV6 : STARK_B2S_IV6;
  v[15] = STARK_B2S_IV7;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    STARK_B2S_G(0, 4, 8, 12, m[b2s_sigma(r, 0)], m[b2s_sigma(r, 1)]);
    STARK_B2S_G(1, 5, 9, 13, m[b2s_sigma(r, 2)], m[b2s_sigma(r, 3)]);
    STARK_B2S_G(2, 6, 10, 14, m[b2s_sigma(r, 4)], m[b2s_sigma(r, 5)]);
    STARK_B2S_G(3, 7, 11, 15, m[b2s_sigma(r, 6)], m[b2s_sigma(r, 7)]);
    STARK_B2S_G(0, 5, 10, 15, m[b2s_sigma(r, 8)], m[b2s_sigma(r, 9)]);
    STARK_B2S_G(1, 6, 11, 12, m[b2s_sigma(r, 10)], m[b2s_sigma(r, 11)]);
    STARK_B2S_G(2, 7, 8, 13, m[b2s_sigma(r, 12)], m[b2s_sigma(r, 13)]);
    STARK_B2S_G(3, 4, 9, 14, m[b2s_sigma(r, 14)], m[b2s_sigma(r, 15)]);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) h[i] ^= v[i] ^ v[i + 8];
}

__host__ __device__ __forceinline__ void b2s_init(uint32_t h[8]) {
  h[0] = STARK_B2S_H0; h[1] = STARK_B2S_IV1; h[2] = STARK_B2S_IV2; h[3] = STARK_B2S_IV3;
  h[4] = STARK_B2S_IV4; h[5] = STARK_B2S_IV5; h[6] = STARK_B2S_IV6; h[7] = STARK_B2S_IV7;
}

// Host: digest of an arbitrary byte string.
inline void b2s_host(const uint8_t* msg, size_t len, uint8_t out[32]) {
  uint32_t h[8];
  b2s_init(h);
  size_t off = 0;
  uint32_t m[16];
  while (len - off > 64) {
    for (int i = 0; i < 16; ++i)
      m[i] = (uint32_t)msg[off + 4 * i] | ((uint32_t)msg[off + 4 * i + 1] << 8) |
             ((uint32_t)msg[off + 4 * i + 2] << 16) | ((uint32_t)msg[off + 4 * i + 3] << 24);
    off += 64;
    b2s_compress(h, m, (uint32_t)off, (uint32_t)((uint64_t)off >> 32), false);
  }
  uint8_t block[64] = {0};
  for (size_t i = off; i < len; ++i) block[i - off] = msg[i];
  for (int i = 0; i < 16; ++i)
    m[i] = (uint32_t)block[4 * i] | ((uint32_t)block[4 * i + 1] << 8) | ((uint32_t)block[4 * i + 2] << 16) |
           ((uint32_t)block[4 * i + 3] << 24);
  b2s_compress(h, m, (uint32_t)len, (uint32_t)((uint64_t)len >> 32), true);
  for (int i = 0; i < 8; ++i) {
    out[4 * i] = (uint8_t)h[i];
    out[4 * i + 1] = (uint8_t)(h[i] >> 8);
    out[4 * i + 2] = (uint8_t)(h[i] >> 16);
    out[4 * i + 3] = (uint8_t)(h[i] >> 24);
  }
}

}  // namespace stark
