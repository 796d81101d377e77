/*
 * oracle.c -- CPU restatement of the stark-pure-rust FRI-prover hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the
 * cpu_baseline leg of bench.py.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline may load liboracle.so; the product library
 * (libstark_hip.so) never links or calls it.
 *
 * Every function restates the reference algorithm *as written* (same loop
 * structure, same thread fan-out) and cites the reference file:line it
 * follows (paths relative to the reference repo root, packages/...).
 *
 * Parity pinning: see tests/test_oracle_kat.py -- Blake2s KATs
 * (fri/src/utils.rs:12-24), pseudorandom-index KATs (fri/src/utils.rs:111-120),
 * Merkle root/path KATs (commitment/src/pallarel_merkle_tree.rs:132-216),
 * Fp codec (ff_utils/src/fp.rs:27-68), multi_inv zero semantics
 * (fri/src/poly_utils.rs:72-91, checked over F7 by the Python restatement),
 * NTT against the DFT definition (naive O(n^2) sum, exact integers).
 *
 * Third-party algorithms restated (absent from /root/reference, pinned in
 * the reference's Cargo.lock): ff 0.10.0 / ff_derive 0.10.0 (Montgomery
 * arithmetic over BN254 Fr, R = 2^256; from_str = decimal reduced mod p),
 * blake2 0.9.1 (Blake2s-256 unkeyed, RFC 7693).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <stdio.h>
#include <pthread.h>

#include "oracle_internal.h"

typedef unsigned __int128 u128;

/* BN254 scalar field r (ff_utils/src/fp.rs:9), little-endian u64 limbs. */
static const uint64_t P[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull,
                              0xb85045b68181585dull, 0x30644e72e131a029ull};
static uint64_t PINV;      /* -p^{-1} mod 2^64 */
static fp R2;              /* R^2 mod p (canonical limbs) */
static fp ONE;             /* R mod p */
static int g_init = 0;

static int geq_p(const uint64_t a[4]) {
  for (int i = 3; i >= 0; i--) {
    if (a[i] > P[i]) return 1;
    if (a[i] < P[i]) return 0;
  }
  return 1;
}
static void sub_p(uint64_t a[4]) {
  u128 borrow = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a[i] - P[i] - borrow;
    a[i] = (uint64_t)d;
    borrow = (d >> 64) ? 1 : 0;
  }
}

fp fp_add(fp a, fp b) {
  fp r; u128 c = 0;
  for (int i = 0; i < 4; i++) { c += (u128)a.v[i] + b.v[i]; r.v[i] = (uint64_t)c; c >>= 64; }
  if (c || geq_p(r.v)) sub_p(r.v);
  return r;
}
fp fp_sub(fp a, fp b) {
  fp r; u128 borrow = 0;
  for (int i = 0; i < 4; i++) {
    u128 d = (u128)a.v[i] - b.v[i] - borrow;
    r.v[i] = (uint64_t)d; borrow = (d >> 64) ? 1 : 0;
  }
  if (borrow) { u128 c = 0; for (int i = 0; i < 4; i++) { c += (u128)r.v[i] + P[i]; r.v[i] = (uint64_t)c; c >>= 64; } }
  return r;
}
/* CIOS Montgomery multiplication: a*b*R^{-1} mod p (ff_derive mul_assign). */
fp fp_mul(fp a, fp b) {
  uint64_t t[6] = {0};
  for (int i = 0; i < 4; i++) {
    u128 c = 0;
    for (int j = 0; j < 4; j++) { c += (u128)a.v[j] * b.v[i] + t[j]; t[j] = (uint64_t)c; c >>= 64; }
    c += t[4]; t[4] = (uint64_t)c; t[5] = (uint64_t)(c >> 64);
    uint64_t m = t[0] * PINV;
    c = (u128)m * P[0] + t[0]; c >>= 64;
    for (int j = 1; j < 4; j++) { c += (u128)m * P[j] + t[j]; t[j - 1] = (uint64_t)c; c >>= 64; }
    c += t[4]; t[3] = (uint64_t)c; t[4] = t[5] + (uint64_t)(c >> 64);
  }
  fp r; memcpy(r.v, t, 32);
  if (t[4] || geq_p(r.v)) sub_p(r.v);
  return r;
}
int fp_eq(fp a, fp b) { return memcmp(a.v, b.v, 32) == 0; }
int fp_is_zero(fp a) { return (a.v[0] | a.v[1] | a.v[2] | a.v[3]) == 0; }

void or_init(void) {
  if (g_init) return;
  uint64_t x = 1; /* Newton iteration for p^{-1} mod 2^64 */
  for (int i = 0; i < 7; i++) x *= 2 - P[0] * x;
  PINV = (uint64_t)(0 - x);
  /* R mod p: 2^256 mod p by doubling 1 256 times; R^2 by doubling 512 times. */
  fp r = {{1, 0, 0, 0}};
  for (int i = 0; i < 512; i++) {
    r = fp_add(r, r);
    if (i == 255) ONE = r;
  }
  R2 = r;
  g_init = 1;
}

/* Canonical little-endian u64[4] <-> Montgomery. Values >= p are reduced
 * (ff from_str semantics used by from_bytes_le, ff_utils/src/fp.rs:70-77). */
fp fp_from_canon(const uint64_t c[4]) {
  fp a; memcpy(a.v, c, 32);
  while (geq_p(a.v)) sub_p(a.v);
  return fp_mul(a, R2);
}
void fp_to_canon(fp a, uint64_t c[4]) {
  fp one = {{1, 0, 0, 0}};
  fp r = fp_mul(a, one);
  memcpy(c, r.v, 32);
}
fp fp_from_u64(uint64_t v) { uint64_t c[4] = {v, 0, 0, 0}; return fp_from_canon(c); }
fp fp_one(void) { return ONE; }
fp fp_zero(void) { fp z = {{0, 0, 0, 0}}; return z; }
/* pow_vartime with a u64-limb exponent, LE limbs (ff Field::pow_vartime). */
fp fp_pow_limbs(fp a, const uint64_t* e, int nlimbs) {
  fp r = ONE;
  for (int i = nlimbs - 1; i >= 0; i--)
    for (int b = 63; b >= 0; b--) {
      r = fp_mul(r, r);
      if ((e[i] >> b) & 1) r = fp_mul(r, a);
    }
  return r;
}
fp fp_pow(fp a, uint64_t e) { return fp_pow_limbs(a, &e, 1); }
fp fp_inv(fp a) { /* invert via Fermat: a^(p-2) */
  uint64_t e[4]; memcpy(e, P, 32); e[0] -= 2;
  return fp_pow_limbs(a, e, 4);
}

/* ------------------------------------------------------------------ */
/* fri/src/fft.rs                                                       */
/* ------------------------------------------------------------------ */

/* expand_root_of_unity, fft.rs:5-14. Returns count; out may be NULL. */
size_t or_expand_root_of_unity(fp root, fp* out, size_t cap) {
  size_t k = 0;
  fp cur = root;
  if (out && k < cap) out[k] = ONE;
  k++;
  while (!fp_eq(cur, ONE)) {
    if (out && k < cap) out[k] = cur;
    k++;
    cur = fp_mul(cur, root);
  }
  return k;
}

static uint32_t bit_reverse(uint32_t n, uint32_t l) {
  uint32_t r = 0;
  for (uint32_t i = 0; i < l; i++) { r = (r << 1) | (n & 1); n >>= 1; }
  return r;
}

/* serial_fft, fft.rs:150-193 (bit-reverse, then log n DIT stages with a
 * running twiddle w *= w_m). */
void or_serial_fft(fp* values, fp root, uint32_t log_n) {
  uint32_t n = 1u << log_n;
  for (uint32_t k = 0; k < n; k++) {
    uint32_t rk = bit_reverse(k, log_n);
    if (k < rk) { fp t = values[rk]; values[rk] = values[k]; values[k] = t; }
  }
  uint32_t m = 1;
  for (uint32_t s = 0; s < log_n; s++) {
    fp w_m = fp_pow(root, n / (2 * m));
    for (uint32_t k = 0; k < n; k += 2 * m) {
      fp w = ONE;
      for (uint32_t j = 0; j < m; j++) {
        fp t = fp_mul(values[k + j + m], w);
        fp tmp = fp_sub(values[k + j], t);
        values[k + j + m] = tmp;
        values[k + j] = fp_add(values[k + j], t);
        w = fp_mul(w, w_m);
      }
    }
    m *= 2;
  }
}

typedef struct {
  const fp* values; fp* tmp; fp root; uint32_t j, log_new_n, log_n, num_cpus;
} pfft_job;

static void* pfft_worker(void* arg) {
  pfft_job* jb = (pfft_job*)arg;
  /* fft.rs:213-233 */
  fp omega_j = fp_pow(jb->root, jb->j);
  fp omega_step = fp_pow(jb->root, (uint64_t)jb->j << jb->log_new_n);
  fp elt = ONE;
  uint32_t new_n = 1u << jb->log_new_n, n = 1u << jb->log_n;
  for (uint32_t i = 0; i < new_n; i++) {
    for (uint32_t s = 0; s < jb->num_cpus; s++) {
      uint32_t idx = (i + (s << jb->log_new_n)) % n;
      fp t = fp_mul(jb->values[idx], elt);
      jb->tmp[i] = fp_add(jb->tmp[i], t);
      elt = fp_mul(elt, omega_step);
    }
    elt = fp_mul(elt, omega_j);
  }
  fp new_omega = fp_pow(jb->root, jb->num_cpus);
  or_serial_fft(jb->tmp, new_omega, jb->log_new_n);
  return NULL;
}

/* parallel_fft, fft.rs:195-251 (bellman split into 2^log_cpus sub-DFTs, one
 * thread each, then the strided gather). */
void or_parallel_fft(fp* values, fp root, uint32_t log_n, uint32_t log_cpus) {
  if (log_cpus > log_n) abort(); /* fft.rs:202 assert */
  uint32_t num_cpus = 1u << log_cpus, log_new_n = log_n - log_cpus;
  size_t new_n = (size_t)1 << log_new_n;
  fp* tmp = (fp*)calloc((size_t)num_cpus * new_n, sizeof(fp));
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * num_cpus);
  pfft_job* jobs = (pfft_job*)malloc(sizeof(pfft_job) * num_cpus);
  for (uint32_t j = 0; j < num_cpus; j++) {
    jobs[j] = (pfft_job){values, tmp + (size_t)j * new_n, root, j, log_new_n, log_n, num_cpus};
    pthread_create(&th[j], NULL, pfft_worker, &jobs[j]);
  }
  for (uint32_t j = 0; j < num_cpus; j++) pthread_join(th[j], NULL);
  uint32_t mask = num_cpus - 1;
  size_t n = (size_t)1 << log_n;
  for (size_t idx = 0; idx < n; idx++) values[idx] = tmp[(idx & mask) * new_n + (idx >> log_cpus)];
  free(tmp); free(th); free(jobs);
}

static uint32_t log2_floor(uint32_t x) { uint32_t r = 0; while ((1u << (r + 1)) <= x) r++; return r; }

/* best_fft, fft.rs:327-357: zero-pad to 2^log_n, serial when cpus == 1 or
 * n <= cpus, else parallel_fft with log2_floor(cpus) (multicore.rs:47-49). */
void or_best_fft_mont(fp* values /* cap 2^log_n, first len filled */, size_t len, fp root,
                      uint32_t log_n, uint32_t cpus) {
  size_t n = (size_t)1 << log_n;
  for (size_t i = len; i < n; i++) values[i] = fp_zero();
  if (cpus == 1 || n <= cpus) or_serial_fft(values, root, log_n);
  else or_parallel_fft(values, root, log_n, log2_floor(cpus));
}

/* inv_serial_fft / inv_parallel_fft, fft.rs:284-309 and inv_best_fft
 * fft.rs:359-379: transform with root^{-1}, then multiply by n^{-1}. */
void or_inv_best_fft_mont(fp* values, size_t len, fp root, uint32_t log_n, uint32_t cpus) {
  size_t n = (size_t)1 << log_n;
  for (size_t i = len; i < n; i++) values[i] = fp_zero();
  fp inv_len = fp_inv(fp_from_u64(n));
  fp inv_root = fp_inv(root);
  if (cpus == 1 || n <= cpus) or_serial_fft(values, inv_root, log_n);
  else or_parallel_fft(values, inv_root, log_n, log2_floor(cpus));
  for (size_t i = 0; i < n; i++) values[i] = fp_mul(values[i], inv_len);
}

/* ------------------------------------------------------------------ */
/* Canonical-limb entry points used by the Python tests / bench.       */
/* Elements cross this boundary as canonical LE u64[4] (= to_bytes_le).*/
/* ------------------------------------------------------------------ */
fp* or_load(const uint64_t* c, size_t len, size_t cap) {
  fp* v = (fp*)malloc(sizeof(fp) * (cap ? cap : 1));
  for (size_t i = 0; i < len; i++) v[i] = fp_from_canon(c + 4 * i);
  return v;
}
void or_store(const fp* v, uint64_t* c, size_t len) {
  for (size_t i = 0; i < len; i++) fp_to_canon(v[i], c + 4 * i);
}

/* out must hold 4*2^log_n u64.  Returns 0 on success, -1 on bad length. */
int oracle_best_fft(const uint64_t* in, size_t len, const uint64_t root[4], uint32_t log_n,
                    uint32_t cpus, uint64_t* out) {
  or_init();
  size_t n = (size_t)1 << log_n;
  if (len > n) return -1;
  fp* v = or_load(in, len, n);
  or_best_fft_mont(v, len, fp_from_canon(root), log_n, cpus);
  or_store(v, out, n); free(v);
  return 0;
}
int oracle_inv_best_fft(const uint64_t* in, size_t len, const uint64_t root[4], uint32_t log_n,
                        uint32_t cpus, uint64_t* out) {
  or_init();
  size_t n = (size_t)1 << log_n;
  if (len > n) return -1;
  fp* v = or_load(in, len, n);
  or_inv_best_fft_mont(v, len, fp_from_canon(root), log_n, cpus);
  or_store(v, out, n); free(v);
  return 0;
}
/* Returns the number of powers; writes min(count, cap) of them. */
size_t oracle_expand_root_of_unity(const uint64_t root[4], uint64_t* out, size_t cap) {
  or_init();
  size_t cnt = or_expand_root_of_unity(fp_from_canon(root), NULL, 0);
  if (out) {
    fp* v = (fp*)malloc(sizeof(fp) * cnt);
    or_expand_root_of_unity(fp_from_canon(root), v, cnt);
    or_store(v, out, cnt < cap ? cnt : cap); free(v);
  }
  return cnt;
}
/* 7^((p-1)/2^log_n): the NTT root the prover builds (r1cs-stark/src/prove.rs:71-82). */
void oracle_root_of_unity(uint32_t log_n, uint64_t out[4]) {
  or_init();
  uint64_t e[4]; memcpy(e, P, 32); e[0] -= 1; /* p - 1 */
  for (uint32_t i = 0; i < log_n; i++) { /* shift right by log_n */
    e[0] = (e[0] >> 1) | (e[1] << 63); e[1] = (e[1] >> 1) | (e[2] << 63);
    e[2] = (e[2] >> 1) | (e[3] << 63); e[3] >>= 1;
  }
  fp g = fp_pow_limbs(fp_from_u64(7), e, 4);
  fp_to_canon(g, out);
}
void oracle_fp_mul(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]) {
  or_init(); fp_to_canon(fp_mul(fp_from_canon(a), fp_from_canon(b)), out);
}
void oracle_fp_inv(const uint64_t a[4], uint64_t out[4]) {
  or_init(); fp_to_canon(fp_inv(fp_from_canon(a)), out);
}
void oracle_fp_pow(const uint64_t a[4], uint64_t e, uint64_t out[4]) {
  or_init(); fp_to_canon(fp_pow(fp_from_canon(a), e), out);
}
/* from_bytes_le (ff_utils/src/fp.rs:74-76): LE integer of up to 32 bytes mod p. */
void oracle_from_bytes_le(const uint8_t* b, size_t len, uint64_t out[4]) {
  or_init();
  uint64_t c[4] = {0, 0, 0, 0};
  for (size_t i = 0; i < len && i < 32; i++) c[i / 8] |= (uint64_t)b[i] << (8 * (i % 8));
  fp_to_canon(fp_from_canon(c), out);
}

/* ------------------------------------------------------------------ */
/* fri/src/poly_utils.rs                                                */
/* ------------------------------------------------------------------ */

/* multi_inv, poly_utils.rs:38-70 (zero maps to zero). */
void or_multi_inv(const fp* values, fp* outputs, size_t n) {
  fp* partials = (fp*)malloc(sizeof(fp) * (n + 1));
  partials[0] = ONE;
  for (size_t i = 0; i < n; i++)
    partials[i + 1] = fp_mul(partials[i], fp_is_zero(values[i]) ? ONE : values[i]);
  fp inv = fp_inv(partials[n]);
  for (size_t i = n; i-- > 0;) {
    outputs[i] = fp_is_zero(values[i]) ? fp_zero() : fp_mul(partials[i], inv);
    inv = fp_mul(inv, fp_is_zero(values[i]) ? ONE : values[i]);
  }
  free(partials);
}
void oracle_multi_inv(const uint64_t* in, size_t n, uint64_t* out) {
  or_init();
  fp* v = or_load(in, n, n); fp* o = (fp*)malloc(sizeof(fp) * (n ? n : 1));
  or_multi_inv(v, o, n); or_store(o, out, n); free(v); free(o);
}

/* eval_poly_at, poly_utils.rs:93-102 (Horner-free power accumulation). */
fp or_eval_poly_at(const fp* poly, size_t deg1, fp x) {
  fp y = fp_zero(), pw = ONE;
  for (size_t i = 0; i < deg1; i++) { y = fp_add(y, fp_mul(pw, poly[i])); pw = fp_mul(pw, x); }
  return y;
}
void oracle_eval_poly_multi(const uint64_t* poly, size_t deg1, const uint64_t* xs, size_t n,
                            uint64_t* out) {
  or_init();
  fp* p = or_load(poly, deg1, deg1);
  for (size_t i = 0; i < n; i++) fp_to_canon(or_eval_poly_at(p, deg1, fp_from_canon(xs + 4 * i)), out + 4 * i);
  free(p);
}

/* eval_quartic, poly_utils.rs:442-446 */
static fp eval_quartic(const fp p[4], fp x) {
  fp xsq = fp_mul(x, x), xcb = fp_mul(xsq, x);
  return fp_add(fp_add(fp_add(p[0], fp_mul(p[1], x)), fp_mul(p[2], xsq)), fp_mul(p[3], xcb));
}
/* multi_interp_4, poly_utils.rs:449-511 */
void or_multi_interp_4(const fp (*xsets)[4], const fp (*ysets)[4], fp (*out)[4], size_t rows) {
  fp (*eqs)[4][4] = malloc(sizeof(fp) * 16 * (rows ? rows : 1));
  fp* inv_targets = (fp*)malloc(sizeof(fp) * 4 * (rows ? rows : 1));
  fp* inv_alls = (fp*)malloc(sizeof(fp) * 4 * (rows ? rows : 1));
  fp zero = fp_zero();
  for (size_t key = 0; key < rows; key++) {
    const fp* xs = xsets[key];
    fp x01 = fp_mul(xs[0], xs[1]), x02 = fp_mul(xs[0], xs[2]), x03 = fp_mul(xs[0], xs[3]);
    fp x12 = fp_mul(xs[1], xs[2]), x13 = fp_mul(xs[1], xs[3]), x23 = fp_mul(xs[2], xs[3]);
    fp (*e)[4] = eqs[key];
    e[0][0] = fp_sub(zero, fp_mul(x12, xs[3])); e[0][1] = fp_add(fp_add(x12, x13), x23);
    e[0][2] = fp_sub(fp_sub(fp_sub(zero, xs[1]), xs[2]), xs[3]); e[0][3] = ONE;
    e[1][0] = fp_sub(zero, fp_mul(x02, xs[3])); e[1][1] = fp_add(fp_add(x02, x03), x23);
    e[1][2] = fp_sub(fp_sub(fp_sub(zero, xs[0]), xs[2]), xs[3]); e[1][3] = ONE;
    e[2][0] = fp_sub(zero, fp_mul(x01, xs[3])); e[2][1] = fp_add(fp_add(x01, x03), x13);
    e[2][2] = fp_sub(fp_sub(fp_sub(zero, xs[0]), xs[1]), xs[3]); e[2][3] = ONE;
    e[3][0] = fp_sub(zero, fp_mul(x01, xs[2])); e[3][1] = fp_add(fp_add(x01, x02), x12);
    e[3][2] = fp_sub(fp_sub(fp_sub(zero, xs[0]), xs[1]), xs[2]); e[3][3] = ONE;
    for (int j = 0; j < 4; j++) inv_targets[4 * key + j] = eval_quartic(e[j], xs[j]);
  }
  or_multi_inv(inv_targets, inv_alls, 4 * rows);
  for (size_t i = 0; i < rows; i++) {
    fp inv_y[4];
    for (int j = 0; j < 4; j++) inv_y[j] = fp_mul(ysets[i][j], inv_alls[4 * i + j]);
    for (int k = 0; k < 4; k++) {
      fp acc = fp_mul(eqs[i][0][k], inv_y[0]);
      for (int j = 1; j < 4; j++) acc = fp_add(acc, fp_mul(eqs[i][j][k], inv_y[j]));
      out[i][k] = acc;
    }
  }
  free(eqs); free(inv_targets); free(inv_alls);
}

/* Canonical-limb entry points of multi_interp_4 and eval_quartic (one quartic per x). */
void oracle_multi_interp_4(const uint64_t* xsets, const uint64_t* ysets, size_t rows, uint64_t* out) {
  or_init();
  fp* x = or_load(xsets, 4 * rows, 4 * rows);
  fp* y = or_load(ysets, 4 * rows, 4 * rows);
  fp* o = (fp*)malloc(sizeof(fp) * 4 * (rows ? rows : 1));
  or_multi_interp_4((const fp (*)[4])x, (const fp (*)[4])y, (fp (*)[4])o, rows);
  or_store(o, out, 4 * rows);
  free(x); free(y); free(o);
}

void oracle_eval_quartic_multi(const uint64_t* polys, const uint64_t* xs, size_t n, uint64_t* out) {
  or_init();
  fp* p = or_load(polys, 4 * n, 4 * n);
  fp* x = or_load(xs, n, n);
  for (size_t i = 0; i < n; i++) x[i] = eval_quartic(p + 4 * i, x[i]);
  or_store(x, out, n);
  free(p); free(x);
}

/* ------------------------------------------------------------------ */
/* Blake2s-256 (blake2 0.9.1; RFC 7693), used by fri/src/utils.rs:5-10   */
/* and commitment/src/utils.rs:5-10.                                   */
/* ------------------------------------------------------------------ */
static const uint32_t B2S_IV[8] = {0x6A09E667, 0xBB67AE85, 0x3C6EF372, 0xA54FF53A,
                                   0x510E527F, 0x9B05688C, 0x1F83D9AB, 0x5BE0CD19};
static const uint8_t B2S_SIGMA[10][16] = {
    {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15}, {14, 10, 4, 8, 9, 15, 13, 6, 1, 12, 0, 2, 11, 7, 5, 3},
    {11, 8, 12, 0, 5, 2, 15, 13, 10, 14, 3, 6, 7, 1, 9, 4}, {7, 9, 3, 1, 13, 12, 11, 14, 2, 6, 5, 10, 4, 0, 15, 8},
    {9, 0, 5, 7, 2, 4, 10, 15, 14, 1, 11, 12, 6, 8, 3, 13}, {2, 12, 6, 10, 0, 11, 8, 3, 4, 13, 7, 5, 15, 14, 1, 9},
    {12, 5, 1, 15, 14, 13, 4, 10, 0, 7, 6, 3, 9, 2, 8, 11}, {13, 11, 7, 14, 12, 1, 3, 9, 5, 0, 15, 4, 8, 6, 2, 10},
    {6, 15, 14, 9, 11, 3, 0, 8, 12, 2, 13, 7, 1, 4, 10, 5}, {10, 2, 8, 4, 7, 6, 1, 5, 15, 11, 9, 14, 3, 12, 13, 0}};
static uint32_t rotr32(uint32_t x, int n) { return (x >> n) | (x << (32 - n)); }
static void b2s_compress(uint32_t h[8], const uint8_t block[64], uint64_t t, int last) {
  uint32_t m[16], v[16];
  for (int i = 0; i < 16; i++)
    m[i] = (uint32_t)block[4 * i] | ((uint32_t)block[4 * i + 1] << 8) | ((uint32_t)block[4 * i + 2] << 16) |
           ((uint32_t)block[4 * i + 3] << 24);
  for (int i = 0; i < 8; i++) { v[i] = h[i]; v[i + 8] = B2S_IV[i]; }
  v[12] ^= (uint32_t)t; v[13] ^= (uint32_t)(t >> 32);
  if (last) v[14] = ~v[14];
#define G(a, b, c, d, x, y)                                  \
  do {                                                       \
    v[a] = v[a] + v[b] + x; v[d] = rotr32(v[d] ^ v[a], 16);  \
    v[c] = v[c] + v[d];     v[b] = rotr32(v[b] ^ v[c], 12);  \
    v[a] = v[a] + v[b] + y; v[d] = rotr32(v[d] ^ v[a], 8);   \
    v[c] = v[c] + v[d];     v[b] = rotr32(v[b] ^ v[c], 7);   \
  } while (0)
  for (int r = 0; r < 10; r++) {
    const uint8_t* s = B2S_SIGMA[r];
    G(0, 4, 8, 12, m[s[0]], m[s[1]]); G(1, 5, 9, 13, m[s[2]], m[s[3]]);
    G(2, 6, 10, 14, m[s[4]], m[s[5]]); G(3, 7, 11, 15, m[s[6]], m[s[7]]);
    G(0, 5, 10, 15, m[s[8]], m[s[9]]); G(1, 6, 11, 12, m[s[10]], m[s[11]]);
    G(2, 7, 8, 13, m[s[12]], m[s[13]]); G(3, 4, 9, 14, m[s[14]], m[s[15]]);
  }
#undef G
  for (int i = 0; i < 8; i++) h[i] ^= v[i] ^ v[i + 8];
}
void oracle_blake2s(const uint8_t* msg, size_t len, uint8_t out[32]) {
  uint32_t h[8];
  memcpy(h, B2S_IV, sizeof h);
  h[0] ^= 0x01010000u ^ 32u; /* digest length 32, no key, fanout 1, depth 1 */
  uint8_t block[64];
  size_t off = 0;
  while (len - off > 64) { b2s_compress(h, msg + off, off + 64, 0); off += 64; }
  memset(block, 0, 64);
  memcpy(block, msg + off, len - off);
  b2s_compress(h, block, len, 1);
  for (int i = 0; i < 8; i++) {
    out[4 * i] = (uint8_t)h[i]; out[4 * i + 1] = (uint8_t)(h[i] >> 8);
    out[4 * i + 2] = (uint8_t)(h[i] >> 16); out[4 * i + 3] = (uint8_t)(h[i] >> 24);
  }
}

/* ------------------------------------------------------------------ */
/* fri/src/utils.rs:82-109 get_pseudorandom_indices                     */
/* ------------------------------------------------------------------ */
int oracle_get_pseudorandom_indices(const uint8_t* seed, size_t seed_len, uint32_t modulus,
                                    size_t count, uint32_t exclude, uint32_t* out) {
  if (modulus >= (1u << 24)) return -1; /* utils.rs:88 assert */
  if (seed_len < 32 && seed_len < 4 * count) return -2; /* data[len-32..] would panic */
  size_t cap = seed_len + 4 * count + 64;
  uint8_t* data = (uint8_t*)malloc(cap);
  memcpy(data, seed, seed_len);
  size_t len = seed_len;
  while (len < 4 * count) { oracle_blake2s(data + len - 32, 32, data + len); len += 32; }
  if (exclude == 0) {
    for (size_t i = 0; i < count; i++) {
      uint32_t w = ((uint32_t)data[4 * i] << 24) | ((uint32_t)data[4 * i + 1] << 16) |
                   ((uint32_t)data[4 * i + 2] << 8) | data[4 * i + 3];
      out[i] = w % modulus;
    }
  } else {
    uint32_t real_modulus = modulus * (exclude - 1) / exclude;
    for (size_t i = 0; i < count; i++) {
      uint32_t w = ((uint32_t)data[4 * i] << 24) | ((uint32_t)data[4 * i + 1] << 16) |
                   ((uint32_t)data[4 * i + 2] << 8) | data[4 * i + 3];
      uint32_t v = w % real_modulus;
      out[i] = v + 1 + v / (exclude - 1);
    }
  }
  free(data);
  return 0;
}

/* ------------------------------------------------------------------ */
/* commitment/src/merkle_proof_in_place.rs                              */
/* ------------------------------------------------------------------ */
typedef struct { uint8_t h[32]; } dg;

/* gen_multi_proofs_in_place, merkle_proof_in_place.rs:54-101.  nodes_out
 * receives, for each index, one sibling per level (appended at *depth). */
static void gen_in_place(dg* layer, size_t len, const size_t* idx, size_t nidx, size_t steps,
                         dg* nodes_out, size_t stride, size_t* depth) {
  size_t lg = 0; while (((size_t)1 << lg) < steps) lg++;
  while (((size_t)1 << lg) < len) {
    for (size_t i = 0; i < nidx; i++) {
      size_t twin = ((idx[i] >> lg) ^ 1) << lg;
      nodes_out[i * stride + depth[i]] = layer[twin];
      depth[i]++;
    }
    size_t interval = (size_t)1 << lg, chunk = interval << 1;
    for (size_t c = 0; c < len; c += chunk) {
      uint8_t msg[64];
      memcpy(msg, layer[c].h, 32); memcpy(msg + 32, layer[c + interval].h, 32);
      oracle_blake2s(msg, 64, layer[c].h);
    }
    lg++;
  }
}

typedef struct { size_t idx, pos; } ipair;
static int ipair_cmp(const void* a, const void* b) {
  const ipair* x = (const ipair*)a; const ipair* y = (const ipair*)b;
  if (x->idx != y->idx) return x->idx < y->idx ? -1 : 1;
  return x->pos < y->pos ? -1 : (x->pos > y->pos); /* stable */
}

/* gen_multi_proofs_multi_core, merkle_proof_in_place.rs:106-206.
 * leaves: n leaves of leaf_len bytes each (n a power of two).
 * chunks: 2^log_num_cpus subtrees (multicore.rs:47-49).
 * root_out: 32 B.  nodes_out: nidx * log2(n) digests in caller index order
 * (leaf -> root); leaves are not copied (the caller holds them).
 * Returns 0, or -1 if n is not a power of two. */
int oracle_merkle_proofs(const uint8_t* leaves, size_t n, size_t leaf_len, const size_t* indices,
                         size_t nidx, size_t chunks, uint8_t* root_out, uint8_t* nodes_out) {
  if (n == 0 || (n & (n - 1))) return -1;
  size_t logn = 0; while (((size_t)1 << logn) < n) logn++;
  ipair* sorted = (ipair*)malloc(sizeof(ipair) * (nidx ? nidx : 1));
  for (size_t i = 0; i < nidx; i++) { sorted[i].idx = indices[i]; sorted[i].pos = i; }
  qsort(sorted, nidx, sizeof(ipair), ipair_cmp);
  dg* cur = (dg*)malloc(sizeof(dg) * n);
  for (size_t i = 0; i < n; i++) oracle_blake2s(leaves + i * leaf_len, leaf_len, cur[i].h);
  if (chunks > n) chunks = n;
  size_t chunk_size = n / chunks;
  dg* sub_nodes = (dg*)malloc(sizeof(dg) * (nidx ? nidx : 1) * (logn ? logn : 1));
  size_t* depth = (size_t*)calloc(nidx ? nidx : 1, sizeof(size_t));
  size_t* sub_idx = (size_t*)malloc(sizeof(size_t) * (nidx ? nidx : 1));
  size_t stride = logn ? logn : 1;
  size_t done = 0;
  for (size_t c = 0; c < chunks; c++) {
    size_t k = 0;
    for (size_t i = 0; i < nidx; i++)
      if (sorted[i].idx >= c * chunk_size && sorted[i].idx < (c + 1) * chunk_size)
        sub_idx[k++] = sorted[i].idx - c * chunk_size;
    gen_in_place(cur + c * chunk_size, chunk_size, sub_idx, k, 1, sub_nodes + done * stride, stride,
                 depth + done);
    done += k;
  }
  /* top tree over subtree roots at multiples of chunk_size (:176-180) */
  size_t* top_idx = (size_t*)malloc(sizeof(size_t) * chunks);
  for (size_t c = 0; c < chunks; c++) top_idx[c] = c * chunk_size;
  size_t top_stride = logn ? logn : 1;
  dg* top_nodes = (dg*)malloc(sizeof(dg) * chunks * top_stride);
  size_t* top_depth = (size_t*)calloc(chunks, sizeof(size_t));
  gen_in_place(cur, n, top_idx, chunks, chunk_size, top_nodes, top_stride, top_depth);
  memcpy(root_out, cur[0].h, 32);
  for (size_t i = 0; i < nidx; i++) { /* :191-197 then restore order :199-204 */
    size_t c = sorted[i].idx / chunk_size;
    for (size_t d = 0; d < top_depth[c]; d++) sub_nodes[i * stride + depth[i] + d] = top_nodes[c * top_stride + d];
    if (depth[i] + top_depth[c] != logn) { abort(); }
    memcpy(nodes_out + sorted[i].pos * logn * 32, sub_nodes + i * stride, logn * 32);
  }
  free(sorted); free(cur); free(sub_nodes); free(depth); free(sub_idx); free(top_idx);
  free(top_nodes); free(top_depth);
  return 0;
}

/* ------------------------------------------------------------------ */
/* fri/src/fri.rs:46-224 prove_low_degree, serialised as the serde_json */
/* compact encoding of Vec<FriProof<BlakeDigest>> (fri.rs:16-26,        */
/* commitment/src/merkle_tree.rs:14-18, blake.rs:8).                    */
/* ------------------------------------------------------------------ */
void sb_put(sbuf* b, const char* s, size_t n) {
  if (b->len + n + 1 > b->cap) { b->cap = (b->len + n + 1) * 2; b->s = (char*)realloc(b->s, b->cap); }
  memcpy(b->s + b->len, s, n); b->len += n; b->s[b->len] = 0;
}
void sb_str(sbuf* b, const char* s) { sb_put(b, s, strlen(s)); }
void sb_bytes(sbuf* b, const uint8_t* p, size_t n) {
  char tmp[8];
  sb_str(b, "[");
  for (size_t i = 0; i < n; i++) { int k = snprintf(tmp, sizeof tmp, i ? ",%u" : "%u", p[i]); sb_put(b, tmp, (size_t)k); }
  sb_str(b, "]");
}
void sb_proofs(sbuf* b, const uint8_t* leaves, size_t leaf_len, const size_t* idx, size_t k,
                      const uint8_t* nodes, size_t logn) {
  sb_str(b, "[");
  for (size_t i = 0; i < k; i++) {
    if (i) sb_str(b, ",");
    sb_str(b, "{\"leaf\":"); sb_bytes(b, leaves + idx[i] * leaf_len, leaf_len);
    sb_str(b, ",\"nodes\":[");
    for (size_t d = 0; d < logn; d++) { if (d) sb_str(b, ","); sb_bytes(b, nodes + (i * logn + d) * 32, 32); }
    sb_str(b, "]}");
  }
  sb_str(b, "]");
}

void fri_rec(sbuf* b, int first, fp* values, size_t nvals, fp root, size_t maxdeg,
                    uint32_t excl, size_t chunks) {
  /* xs = expand_root_of_unity(root) (fri.rs:84) */
  size_t nxs = or_expand_root_of_unity(root, NULL, 0);
  if (!first) sb_str(b, ",");
  if (maxdeg <= 16) { /* fri.rs:88-111 (degree check is debug_assert only) */
    sb_str(b, "{\"Last\":{\"last\":[");
    for (size_t i = 0; i < nvals; i++) {
      uint64_t c[4]; fp_to_canon(values[i], c);
      if (i) sb_str(b, ",");
      sb_bytes(b, (const uint8_t*)c, 32);
    }
    sb_str(b, "]}}");
    return;
  }
  fp* xs = (fp*)malloc(sizeof(fp) * nxs);
  or_expand_root_of_unity(root, xs, nxs);
  /* encoded values (to_bytes_le) -> m_tree root (fri.rs:120-131) */
  uint8_t* enc = (uint8_t*)malloc(32 * nvals);
  for (size_t i = 0; i < nvals; i++) fp_to_canon(values[i], (uint64_t*)(enc + 32 * i));
  uint8_t m_root[32];
  oracle_merkle_proofs(enc, nvals, 32, NULL, 0, chunks, m_root, NULL);
  fp special_x; { uint64_t c[4]; oracle_from_bytes_le(m_root, 32, c); special_x = fp_from_canon(c); }
  size_t q = nxs / 4; /* fri.rs:141 */
  fp (*xsets)[4] = malloc(sizeof(fp) * 4 * q);
  fp (*ysets)[4] = malloc(sizeof(fp) * 4 * q);
  fp (*polys)[4] = malloc(sizeof(fp) * 4 * q);
  for (size_t i = 0; i < q; i++)
    for (int j = 0; j < 4; j++) { xsets[i][j] = xs[i + q * j]; ysets[i][j] = values[i + q * j]; }
  or_multi_interp_4((const fp (*)[4])xsets, (const fp (*)[4])ysets, polys, q);
  fp* column = (fp*)malloc(sizeof(fp) * q);
  for (size_t i = 0; i < q; i++) column[i] = eval_quartic(polys[i], special_x);
  uint8_t* enc_col = (uint8_t*)malloc(32 * q);
  for (size_t i = 0; i < q; i++) fp_to_canon(column[i], (uint64_t*)(enc_col + 32 * i));
  uint8_t m2_root[32];
  oracle_merkle_proofs(enc_col, q, 32, NULL, 0, chunks, m2_root, NULL);
  uint32_t ys[40];
  oracle_get_pseudorandom_indices(m2_root, 32, (uint32_t)q, 40, excl, ys); /* fri.rs:181-189 */
  size_t ysz[40], pos[160];
  for (int i = 0; i < 40; i++) ysz[i] = ys[i];
  for (int i = 0; i < 40; i++)
    for (int j = 0; j < 4; j++) pos[4 * i + j] = ys[i] + (nxs / 4) * j; /* fri.rs:193-204 */
  size_t logq = 0; while (((size_t)1 << logq) < q) logq++;
  size_t logn = 0; while (((size_t)1 << logn) < nvals) logn++;
  uint8_t* col_nodes = (uint8_t*)malloc(40 * (logq ? logq : 1) * 32);
  uint8_t* poly_nodes = (uint8_t*)malloc(160 * (logn ? logn : 1) * 32);
  uint8_t rtmp[32];
  oracle_merkle_proofs(enc_col, q, 32, ysz, 40, chunks, rtmp, col_nodes);
  oracle_merkle_proofs(enc, nvals, 32, pos, 160, chunks, rtmp, poly_nodes);
  sb_str(b, "{\"Middle\":{\"root2\":"); sb_bytes(b, m2_root, 32);
  sb_str(b, ",\"column_branches\":"); sb_proofs(b, enc_col, 32, ysz, 40, col_nodes, logq);
  sb_str(b, ",\"poly_branches\":"); sb_proofs(b, enc, 32, pos, 160, poly_nodes, logn);
  sb_str(b, "}}");
  free(xs); free(enc); free(xsets); free(ysets); free(polys); free(enc_col);
  free(col_nodes); free(poly_nodes);
  fri_rec(b, 0, column, q, fp_pow(root, 4), maxdeg / 4, excl, chunks); /* fri.rs:215-223 */
  free(column);
}

/* Returns a malloc'd NUL-terminated JSON string (free with oracle_free). */
char* oracle_prove_low_degree_json(const uint64_t* values, size_t n, const uint64_t root[4],
                                   size_t max_deg_plus_1, uint32_t exclude, size_t chunks) {
  or_init();
  fp* v = or_load(values, n, n);
  sbuf b = {0, 0, 0};
  sb_str(&b, "[");
  fri_rec(&b, 1, v, n, fp_from_canon(root), max_deg_plus_1, exclude, chunks);
  sb_str(&b, "]");
  free(v);
  return b.s;
}
void oracle_free(void* p) { free(p); }
