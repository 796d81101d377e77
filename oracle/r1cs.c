/*
 * r1cs.c -- CPU restatement of mk_r1cs_proof
 * (packages/r1cs-stark/src/prove.rs:14-378 with the helpers of
 * packages/r1cs-stark/src/utils.rs:14-524), emitting the serde_json compact
 * encoding of StarkProof<BlakeDigest> (utils.rs:122-130) that run.rs:549
 * writes.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.c): the parity checker for
 * libstark_hip's stark_mk_r1cs_proof.  Statement order, loop structure and
 * index arithmetic follow the reference line by line; every step cites the
 * line it restates.  The NTTs, multi_inv, Merkle trees and FRI come from
 * oracle.c (themselves restatements of packages/fri and packages/commitment).
 *
 * Parity: the reference commits no golden proof; this
 * restatement is pinned through its parts (oracle.c KATs), by the restated
 * verifier (oracle/stark_verify.py, verify.rs:13-258 + fri.rs:226-404) accepting
 * its proofs, and by the committed digests in tests/golden/r1cs_proofs.json.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle_internal.h"

#define EXTENSION_FACTOR 8         /* utils.rs:135 */
#define LOG_EXTENSION_FACTOR 3     /* utils.rs:134 */
#define SPOT_CHECK_SECURITY_FACTOR 80 /* utils.rs:136 */

/* log2_ceil, utils.rs:14-23 (floor(log2 v) + 1 for v >= 1; 1 for v = 0). */
static uint32_t log2_ceil_ref(size_t value) {
  uint32_t log_value = 1;
  size_t tmp = value;
  while (tmp > 1) { tmp /= 2; log_value++; }
  return log_value;
}

static fp from_u64(uint64_t v) { return fp_from_u64(v); }

/* T::from_str(decimal of big-endian bytes) (utils.rs:25-27, 51-57): BE integer mod p. */
static fp from_be_bytes(const uint8_t* b, size_t len) {
  uint8_t le[32];
  memset(le, 0, 32);
  for (size_t i = 0; i < len && i < 32; i++) le[i] = b[len - 1 - i];
  uint64_t c[4];
  oracle_from_bytes_le(le, 32, c);
  return fp_from_canon(c);
}

/* LDE of a step column: inv_best_fft(v, g1, log_steps) then best_fft(., g2, log_precision)
 * (prove.rs:100-101 and the eight identical pairs after it). `len` may be below steps:
 * inv_best_fft zero-pads (fft.rs:359-379). */
static fp* lde(const fp* v, size_t len, fp g1, uint32_t log_steps, fp g2, uint32_t log_prec, uint32_t cpus) {
  size_t steps = (size_t)1 << log_steps, prec = (size_t)1 << log_prec;
  fp* poly = (fp*)malloc(sizeof(fp) * prec);
  memcpy(poly, v, sizeof(fp) * len);
  or_inv_best_fft_mont(poly, len, g1, log_steps, cpus);
  or_best_fft_mont(poly, steps, g2, log_prec, cpus);
  return poly;
}

/* zpoly, poly_utils.rs:362-373 (returns the coefficient vector, low degree first, n+1 long). */
static fp* zpoly(const fp* xs, size_t n) {
  fp* root = (fp*)malloc(sizeof(fp) * (n + 1));
  root[0] = fp_one();
  for (size_t i = 0; i < n; i++) {
    root[i + 1] = fp_zero();
    for (size_t j = i + 1; j-- > 0;) root[j + 1] = fp_sub(root[j + 1], fp_mul(root[j], xs[i]));
  }
  for (size_t i = 0; i < (n + 1) / 2; i++) { fp t = root[i]; root[i] = root[n - i]; root[n - i] = t; }
  return root;
}

/* div_polys(a, [-x, 1]), poly_utils.rs:235-289 specialised to a monic linear divisor. */
static void div_linear(const fp* a, size_t alen, fp x, fp* out /* alen - 1 */) {
  fp* c = (fp*)malloc(sizeof(fp) * alen);
  memcpy(c, a, sizeof(fp) * alen);
  const fp b0 = fp_sub(fp_zero(), x);
  size_t apos = alen - 1;
  const size_t diff = alen - 2;
  for (size_t d = diff + 1; d-- > 0;) {
    fp quot = c[apos];          /* c[apos] * b[1]^-1, b[1] = 1 */
    out[d] = quot;              /* o.push then o.reverse() */
    c[d + 1] = fp_sub(c[d + 1], quot);
    c[d] = fp_sub(c[d], fp_mul(b0, quot));
    apos--;
  }
  free(c);
}

/* lagrange_interp, poly_utils.rs:409-439. Returns n coefficients. */
static fp* lagrange_interp(const fp* xs, const fp* ys, size_t n) {
  fp* root = zpoly(xs, n);
  fp* nums = (fp*)malloc(sizeof(fp) * n * (n ? n : 1));
  for (size_t i = 0; i < n; i++) div_linear(root, n + 1, xs[i], nums + i * n);
  fp* denoms = (fp*)malloc(sizeof(fp) * (n ? n : 1));
  for (size_t i = 0; i < n; i++) denoms[i] = or_eval_poly_at(nums + i * n, n, xs[i]);
  fp* inv_denoms = (fp*)malloc(sizeof(fp) * (n ? n : 1));
  or_multi_inv(denoms, inv_denoms, n);
  fp* b = (fp*)calloc(n ? n : 1, sizeof(fp));
  for (size_t i = 0; i < n; i++) {
    fp yslice = fp_mul(ys[i], inv_denoms[i]);
    for (size_t j = 0; j < n; j++)
      if (!fp_is_zero(nums[i * n + j]) && !fp_is_zero(ys[i])) b[j] = fp_add(b[j], fp_mul(nums[i * n + j], yslice));
  }
  free(root); free(nums); free(denoms); free(inv_denoms);
  return b;
}

static void enc(fp v, uint8_t* out) { fp_to_canon(v, (uint64_t*)out); }

/*
 * Returns a malloc'd JSON string, or NULL with *err set:
 *   1 = an input assert of prove.rs:32-35/53 failed (or original_steps < 5, where the
 *       reference's steps/log_steps disagree: prove.rs:37-41),
 *   2 = a divisibility assert (utils.rs:379-418 D1-D3, :477-524 B2/B3) failed.
 * Elements are canonical LE u64[4]; public_first_indices holds (k, w) pairs.
 */
/* rows_out != NULL: stop once the main-tree rows exist and hand them (precision x 256 B)
 * and a_root to the caller (the distributed-prover tests' per-rank slices). */
static char* mk_proof(const uint64_t* witness_trace_c, const uint64_t* computational_trace_c,
                      size_t original_steps, const uint64_t* public_wires_c, size_t n_public,
                      const size_t* public_first_indices, size_t n_pfi,
                      const size_t* permuted_indices_in, const uint64_t* coefficients_c,
                      const uint64_t* flag0_c, const uint64_t* flag1_c, const uint64_t* flag2_c,
                      size_t n_constraints, size_t n_wires, uint32_t cpus, int* err,
                      uint8_t** rows_out, uint8_t* a_root_out) {
  or_init();
  *err = 0;
  if (!(original_steps <= 3 * n_constraints * n_wires) || original_steps % 3 != 0 || original_steps < 5) {
    *err = 1; /* prove.rs:32-33 */
    return NULL;
  }
  const uint32_t log_steps = log2_ceil_ref(original_steps - 1); /* prove.rs:37 */
  size_t steps = (size_t)1 << log_steps;
  if (steps < 8) steps = 8;                                      /* prove.rs:38-41 */
  const size_t precision = steps * EXTENSION_FACTOR;             /* prove.rs:43 */
  const uint32_t log_precision = log_steps + LOG_EXTENSION_FACTOR;
  if (log_precision >= 24) { *err = 1; return NULL; } /* prove.rs:51-53; precision < 2^24 (fri/src/utils.rs:88) */

  /* prove.rs:55-69: pad to steps */
  size_t* permuted_indices = (size_t*)malloc(sizeof(size_t) * steps);
  memcpy(permuted_indices, permuted_indices_in, sizeof(size_t) * original_steps);
  for (size_t i = original_steps; i < steps; i++) permuted_indices[i] = i;
  fp* coefficients = or_load(coefficients_c, original_steps, steps);
  fp* witness_trace = or_load(witness_trace_c, original_steps, steps);
  fp* computational_trace = or_load(computational_trace_c, original_steps, steps);
  for (size_t i = original_steps; i < steps; i++)
    coefficients[i] = witness_trace[i] = computational_trace[i] = fp_zero();
  fp* flag0 = or_load(flag0_c, original_steps, original_steps);
  fp* flag1 = or_load(flag1_c, original_steps, original_steps);
  fp* flag2 = or_load(flag2_c, original_steps, original_steps);
  fp* public_wires = or_load(public_wires_c, n_public, n_public);

  /* g2 = 7^((p-1)/precision), xs = expand_root_of_unity(g2), g1 = xs[8] (prove.rs:71-92) */
  uint64_t g2c[4];
  oracle_root_of_unity(log_precision, g2c);
  const fp g2 = fp_from_canon(g2c);
  fp* xs = (fp*)malloc(sizeof(fp) * precision);
  or_expand_root_of_unity(g2, xs, precision);
  const size_t skips = precision / steps;
  const fp g1 = xs[skips];

  /* LDEs (prove.rs:100-126) */
  fp* k_ev = lde(coefficients, steps, g1, log_steps, g2, log_precision, cpus);
  fp* f0_ev = lde(flag0, original_steps, g1, log_steps, g2, log_precision, cpus);
  fp* f1_ev = lde(flag1, original_steps, g1, log_steps, g2, log_precision, cpus);
  fp* f2_ev = lde(flag2, original_steps, g1, log_steps, g2, log_precision, cpus);
  fp* s_ev = lde(witness_trace, steps, g1, log_steps, g2, log_precision, cpus);
  fp* p_ev = lde(computational_trace, steps, g1, log_steps, g2, log_precision, cpus);

  /* Z = X^steps - 1 (utils.rs:173-178), best_fft at g2 (prove.rs:128-129) */
  fp* z_ev = (fp*)malloc(sizeof(fp) * precision);
  for (size_t i = 0; i <= steps; i++) z_ev[i] = fp_zero();
  z_ev[0] = fp_sub(fp_zero(), fp_one());
  z_ev[steps] = fp_one();
  or_best_fft_mont(z_ev, steps + 1, g2, log_precision, cpus);

  /* Q1, utils.rs:181-213 */
  fp* q1 = (fp*)malloc(sizeof(fp) * precision);
  for (size_t j = 0; j < precision; j++) {
    fp p_prev = p_ev[(j + precision - skips) % precision];
    q1[j] = fp_mul(f0_ev[j], fp_sub(fp_sub(p_ev[j], fp_mul(f1_ev[j], p_prev)), fp_mul(k_ev[j], s_ev[j])));
  }
  /* Q2, utils.rs:217-248 */
  fp* q2 = (fp*)malloc(sizeof(fp) * precision);
  for (size_t j = 0; j < precision; j++) {
    size_t j2 = (j + original_steps / 3 * skips) % precision;
    size_t j3 = (j + original_steps / 3 * 2 * skips) % precision;
    q2[j] = fp_mul(f2_ev[j], fp_sub(p_ev[j3], fp_mul(p_ev[j], p_ev[j2])));
  }

  /* index columns (prove.rs:160-167, utils.rs:164-170) */
  fp* idx = (fp*)malloc(sizeof(fp) * steps);
  fp* pidx = (fp*)malloc(sizeof(fp) * steps);
  for (size_t i = 0; i < steps; i++) { idx[i] = from_u64(i); pidx[i] = from_u64(permuted_indices[i]); }
  fp* ext_idx = lde(idx, steps, g1, log_steps, g2, log_precision, cpus);
  fp* ext_pidx = lde(pidx, steps, g1, log_steps, g2, log_precision, cpus);

  /* accumulator tree root (utils.rs:250-270): leaf = u64 LE index || to_bytes_le(w) */
  uint8_t a_root[32];
  {
    uint8_t* leaves = (uint8_t*)malloc(40 * steps);
    for (size_t i = 0; i < steps; i++) {
      uint64_t pv = (uint64_t)permuted_indices[i];
      memcpy(leaves + 40 * i, &pv, 8);
      enc(witness_trace[i], leaves + 40 * i + 8);
    }
    oracle_merkle_proofs(leaves, steps, 40, NULL, 0, cpus, a_root, NULL);
    free(leaves);
  }
  /* r = get_random_ff_values(a_root, precision, 3, 0) (utils.rs:272-290) */
  fp r[3];
  {
    uint32_t rnd[24];
    oracle_get_pseudorandom_indices(a_root, 32, (uint32_t)precision, 24, 0, rnd);
    for (int c = 0; c < 3; c++) {
      uint8_t be[32];
      for (int i = 0; i < 8; i++) {
        uint32_t v = rnd[8 * c + i];
        be[4 * i] = (uint8_t)(v >> 24); be[4 * i + 1] = (uint8_t)(v >> 16);
        be[4 * i + 2] = (uint8_t)(v >> 8); be[4 * i + 3] = (uint8_t)v;
      }
      uint64_t cc[4];
      oracle_from_bytes_le(be, 32, cc); /* from_bytes_le of BE-written words (utils.rs:284) */
      r[c] = fp_from_canon(cc);
    }
  }
  /* calc_a_mini_evaluations, utils.rs:293-339 */
  fp* a_mini = (fp*)malloc(sizeof(fp) * steps);
  {
    fp* nmr = (fp*)malloc(sizeof(fp) * steps);
    fp* dnm = (fp*)malloc(sizeof(fp) * steps);
    for (size_t j = 0; j < steps; j++) {
      fp last_nmr = j ? nmr[j - 1] : fp_one();
      fp last_dnm = j ? dnm[j - 1] : fp_one();
      fp val_nmr = fp_add(fp_add(r[0], fp_mul(r[1], ext_idx[j * skips])), fp_mul(r[2], witness_trace[j]));
      fp val_dnm = fp_add(fp_add(r[0], fp_mul(r[1], ext_pidx[j * skips])), fp_mul(r[2], witness_trace[j]));
      nmr[j] = fp_mul(val_nmr, last_nmr);
      dnm[j] = fp_mul(val_dnm, last_dnm);
    }
    fp* inv_dnm = (fp*)malloc(sizeof(fp) * steps);
    or_multi_inv(dnm, inv_dnm, steps);
    for (size_t j = 0; j < steps; j++) a_mini[j] = fp_mul(nmr[j], inv_dnm[j]);
    free(nmr); free(dnm); free(inv_dnm);
  }
  fp* a_ev = lde(a_mini, steps, g1, log_steps, g2, log_precision, cpus); /* prove.rs:183-184 */

  /* Q3, utils.rs:344-376 */
  fp* q3 = (fp*)malloc(sizeof(fp) * precision);
  for (size_t j = 0; j < precision; j++) {
    fp val_nmr = fp_add(fp_add(r[0], fp_mul(r[1], ext_idx[j])), fp_mul(r[2], s_ev[j]));
    fp val_dnm = fp_add(fp_add(r[0], fp_mul(r[1], ext_pidx[j])), fp_mul(r[2], s_ev[j]));
    size_t prev_j = (j + precision - skips) % precision;
    q3[j] = fp_sub(fp_mul(a_ev[j], val_dnm), fp_mul(a_ev[prev_j], val_nmr));
  }

  char* out = NULL;
  fp* inv_z = (fp*)malloc(sizeof(fp) * precision);
  or_multi_inv(z_ev, inv_z, precision); /* prove.rs:203 */
  fp* d1 = (fp*)malloc(sizeof(fp) * precision);
  fp* d2 = (fp*)malloc(sizeof(fp) * precision);
  fp* d3 = (fp*)malloc(sizeof(fp) * precision);
  for (size_t j = 0; j < precision; j++) { /* utils.rs:379-418 */
    if (fp_is_zero(inv_z[j]) && (!fp_is_zero(q1[j]) || !fp_is_zero(q2[j]) || !fp_is_zero(q3[j]))) *err = 2;
    d1[j] = fp_mul(q1[j], inv_z[j]);
    d2[j] = fp_mul(q2[j], inv_z[j]);
    d3[j] = fp_mul(q3[j], inv_z[j]);
  }

  /* I2 (utils.rs:421-435), I3 (:458-463) and their evaluations (prove.rs:216-220) */
  fp* i2_ev = (fp*)malloc(sizeof(fp) * precision);
  fp* i3_ev = (fp*)malloc(sizeof(fp) * precision);
  {
    fp* xv = (fp*)malloc(sizeof(fp) * (n_pfi ? n_pfi : 1));
    fp* yv = (fp*)malloc(sizeof(fp) * (n_pfi ? n_pfi : 1));
    for (size_t i = 0; i < n_pfi; i++) {
      xv[i] = xs[skips * public_first_indices[2 * i + 1]];
      yv[i] = public_wires[public_first_indices[2 * i]];
    }
    fp* interp2 = lagrange_interp(xv, yv, n_pfi);
    fp x_last = xs[precision - skips];
    fp one = fp_one();
    fp* interp3 = lagrange_interp(&x_last, &one, 1);
    for (size_t i = 0; i < precision; i++) {
      i2_ev[i] = or_eval_poly_at(interp2, n_pfi, xs[i]);
      i3_ev[i] = or_eval_poly_at(interp3, 1, xs[i]);
    }
    free(xv); free(yv); free(interp2); free(interp3);
  }
  /* Zb2 (utils.rs:438-455), Zb3 (:466-474) */
  fp* zb2 = (fp*)malloc(sizeof(fp) * precision);
  fp* zb3 = (fp*)malloc(sizeof(fp) * precision);
  for (size_t i = 0; i < precision; i++) zb2[i] = fp_one();
  for (size_t k = 0; k < n_pfi; k++) {
    size_t j = public_first_indices[2 * k + 1] * skips;
    for (size_t i = 0; i < precision; i++) zb2[i] = fp_mul(zb2[i], fp_sub(xs[i], xs[j]));
  }
  {
    fp x_last = xs[precision - skips];
    for (size_t i = 0; i < precision; i++) zb3[i] = fp_mul(fp_one(), fp_sub(xs[i], x_last));
  }
  fp* inv_zb2 = (fp*)malloc(sizeof(fp) * precision);
  fp* inv_zb3 = (fp*)malloc(sizeof(fp) * precision);
  or_multi_inv(zb2, inv_zb2, precision);
  or_multi_inv(zb3, inv_zb3, precision);
  fp* b2 = (fp*)malloc(sizeof(fp) * precision);
  fp* b3 = (fp*)malloc(sizeof(fp) * precision);
  for (size_t i = 0; i < precision; i++) { /* utils.rs:477-524 */
    if (fp_is_zero(inv_zb2[i]) && !fp_eq(s_ev[i], i2_ev[i])) *err = 2;
    if (fp_is_zero(inv_zb3[i]) && !fp_eq(a_ev[i], i3_ev[i])) *err = 2;
    b2[i] = fp_mul(fp_sub(s_ev[i], i2_ev[i]), inv_zb2[i]);
    b3[i] = fp_mul(fp_sub(a_ev[i], i3_ev[i]), inv_zb3[i]);
  }
  if (*err) goto done;

  {
    /* main leaves P||A||S||D1||D2||D3||B2||B3 (prove.rs:235-258) and m_root (:261-264) */
    uint8_t* main_leaves = (uint8_t*)malloc(256 * precision);
    for (size_t i = 0; i < precision; i++) {
      uint8_t* row = main_leaves + 256 * i;
      enc(p_ev[i], row); enc(a_ev[i], row + 32); enc(s_ev[i], row + 64); enc(d1[i], row + 96);
      enc(d2[i], row + 128); enc(d3[i], row + 160); enc(b2[i], row + 192); enc(b3[i], row + 224);
    }
    if (rows_out) {
      *rows_out = main_leaves;
      memcpy(a_root_out, a_root, 32);
      goto done;
    }
    uint8_t m_root[32];
    oracle_merkle_proofs(main_leaves, precision, 256, NULL, 0, cpus, m_root, NULL);
    /* k (prove.rs:274-283) */
    fp k[11];
    k[0] = fp_one();
    for (int i = 1; i < 11; i++) {
      uint8_t msg[33], h[32];
      memcpy(msg, m_root, 32);
      msg[32] = (uint8_t)i;
      oracle_blake2s(msg, 33, h);
      k[i] = from_be_bytes(h, 32);
    }
    /* powers of g2^steps (prove.rs:287-291) and L (:293-322) */
    const fp g2s = xs[steps];
    fp pw = fp_one();
    fp* l_ev = (fp*)malloc(sizeof(fp) * precision);
    for (size_t i = 0; i < precision; i++) {
      if (i) pw = fp_mul(g2s, pw);
      fp acc = fp_mul(k[0], d1[i]);
      acc = fp_add(acc, fp_mul(k[1], d2[i]));
      acc = fp_add(acc, fp_mul(k[2], d3[i]));
      acc = fp_add(acc, fp_mul(k[3], p_ev[i]));
      acc = fp_add(acc, fp_mul(fp_mul(k[4], p_ev[i]), pw));
      acc = fp_add(acc, fp_mul(k[5], b2[i]));
      acc = fp_add(acc, fp_mul(fp_mul(k[6], b2[i]), pw));
      acc = fp_add(acc, fp_mul(k[7], b3[i]));
      acc = fp_add(acc, fp_mul(fp_mul(k[8], b3[i]), pw));
      acc = fp_add(acc, fp_mul(k[9], a_ev[i]));
      acc = fp_add(acc, fp_mul(k[10], s_ev[i]));
      l_ev[i] = acc;
    }
    uint8_t* l_leaves = (uint8_t*)malloc(32 * precision);
    for (size_t i = 0; i < precision; i++) enc(l_ev[i], l_leaves + 32 * i);
    uint8_t l_root[32];
    oracle_merkle_proofs(l_leaves, precision, 32, NULL, 0, cpus, l_root, NULL); /* prove.rs:329-332 */
    /* positions (prove.rs:337-345) */
    uint32_t pos32[SPOT_CHECK_SECURITY_FACTOR];
    oracle_get_pseudorandom_indices(l_root, 32, (uint32_t)precision, SPOT_CHECK_SECURITY_FACTOR, (uint32_t)skips,
                                    pos32);
    size_t positions[SPOT_CHECK_SECURITY_FACTOR], aug[4 * SPOT_CHECK_SECURITY_FACTOR];
    for (int i = 0; i < SPOT_CHECK_SECURITY_FACTOR; i++) positions[i] = pos32[i];
    for (int i = 0; i < SPOT_CHECK_SECURITY_FACTOR; i++) { /* prove.rs:351-359 */
      size_t j = positions[i];
      aug[4 * i] = j;
      aug[4 * i + 1] = (j + precision - skips) % precision;
      aug[4 * i + 2] = (j + original_steps / 3 * skips) % precision;
      aug[4 * i + 3] = (j + original_steps / 3 * 2 * skips) % precision;
    }
    const size_t logp = log_precision;
    uint8_t rtmp[32];
    uint8_t* l_nodes = (uint8_t*)malloc(SPOT_CHECK_SECURITY_FACTOR * logp * 32);
    oracle_merkle_proofs(l_leaves, precision, 32, positions, SPOT_CHECK_SECURITY_FACTOR, cpus, rtmp, l_nodes);
    uint8_t* m_nodes = (uint8_t*)malloc(4 * SPOT_CHECK_SECURITY_FACTOR * logp * 32);
    oracle_merkle_proofs(main_leaves, precision, 256, aug, 4 * SPOT_CHECK_SECURITY_FACTOR, cpus, rtmp, m_nodes);

    /* StarkProof JSON (utils.rs:122-130, run.rs:549) */
    sbuf b = {0, 0, 0};
    sb_str(&b, "{\"m_root\":"); sb_bytes(&b, m_root, 32);
    sb_str(&b, ",\"l_root\":"); sb_bytes(&b, l_root, 32);
    sb_str(&b, ",\"a_root\":"); sb_bytes(&b, a_root, 32);
    sb_str(&b, ",\"main_branches\":");
    sb_proofs(&b, main_leaves, 256, aug, 4 * SPOT_CHECK_SECURITY_FACTOR, m_nodes, logp);
    sb_str(&b, ",\"linear_comb_branches\":");
    sb_proofs(&b, l_leaves, 32, positions, SPOT_CHECK_SECURITY_FACTOR, l_nodes, logp);
    /* prove_low_degree(L, g2, precision / 4, skips) (prove.rs:367) */
    sb_str(&b, ",\"fri_proof\":[");
    fri_rec(&b, 1, l_ev, precision, g2, precision / 4, (uint32_t)skips, cpus);
    sb_str(&b, "]}");
    out = b.s;
    free(main_leaves); free(l_ev); free(l_leaves); free(l_nodes); free(m_nodes);
  }
done:
  free(permuted_indices); free(coefficients); free(witness_trace); free(computational_trace);
  free(flag0); free(flag1); free(flag2); free(public_wires); free(xs);
  free(k_ev); free(f0_ev); free(f1_ev); free(f2_ev); free(s_ev); free(p_ev); free(z_ev);
  free(q1); free(q2); free(q3); free(idx); free(pidx); free(ext_idx); free(ext_pidx);
  free(a_mini); free(a_ev); free(inv_z); free(d1); free(d2); free(d3);
  free(i2_ev); free(i3_ev); free(zb2); free(zb3); free(inv_zb2); free(inv_zb3); free(b2); free(b3);
  return out;
}

char* oracle_mk_r1cs_proof_json(const uint64_t* witness_trace_c, const uint64_t* computational_trace_c,
                                size_t original_steps, const uint64_t* public_wires_c, size_t n_public,
                                const size_t* public_first_indices, size_t n_pfi,
                                const size_t* permuted_indices_in, const uint64_t* coefficients_c,
                                const uint64_t* flag0_c, const uint64_t* flag1_c, const uint64_t* flag2_c,
                                size_t n_constraints, size_t n_wires, uint32_t cpus, int* err) {
  return mk_proof(witness_trace_c, computational_trace_c, original_steps, public_wires_c, n_public,
                  public_first_indices, n_pfi, permuted_indices_in, coefficients_c, flag0_c, flag1_c, flag2_c,
                  n_constraints, n_wires, cpus, err, NULL, NULL);
}

/* The main-tree rows P|A|S|D1|D2|D3|B2|B3 of every precision point (prove.rs:235-258)
 * and a_root; free the rows with oracle_free. */
uint8_t* oracle_r1cs_rows(const uint64_t* witness_trace_c, const uint64_t* computational_trace_c,
                          size_t original_steps, const uint64_t* public_wires_c, size_t n_public,
                          const size_t* public_first_indices, size_t n_pfi, const size_t* permuted_indices_in,
                          const uint64_t* coefficients_c, const uint64_t* flag0_c, const uint64_t* flag1_c,
                          const uint64_t* flag2_c, size_t n_constraints, size_t n_wires, uint32_t cpus, int* err,
                          uint8_t a_root[32]) {
  uint8_t* rows = NULL;
  mk_proof(witness_trace_c, computational_trace_c, original_steps, public_wires_c, n_public, public_first_indices,
           n_pfi, permuted_indices_in, coefficients_c, flag0_c, flag1_c, flag2_c, n_constraints, n_wires, cpus, err,
           &rows, a_root);
  return rows;
}
