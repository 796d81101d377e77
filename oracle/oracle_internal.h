/*
 * oracle_internal.h -- shared declarations of the CPU oracle's translation
 * units (oracle.c: field, NTT, Merkle, FRI; r1cs.c: mk_r1cs_proof).
 *
 * TEST INFRASTRUCTURE ONLY (see the header of oracle.c).
 */
#pragma once
#include <stddef.h>
#include <stdint.h>

typedef struct { uint64_t v[4]; } fp; /* Montgomery form, R = 2^256 */
typedef struct { char* s; size_t len, cap; } sbuf;

void or_init(void);
fp fp_add(fp a, fp b);
fp fp_sub(fp a, fp b);
fp fp_mul(fp a, fp b);
int fp_eq(fp a, fp b);
int fp_is_zero(fp a);
fp fp_from_canon(const uint64_t c[4]);
void fp_to_canon(fp a, uint64_t c[4]);
fp fp_from_u64(uint64_t v);
fp fp_one(void);
fp fp_zero(void);
fp fp_pow_limbs(fp a, const uint64_t* e, int nlimbs);
fp fp_pow(fp a, uint64_t e);
fp fp_inv(fp a);

size_t or_expand_root_of_unity(fp root, fp* out, size_t cap);
void or_best_fft_mont(fp* values, size_t len, fp root, uint32_t log_n, uint32_t cpus);
void or_inv_best_fft_mont(fp* values, size_t len, fp root, uint32_t log_n, uint32_t cpus);
fp* or_load(const uint64_t* c, size_t len, size_t cap);
void or_store(const fp* v, uint64_t* c, size_t len);
void or_multi_inv(const fp* values, fp* outputs, size_t n);
fp or_eval_poly_at(const fp* poly, size_t deg1, fp x);

void oracle_root_of_unity(uint32_t log_n, uint64_t out[4]);
void oracle_from_bytes_le(const uint8_t* b, size_t len, uint64_t out[4]);
void oracle_blake2s(const uint8_t* msg, size_t len, uint8_t out[32]);
int oracle_get_pseudorandom_indices(const uint8_t* seed, size_t seed_len, uint32_t modulus, size_t count,
                                    uint32_t exclude, uint32_t* out);
int oracle_merkle_proofs(const uint8_t* leaves, size_t n, size_t leaf_len, const size_t* indices, size_t nidx,
                         size_t chunks, uint8_t* root_out, uint8_t* nodes_out);

void sb_put(sbuf* b, const char* s, size_t n);
void sb_str(sbuf* b, const char* s);
void sb_bytes(sbuf* b, const uint8_t* p, size_t n);
void sb_proofs(sbuf* b, const uint8_t* leaves, size_t leaf_len, const size_t* idx, size_t k, const uint8_t* nodes,
               size_t logn);
void fri_rec(sbuf* b, int first, fp* values, size_t nvals, fp root, size_t maxdeg, uint32_t excl, size_t chunks);
