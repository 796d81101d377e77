/*
 * stark_hip.h -- C ABI of the MI355X (gfx950) FRI-prover hot path.
 *
 * Drop-in boundary for the reference's Rust hot path
 * (InternetMaximalism/stark-pure-rust).  Each entry point names the reference
 * item it replaces (path:line, relative to the reference repo root).  A Rust
 * `extern "C"` shim that binds these is in INTEGRATION.md.
 *
 * Conventions
 *  - Field elements are BN254 Fr values as 4 little-endian u64 limbs, i.e. the
 *    32-byte canonical image `Fp::to_bytes_le` produces
 *    (packages/ff_utils/src/fp.rs:35-44).  Inputs must be < p (every Fp value
 *    is); outputs are always fully reduced.
 *  - Host-buffer entry points copy in, compute on the context's GPU, copy out,
 *    and never retain caller pointers after returning.  Device entry points
 *    (suffix _dev) take device pointers and a hipStream_t (NULL = the context
 *    stream) and are asynchronous on that stream.
 *  - Every call returns a stark_status; 0 = success.  Nothing unwinds.
 *  - One context per GPU; a context is not shared between threads.  Calls on one context may take
 *    different streams: the context's own buffers and cached tables are ordered across streams
 *    by the library (events), so results never depend on which stream a call used.  A stream
 *    handed to a call must stay valid until the context's next call on another stream (the
 *    library then records an event on it) or until stark_ctx_synchronize.
 *  - ABI changes bump STARK_ABI_VERSION; a client built against this header checks
 *    stark_abi_version() == STARK_ABI_VERSION at start-up (INTEGRATION.md lists the changes).
 */
#ifndef STARK_HIP_H
#define STARK_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: stark_r1cs_proof_branches takes leaves_cap / nodes_cap (round 4).
 * 3: device groups, stark_group_* (round 6). */
#define STARK_ABI_VERSION 3u
/* The ABI version the loaded library implements (no reference counterpart: a linking check). */
uint32_t stark_abi_version(void);
/* Paths per SIMD register of the verifier's host Merkle path checks on this CPU (16 AVX-512, 8 AVX2,
 * 4 SSE2; the environment variable STARK_B2S_WIDTH=4|8 narrows it).  A diagnostic with no reference
 * counterpart (Proof::validate, commitment/src/merkle_tree.rs:25-43, is what those checks restate). */
uint32_t stark_verify_simd_width(void);
/* Bytes per SIMD register of the proof JSON writer's byte-array digits on this CPU (64 with AVX-512
 * VBMI2, else 1: one table store per byte; STARK_JSON_SIMD=0 forces 1).  A diagnostic: the text is the
 * same either way (serde_json's, utils.rs:122-130 / fri.rs:16-26). */
uint32_t stark_json_simd_width(void);

typedef enum {
  STARK_OK = 0,
  STARK_ERR_BAD_LENGTH = 1,   /* len > 2^log_n, or not a power of two where one is required
                                 (fft.rs:162 assert, merkle_proof_in_place.rs:113 assert) */
  STARK_ERR_BAD_ROOT = 2,     /* root is not a primitive 2^log_n-th root of unity */
  STARK_ERR_BAD_ARG = 3,      /* null pointer, index out of range, modulus >= 2^24
                                 (fri/src/utils.rs:88 assert), ... */
  STARK_ERR_OOM = 4,          /* device or host allocation failed */
  STARK_ERR_HIP = 5,          /* a HIP runtime call failed */
  STARK_ERR_NO_DEVICE = 6,    /* no gfx950 device / bad device ordinal */
  STARK_ERR_STATE = 7,        /* API used out of order (e.g. proofs before update) */
  STARK_ERR_CHECK = 8         /* the witness does not satisfy the R1CS: a divisibility assert of
                                 r1cs-stark/src/utils.rs:379-418 (D1-D3) or :477-524 (B2, B3) */
} stark_status;

typedef struct stark_ctx stark_ctx;
typedef struct stark_merkle_tree stark_merkle_tree;
typedef struct stark_fri_proof stark_fri_proof;
typedef struct stark_r1cs_proof stark_r1cs_proof;
typedef struct stark_r1cs_trace stark_r1cs_trace;
typedef struct stark_dprove stark_dprove;
typedef struct stark_r1cs_circuit stark_r1cs_circuit;

/* ---- context ------------------------------------------------------------ */
/* Replaces commitment::multicore::Worker::new (packages/commitment/src/multicore.rs:43-45):
 * the unit of parallel execution is one GPU instead of a thread pool. */
stark_status stark_ctx_create(int device, stark_ctx** out);
void stark_ctx_destroy(stark_ctx* ctx);
const char* stark_status_str(stark_status s);
/* Last HIP error string recorded by the context (for STARK_ERR_HIP). */
const char* stark_ctx_last_error(const stark_ctx* ctx);
/* Returns the HIP stream the context launches on (as void* = hipStream_t). */
void* stark_ctx_stream(stark_ctx* ctx);
/* Memory bound of the context's caches (no reference counterpart: the reference recomputes its
 * twiddles per call, fft.rs:173).  The context caches the last NTT pass's full twiddle table per
 * (root, size, direction) -- 2^log_n x 32 B, 512 MB at 2^24 -- and the extension of the index
 * column per trace size (precision x 32 B).  Together they stay at or below `bytes` (default 4 GiB):
 * least recently used entries are freed first (after a device synchronisation), a table that does
 * not fit is not cached (the NTT's last pass then forms its twiddles from the two-level tables, same
 * outputs).  Setting a lower cap frees down to it at once. */
stark_status stark_ctx_set_cache_limit(stark_ctx* ctx, size_t bytes);
/* Device bytes the context holds: cached tables (<= *cache_limit), and everything resident
 * (cached tables, the small per-root twiddle tables, working arenas, context-owned trees).  Any
 * pointer may be NULL. */
stark_status stark_ctx_memory(const stark_ctx* ctx, size_t* cached_bytes, size_t* cache_limit,
                              size_t* resident_bytes);

/* ---- NTT (packages/fri/src/fft.rs) --------------------------------------- */
/* best_fft<T>(coefficients: Vec<T>, root_of_unity: &T, log_order_of_root: u32) -> Vec<T>
 * (fft.rs:327-357).  Zero-pads `len` coefficients to n = 2^log_n and writes the
 * n evaluations out[i] = sum_j c_j * root^(i*j) to `out` (4*n u64; may alias
 * `coeffs` when it has room for 4*n u64). */
stark_status stark_best_fft(stark_ctx* ctx, const uint64_t* coeffs, size_t len, const uint64_t root[4],
                            uint32_t log_n, uint64_t* out);
/* inv_best_fft<T>(evaluations, root_of_unity, log_order_of_root) (fft.rs:359-379):
 * pad, transform with root^-1, scale by n^-1. */
stark_status stark_inv_best_fft(stark_ctx* ctx, const uint64_t* evals, size_t len, const uint64_t root[4],
                                uint32_t log_n, uint64_t* out);
/* serial_fft / parallel_fft / inv_serial_fft / inv_parallel_fft (fft.rs:150, 195, 284, 295):
 * in place on exactly 2^log_n values (no padding). */
stark_status stark_fft_in_place(stark_ctx* ctx, uint64_t* values, const uint64_t root[4], uint32_t log_n,
                                int inverse);
/* Device-resident batched NTT: `batch` transforms of n = 2^log_n elements,
 * transform b at d_data + b*4*n u64.  In place.  inverse != 0 => inv_best_fft
 * semantics.  Asynchronous on `stream` (NULL = context stream). */
stark_status stark_ntt_dev(stark_ctx* ctx, uint64_t* d_data, uint32_t log_n, uint32_t batch,
                           const uint64_t root[4], int inverse, void* stream);
/* Diagnostics, no reference counterpart: the Stockham pass plan of a 2^log_n transform.
 * Writes up to `cap` log2 radices (first pass first) to log_r and returns the number of
 * passes (0 for log_n < 2, where no pass kernel runs).  bench.py prices its roofline with it. */
uint32_t stark_ntt_plan(uint32_t log_n, uint32_t* log_r, uint32_t cap);
/* Low-degree extension, the pattern of r1cs-stark/src/prove.rs:100-101 (and
 * :160-167, 183-184): inv_best_fft(values, g1, log2 steps) followed by
 * best_fft(coefficients zero-padded to steps << log_blowup, g2), where g2 is a
 * primitive (steps << log_blowup)-th root and g1 = g2^(2^log_blowup)
 * (prove.rs:71-94).  out holds steps << log_blowup elements.  The padding is
 * never materialised (the first forward pass reads the coefficients only). */
stark_status stark_lde(stark_ctx* ctx, const uint64_t* values, size_t steps, const uint64_t g1[4],
                       uint32_t log_blowup, const uint64_t g2[4], uint64_t* out);
/* Device-resident, batched: `batch` columns of 2^log_steps values at d_values
 * (overwritten with their coefficients) -> `batch` columns of
 * 2^(log_steps + log_blowup) evaluations at d_out.  Asynchronous on `stream`. */
stark_status stark_lde_dev(stark_ctx* ctx, uint64_t* d_values, uint64_t* d_out, uint32_t log_steps,
                           uint32_t log_blowup, uint32_t batch, const uint64_t g1[4], const uint64_t g2[4],
                           void* stream);
/* expand_root_of_unity<T>(root) -> Vec<T> (fft.rs:5-14): writes
 * min(order, cap) powers [1, w, w^2, ...] and stores the order in *count.
 * The order must be a power of two <= 2^28. */
stark_status stark_expand_root_of_unity(stark_ctx* ctx, const uint64_t root[4], uint64_t* out, size_t cap,
                                        size_t* count);

/* ---- field-vector kernels (packages/fri/src/poly_utils.rs) --------------- */
/* multi_inv<T>(values) -> Vec<T> (poly_utils.rs:38-70); zero maps to zero. */
stark_status stark_multi_inv(stark_ctx* ctx, const uint64_t* values, size_t n, uint64_t* out);
/* xs.map(|x| eval_poly_at(poly, x)) (poly_utils.rs:93-102 as used at
 * r1cs-stark/src/prove.rs:216-220): out[i] = sum_k poly[k] * xs[i]^k. */
stark_status stark_eval_poly_at_multi(stark_ctx* ctx, const uint64_t* poly, size_t deg_plus_1,
                                      const uint64_t* xs, size_t n, uint64_t* out);
/* multi_interp_4<T>(xsets, ysets) -> Vec<[T; 4]> (poly_utils.rs:449-511): for
 * each row the coefficients of the cubic through (xs[k], ys[k]), k < 4; rows
 * x 4 elements in, rows x 4 coefficients out (zero denominators map to zero
 * through multi_inv, as in the reference). */
stark_status stark_multi_interp_4(stark_ctx* ctx, const uint64_t* xsets, const uint64_t* ysets, size_t rows,
                                  uint64_t* out);
/* eval_quartic<T>(p, x) (poly_utils.rs:442-446) for n (p, x) pairs: polys is
 * n x 4 coefficients, out[i] = p0 + p1 x + p2 x^2 + p3 x^3. */
stark_status stark_eval_quartic_multi(stark_ctx* ctx, const uint64_t* polys, const uint64_t* xs, size_t n,
                                      uint64_t* out);
/* Field linear combination out[i] = sum_c coeffs[c] * cols[c][i] over n_cols
 * columns of n elements (the shape of the L combination, prove.rs:287-322). */
stark_status stark_lincomb(stark_ctx* ctx, const uint64_t* cols, uint32_t n_cols, size_t n, const uint64_t* coeffs,
                           uint64_t* out);
/* Device-resident form (columns back to back at d_cols); synchronous. */
stark_status stark_lincomb_dev(stark_ctx* ctx, const uint64_t* d_cols, uint32_t n_cols, size_t n,
                               const uint64_t* coeffs, uint64_t* d_out, void* stream);

/* ---- Blake2s + index sampler (packages/fri/src/utils.rs) ------------------ */
/* blake(message) -> Vec<u8> (fri/src/utils.rs:5-10): Blake2s-256, unkeyed. */
void stark_blake(const uint8_t* msg, size_t len, uint8_t out[32]);
/* get_pseudorandom_indices(seed, modulus, count, exclude_multiples_of) (fri/src/utils.rs:82-109). */
stark_status stark_get_pseudorandom_indices(const uint8_t* seed, size_t seed_len, uint32_t modulus,
                                            size_t count, uint32_t exclude_multiples_of, uint32_t* out);

/* ---- Merkle commitment (packages/commitment/src) --------------------------
 * MerkleTree<Vec<u8>, BlakeDigest> implemented by MerkleProofInPlace
 * (merkle_tree.rs:60-73, merkle_proof_in_place.rs:9-50).  The tree lives in
 * HBM; gen_proofs does not rebuild it (the reference rebuilds on every call,
 * with identical results). */
/* MerkleProofInPlace::new (merkle_proof_in_place.rs:16-25) */
stark_status stark_merkle_new(stark_ctx* ctx, stark_merkle_tree** out);
void stark_merkle_free(stark_merkle_tree* tree);
/* update(leaves) (merkle_proof_in_place.rs:37-42) + the hashing of
 * gen_multi_proofs_multi_core (:106-189): n leaves of leaf_len bytes each,
 * packed back to back.  n must be a power of two. */
stark_status stark_merkle_update(stark_merkle_tree* tree, const uint8_t* leaves, size_t n, size_t leaf_len);
/* Same, leaves already in device memory. */
stark_status stark_merkle_update_dev(stark_merkle_tree* tree, const uint8_t* d_leaves, size_t n,
                                     size_t leaf_len, void* stream);
/* width() (merkle_tree.rs:62) */
size_t stark_merkle_width(const stark_merkle_tree* tree);
/* Bytes per leaf of the last update (0 before one): sizes gen_proofs' leaves_out for a caller
 * that, like MerkleTree::gen_proofs, does not keep the leaves (no reference counterpart). */
size_t stark_merkle_leaf_len(const stark_merkle_tree* tree);
/* get_root() (merkle_tree.rs:66): *root_len = 32, or 0 before the first
 * gen_proofs (the reference's H::default() = empty digest, :19). */
stark_status stark_merkle_get_root(const stark_merkle_tree* tree, uint8_t root[32], size_t* root_len);
/* gen_proofs(indices) -> Vec<Proof> (merkle_tree.rs:72, merkle_proof_in_place.rs:44-49):
 * for each of the k indices (caller order, duplicates allowed) writes the leaf
 * (leaf_len bytes) to leaves_out + i*leaf_len and log2(n) sibling digests
 * leaf->root to nodes_out + i*log2(n)*32.  Either output may be NULL when
 * k == 0.  Sets the root returned by get_root. */
stark_status stark_merkle_gen_proofs(stark_merkle_tree* tree, const size_t* indices, size_t k,
                                     uint8_t* leaves_out, uint8_t* nodes_out);
/* verify_multi_branch / Proof::validate (merkle_tree.rs:25-58), host side:
 * returns STARK_OK when every path hashes to root. */
stark_status stark_merkle_verify(const uint8_t root[32], const size_t* indices, size_t k,
                                 const uint8_t* leaves, size_t leaf_len, const uint8_t* nodes, size_t depth);

/* ---- FRI (packages/fri/src/fri.rs) ---------------------------------------- */
/* prove_low_degree<T, H=BlakeDigest>(values, root_of_unity, max_deg_plus_1,
 * exclude_multiples_of) -> Vec<FriProof<H>> (fri.rs:46-224).  n = len(values)
 * must equal the (power-of-two) order of root_of_unity. */
stark_status stark_prove_low_degree(stark_ctx* ctx, const uint64_t* values, size_t n, const uint64_t root[4],
                                    size_t max_deg_plus_1, uint32_t exclude_multiples_of,
                                    stark_fri_proof** out);
/* Same with values already in device memory (not modified). */
stark_status stark_prove_low_degree_dev(stark_ctx* ctx, const uint64_t* d_values, size_t n,
                                        const uint64_t root[4], size_t max_deg_plus_1,
                                        uint32_t exclude_multiples_of, stark_fri_proof** out);
void stark_fri_proof_free(stark_fri_proof* proof);
/* serde_json (compact) encoding of Vec<FriProof<BlakeDigest>> (fri.rs:16-26).
 * Writes up to cap bytes (NUL-terminated if room) and the full length to *len. */
stark_status stark_fri_proof_json(const stark_fri_proof* proof, char* buf, size_t cap, size_t* len);
/* Structured access: number of FriProof entries (Middle... then one Last). */
size_t stark_fri_proof_num_layers(const stark_fri_proof* proof);
/* Layer i: *is_last, root2 (Middle), number of column / poly branches, depth of each. */
stark_status stark_fri_proof_layer_info(const stark_fri_proof* proof, size_t i, int* is_last, uint8_t root2[32],
                                        size_t* n_column, size_t* column_depth, size_t* n_poly,
                                        size_t* poly_depth, size_t* n_last);
/* Layer i's bytes (any pointer may be NULL): n_column 32-B column leaves and n_column x column_depth
 * 32-B siblings (leaf to root), the same for the n_poly poly openings, and n_last 32-B values of the
 * Last entry -- everything a caller needs to build FriProof<H> values itself (fri.rs:16-26) without
 * going through serde.  Each non-NULL output comes with its capacity in bytes; the sizes it needs are
 * (from stark_fri_proof_layer_info) column_leaves 32 n_column, column_nodes 32 n_column column_depth,
 * poly_leaves 32 n_poly, poly_nodes 32 n_poly poly_depth, last_values 32 n_last.  A capacity below
 * that is STARK_ERR_BAD_LENGTH, and then no output is written. */
stark_status stark_fri_proof_layer_data(const stark_fri_proof* proof, size_t i, uint8_t* column_leaves,
                                        size_t column_leaves_cap, uint8_t* column_nodes, size_t column_nodes_cap,
                                        uint8_t* poly_leaves, size_t poly_leaves_cap, uint8_t* poly_nodes,
                                        size_t poly_nodes_cap, uint8_t* last_values, size_t last_values_cap);

/* ---- R1CS STARK prover (packages/r1cs-stark) -------------------------------- */
/* mk_r1cs_proof<Fp, BlakeDigest>(witness_trace, computational_trace, public_wires,
 * public_first_indices, permuted_indices, coefficients, flag0, flag1, flag2,
 * n_constraints, n_wires) -> StarkProof (prove.rs:14-378), resident on the GPU.
 * Step vectors have original_steps elements (canonical u64[4] each);
 * public_first_indices holds n_public_first (wire k, trace position w) pairs.
 * Returns STARK_ERR_CHECK where the reference's D/B asserts would panic. */
stark_status stark_mk_r1cs_proof(stark_ctx* ctx, const uint64_t* witness_trace, const uint64_t* computational_trace,
                                 size_t original_steps, const uint64_t* public_wires, size_t n_public,
                                 const size_t* public_first_indices, size_t n_public_first,
                                 const size_t* permuted_indices, const uint64_t* coefficients,
                                 const uint64_t* flag0, const uint64_t* flag1, const uint64_t* flag2,
                                 size_t n_constraints, size_t n_wires, stark_r1cs_proof** out);
/* serde_json::to_string(&StarkProof<BlakeDigest>) (utils.rs:122-130, run.rs:549). */
stark_status stark_r1cs_proof_json(const stark_r1cs_proof* proof, char* buf, size_t cap, size_t* len);
/* The same text without a copy: *data points into the proof (NUL-terminated, *len bytes) and stays
 * valid until stark_r1cs_proof_free(proof). */
stark_status stark_r1cs_proof_json_view(const stark_r1cs_proof* proof, const char** data, size_t* len);
stark_status stark_r1cs_proof_roots(const stark_r1cs_proof* proof, uint8_t m_root[32], uint8_t l_root[32],
                                    uint8_t a_root[32]);
/* StarkProof's openings (utils.rs:122-130): which = 0 main_branches (k = 320, 256-B leaves),
 * 1 linear_comb_branches (k = 80, 32-B leaves); leaves k x leaf_len bytes, nodes k x depth x 32 bytes
 * (siblings leaf to root).  Any output pointer may be NULL (query the sizes first); leaves_cap and
 * nodes_cap are the byte capacities of the two buffers, and one below k x leaf_len (resp.
 * k x depth x 32) is STARK_ERR_BAD_LENGTH with neither buffer written. */
stark_status stark_r1cs_proof_branches(const stark_r1cs_proof* proof, int which, size_t* k, size_t* leaf_len,
                                       size_t* depth, uint8_t* leaves, size_t leaves_cap, uint8_t* nodes,
                                       size_t nodes_cap);
/* StarkProof's fri_proof, borrowed (valid until stark_r1cs_proof_free); read it with the
 * stark_fri_proof_* accessors. */
const stark_fri_proof* stark_r1cs_proof_fri(const stark_r1cs_proof* proof);
void stark_r1cs_proof_free(stark_r1cs_proof* proof);

/* R1CS front end (host): read_r1cs (circom2bellman_core/src/reader.rs:4-89) +
 * read_witness (r1cs-stark/src/reader.rs:7-42) + the trace construction of
 * prove_with_witness (run.rs:310-437: calc_coefficients_and_witness :109-281,
 * calc_flags :283-308, permuted indices :388-401, public_first_indices :411-419).
 * STARK_ERR_BAD_ARG on a malformed file, a prime other than BN254 r
 * (run.rs:344-350) or witness[0] != 1 (run.rs:358). */
stark_status stark_r1cs_trace_build(const uint8_t* r1cs, size_t r1cs_len, const uint8_t* wtns, size_t wtns_len,
                                    stark_r1cs_trace** out);
stark_status stark_r1cs_trace_dims(const stark_r1cs_trace* trace, size_t* original_steps, size_t* n_public,
                                   size_t* n_public_first, size_t* n_constraints, size_t* n_wires);
/* Copies the mk_r1cs_proof arguments out (any pointer may be NULL). */
stark_status stark_r1cs_trace_export(const stark_r1cs_trace* trace, uint64_t* witness_trace,
                                     uint64_t* computational_trace, uint64_t* coefficients, uint64_t* flag0,
                                     uint64_t* flag1, uint64_t* flag2, size_t* permuted_indices,
                                     uint64_t* public_wires, size_t* public_first_indices);
void stark_r1cs_trace_free(stark_r1cs_trace* trace);
/* prove_with_witness (run.rs:310-452) = stark_mk_r1cs_proof on a built trace. */
stark_status stark_prove_r1cs_trace(stark_ctx* ctx, const stark_r1cs_trace* trace, stark_r1cs_proof** out);
/* prove_with_witness (run.rs:310-452) with the trace built on the GPU: the raw
 * .r1cs / .wtns bytes are parsed (headers and record counts on the host), the
 * trace columns, flags and permutation are constructed in HBM and proved in
 * place.  The proof is identical to stark_r1cs_trace_build +
 * stark_prove_r1cs_trace on the same bytes. */
stark_status stark_prove_r1cs_bytes(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len, const uint8_t* wtns,
                                    size_t wtns_len, stark_r1cs_proof** out);

/* Prove many witnesses of one circuit: stark_r1cs_circuit_new does, once, all of
 * prove_with_witness that depends on the .r1cs alone (slot layout, coefficients,
 * flags, permutation, public first uses, and the LDEs of K, F0-F2, IDX, PIDX);
 * stark_prove_r1cs_circuit then builds the witness columns and extends only S, P
 * and A.  The proof equals stark_prove_r1cs_bytes on the same bytes.  A circuit
 * is bound to the context that prepared it. */
stark_status stark_r1cs_circuit_new(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len, stark_r1cs_circuit** out);
void stark_r1cs_circuit_free(stark_r1cs_circuit* circuit);
stark_status stark_prove_r1cs_circuit(stark_ctx* ctx, const stark_r1cs_circuit* circuit, const uint8_t* wtns,
                                      size_t wtns_len, stark_r1cs_proof** out);

/* ---- multi-GPU four-step NTT building blocks (no reference counterpart;
 * the reference is single-process).  The exchanges are RCCL
 * all-to-alls issued by the caller; see stark-pure-rust_amd/stark_amd/distributed.py. */
/* dst[c][r] = src[r][c] for `batch` row-major rows x cols matrices of elements. */
stark_status stark_transpose_dev(stark_ctx* ctx, const uint64_t* d_src, uint64_t* d_dst, size_t rows, size_t cols,
                                 uint32_t batch, void* stream);
/* d_data[i][j] *= root^((row_base + i) * (col_base + j)) for a rows x cols matrix;
 * root must be a primitive 2^log_order-th root of unity. */
stark_status stark_twiddle2d_dev(stark_ctx* ctx, uint64_t* d_data, size_t rows, size_t cols, uint64_t row_base,
                                 uint64_t col_base, const uint64_t root[4], uint32_t log_order, void* stream);

/* In-place small DFTs across a stride: for each i < stride, the 2^log_g points
 * d[i + stride*j] become sum_j d[i + stride*j] root^(j*k) (inverse: root^-1 and
 * scaled by 2^-log_g).  root is a primitive 2^log_g-th root; log_g <= 4.  This is
 * the cross-rank DFT of the one-exchange distributed NTT. */
stark_status stark_ntt_strided_dev(stark_ctx* ctx, uint64_t* d_data, uint32_t log_g, size_t stride,
                                   const uint64_t root[4], int inverse, void* stream);
/* The one-exchange distributed NTT's first step on rank `rank` of G = 2^log_g (stark_amd/distributed.py
 * cyclic_ntt; no reference counterpart: the reference's only parallelism is parallel_fft's threads,
 * fft.rs:195-251): the rank's cyclic shard of M = 2^(log_n - log_g) points (x[rank + G j]) is
 * transformed in place with root w^G, w = root of order 2^log_n, and output k is multiplied by
 * w^(rank k) in the same last pass (w^-1, and the 1/M scale, with inverse != 0).  What the all-to-all
 * then sends; stark_ntt_strided_dev finishes the transform on the receiving rank.  The twiddle table
 * (M x 32 B per rank and direction) is cached under the context's cap.  Asynchronous on `stream`. */
stark_status stark_cyclic_ntt_local_dev(stark_ctx* ctx, uint64_t* d_data, uint32_t log_n, uint32_t log_g,
                                        uint32_t rank, const uint64_t root[4], int inverse, void* stream);
/* The same, after first scaling d[i + stride*j] by tw_root^(j*(tw_base + i))
 * (tw_root a primitive 2^log_order-th root): the receiver-side twiddle of the
 * one-exchange distributed NTT, fused into its cross-rank DFT. */
stark_status stark_ntt_strided_tw_dev(stark_ctx* ctx, uint64_t* d_data, uint32_t log_g, size_t stride,
                                      const uint64_t root[4], int inverse, const uint64_t tw_root[4],
                                      uint32_t log_order, uint64_t tw_base, void* stream);

/* ---- distributed Merkle / FRI / prover building blocks ---------------------
 * (no reference counterpart: the reference prover is single-process; these let
 * `world` GPUs share one proof, see stark-pure-rust_amd/stark_amd/dprove.py.)
 * Vectors are distributed by residue class: rank r holds the points
 * r, r + world, r + 2 world, ...; world is a power of two <= 8. */
/* Leaf digests only: d_digests[i] = Blake2s(leaf i) (the level-0 nodes of
 * merkle_proof_in_place.rs:125-140), n leaves of leaf_len bytes. */
stark_status stark_merkle_leaf_digests_dev(stark_ctx* ctx, const uint8_t* d_leaves, size_t n, size_t leaf_len,
                                           uint8_t* d_digests, void* stream);
/* Builds a tree whose level 0 is given: d_digests holds `interleave` chunks of
 * n/interleave digests (chunk r = the residue class r of the leaves), so leaf
 * interleave*m + r is chunk r's m-th digest.  gen_proofs then returns the leaf
 * digest as the leaf bytes. */
stark_status stark_merkle_update_digests_dev(stark_merkle_tree* tree, const uint8_t* d_digests, size_t n,
                                             uint32_t interleave, void* stream);
/* The tree's root digest copied to device memory d_out (32 B), asynchronously on `stream`: the
 * distributed prover all-gathers subtree roots without a host round trip. */
stark_status stark_merkle_root_dev(const stark_merkle_tree* tree, uint8_t* d_out, void* stream);
/* The top of a tree split into g subtrees (merkle_proof_in_place.rs:176-180, the chunk roots hashed as
 * a tree of their own), on the device: d_roots holds the g subtree roots (g a power of two <= 1024,
 * 32 B each), d_levels receives the g - 1 digests above them level by level (the g/2 parents of the
 * roots first, the root last).  Both 16-B aligned.  Asynchronous on `stream`. */
stark_status stark_merkle_top_dev(stark_ctx* ctx, const uint8_t* d_roots, size_t g, uint8_t* d_levels,
                                  void* stream);
/* Many openings in one launch: request i gathers, for its k indices, the leaves
 * (leaf_len bytes each) and log2(n) sibling digests of `tree`, or, when tree is
 * NULL, only the rows (row_bytes each) of the device buffer d_rows (n_rows rows).
 * Either output may be NULL. */
typedef struct stark_open_req {
  stark_merkle_tree* tree;
  const uint8_t* d_rows;
  size_t row_bytes, n_rows;
  const size_t* idx;
  size_t k;
  uint8_t* leaves_out;
  uint8_t* nodes_out;
} stark_open_req;
stark_status stark_open_batch(stark_ctx* ctx, const stark_open_req* reqs, size_t n_req, void* stream);
/* One FRI fold (fri.rs:135-164) on a residue class: `values` = the layer's n
 * values at points rank + world j (n/world of them, root = the layer's root of
 * unity), `column` = the folded column's rows rank + world j (n/(4 world));
 * special_x = from_bytes_le(m_root).  Requires world | n/4. */
stark_status stark_fri_fold_dev(stark_ctx* ctx, const uint64_t* values, uint64_t* column, size_t n,
                                const uint64_t root[4], const uint8_t m_root[32], uint32_t world, uint32_t rank,
                                void* stream);
/* Same with the layer's Merkle root in device memory (d_m_root, 32 B, 4-B aligned): special_x is
 * derived on the device and nothing waits for the host (asynchronous on `stream`). */
stark_status stark_fri_fold_dev_root(stark_ctx* ctx, const uint64_t* values, uint64_t* column, size_t n,
                                     const uint64_t root[4], const uint8_t* d_m_root, uint32_t world, uint32_t rank,
                                     void* stream);
/* serde_json of StarkProof (utils.rs:122-130) from its parts. */
typedef struct stark_branches {
  const uint8_t* leaves; /* k * leaf_len bytes */
  const uint8_t* nodes;  /* k * depth * 32 bytes, leaf -> root per proof */
  size_t k, leaf_len, depth;
} stark_branches;
typedef struct stark_fri_layer_parts {
  const uint8_t* root2; /* 32 bytes */
  stark_branches column, poly;
} stark_fri_layer_parts;
stark_status stark_r1cs_proof_json_from_parts(const uint8_t m_root[32], const uint8_t l_root[32],
                                              const uint8_t a_root[32], const stark_branches* main_branches,
                                              const stark_branches* linear_comb_branches,
                                              const stark_fri_layer_parts* layers, size_t n_layers,
                                              const uint8_t* last_values, size_t n_last, char* buf, size_t cap,
                                              size_t* len);
/* mk_r1cs_proof (prove.rs:14-264) for rank `rank` of `world`: the trace set-up,
 * accumulator tree and transcript r on every rank, then this rank's residue
 * class of the precision domain: coset LDEs (no exchange: degree < steps <=
 * precision/world), A, Zb, the constraint kernel and the 256-B main-tree rows.
 * Arguments as stark_mk_r1cs_proof; work is enqueued on `stream` (NULL = the
 * context stream) and finished on return. */
stark_status stark_dprove_begin(stark_ctx* ctx, uint32_t world, uint32_t rank, const uint64_t* witness_trace,
                                const uint64_t* computational_trace, size_t original_steps,
                                const uint64_t* public_wires, size_t n_public, const size_t* public_first_indices,
                                size_t n_public_first, const size_t* permuted_indices, const uint64_t* coefficients,
                                const uint64_t* flag0, const uint64_t* flag1, const uint64_t* flag2,
                                size_t n_constraints, size_t n_wires, void* stream, stark_dprove** out);
/* The same from raw .r1cs / .wtns bytes, trace built on this GPU (as stark_prove_r1cs_bytes). */
stark_status stark_dprove_begin_bytes(stark_ctx* ctx, uint32_t world, uint32_t rank, const uint8_t* r1cs,
                                      size_t r1cs_len, const uint8_t* wtns, size_t wtns_len, void* stream,
                                      stark_dprove** out);
/* A circuit prepared for rank `rank` of `world` (as stark_r1cs_circuit_new, with this rank's
 * coset LDEs and Zb inverses), and the distributed proof of one witness with it.  The proofs
 * equal stark_dprove_begin_bytes' on the same bytes. */
stark_status stark_dprove_circuit_new(stark_ctx* ctx, uint32_t world, uint32_t rank, const uint8_t* r1cs,
                                      size_t r1cs_len, stark_r1cs_circuit** out);
stark_status stark_dprove_begin_circuit(stark_ctx* ctx, const stark_r1cs_circuit* circuit, const uint8_t* wtns,
                                        size_t wtns_len, void* stream, stark_dprove** out);
/* Sizes, g2 = 7^((p-1)/precision) (prove.rs:71-82) and a_root; STARK_ERR_CHECK
 * where the reference's D/B asserts would panic (on this rank's points). */
stark_status stark_dprove_info(stark_dprove* h, size_t* precision, size_t* n_local, size_t* original_steps,
                               uint64_t g2[4], uint8_t a_root[32]);
/* This rank's main-tree rows P|A|S|D1|D2|D3|B2|B3 (n_local x 256 B, device). */
stark_status stark_dprove_rows(stark_dprove* h, uint8_t** rows_dev);
/* k from m_root (prove.rs:274-283) and L at this rank's points (prove.rs:287-322). */
stark_status stark_dprove_lincomb(stark_dprove* h, const uint8_t m_root[32], uint64_t** l_dev);
/* Same with m_root in device memory (4-B aligned): asynchronous on the stream given at begin. */
stark_status stark_dprove_lincomb_dev(stark_dprove* h, const uint8_t* d_m_root, uint64_t** l_dev);
void stark_dprove_free(stark_dprove* h);

/* ---- device groups: one call over G GPUs (SURVEY.md 8(b) "Multi-GPU is a ctx group created once", 8(e))
 * The reference parallelises a call over the thread pool the call builds (Worker::new inside best_fft,
 * fri/src/fft.rs:332; commitment/src/multicore.rs:43-45).  A group is that pool with GPUs as its workers:
 * created once from a device list (a device may repeat: G contexts on one GPU run the same code), then
 * passed to the group entry points, which keep the reference's signatures and return what the
 * single-context calls return, bit for bit.  The members exchange data by peer copies on their own
 * streams (xGMI between devices); no collective library and no process per GPU is needed.  A group is
 * not shared between threads (it runs its members on g - 1 host threads of its own, parked between calls
 * and joined by stark_group_destroy). */
typedef struct stark_group stark_group;
typedef struct stark_group_tree stark_group_tree;
/* g = 1, 2, 4 or 8 members on devices[0..g). */
stark_status stark_group_create(const int* devices, uint32_t g, stark_group** out);
void stark_group_destroy(stark_group* group);
uint32_t stark_group_size(const stark_group* group);
/* Member i's context (owned by the group): for _dev calls and device memory on that member. */
stark_ctx* stark_group_ctx(stark_group* group, uint32_t i);
const char* stark_group_last_error(const stark_group* group);
stark_status stark_group_synchronize(stark_group* group);
/* best_fft / inv_best_fft (fft.rs:327-379) with the group as the worker pool: the one-exchange cyclic
 * NTT (member r transforms x[r + G j], one all-to-all, G-point DFTs across the received chunks);
 * transforms smaller than 2^(2 log2 G) run on member 0.  Same arguments and output as stark_best_fft. */
stark_status stark_group_best_fft(stark_group* group, const uint64_t* coeffs, size_t len, const uint64_t root[4],
                                  uint32_t log_n, uint64_t* out);
stark_status stark_group_inv_best_fft(stark_group* group, const uint64_t* evals, size_t len, const uint64_t root[4],
                                      uint32_t log_n, uint64_t* out);
/* Device-resident form: member r's d_shards[r] holds x[r + G j], j < M = 2^log_n / G (destroyed);
 * d_out[r] receives X[r c + i + M k1] at k1 c + i, k1 < G, i < c = M / G.  log_n >= 2 log2 G.
 * Asynchronous on the member contexts' streams (stark_group_synchronize). */
stark_status stark_group_ntt_dev(stark_group* group, uint64_t* const* d_shards, uint64_t* const* d_out,
                                 uint32_t log_n, const uint64_t root[4], int inverse);
/* MerkleTree<Vec<u8>, BlakeDigest> (merkle_tree.rs:60-73) over the group: member r hashes leaves
 * [r m, (r+1) m), m = n / G (n >= G; smaller trees live on member 0), its subtree root goes to
 * member 0, which hashes the top log2 G levels -- the reference's own subtree + top-tree split
 * (merkle_proof_in_place.rs:106-206), so roots and paths equal the single tree's. */
stark_status stark_group_merkle_new(stark_group* group, stark_group_tree** out);
void stark_group_merkle_free(stark_group_tree* tree);
/* update(leaves) (merkle_proof_in_place.rs:37-42): n (a power of two) leaves of leaf_len bytes. */
stark_status stark_group_merkle_update(stark_group_tree* tree, const uint8_t* leaves, size_t n, size_t leaf_len);
/* Same with the leaves in device memory: d_blocks[r] = member r's block of m leaves (d_blocks[0] = all n
 * leaves when n < G). */
stark_status stark_group_merkle_update_dev(stark_group_tree* tree, const uint8_t* const* d_blocks, size_t n,
                                           size_t leaf_len);
size_t stark_group_merkle_width(const stark_group_tree* tree);
/* get_root() / gen_proofs(indices) as stark_merkle_get_root / stark_merkle_gen_proofs. */
stark_status stark_group_merkle_get_root(const stark_group_tree* tree, uint8_t root[32], size_t* root_len);
stark_status stark_group_merkle_gen_proofs(stark_group_tree* tree, const size_t* indices, size_t k,
                                           uint8_t* leaves_out, uint8_t* nodes_out);
/* prove_with_witness (run.rs:310-452) with one proof shared by the group: member r owns
 * the precision-domain points r + G j; coset LDEs, constraints and FRI folds are local, each Merkle tree
 * is one digest all-to-all; the proof equals stark_prove_r1cs_bytes' byte for byte. */
stark_status stark_group_prove_r1cs_bytes(stark_group* group, const uint8_t* r1cs, size_t r1cs_len,
                                          const uint8_t* wtns, size_t wtns_len, stark_r1cs_proof** out);
/* The .r1cs-only work of that proof done once per member (circuits[r] on member r, G handles, freed with
 * stark_r1cs_circuit_free), and a proof of one witness with it (as stark_r1cs_circuit_new / _prove). */
stark_status stark_group_circuit_new(stark_group* group, const uint8_t* r1cs, size_t r1cs_len,
                                     stark_r1cs_circuit** circuits);
stark_status stark_group_prove_r1cs_circuit(stark_group* group, stark_r1cs_circuit* const* circuits,
                                            const uint8_t* wtns, size_t wtns_len, stark_r1cs_proof** out);

/* ---- device memory helpers (for callers without their own allocator) ------ */
stark_status stark_dev_alloc(stark_ctx* ctx, size_t bytes, void** d_ptr);
stark_status stark_dev_free(stark_ctx* ctx, void* d_ptr);
stark_status stark_memcpy_h2d(stark_ctx* ctx, void* d_dst, const void* h_src, size_t bytes);
stark_status stark_memcpy_d2h(stark_ctx* ctx, void* h_dst, const void* d_src, size_t bytes);
stark_status stark_ctx_synchronize(stark_ctx* ctx);

/* ---- Verifier (packages/fri/src/fri.rs:226-404, packages/r1cs-stark/src/verify.rs:13-258,
 * run.rs:454-526, 556-592) ------------------------------------------------------------
 * STARK_OK: the proof verifies.  STARK_ERR_CHECK: the reference would fail an assert
 * (an invalid proof).  STARK_ERR_BAD_ARG: malformed input, including a proof JSON that
 * serde_json would not parse as StarkProof<BlakeDigest>.  The circuit-only extensions
 * (K, F0-F2, IDX, PIDX over the precision domain) come from a prepared circuit on the
 * GPU; the Merkle paths, FRI layer checks and the 80 spot checks run on the host. */

/* verify_low_degree_proof (fri.rs:226-242): layers[0..n_layers) are the Middle layers,
 * last_values[i] (last_lens[i] bytes) the Last layer's values; root_of_unity canonical. */
stark_status stark_verify_low_degree_proof(const uint8_t merkle_root[32], const uint64_t root_of_unity[4],
                                           const stark_fri_layer_parts* layers, size_t n_layers,
                                           const uint8_t* const* last_values, const size_t* last_lens,
                                           size_t n_last, size_t max_deg_plus_1, uint32_t exclude_multiples_of);
/* verify_with_witness (run.rs:454-526) on a prepared circuit; public_wires = n_public
 * 32-byte little-endian integers (n_public >= 1 + n_public_inputs + n_public_outputs). */
stark_status stark_verify_r1cs_circuit(stark_ctx* ctx, const stark_r1cs_circuit* circuit,
                                       const uint8_t* public_wires, size_t n_public, const char* proof_json,
                                       size_t json_len);
/* The same from the .r1cs bytes (read_r1cs + verify_with_witness). */
stark_status stark_verify_r1cs_bytes(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len,
                                     const uint8_t* public_wires, size_t n_public, const char* proof_json,
                                     size_t json_len);
/* verify_with_file_path (run.rs:556-592) on bytes: the public wires are the first
 * 1 + n_public_inputs + n_public_outputs witness values. */
stark_status stark_verify_with_witness(stark_ctx* ctx, const uint8_t* r1cs, size_t r1cs_len, const uint8_t* wtns,
                                       size_t wtns_len, const char* proof_json, size_t json_len);

#ifdef __cplusplus
}
#endif
#endif /* STARK_HIP_H */
