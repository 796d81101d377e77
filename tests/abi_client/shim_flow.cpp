// A non-Python caller of libstark_hip.so making exactly the calls of the Rust shim in
// INTEGRATION.md, in the order packages/fri and packages/commitment make them:
//   fri::fft::best_fft (fft.rs:327)            -> stark_best_fft
//   MerkleProofInPlace::new/update/gen_proofs/get_root (merkle_proof_in_place.rs:15-50)
//                                              -> stark_merkle_new / _update / _gen_proofs / _get_root
//   fri::fri::prove_low_degree (fri.rs:46)     -> stark_prove_low_degree + stark_fri_proof_json
// Test infrastructure (tests/test_abi_client.py): reads the coefficients, root and indices the test
// wrote, writes every output, and the test compares them with the oracle.
//   usage: shim_flow <in.bin> <out_dir>
//   in.bin: u32 log_n, u32 n_coeffs, u32 k, u32 exclude; u64 root[4]; u64 coeffs[4 * n_coeffs]; u64 idx[k]
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "stark_hip.h"

static void check(stark_status rc, const char* what) {
  if (rc != STARK_OK) {  // the shim's ok(): a non-zero status is a panic
    fprintf(stderr, "%s: %s\n", what, stark_status_str(rc));
    exit(2);
  }
}

static void write_file(const std::string& path, const void* data, size_t len) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f || fwrite(data, 1, len, f) != len) {
    fprintf(stderr, "cannot write %s\n", path.c_str());
    exit(3);
  }
  fclose(f);
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: shim_flow <in.bin> <out_dir>\n");
    return 1;
  }
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 1;
  uint32_t hdr[4];
  uint64_t root[4];
  if (fread(hdr, 4, 4, f) != 4 || fread(root, 8, 4, f) != 4) return 1;
  const uint32_t log_n = hdr[0], n_coeffs = hdr[1], k = hdr[2], exclude = hdr[3];
  const size_t n = (size_t)1 << log_n;
  std::vector<uint64_t> coeffs(4 * (size_t)n_coeffs);
  std::vector<uint64_t> idx64(k);
  if (fread(coeffs.data(), 8, coeffs.size(), f) != coeffs.size() || fread(idx64.data(), 8, k, f) != k) return 1;
  fclose(f);
  const std::string out = argv[2];

  stark_ctx* ctx = nullptr;
  check(stark_ctx_create(0, &ctx), "stark_ctx_create");

  // best_fft(coefficients, &root, log_n): zero-padded to n, evaluations in natural order.
  std::vector<uint64_t> evals(4 * n);
  check(stark_best_fft(ctx, coeffs.data(), n_coeffs, root, log_n, evals.data()), "best_fft");
  write_file(out + "/evals.bin", evals.data(), evals.size() * 8);

  // MerkleProofInPlace<Vec<u8>, BlakeDigest> over the evaluations' to_bytes_le leaves.
  stark_merkle_tree* tree = nullptr;
  check(stark_merkle_new(ctx, &tree), "MerkleProofInPlace::new");
  uint8_t root_before[32];
  size_t root_len = 99;
  check(stark_merkle_get_root(tree, root_before, &root_len), "get_root");
  if (root_len != 0) return 4;  // H::default() (empty BlakeDigest) before gen_proofs
  check(stark_merkle_update(tree, (const uint8_t*)evals.data(), n, 32), "update");
  if (stark_merkle_width(tree) != n || stark_merkle_leaf_len(tree) != 32) return 5;
  std::vector<size_t> idx(idx64.begin(), idx64.end());
  std::vector<uint8_t> leaves(32 * (size_t)k), nodes(32 * (size_t)k * log_n);
  check(stark_merkle_gen_proofs(tree, idx.data(), k, leaves.data(), nodes.data()), "gen_proofs");
  uint8_t mroot[32];
  check(stark_merkle_get_root(tree, mroot, &root_len), "get_root");
  if (root_len != 32) return 6;
  check(stark_merkle_verify(mroot, idx.data(), k, leaves.data(), 32, nodes.data(), log_n), "verify_multi_branch");
  write_file(out + "/merkle_root.bin", mroot, 32);
  write_file(out + "/merkle_leaves.bin", leaves.data(), leaves.size());
  write_file(out + "/merkle_nodes.bin", nodes.data(), nodes.size());
  stark_merkle_free(tree);

  // prove_low_degree::<Fp, BlakeDigest>(&values, root, n / 4, exclude) -> serde_json.
  stark_fri_proof* proof = nullptr;
  check(stark_prove_low_degree(ctx, evals.data(), n, root, n / 4, exclude, &proof), "prove_low_degree");
  size_t len = 0;
  check(stark_fri_proof_json(proof, nullptr, 0, &len), "fri_proof_json (size)");
  std::string json(len + 1, '\0');
  check(stark_fri_proof_json(proof, &json[0], json.size(), &len), "fri_proof_json");
  write_file(out + "/fri.json", json.data(), len);
  stark_fri_proof_free(proof);
  stark_ctx_destroy(ctx);
  printf("shim_flow ok: n=%zu k=%u json=%zu B\n", n, k, len);
  return 0;
}
