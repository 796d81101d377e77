// A non-Python caller of the device-group entry points (include/stark_hip.h stark_group_*), making the
// calls INTEGRATION.md section 6's Rust shim makes when a group exists:
//   best_fft / inv_best_fft (fft.rs:327-379)              -> stark_group_best_fft / _inv_best_fft
//   MerkleProofInPlace update / gen_proofs / get_root      -> stark_group_merkle_*
//     (merkle_tree.rs:60-73)
//   prove_with_witness (run.rs:310-452)                    -> stark_group_prove_r1cs_bytes, and the
//                                                             prepared-circuit form
// on a group of G members (all on device 0 unless STARK_GROUP_DEVICES lists them, e.g. "0,1,2,3").
// Test infrastructure (tests/test_abi_client.py): writes the outputs for the test to compare with the
// oracle and the golden digests.
//   usage: group_flow <G> <in.bin> <file.r1cs> <file.wtns> <out_dir>
//   in.bin: u32 log_n, u32 len, u32 k, u32 unused; root (4 x u64); len coefficients (4 x u64 each);
//           k u64 leaf indices.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "stark_hip.h"

static stark_group* g_group = nullptr;

static void check(stark_status rc, const char* what) {
  if (rc != STARK_OK) {
    fprintf(stderr, "%s: %s (%s)\n", what, stark_status_str(rc), g_group ? stark_group_last_error(g_group) : "");
    exit(2);
  }
}

static std::vector<uint8_t> read_file(const char* path) {
  FILE* f = fopen(path, "rb");
  if (!f) {
    fprintf(stderr, "cannot read %s\n", path);
    exit(3);
  }
  std::vector<uint8_t> b;
  uint8_t buf[1 << 16];
  size_t k;
  while ((k = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + k);
  fclose(f);
  return b;
}

static void write_file(const std::string& path, const void* p, size_t n) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f || fwrite(p, 1, n, f) != n) {
    fprintf(stderr, "cannot write %s\n", path.c_str());
    exit(3);
  }
  fclose(f);
}

static void write_proof(const std::string& path, const stark_r1cs_proof* p) {
  size_t len = 0;
  check(stark_r1cs_proof_json(p, nullptr, 0, &len), "r1cs_proof_json (size)");
  std::string s(len + 1, '\0');
  check(stark_r1cs_proof_json(p, &s[0], s.size(), &len), "r1cs_proof_json");
  write_file(path, s.data(), len);
}

int main(int argc, char** argv) {
  if (argc != 6) {
    fprintf(stderr, "usage: group_flow <G> <in.bin> <file.r1cs> <file.wtns> <out_dir>\n");
    return 1;
  }
  if (stark_abi_version() != STARK_ABI_VERSION) {
    fprintf(stderr, "library ABI %u, header %u\n", stark_abi_version(), STARK_ABI_VERSION);
    return 1;
  }
  const uint32_t G = (uint32_t)atoi(argv[1]);
  std::vector<int> devices(G, 0);
  if (const char* list = getenv("STARK_GROUP_DEVICES")) {
    const char* p = list;
    for (uint32_t i = 0; i < G && *p; ++i) {
      devices[i] = atoi(p);
      while (*p && *p != ',') ++p;
      if (*p == ',') ++p;
    }
  }
  const std::vector<uint8_t> in = read_file(argv[2]);
  const std::vector<uint8_t> r1cs = read_file(argv[3]), wtns = read_file(argv[4]);
  const std::string out = argv[5];
  uint32_t hdr[4];
  memcpy(hdr, in.data(), 16);
  const uint32_t log_n = hdr[0], len = hdr[1], k = hdr[2];
  const size_t n = (size_t)1 << log_n;
  uint64_t root[4];
  memcpy(root, in.data() + 16, 32);
  std::vector<uint64_t> coeffs(4 * (size_t)len);
  memcpy(coeffs.data(), in.data() + 48, 32 * (size_t)len);
  std::vector<size_t> idx(k);
  for (uint32_t i = 0; i < k; ++i) {
    uint64_t v;
    memcpy(&v, in.data() + 48 + 32 * (size_t)len + 8 * i, 8);
    idx[i] = (size_t)v;
  }

  check(stark_group_create(devices.data(), G, &g_group), "stark_group_create");
  if (stark_group_size(g_group) != G || !stark_group_ctx(g_group, G - 1)) {
    fprintf(stderr, "group size / member context\n");
    return 1;
  }

  // best_fft then inv_best_fft of the evaluations (the padded coefficients back)
  std::vector<uint64_t> evals(4 * n), back(4 * n);
  check(stark_group_best_fft(g_group, coeffs.data(), len, root, log_n, evals.data()), "group best_fft");
  check(stark_group_inv_best_fft(g_group, evals.data(), n, root, log_n, back.data()), "group inv_best_fft");
  write_file(out + "/evals.bin", evals.data(), 32 * n);
  write_file(out + "/inv.bin", back.data(), 32 * n);

  // MerkleTree over the evaluations as 32-B leaves (the FRI / L tree shape)
  stark_group_tree* t = nullptr;
  check(stark_group_merkle_new(g_group, &t), "group merkle new");
  check(stark_group_merkle_update(t, (const uint8_t*)evals.data(), n, 32), "group merkle update");
  uint8_t mroot[32];
  size_t rl = 1;
  check(stark_group_merkle_get_root(t, mroot, &rl), "group get_root");
  if (rl != 0) {  // H::default() before gen_proofs (merkle_tree.rs:19, 66)
    fprintf(stderr, "root before gen_proofs\n");
    return 1;
  }
  std::vector<uint8_t> leaves(32 * (size_t)k + 1), nodes(32 * (size_t)k * log_n + 1);
  check(stark_group_merkle_gen_proofs(t, idx.data(), k, leaves.data(), nodes.data()), "group gen_proofs");
  check(stark_group_merkle_get_root(t, mroot, &rl), "group get_root");
  write_file(out + "/merkle_root.bin", mroot, 32);
  write_file(out + "/merkle_leaves.bin", leaves.data(), 32 * (size_t)k);
  write_file(out + "/merkle_nodes.bin", nodes.data(), 32 * (size_t)k * log_n);
  check(stark_merkle_verify(mroot, idx.data(), k, leaves.data(), 32, nodes.data(), log_n), "verify_multi_branch");
  stark_group_merkle_free(t);

  // prove_with_witness, cold and from circuits prepared on every member
  stark_r1cs_proof* p = nullptr;
  check(stark_group_prove_r1cs_bytes(g_group, r1cs.data(), r1cs.size(), wtns.data(), wtns.size(), &p),
        "group prove_with_witness");
  write_proof(out + "/proof.json", p);
  stark_r1cs_proof_free(p);
  std::vector<stark_r1cs_circuit*> circ(G, nullptr);
  check(stark_group_circuit_new(g_group, r1cs.data(), r1cs.size(), circ.data()), "group circuit_new");
  check(stark_group_prove_r1cs_circuit(g_group, circ.data(), wtns.data(), wtns.size(), &p), "group prove circuit");
  write_proof(out + "/proof_circuit.json", p);
  stark_r1cs_proof_free(p);
  for (stark_r1cs_circuit* c : circ) stark_r1cs_circuit_free(c);
  stark_group_destroy(g_group);
  return 0;
}
