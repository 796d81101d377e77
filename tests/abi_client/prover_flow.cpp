// A non-Python caller of libstark_hip.so making the calls of INTEGRATION.md section 5's Rust shim of
// the whole prover, in the order r1cs-stark makes them:
//   run.rs:310-452 prove_with_witness on raw bytes  -> stark_prove_r1cs_bytes
//   prove.rs:14 mk_r1cs_proof on trace vectors      -> stark_r1cs_trace_build / _export (the reference's
//                                                      read_r1cs + run.rs trace) + stark_mk_r1cs_proof
// and builds StarkProof (utils.rs:122-130) from the library's structured parts -- roots, branches,
// FRI layers -- the way the shim builds a StarkProof<H> value with H::from_blake2s and no serde:
//   stark_r1cs_proof_roots / _branches / _fri, stark_fri_proof_num_layers / _layer_info / _layer_data.
// Test infrastructure (tests/test_abi_client.py): writes three JSON texts -- the library's own
// serialisation of each route and this program's rendering of the parts (serde_json's compact
// encoding of StarkProof<BlakeDigest>) -- which the test compares with the golden digests.
//   usage: prover_flow <file.r1cs> <file.wtns> <out_dir>
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

static void write_file(const std::string& path, const std::string& s) {
  FILE* f = fopen(path.c_str(), "wb");
  if (!f || fwrite(s.data(), 1, s.size(), f) != s.size()) {
    fprintf(stderr, "cannot write %s\n", path.c_str());
    exit(3);
  }
  fclose(f);
}

// serde_json compact encodings: Vec<u8> / BlakeDigest(Vec<u8>) as a number array, Proof<Vec<u8>, H> as
// {"leaf":[..],"nodes":[[..],..]} (merkle_tree.rs:14-18).
static void bytes(std::string& o, const uint8_t* p, size_t n) {
  o += '[';
  for (size_t i = 0; i < n; ++i) {
    if (i) o += ',';
    o += std::to_string(p[i]);
  }
  o += ']';
}

static void branches(std::string& o, const std::vector<uint8_t>& leaves, size_t leaf_len,
                     const std::vector<uint8_t>& nodes, size_t k, size_t depth) {
  o += '[';
  for (size_t i = 0; i < k; ++i) {
    if (i) o += ',';
    o += "{\"leaf\":";
    bytes(o, &leaves[i * leaf_len], leaf_len);
    o += ",\"nodes\":[";
    for (size_t d = 0; d < depth; ++d) {
      if (d) o += ',';
      bytes(o, &nodes[(i * depth + d) * 32], 32);
    }
    o += "]}";
  }
  o += ']';
}

// Vec<FriProof<H>> (fri.rs:16-26, externally tagged enum) from the structured accessors.
static void fri_proof(std::string& o, const stark_fri_proof* p) {
  const size_t n = stark_fri_proof_num_layers(p);
  o += '[';
  for (size_t i = 0; i < n; ++i) {
    int is_last = 0;
    uint8_t root2[32];
    size_t nc = 0, cd = 0, np = 0, pd = 0, nl = 0;
    check(stark_fri_proof_layer_info(p, i, &is_last, root2, &nc, &cd, &np, &pd, &nl), "fri layer info");
    std::vector<uint8_t> cl(32 * nc), cn(32 * nc * cd), pl(32 * np), pn(32 * np * pd), last(32 * nl);
    // a buffer one byte short must be refused untouched (capacity check), the exact sizes accepted
    if (!cl.empty() && stark_fri_proof_layer_data(p, i, cl.data(), cl.size() - 1, nullptr, 0, nullptr, 0, nullptr, 0,
                                                  nullptr, 0) != STARK_ERR_BAD_LENGTH) {
      fprintf(stderr, "stark_fri_proof_layer_data: short buffer accepted\n");
      exit(1);
    }
    check(stark_fri_proof_layer_data(p, i, cl.data(), cl.size(), cn.data(), cn.size(), pl.data(), pl.size(),
                                     pn.data(), pn.size(), last.data(), last.size()),
          "fri layer data");
    if (i) o += ',';
    if (is_last) {
      o += "{\"Last\":{\"last\":[";
      for (size_t j = 0; j < nl; ++j) {
        if (j) o += ',';
        bytes(o, &last[32 * j], 32);
      }
      o += "]}}";
    } else {
      o += "{\"Middle\":{\"root2\":";
      bytes(o, root2, 32);
      o += ",\"column_branches\":";
      branches(o, cl, 32, cn, nc, cd);
      o += ",\"poly_branches\":";
      branches(o, pl, 32, pn, np, pd);
      o += "}}";
    }
  }
  o += ']';
}

// StarkProof<H> (utils.rs:122-130) from the parts.
static std::string from_parts(const stark_r1cs_proof* p) {
  uint8_t m[32], l[32], a[32];
  check(stark_r1cs_proof_roots(p, m, l, a), "roots");
  std::string o = "{\"m_root\":";
  bytes(o, m, 32);
  o += ",\"l_root\":";
  bytes(o, l, 32);
  o += ",\"a_root\":";
  bytes(o, a, 32);
  for (int which = 0; which < 2; ++which) {
    size_t k = 0, ll = 0, depth = 0;
    check(stark_r1cs_proof_branches(p, which, &k, &ll, &depth, nullptr, 0, nullptr, 0), "branches (sizes)");
    std::vector<uint8_t> leaves(k * ll), nodes(k * depth * 32);
    if (stark_r1cs_proof_branches(p, which, &k, &ll, &depth, leaves.data(), leaves.size(), nodes.data(),
                                  nodes.size() - 1) != STARK_ERR_BAD_LENGTH) {
      fprintf(stderr, "stark_r1cs_proof_branches: short buffer accepted\n");
      exit(1);
    }
    check(stark_r1cs_proof_branches(p, which, &k, &ll, &depth, leaves.data(), leaves.size(), nodes.data(),
                                    nodes.size()),
          "branches");
    o += which == 0 ? ",\"main_branches\":" : ",\"linear_comb_branches\":";
    branches(o, leaves, ll, nodes, k, depth);
  }
  o += ",\"fri_proof\":";
  const stark_fri_proof* fri = stark_r1cs_proof_fri(p);
  if (!fri) {
    fprintf(stderr, "stark_r1cs_proof_fri: null\n");
    exit(4);
  }
  fri_proof(o, fri);
  o += '}';
  return o;
}

static std::string lib_json(const stark_r1cs_proof* p) {
  size_t len = 0;
  check(stark_r1cs_proof_json(p, nullptr, 0, &len), "r1cs_proof_json (size)");
  std::string s(len + 1, '\0');
  check(stark_r1cs_proof_json(p, &s[0], s.size(), &len), "r1cs_proof_json");
  s.resize(len);
  return s;
}

int main(int argc, char** argv) {
  if (argc != 4) {
    fprintf(stderr, "usage: prover_flow <file.r1cs> <file.wtns> <out_dir>\n");
    return 1;
  }
  const std::vector<uint8_t> r1cs = read_file(argv[1]), wtns = read_file(argv[2]);
  const std::string out = argv[3];
  stark_ctx* ctx = nullptr;
  check(stark_ctx_create(0, &ctx), "stark_ctx_create");

  // prove_with_witness (run.rs:310-452) on the raw bytes.
  stark_r1cs_proof* p = nullptr;
  check(stark_prove_r1cs_bytes(ctx, r1cs.data(), r1cs.size(), wtns.data(), wtns.size(), &p), "prove_with_witness");
  write_file(out + "/bytes.json", lib_json(p));
  write_file(out + "/bytes_parts.json", from_parts(p));
  stark_r1cs_proof_free(p);

  // mk_r1cs_proof (prove.rs:14) on the trace vectors, the arguments the reference's prove_with_witness
  // passes it (run.rs:437-452).
  stark_r1cs_trace* tr = nullptr;
  check(stark_r1cs_trace_build(r1cs.data(), r1cs.size(), wtns.data(), wtns.size(), &tr), "trace build");
  size_t os = 0, n_pub = 0, n_pfi = 0, n_c = 0, n_w = 0;
  check(stark_r1cs_trace_dims(tr, &os, &n_pub, &n_pfi, &n_c, &n_w), "trace dims");
  std::vector<uint64_t> wit(4 * os), comp(4 * os), coef(4 * os), f0(4 * os), f1(4 * os), f2(4 * os);
  std::vector<uint64_t> pub(4 * (n_pub ? n_pub : 1));
  std::vector<size_t> perm(os), pfi(2 * (n_pfi ? n_pfi : 1));
  check(stark_r1cs_trace_export(tr, wit.data(), comp.data(), coef.data(), f0.data(), f1.data(), f2.data(),
                                perm.data(), pub.data(), pfi.data()),
        "trace export");
  stark_r1cs_trace_free(tr);
  check(stark_mk_r1cs_proof(ctx, wit.data(), comp.data(), os, pub.data(), n_pub, pfi.data(), n_pfi, perm.data(),
                            coef.data(), f0.data(), f1.data(), f2.data(), n_c, n_w, &p),
        "mk_r1cs_proof");
  write_file(out + "/mk.json", lib_json(p));
  write_file(out + "/mk_parts.json", from_parts(p));
  stark_r1cs_proof_free(p);
  stark_ctx_destroy(ctx);
  printf("prover_flow ok: original_steps=%zu\n", os);
  return 0;
}
