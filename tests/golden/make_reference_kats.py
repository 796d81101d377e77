"""Writes reference_kats.json: the known-answer vectors the reference's own
unit tests hold for the hot path, transcribed as data with their source
(file:line in the reference repo).  Run once; the JSON is committed."""
import json
import os

KATS = {
    "blake": {  # packages/fri/src/utils.rs:12-24 (same in commitment/src/utils.rs:12-24)
        "source": "packages/fri/src/utils.rs:12-24",
        "vectors": [
            {"msg_hex": b"hello world".hex(),
             "digest_hex": "9aec6806794561107e594b1f6a8a6b0c92a0cba9acf5e5e93cca06f781813b0b"},
            {"msg_hex": "9aec6806794561107e594b1f6a8a6b0c92a0cba9acf5e5e93cca06f781813b0b",
             "digest_hex": "8ea974646c2be3c16f9f52a2e5ebb3d2df7ba184a6440e47fc6fcce6e9d9bdc4"},
        ],
    },
    "pseudorandom_indices": {  # packages/fri/src/utils.rs:111-120
        "source": "packages/fri/src/utils.rs:111-120",
        "vectors": [
            {"seed_msg": "hello world", "modulus": 7, "count": 5, "exclude": 0, "out": [5, 5, 5, 3, 5]},
            {"seed_msg": "hello another world", "modulus": 7, "count": 20, "exclude": 0,
             "out": [3, 0, 2, 4, 4, 1, 4, 2, 5, 1, 3, 2, 1, 0, 0, 1, 6, 5, 2, 3]},
        ],
    },
    "merkle_16": {  # packages/commitment/src/pallarel_merkle_tree.rs:132-179
        "source": "packages/commitment/src/pallarel_merkle_tree.rs:132-179",
        "leaves_hex": ["7fffffff", "80000000", "00000003", "00000000", "7ffffffe", "80000001", "00000004",
                       "00000001", "7ffffffd", "80000002", "00000005", "00000002", "7ffffffc", "80000003",
                       "00000006", "00000003"],
        "root_hex": "9f04496db6a8c505e88a7db289161a540a0cb953ef81c9b86103f0d6d12e8e15",
        "index": 2,
        "leaf_hex": "00000003",
        "nodes_hex": ["4cd90cc0d54239ee5b3fd9989b4ef4cbebbbdd08410758cbd2d291fa364c82d5",
                      "2e3d3579213e0a992d60b503f1d8fe331b8bd548e227e8dbd741ca1752077b84",
                      "9a8c87bb98f1b2e0f7036a27a343dc8fd649bedc737093c2080a34c6b9f6f375",
                      "ef459d75e20ce2f3fc4378ff20fe2d594fbcf16cccd986c2e0d3df41bd3bbe44"],
    },
    "merkle_4096": {  # packages/commitment/src/pallarel_merkle_tree.rs:181-216
        "source": "packages/commitment/src/pallarel_merkle_tree.rs:181-216",
        "leaf_hex": "7fffffff",
        "n": 4096,
        "indices": [2, 7, 13],
        "root_hex": "a0d91c3115f9e4d9f142e7cb2f413c10f0f2f9f65d9f918b80f852f9ebc06ebc",
        "proof0_node0_hex": "b72b5371ceffa4e01aa1849cdb8705406e14791db359f826bc01a392ed26b6b9",
    },
    "merkle_multi_core": {  # packages/commitment/src/merkle_proof_in_place.rs:208-259
        "source": "packages/commitment/src/merkle_proof_in_place.rs:208-259",
        "leaves": "hex::decode(format!(\"{:08x}\", i)) for i in 0..16",
        "cpus": 4,
        "indices": [10, 4, 6, 3, 6, 8],
    },
    "fp_codec": {  # packages/ff_utils/src/fp.rs:27-68
        "source": "packages/ff_utils/src/fp.rs:27-68",
        "value": 31,
        "hex": "%064x" % 31,
        "bytes_be": [0] * 31 + [31],
        "bytes_le": [31] + [0] * 31,
    },
    "multi_inv_f7": {  # packages/fri/src/poly_utils.rs:72-91 (toy field F7)
        "source": "packages/fri/src/poly_utils.rs:72-91",
        "p": 7,
        "vectors": [
            {"in": [1, 3, 2, 6, 4, 5], "out": [1, 5, 4, 6, 2, 3]},
            {"in": [0, 1, 5, 4, 0, 6, 2, 3, 0], "out": [0, 1, 3, 2, 0, 6, 4, 5, 0]},
        ],
    },
    "expand_root_f7": {  # packages/fri/src/fft.rs:16-41
        "source": "packages/fri/src/fft.rs:16-41",
        "p": 7, "root": 3, "out": [1, 3, 2, 6, 4, 5],
        "bn254_order_65536_len": 65536,
    },
    "simple_ft_f7": {  # packages/fri/src/fft.rs:84-99 (_simple_ft over F7, roots [1,2,4])
        "source": "packages/fri/src/fft.rs:84-99",
        "p": 7, "roots": [1, 2, 4],
        "vectors": [{"in": [1, 2, 0], "out": [3, 5, 2]}, {"in": [0, 1, 1, 0], "out": [2, 6, 6]}],
    },
    "parse_bytes_to_u64_vec": {  # packages/fri/src/utils.rs:148-154
        "source": "packages/fri/src/utils.rs:148-154",
        "in": [1, 1, 0, 0, 0, 0, 0, 0, 255, 0], "out": [257, 255],
    },
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "reference_kats.json")
    with open(out, "w") as f:
        json.dump(KATS, f, indent=1)
    print("wrote", out)
