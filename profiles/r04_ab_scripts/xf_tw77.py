# Transform for tools/build_variant.sh (VARIANT_FILE-free: edits ntt.hip and, through a side file, internal.h):
# the 16 x 16 twiddle tables without the e = 0 constant (77 instead of 78, 21,560 B of LDS); the lanes with
# t = 0 (w_R^0 = 1) take a masked lazy reduction instead of a product.
import os
import re

out = s  # noqa: F821  (set by build_variant.sh)
d = os.path.dirname(os.path.abspath(__import__("sys").argv[1]))
ih = os.path.join(d, "internal.h")
t = open(ih).read()
t = t.replace("constexpr uint32_t kTw16Consts = 78;", "constexpr uint32_t kTw16Consts = 77;")
open(ih, "w").write(t)


def rep(a, b):
    global out
    assert a in out, a
    out = out.replace(a, b, 1)


rep("      for (uint32_t e = 0; e < 128; ++e)\n        if (seen[e]) es.push_back(e);",
    "      for (uint32_t e = 1; e < 128; ++e)\n        if (seen[e]) es.push_back(e);")
rep("        const uint32_t idx = (uint32_t)(std::lower_bound(es.begin(), es.end(), e & 127) - es.begin());",
    "        const uint32_t idx = (e & 127) == 0 ? 0x7fu\n"
    "                             : (uint32_t)(std::lower_bound(es.begin(), es.end(), e & 127) - es.begin());")
rep("            x[k] = fe_mul_db_split(u, A, Bp);  // [0, 2p)",
    "            if (idx == 0x7fu) {\n              x[k] = v;\n              fe_csub2p(x[k]);\n"
    "            } else {\n              x[k] = fe_mul_db_split(u, A, Bp);  // [0, 2p)\n            }")
