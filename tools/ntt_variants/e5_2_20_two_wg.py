# Variant E5 (round 6, timing only, built but not yet measured: the GPU pool had no box): 2^20's passes capped at
# two workgroups per CU by raising the launch's dynamic LDS to 56 KB (OCC=last: the last pass only), to test whether
# two full rounds beat 1.33 rounds at three per CU (profiles/r06_ntt_2_20_pass_trace.txt).
# usage: OCC=all|last tools/build_variant.sh ab/occ.so @tools/ntt_variants/e5_2_20_two_wg.py
import os
def apply(s):
    old = "    const size_t lds = (image + db_lds_fe(lr, col)) * sizeof(fe);\n"
    assert s.count(old) == 1
    cond = "log_n == 20" + (" && last" if os.environ["OCC"] == "last" else "")
    new = ("    size_t lds = (image + db_lds_fe(lr, col)) * sizeof(fe);\n"
           f"    if ({cond} && lds < 56 * 1024) lds = 56 * 1024;\n")
    return s.replace(old, new)
