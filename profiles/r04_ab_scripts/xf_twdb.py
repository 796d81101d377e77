# Timing-only transform of csrc/ntt.hip (tools/build_variant.sh): the 16 x 16 passes' internal twiddles
# by the digit-basis product from an LDS table of TW_ENTRIES constants (w_R^(e mod TW_ENTRIES): WRONG
# results unless TW_ENTRIES covers every e -- it prices the product form and the LDS size, nothing else),
# with the 4p - a input negation for r1 > 8 and an extra STARK_LDS_PAD bytes of LDS per workgroup.
import os

n = int(os.environ.get("TW_ENTRIES", "64"))
out = s  # noqa: F821  (set by build_variant.sh)


def rep(a, b):
    global out
    assert a in out, a
    out = out.replace(a, b, 1)


rep("  static constexpr uint32_t stride = 4;             // the table holds w_R^(4 k), k < R / 8\n"
    "  static constexpr uint32_t entries = (on && !four) ? (1u << LOG_R) / (2 * stride) : 0;",
    "  static constexpr bool twdb = four && LOG_R == 8 && COL != kColSparse;\n"
    "  static constexpr uint32_t stride = twdb ? 1 : 4;\n"
    f"  static constexpr uint32_t entries = (on && !four) ? (1u << LOG_R) / (2 * stride) : twdb ? {n} : 0;")
rep("static constexpr uint32_t shoup_fe = last ? 0 : four ? 2 * (1u << LOG_R) : (1u << LOG_R);",
    "static constexpr uint32_t shoup_fe = last ? 0 : four ? (twdb ? 0 : 2 * (1u << LOG_R)) : (1u << LOG_R);")
rep("        x[k] = fe_mul_shoup(v, sm[2 * e], sm[2 * e + 1]);                      // [0, 2p)",
    """        if constexpr (DB::twdb) {
          const uint32_t r1 = __builtin_bitreverse32((a << 2) + k) >> 28;
          fe u = v;
          if (r1 > 8) {
            fe d;
            asm("v_sub_co_u32 %0, vcc, %8, %16\\n\\t"
                "v_subb_co_u32 %1, vcc, %9, %17, vcc\\n\\t"
                "v_subb_co_u32 %2, vcc, %10, %18, vcc\\n\\t"
                "v_subb_co_u32 %3, vcc, %11, %19, vcc\\n\\t"
                "v_subb_co_u32 %4, vcc, %12, %20, vcc\\n\\t"
                "v_subb_co_u32 %5, vcc, %13, %21, vcc\\n\\t"
                "v_subb_co_u32 %6, vcc, %14, %22, vcc\\n\\t"
                "v_subb_co_u32 %7, vcc, %15, %23, vcc"
                : "=&v"(d.w[0]), "=&v"(d.w[1]), "=&v"(d.w[2]), "=&v"(d.w[3]), "=&v"(d.w[4]), "=&v"(d.w[5]),
                  "=&v"(d.w[6]), "=&v"(d.w[7])
                : "v"(0xc0000004u), "v"(0x0f87d64fu), "v"(0xe6e5c245u), "v"(0xa0cfa121u), "v"(0x06056174u),
                  "v"(0xe14116dau), "v"(0x84c680a6u), "v"(0xc19139cbu), "v"(v.w[0]), "v"(v.w[1]), "v"(v.w[2]),
                  "v"(v.w[3]), "v"(v.w[4]), "v"(v.w[5]), "v"(v.w[6]), "v"(v.w[7])
                : "vcc");
            const bool ng = (e & 128) != 0;
#pragma unroll
            for (int i = 0; i < 8; ++i) u.w[i] = ng ? d.w[i] : v.w[i];
          }
          x[k] = fe_mul_db(u, dbt(sdb, (e & 127) % DB::entries));
        } else {
          x[k] = fe_mul_shoup(v, sm[2 * e], sm[2 * e + 1]);                      // [0, 2p)
        }""")
rep("    const size_t lds = (image + db_lds_fe(lr, col)) * sizeof(fe);",
    "    const size_t lds = (image + db_lds_fe(lr, col)) * sizeof(fe) +\n"
    "        ((lr == 8 && col != kColSparse && getenv(\"STARK_LDS_PAD\")) ? atoi(getenv(\"STARK_LDS_PAD\")) : 0);")
