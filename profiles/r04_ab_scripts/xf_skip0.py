# Transform for tools/build_variant.sh: the 16 x 16 passes skip the internal twiddle of the r1 = 0 group
# (w_R^0 = 1; wave-uniform in 1024-element tiles) with a lazy reduction in place of the Shoup product.
out = s  # noqa: F821  (set by build_variant.sh)
a = """        const uint32_t e = (__builtin_bitreverse32((a << 2) + k) >> 28) * t;  // rev4(g) k1, < R
        x[k] = fe_mul_shoup(v, sm[2 * e], sm[2 * e + 1]);                      // [0, 2p)"""
b = """        const uint32_t r1 = __builtin_bitreverse32((a << 2) + k) >> 28;  // rev4(g)
        if (r1 == 0) {  // w_R^0 = 1 for the whole group (a wave-uniform branch in 1024-element tiles)
          x[k] = v;
          fe_csub2p(x[k]);
        } else {
          const uint32_t e = r1 * t;  // rev4(g) k1, < R
          x[k] = fe_mul_shoup(v, sm[2 * e], sm[2 * e + 1]);  // [0, 2p)
        }"""
assert a in out
out = out.replace(a, b, 1)
