# Variant E2 (round 6, timing only): in the 16 x 16 passes the twiddle of image group g = 0 is w^0 = 1, so the
# wave with a = 0 (wave-uniform) skips the Shoup product of its k = 0 element (1/16 of the pass's twiddle
# products) and only reduces it below 2p.
def apply(s):
    old = '''      fe x[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const fe v = XI.ld(i0 + k * st);
        const uint32_t e = (__builtin_bitreverse32((a << 2) + k) >> 28) * t;  // rev4(g) k1, < R
        x[k] = fe_mul_shoup(v, sm[2 * e], sm[2 * e + 1]);                      // [0, 2p)
      }'''
    new = '''      fe x[4];
      // (group g = 0's twiddle is w^0: with one a per wave the a = 0 waves skip that product)
      const bool unit0 = ((64u >> log_b) <= (1u << LT) ? __builtin_amdgcn_readfirstlane(a) : a) == 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const fe v = XI.ld(i0 + k * st);
        if (k == 0 && unit0) {
          x[0] = v;
          fe_csub2p(x[0]);  // [0, 4p) -> [0, 2p)
          continue;
        }
        const uint32_t e = (__builtin_bitreverse32((a << 2) + k) >> 28) * t;  // rev4(g) k1, < R
        x[k] = fe_mul_shoup(v, sm[2 * e], sm[2 * e + 1]);                      // [0, 2p)
      }'''
    assert old in s
    return s.replace(old, new)
