# Variant E1 (round 6, timing only): the last pass's full column-twiddle table as Shoup pairs (64 B per entry,
# fe_mul_shoup ~245 VALU) instead of Montgomery images (32 B, fe_mul_lazy ~280 VALU).
def apply(s):
    rep = [
        ('''#pragma unroll
        for (int t = 0; t < 4; ++t) tw[t] = fe_load_nt(ct.full + ((((j0 + eb[t]) & ns_mask) << LOG_R) + er[t]));
        // Montgomery images (the table streams from HBM once per transform, so it stays 32 B per
        // entry): v < 4p, tw < p -> [0, 2p); two interleaved products per block
        mul2(v[0], v[1], v[0], tw[0], v[1], tw[1]);
        mul2(v[2], v[3], v[2], tw[2], v[3], tw[3]);''',
         '''        fe twq[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const fe* e = ct.full + 2 * ((((j0 + eb[t]) & ns_mask) << LOG_R) + er[t]);
          tw[t] = fe_load_nt(e);
          twq[t] = fe_load_nt(e + 1);
        }
        shoup2(v[0], v[1], v[0], tw[0], twq[0], v[1], tw[1], twq[1]);
        shoup2(v[2], v[3], v[2], tw[2], twq[2], v[3], tw[3], twq[3]);'''),
        ('''  fe t = fe_mul(lo[e & (((uint64_t)1 << kb) - 1)], hi[e >> kb]);
  if (do_scale) t = fe_mul(t, scale);
  fe_store(out + g, t);''',
         '''  fe t = fe_mul(lo[e & (((uint64_t)1 << kb) - 1)], hi[e >> kb]);
  if (do_scale) t = fe_mul(t, scale);
  // Shoup pair of the value whose Montgomery image is t: w = montmul(t, 1), wq = (2^256 - t) p^-1 mod 2^256
  fe one = fe_zero();
  one.w[0] = 1;
  const fe w = fe_mul(t, one);
  const uint32_t pinv[8] = {0x10000001u, 0x3d1e0a6cu, 0xb396ee4cu, 0x9a7979b4u, 0x66f9dc6eu, 0x1c6567d7u, 0xf27cbe4du, 0x8c07d0e2u};
  uint32_t neg[8];
  uint64_t br = 0;
  for (int i = 0; i < 8; ++i) {
    const uint64_t d = (uint64_t)0 - t.w[i] - br;
    neg[i] = (uint32_t)d;
    br = (d >> 32) ? 1 : 0;
  }
  uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 8; ++i) {
    uint64_t c = 0;
    for (int j = 0; i + j < 8; ++j) {
      const uint64_t x = (uint64_t)neg[i] * pinv[j] + q[i + j] + c;
      q[i + j] = (uint32_t)x;
      c = x >> 32;
    }
  }
  fe wq;
  for (int i = 0; i < 8; ++i) wq.w[i] = q[i];
  fe_store(out + 2 * g, w);
  fe_store(out + 2 * g + 1, wq);'''),
        ('''    if (!cache_reserve(ctx, n * sizeof(fe), false) || hipMalloc(&p, n * sizeof(fe)) != hipSuccess) {''',
         '''    if (!cache_reserve(ctx, 2 * n * sizeof(fe), false) || hipMalloc(&p, 2 * n * sizeof(fe)) != hipSuccess) {'''),
    ]
    for a, b in rep:
        assert a in s, a[:80]
        s = s.replace(a, b)
    return s
