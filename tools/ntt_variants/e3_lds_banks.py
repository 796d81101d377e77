# Variant E3 (round 6): LDS bank conflicts of the dense radix-2^8 (16 x 16) passes.
#  * image: the 16-B slot of column b in row r is b ^ f(r), f(r) = ((r >> 4) ^ (r >> 6)) & 3 (B = 4), so the
#    bit-reversed scatter (16-lane groups over rows 64 apart) and the jj-major step (rows 16 apart) hit
#    distinct banks; the twiddle step and the last step (rows 1 apart within a group) stay conflict-free;
#  * twiddle pairs: 16 B of padding after every 4 Shoup pairs (pair e at 16-B unit 4 e + (e >> 2)), so the
#    pairs e = rev4(g) t of 4 adjacent t hit distinct banks for even rev4(g) too.
def rep(s, a, b, cnt=1):
    assert s.count(a) == cnt, (s.count(a), a[:80])
    return s.replace(a, b)

def apply(s):
    s = rep(s, '''  static constexpr uint32_t shoup_fe = last ? 0 : four ? 2 * (1u << LOG_R) : (1u << LOG_R);''',
            '''  // (four: 16 B of padding after every 4 pairs, see sm_pair)
  static constexpr uint32_t shoup_fe = last ? 0 : four ? 2 * (1u << LOG_R) + (1u << LOG_R) / 8 : (1u << LOG_R);''')
    s = rep(s, '''  const uint32_t tile = blockIdx.x;
  if (tile >= total_tiles) return;  // (uniform per workgroup)
''', '''  const uint32_t tile = blockIdx.x;
  if (tile >= total_tiles) return;  // (uniform per workgroup)
  // Image slot swizzle of the dense radix-2^8 passes at B = 4 (column b of row r at slot b ^ f(r)); every
  // image access of those passes goes through px.
  const bool swz = LOG_R == 8 && COL != kColSparse && sp.skip == 0 && log_b == 2;
  auto px = [&](uint32_t i) { return swz ? i ^ (((i >> 6) ^ (i >> 8)) & 3u) : i; };
''')
    s = rep(s, '''    constexpr uint32_t kSm = 2 * DB::shoup_fe, kDb = DB::on ? DB::entries * 18 : 0;  // 16-B units''',
            '''    constexpr uint32_t kSm = DB::four ? 4u << LOG_R : 2 * DB::shoup_fe, kDb = DB::on ? DB::entries * 18 : 0;  // 16-B units
    auto sm_dst = [&](uint32_t k) { return DB::four ? k + (k >> 4) : k; };''')
    s = rep(s, '''        if (in_sm(i)) sm4[tid + i * kPassThreads] = ts[i];''',
            '''        if (in_sm(i)) sm4[sm_dst(tid + i * kPassThreads)] = ts[i];''')
    s = rep(s, '''      for (uint32_t k = tid; k < kSm; k += blockDim.x) sm4[k] = small4[k];''',
            '''      for (uint32_t k = tid; k < kSm; k += blockDim.x) sm4[sm_dst(k)] = small4[k];''')
    s = rep(s, '''        XI.st((rr << log_b) + eb[t], v[t]);''', '''        XI.st(px((rr << log_b) + eb[t]), v[t]);''')
    s = rep(s, '''      fe x0 = XI.ld(i0), x1 = XI.ld(i0 + st), x2 = XI.ld(i0 + 2 * st), x3 = XI.ld(i0 + 3 * st);
      if (jj == 0) {''', '''      fe x0 = XI.ld(px(i0)), x1 = XI.ld(px(i0 + st)), x2 = XI.ld(px(i0 + 2 * st)), x3 = XI.ld(px(i0 + 3 * st));
      if (jj == 0) {''')
    s = rep(s, '''      XI.st(i0, x0);
      XI.st(i0 + 2 * st, x2);
      XI.st(i0 + st, x1);
      XI.st(i0 + 3 * st, x3);
    }
    __syncthreads();
    s = kS0 + 2;''', '''      XI.st(px(i0), x0);
      XI.st(px(i0 + 2 * st), x2);
      XI.st(px(i0 + st), x1);
      XI.st(px(i0 + 3 * st), x3);
    }
    __syncthreads();
    s = kS0 + 2;''')
    s = rep(s, '''        const fe v = XI.ld(i0 + k * st);
        if (k == 0 && unit0) {''', '''        const fe v = XI.ld(px(i0 + k * st));
        if (k == 0 && unit0) {''')
    s = rep(s, '''        x[k] = fe_mul_shoup(v, sm[2 * e], sm[2 * e + 1]);                      // [0, 2p)''',
            '''        fe w, wq;
        {  // pair e at 16-B unit 4 e + (e >> 2) (DbPlan::shoup_fe)
          const uint4* pe = reinterpret_cast<const uint4*>(sm) + 4 * e + (e >> 2);
          const uint4 u0 = pe[0], u1 = pe[1], u2 = pe[2], u3 = pe[3];
          w.w[0] = u0.x; w.w[1] = u0.y; w.w[2] = u0.z; w.w[3] = u0.w;
          w.w[4] = u1.x; w.w[5] = u1.y; w.w[6] = u1.z; w.w[7] = u1.w;
          wq.w[0] = u2.x; wq.w[1] = u2.y; wq.w[2] = u2.z; wq.w[3] = u2.w;
          wq.w[4] = u3.x; wq.w[5] = u3.y; wq.w[6] = u3.z; wq.w[7] = u3.w;
        }
        x[k] = fe_mul_shoup(v, w, wq);  // [0, 2p)''')
    s = rep(s, '''      for (int k = 0; k < 4; ++k) XI.st(i0 + k * st, x[k]);''',
            '''      for (int k = 0; k < 4; ++k) XI.st(px(i0 + k * st), x[k]);''')
    s = rep(s, '''      const uint32_t i0 = (q << log_b) + b, st = (R / 4) << log_b;
      fe x0 = XI.ld(i0), x1 = XI.ld(i0 + st), x2 = XI.ld(i0 + 2 * st), x3 = XI.ld(i0 + 3 * st);
      auto step''', '''      const uint32_t i0 = (q << log_b) + b, st = (R / 4) << log_b;
      fe x0 = XI.ld(px(i0)), x1 = XI.ld(px(i0 + st)), x2 = XI.ld(px(i0 + 2 * st)), x3 = XI.ld(px(i0 + 3 * st));
      auto step''')
    return s
