// Host-side BN254 Fr scalar arithmetic for setup work only (root checks,
// twiddle seeds, transcript values such as special_x).  The hot loops run on
// the GPU (fp_dev.h).  Same Montgomery convention: R = 2^256.
#pragma once
#include <stdint.h>
#include <string.h>

namespace stark {

struct HostFp {
  uint64_t v[4];  // Montgomery form
};

class FieldHost {
 public:
  static constexpr uint64_t kP[4] = {0x43e1f593f0000001ull, 0x2833e84879b97091ull, 0xb85045b68181585dull,
                                     0x30644e72e131a029ull};
  static const FieldHost& get() {
    static FieldHost f;
    return f;
  }

  HostFp one() const { return one_; }
  HostFp zero() const { return HostFp{{0, 0, 0, 0}}; }

  static bool ge_p(const uint64_t a[4]) {
    for (int i = 3; i >= 0; --i) {
      if (a[i] != kP[i]) return a[i] > kP[i];
    }
    return true;
  }
  static void sub_p_in_place(uint64_t a[4]) {
    unsigned __int128 br = 0;
    for (int i = 0; i < 4; ++i) {
      unsigned __int128 d = (unsigned __int128)a[i] - kP[i] - br;
      a[i] = (uint64_t)d;
      br = (uint64_t)(d >> 64) ? 1 : 0;
    }
  }

  HostFp add(const HostFp& a, const HostFp& b) const {
    HostFp r;
    unsigned __int128 c = 0;
    for (int i = 0; i < 4; ++i) {
      c += (unsigned __int128)a.v[i] + b.v[i];
      r.v[i] = (uint64_t)c;
      c >>= 64;
    }
    if (ge_p(r.v)) sub_p_in_place(r.v);
    return r;
  }
  HostFp sub(const HostFp& a, const HostFp& b) const {
    HostFp r;
    unsigned __int128 br = 0;
    for (int i = 0; i < 4; ++i) {
      unsigned __int128 d = (unsigned __int128)a.v[i] - b.v[i] - br;
      r.v[i] = (uint64_t)d;
      br = (uint64_t)(d >> 64) ? 1 : 0;
    }
    if (br) {
      unsigned __int128 c = 0;
      for (int i = 0; i < 4; ++i) {
        c += (unsigned __int128)r.v[i] + kP[i];
        r.v[i] = (uint64_t)c;
        c >>= 64;
      }
    }
    return r;
  }
  // Separated-operand-scanning Montgomery product (64-bit limbs).
  HostFp mul(const HostFp& a, const HostFp& b) const {
    uint64_t t[9] = {0};
    for (int i = 0; i < 4; ++i) {
      unsigned __int128 c = 0;
      for (int j = 0; j < 4; ++j) {
        c += (unsigned __int128)a.v[j] * b.v[i] + t[j];
        t[j] = (uint64_t)c;
        c >>= 64;
      }
      unsigned __int128 top = (unsigned __int128)t[4] + (uint64_t)c;
      t[4] = (uint64_t)top;
      t[5] = (uint64_t)(top >> 64);
      const uint64_t m = t[0] * pinv_;
      c = ((unsigned __int128)m * kP[0] + t[0]) >> 64;
      for (int j = 1; j < 4; ++j) {
        c += (unsigned __int128)m * kP[j] + t[j];
        t[j - 1] = (uint64_t)c;
        c >>= 64;
      }
      top = (unsigned __int128)t[4] + (uint64_t)c;
      t[3] = (uint64_t)top;
      t[4] = t[5] + (uint64_t)(top >> 64);
    }
    HostFp r;
    memcpy(r.v, t, 32);
    if (t[4] || ge_p(r.v)) sub_p_in_place(r.v);
    return r;
  }
  // Canonical (any 256-bit value, reduced mod p) -> Montgomery.
  HostFp from_canonical(const uint64_t c[4]) const {
    HostFp a;
    memcpy(a.v, c, 32);
    while (ge_p(a.v)) sub_p_in_place(a.v);
    return mul(a, r2_);
  }
  void to_canonical(const HostFp& a, uint64_t out[4]) const {
    HostFp unit{{1, 0, 0, 0}};
    HostFp r = mul(a, unit);
    memcpy(out, r.v, 32);
  }
  HostFp from_u64(uint64_t x) const {
    uint64_t c[4] = {x, 0, 0, 0};
    return from_canonical(c);
  }
  HostFp pow(const HostFp& a, const uint64_t* e, int nlimbs) const {
    HostFp r = one_;
    bool started = false;  // squarings of one before the top set bit are skipped
    for (int i = nlimbs - 1; i >= 0; --i)
      for (int bit = 63; bit >= 0; --bit) {
        if (started) r = mul(r, r);
        if ((e[i] >> bit) & 1) {
          r = started ? mul(r, a) : a;
          started = true;
        }
      }
    return r;
  }
  HostFp pow_u64(const HostFp& a, uint64_t e) const { return pow(a, &e, 1); }
  HostFp inv(const HostFp& a) const {
    uint64_t e[4] = {kP[0] - 2, kP[1], kP[2], kP[3]};
    return pow(a, e, 4);
  }
  static bool eq(const HostFp& a, const HostFp& b) { return memcmp(a.v, b.v, 32) == 0; }
  // from_bytes_le (ff_utils/src/fp.rs:74-76): the little-endian integer of up
  // to 32 bytes, reduced mod p (ff from_str semantics), in canonical form (no
  // Montgomery conversion).  The host is little endian, so the bytes are the
  // limbs.
  HostFp reduce_bytes_le(const uint8_t* b, size_t len) const {
    HostFp a{{0, 0, 0, 0}};
    memcpy(a.v, b, len < 32 ? len : 32);
    while (ge_p(a.v)) sub_p_in_place(a.v);
    return a;
  }
  // The same value as a Montgomery image.
  HostFp from_bytes_le(const uint8_t* b, size_t len) const {
    const HostFp c = reduce_bytes_le(b, len);
    return from_canonical(c.v);
  }

 private:
  FieldHost() {
    uint64_t x = 1;
    for (int i = 0; i < 7; ++i) x *= 2 - kP[0] * x;
    pinv_ = 0 - x;
    HostFp r{{1, 0, 0, 0}};
    for (int i = 0; i < 512; ++i) {
      r = add(r, r);
      if (i == 255) one_ = r;
    }
    r2_ = r;
  }
  uint64_t pinv_ = 0;
  HostFp one_{};
  HostFp r2_{};
};

}  // namespace stark
