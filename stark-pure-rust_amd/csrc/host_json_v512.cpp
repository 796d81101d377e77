// AVX-512 (BW + VBMI + VBMI2) digits for the JSON byte-array writer (host_json.h).  Built with those
// features enabled; only called once host_json.cpp has found them on the CPU.
#include <immintrin.h>

#include "host_json.h"

namespace stark {

namespace {

// 16 bytes -> their decimal text with a comma after each item, compressed to its exact length.
// Each byte owns a 4-byte slot [hundreds, tens, ones, ','] in one 64-byte register, and the leading
// zeros are dropped by the compress mask (hundreds kept from 100, tens from 10).
struct Digits {
  __m512i spread, tens_lo, tens_hi, ones_lo, ones_hi, c100, c10, comma;
  __mmask64 p0, p1, p2, p3;
  Digits() {
    alignas(64) uint8_t sp[64], tl[64], th[64], ol[64], oh[64];
    for (int i = 0; i < 64; ++i) {
      sp[i] = (uint8_t)(i / 4);  // slot i/4 reads input byte i/4
      tl[i] = (uint8_t)('0' + i / 10);
      th[i] = (uint8_t)('0' + ((i + 64) / 10) % 10);
      ol[i] = (uint8_t)('0' + i % 10);
      oh[i] = (uint8_t)('0' + (i + 64) % 10);
    }
    spread = _mm512_load_si512(sp);
    tens_lo = _mm512_load_si512(tl);
    tens_hi = _mm512_load_si512(th);
    ones_lo = _mm512_load_si512(ol);
    ones_hi = _mm512_load_si512(oh);
    c100 = _mm512_set1_epi8(100);
    c10 = _mm512_set1_epi8(10);
    comma = _mm512_set1_epi8(',');
    p0 = (__mmask64)0x1111111111111111ull;
    p1 = p0 << 1;
    p2 = p0 << 2;
    p3 = p0 << 3;
  }
};

// full: store all 64 bytes (the caller's next group overwrites what lies past this one's end)
template <bool full>
inline char* items16(char* w, const uint8_t* p, const Digits& D) {
  const __m512i in = _mm512_castsi128_si512(_mm_loadu_si128(reinterpret_cast<const __m128i*>(p)));
  const __m512i b = _mm512_permutexvar_epi8(D.spread, in);  // byte i/4 in every lane of slot i/4
  const __mmask64 ge100 = _mm512_cmpge_epu8_mask(b, D.c100);
  const __mmask64 ge200 = _mm512_cmpge_epu8_mask(b, _mm512_set1_epi8((char)200));
  const __mmask64 ge10 = _mm512_cmpge_epu8_mask(b, D.c10);
  // r = b mod 100 (< 100: a 7-bit index into the 128-entry tens / ones tables)
  __m512i r = _mm512_mask_sub_epi8(b, ge100, b, D.c100);
  r = _mm512_mask_sub_epi8(r, ge200, r, D.c100);
  const __m512i tens = _mm512_permutex2var_epi8(D.tens_lo, r, D.tens_hi);
  const __m512i ones = _mm512_permutex2var_epi8(D.ones_lo, r, D.ones_hi);
  __m512i hund = _mm512_set1_epi8('0');
  hund = _mm512_mask_add_epi8(hund, ge100, hund, _mm512_set1_epi8(1));
  hund = _mm512_mask_add_epi8(hund, ge200, hund, _mm512_set1_epi8(1));
  __m512i t = _mm512_mask_blend_epi8(D.p0, D.comma, hund);
  t = _mm512_mask_blend_epi8(D.p1, t, tens);
  t = _mm512_mask_blend_epi8(D.p2, t, ones);
  const __mmask64 keep = (ge100 & D.p0) | (ge10 & D.p1) | D.p2 | D.p3;
  const __m512i out = _mm512_maskz_compress_epi8(keep, t);
  const unsigned len = (unsigned)_mm_popcnt_u64((unsigned long long)keep);
  if (full) _mm512_storeu_si512(w, out);
  else _mm512_mask_storeu_epi8(w, (__mmask64)(len == 64 ? ~0ull : ((1ull << len) - 1)), out);
  return w + len;
}

}  // namespace

char* json_items16_v512(char* w, const uint8_t* p, size_t k) {
  static const Digits D;
  if (!k) return w;
  for (size_t i = 0; i + 1 < k; ++i) w = items16<true>(w, p + 16 * i, D);
  return items16<false>(w, p + 16 * (k - 1), D);  // the last group writes nothing past its end
}

size_t json_digits_v512(const uint8_t* p, size_t n) {
  const __m512i c100 = _mm512_set1_epi8(100), c10 = _mm512_set1_epi8(10);
  size_t d = n;
  for (size_t i = 0; i < n; i += 64) {
    const size_t m = n - i < 64 ? n - i : 64;
    const __mmask64 live = m == 64 ? ~(__mmask64)0 : (((__mmask64)1 << m) - 1);
    const __m512i b = _mm512_maskz_loadu_epi8(live, p + i);  // (masked-off lanes read as 0: no digit)
    d += (size_t)_mm_popcnt_u64(_mm512_cmpge_epu8_mask(b, c10)) + (size_t)_mm_popcnt_u64(_mm512_cmpge_epu8_mask(b, c100));
  }
  return d;
}

}  // namespace stark
