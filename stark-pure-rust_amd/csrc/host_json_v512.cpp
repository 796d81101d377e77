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

// The compact u8 array text after its '[' ("d,d,...,d]": 1-3 digits per number, no leading zero, at
// most 255, no whitespace), 16 numbers per step: the commas' positions (compressed byte indices) give
// each number's end, the previous end its start, and the digits are gathered right-aligned.  nullptr
// for any other text (the caller's scalar reader decides it), or past max numbers.
const char* json_u8s_v512(const char* p, const char* e, uint8_t* out, size_t max, size_t* count) {
  alignas(64) static const uint8_t kIota[64] = {0,  1,  2,  3,  4,  5,  6,  7,  8,  9,  10, 11, 12, 13, 14, 15,
                                                16, 17, 18, 19, 20, 21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31,
                                                32, 33, 34, 35, 36, 37, 38, 39, 40, 41, 42, 43, 44, 45, 46, 47,
                                                48, 49, 50, 51, 52, 53, 54, 55, 56, 57, 58, 59, 60, 61, 62, 63};
  const __m512i iota = _mm512_load_si512(kIota);
  const __m512i zero_ch = _mm512_set1_epi8('0'), ten = _mm512_set1_epi8(10);
  size_t k = 0;
  while (p < e) {
    const size_t avail = (size_t)(e - p);
    const __mmask64 live = avail >= 64 ? ~(__mmask64)0 : (((__mmask64)1 << avail) - 1);
    const __m512i c = _mm512_maskz_loadu_epi8(live, p);
    const __mmask64 dig = _mm512_cmplt_epu8_mask(_mm512_sub_epi8(c, zero_ch), ten) & live;
    const __mmask64 com = _mm512_cmpeq_epi8_mask(c, _mm512_set1_epi8(',')) & live;
    const __mmask64 other = ~(dig | com);
    const unsigned lim = other ? (unsigned)_tzcnt_u64(other) : 64u;
    const bool term = lim < 64 && lim < avail && p[lim] == ']';
    const __mmask64 below = lim >= 64 ? ~(__mmask64)0 : (((__mmask64)1 << lim) - 1);
    __mmask64 ends = (com & below) | (term ? (__mmask64)1 << lim : 0);
    if (!ends) return nullptr;
    const unsigned n_all = (unsigned)_mm_popcnt_u64(ends);
    const unsigned n = n_all < 16 ? n_all : 16;
    if (n < n_all) ends = _pdep_u64((1ull << 16) - 1, ends);  // the first 16 ends
    if (k + n > max) return nullptr;
    // end positions e_j (bytes 0..n-1) and starts s_j = e_(j-1) + 1 (s_0 = 0)
    const __m128i en = _mm512_castsi512_si128(_mm512_maskz_compress_epi8(ends, iota));
    const __m128i st = _mm_add_epi8(_mm_slli_si128(en, 1), _mm_set_epi8(1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0));
    const __mmask16 lanes = (__mmask16)((1u << n) - 1);
    const __m128i len = _mm_sub_epi8(en, st);
    // 1..3 digits per number
    if (_mm_mask_cmpgt_epu8_mask(lanes, _mm_set1_epi8(1), len) || _mm_mask_cmpgt_epu8_mask(lanes, len, _mm_set1_epi8(3)))
      return nullptr;
    const __mmask16 has2 = _mm_mask_cmpge_epu8_mask(lanes, len, _mm_set1_epi8(2));
    const __mmask16 has3 = _mm_mask_cmpge_epu8_mask(lanes, len, _mm_set1_epi8(3));
    const __m512i d = _mm512_sub_epi8(c, zero_ch);
    const __m128i ones = _mm512_castsi512_si128(
        _mm512_permutexvar_epi8(_mm512_castsi128_si512(_mm_sub_epi8(en, _mm_set1_epi8(1))), d));
    const __m128i tens = _mm_maskz_mov_epi8(has2, _mm512_castsi512_si128(_mm512_permutexvar_epi8(
                                                      _mm512_castsi128_si512(_mm_sub_epi8(en, _mm_set1_epi8(2))), d)));
    const __m128i hund = _mm_maskz_mov_epi8(has3, _mm512_castsi512_si128(_mm512_permutexvar_epi8(
                                                      _mm512_castsi128_si512(_mm_sub_epi8(en, _mm_set1_epi8(3))), d)));
    const __m128i first = _mm_mask_mov_epi8(_mm_mask_mov_epi8(ones, has2, tens), has3, hund);
    // no leading zero: a number of two or more digits starts with 1-9
    if (_mm_mask_cmpeq_epi8_mask(has2, first, _mm_setzero_si128())) return nullptr;
    const __m256i v = _mm256_add_epi16(_mm256_add_epi16(_mm256_cvtepu8_epi16(ones),
                                                        _mm256_mullo_epi16(_mm256_cvtepu8_epi16(tens), _mm256_set1_epi16(10))),
                                       _mm256_mullo_epi16(_mm256_cvtepu8_epi16(hund), _mm256_set1_epi16(100)));
    if (_mm256_mask_cmpgt_epu16_mask(lanes, v, _mm256_set1_epi16(255))) return nullptr;
    _mm_mask_storeu_epi8(out + k, lanes, _mm256_cvtepi16_epi8(v));
    k += n;
    alignas(16) uint8_t eb[16];
    _mm_store_si128(reinterpret_cast<__m128i*>(eb), en);
    const unsigned last_end = eb[n - 1];
    if (term && n == n_all) {  // the ']' ended the last number
      *count = k;
      return p + lim + 1;
    }
    p += last_end + 1;  // past the comma of the last number taken
  }
  return nullptr;
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
