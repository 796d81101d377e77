// serde_json's text of a byte array (Vec<u8> / [u8; 32]: "[b0,b1,...]", no spaces) for the proof
// writers (fri.hip json_bytes_at).  The digits of 64 bytes at a time in AVX-512 registers
// (host_json_v512.cpp) when the CPU has VBMI2's byte compress, else one table store per byte.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace stark {

// Writes "b," for each of the 16 k bytes at p (every item followed by its comma) and returns the end;
// nothing past the end is written.
char* json_items16_v512(char* w, const uint8_t* p, size_t k);
// The reader's side: the numbers of a compact u8 array whose text starts after its '[' at p, written to
// out[0..max), their count in *count and the end (past ']') returned; nullptr when the text is anything
// but "d,d,...,d]" with serde_json's canonical numbers 0..255 (the scalar reader then decides it).
const char* json_u8s_v512(const char* p, const char* e, uint8_t* out, size_t max, size_t* count);
// Number of decimal digits of the n bytes at p.
size_t json_digits_v512(const uint8_t* p, size_t n);

// The width the writers use: 64 (AVX-512 VBMI2) or 1 (scalar).  STARK_JSON_SIMD=0 forces the scalar
// path (the tests compare both on one host).
int json_simd_width();

}  // namespace stark
