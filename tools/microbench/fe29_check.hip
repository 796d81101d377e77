// Building-block check of fp29_dev.h against tools/fe29_check.py (inputs/outputs as raw u32 files).
#include "../../stark-pure-rust_amd/csrc/fp29_dev.h"
#include <cstdio>
#include <cstdlib>
using namespace stark;
// in: per case 32 dwords: a (8), b (8), w (8, canonical), m (8, Montgomery image of w)
// out: per case 64 dwords: to32(from32(a)) (8), canonical(from32(a)) (8), a*w via pair_from_mont (8),
//      a*w via pair_from_shoup(w, q32) with q32 from the mont path (8), pair wq from mont (9) + pad,
//      canonical(subk(from32(a), from32(b))) = a - b + 4p mod p (8), canonical(a + b) (8), spare
__global__ void k(const uint32_t* in, uint32_t* out, int n) {
  const int g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  fe a, b, w, m;
  for (int i = 0; i < 8; ++i) {
    a.w[i] = in[32 * g + i]; b.w[i] = in[32 * g + 8 + i]; w.w[i] = in[32 * g + 16 + i]; m.w[i] = in[32 * g + 24 + i];
  }
  uint32_t* o = out + 64 * g;
  const fe29 a29 = fe29_from32(a), b29 = fe29_from32(b);
  fe r = fe29_to32(a29);
  for (int i = 0; i < 8; ++i) o[i] = r.w[i];
  r = fe29_canonical(a29);
  for (int i = 0; i < 8; ++i) o[8 + i] = r.w[i];
  const fe29p pm = pair29_from_mont(m);
  fe29 w29, wq29;
  for (int i = 0; i < 9; ++i) { w29.l[i] = pm.w[i]; wq29.l[i] = pm.wq[i]; }
  r = fe29_canonical(fe29_mul_shoup(a29, w29, wq29));
  for (int i = 0; i < 8; ++i) o[16 + i] = r.w[i];
  r = fe29_canonical(fe29_mul_pair(a29, &pm));
  for (int i = 0; i < 8; ++i) o[24 + i] = r.w[i];
  for (int i = 0; i < 9; ++i) o[32 + i] = pm.wq[i];
  r = fe29_canonical(fe29_subk(a29, b29));
  for (int i = 0; i < 8; ++i) o[41 + i] = r.w[i];
  fe29 s = a29;
  fe29_add(s, b29);
  r = fe29_canonical(s);
  for (int i = 0; i < 8; ++i) o[49 + i] = r.w[i];
  for (int i = 0; i < 9; ++i) o[57 + i < 64 ? 57 + i : 63] = pm.w[i];
}
int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  fseek(f, 0, SEEK_END);
  const long bytes = ftell(f);
  fseek(f, 0, SEEK_SET);
  const int n = (int)(bytes / 128);
  uint32_t* h = (uint32_t*)malloc(bytes);
  if (fread(h, 1, bytes, f) != (size_t)bytes) return 1;
  fclose(f);
  uint32_t *din, *dout;
  (void)hipMalloc(&din, bytes);
  (void)hipMalloc(&dout, (size_t)n * 256);
  (void)hipMemcpy(din, h, bytes, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3((n + 63) / 64), dim3(64), 0, 0, din, dout, n);
  uint32_t* ho = (uint32_t*)malloc((size_t)n * 256);
  (void)hipMemcpy(ho, dout, (size_t)n * 256, hipMemcpyDeviceToHost);
  f = fopen(argv[2], "wb");
  fwrite(ho, 1, (size_t)n * 256, f);
  fclose(f);
  printf("%d cases\n", n);
  return 0;
}
