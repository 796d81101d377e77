// Shoup constant product (fe_mul_shoup) vs the Montgomery product (fe_mul_lazy):
//   check: reads shoup_in.bin (n x [a, w, wq, w_mont] 32-B LE elements, made by shoup_check.py),
//          writes shoup_out.bin (n x [shoup(a, w, wq), mont(a, w_mont)]);
//   rate:  G products/s of each form, 4 and 8 waves per SIMD.
#include "../../stark-pure-rust_amd/csrc/fp_dev.h"

#include <cstdio>
#include <vector>
using namespace stark;

__global__ void check_k(const fe* in, fe* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const fe a = in[4 * i], w = in[4 * i + 1], wq = in[4 * i + 2], wm = in[4 * i + 3];
  out[2 * i] = fe_mul_shoup(a, w, wq);
  out[2 * i + 1] = fe_mul_lazy(a, wm);
}

#define ITERS 256
template <int V>
__global__ __launch_bounds__(256) void rate_k(fe* out, fe a0, fe w, fe wq) {
  fe a = a0;
  a.w[0] += threadIdx.x;
  w.w[1] ^= threadIdx.x & 7;
  for (int i = 0; i < ITERS; ++i) {
    if (V == 0) a = fe_mul_lazy(a, w);
    if (V == 1) a = fe_mul_shoup(a, w, wq);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a;
}
template <int V>
void rate(fe* out, fe a0, fe w, fe wq, int waves) {
  const int blocks = 256 * waves;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(rate_k<V>, dim3(blocks), dim3(256), 0, 0, out, a0, w, wq);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(rate_k<V>, dim3(blocks), dim3(256), 0, 0, out, a0, w, wq);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= 5;
  printf("%-10s waves/SIMD %d: %.2f G products/s\n", V ? "shoup" : "montgomery", waves,
         (double)blocks * 256 * ITERS / ms / 1e6);
}
int main(int argc, char** argv) {
  const char* inp = argc > 1 ? argv[1] : "shoup_in.bin";
  const char* outp = argc > 2 ? argv[2] : "shoup_out.bin";
  FILE* f = fopen(inp, "rb");
  if (!f) { printf("no %s\n", inp); return 1; }
  fseek(f, 0, SEEK_END);
  const long bytes = ftell(f);
  fseek(f, 0, SEEK_SET);
  const int n = (int)(bytes / (4 * sizeof(fe)));
  std::vector<fe> h(4 * (size_t)n), o(2 * (size_t)n);
  if (fread(h.data(), sizeof(fe), h.size(), f) != h.size()) return 1;
  fclose(f);
  fe *din, *dout;
  (void)hipMalloc(&din, h.size() * sizeof(fe));
  (void)hipMalloc(&dout, (size_t)256 * 8 * 256 * sizeof(fe) > o.size() * sizeof(fe) ? (size_t)256 * 8 * 256 * sizeof(fe)
                                                                                       : o.size() * sizeof(fe));
  (void)hipMemcpy(din, h.data(), h.size() * sizeof(fe), hipMemcpyHostToDevice);
  hipLaunchKernelGGL(check_k, dim3((n + 255) / 256), dim3(256), 0, 0, din, dout, n);
  (void)hipMemcpy(o.data(), dout, o.size() * sizeof(fe), hipMemcpyDeviceToHost);
  FILE* g = fopen(outp, "wb");
  fwrite(o.data(), sizeof(fe), o.size(), g);
  fclose(g);
  printf("checked %d products -> %s\n", n, outp);
  for (int w : {4, 8}) {
    rate<0>(dout, h[0], h[1], h[2], w);
    rate<1>(dout, h[0], h[1], h[2], w);
  }
  return 0;
}
