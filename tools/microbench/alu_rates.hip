// Microbenchmark: issue rates of the integer multiply forms a 256-bit Montgomery
// multiply can be built from on gfx950, plus FP64 FMA for comparison.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 4096
#pragma clang diagnostic ignored "-Wunused-result"
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void k_mad64(uint64_t* out, uint32_t a, uint32_t b) {
  uint32_t x = a + threadIdx.x;
  uint64_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i + threadIdx.x;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = (uint64_t)(uint32_t)acc[i] * (uint32_t)(b + i) + (acc[i] >> 32);
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mullo(uint32_t* out, uint32_t a, uint32_t b) {
  uint32_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i + threadIdx.x + a;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = acc[i] * (b + i);
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_mulhi(uint32_t* out, uint32_t a, uint32_t b) {
  uint32_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i + threadIdx.x + a;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = __umulhi(acc[i], b + i) + 1u;
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_addc(uint32_t* out, uint32_t a, uint32_t b) {
  uint64_t acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i + threadIdx.x + a;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = acc[i] + (uint64_t)(b + i) * 0x100000001ull;
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}
__global__ void k_fma64(double* out, double a, double b) {
  double acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i + threadIdx.x + a;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = fma(acc[i], b, 1e-300);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_fma32(float* out, float a, float b) {
  float acc[8];
#pragma unroll
  for (int i = 0; i < 8; i++) acc[i] = i + threadIdx.x + a;
  for (int it = 0; it < ITERS; it++) {
#pragma unroll
    for (int i = 0; i < 8; i++) acc[i] = fmaf(acc[i], b, 1e-30f);
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename F>
static float timeit(F launch) {
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  launch(); hipDeviceSynchronize();
  hipEventRecord(a);
  for (int i = 0; i < 5; i++) launch();
  hipEventRecord(b); hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 5;
}

int main() {
  const int blocks = 256 * 8, threads = 256;
  const double ops = (double)blocks * threads * ITERS * 8;
  void* buf; CHK(hipMalloc(&buf, (size_t)blocks * threads * 8));
  float t;
  t = timeit([&] { k_mad64<<<blocks, threads>>>((uint64_t*)buf, 3, 5); });
  printf("v_mad_u64_u32  : %.3f ms  %.2f Tops/s\n", t, ops / t / 1e9);
  t = timeit([&] { k_mullo<<<blocks, threads>>>((uint32_t*)buf, 3, 5); });
  printf("v_mul_lo_u32   : %.3f ms  %.2f Tops/s\n", t, ops / t / 1e9);
  t = timeit([&] { k_mulhi<<<blocks, threads>>>((uint32_t*)buf, 3, 5); });
  printf("v_mul_hi_u32+add: %.3f ms  %.2f Tops/s\n", t, ops / t / 1e9);
  t = timeit([&] { k_addc<<<blocks, threads>>>((uint32_t*)buf, 3, 5); });
  printf("u64 add (co+addc): %.3f ms  %.2f Tops/s\n", t, ops / t / 1e9);
  t = timeit([&] { k_fma64<<<blocks, threads>>>((double*)buf, 1.0, 0.999); });
  printf("v_fma_f64      : %.3f ms  %.2f Tops/s\n", t, ops / t / 1e9);
  t = timeit([&] { k_fma32<<<blocks, threads>>>((float*)buf, 1.0f, 0.999f); });
  printf("v_fma_f32      : %.3f ms  %.2f Tops/s\n", t, ops / t / 1e9);
  return 0;
}
