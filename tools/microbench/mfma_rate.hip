// MFMA issue-rate microbenchmark (gfx950): f64 16x16x4 vs f32 16x16x4 vs bf16 16x16x32, 8
// independent accumulators per wave, no memory traffic. Prints achieved TFLOP/s per form.
// Build: hipcc --offload-arch=gfx950 -O3 tools/microbench/mfma_rate.hip -o /tmp/mfma_rate
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double f64x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

template <int FORM>
__global__ __launch_bounds__(256) void k_rate(float* out, int iters) {
  const int l = threadIdx.x;
  if constexpr (FORM == 0) {
    f64x4 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = f64x4{0, 0, 0, 0};
    double a = 1e-3 * l, b = 2e-3 * l;
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[j], 0, 0, 0);
    double s = 0;
    for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][3];
    if (s == 12345.0) out[0] = (float)s;
  } else if constexpr (FORM == 1) {
    f32x4 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = f32x4{0, 0, 0, 0};
    float a = 1e-3f * l, b = 2e-3f * l;
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
    float s = 0;
    for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][3];
    if (s == 12345.f) out[0] = s;
  } else {
    f32x4 acc[8];
    for (int j = 0; j < 8; ++j) acc[j] = f32x4{0, 0, 0, 0};
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) { a[j] = (__bf16)(1e-3f * (l + j)); b[j] = (__bf16)(2e-3f * (l - j)); }
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
    float s = 0;
    for (int j = 0; j < 8; ++j) s += acc[j][0] + acc[j][3];
    if (s == 12345.f) out[0] = s;
  }
}

template <int FORM>
static void run(const char* name, double flop_per_mfma, float* out) {
  const int blocks = 2048, iters = 2000;
  hipLaunchKernelGGL(k_rate<FORM>, dim3(blocks), dim3(256), 0, 0, out, 10);
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(k_rate<FORM>, dim3(blocks), dim3(256), 0, 0, out, iters);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  const double n = (double)blocks * 4 * iters * 8;     // MFMAs (4 waves per block)
  printf("%-24s %8.3f ms  %8.1f TFLOP/s  %6.2f ns per MFMA per SIMD (1024 SIMDs)\n", name, ms,
         n * flop_per_mfma / (ms * 1e-3) / 1e12, ms * 1e6 / (n / 1024));
}

int main() {
  float* out;
  hipMalloc(&out, 4);
  run<0>("f64 16x16x4", 16 * 16 * 4 * 2, out);
  run<1>("f32 16x16x4", 16 * 16 * 4 * 2, out);
  run<2>("bf16 16x16x32", 16 * 16 * 32 * 2, out);
  hipFree(out);
  return 0;
}
