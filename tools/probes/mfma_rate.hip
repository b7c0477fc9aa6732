// MFMA issue-rate probe (diagnostic, not product): cycles per instruction of
// v_mfma_f32_16x16x32_bf16 and v_mfma_f32_16x16x16_bf16 (the 1k form), one
// wave per SIMD, 4 independent accumulators.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int K>
__global__ __launch_bounds__(256) void probe(float* out, long long* cyc, int iters) {
  f32x4 acc[4] = {};
  bf16x8 a8, b8;
  s16x4 a4, b4;
  for (int i = 0; i < 8; ++i) { a8[i] = (__bf16)(threadIdx.x * 0.001f + i); b8[i] = (__bf16)(i * 0.5f); }
  for (int i = 0; i < 4; ++i) { a4[i] = (short)(threadIdx.x + i); b4[i] = (short)(i * 3); }
  const long long t0 = clock64();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if constexpr (K == 32) acc[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a8, b8, acc[q], 0, 0, 0);
      else acc[q] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(a4, b4, acc[q], 0, 0, 0);
    }
  }
  const long long t1 = clock64();
  float s = 0.f;
  for (int q = 0; q < 4; ++q) s += acc[q][0] + acc[q][1] + acc[q][2] + acc[q][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out; long long* cyc;
  hipMalloc(&out, 256 * 256 * 4); hipMalloc(&cyc, 256 * 8);
  const int iters = 4096;
  long long h[256];
  for (int k = 0; k < 2; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      if (k == 0) hipLaunchKernelGGL(probe<32>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
      else hipLaunchKernelGGL(probe<16>, dim3(256), dim3(256), 0, 0, out, cyc, iters);
      hipDeviceSynchronize();
    }
    hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    std::printf("16x16x%d bf16: %.2f cycles per MFMA (s_memtime clock, 1 wave/SIMD, 4 chains)\n", k == 0 ? 32 : 16,
                (double)h[0] / (iters * 4.0));
  }
  return 0;
}
