// Standalone probe: variants of the fused cosine + weighted-MSE fwd/bwd
// streaming kernel (tt_cosine.hip) against a same-shaped float4 copy
// (2 read streams -> 2 write streams).  B = 4M pairs, D = 128, fp32.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 cos_probe.hip -o cos_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cstring>

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row_reduce16(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  v += dpp_mov<0x140>(v);
  return v;
}
template <int LPR>
__device__ __forceinline__ float red_lpr(float v) {
  v += dpp_mov<0xB1>(v);
  v += dpp_mov<0x4E>(v);
  v += dpp_mov<0x141>(v);
  if constexpr (LPR == 16) v += dpp_mov<0x140>(v);
  return v;
}

template <bool NT>
__device__ __forceinline__ f32x4 ld4(const f32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st4(f32x4 v, f32x4* p) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// NV4 float4 per lane per row (16 lanes per row), RPG rows per 16-lane group per iteration
template <int NV4, int RPG, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_cos(const float* __restrict__ U, const float* __restrict__ V,
                                             const float* __restrict__ tgt, const float* __restrict__ wgt, int64_t B,
                                             int D, float s, float inv_batch, float* __restrict__ score,
                                             float* __restrict__ dU, float* __restrict__ dV, float* loss_sum) {
  const int r = threadIdx.x & 15;
  const int grp = threadIdx.x >> 4;  // 16 groups per block
  float loss_p = 0.f;
  const int64_t rows_per_iter = (int64_t)gridDim.x * 16 * RPG;
  for (int64_t base = ((int64_t)blockIdx.x * 16 + grp) * RPG; base < B; base += rows_per_iter) {
    f32x4 uu[RPG][NV4], vv[RPG][NV4];
    float tg[RPG], wt[RPG];
#pragma unroll
    for (int q = 0; q < RPG; ++q) {
      const int64_t row = min(base + q, B - 1);
      const f32x4* u4 = reinterpret_cast<const f32x4*>(U + row * D);
      const f32x4* v4 = reinterpret_cast<const f32x4*>(V + row * D);
#pragma unroll
      for (int k = 0; k < NV4; ++k) {
        uu[q][k] = ld4<NTL>(u4 + r + 16 * k);
        vv[q][k] = ld4<NTL>(v4 + r + 16 * k);
      }
      tg[q] = tgt[row];
      wt[q] = wgt[row];
    }
#pragma unroll
    for (int q = 0; q < RPG; ++q) {
      const int64_t row = base + q;
      float uv = 0.f, nuu = 0.f, nvv = 0.f;
#pragma unroll
      for (int k = 0; k < NV4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          uv += uu[q][k][e] * vv[q][k][e];
          nuu += uu[q][k][e] * uu[q][k][e];
          nvv += vv[q][k][e] * vv[q][k][e];
        }
      uv = row_reduce16(uv);
      nuu = row_reduce16(nuu);
      nvv = row_reduce16(nvv);
      const float nu = sqrtf(nuu), nv = sqrtf(nvv);
      const float c = uv / (nu * nv);
      const float sc = c * s;
      const bool ok = row < B;
      if (r == 0 && ok) score[row] = sc;
      const float diff = sc - tg[q];
      const float ds = 2.f * diff * (wt[q] * inv_batch);
      if (r == 0 && ok) loss_p += wt[q] * diff * diff;
      const float dc = ds * s;
      const float a_u = dc / (nu * nv), b_u = dc * c / (nu * nu);
      const float a_v = a_u, b_v = dc * c / (nv * nv);
      if (ok) {
        f32x4* du4 = reinterpret_cast<f32x4*>(dU + row * D);
        f32x4* dv4 = reinterpret_cast<f32x4*>(dV + row * D);
#pragma unroll
        for (int k = 0; k < NV4; ++k) {
          st4<NTS>(a_u * vv[q][k] - b_u * uu[q][k], du4 + r + 16 * k);
          st4<NTS>(a_v * uu[q][k] - b_v * vv[q][k], dv4 + r + 16 * k);
        }
      }
    }
  }
  if (r == 0 && loss_p != 0.f) atomicAdd(loss_sum, loss_p * inv_batch);
}

// generalized: LPR lanes per row, RPG rows per lane group, PF: next iteration's loads before this one's math
template <int LPR, int RPG, bool PF>
__global__ __launch_bounds__(256) void k_cos2(const float* __restrict__ U, const float* __restrict__ V,
                                              const float* __restrict__ tgt, const float* __restrict__ wgt, int64_t B,
                                              int D, float s, float inv_batch, float* __restrict__ score,
                                              float* __restrict__ dU, float* __restrict__ dV, float* loss_sum) {
  constexpr int NV4 = 32 / LPR;  // D = 128
  constexpr int GPB = 256 / LPR;
  const int r = threadIdx.x & (LPR - 1);
  const int grp = threadIdx.x / LPR;
  float loss_p = 0.f;
  const int64_t rows_per_iter = (int64_t)gridDim.x * GPB * RPG;
  int64_t base = ((int64_t)blockIdx.x * GPB + grp) * RPG;
  f32x4 uu[RPG][NV4], vv[RPG][NV4];
  float tg[RPG], wt[RPG];
  auto load = [&](int64_t b0) {
#pragma unroll
    for (int q = 0; q < RPG; ++q) {
      const int64_t row = min(b0 + q, B - 1);
      const f32x4* u4 = reinterpret_cast<const f32x4*>(U + row * D);
      const f32x4* v4 = reinterpret_cast<const f32x4*>(V + row * D);
#pragma unroll
      for (int k = 0; k < NV4; ++k) {
        uu[q][k] = __builtin_nontemporal_load(u4 + r + LPR * k);
        vv[q][k] = __builtin_nontemporal_load(v4 + r + LPR * k);
      }
      tg[q] = tgt[row];
      wt[q] = wgt[row];
    }
  };
  if (base < B) load(base);
  for (; base < B; base += rows_per_iter) {
    f32x4 cu[RPG][NV4], cv[RPG][NV4];
    float ct[RPG], cw[RPG];
#pragma unroll
    for (int q = 0; q < RPG; ++q) {
      ct[q] = tg[q]; cw[q] = wt[q];
#pragma unroll
      for (int k = 0; k < NV4; ++k) { cu[q][k] = uu[q][k]; cv[q][k] = vv[q][k]; }
    }
    if (PF && base + rows_per_iter < B) load(base + rows_per_iter);
#pragma unroll
    for (int q = 0; q < RPG; ++q) {
      const int64_t row = base + q;
      float uv = 0.f, nuu = 0.f, nvv = 0.f;
#pragma unroll
      for (int k = 0; k < NV4; ++k)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          uv += cu[q][k][e] * cv[q][k][e];
          nuu += cu[q][k][e] * cu[q][k][e];
          nvv += cv[q][k][e] * cv[q][k][e];
        }
      uv = red_lpr<LPR>(uv);
      nuu = red_lpr<LPR>(nuu);
      nvv = red_lpr<LPR>(nvv);
      const float nu = sqrtf(nuu), nv = sqrtf(nvv);
      const float c = uv / (nu * nv);
      const float sc = c * s;
      const bool ok = row < B;
      if (r == 0 && ok) score[row] = sc;
      const float diff = sc - ct[q];
      const float ds = 2.f * diff * (cw[q] * inv_batch);
      if (r == 0 && ok) loss_p += cw[q] * diff * diff;
      const float dc = ds * s;
      const float a_u = dc / (nu * nv), b_u = dc * c / (nu * nu);
      const float a_v = a_u, b_v = dc * c / (nv * nv);
      if (ok) {
        f32x4* du4 = reinterpret_cast<f32x4*>(dU + row * D);
        f32x4* dv4 = reinterpret_cast<f32x4*>(dV + row * D);
#pragma unroll
        for (int k = 0; k < NV4; ++k) {
          __builtin_nontemporal_store(a_u * cv[q][k] - b_u * cu[q][k], du4 + r + LPR * k);
          __builtin_nontemporal_store(a_v * cu[q][k] - b_v * cv[q][k], dv4 + r + LPR * k);
        }
      }
    }
    if (!PF && base + rows_per_iter < B) load(base + rows_per_iter);
  }
  if (r == 0 && loss_p != 0.f) atomicAdd(loss_sum, loss_p * inv_batch);
}

template <bool NT>
__global__ __launch_bounds__(256) void k_copy2(const f32x4* __restrict__ a, const f32x4* __restrict__ b,
                                               f32x4* __restrict__ x, f32x4* __restrict__ y, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const f32x4 p = ld4<NT>(a + i), q = ld4<NT>(b + i);
    st4<NT>(p, x + i);
    st4<NT>(q, y + i);
  }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

int main() {
  const int64_t B = 4194304;
  const int D = 128;
  const size_t nbytes = (size_t)B * D * 4;
  float *U, *V, *T, *W, *S, *dU, *dV, *L;
  CK(hipMalloc(&U, nbytes)); CK(hipMalloc(&V, nbytes)); CK(hipMalloc(&dU, nbytes)); CK(hipMalloc(&dV, nbytes));
  CK(hipMalloc(&T, B * 4)); CK(hipMalloc(&W, B * 4)); CK(hipMalloc(&S, B * 4)); CK(hipMalloc(&L, 4));
  {
    std::vector<float> h((size_t)B * D);
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 1000) / 500.f - 1.f;
    CK(hipMemcpy(U, h.data(), nbytes, hipMemcpyHostToDevice));
    for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 40503u + 7) % 997) / 498.f - 1.f;
    CK(hipMemcpy(V, h.data(), nbytes, hipMemcpyHostToDevice));
    std::vector<float> t(B), w(B);
    for (int64_t i = 0; i < B; ++i) { t[i] = (float)(i % 17) / 8.f - 1.f; w[i] = 1.f + (float)(i % 13); }
    CK(hipMemcpy(T, t.data(), B * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(W, w.data(), B * 4, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  const double bytes = (double)B * 4 * (4.0 * D + 3);
  const int iters = 20;
  auto timeit = [&](const char* name, auto launch) {
    launch(); launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    const double us = ms * 1000.0 / iters;
    printf("%-40s %9.1f us  %7.1f GB/s\n", name, us, bytes / (us * 1e-6) / 1e9);
    fflush(stdout);
  };
  std::vector<float> ref(1024), got(1024);
  auto check = [&](const char* name) {
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), dU + (size_t)(B - 8) * D, 1024 * 4, hipMemcpyDeviceToHost));
    if (memcmp(got.data(), ref.data(), 4096)) printf("  MISMATCH %s\n", name);
  };
  const float s = 14.2857f, ib = 1.f / B;
#define RUN(NV, RPG, NTL, NTS, GRID)                                                                          \
  {                                                                                                           \
    char nm[96];                                                                                              \
    snprintf(nm, 96, "cos NV%d RPG%d ntl%d nts%d grid%d", NV, RPG, NTL, NTS, GRID);                           \
    timeit(nm, [&] { hipLaunchKernelGGL((k_cos<NV, RPG, NTL, NTS>), dim3(GRID), dim3(256), 0, 0, U, V, T, W, B, D, s, ib, S, dU, dV, L); }); \
    check(nm);                                                                                                \
  }
  hipLaunchKernelGGL((k_cos<2, 1, true, true>), dim3(4096), dim3(256), 0, 0, U, V, T, W, B, D, s, ib, S, dU, dV, L);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(ref.data(), dU + (size_t)(B - 8) * D, 4096, hipMemcpyDeviceToHost));
#define RUN2(LPR, RPG, PF, GRID)                                                                          \
  {                                                                                                           \
    char nm[96];                                                                                              \
    snprintf(nm, 96, "cos2 LPR%d RPG%d PF%d grid%d", LPR, RPG, PF, GRID);                                     \
    timeit(nm, [&] { hipLaunchKernelGGL((k_cos2<LPR, RPG, PF>), dim3(GRID), dim3(256), 0, 0, U, V, T, W, B, D, s, ib, S, dU, dV, L); }); \
    check(nm);                                                                                                \
  }
  RUN2(16, 2, true, 4096)
  RUN2(16, 2, true, 4096)
  // placement: the four streams in one pool, stream k at k * (nbytes + delta)
  {
    char* pool;
    const size_t slack = (size_t)64 << 20;
    CK(hipMalloc(&pool, 4 * (nbytes + slack)));
    for (size_t delta : {(size_t)0, (size_t)256, (size_t)4096, (size_t)65536, (size_t)1 << 20, ((size_t)2 << 20) + 4096,
                         (size_t)5 << 20, ((size_t)13 << 20) + 8192}) {
      float* u2 = (float*)(pool);
      float* v2 = (float*)(pool + 1 * (nbytes + delta));
      float* du2 = (float*)(pool + 2 * (nbytes + delta));
      float* dv2 = (float*)(pool + 3 * (nbytes + delta));
      CK(hipMemcpy(u2, U, nbytes, hipMemcpyDeviceToDevice));
      CK(hipMemcpy(v2, V, nbytes, hipMemcpyDeviceToDevice));
      char nm[96];
      snprintf(nm, 96, "cos2 pooled delta=%zu", delta);
      timeit(nm, [&] { hipLaunchKernelGGL((k_cos2<16, 2, true>), dim3(4096), dim3(256), 0, 0, u2, v2, T, W, B, D, s, ib, S, du2, dv2, L); });
      snprintf(nm, 96, "copy2 pooled delta=%zu", delta);
      timeit(nm, [&] { hipLaunchKernelGGL((k_copy2<true>), dim3(8192), dim3(256), 0, 0, (f32x4*)u2, (f32x4*)v2, (f32x4*)du2, (f32x4*)dv2, B * D / 4); });
    }
    CK(hipFree(pool));
  }
  printf("U %p V %p dU %p dV %p\n", (void*)U, (void*)V, (void*)dU, (void*)dV);
  printf("done\n");
  return 0;
}
