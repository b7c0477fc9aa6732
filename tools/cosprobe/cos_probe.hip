// Shapes of the fused cosine + weighted-MSE fwd/bwd stream (k_cosine) for the
// probe in cos_probe.py: LPR lanes per row, NV float4 of u and of v per lane,
// grid-stride over rows with a chosen grid.  Same arithmetic as k_cosine.
#include "../../ceo-recommender_amd/csrc/tt_common.h"
#include "../../ceo-recommender_amd/csrc/tt_cosine.hip"
using namespace tt;

template <int LPR>
__device__ __forceinline__ float rsum(float v) {
  v = row_reduce16(v);
  if constexpr (LPR >= 32) v = xrow16_add(v);
  if constexpr (LPR >= 64) v = xrow32_add(v);
  return v;
}

template <int LPR, int NV>
__global__ __launch_bounds__(256) void k_cos_probe(const float* __restrict__ U, const float* __restrict__ V,
                                                   const float* __restrict__ tgt, const float* __restrict__ wgt,
                                                   int64_t B, int D, const float* logit_scale, float inv_batch,
                                                   float* __restrict__ score, float* __restrict__ dU,
                                                   float* __restrict__ dV, float* loss_sum, float* dls_sum) {
  constexpr int RPB = 256 / LPR;
  __shared__ float red[2][4];
  const int rl = (int)threadIdx.x % LPR;
  const int n4 = D >> 2;
  const float s = expf(*logit_scale);
  float loss_p = 0.f, dls_p = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * RPB + (int)threadIdx.x / LPR; row < B; row += (int64_t)gridDim.x * RPB) {
    const f32x4* u4 = reinterpret_cast<const f32x4*>(U + row * D);
    const f32x4* v4 = reinterpret_cast<const f32x4*>(V + row * D);
    f32x4 uu[NV], vv[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int c = min(rl + LPR * k, n4 - 1);
      uu[k] = __builtin_nontemporal_load(u4 + c);
      vv[k] = __builtin_nontemporal_load(v4 + c);
    }
    const float tg = tgt[row], wt = wgt[row];
    float uv = 0.f, nuu = 0.f, nvv = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if (rl + LPR * k >= n4) uu[k] = vv[k] = zero4();
      const f32x4 a = uu[k], b = vv[k];
      uv += a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
      nuu += a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
      nvv += b[0] * b[0] + b[1] * b[1] + b[2] * b[2] + b[3] * b[3];
    }
    uv = rsum<LPR>(uv);
    nuu = rsum<LPR>(nuu);
    nvv = rsum<LPR>(nvv);
    const float nu = sqrtf(nuu), nv = sqrtf(nvv);
    const float c = uv / (nu * nv), sc = c * s;
    if (rl == 0) score[row] = sc;
    const float diff = sc - tg, ds = 2.f * diff * (wt * inv_batch);
    if (rl == 0) {
      loss_p += wt * diff * diff;
      dls_p += ds * sc;
    }
    const float dc = ds * s;
    const float a_u = dc / (nu * nv), b_u = dc * c / (nu * nu), b_v = dc * c / (nv * nv);
    f32x4* du4 = reinterpret_cast<f32x4*>(dU + row * D);
    f32x4* dv4 = reinterpret_cast<f32x4*>(dV + row * D);
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int cc = rl + LPR * k;
      if (cc < n4) {
        __builtin_nontemporal_store(a_u * vv[k] - b_u * uu[k], du4 + cc);
        __builtin_nontemporal_store(a_u * uu[k] - b_v * vv[k], dv4 + cc);
      }
    }
  }
  loss_p = wave_reduce(loss_p);
  dls_p = wave_reduce(dls_p);
  if (lane_id() == 0) {
    red[0][wave_id()] = loss_p;
    red[1][wave_id()] = dls_p;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(loss_sum, ((red[0][0] + red[0][1]) + (red[0][2] + red[0][3])) * inv_batch);
    atomicAdd(dls_sum, (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
  }
}

extern "C" int cos_probe(int lpr, int nv, int64_t grid, const float* u, const float* v, const float* tg,
                         const float* wt, int64_t B, int D, const float* ls, float inv, float* score, float* du,
                         float* dv, float* loss, float* dls, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const dim3 g((unsigned)grid), t(256);
#define P(L, N) \
  if (lpr == L && nv == N) { hipLaunchKernelGGL((k_cos_probe<L, N>), g, t, 0, s, u, v, tg, wt, B, D, ls, inv, score, du, dv, loss, dls); return (int)hipGetLastError(); }
  P(16, 2) P(32, 1) P(64, 1) P(16, 1) P(8, 4)
#undef P
  if (lpr == 0) {  // the shipped k_cosine (2 rows per 16-lane group, next rows prefetched) at this grid
    hipLaunchKernelGGL((k_cosine<2, true>), g, t, 0, s, u, v, tg, wt, B, D, ls, inv, score, du, dv, loss, dls);
    return (int)hipGetLastError();
  }
  return -1;
}
