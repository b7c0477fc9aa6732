// k_cosine shapes, second probe: LPR lanes per row, NV float4 of u / v per
// lane, RPG rows per lane group per iteration, the next iteration's rows
// prefetched (PF) or not, nontemporal or plain loads (NTL).  Grid-stride over
// rows; the loss / dls partials as k_cosine (one atomic pair per block).
#include "../../ceo-recommender_amd/csrc/tt_common.h"
using namespace tt;

template <int LPR>
__device__ __forceinline__ float rsum(float v) {
  if constexpr (LPR >= 4) { v += dpp_mov<0xB1>(v); v += dpp_mov<0x4E>(v); }
  if constexpr (LPR >= 8) v += dpp_mov<0x141>(v);
  if constexpr (LPR >= 16) v += dpp_mov<0x140>(v);
  if constexpr (LPR >= 32) v = xrow16_add(v);
  return v;
}

template <int LPR, int NV, int RPG, bool PF, bool NTL>
__global__ __launch_bounds__(256) void k_cos2(const float* __restrict__ U, const float* __restrict__ V,
                                              const float* __restrict__ tgt, const float* __restrict__ wgt,
                                              int64_t B, int D, const float* logit_scale, float inv_batch,
                                              float* __restrict__ score, float* __restrict__ dU,
                                              float* __restrict__ dV, float* loss_sum, float* dls_sum) {
  constexpr int GPB = 256 / LPR;           // lane groups per block
  constexpr int RPB = GPB * RPG;           // rows per block per iteration
  __shared__ float red[2][4];
  const int rl = (int)threadIdx.x % LPR, grp = (int)threadIdx.x / LPR;
  const int n4 = D >> 2;
  const float s = expf(*logit_scale);
  float loss_p = 0.f, dls_p = 0.f;
  const int64_t stride = (int64_t)gridDim.x * RPB;
  int64_t base = ((int64_t)blockIdx.x * GPB + grp) * RPG;
  f32x4 nu[RPG][NV], nv[RPG][NV];
  float ntg[RPG], nwt[RPG];
  auto load = [&](int64_t b0) {
#pragma unroll
    for (int q = 0; q < RPG; ++q) {
      const int64_t row = min(b0 + q, B - 1);
      const f32x4* u4 = reinterpret_cast<const f32x4*>(U + row * D);
      const f32x4* v4 = reinterpret_cast<const f32x4*>(V + row * D);
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int c = min(rl + LPR * k, n4 - 1);
        if constexpr (NTL) { nu[q][k] = __builtin_nontemporal_load(u4 + c); nv[q][k] = __builtin_nontemporal_load(v4 + c); }
        else { nu[q][k] = u4[c]; nv[q][k] = v4[c]; }
      }
      ntg[q] = tgt[row];
      nwt[q] = wgt[row];
    }
  };
  if (base < B) load(base);
  for (; base < B; base += stride) {
    f32x4 uu[RPG][NV], vv[RPG][NV];
    float tg[RPG], wt[RPG];
    if constexpr (!PF) load(base);
#pragma unroll
    for (int q = 0; q < RPG; ++q) {
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const bool in = rl + LPR * k < n4;
        uu[q][k] = in ? nu[q][k] : zero4();
        vv[q][k] = in ? nv[q][k] : zero4();
      }
      tg[q] = ntg[q];
      wt[q] = nwt[q];
    }
    if constexpr (PF) { if (base + stride < B) load(base + stride); }
#pragma unroll
    for (int q = 0; q < RPG; ++q) {
      const int64_t row = base + q;
      const bool valid = row < B;
      float uv = 0.f, nuu = 0.f, nvv = 0.f;
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const f32x4 a = uu[q][k], b = vv[q][k];
        uv += a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
        nuu += a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
        nvv += b[0] * b[0] + b[1] * b[1] + b[2] * b[2] + b[3] * b[3];
      }
      uv = rsum<LPR>(uv);
      nuu = rsum<LPR>(nuu);
      nvv = rsum<LPR>(nvv);
      const float nu_ = sqrtf(nuu), nv_ = sqrtf(nvv);
      const float c = uv / (nu_ * nv_), sc = c * s;
      if (rl == 0 && valid) score[row] = sc;
      const float diff = sc - tg[q], ds = 2.f * diff * (wt[q] * inv_batch);
      if (rl == 0 && valid) { loss_p += wt[q] * diff * diff; dls_p += ds * sc; }
      const float dc = ds * s;
      const float a_u = dc / (nu_ * nv_), b_u = dc * c / (nu_ * nu_), b_v = dc * c / (nv_ * nv_);
      f32x4* du4 = reinterpret_cast<f32x4*>(dU + row * D);
      f32x4* dv4 = reinterpret_cast<f32x4*>(dV + row * D);
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        const int cc = rl + LPR * k;
        if (valid && cc < n4) {
          __builtin_nontemporal_store(a_u * vv[q][k] - b_u * uu[q][k], du4 + cc);
          __builtin_nontemporal_store(a_u * uu[q][k] - b_v * vv[q][k], dv4 + cc);
        }
      }
    }
  }
  loss_p = wave_reduce(loss_p);
  dls_p = wave_reduce(dls_p);
  if (lane_id() == 0) { red[0][wave_id()] = loss_p; red[1][wave_id()] = dls_p; }
  __syncthreads();
  if (threadIdx.x == 0) {
    atomicAdd(loss_sum, ((red[0][0] + red[0][1]) + (red[0][2] + red[0][3])) * inv_batch);
    atomicAdd(dls_sum, (red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
  }
}

extern "C" int cos_probe2(int v, int64_t grid, const float* u, const float* vv, const float* tg, const float* wt,
                          int64_t B, int D, const float* ls, float inv, float* score, float* du, float* dv,
                          float* loss, float* dls, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const dim3 g((unsigned)grid), t(256);
#define P(ID, L, N, R, PF, NT) \
  if (v == ID) { hipLaunchKernelGGL((k_cos2<L, N, R, PF, NT>), g, t, 0, s, u, vv, tg, wt, B, D, ls, inv, score, du, dv, loss, dls); return (int)hipGetLastError(); }
  P(0, 16, 2, 2, true, true)    // = k_cosine<2>
  P(1, 16, 2, 1, true, true)
  P(2, 16, 2, 4, true, true)
  P(3, 16, 2, 2, true, false)
  P(4, 8, 4, 1, true, true)
  P(5, 8, 4, 2, true, true)
  P(6, 32, 1, 2, true, true)
  P(7, 32, 1, 4, true, true)
  P(8, 16, 2, 2, false, true)
  P(9, 8, 4, 1, false, true)
  P(10, 4, 8, 1, true, true)
#undef P
  return -1;
}
