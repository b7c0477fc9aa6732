// Standalone fused L2-normalise + scaled cosine (+ weighted MSE fwd/bwd)
// over precomputed tower outputs (gfx950).
//
// Reference: model.py:79-87 (u/|u|, v/|v| without eps, exp(logit_scale) *
// row dot) and training.py:52 (mean of w (score - t)^2), plus their autograd
// reverse (SURVEY.md 3D closed form).
//
// HBM-bound streaming kernel: one row per 16-lane group (4 rows per wave in
// flight), 16-byte loads/stores, row reductions with DPP, each
// row's u and v kept in registers between the reduction and the gradient
// (read once, written once: 4(4D+3) bytes per pair for fwd+bwd).  Loss and
// logit-scale partials are reduced per block and added with one atomic each.
#include "tt_common.h"

namespace tt {

constexpr int COS_THREADS = 256;
constexpr int COS_ROWS_PER_BLOCK_ITER = COS_THREADS / 16;

template <int NV4, bool BWD>
__global__ __launch_bounds__(COS_THREADS) void k_cosine(const float* __restrict__ U, const float* __restrict__ V,
                                                        const float* __restrict__ tgt, const float* __restrict__ wgt,
                                                        int64_t B, int D, const float* logit_scale, float inv_batch,
                                                        float* __restrict__ score, float* __restrict__ dU,
                                                        float* __restrict__ dV, float* loss_sum, float* dls_sum) {
  __shared__ float red[2][COS_THREADS / 64];
  const int l = lane_id(), r = l & 15;
  const int n4 = D >> 2;
  const float s = expf(*logit_scale);
  float loss_p = 0.f, dls_p = 0.f;
  const int64_t stride = (int64_t)gridDim.x * COS_ROWS_PER_BLOCK_ITER;
  for (int64_t row = (int64_t)blockIdx.x * COS_ROWS_PER_BLOCK_ITER + (threadIdx.x >> 4); row < B; row += stride) {
    const float4* u4 = reinterpret_cast<const float4*>(U + row * D);
    const float4* v4 = reinterpret_cast<const float4*>(V + row * D);
    float4 uu[NV4], vv[NV4];
    float uv = 0.f, nuu = 0.f, nvv = 0.f;
#pragma unroll
    for (int k = 0; k < NV4; ++k) {
      const int c = r + 16 * k;
      if (c < n4) {
        const f32x4 a = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(u4 + c));
        const f32x4 b = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(v4 + c));
        uu[k] = make_float4(a[0], a[1], a[2], a[3]);
        vv[k] = make_float4(b[0], b[1], b[2], b[3]);
      } else {
        uu[k] = make_float4(0.f, 0.f, 0.f, 0.f);
        vv[k] = uu[k];
      }
      uv += uu[k].x * vv[k].x + uu[k].y * vv[k].y + uu[k].z * vv[k].z + uu[k].w * vv[k].w;
      nuu += uu[k].x * uu[k].x + uu[k].y * uu[k].y + uu[k].z * uu[k].z + uu[k].w * uu[k].w;
      nvv += vv[k].x * vv[k].x + vv[k].y * vv[k].y + vv[k].z * vv[k].z + vv[k].w * vv[k].w;
    }
    uv = row_reduce16(uv);
    nuu = row_reduce16(nuu);
    nvv = row_reduce16(nvv);
    const float nu = sqrtf(nuu), nv = sqrtf(nvv);
    const float c = uv / (nu * nv);
    const float sc = c * s;
    if (r == 0) score[row] = sc;
    if (BWD) {
      const float wt = wgt[row];
      const float diff = sc - tgt[row];
      const float ds = 2.f * diff * (wt * inv_batch);
      if (r == 0) {
        loss_p += wt * diff * diff;
        dls_p += ds * sc;
      }
      const float dc = ds * s;
      const float a_u = dc / (nu * nv), b_u = dc * c / (nu * nu);
      const float a_v = dc / (nu * nv), b_v = dc * c / (nv * nv);
      float4* du4 = reinterpret_cast<float4*>(dU + row * D);
      float4* dv4 = reinterpret_cast<float4*>(dV + row * D);
#pragma unroll
      for (int k = 0; k < NV4; ++k) {
        const int cc = r + 16 * k;
        if (cc < n4) {
          float4 gu, gv;
          gu.x = a_u * vv[k].x - b_u * uu[k].x;
          gu.y = a_u * vv[k].y - b_u * uu[k].y;
          gu.z = a_u * vv[k].z - b_u * uu[k].z;
          gu.w = a_u * vv[k].w - b_u * uu[k].w;
          gv.x = a_v * uu[k].x - b_v * vv[k].x;
          gv.y = a_v * uu[k].y - b_v * vv[k].y;
          gv.z = a_v * uu[k].z - b_v * vv[k].z;
          gv.w = a_v * uu[k].w - b_v * vv[k].w;
          __builtin_nontemporal_store(f32x4{gu.x, gu.y, gu.z, gu.w}, reinterpret_cast<f32x4*>(du4 + cc));
          __builtin_nontemporal_store(f32x4{gv.x, gv.y, gv.z, gv.w}, reinterpret_cast<f32x4*>(dv4 + cc));
        }
      }
    }
  }
  if (BWD) {
    loss_p = wave_reduce(loss_p);
    dls_p = wave_reduce(dls_p);
    if (l == 0) {
      red[0][wave_id()] = loss_p;
      red[1][wave_id()] = dls_p;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      float a = 0.f, b = 0.f;
      for (int k = 0; k < COS_THREADS / 64; ++k) {
        a += red[0][k];
        b += red[1][k];
      }
      atomicAdd(loss_sum, a * inv_batch);
      atomicAdd(dls_sum, b);
    }
  }
}

// scalar fallback for D % 4 != 0 (e.g. LATENT_DIM = 60 is fine: 60 % 4 == 0)
template <bool BWD>
__global__ __launch_bounds__(COS_THREADS) void k_cosine_scalar(const float* __restrict__ U, const float* __restrict__ V,
                                                               const float* __restrict__ tgt, const float* __restrict__ wgt,
                                                               int64_t B, int D, const float* logit_scale, float inv_batch,
                                                               float* __restrict__ score, float* __restrict__ dU,
                                                               float* __restrict__ dV, float* loss_sum, float* dls_sum) {
  const int r = lane_id() & 15;
  const float s = expf(*logit_scale);
  const int64_t stride = (int64_t)gridDim.x * COS_ROWS_PER_BLOCK_ITER;
  float loss_p = 0.f, dls_p = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * COS_ROWS_PER_BLOCK_ITER + (threadIdx.x >> 4); row < B; row += stride) {
    float uv = 0.f, nuu = 0.f, nvv = 0.f;
    for (int d = r; d < D; d += 16) {
      const float x = U[row * D + d], y = V[row * D + d];
      uv += x * y;
      nuu += x * x;
      nvv += y * y;
    }
    uv = row_reduce16(uv);
    nuu = row_reduce16(nuu);
    nvv = row_reduce16(nvv);
    const float nu = sqrtf(nuu), nv = sqrtf(nvv);
    const float c = uv / (nu * nv), sc = c * s;
    if (r == 0) score[row] = sc;
    if (BWD) {
      const float wt = wgt[row], diff = sc - tgt[row];
      const float ds = 2.f * diff * (wt * inv_batch);
      if (r == 0) {
        loss_p += wt * diff * diff;
        dls_p += ds * sc;
      }
      const float dc = ds * s;
      for (int d = r; d < D; d += 16) {
        const float x = U[row * D + d], y = V[row * D + d];
        dU[row * D + d] = dc / (nu * nv) * y - dc * c / (nu * nu) * x;
        dV[row * D + d] = dc / (nu * nv) * x - dc * c / (nv * nv) * y;
      }
    }
  }
  if (BWD) {
    loss_p = wave_reduce(loss_p);
    dls_p = wave_reduce(dls_p);
    if (lane_id() == 0) {
      atomicAdd(loss_sum, loss_p * inv_batch);
      atomicAdd(dls_sum, dls_p);
    }
  }
}




}  // namespace tt
