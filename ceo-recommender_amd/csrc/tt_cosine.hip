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
constexpr int COS_RPG = 2;  // rows per 16-lane group per iteration
constexpr int COS_ROWS_PER_BLOCK = COS_ROWS_PER_BLOCK_ITER * COS_RPG;

// One 16-lane group owns COS_RPG rows per iteration and issues the NEXT
// iteration's loads (clamped addresses, no branches around loads) before
// this iteration's math and stores: 2 x NV4 x 2 float4 per lane in flight
// across the reduction, 5.6 TB/s vs 5.2 TB/s for one row without
// prefetch (tools/probes/cos_probe.hip, B = 4M, D = 128).
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
  const int64_t stride = (int64_t)gridDim.x * COS_ROWS_PER_BLOCK;
  int64_t base = ((int64_t)blockIdx.x * COS_ROWS_PER_BLOCK_ITER + (threadIdx.x >> 4)) * COS_RPG;
  f32x4 nu4[COS_RPG][NV4], nv4[COS_RPG][NV4];
  float ntg[COS_RPG], nwt[COS_RPG];
  auto load = [&](int64_t b0) {
#pragma unroll
    for (int q = 0; q < COS_RPG; ++q) {
      const int64_t row = min(b0 + q, B - 1);
      const f32x4* u4 = reinterpret_cast<const f32x4*>(U + row * D);
      const f32x4* v4 = reinterpret_cast<const f32x4*>(V + row * D);
#pragma unroll
      for (int k = 0; k < NV4; ++k) {
        const int c = min(r + 16 * k, n4 - 1);
        nu4[q][k] = __builtin_nontemporal_load(u4 + c);
        nv4[q][k] = __builtin_nontemporal_load(v4 + c);
      }
      if (BWD) {
        ntg[q] = tgt[row];
        nwt[q] = wgt[row];
      }
    }
  };
  if (base < B) load(base);
  for (; base < B; base += stride) {
    f32x4 uu[COS_RPG][NV4], vv[COS_RPG][NV4];
    float tg[COS_RPG], wt[COS_RPG];
#pragma unroll
    for (int q = 0; q < COS_RPG; ++q) {
#pragma unroll
      for (int k = 0; k < NV4; ++k) {
        const bool in = r + 16 * k < n4;
        uu[q][k] = in ? nu4[q][k] : zero4();
        vv[q][k] = in ? nv4[q][k] : zero4();
      }
      tg[q] = ntg[q];
      wt[q] = nwt[q];
    }
    if (base + stride < B) load(base + stride);
#pragma unroll
    for (int q = 0; q < COS_RPG; ++q) {
      const int64_t row = base + q;
      const bool valid = row < B;
      float uv = 0.f, nuu = 0.f, nvv = 0.f;
#pragma unroll
      for (int k = 0; k < NV4; ++k) {
        const f32x4 a = uu[q][k], b = vv[q][k];
        uv += a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
        nuu += a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
        nvv += b[0] * b[0] + b[1] * b[1] + b[2] * b[2] + b[3] * b[3];
      }
      uv = row_reduce16(uv);
      nuu = row_reduce16(nuu);
      nvv = row_reduce16(nvv);
      const float nu = sqrtf(nuu), nv = sqrtf(nvv);
      const float c = uv / (nu * nv);
      const float sc = c * s;
      if (r == 0 && valid) score[row] = sc;
      if (BWD) {
        const float diff = sc - tg[q];
        const float ds = 2.f * diff * (wt[q] * inv_batch);
        if (r == 0 && valid) {
          loss_p += wt[q] * diff * diff;
          dls_p += ds * sc;
        }
        const float dc = ds * s;
        const float a_u = dc / (nu * nv), b_u = dc * c / (nu * nu);
        const float a_v = dc / (nu * nv), b_v = dc * c / (nv * nv);
        f32x4* du4 = reinterpret_cast<f32x4*>(dU + row * D);
        f32x4* dv4 = reinterpret_cast<f32x4*>(dV + row * D);
#pragma unroll
        for (int k = 0; k < NV4; ++k) {
          const int cc = r + 16 * k;
          if (valid && cc < n4) {
            __builtin_nontemporal_store(a_u * vv[q][k] - b_u * uu[q][k], du4 + cc);
            __builtin_nontemporal_store(a_v * uu[q][k] - b_v * vv[q][k], dv4 + cc);
          }
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




// HBM stream ceiling (tt_stream_copy): one 16-B nontemporal load and store
// per thread, each block a contiguous 4 KiB, one block per 256 float4 (no
// grid-stride loop).  Of the shapes probed on the box (tools/copyprobe: 1 /
// 2 / 4 / 8 float4 per thread, block-contiguous or grid-stride, plain or
// nontemporal) this one moves the most: 6.3-6.5 TB/s read + write over 2 GiB
// against 4.4 TB/s for a grid-stride loop of 4 float4 per thread
// (bench.py cosine_roofline).
constexpr int COPY_THREADS = 256;

__global__ __launch_bounds__(COPY_THREADS) void k_stream_copy(const float4* __restrict__ src,
                                                              float4* __restrict__ dst, int64_t n4) {
  typedef float v4f __attribute__((ext_vector_type(4)));
  const int64_t i = (int64_t)blockIdx.x * COPY_THREADS + threadIdx.x;
  if (i < n4)
    __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const v4f*>(src) + i),
                                reinterpret_cast<v4f*>(dst) + i);
}

}  // namespace tt
