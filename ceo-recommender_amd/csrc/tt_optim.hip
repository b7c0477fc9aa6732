// Gradient reduction + Adam over the flat parameter arena (gfx950).
//
// k_reduce_adam : for every parameter element, sum its per-row-tile partial
//   slabs (dW/db written by the tower kernels) in a fixed order -- or take the
//   atomically accumulated value (BN affine, embeddings, logit_scale) -- write
//   the full gradient, zero the accumulators for the next step, and optionally
//   apply Adam in the same pass (single-GPU training: one launch for K10+K11).
// k_adam : Adam alone (data-parallel: after the RCCL all-reduce of `grad`).
//
// Adam arithmetic follows torch 2.10 _single_tensor_adam (optim.Adam.step,
// training.py:55):  m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
//   denom = sqrt(v) / sqrt(bc2) + eps;  p.addcdiv_(m, denom, -lr/bc1)
// with bias corrections in double precision, element math in fp32.
#include "tt_common.h"

namespace tt {

struct AdamCoef {
  float w1, c2, b2, step_size, bc2s, eps;
};

__device__ __forceinline__ AdamCoef adam_coef(float lr, float b1, float b2, float eps, int64_t t) {
  const double bc1 = 1.0 - pow((double)b1, (double)t);
  const double bc2 = 1.0 - pow((double)b2, (double)t);
  AdamCoef c;
  c.w1 = (float)(1.0 - (double)b1);
  c.c2 = (float)(1.0 - (double)b2);
  c.b2 = b2;
  c.step_size = (float)((double)lr / bc1);
  c.bc2s = (float)sqrt(bc2);
  c.eps = eps;
  return c;
}

__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamCoef& c) {
  m = m + c.w1 * (g - m);           // lerp, weight < 0.5 branch
  v = v * c.b2 + (c.c2 * g) * g;    // mul_ + addcmul_
  const float denom = sqrtf(v) / c.bc2s + c.eps;
  p = p + (-c.step_size) * (m / denom);
}

__global__ __launch_bounds__(RED_E* RED_G, TT_RED_MINW) void k_reduce_adam(RedArgs a) {
  __shared__ float part[RED_G][RED_E];
  TT_STAMP(5, 0);
  // the step first: a later load would make its wait (in-order vmcnt) wait for the slabs
  const int64_t t = a.state ? a.state->step_cur : a.step_host;
  const int el = threadIdx.x & (RED_E - 1), pg = threadIdx.x / RED_E;
  const int64_t e = (int64_t)blockIdx.x * RED_E + el;
  int si = -1;
  if (e < a.n)
    for (int k = 0; k < a.n_seg; ++k)
      if (e >= a.seg[k].off && e < a.seg[k].off + a.seg[k].len) { si = k; break; }
  // the Adam state of this element is loaded up front: its latency overlaps the slab loads
  const bool owner = pg == 0 && si >= 0;
  float pp = 0.f, pm = 0.f, pv = 0.f;
  if (owner && a.apply_adam) {
    pp = a.p[e];
    pm = a.m[e];
    pv = a.v[e];
  }
  float acc = 0.f;
  // Adam's bias corrections (double pow: a long dependent chain) are computed
  // by the owner lanes between issuing the slab loads and summing them (was:
  // after the barrier, on the critical path; 8.2 -> 7.3 us).  Owner lanes
  // only: the same pow in every wave costs more (11.4 us) than it hides.
  // (The code shape matters: an equivalent lambda form measured 10.1 us.)
  AdamCoef c{};
  const bool adam_here = owner && a.apply_adam;
  bool coef_done = false;
  if (si >= 0) {
    const Seg& S = a.seg[si];
    if (S.kind == 0) {
      // fixed summation order (deterministic); UNR independent loads in flight
      constexpr int UNR = 256 / RED_G;  // 256 slabs / RED_G groups: every load of a thread in flight at once
      const float* base = a.slab[S.tower] + S.slab_off + (e - S.off);
      const int n = S.n_slabs;
      for (int p0 = pg; p0 < n; p0 += RED_G * UNR) {
        float v[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
          const int p = min(p0 + k * RED_G, n - 1);
          v[k] = base[(int64_t)p * a.slab_ld];
        }
        if (!coef_done) {
          if (adam_here) c = adam_coef(a.lr, a.b1, a.b2, a.eps, t);
          coef_done = true;
        }
#pragma unroll
        for (int k = 0; k < UNR; ++k) acc += (p0 + k * RED_G < n) ? v[k] : 0.f;
      }
    } else if (S.kind == 1) {
      if (pg == 0) acc = a.gacc[e];
    } else {  // replicas: group pg sums replicas pg, pg + RED_G, ... (fixed order) and zeroes them
      float* rp = S.rep + (e - S.off);
#pragma unroll
      for (int q = pg; q < NREP; q += RED_G) {
        acc += rp[q * S.rep_stride];
        rp[q * S.rep_stride] = 0.f;
      }
    }
  }
  if (!coef_done && adam_here) c = adam_coef(a.lr, a.b1, a.b2, a.eps, t);
  part[pg][el] = acc;
  // zero the BN moment sums consumed by this step (one element per thread of
  // the leading blocks); fold the loss replicas (block 0)
  {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      if (i >= 0 && i < a.zero_len[b]) a.zero_buf[b][i] = 0.f;
      i -= a.zero_len[b];
    }
  }
  if (blockIdx.x == 0) {
    if (a.lsr && threadIdx.x == 0) {
      float l = 0.f;
      for (int q = 0; q < NREP; ++q) {
        l += a.lsr[q * LSR + 1];
        a.lsr[q * LSR + 1] = 0.f;
      }
      if (a.loss_state) a.loss_state->loss_sum += l;
    }
  }
  __syncthreads();
  TT_STAMP(5, 1);
  if (!owner) return;
  float gsum = 0.f;
#pragma unroll
  for (int k = 0; k < RED_G; ++k) gsum += part[k][el];
  a.grad[e] = gsum;
  if (a.seg[si].kind == 1) a.gacc[e] = 0.f;
  if (a.apply_adam) {
    adam_elem(pp, pm, pv, gsum, c);
    a.p[e] = pp;
    a.m[e] = pm;
    a.v[e] = pv;
    if (a.state && blockIdx.x == 0 && el == 0) a.state->step_done = t;
  }
}

__global__ __launch_bounds__(256) void k_adam(float* __restrict__ P, const float* __restrict__ G,
                                              float* __restrict__ M, float* __restrict__ V, int64_t n,
                                              float lr, float b1, float b2, float eps, tt_state* state,
                                              int64_t step_host) {
  const int64_t t = state ? state->step_cur : step_host;
  const AdamCoef c = adam_coef(lr, b1, b2, eps, t);
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    float p = P[e], m = M[e], v = V[e];
    adam_elem(p, m, v, G[e], c);
    P[e] = p;
    M[e] = m;
    V[e] = v;
  }
  if (state && blockIdx.x == 0 && threadIdx.x == 0) state->step_done = t;
}

}  // namespace tt
