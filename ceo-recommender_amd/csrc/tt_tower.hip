// Fused CEOFirmMatcher tower kernels for gfx950 (MI355X).
//
// One training step over a batch of B pairs is five tower kernels + one
// reduce/Adam kernel (tt_optim.hip).  Every tower kernel works on R-row tiles
// of the batch (R/16 waves, one 16-row strip per wave) and keeps activations
// in LDS / registers; between kernels only the pre-BatchNorm activations
// (Z0, Z4), the post-ReLU grads (dY0, dY1), BN moment sums and per-tile
// weight-gradient partial slabs travel through memory (at B = 16K all of them
// sit in the 256 MB Infinity Cache).
//
//   k_l0_fwd    Z0 = X W0^T + b0 (X gathered: numeric ++ embeddings), BN0 sums
//               model.py:69-71 (embedding gather + concat), :38 (Linear)
//   k_l4_fwd    A0 = Dropout(ReLU(BN0(Z0))); Z4 = A0 W4^T + b4,       BN1 sums
//               model.py:39-42
//   k_top       A1 = Dropout(ReLU(BN1(Z4))) of BOTH towers; U,V = A1 W8^T + b8;
//               cosine score; weighted MSE; dU/dV; dW8, db8; dY1; dgamma1/dbeta1
//               model.py:43-46, :79-87, training.py:52 and their autograd
//   k_bwd_mid   dZ4 (BN1 backward); dW4, db4; dA0 = dZ4 W4; dY0; dgamma0/dbeta0
//   k_bwd_first dZ0 (BN0 backward); dW0, db0; dX -> embedding grads (K1 bwd)
//
// GEMMs run on v_mfma_f32_16x16x4_f32 (exact fp32).  Row-wise products
// (X W^T, dZ W) read LDS operands (ds_read_b128 where the layout allows); the
// row-contracted weight-gradient products (dZ^T X) are owned tile-by-tile by
// the waves and read transposed LDS images written straight from the MFMA
// accumulator layout (one ds_write_b128 per 16x16 tile).
//
// Latency discipline (B = 16K is a latency-bound size):
//  * every global load of a phase is issued before its first use (batched
//    16-B loads, small parameters prefetched at kernel entry);
//  * no per-element guards around memory operations on the hot path: hipcc
//    drains vmcnt(0) at every join of such guards.  Row indices are clamped
//    for loads, the workspace is padded to whole tiles so per-row stores need
//    no guard, and rows beyond B are masked out of statistics with selects.
#include "tt_common.h"

namespace tt {

// ---------------------------------------------------------------------------
// shared pieces
// ---------------------------------------------------------------------------

// BN coefficients of column c (train: shifted moment sums of this batch;
// eval: running stats).  `update`: fold the batch stats into the running
// estimates (momentum, unbiased variance, torch semantics) and publish
// mean|invstd for the backward kernels.
__device__ __forceinline__ void bn_coefs(const StepArgs& a, int H, const float* st, const float* shift,
                                         float* rm, float* rv, int64_t* nbt, float* fin, bool update,
                                         int c, float* mean_out, float* inv_out) {
  float mean, var;
  if (a.train) {
    const double Bd = (double)a.B;
    const float m1 = st[c] / (float)Bd;  // st: replica-summed S1|S2 (LDS)
    var = st[H + c] / (float)Bd - m1 * m1;
    var = var < 0.f ? 0.f : var;
    mean = shift[c] + m1;
    if (update) {
      const float mom = a.momentum;
      rm[c] = (1.f - mom) * rm[c] + mom * mean;
      rv[c] = (1.f - mom) * rv[c] + mom * (var * (float)(Bd / (Bd - 1.0)));
      fin[c] = mean;
      fin[H + c] = 1.f / sqrtf(var + a.eps);
      if (c == 0) *nbt += 1;
    }
  } else {
    mean = rm[c];
    var = rv[c];
  }
  *mean_out = mean;
  *inv_out = 1.f / sqrtf(var + a.eps);
}

// BN apply + ReLU + (train) dropout of one element.
__device__ __forceinline__ float bn_relu_drop(float z, float mean, float alpha, float beta, bool drop,
                                              uint64_t key, uint64_t ctr, uint32_t thr, float scale) {
  float y = (z - mean) * alpha + beta;
  y = y > 0.f ? y : 0.f;
  if (drop) y = dropout_keep(key, ctr, thr) ? y * scale : 0.f;
  return y;
}

// Sum the NREP replicas of N consecutive cross-block accumulators (replica
// stride `stride`) into dst[N] (LDS) with the whole block: every thread issues
// its NREP/G loads at once (G = groups of N threads), fixed summation order.
// Ends with dst visible to the block.  scratch: NTH floats of LDS.
template <int NTH, int N>
__device__ __forceinline__ void rep_sum(const float* rep, int stride, float* scratch, float* dst) {
  constexpr int G0 = NTH / N;
  constexpr int G = G0 < NREP ? G0 : NREP;
  constexpr int PER = NREP / G;
  static_assert(NTH % N == 0 && NREP % G == 0, "replica groups");
  const int c = (int)threadIdx.x % N, grp = (int)threadIdx.x / N;
  if (grp < G) {
    float v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = rep[(grp + k * G) * stride + c];
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) sum += v[k];
    scratch[grp * N + c] = sum;
  }
  __syncthreads();
  if (threadIdx.x < N) {
    float sum = 0.f;
#pragma unroll
    for (int q = 0; q < G; ++q) sum += scratch[q * N + threadIdx.x];
    dst[threadIdx.x] = sum;
  }
  __syncthreads();
}

// Block-wide column sums of NT C-layout tiles into LDS `red` (ds_add_f32).
template <int NT>
__device__ __forceinline__ void cols_to_lds(const float (&s)[NT], float* red) {
  const int l = lane_id(), r = l & 15, g = l >> 4;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const float v = col_reduce(s[j]);
    if (g == 0) atomicAdd(&red[16 * j + r], v);
  }
}

// Dataset rows of this tile (clamped into the batch) -> LDS.
template <int R>
__device__ __forceinline__ void stage_ridx(const StepArgs& a, int64_t base, int64_t r0, int64_t* ridx) {
  if (threadIdx.x < R) {
    const int64_t row = min(r0 + (int64_t)threadIdx.x, a.B - 1);
    ridx[threadIdx.x] = data_row(a, base, row);
  }
}

// Tower-input tile X[R][kp] gathered by ridx into LDS (needs ridx visible).
// Padding columns in_dim..kp are zero; rows beyond B hold a duplicate row.
template <int R, int NTH>
__device__ __forceinline__ void stage_x(const TowerDev& T, const int64_t* ridx, float* Xs, int ldk) {
  const int kp = T.kp;
  if (T.num_vec) {
    const int c4 = T.n_num >> 2, n4 = R * c4;
    constexpr int UNR = 4;
    if (n4 % (NTH * UNR) == 0) {
      for (int base = 0; base < n4; base += NTH * UNR) {
        float4 v[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
          const int e = base + (int)threadIdx.x + k * NTH;
          const int r = e / c4, c = e - r * c4;
          v[k] = *reinterpret_cast<const float4*>(T.num + ridx[r] * T.num_ld + 4 * c);
        }
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
          const int e = base + (int)threadIdx.x + k * NTH;
          const int r = e / c4, c = e - r * c4;
          *reinterpret_cast<float4*>(Xs + r * ldk + 4 * c) = v[k];
        }
      }
    } else {
      for (int base = 0; base < n4; base += NTH * UNR) {
        float4 v[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
          const int e = min(base + (int)threadIdx.x + k * NTH, n4 - 1);
          const int r = e / c4, c = e - r * c4;
          v[k] = *reinterpret_cast<const float4*>(T.num + ridx[r] * T.num_ld + 4 * c);
        }
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
          const int e = base + (int)threadIdx.x + k * NTH;
          if (e < n4) {
            const int r = e / c4, c = e - r * c4;
            *reinterpret_cast<float4*>(Xs + r * ldk + 4 * c) = v[k];
          }
        }
      }
    }
    zero_cols<NTH>(Xs, ldk, R, T.n_num, kp);
  } else {
    constexpr int UNR = 8;
    const int n = R * kp;
    for (int base = 0; base < n; base += NTH * UNR) {
      float v[UNR];
#pragma unroll
      for (int k = 0; k < UNR; ++k) {
        const int e = min(base + (int)threadIdx.x + k * NTH, n - 1);
        const int r = e / kp, c = e - r * kp;
        v[k] = tower_x(T, ridx[r], c);
      }
#pragma unroll
      for (int k = 0; k < UNR; ++k) {
        const int e = base + (int)threadIdx.x + k * NTH;
        if (e < n) {
          const int r = e / kp, c = e - r * kp;
          Xs[r * ldk + c] = v[k];
        }
      }
    }
  }
}

// Weight [N][K] (nn.Linear layout) -> LDS row-major [N][ld] (cols K..Kp zero)
template <int NTH>
__device__ __forceinline__ void stage_w(const float* W, int N, int K, int Kp, float* s, int ld) {
  if ((K & 3) == 0)
    g2s_f4<NTH, 4>(W, K, s, ld, N, K);
  else
    g2s_f1<NTH, 8>(W, K, s, ld, N, K);
  zero_cols<NTH>(s, ld, N, K, Kp);
}

// Block-parallel dot products  out[c] = bias[c] + sum_k x[k] * W[c][k]  for
// c < C (C*4 <= NTH): 4 threads per output, fixed summation order (so every
// block computes bitwise the same value).  `part` is LDS scratch [4][C].
template <int NTH>
__device__ __forceinline__ void row_dot(const float* x, const float* W, int ld, int K, int C, const float* bias,
                                        float* part, float* out) {
  const int c = threadIdx.x % C, q = threadIdx.x / C;
  if (q < 4) {
    const int k0 = (K * q) / 4, k1 = (K * (q + 1)) / 4;
    float z = 0.f;
    for (int k = k0; k < k1; ++k) z = fmaf(x[k], W[c * ld + k], z);
    part[q * C + c] = z;
  }
  __syncthreads();
  if (threadIdx.x < C) out[threadIdx.x] = ((part[threadIdx.x] + part[C + threadIdx.x]) +
                                           (part[2 * C + threadIdx.x] + part[3 * C + threadIdx.x])) +
                                          bias[threadIdx.x];
}

// ---------------------------------------------------------------------------
// k_l0_fwd : Z0 = X W0^T + b0 ; BN0 shifted moment sums ; (target, weight)
// ---------------------------------------------------------------------------
template <int R>
struct L0Lds {
  static size_t bytes(int kp) {
    return sizeof(float) * ((size_t)(H0 + R) * (kp + 4) + 2 * H0 + H0 + kp + 4 * H0) + sizeof(int64_t) * R;
  }
};

template <int R>
__global__ __launch_bounds__(R * 4) void k_l0_fwd(StepArgs a) {
  constexpr int NTH = R * 4;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int64_t step = step_for_first_kernel(a);
  const int64_t base = batch_row0(a, step);
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int kp = T.kp, ldk = kp + 4;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  int64_t* ridx = reinterpret_cast<int64_t*>(smem);  // [R]
  float* Ws = smem + 2 * R;        // [64][ldk]
  float* Xs = Ws + H0 * ldk;       // [R][ldk]
  float* red = Xs + R * ldk;       // [128]
  float* shl = red + 2 * H0;       // [64] moment shift = Z0 of batch row 0
  float* x0 = shl + H0;            // [kp] X of batch row 0
  float* part = x0 + kp;           // [4][64]
  TT_STAMP(0, 0);

  float bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bias[j] = T.b0[16 * j + r];
  if (a.state && blockIdx.x == 0 && t == 0 && threadIdx.x == 0) a.state->step_cur = step;
  stage_ridx<R>(a, base, r0, ridx);
  if (threadIdx.x < 2 * H0) red[threadIdx.x] = 0.f;
  if (a.train) {
    const int64_t dr0 = data_row(a, base, 0);
    for (int c = threadIdx.x; c < kp; c += NTH) x0[c] = tower_x(T, dr0, c);
  }
  stage_w<NTH>(T.W0, H0, T.in_dim, kp, Ws, ldk);
  __syncthreads();
  TT_STAMP(0, 1);
  if (t == 0 && a.target && threadIdx.x < R) {  // (target, weight) of the tile's rows for k_top
    const int64_t dr = ridx[threadIdx.x];
    const float tv = a.target[dr], wv = a.weight[dr];
    *reinterpret_cast<float2*>(a.tgw + 2 * (r0 + threadIdx.x)) = make_float2(tv, wv);
  }
  stage_x<R, NTH>(T, ridx, Xs, ldk);
  __syncthreads();
  TT_STAMP(0, 2);

  if (a.train) {
    // Shifted moment sums: every block derives the same shift (Z0 of the
    // batch's first row, identical fp32 ops in every block), which keeps
    // var = S2/B - (S1/B)^2 free of cancellation for any data offset.
    row_dot<NTH>(x0, Ws, ldk, T.in_dim, H0, T.b0, part, shl);
    if (blockIdx.x == 0 && threadIdx.x < H0) T.shift0[threadIdx.x] = shl[threadIdx.x];
  }
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = zero4();
  strip_gemm_nt<4>(Xs + 16 * w * ldk, ldk, Ws, ldk, kp, acc);
  __syncthreads();
  TT_STAMP(0, 3);

  float s1[4], s2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
    const float sh = a.train ? shl[col] : 0.f;
    s1[j] = 0.f;
    s2[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      const float z = acc[j][i] + bias[j];
      acc[j][i] = z;
      const float d = row < a.B ? z - sh : 0.f;
      s1[j] += d;
      s2[j] += d * d;
    }
  }
  if (a.train) {
    cols_to_lds<4>(s1, red);
    cols_to_lds<4>(s2, red + H0);
  }
  // Z0 (workspace rows are padded to whole tiles: no guard)
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) T.Z0[(r0 + 16 * w + 4 * g + i) * H0 + 16 * j + r] = acc[j][i];
  if (a.train) {
    __syncthreads();
    if (threadIdx.x < 2 * H0) atomicAdd(&T.st0[rep_of_block() * 2 * H0 + threadIdx.x], red[threadIdx.x]);
  }
  TT_STAMP(0, 4);
}

// ---------------------------------------------------------------------------
// k_l4_fwd : A0 = Drop(ReLU(BN0(Z0))) ; Z4 = A0 W4^T + b4 ; BN1 sums
// ---------------------------------------------------------------------------
template <int R>
struct L4Lds {
  static constexpr int LD = H0 + 4;
  static constexpr size_t bytes =
      sizeof(float) * ((size_t)(H1 + R) * LD + 3 * H0 + 2 * H1 + H0 + H1 + 4 * H1 + 4 * R + 2 * H0);
};

template <int R>
__global__ __launch_bounds__(R * 4) void k_l4_fwd(StepArgs a) {
  constexpr int NTH = R * 4;
  constexpr int LD = L4Lds<R>::LD;
  constexpr int Z4PT = R * (H0 / 4) / NTH;  // float4 of Z0 per thread
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int64_t step = step_current(a);
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  float* W4s = smem;               // [32][68]
  float* A0s = W4s + H1 * LD;      // [R][68]
  float* cf = A0s + R * LD;        // mean[64] alpha[64] beta[64]
  float* red = cf + 3 * H0;        // [64]
  float* a0r = red + 2 * H1;       // [64] A0 of batch row 0
  float* shl = a0r + H0;           // [32] moment shift = Z4 of batch row 0
  float* part = shl + H1;          // [4][32]
  float* rsc = part + 4 * H1;      // [NTH] replica-sum scratch
  float* rst = rsc + NTH;          // [2*64] BN0 moment sums S1|S2
  TT_STAMP(1, 0);

  // issue every load of the phase first (Z0 rows are padded: no clamp needed)
  float4 z[Z4PT];
#pragma unroll
  for (int k = 0; k < Z4PT; ++k) {
    const int e = threadIdx.x + k * NTH;
    const int rl = e >> 4, c4 = (e & 15) * 4;
    z[k] = *reinterpret_cast<const float4*>(T.Z0 + (r0 + rl) * H0 + c4);
  }
  float bias[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bias[j] = T.b4[16 * j + r];
  const float z0r = threadIdx.x < H0 ? T.Z0[threadIdx.x] : 0.f;
  if (a.train) rep_sum<NTH, 2 * H0>(T.st0, 2 * H0, rsc, rst);
  if (threadIdx.x < H0) {
    const int c = threadIdx.x;
    float mean, inv;
    bn_coefs(a, H0, rst, T.shift0, T.rm0, T.rv0, T.nbt0, T.fin0, a.update_stats && blockIdx.x == 0, c, &mean,
             &inv);
    cf[c] = mean;
    cf[H0 + c] = inv * T.g0[c];
    cf[2 * H0 + c] = T.be0[c];
  }
  if (threadIdx.x < 2 * H1) red[threadIdx.x] = 0.f;
  g2s_f4<NTH, 2>(T.W4, H0, W4s, LD, H1, H0);
  __syncthreads();
  TT_STAMP(1, 1);

  const bool drop = a.train && a.drop_thr > 0;
  const uint64_t key = dropout_key(a.seed, (uint64_t)step, t, 0);
#pragma unroll
  for (int k = 0; k < Z4PT; ++k) {
    const int e = threadIdx.x + k * NTH;
    const int rl = e >> 4, c4 = (e & 15) * 4;
    const uint64_t ctr = (uint64_t)(r0 + rl) * H0 + c4;
    float4 o;
    o.x = bn_relu_drop(z[k].x, cf[c4 + 0], cf[H0 + c4 + 0], cf[2 * H0 + c4 + 0], drop, key, ctr + 0, a.drop_thr, a.drop_scale);
    o.y = bn_relu_drop(z[k].y, cf[c4 + 1], cf[H0 + c4 + 1], cf[2 * H0 + c4 + 1], drop, key, ctr + 1, a.drop_thr, a.drop_scale);
    o.z = bn_relu_drop(z[k].z, cf[c4 + 2], cf[H0 + c4 + 2], cf[2 * H0 + c4 + 2], drop, key, ctr + 2, a.drop_thr, a.drop_scale);
    o.w = bn_relu_drop(z[k].w, cf[c4 + 3], cf[H0 + c4 + 3], cf[2 * H0 + c4 + 3], drop, key, ctr + 3, a.drop_thr, a.drop_scale);
    *reinterpret_cast<float4*>(A0s + rl * LD + c4) = o;
  }
  if (a.train && threadIdx.x < H0) {
    const int c = threadIdx.x;
    a0r[c] = bn_relu_drop(z0r, cf[c], cf[H0 + c], cf[2 * H0 + c], drop, key, (uint64_t)c, a.drop_thr, a.drop_scale);
  }
  __syncthreads();
  TT_STAMP(1, 2);

  if (a.train) {  // shift for the BN1 moment sums (see k_l0_fwd)
    row_dot<NTH>(a0r, W4s, LD, H0, H1, T.b4, part, shl);
    if (blockIdx.x == 0 && threadIdx.x < H1) T.shift1[threadIdx.x] = shl[threadIdx.x];
  }
  f32x4 acc[2] = {zero4(), zero4()};
  strip_gemm_nt<2>(A0s + 16 * w * LD, LD, W4s, LD, H0, acc);
  __syncthreads();
  TT_STAMP(1, 3);

  float s1[2], s2[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = 16 * j + r;
    const float sh = a.train ? shl[col] : 0.f;
    s1[j] = 0.f;
    s2[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      const float zz = acc[j][i] + bias[j];
      acc[j][i] = zz;
      const float d = row < a.B ? zz - sh : 0.f;
      s1[j] += d;
      s2[j] += d * d;
    }
  }
  if (a.train) {
    cols_to_lds<2>(s1, red);
    cols_to_lds<2>(s2, red + H1);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) T.Z4[(r0 + 16 * w + 4 * g + i) * H1 + 16 * j + r] = acc[j][i];
  if (a.train) {
    __syncthreads();
    if (threadIdx.x < 2 * H1) atomicAdd(&T.st1[rep_of_block() * 2 * H1 + threadIdx.x], red[threadIdx.x]);
  }
  TT_STAMP(1, 4);
}

// ---------------------------------------------------------------------------
// k_top : both towers' last layer, cosine score, loss, own-tower backward
// ---------------------------------------------------------------------------
template <int NDT, int R>
struct TopLds {
  static constexpr int DP = 16 * NDT;
  static constexpr int LDA = H1 + 4;
  static constexpr int W8s = 0;
  static constexpr int A1s = W8s + DP * LDA;
  static constexpr int Z4s = A1s + R * LDA;
  static constexpr int LDT = R + 4;            // transposed images [col][row]
  static constexpr int A1T = Z4s + R * LDA;    // [32][R+4]
  static constexpr int dUT = A1T + H1 * LDT;   // [DP][R+4]
  static constexpr int db8 = dUT + DP * LDT;
  static constexpr int cf1 = db8 + DP;
  static constexpr int red = cf1 + 2 * 4 * H1;
  static constexpr int scal = red + 2 * H1;  // [0] loss part [1] dls part
  static constexpr int rsc = scal + 4;        // [4R] replica-sum scratch
  static constexpr int rst = rsc + 4 * R;     // [2][2*32] BN1 moment sums S1|S2 per tower
  static constexpr int total = rst + 4 * H1;
};

template <int NDT, int R>
__global__ __launch_bounds__(R * 4) void k_top(StepArgs a) {
  using L = TopLds<NDT, R>;
  constexpr int NTH = R * 4;
  constexpr int ZPT = R * (H1 / 4) / NTH;                // float4 of Z4 per thread (2)
  constexpr int WPT = (L::DP * H1 / 4 + NTH - 1) / NTH;  // float4 of W8 per thread
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const bool bwd = a.mode != TOP_FWD;
  const int own = bwd ? (int)blockIdx.y : 0;
  const int oth = 1 - own;
  const int64_t step = step_current(a);
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  const int D = a.D;
  float* W8s = smem + L::W8s;
  float* A1s = smem + L::A1s;
  float* Z4s = smem + L::Z4s;
  TT_STAMP(2, 0);

  // ---- phase 0: issue every load: both towers' Z4 tile and W8, biases,
  // logit_scale, per-row (target, weight) or dscore
  float4 zo[ZPT], zs[ZPT], wo[WPT], ws[WPT];
#pragma unroll
  for (int k = 0; k < ZPT; ++k) {
    const int e = threadIdx.x + k * NTH;
    const int rl = e >> 3, c4 = (e & 7) * 4;
    zo[k] = *reinterpret_cast<const float4*>(a.tw[oth].Z4 + (r0 + rl) * H1 + c4);
    zs[k] = *reinterpret_cast<const float4*>(a.tw[own].Z4 + (r0 + rl) * H1 + c4);
  }
#pragma unroll
  for (int k = 0; k < WPT; ++k) {
    const int e = min((int)threadIdx.x + k * NTH, D * (H1 / 4) - 1);
    wo[k] = reinterpret_cast<const float4*>(a.tw[oth].W8)[e];
    ws[k] = reinterpret_cast<const float4*>(a.tw[own].W8)[e];
  }
  float bo[NDT], bs[NDT];
#pragma unroll
  for (int j = 0; j < NDT; ++j) {
    const int d = min(16 * j + r, D - 1);
    bo[j] = a.tw[oth].b8[d];
    bs[j] = a.tw[own].b8[d];
  }
  const float lsc = *a.logit_scale;
  float tg[4], wt[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t row = r0 + 16 * w + 4 * g + i;
    tg[i] = 0.f;
    wt[i] = 0.f;
    if (a.mode == TOP_TRAIN) {
      const float2 v = *reinterpret_cast<const float2*>(a.tgw + 2 * row);
      tg[i] = v.x;
      wt[i] = v.y;
    } else if (a.mode == TOP_BWD_GIVEN) {
      tg[i] = a.dscore[min(row, a.B - 1)];
    }
  }
  if (a.train) {
    rep_sum<NTH, 2 * H1>(a.tw[0].st1, 2 * H1, smem + L::rsc, smem + L::rst);
    rep_sum<NTH, 2 * H1>(a.tw[1].st1, 2 * H1, smem + L::rsc, smem + L::rst + 2 * H1);
  }
  if (threadIdx.x < 2 * H1) {
    const int tau = threadIdx.x / H1, c = threadIdx.x % H1;
    const TowerDev& T = a.tw[tau];
    const bool upd = a.update_stats && blockIdx.x == 0 && (bwd ? tau == own : true);
    float mean, inv;
    bn_coefs(a, H1, smem + L::rst + tau * 2 * H1, T.shift1, T.rm1, T.rv1, T.nbt1, T.fin1, upd, c, &mean, &inv);
    float* cf = smem + L::cf1 + tau * 4 * H1;
    cf[c] = mean;
    cf[H1 + c] = inv * T.g1[c];
    cf[2 * H1 + c] = T.be1[c];
    cf[3 * H1 + c] = inv;
  }
  if (threadIdx.x < L::DP) smem[L::db8 + threadIdx.x] = 0.f;
  if (threadIdx.x < 2 * H1 + 4) smem[L::red + threadIdx.x] = 0.f;  // red + scal
  __syncthreads();
  TT_STAMP(2, 1);

  const bool drop = a.train && a.drop_thr > 0;
  // write one tower's A1 (and optionally raw Z4) + W8 into LDS
  auto put = [&](int tau, const float4(&zz)[ZPT], const float4(&ww)[WPT], bool keep_z) {
    const float* cf = smem + L::cf1 + tau * 4 * H1;
    const uint64_t key = dropout_key(a.seed, (uint64_t)step, tau, 1);
#pragma unroll
    for (int k = 0; k < ZPT; ++k) {
      const int e = threadIdx.x + k * NTH;
      const int rl = e >> 3, c4 = (e & 7) * 4;
      const uint64_t ctr = (uint64_t)(r0 + rl) * H1 + c4;
      float4 o;
      o.x = bn_relu_drop(zz[k].x, cf[c4 + 0], cf[H1 + c4 + 0], cf[2 * H1 + c4 + 0], drop, key, ctr + 0, a.drop_thr, a.drop_scale);
      o.y = bn_relu_drop(zz[k].y, cf[c4 + 1], cf[H1 + c4 + 1], cf[2 * H1 + c4 + 1], drop, key, ctr + 1, a.drop_thr, a.drop_scale);
      o.z = bn_relu_drop(zz[k].z, cf[c4 + 2], cf[H1 + c4 + 2], cf[2 * H1 + c4 + 2], drop, key, ctr + 2, a.drop_thr, a.drop_scale);
      o.w = bn_relu_drop(zz[k].w, cf[c4 + 3], cf[H1 + c4 + 3], cf[2 * H1 + c4 + 3], drop, key, ctr + 3, a.drop_thr, a.drop_scale);
      *reinterpret_cast<float4*>(A1s + rl * L::LDA + c4) = o;
      if (keep_z) *reinterpret_cast<float4*>(Z4s + rl * L::LDA + c4) = zz[k];
    }
#pragma unroll
    for (int k = 0; k < WPT; ++k) {
      const int e = threadIdx.x + k * NTH;
      if (e < L::DP * (H1 / 4)) {
        const int d = e >> 3, c4 = (e & 7) * 4;
        const float4 v = d < D ? ww[k] : make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(W8s + d * L::LDA + c4) = v;
      }
    }
  };
  auto gemm = [&](const float(&bias)[NDT], f32x4(&acc)[NDT]) {
#pragma unroll
    for (int j = 0; j < NDT; ++j) acc[j] = zero4();
    strip_gemm_nt<NDT>(A1s + 16 * w * L::LDA, L::LDA, W8s, L::LDA, H1, acc);
#pragma unroll
    for (int j = 0; j < NDT; ++j) acc[j] += (16 * j + r < D) ? bias[j] : 0.f;
  };

  f32x4 accO[NDT], accS[NDT];
  put(oth, zo, wo, false);
  __syncthreads();
  TT_STAMP(2, 2);
  gemm(bo, accO);
  __syncthreads();
  TT_STAMP(2, 3);
  put(own, zs, ws, bwd);
  __syncthreads();
  TT_STAMP(2, 4);
  gemm(bs, accS);

  // ---- cosine (symmetric in own/other: no runtime choice of register arrays)
  const float s = expf(lsc);
  float ino[4], int_[4], cs[4], ds[4], sc[4];
  bool valid[4];
  float loss_p = 0.f, dls_p = 0.f;
  const float inv_b = 1.f / (float)a.B;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float uv = 0.f, oo = 0.f, tt2 = 0.f;
#pragma unroll
    for (int j = 0; j < NDT; ++j) {
      uv += accS[j][i] * accO[j][i];
      oo += accS[j][i] * accS[j][i];
      tt2 += accO[j][i] * accO[j][i];
    }
    uv = row_reduce16(uv);
    oo = row_reduce16(oo);
    tt2 = row_reduce16(tt2);
    ino[i] = __builtin_amdgcn_rsqf(oo);  // v_rsq_f32 (1 ulp): no IEEE divides
    int_[i] = __builtin_amdgcn_rsqf(tt2);
    cs[i] = uv * ino[i] * int_[i];
    sc[i] = cs[i] * s;
    const int64_t row = r0 + 16 * w + 4 * g + i;
    valid[i] = row < a.B;
    float dsi = 0.f;
    if (a.mode == TOP_TRAIN) {
      const float diff = sc[i] - tg[i];
      dsi = 2.f * diff * (wt[i] * inv_b);
      loss_p += valid[i] ? wt[i] * diff * diff : 0.f;
    } else if (a.mode == TOP_BWD_GIVEN) {
      dsi = tg[i];
    }
    ds[i] = valid[i] ? dsi : 0.f;
    dls_p += ds[i] * sc[i];
  }
  if (a.score && own == 0 && r == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      if (row < a.B) a.score[row] = sc[i];
    }
  }
  if (!bwd) return;

  if (own == 0) {  // loss + logit_scale grad once per row tile
    // every lane of a row group holds the same loss_p / dls_p: sum over g
    const float lp = col_reduce(loss_p), dp = col_reduce(dls_p);
    if (l == 0) {
      atomicAdd(smem + L::scal + 0, lp);
      atomicAdd(smem + L::scal + 1, dp);
    }
  }

  // own-tower output gradient in C layout (SURVEY 3D closed form),
  // d(own) = dc * (oth/|oth| - own * cos/|own|) / |own|
  f32x4 dO[NDT];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float dc = ds[i] * s;
    const float ka = valid[i] ? dc * ino[i] * int_[i] : 0.f;
    const float kb = valid[i] ? dc * cs[i] * ino[i] * ino[i] : 0.f;
#pragma unroll
    for (int j = 0; j < NDT; ++j) dO[j][i] = ka * accO[j][i] - kb * accS[j][i];
  }

  const TowerDev& T = a.tw[own];
  float* A1T = smem + L::A1T;
  float* dUT = smem + L::dUT;
  const float* cf = smem + L::cf1 + own * 4 * H1;
  f32x4 a1[2], z4[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a1[q][i] = A1s[(16 * w + 4 * g + i) * L::LDA + 16 * q + r];
      z4[q][i] = Z4s[(16 * w + 4 * g + i) * L::LDA + 16 * q + r];
    }
    store_tile_T(A1T, L::LDT, 16 * q, 16 * w, a1[q]);
  }
  // transposed dU image (one ds_write_b128 per tile) + db8 column sums
#pragma unroll
  for (int j = 0; j < NDT; ++j) {
    store_tile_T(dUT, L::LDT, 16 * j, 16 * w, dO[j]);
    const float cb = col_reduce(dO[j][0] + dO[j][1] + dO[j][2] + dO[j][3]);
    if (g == 0) atomicAdd(smem + L::db8 + 16 * j + r, cb);
  }
  __syncthreads();
  TT_STAMP(2, 5);

  // dW8 = dU^T A1 over all R rows of the tile: each wave owns whole output
  // tiles (no cross-wave reduction) and stores them into this tile's slab
  // (rows d >= D of dU are zero: the padded slab rows are never read).
  float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
  for (int p = w; p < NDT; p += R / 16) {
    f32x4 acc[2] = {zero4(), zero4()};
    strip_gemm_nt<2>(dUT + 16 * p * L::LDT, L::LDT, A1T, L::LDT, R, acc);
    if (16 * p + 16 <= D) {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) slab[T.so_W8 + (16 * p + 4 * g + i) * H1 + 16 * q + r] = acc[q][i];
    } else {
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int d = 16 * p + 4 * g + i;
          if (d < D) slab[T.so_W8 + d * H1 + 16 * q + r] = acc[q][i];
        }
    }
  }

  // dA1 = dU W8  (A from the transposed dU image, W8s row-major [d][k])
  f32x4 dA[2] = {zero4(), zero4()};
  strip_gemm_tn<2>(dUT + 16 * w, L::LDT, W8s, L::LDA, L::DP, dA);

  // dY1 = dA1 * mask*scale * [Y1 > 0]  ==  [A1 > 0] * dA1 * scale
  const float scl = (a.drop_thr > 0) ? a.drop_scale : 1.f;
  float sg[2], sb[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int col = 16 * q + r;
    const float mean = cf[col], inv = cf[3 * H1 + col];
    sg[q] = 0.f;
    sb[q] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float dy = a1[q][i] > 0.f ? dA[q][i] * scl : 0.f;  // 0 on rows >= B (dU = 0)
      T.dY1[(r0 + 16 * w + 4 * g + i) * H1 + col] = dy;
      sg[q] += dy * ((z4[q][i] - mean) * inv);
      sb[q] += dy;
    }
  }
  cols_to_lds<2>(sg, smem + L::red);
  cols_to_lds<2>(sb, smem + L::red + H1);
  __syncthreads();
  TT_STAMP(2, 6);

  if (threadIdx.x < H1) {
    atomicAdd(&T.gg1[rep_of_block() * BNG + threadIdx.x], smem[L::red + threadIdx.x]);
    atomicAdd(&T.gbe1[rep_of_block() * BNG + threadIdx.x], smem[L::red + H1 + threadIdx.x]);
  }
  if (own == 0 && threadIdx.x == 0) {
    float* lr = a.lsr + rep_of_block() * LSR;
    atomicAdd(lr, smem[L::scal + 1]);
    if (a.mode == TOP_TRAIN) atomicAdd(lr + 1, smem[L::scal + 0] / (float)a.B);
  }
  if (threadIdx.x < D) slab[T.so_b8 + threadIdx.x] = smem[L::db8 + threadIdx.x];
  TT_STAMP(2, 7);
}

// ---------------------------------------------------------------------------
// k_bwd_mid : BN1 backward -> dZ4 ; dW4, db4 ; dA0 = dZ4 W4 ; dY0 ; dgamma0/dbeta0
// ---------------------------------------------------------------------------
template <int R>
struct MidLds {
  static constexpr int LDW = H0 + 4;   // W4 row-major [32][68]
  static constexpr int LDT = R + 4;    // transposed images [col][row]
  static constexpr size_t bytes =
      sizeof(float) * ((size_t)H1 * LDW + (size_t)(H1 + H0) * LDT + H1 + 5 * H1 + 4 * H0 + 2 * H0 + 4 * R +
                       2 * H1);
};

template <int R>
__global__ __launch_bounds__(R * 4) void k_bwd_mid(StepArgs a) {
  static_assert(R == 64, "dW4 tile ownership assumes 4 waves");
  constexpr int NTH = R * 4;
  constexpr int LDW = MidLds<R>::LDW, LDT = MidLds<R>::LDT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int64_t step = step_current(a);
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  float* W4s = smem;                  // [32][68]  W4 row-major
  float* dZT = W4s + H1 * LDW;        // [32][R+4] dZ4^T
  float* A0T = dZT + H1 * LDT;        // [64][R+4] A0^T
  float* db4 = A0T + H0 * LDT;        // [32]
  float* c1 = db4 + H1;               // k1[32] mb[32] mg[32] mean1[32] inv1[32]
  float* c0 = c1 + 5 * H1;            // mean0[64] alpha0[64] beta0[64] inv0[64]
  float* red = c0 + 4 * H0;           // [128]
  float* rsc = red + 2 * H0;          // [NTH] replica-sum scratch
  float* rst = rsc + NTH;             // [2*32] sum dgamma1 | sum dbeta1
  TT_STAMP(3, 0);

  // issue the phase's loads: dY1, Z4 (2 tiles), Z0 (4 tiles) in C layout
  f32x4 dy1[2], zz4[2], zz0[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t row = r0 + 16 * w + 4 * g + i;
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      dy1[q][i] = T.dY1[row * H1 + 16 * q + r];
      zz4[q][i] = T.Z4[row * H1 + 16 * q + r];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) zz0[j][i] = T.Z0[row * H0 + 16 * j + r];
  }
  const float invB = 1.f / (float)a.B;
  rep_sum<NTH, 2 * H1>(T.gg1, BNG, rsc, rst);  // gg1|gbe1 are adjacent in a replica
  if (threadIdx.x < H1) {
    const int c = threadIdx.x;
    const float inv = T.fin1[H1 + c];
    c1[c] = inv * T.g1[c];
    c1[H1 + c] = rst[H1 + c] * invB;
    c1[2 * H1 + c] = rst[c] * invB;
    c1[3 * H1 + c] = T.fin1[c];
    c1[4 * H1 + c] = inv;
  } else if (threadIdx.x < H1 + H0) {
    const int c = threadIdx.x - H1;
    const float inv = T.fin0[H0 + c];
    c0[c] = T.fin0[c];
    c0[H0 + c] = inv * T.g0[c];
    c0[2 * H0 + c] = T.be0[c];
    c0[3 * H0 + c] = inv;
  }
  if (threadIdx.x < H1) db4[threadIdx.x] = 0.f;
  if (threadIdx.x < 2 * H0) red[threadIdx.x] = 0.f;
  g2s_f4<NTH, 2>(T.W4, H0, W4s, LDW, H1, H0);
  __syncthreads();
  TT_STAMP(3, 1);

  // dZ4 (BN1 backward) and the recomputed A0 / normalised Z0, all C layout;
  // transposed images for the rows-contracted dW4 product
  f32x4 dz[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int col = 16 * q + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      const float zh = (zz4[q][i] - c1[3 * H1 + col]) * c1[4 * H1 + col];
      const float v = c1[col] * (dy1[q][i] - c1[H1 + col] - zh * c1[2 * H1 + col]);
      dz[q][i] = row < a.B ? v : 0.f;
    }
    store_tile_T(dZT, LDT, 16 * q, 16 * w, dz[q]);
    const float cb = col_reduce(dz[q][0] + dz[q][1] + dz[q][2] + dz[q][3]);
    if (g == 0) atomicAdd(db4 + col, cb);
  }
  const bool drop = a.drop_thr > 0;
  const uint64_t key = dropout_key(a.seed, (uint64_t)step, t, 0);
  f32x4 a0[4], zh0[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      const float z = zz0[j][i];
      const bool ok = row < a.B;
      const float av = bn_relu_drop(z, c0[col], c0[H0 + col], c0[2 * H0 + col], drop, key,
                                    (uint64_t)row * H0 + col, a.drop_thr, a.drop_scale);
      a0[j][i] = ok ? av : 0.f;
      zh0[j][i] = ok ? (z - c0[col]) * c0[3 * H0 + col] : 0.f;
    }
    store_tile_T(A0T, LDT, 16 * j, 16 * w, a0[j]);
  }
  __syncthreads();
  TT_STAMP(3, 2);

  // dW4 = dZ4^T A0 over the tile's rows: wave w owns h1-tile (w&1) x h0-tiles
  // 2*(w>>1)..+1 and writes them straight into this tile's slab
  float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
  {
    const int p = w & 1, q0 = 2 * (w >> 1);
    f32x4 acc[2] = {zero4(), zero4()};
    strip_gemm_nt<2>(dZT + 16 * p * LDT, LDT, A0T + 16 * q0 * LDT, LDT, R, acc);
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) slab[T.so_W4 + (16 * p + 4 * g + i) * H0 + 16 * (q0 + q) + r] = acc[q][i];
  }

  // dA0 = dZ4 W4  (K = 32; A from the transposed image, W4 row-major)
  f32x4 dA[4] = {zero4(), zero4(), zero4(), zero4()};
  strip_gemm_tn<4>(dZT + 16 * w, LDT, W4s, LDW, H1, dA);
  const float scl = drop ? a.drop_scale : 1.f;
  float sg[4], sb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
    sg[j] = 0.f;
    sb[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float dy = a0[j][i] > 0.f ? dA[j][i] * scl : 0.f;  // 0 on rows >= B (a0 = 0)
      T.dY0[(r0 + 16 * w + 4 * g + i) * H0 + col] = dy;
      sg[j] += dy * zh0[j][i];
      sb[j] += dy;
    }
  }
  cols_to_lds<4>(sg, red);
  cols_to_lds<4>(sb, red + H0);
  __syncthreads();
  TT_STAMP(3, 3);
  if (threadIdx.x < H0) {
    atomicAdd(&T.gg0[rep_of_block() * BNG + threadIdx.x], red[threadIdx.x]);
    atomicAdd(&T.gbe0[rep_of_block() * BNG + threadIdx.x], red[H0 + threadIdx.x]);
  }
  if (threadIdx.x < H1) slab[T.so_b4 + threadIdx.x] = db4[threadIdx.x];
  TT_STAMP(3, 4);
}

// ---------------------------------------------------------------------------
// k_bwd_first : BN0 backward -> dZ0 ; dW0 = dZ0^T X ; db0 ; dX -> embedding grads
// ---------------------------------------------------------------------------
template <int R>
struct FirstLds {
  static constexpr int LDT = R + 4;
  // XT [kp][R+4] (X^T; reused as W0 [64][kp+4] by the embedding pass) | dZT [64][R+4]
  __host__ __device__ static size_t xt_floats(int kp) {
    const size_t a = (size_t)kp * LDT, b = (size_t)H0 * (kp + 4);
    return a > b ? a : b;
  }
  static size_t bytes(int kp) {
    return sizeof(float) * (xt_floats(kp) + (size_t)H0 * LDT + H0 + 5 * H0 + 2 * R + 4 * R + 2 * H0);
  }
};

template <int R>
__global__ __launch_bounds__(R * 4) void k_bwd_first(StepArgs a) {
  static_assert(R == 64, "dW0 tile ownership assumes 4 waves (one per 16 outputs of 64)");
  constexpr int NTH = R * 4;
  constexpr int LDT = FirstLds<R>::LDT;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int64_t step = step_current(a);
  const int64_t base = batch_row0(a, step);
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  const int kp = T.kp, ldk = kp + 4, KT = kp / 16;
  const bool emb = T.n_cat > 0;
  int64_t* ridx = reinterpret_cast<int64_t*>(smem);  // [R]
  float* XT = smem + 2 * R;                            // [kp][R+4]
  float* dZT = XT + FirstLds<R>::xt_floats(kp);        // [64][R+4]
  float* db0 = dZT + H0 * LDT;                         // [64]
  float* c0 = db0 + H0;                                // k0[64] mb[64] mg[64] mean0[64] inv0[64]
  float* rsc = c0 + 5 * H0;                            // [NTH] replica-sum scratch
  float* rst = rsc + NTH;                              // [2*64] sum dgamma0 | sum dbeta0
  TT_STAMP(4, 0);

  f32x4 dy0[4], zz0[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t row = r0 + 16 * w + 4 * g + i;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      dy0[j][i] = T.dY0[row * H0 + 16 * j + r];
      zz0[j][i] = T.Z0[row * H0 + 16 * j + r];
    }
  }
  stage_ridx<R>(a, base, r0, ridx);
  const float invB = 1.f / (float)a.B;
  rep_sum<NTH, 2 * H0>(T.gg0, BNG, rsc, rst);  // gg0|gbe0 are adjacent in a replica
  if (threadIdx.x < H0) {
    const int c = threadIdx.x;
    const float inv = T.fin0[H0 + c];
    c0[c] = inv * T.g0[c];
    c0[H0 + c] = rst[H0 + c] * invB;
    c0[2 * H0 + c] = rst[c] * invB;
    c0[3 * H0 + c] = T.fin0[c];
    c0[4 * H0 + c] = inv;
    db0[c] = 0.f;
  }
  __syncthreads();
  TT_STAMP(4, 1);

  // X^T tile: consecutive threads take consecutive rows (conflict-free LDS
  // writes); gathered 16-B row loads, all issued before the stores
  if (T.num_vec) {
    const int c4n = T.n_num >> 2, n4 = R * c4n;
    constexpr int UNR = 4;
    if (n4 % (NTH * UNR) == 0) {
      for (int b0 = 0; b0 < n4; b0 += NTH * UNR) {
        float4 v[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
          const int e = b0 + (int)threadIdx.x + k * NTH;
          v[k] = *reinterpret_cast<const float4*>(T.num + ridx[e % R] * T.num_ld + 4 * (e / R));
        }
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
          const int e = b0 + (int)threadIdx.x + k * NTH;
          const int rr = e % R, c = 4 * (e / R);
          XT[(c + 0) * LDT + rr] = v[k].x;
          XT[(c + 1) * LDT + rr] = v[k].y;
          XT[(c + 2) * LDT + rr] = v[k].z;
          XT[(c + 3) * LDT + rr] = v[k].w;
        }
      }
    } else {
      for (int b0 = 0; b0 < n4; b0 += NTH * UNR) {
        float4 v[UNR];
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
          const int e = min(b0 + (int)threadIdx.x + k * NTH, n4 - 1);
          v[k] = *reinterpret_cast<const float4*>(T.num + ridx[e % R] * T.num_ld + 4 * (e / R));
        }
#pragma unroll
        for (int k = 0; k < UNR; ++k) {
          const int e = b0 + (int)threadIdx.x + k * NTH;
          if (e < n4) {
            const int rr = e % R, c = 4 * (e / R);
            XT[(c + 0) * LDT + rr] = v[k].x;
            XT[(c + 1) * LDT + rr] = v[k].y;
            XT[(c + 2) * LDT + rr] = v[k].z;
            XT[(c + 3) * LDT + rr] = v[k].w;
          }
        }
      }
    }
    for (int e = threadIdx.x; e < (kp - T.n_num) * R; e += NTH) XT[(T.n_num + e / R) * LDT + e % R] = 0.f;
  } else {
    constexpr int UNR = 8;
    const int n = R * kp;
    for (int b0 = 0; b0 < n; b0 += NTH * UNR) {
      float v[UNR];
#pragma unroll
      for (int k = 0; k < UNR; ++k) {
        const int e = min(b0 + (int)threadIdx.x + k * NTH, n - 1);
        v[k] = tower_x(T, ridx[e % R], e / R);
      }
#pragma unroll
      for (int k = 0; k < UNR; ++k) {
        const int e = b0 + (int)threadIdx.x + k * NTH;
        if (e < n) XT[(e / R) * LDT + e % R] = v[k];
      }
    }
  }

  // dZ0 (BN0 backward), C layout -> transposed image; db0 column sums
  f32x4 dz[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      const float zh = (zz0[j][i] - c0[3 * H0 + col]) * c0[4 * H0 + col];
      const float v = c0[col] * (dy0[j][i] - c0[H0 + col] - zh * c0[2 * H0 + col]);
      dz[j][i] = row < a.B ? v : 0.f;
    }
    store_tile_T(dZT, LDT, 16 * j, 16 * w, dz[j]);
    const float cb = col_reduce(dz[j][0] + dz[j][1] + dz[j][2] + dz[j][3]);
    if (g == 0) atomicAdd(db0 + col, cb);
  }
  __syncthreads();
  TT_STAMP(4, 2);

  // dW0 = dZ0^T X over the tile's rows: wave w owns outputs 16w..16w+15 and
  // every input column tile; results go straight into this tile's slab
  float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
  const int in = T.in_dim;
  auto put_w0 = [&](int kt, const f32x4& acc) {
    const int k = 16 * kt + r;
    float* dst = slab + T.so_W0 + (16 * w + 4 * g) * in + k;
    if (16 * kt + 16 <= in) {
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[i * in] = acc[i];
    } else if (k < in) {
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[i * in] = acc[i];
    }
  };
  int kt = 0;
  for (; kt + 4 <= KT; kt += 4) {
    f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
    strip_gemm_nt<4>(dZT + 16 * w * LDT, LDT, XT + 16 * kt * LDT, LDT, R, acc);
#pragma unroll
    for (int q = 0; q < 4; ++q) put_w0(kt + q, acc[q]);
  }
  for (; kt < KT; ++kt) {
    f32x4 acc[1] = {zero4()};
    strip_gemm_nt<1>(dZT + 16 * w * LDT, LDT, XT + 16 * kt * LDT, LDT, R, acc);
    put_w0(kt, acc[0]);
  }
  if (emb) {
    // dX = dZ0 W0 on the embedding columns -> scatter-add into the tables.
    // W0 (row-major [64][ldk]) takes over the X^T image's LDS.
    __syncthreads();
    float* W0s = XT;
    stage_w<NTH>(T.W0, H0, T.in_dim, kp, W0s, ldk);
    __syncthreads();
    for (int ktt = T.n_num / 16; ktt < KT; ++ktt) {
      f32x4 dx[1] = {zero4()};
      strip_gemm_tn<1>(dZT + 16 * w, LDT, W0s + 16 * ktt, ldk, H0, dx);
      const int col = 16 * ktt + r;
      if (col >= T.n_num && col < T.in_dim) {
        const int c = col - T.n_num;
        const int jj = c / T.emb_dim, e = c - jj * T.emb_dim;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rl = 16 * w + 4 * g + i;
          if (r0 + rl >= a.B) continue;
          int64_t code = T.cat[ridx[rl] * T.cat_ld + jj];
          code = code < 0 ? 0 : (code >= T.emb_rows[jj] ? T.emb_rows[jj] - 1 : code);
          atomicAdd(T.gemb[jj] + code * T.emb_dim + e, dx[0][i]);
        }
      }
    }
  }
  if (threadIdx.x < H0) slab[T.so_b0 + threadIdx.x] = db0[threadIdx.x];
  TT_STAMP(4, 3);
}

template __global__ void k_l0_fwd<64>(StepArgs);
template __global__ void k_l4_fwd<64>(StepArgs);
template __global__ void k_top<4, 64>(StepArgs);
template __global__ void k_top<8, 64>(StepArgs);
template __global__ void k_top<4, 128>(StepArgs);
template __global__ void k_top<8, 128>(StepArgs);
template __global__ void k_bwd_mid<64>(StepArgs);
template __global__ void k_bwd_first<64>(StepArgs);

}  // namespace tt
