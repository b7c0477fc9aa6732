// Fused CEOFirmMatcher tower kernels for gfx950 (MI355X).
//
// One training step over a batch of B pairs is five tower kernels + one
// reduce/Adam kernel (tt_optim.hip).  Every tower kernel works on 64-row tiles
// of the batch (4 waves, one 16-row strip per wave) for one tower
// (blockIdx.y = tower) and keeps activations in LDS / registers; between
// kernels only the pre-BatchNorm activations (Z0, Z4), the post-ReLU grads
// (dY0, dY1), BN moment sums and per-tile weight-gradient partial slabs travel
// through HBM (all of them sit in the 256 MB Infinity Cache at B=16384).
//
//   k_l0_fwd   Z0 = X W0^T + b0 (X gathered: numeric ++ embeddings),   BN0 sums
//              model.py:69-71 (embedding gather+concat), :38 (Linear)
//   k_l4_fwd   A0 = Dropout(ReLU(BN0(Z0))); Z4 = A0 W4^T + b4,         BN1 sums
//              model.py:39-42
//   k_top      A1 = Dropout(ReLU(BN1(Z4))) for BOTH towers; U,V = A1 W8^T + b8;
//              cosine score; weighted MSE; dU/dV; dW8, db8; dY1; dgamma1/dbeta1
//              model.py:43-46, :79-87, training.py:52, autograd of those
//   k_bwd_mid  dZ4 (BN1 backward); dW4, db4; dA0 = dZ4 W4; dY0; dgamma0/dbeta0
//   k_bwd_first dZ0 (BN0 backward); dW0, db0; dX -> embedding grads (K1 bwd)
//
// GEMMs run on v_mfma_f32_16x16x4_f32 (exact fp32).  Row-wise products
// (X W^T, dZ W) read both operands from LDS with ds_read_b128; the
// row-contracted weight-gradient products (dZ^T X) take their operands
// straight from the MFMA accumulator layout (tt_common.h cl_gemm_tn).
#include "tt_common.h"

namespace tt {

// ---------------------------------------------------------------------------
// shared pieces
// ---------------------------------------------------------------------------

// BN coefficients for H columns of tower T (train: from the shifted moment
// sums of this batch; eval: running stats).  Writes mean / invstd to LDS.
// When `update` the caller's block also folds the batch stats into the
// running estimates (torch: momentum 0.1, unbiased variance) and publishes
// mean|invstd for the backward kernels.
__device__ __forceinline__ void bn_coefs(const StepArgs& a, int H, const float* st, const float* shift,
                                         float* rm, float* rv, int64_t* nbt, float* fin, bool update,
                                         int c, float* mean_out, float* inv_out) {
  float mean, var;
  if (a.train) {
    const double Bd = (double)a.B;
    const float m1 = st[c] / (float)Bd;
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

// Block-wide column sums of NT C-layout tiles (valid rows only are non-zero),
// accumulated into LDS `red` (must be zeroed) with ds_add_f32.
template <int NT>
__device__ __forceinline__ void cols_to_lds(const float (&s)[NT], float* red) {
  const int l = lane_id(), r = l & 15, g = l >> 4;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const float v = col_reduce(s[j]);
    if (g == 0) atomicAdd(&red[16 * j + r], v);
  }
}

// Stage a tower input tile X[ROWS][kp] (rows beyond B zero) into LDS.
__device__ __forceinline__ void stage_x(const StepArgs& a, const TowerDev& T, int64_t base, int64_t r0,
                                        float* Xs, int ldk) {
  const int kp = T.kp;
  if (T.n_cat == 0 && (T.n_num & 3) == 0 && (T.num_ld & 3) == 0) {
    const int q = kp >> 2;  // float4 per row
    for (int e = threadIdx.x; e < ROWS * q; e += THREADS) {
      const int rl = e / q, c4 = (e - rl * q) * 4;
      const int64_t row = r0 + rl;
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < a.B && c4 < T.n_num) {
        const int64_t dr = data_row(a, base, row);
        v = *reinterpret_cast<const float4*>(T.num + dr * T.num_ld + c4);
      }
      *reinterpret_cast<float4*>(Xs + rl * ldk + c4) = v;
    }
  } else {
    for (int e = threadIdx.x; e < ROWS * kp; e += THREADS) {
      const int rl = e / kp, c = e - rl * kp;
      const int64_t row = r0 + rl;
      float v = 0.f;
      if (row < a.B) v = tower_x(T, data_row(a, base, row), c);
      Xs[rl * ldk + c] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// k_l0_fwd : Z0 = X W0^T + b0 ; BN0 shifted moment sums
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(THREADS) void k_l0_fwd(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int64_t step = step_for_first_kernel(a);
  const int64_t base = batch_row0(a, step);
  const int64_t r0 = (int64_t)blockIdx.x * ROWS;
  const int kp = T.kp, ldk = kp + 4;
  float* Ws = smem;             // [64][ldk]
  float* Xs = Ws + H0 * ldk;    // [ROWS][ldk]
  float* red = Xs + ROWS * ldk; // [128]
  float* shl = red + 2 * H0;    // [64] moment shift = Z0 of batch row 0

  if (a.state && blockIdx.x == 0 && t == 0 && threadIdx.x == 0) a.state->step_cur = step;
  if (threadIdx.x < 2 * H0) red[threadIdx.x] = 0.f;

  for (int e = threadIdx.x; e < H0 * kp; e += THREADS) {
    const int n = e / kp, k = e - n * kp;
    Ws[n * ldk + k] = k < T.in_dim ? T.W0[n * T.in_dim + k] : 0.f;
  }
  stage_x(a, T, base, r0, Xs, ldk);
  __syncthreads();
  if (a.train && threadIdx.x < H0) {
    // Shifted moment sums: every block derives the same shift (Z0 of the
    // batch's first row, identical fp32 ops in every block), which keeps
    // var = S2/B - (S1/B)^2 free of cancellation for any data offset.
    const int c = threadIdx.x;
    const int64_t dr0 = data_row(a, base, 0);
    float z = 0.f;
    for (int k = 0; k < T.in_dim; ++k) z = fmaf(tower_x(T, dr0, k), Ws[c * ldk + k], z);
    z += T.b0[c];
    shl[c] = z;
    if (blockIdx.x == 0) T.shift0[c] = z;
  }
  __syncthreads();

  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = zero4();
  strip_gemm_nt<4>(Xs + 16 * w * ldk, ldk, Ws, ldk, kp, acc);

  float s1[4], s2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
    const float bias = T.b0[col];
    const float sh = a.train ? shl[col] : 0.f;
    s1[j] = 0.f;
    s2[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      const float z = acc[j][i] + bias;
      if (row < a.B) {
        T.Z0[row * H0 + col] = z;
        const float d = z - sh;
        s1[j] += d;
        s2[j] += d * d;
      }
    }
  }
  if (a.train) {
    cols_to_lds<4>(s1, red);
    cols_to_lds<4>(s2, red + H0);
    __syncthreads();
    if (threadIdx.x < 2 * H0) atomicAdd(&T.st0[threadIdx.x], red[threadIdx.x]);
  }
}

// ---------------------------------------------------------------------------
// k_l4_fwd : A0 = Drop(ReLU(BN0(Z0))) ; Z4 = A0 W4^T + b4 ; BN1 sums
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(THREADS) void k_l4_fwd(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int64_t step = step_current(a);
  const int64_t r0 = (int64_t)blockIdx.x * ROWS;
  constexpr int LD = H0 + 4;
  float* W4s = smem;                // [32][68]
  float* A0s = W4s + H1 * LD;       // [ROWS][68]
  float* cf = A0s + ROWS * LD;      // mean[64] alpha[64] beta[64]
  float* red = cf + 3 * H0;         // [64]
  float* a0r = red + 2 * H1;        // [64] A0 of batch row 0
  float* shl = a0r + H0;            // [32] moment shift = Z4 of batch row 0

  if (threadIdx.x < H0) {
    const int c = threadIdx.x;
    float mean, inv;
    bn_coefs(a, H0, T.st0, T.shift0, T.rm0, T.rv0, T.nbt0, T.fin0, a.update_stats && blockIdx.x == 0, c, &mean, &inv);
    cf[c] = mean;
    cf[H0 + c] = inv * T.g0[c];
    cf[2 * H0 + c] = T.be0[c];
  }
  if (threadIdx.x < 2 * H1) red[threadIdx.x] = 0.f;
  for (int e = threadIdx.x; e < H1 * H0; e += THREADS) {
    const int n = e / H0, k = e - n * H0;
    W4s[n * LD + k] = T.W4[e];
  }
  __syncthreads();

  const bool drop = a.train && a.drop_thr > 0;
  const uint64_t key = dropout_key(a.seed, (uint64_t)step, t, 0);
  if (a.train) {  // shift for the BN1 moment sums: Z4 of batch row 0 (see k_l0_fwd)
    if (threadIdx.x < H0) {
      const int c = threadIdx.x;
      a0r[c] = bn_relu_drop(T.Z0[c], cf[c], cf[H0 + c], cf[2 * H0 + c], drop, key, (uint64_t)c, a.drop_thr,
                            a.drop_scale);
    }
    __syncthreads();
    if (threadIdx.x < H1) {
      const int c = threadIdx.x;
      float z = 0.f;
      for (int k = 0; k < H0; ++k) z = fmaf(a0r[k], W4s[c * LD + k], z);
      z += T.b4[c];
      shl[c] = z;
      if (blockIdx.x == 0) T.shift1[c] = z;
    }
  }
  for (int e = threadIdx.x; e < ROWS * (H0 / 4); e += THREADS) {
    const int rl = e >> 4, c4 = (e & 15) * 4;
    const int64_t row = r0 + rl;
    float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
    if (row < a.B) {
      const float4 z = *reinterpret_cast<const float4*>(T.Z0 + row * H0 + c4);
      const uint64_t ctr = (uint64_t)row * H0 + c4;
      o.x = bn_relu_drop(z.x, cf[c4 + 0], cf[H0 + c4 + 0], cf[2 * H0 + c4 + 0], drop, key, ctr + 0, a.drop_thr, a.drop_scale);
      o.y = bn_relu_drop(z.y, cf[c4 + 1], cf[H0 + c4 + 1], cf[2 * H0 + c4 + 1], drop, key, ctr + 1, a.drop_thr, a.drop_scale);
      o.z = bn_relu_drop(z.z, cf[c4 + 2], cf[H0 + c4 + 2], cf[2 * H0 + c4 + 2], drop, key, ctr + 2, a.drop_thr, a.drop_scale);
      o.w = bn_relu_drop(z.w, cf[c4 + 3], cf[H0 + c4 + 3], cf[2 * H0 + c4 + 3], drop, key, ctr + 3, a.drop_thr, a.drop_scale);
    }
    *reinterpret_cast<float4*>(A0s + rl * LD + c4) = o;
  }
  __syncthreads();

  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  f32x4 acc[2] = {zero4(), zero4()};
  strip_gemm_nt<2>(A0s + 16 * w * LD, LD, W4s, LD, H0, acc);

  float s1[2], s2[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = 16 * j + r;
    const float bias = T.b4[col];
    const float sh = a.train ? shl[col] : 0.f;
    s1[j] = 0.f;
    s2[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      const float z = acc[j][i] + bias;
      if (row < a.B) {
        T.Z4[row * H1 + col] = z;
        const float d = z - sh;
        s1[j] += d;
        s2[j] += d * d;
      }
    }
  }
  if (a.train) {
    cols_to_lds<2>(s1, red);
    cols_to_lds<2>(s2, red + H1);
    __syncthreads();
    if (threadIdx.x < 2 * H1) atomicAdd(&T.st1[threadIdx.x], red[threadIdx.x]);
  }
}

// ---------------------------------------------------------------------------
// k_top : both towers' last layer, cosine score, loss, own-tower backward
// ---------------------------------------------------------------------------
// LDS layout (floats):  W8s[DP][36] | W8Ts[32][DP+4] | A1s[ROWS][36] |
//   Z4s[ROWS][36] | dUs[ROWS][DP+4] | dW8acc[DP][32] | db8acc[DP] |
//   cf1[2 towers][mean,alpha,beta,inv][32] | red[64] | rowred[ROWS*?]
template <int NDT>
struct TopLds {
  static constexpr int DP = 16 * NDT;
  static constexpr int LDA = H1 + 4;
  static constexpr int LDD = DP + 4;
  static constexpr int W8s = 0;
  static constexpr int W8Ts = W8s + DP * LDA;
  static constexpr int A1s = W8Ts + H1 * LDD;
  static constexpr int Z4s = A1s + ROWS * LDA;
  static constexpr int dUs = Z4s + ROWS * LDA;
  static constexpr int dW8 = dUs + ROWS * LDD;
  static constexpr int db8 = dW8 + DP * H1;
  static constexpr int cf1 = db8 + DP;
  static constexpr int red = cf1 + 2 * 4 * H1;
  static constexpr int scal = red + 2 * H1;  // [0]=loss part [1]=dls part
  static constexpr int total = scal + 4;
};

// Stage tower tau's W8 (and W8^T when `want_t`) and its A1 tile into LDS.
template <int NDT>
__device__ __forceinline__ void top_stage(const StepArgs& a, int tau, int64_t r0, uint64_t step, bool want_t,
                                          bool keep_z, float* smem) {
  using L = TopLds<NDT>;
  const TowerDev& T = a.tw[tau];
  const int D = a.D;
  float* W8s = smem + L::W8s;
  float* W8Ts = smem + L::W8Ts;
  float* A1s = smem + L::A1s;
  float* Z4s = smem + L::Z4s;
  const float* cf = smem + L::cf1 + tau * 4 * H1;
  for (int e = threadIdx.x; e < L::DP * H1; e += THREADS) {
    const int d = e >> 5, k = e & 31;
    const float v = d < D ? T.W8[d * H1 + k] : 0.f;
    W8s[d * L::LDA + k] = v;
    if (want_t) W8Ts[k * L::LDD + d] = v;
  }
  const bool drop = a.train && a.drop_thr > 0;
  const uint64_t key = dropout_key(a.seed, step, tau, 1);
  for (int e = threadIdx.x; e < ROWS * (H1 / 4); e += THREADS) {
    const int rl = e >> 3, c4 = (e & 7) * 4;
    const int64_t row = r0 + rl;
    float4 z = make_float4(0.f, 0.f, 0.f, 0.f), o = z;
    if (row < a.B) {
      z = *reinterpret_cast<const float4*>(T.Z4 + row * H1 + c4);
      const uint64_t ctr = (uint64_t)row * H1 + c4;
      o.x = bn_relu_drop(z.x, cf[c4 + 0], cf[H1 + c4 + 0], cf[2 * H1 + c4 + 0], drop, key, ctr + 0, a.drop_thr, a.drop_scale);
      o.y = bn_relu_drop(z.y, cf[c4 + 1], cf[H1 + c4 + 1], cf[2 * H1 + c4 + 1], drop, key, ctr + 1, a.drop_thr, a.drop_scale);
      o.z = bn_relu_drop(z.z, cf[c4 + 2], cf[H1 + c4 + 2], cf[2 * H1 + c4 + 2], drop, key, ctr + 2, a.drop_thr, a.drop_scale);
      o.w = bn_relu_drop(z.w, cf[c4 + 3], cf[H1 + c4 + 3], cf[2 * H1 + c4 + 3], drop, key, ctr + 3, a.drop_thr, a.drop_scale);
    }
    *reinterpret_cast<float4*>(A1s + rl * L::LDA + c4) = o;
    if (keep_z) *reinterpret_cast<float4*>(Z4s + rl * L::LDA + c4) = z;
  }
}

template <int NDT>
__device__ __forceinline__ void top_gemm(const StepArgs& a, int tau, const float* smem, f32x4 (&acc)[NDT]) {
  using L = TopLds<NDT>;
  const int w = wave_id(), r = lane_id() & 15;
#pragma unroll
  for (int j = 0; j < NDT; ++j) acc[j] = zero4();
  strip_gemm_nt<NDT>(smem + L::A1s + 16 * w * L::LDA, L::LDA, smem + L::W8s, L::LDA, H1, acc);
  const TowerDev& T = a.tw[tau];
#pragma unroll
  for (int j = 0; j < NDT; ++j) {
    const int d = 16 * j + r;
    const float b = d < a.D ? T.b8[d] : 0.f;
    acc[j] += b;
  }
}

template <int NDT>
__global__ __launch_bounds__(THREADS) void k_top(StepArgs a) {
  using L = TopLds<NDT>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const bool bwd = a.mode != TOP_FWD;
  const int own = bwd ? (int)blockIdx.y : 0;
  const int oth = 1 - own;
  const int64_t step = step_current(a);
  const int64_t base = batch_row0(a, step);
  const int64_t r0 = (int64_t)blockIdx.x * ROWS;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;

  // BN1 coefficients of both towers
  if (threadIdx.x < 2 * H1) {
    const int tau = threadIdx.x / H1, c = threadIdx.x % H1;
    const TowerDev& T = a.tw[tau];
    const bool upd = a.update_stats && blockIdx.x == 0 && (bwd ? tau == own : true);
    float mean, inv;
    bn_coefs(a, H1, T.st1, T.shift1, T.rm1, T.rv1, T.nbt1, T.fin1, upd, c, &mean, &inv);
    float* cf = smem + L::cf1 + tau * 4 * H1;
    cf[c] = mean;
    cf[H1 + c] = inv * T.g1[c];
    cf[2 * H1 + c] = T.be1[c];
    cf[3 * H1 + c] = inv;
  }
  for (int e = threadIdx.x; e < L::DP * H1 + L::DP; e += THREADS) smem[L::dW8 + e] = 0.f;  // dW8 + db8
  if (threadIdx.x < 2 * H1 + 4) smem[L::red + threadIdx.x] = 0.f;                       // red + scal
  __syncthreads();

  // pass 1: the other tower (forward only), pass 2: own tower (kept for bwd)
  f32x4 accO[NDT], accS[NDT];
  top_stage<NDT>(a, oth, r0, (uint64_t)step, false, false, smem);
  __syncthreads();
  top_gemm<NDT>(a, oth, smem, accO);
  __syncthreads();
  top_stage<NDT>(a, own, r0, (uint64_t)step, bwd, bwd, smem);
  __syncthreads();
  top_gemm<NDT>(a, own, smem, accS);

  // cosine is symmetric in (own, other): no runtime selection of register arrays
  const float s = expf(*a.logit_scale);
  float no[4], nt[4], cs[4], ds[4], sc[4];
  bool valid[4];
  float loss_p = 0.f, dls_p = 0.f;
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
    no[i] = sqrtf(oo);
    nt[i] = sqrtf(tt2);
    cs[i] = uv / (no[i] * nt[i]);
    sc[i] = cs[i] * s;
    const int64_t row = r0 + 16 * w + 4 * g + i;
    valid[i] = row < a.B;
    ds[i] = 0.f;
    if (valid[i]) {
      if (a.mode == TOP_TRAIN) {
        const int64_t dr = data_row(a, base, row);
        const float wt = a.weight[dr];
        const float diff = sc[i] - a.target[dr];
        const float invB = 1.f / (float)a.B;
        ds[i] = 2.f * diff * (wt * invB);
        loss_p += wt * diff * diff;
      } else if (a.mode == TOP_BWD_GIVEN) {
        ds[i] = a.dscore[row];
      }
      dls_p += ds[i] * sc[i];
      if (a.score && r == 0 && own == 0) a.score[row] = sc[i];
    }
  }
  if (!bwd) return;

  // logit_scale grad and loss: once per row tile (tower-0 block)
  if (own == 0) {
    // every lane of a 16-lane row group holds the same row values: count once
    float lp = (r == 0) ? loss_p : 0.f, dp = (r == 0) ? dls_p : 0.f;
    for (int o = 32; o > 0; o >>= 1) {
      lp += __shfl_xor(lp, o);
      dp += __shfl_xor(dp, o);
    }
    if (l == 0) {
      atomicAdd(smem + L::scal + 0, lp);
      atomicAdd(smem + L::scal + 1, dp);
    }
  }

  // own-tower output gradient in C layout
  f32x4 dO[NDT];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float dc = ds[i] * s;
#pragma unroll
    for (int j = 0; j < NDT; ++j) {
      const float so = accS[j][i], ot = accO[j][i];
      // d/d(own) of s*<own/|own|, oth/|oth|>  (SURVEY 3D closed form)
      dO[j][i] = valid[i] ? dc * (ot / nt[i] - so * cs[i] / no[i]) / no[i] : 0.f;
    }
  }

  const TowerDev& T = a.tw[own];
  float* A1s = smem + L::A1s;
  float* Z4s = smem + L::Z4s;
  float* dUs = smem + L::dUs;
  const float* cf = smem + L::cf1 + own * 4 * H1;

  // A1 of this wave's rows in C layout
  f32x4 a1[2], z4[2];
#pragma unroll
  for (int q = 0; q < 2; ++q)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a1[q][i] = A1s[(16 * w + 4 * g + i) * L::LDA + 16 * q + r];
      z4[q][i] = Z4s[(16 * w + 4 * g + i) * L::LDA + 16 * q + r];
    }

  // dW8 (rows-contracted from registers) and db8
#pragma unroll
  for (int j = 0; j < NDT; ++j) {
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      f32x4 acc = zero4();
      cl_gemm_tn(dO[j], a1[q], acc);
#pragma unroll
      for (int i = 0; i < 4; ++i) atomicAdd(smem + L::dW8 + (16 * j + 4 * g + i) * H1 + 16 * q + r, acc[i]);
    }
    const float cb = col_reduce(dO[j][0] + dO[j][1] + dO[j][2] + dO[j][3]);
    if (g == 0) atomicAdd(smem + L::db8 + 16 * j + r, cb);
    // dU strip, row-major, for dA1 = dU W8
#pragma unroll
    for (int i = 0; i < 4; ++i) dUs[(16 * w + 4 * g + i) * L::LDD + 16 * j + r] = dO[j][i];
  }
  __syncthreads();

  f32x4 dA[2] = {zero4(), zero4()};
  strip_gemm_nt<2>(dUs + 16 * w * L::LDD, L::LDD, smem + L::W8Ts, L::LDD, L::DP, dA);

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
      const int64_t row = r0 + 16 * w + 4 * g + i;
      const float dy = a1[q][i] > 0.f ? dA[q][i] * scl : 0.f;
      if (row < a.B) {
        T.dY1[row * H1 + col] = dy;
        sg[q] += dy * ((z4[q][i] - mean) * inv);
        sb[q] += dy;
      }
    }
  }
  cols_to_lds<2>(sg, smem + L::red);
  cols_to_lds<2>(sb, smem + L::red + H1);
  __syncthreads();

  if (threadIdx.x < H1) {
    atomicAdd(&T.gg1[threadIdx.x], smem[L::red + threadIdx.x]);
    atomicAdd(&T.gbe1[threadIdx.x], smem[L::red + H1 + threadIdx.x]);
  }
  if (own == 0 && threadIdx.x == 0) {
    atomicAdd(a.g_ls, smem[L::scal + 1]);
    if (a.mode == TOP_TRAIN && a.loss_sum) atomicAdd(a.loss_sum, smem[L::scal + 0] / (float)a.B);
  }
  float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
  const int D = a.D;
  for (int e = threadIdx.x; e < D * H1; e += THREADS) slab[T.so_W8 + e] = smem[L::dW8 + e];
  for (int e = threadIdx.x; e < D; e += THREADS) slab[T.so_b8 + e] = smem[L::db8 + e];
}

// ---------------------------------------------------------------------------
// k_bwd_mid : BN1 backward -> dZ4 ; dW4, db4 ; dA0 = dZ4 W4 ; dY0 ; dgamma0/dbeta0
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(THREADS) void k_bwd_mid(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int64_t step = step_current(a);
  const int64_t r0 = (int64_t)blockIdx.x * ROWS;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  constexpr int LD4 = H1 + 4;
  float* W4Ts = smem;                 // [64][36]  W4^T
  float* dZs = W4Ts + H0 * LD4;       // [ROWS][36]
  float* dW4 = dZs + ROWS * LD4;      // [32][64]
  float* db4 = dW4 + H1 * H0;         // [32]
  float* c1 = db4 + H1;               // k1[32] mb[32] mg[32] mean1[32] inv1[32]
  float* c0 = c1 + 5 * H1;            // mean0[64] alpha0[64] beta0[64] inv0[64]
  float* red = c0 + 4 * H0;           // [128]

  const float invB = 1.f / (float)a.B;
  if (threadIdx.x < H1) {
    const int c = threadIdx.x;
    const float inv = T.fin1[H1 + c];
    c1[c] = inv * T.g1[c];
    c1[H1 + c] = T.gbe1[c] * invB;
    c1[2 * H1 + c] = T.gg1[c] * invB;
    c1[3 * H1 + c] = T.fin1[c];
    c1[4 * H1 + c] = inv;
  }
  if (threadIdx.x < H0) {
    const int c = threadIdx.x;
    const float inv = T.fin0[H0 + c];
    c0[c] = T.fin0[c];
    c0[H0 + c] = inv * T.g0[c];
    c0[2 * H0 + c] = T.be0[c];
    c0[3 * H0 + c] = inv;
  }
  for (int e = threadIdx.x; e < H1 * H0 + H1; e += THREADS) dW4[e] = 0.f;
  if (threadIdx.x < 2 * H0) red[threadIdx.x] = 0.f;
  for (int e = threadIdx.x; e < H1 * H0; e += THREADS) {
    const int h1 = e / H0, h0 = e - h1 * H0;
    W4Ts[h0 * LD4 + h1] = T.W4[e];
  }
  __syncthreads();

  // dZ4 in C layout (2 tiles)
  f32x4 dz[2];
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    const int col = 16 * q + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      float v = 0.f;
      if (row < a.B) {
        const float dy = T.dY1[row * H1 + col];
        const float zh = (T.Z4[row * H1 + col] - c1[3 * H1 + col]) * c1[4 * H1 + col];
        v = c1[col] * (dy - c1[H1 + col] - zh * c1[2 * H1 + col]);
      }
      dz[q][i] = v;
      dZs[(16 * w + 4 * g + i) * LD4 + col] = v;
    }
  }
  // A0 (recomputed) in C layout (4 tiles), and the normalised Z0
  const bool drop = a.drop_thr > 0;
  const uint64_t key = dropout_key(a.seed, (uint64_t)step, t, 0);
  f32x4 a0[4], zh0[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      float av = 0.f, zh = 0.f;
      if (row < a.B) {
        const float z = T.Z0[row * H0 + col];
        av = bn_relu_drop(z, c0[col], c0[H0 + col], c0[2 * H0 + col], drop, key, (uint64_t)row * H0 + col,
                          a.drop_thr, a.drop_scale);
        zh = (z - c0[col]) * c0[3 * H0 + col];
      }
      a0[j][i] = av;
      zh0[j][i] = zh;
    }
  }
  // dW4 = dZ4^T A0 ; db4
#pragma unroll
  for (int q = 0; q < 2; ++q) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 acc = zero4();
      cl_gemm_tn(dz[q], a0[j], acc);
#pragma unroll
      for (int i = 0; i < 4; ++i) atomicAdd(dW4 + (16 * q + 4 * g + i) * H0 + 16 * j + r, acc[i]);
    }
    const float cb = col_reduce(dz[q][0] + dz[q][1] + dz[q][2] + dz[q][3]);
    if (g == 0) atomicAdd(db4 + 16 * q + r, cb);
  }
  __syncthreads();

  // dA0 = dZ4 W4  (K = 32)
  f32x4 dA[4] = {zero4(), zero4(), zero4(), zero4()};
  strip_gemm_nt<4>(dZs + 16 * w * LD4, LD4, W4Ts, LD4, H1, dA);
  const float scl = drop ? a.drop_scale : 1.f;
  float sg[4], sb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
    sg[j] = 0.f;
    sb[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      const float dy = a0[j][i] > 0.f ? dA[j][i] * scl : 0.f;
      if (row < a.B) {
        T.dY0[row * H0 + col] = dy;
        sg[j] += dy * zh0[j][i];
        sb[j] += dy;
      }
    }
  }
  cols_to_lds<4>(sg, red);
  cols_to_lds<4>(sb, red + H0);
  __syncthreads();
  if (threadIdx.x < H0) {
    atomicAdd(&T.gg0[threadIdx.x], red[threadIdx.x]);
    atomicAdd(&T.gbe0[threadIdx.x], red[H0 + threadIdx.x]);
  }
  float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
  for (int e = threadIdx.x; e < H1 * H0; e += THREADS) slab[T.so_W4 + e] = dW4[e];
  if (threadIdx.x < H1) slab[T.so_b4 + threadIdx.x] = db4[threadIdx.x];
}

// ---------------------------------------------------------------------------
// k_bwd_first : BN0 backward -> dZ0 ; dW0 = dZ0^T X ; db0 ; dX -> embedding grads
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(THREADS) void k_bwd_first(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int64_t step = step_current(a);
  const int64_t base = batch_row0(a, step);
  const int64_t r0 = (int64_t)blockIdx.x * ROWS;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  const int kp = T.kp;
  constexpr int LD0 = H0 + 4;
  float* dW0 = smem;                 // [64][kp]
  float* db0 = dW0 + H0 * kp;        // [64]
  float* c0 = db0 + H0;              // k0[64] mb[64] mg[64] mean0[64] inv0[64]
  float* dZs = c0 + 5 * H0;          // [ROWS][68]   (only with embeddings)
  float* W0Ts = dZs + ROWS * LD0;    // [kp][68]     (only with embeddings)

  const float invB = 1.f / (float)a.B;
  if (threadIdx.x < H0) {
    const int c = threadIdx.x;
    const float inv = T.fin0[H0 + c];
    c0[c] = inv * T.g0[c];
    c0[H0 + c] = T.gbe0[c] * invB;
    c0[2 * H0 + c] = T.gg0[c] * invB;
    c0[3 * H0 + c] = T.fin0[c];
    c0[4 * H0 + c] = inv;
  }
  for (int e = threadIdx.x; e < H0 * kp + H0; e += THREADS) dW0[e] = 0.f;
  const bool emb = T.n_cat > 0;
  if (emb) {
    for (int e = threadIdx.x; e < H0 * kp; e += THREADS) {
      const int n = e / kp, k = e - n * kp;
      W0Ts[k * LD0 + n] = k < T.in_dim ? T.W0[n * T.in_dim + k] : 0.f;
    }
  }
  __syncthreads();

  f32x4 dz[4];
  int64_t drow[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t row = r0 + 16 * w + 4 * g + i;
    drow[i] = row < a.B ? data_row(a, base, row) : -1;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      float v = 0.f;
      if (row < a.B) {
        const float dy = T.dY0[row * H0 + col];
        const float zh = (T.Z0[row * H0 + col] - c0[3 * H0 + col]) * c0[4 * H0 + col];
        v = c0[col] * (dy - c0[H0 + col] - zh * c0[2 * H0 + col]);
      }
      dz[j][i] = v;
      if (emb) dZs[(16 * w + 4 * g + i) * LD0 + col] = v;
    }
    const float cb = col_reduce(dz[j][0] + dz[j][1] + dz[j][2] + dz[j][3]);
    if (g == 0) atomicAdd(db0 + col, cb);
  }
  // dW0 = dZ0^T X, one 16-column tile of X at a time (X in C layout)
  for (int kt = 0; kt < kp / 16; ++kt) {
    f32x4 x;
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = drow[i] >= 0 ? tower_x(T, drow[i], 16 * kt + r) : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 acc = zero4();
      cl_gemm_tn(dz[j], x, acc);
#pragma unroll
      for (int i = 0; i < 4; ++i) atomicAdd(dW0 + (16 * j + 4 * g + i) * kp + 16 * kt + r, acc[i]);
    }
  }
  if (emb) {
    __syncthreads();
    // dX = dZ0 W0 on the embedding columns -> scatter-add into the tables
    const int kt0 = T.n_num / 16;
    for (int kt = kt0; kt < kp / 16; ++kt) {
      f32x4 dx[1] = {zero4()};
      strip_gemm_nt<1>(dZs + 16 * w * LD0, LD0, W0Ts + 16 * kt * LD0, LD0, H0, dx);
      const int col = 16 * kt + r;
      if (col >= T.n_num && col < T.in_dim) {
        const int c = col - T.n_num;
        const int jj = c / T.emb_dim, e = c - jj * T.emb_dim;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (drow[i] < 0) continue;
          int64_t code = T.cat[drow[i] * T.cat_ld + jj];
          code = code < 0 ? 0 : (code >= T.emb_rows[jj] ? T.emb_rows[jj] - 1 : code);
          atomicAdd(T.gemb[jj] + code * T.emb_dim + e, dx[0][i]);
        }
      }
    }
  }
  __syncthreads();
  float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
  const int in = T.in_dim;
  for (int e = threadIdx.x; e < H0 * in; e += THREADS) {
    const int n = e / in, k = e - n * in;
    slab[T.so_W0 + e] = dW0[n * kp + k];
  }
  if (threadIdx.x < H0) slab[T.so_b0 + threadIdx.x] = db0[threadIdx.x];
}

template __global__ void k_top<4>(StepArgs);
template __global__ void k_top<8>(StepArgs);

// LDS bytes per kernel (used by the launcher)
size_t lds_l0_fwd(int kp) { return sizeof(float) * ((size_t)(H0 + ROWS) * (kp + 4) + 3 * H0); }
size_t lds_l4_fwd() { return sizeof(float) * ((size_t)(H1 + ROWS) * (H0 + 4) + 3 * H0 + 2 * H1 + H0 + H1); }
size_t lds_top(int ndt) {
  return sizeof(float) * (size_t)(ndt == 4 ? TopLds<4>::total : TopLds<8>::total);
}
size_t lds_bwd_mid() {
  return sizeof(float) * ((size_t)(H0 + ROWS) * (H1 + 4) + H1 * H0 + H1 + 5 * H1 + 4 * H0 + 2 * H0);
}
size_t lds_bwd_first(int kp, bool emb) {
  size_t n = (size_t)H0 * kp + H0 + 5 * H0;
  if (emb) n += (size_t)(ROWS + kp) * (H0 + 4);
  return sizeof(float) * n;
}

}  // namespace tt
