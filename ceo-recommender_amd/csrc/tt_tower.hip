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
//   k_l0_fwd    Z0 = X W0^T + b0 (X gathered per lane: numeric ++ embeddings), BN0 sums
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
#include "tt_reduce.h"

namespace tt {

// ---------------------------------------------------------------------------
// shared pieces
// ---------------------------------------------------------------------------

// BN coefficients of column c (train: shifted moment sums of this batch;
// eval: running stats).  `update`: fold the batch stats into the running
// estimates (momentum, unbiased variance, torch semantics) and publish
// mean|invstd for the backward kernels.
// (bn_coefs_pre: the same on shift[c], rm[c], rv[c] loaded by the caller)
__device__ __forceinline__ void bn_coefs_pre(const StepArgs& a, int H, const float* st, float shift_c, float rm_c,
                                             float rv_c, float* rm, float* rv, int64_t* nbt, float* fin,
                                             bool update, int c, float* mean_out, float* inv_out) {
  float mean, var;
  if (a.train) {
    const double Bd = (double)a.B;
    const float m1 = st[c] / (float)Bd;  // st: replica-summed S1|S2 (LDS)
    var = st[H + c] / (float)Bd - m1 * m1;
    var = var < 0.f ? 0.f : var;
    mean = shift_c + m1;
    if (update) {
      const float mom = a.momentum;
      rm[c] = (1.f - mom) * rm_c + mom * mean;
      rv[c] = (1.f - mom) * rv_c + mom * (var * (float)(Bd / (Bd - 1.0)));
      fin[c] = mean;
      fin[H + c] = 1.f / sqrtf(var + a.eps);
      if (c == 0) *nbt += 1;
    }
  } else {
    mean = rm_c;
    var = rv_c;
    // eval: publish the running-stat coefficients the eval-mode backward
    // recomputes the activations with (block 0; every writer stores the same)
    if (blockIdx.x == 0 && fin) {
      fin[c] = mean;
      fin[H + c] = 1.f / sqrtf(var + a.eps);
    }
  }
  *mean_out = mean;
  *inv_out = 1.f / sqrtf(var + a.eps);
}
__device__ __forceinline__ void bn_coefs(const StepArgs& a, int H, const float* st, const float* shift,
                                         float* rm, float* rv, int64_t* nbt, float* fin, bool update,
                                         int c, float* mean_out, float* inv_out) {
  bn_coefs_pre(a, H, st, shift[c], rm[c], rv[c], rm, rv, nbt, fin, update, c, mean_out, inv_out);
}

// BN apply + ReLU + (train) dropout of one element.
__device__ __forceinline__ float bn_relu_drop(float z, float mean, float alpha, float beta, bool drop,
                                              uint32_t rk, int col, uint32_t thr, float scale) {
  float y = (z - mean) * alpha + beta;
  y = y > 0.f ? y : 0.f;
  if (drop) y = dropout_keep_rk<DROP_HB0>(rk, col, thr) ? y * scale : 0.f;
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

// rep_sum split in two (issue / finish) so the replica loads can be issued
// ahead of a kernel's tile loads: vmcnt retires in issue order, so the sum
// (and the BN-coefficient chain behind it) then waits for the replicas only,
// not for every tile load issued before them.
template <int NTH, int N>
struct RepSum1 {
  static constexpr int G0 = NTH / N;
  static constexpr int G = G0 < NREP ? G0 : NREP;
  static constexpr int PER = NREP / G;
  static_assert(NTH % N == 0 && NREP % G == 0, "replica groups");
  float v[PER];
  __device__ __forceinline__ void issue(const float* rep, int stride) {
    // groups beyond G re-read group G - 1 (ignored by finish): no branch join
    const int c = (int)threadIdx.x % N, grp = min((int)threadIdx.x / N, G - 1);
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = rep[(grp + k * G) * stride + c];
  }
  __device__ __forceinline__ void finish(float* scratch, float* dst) {
    const int c = (int)threadIdx.x % N, grp = (int)threadIdx.x / N;
    if (grp < G) {
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
};

// rep_sum of two equally shaped replica sets at once (one load round trip),
// split in two so the caller can work while the loads are in flight:
//   RepSum2<NTH, N> rs; rs.issue(rep0, rep1, stride);  ...  rs.finish(scratch, dst);
// dst[0..N) from rep0, dst[N..2N) from rep1 (LDS, visible to the block after
// finish).  scratch: NTH floats of LDS.
template <int NTH, int N>
struct RepSum2 {
  static constexpr int N2 = 2 * N;
  static constexpr int G0 = NTH / N2;
  static constexpr int G = G0 < NREP ? G0 : NREP;
  static constexpr int PER = NREP / G;
  static_assert(NTH % N2 == 0 && NREP % G == 0, "replica groups");
  float v[PER];
  __device__ __forceinline__ void issue(const float* rep0, const float* rep1, int stride) {
    // every thread loads (groups beyond G re-read group G - 1, ignored by
    // finish): no branch join that would make hipcc wait for the loads here
    const int c2 = (int)threadIdx.x % N2, grp = min((int)threadIdx.x / N2, G - 1);
    const float* rep = c2 < N ? rep0 : rep1;
    const int c = c2 < N ? c2 : c2 - N;
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = rep[(grp + k * G) * stride + c];
  }
  __device__ __forceinline__ void finish(float* scratch, float* dst) {
    const int c2 = (int)threadIdx.x % N2, grp = (int)threadIdx.x / N2;
    if (grp < G) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < PER; ++k) sum += v[k];
      scratch[grp * N2 + c2] = sum;
    }
    __syncthreads();
    if (threadIdx.x < N2) {
      float sum = 0.f;
#pragma unroll
      for (int q = 0; q < G; ++q) sum += scratch[q * N2 + threadIdx.x];
      dst[threadIdx.x] = sum;
    }
    __syncthreads();
  }
};

// Block-wide column sums of NT C-layout tiles: wave w stores its column
// totals into its own LDS row red[w * ld + ...] (no LDS atomics, whose
// arrival order would decide the rounding); wave_rows_sum adds the rows in
// wave order, so a block's sum is bitwise repeatable.
template <int NT>
__device__ __forceinline__ void cols_to_lds(const float (&s)[NT], float* red, int ld) {
  const int l = lane_id(), r = l & 15, g = l >> 4, w = wave_id();
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const float v = col_reduce(s[j]);
    if (g == 0) red[w * ld + 16 * j + r] = v;
  }
}
template <int NW>
__device__ __forceinline__ float wave_rows_sum(const float* red, int ld, int c) {
  float v = red[c];
#pragma unroll
  for (int w = 1; w < NW; ++w) v += red[w * ld + c];
  return v;
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
// X W0^T on the bf16x3 MFMA core: each lane gathers the 8-column slices of
// its own row that it supplies as the A operand (no X tile in LDS, no
// gather -> LDS -> barrier chain); W0 is staged once per block as bf16 planes.
// Instances: KS = 32-wide K steps (tower inputs up to 32 KS columns, zero
// padded), VEC = numeric-only towers with 16-B aligned rows.  The issue phase
// is straight-line code -- every load unconditional at a clamped address,
// out-of-range values zeroed by selects afterwards -- because a branch around
// a load makes the compiler drain vmcnt at the join, which serialises the
// gathers behind one another.
constexpr int l0_ks(int kp) { return kp <= 32 ? 1 : kp <= 64 ? 2 : kp <= 128 ? 4 : 8; }
template <int R>
struct L0Lds {
  __host__ __device__ static constexpr int ldk(int ks) { return 32 * ks + 16; }  // 32-B pad: conflict-free reads
  // bf16 planes [3][H0][ldk] | red [4 waves][2*H0] | shl [H0]
  static size_t bytes(int kp) {
    return sizeof(uint16_t) * 3 * (size_t)H0 * ldk(l0_ks(kp)) + sizeof(float) * 9 * H0;
  }
};

// 8 consecutive tower-input columns c0..c0+7 of dataset row drow, raw
// (VEC: two float4 at clamped addresses; zero_x8 masks columns >= n_num)
template <bool VEC>
__device__ __forceinline__ void tower_x8(const TowerDev& T, int64_t drow, int c0, float (&x)[8]) {
  if constexpr (VEC) {
    const float* src = T.num + drow * T.num_ld;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const float4 v = *reinterpret_cast<const float4*>(src + min(c0 + 4 * h, T.n_num - 4));
      x[4 * h + 0] = v.x;
      x[4 * h + 1] = v.y;
      x[4 * h + 2] = v.z;
      x[4 * h + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = tower_x(T, drow, c0 + e);
  }
}
template <bool VEC>
__device__ __forceinline__ void zero_x8(const TowerDev& T, int c0, float (&x)[8]) {
  if constexpr (VEC) {
#pragma unroll
    for (int e = 0; e < 8; ++e) x[e] = c0 + e < T.n_num ? x[e] : 0.f;
  }
}

// LATE: blocks x >= a.l0_gx run the previous step's deferred late half of
// the gradient reduction (TT_FLAG_DEFER_LATE: W4, BN1 affine, W8, b8,
// logit_scale and the loss fold) beside the row tiles -- none of which reads
// or writes what this kernel does.
template <int R, int KS, bool VEC, bool LATE>
__global__ __launch_bounds__(R * 4) TT_WPE(TT_WPE_L0) void k_l0_fwd(StepArgs a, LateRed late) {
  constexpr int NTH = R * 4;
  constexpr int KC = 32 * KS, LDK = L0Lds<R>::ldk(KS), PL = H0 * LDK;
  constexpr int C4N = KC / 4, N4 = H0 * C4N, WPT = N4 / NTH;  // W0 float4 per thread
  constexpr int NW = R / 16, SPW = 4 / NW;  // waves; shift-row tiles per wave
  static_assert((R == 64 || (R == 32 && !LATE)) && N4 % NTH == 0, "4 (or 2) waves x 16 rows");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  if constexpr (LATE) {
    static_assert(LATE_G * RED_E == NTH, "a late-half block is one k_l0_fwd block");
    if ((int)blockIdx.x >= a.l0_gx) {
      const int bid = ((int)blockIdx.x - a.l0_gx) * 2 + (int)blockIdx.y;
      reduce_body<LateRed, LATE_G, true, false, true>(late, bid, smem, smem + LATE_G * RED_E,
                                                      reinterpret_cast<int*>(smem + 5 * LATE_G * RED_E));
      return;
    }
  }
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int64_t step = step_for_first_kernel(a);
  const int64_t base = batch_row0(a, step);
  const int64_t r0 = (int64_t)(R == 64 ? tile64(a) : (int)blockIdx.x) * R;
  const int in = T.in_dim;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  uint16_t* Wh = reinterpret_cast<uint16_t*>(smem);
  float* red = reinterpret_cast<float*>(Wh + 3 * PL);  // [NW waves][128]
  float* shl = red + 4 * 2 * H0;                       // [64] moment shift = Z0 of batch row 0
  TT_STAMP(0, 0);

  // ---- issue (straight line): row indices; W0 (raw, clamped); this lane's
  // X slices (A operand: row 16w + r, columns 32kk + 8g .. +7; rows beyond B
  // gather a duplicate row) and the same slices of the batch's row 0
  const int64_t dr = data_row_nb(a, base, min(r0 + 16 * w + r, a.B - 1));
  const int64_t dr0 = data_row_nb(a, base, 0);
  float4 wv[WPT];
#pragma unroll
  for (int k = 0; k < WPT; ++k) {
    const int e = k * NTH + (int)threadIdx.x;
    const int h = e / C4N, c = 4 * (e - h * C4N);
    const float* rw = T.W0 + (int64_t)h * in;
    if constexpr (VEC)
      wv[k] = *reinterpret_cast<const float4*>(rw + min(c, in - 4));
    else
      wv[k] = make_float4(rw[min(c, in - 1)], rw[min(c + 1, in - 1)], rw[min(c + 2, in - 1)], rw[min(c + 3, in - 1)]);
  }
  float xr[KS][8], x0[KS][8];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    tower_x8<VEC>(T, dr, 32 * kk + 8 * g, xr[kk]);
    tower_x8<VEC>(T, dr0, 32 * kk + 8 * g, x0[kk]);
  }
  float bias[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) bias[j] = T.b0[16 * j + r];
  float bsh[SPW];  // the shift row's tiles of this wave: w, w + NW, ...
#pragma unroll
  for (int i = 0; i < SPW; ++i) bsh[i] = T.b0[16 * (w + NW * i) + r];
  // (target, weight) of this lane's row for the top kernel (tower-0 blocks
  // store them at the end): issued last, from the row index the lane already
  // holds, unconditionally (valid dummy address without a target) -- no
  // index load and no load chain at the end of the kernel (was 1.1-1.3 us)
  // (tower-1 blocks read one shared line instead: the random gather is
  // tower 0's alone)
  const bool tgw_on = a.target != nullptr;
  const int64_t tgr = tgw_on && t == 0 ? dr : 0;
  const float tg_v = (tgw_on ? a.target : T.b0)[tgr];
  const float wt_v = (tgw_on ? a.weight : T.b0)[tgr];
  // W0 image: zero columns >= in, split, store
#pragma unroll
  for (int k = 0; k < WPT; ++k) {
    const int e = k * NTH + (int)threadIdx.x;
    const int h = e / C4N, c = 4 * (e - h * C4N);
    const float4 u = make_float4(c + 0 < in ? wv[k].x : 0.f, c + 1 < in ? wv[k].y : 0.f, c + 2 < in ? wv[k].z : 0.f,
                                 c + 3 < in ? wv[k].w : 0.f);
    put_planes4(Wh + h * LDK + c, PL, u);
  }
  __syncthreads();
  TT_STAMP(0, 1);

  // ---- Z0 = X W0^T (+ b0): lane (r, g) of wave w gets rows 16w + 4g + i,
  // column 16j + r.  Shift row: wave w computes Z0[row 0] columns 16w..16w+15
  // with the same MFMA sequence in every block (bitwise one shift for all),
  // which keeps var = S2/B - (S1/B)^2 free of cancellation for any data offset.
  f32x4 acc[4], accs[SPW];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = zero4();
#pragma unroll
  for (int i = 0; i < SPW; ++i) accs[i] = zero4();
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    zero_x8<VEC>(T, 32 * kk + 8 * g, xr[kk]);
    zero_x8<VEC>(T, 32 * kk + 8 * g, x0[kk]);
    bf16x8 xa[3], xs[3];
    split8x3(xr[kk], xa);
    split8x3(x0[kk], xs);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x8 wf[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        wf[p] = *reinterpret_cast<const bf16x8*>(Wh + p * PL + (16 * j + r) * LDK + 32 * kk + 8 * g);
      mfma_x3(xa, wf, acc[j]);
    }
    // the shift row's tiles w, w + NW, ...: their own fragment reads (no
    // per-tile branch between the MFMA chains), the same six-product sequence
    // in every block
#pragma unroll
    for (int i = 0; i < SPW; ++i) {
      bf16x8 ws[3];
#pragma unroll
      for (int p = 0; p < 3; ++p)
        ws[p] = *reinterpret_cast<const bf16x8*>(Wh + p * PL + (16 * (w + NW * i) + r) * LDK + 32 * kk + 8 * g);
      mfma_x3(xs, ws, accs[i]);
    }
  }
  if (a.train) {
    if (g == 0) {
#pragma unroll
      for (int i = 0; i < SPW; ++i) {
        const float sh = accs[i][0] + bsh[i];
        shl[16 * (w + NW * i) + r] = sh;
        if (blockIdx.x == 0) T.shift0[16 * (w + NW * i) + r] = sh;
      }
    }
    __syncthreads();  // shl
  }
  TT_STAMP(0, 2);

  float s1[4], s2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
    const float sh = a.train ? shl[col] : 0.f;
    s1[j] = 0.f;
    s2[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t rw = r0 + 16 * w + 4 * g + i;
      const float z = acc[j][i] + bias[j];
      acc[j][i] = z;
      const float d = rw < a.B ? z - sh : 0.f;
      s1[j] += d;
      s2[j] += d * d;
    }
  }
  if (a.train) {
    cols_to_lds<4>(s1, red, 2 * H0);
    cols_to_lds<4>(s2, red + H0, 2 * H0);
  }
  // Z0 (workspace rows are padded to whole tiles: no guard), row-major via
  // quad transposes, 16-B write-through stores
#pragma unroll
  for (int j = 0; j < 4; ++j) store_tile_rm_wt<TT_HANDOFF_AUX>(T.Z0 + r0 * H0, 16 * w * H0 + 16 * j, H0, acc[j]);
  if (t == 0 && tgw_on && g == 0)  // rows r0 + 16 w + r: the whole tile (tgw is padded to whole tiles)
    *reinterpret_cast<float2*>(a.tgw + 2 * (r0 + 16 * w + r)) = make_float2(tg_v, wt_v);
  if (a.state && blockIdx.x == 0 && t == 0 && threadIdx.x == 0) a.state->step_cur = step;
  // Adam's coefficients for this step: normally cached by the previous
  // step's k_reduce_adam (AdamSlot); recomputed here when the slot does not
  // match (first step, counter or hyperparameters changed by the host)
  if (a.adam_slots && blockIdx.x == 0 && t == 0 && threadIdx.x == 64) {
    AdamSlot& sl = a.adam_slots[step & 1];
    if (!adam_slot_ok(sl, step, a.adam_lr, a.adam_b1, a.adam_b2, a.adam_eps))
      adam_slot_fill(sl, step, a.adam_lr, a.adam_b1, a.adam_b2, a.adam_eps);
  }
  if (a.train) {
    __syncthreads();
    if (threadIdx.x < 2 * H0)
      xblock_add(a.det, T.st0, ST0S, T.dslot, 2 * H0, threadIdx.x, wave_rows_sum<NW>(red, 2 * H0, threadIdx.x));
  }
  // the folded BN0 backward's replicas start every step at zero (k_bwd_mid
  // accumulates them, k_reduce_adam only reads them)
  if (a.fr_zero) {  // (the row-tile blocks only: with LATE l0_gx, not gridDim.x)
    const int gx = LATE ? a.l0_gx : (int)gridDim.x;
    const int nthr = gx * (int)gridDim.y * NTH;
    for (int i = (int)((blockIdx.y * gx + blockIdx.x) * NTH + threadIdx.x); i < a.fr_zero_len; i += nthr)
      a.fr_zero[i] = 0.f;
  }
  TT_STAMP(0, 3);
}

// ---------------------------------------------------------------------------
// k_l4_fwd : A0 = Drop(ReLU(BN0(Z0))) ; Z4 = A0 W4^T + b4 ; BN1 sums
//
// Z4 = A0 W4^T on the bf16x3 MFMA core with the A operand straight from
// registers: lane (r, g) of wave w loads the Z0 slices it supplies as the A
// operand of v_mfma_f32_16x16x32_bf16 -- row 16w + r, columns 8g .. 8g + 7
// (K step 0) and 32 + 8g .. (K step 1) -- applies BN0 / ReLU / dropout and
// splits them into planes in place: no A0 tile in LDS, no barrier between the
// activation and the GEMM.  The dropout pair of layer 0 is (c, c + 32)
// (DROP_HB0 = 5): both halves of every permutation are this lane's.  W4 is
// staged once per block as bf16 planes (the B operand, l0's padded layout).
// ---------------------------------------------------------------------------
template <int R>
struct L4Lds {
  static constexpr int LDK = H0 + 16;  // bf16 row stride of the W4 image (32-B pad: conflict-free reads)
  static constexpr int PL = H1 * LDK;  // one W4 plane
  // W4 planes [3][32][LDK] (bf16) | cf [3][64] | red [4][64] | a0r [64] | shl [32] | rsc [NTH] | rst [128]
  static constexpr int f_cf = 3 * PL / 2;
  static constexpr int f_red = f_cf + 3 * H0;
  static constexpr int f_a0r = f_red + 8 * H1;
  static constexpr int f_shl = f_a0r + H0;
  static constexpr int f_rsc = f_shl + H1;
  static constexpr int f_rst = f_rsc + 4 * R;
  static constexpr size_t bytes = sizeof(float) * ((size_t)f_rst + 2 * H0);
  static_assert(PL % 8 == 0, "16-B aligned planes");
};

template <int R>
__global__ __launch_bounds__(R * 4) TT_WPE(TT_WPE_L4) void k_l4_fwd(StepArgs a) {
  using L = L4Lds<R>;
  constexpr int NTH = R * 4, LDK = L::LDK, PL = L::PL, NW = R / 16;
  static_assert((R == 64 || R == 32) && H0 == 64 && H1 == 32, "4 (or 2) waves x 16 rows, two 32-deep K steps");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int64_t step = step_current(a);
  const int64_t r0 = (int64_t)(R == 64 ? tile64(a) : (int)blockIdx.x) * R;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  uint16_t* Wh = reinterpret_cast<uint16_t*>(smem);  // W4 planes
  float* cf = smem + L::f_cf;                        // mean[64] alpha[64] beta[64]
  float* red = smem + L::f_red;                      // [4 waves][64]
  float* a0r = smem + L::f_a0r;                      // [64] A0 of batch row 0
  float* shl = smem + L::f_shl;                      // [32] moment shift = Z4 of batch row 0
  float* rsc = smem + L::f_rsc;                      // [NTH] replica-sum scratch
  float* rst = smem + L::f_rst;                      // [2*64] BN0 moment sums S1|S2
  TT_STAMP(1, 0);
#ifdef TT_DIAG_KARG  // diagnostic stamps build: slot 1 = when the kernel arguments have arrived
  asm volatile("; karg %0 %1" ::"s"(a.tw[0].st0), "s"(a.state));
  TT_STAMP(1, 1);
#endif

  // ---- issue every load of the phase first (Z0 rows are padded: no clamp):
  // the BN0 moment replicas first (their sum and the coefficient chain wait
  // for them alone), then this lane's A-operand slices of Z0: row 16w + r,
  // columns 8g.. and 32 + 8g..
  RepSum1<NTH, 2 * H0> rs;
#ifdef TT_DIAG_REP
  rs.issue(T.Z0 + (int64_t)(a.B / 2) * H0, 2 * H0);  // diagnostic (wrong values): plain-stored lines instead of the atomically built replicas
#else
  rs.issue(T.st0, ST0S);
#endif
  float bias[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) bias[j] = T.b4[16 * j + r];
  const float z0r_raw = T.Z0[min((int)threadIdx.x, H0 - 1)];
  const float z0r = threadIdx.x < H0 ? z0r_raw : 0.f;
  // W4 (raw) and wave 0's BN0 parameters are issued with the Z0 loads: one
  // round trip for the whole phase
  constexpr int W4T = H1 * H0 / 4 / NTH;  // W4 float4 per thread (2, or 4 at 32 rows); BN0: wave 0
  static_assert(H1 * H0 / 4 == W4T * NTH, "whole W4 float4 rounds");
  float4 w4v[W4T];
#pragma unroll
  for (int k = 0; k < W4T; ++k) {
    const int we = (int)threadIdx.x + k * NTH;
    w4v[k] = *reinterpret_cast<const float4*>(T.W4 + (we >> 4) * H0 + 4 * (we & 15));
  }
  // (every wave loads them -- wave 0 uses them: a load under a branch would
  // make hipcc drain vmcnt at the join, i.e. wait for the whole phase here)
  const float* rmp = T.rm0 ? T.rm0 : T.g0;  // running stats NULL without buffers (never read then)
  const float* rvp = T.rv0 ? T.rv0 : T.g0;
  const float bn_sh = T.shift0[l], bn_rm = rmp[l], bn_rv = rvp[l], bn_g = T.g0[l], bn_be = T.be0[l];
  // the Z0 tile last: needed only after the phase's barrier
  const float* zr = T.Z0 + (r0 + 16 * w + r) * H0 + 8 * g;
  const float4 za0 = *reinterpret_cast<const float4*>(zr), za1 = *reinterpret_cast<const float4*>(zr + 4);
  const float4 zb0 = *reinterpret_cast<const float4*>(zr + 32), zb1 = *reinterpret_cast<const float4*>(zr + 36);
  const bool drop = a.train && a.drop_thr > 0;
  const uint64_t key = dropout_key(a.seed, (uint64_t)step, t, 0);
#ifndef TT_DIAG_KARG
  TT_STAMP(1, 1);
#endif
  if (a.train) rs.finish(rsc, rst);
  TT_STAMP(1, 2);
  if (threadIdx.x < H0) {
    const int c = threadIdx.x;
    float mean, inv;
    bn_coefs_pre(a, H0, rst, bn_sh, bn_rm, bn_rv, T.rm0, T.rv0, T.nbt0, T.fin0, a.update_stats && blockIdx.x == 0,
                 c, &mean, &inv);
    const float alpha = inv * bn_g;
    cf[c] = mean;
    cf[H0 + c] = alpha;
    cf[2 * H0 + c] = bn_be;
    // A0 of the batch's row 0 (the BN1 moment shift's input), bitwise as the
    // tile rows compute it
    if (a.train)
      a0r[c] = bn_relu_drop(z0r, mean, alpha, bn_be, drop, dropout_row_key(key, 0), c, a.drop_thr, a.drop_scale);
  }
  TT_STAMP(1, 3);
#pragma unroll
  for (int k = 0; k < W4T; ++k) {
    const int we = (int)threadIdx.x + k * NTH;
    put_planes4(Wh + (we >> 4) * LDK + 4 * (we & 15), PL, w4v[k]);
  }
  __syncthreads();
  TT_STAMP(1, 4);

  // ---- A0 of this lane's 16 elements (columns c = 8g + e and c + 32), split
  // into the two K steps' A operands
  bf16x8 xa[2][3];
  {
    const f32x4* cv = reinterpret_cast<const f32x4*>(cf + 8 * g);
    const f32x4 mu[4] = {cv[0], cv[1], cv[8], cv[9]};
    const f32x4 al[4] = {cv[H0 / 4], cv[H0 / 4 + 1], cv[H0 / 4 + 8], cv[H0 / 4 + 9]};
    const f32x4 be[4] = {cv[H0 / 2], cv[H0 / 2 + 1], cv[H0 / 2 + 8], cv[H0 / 2 + 9]};
    const float zz[16] = {za0.x, za0.y, za0.z, za0.w, za1.x, za1.y, za1.z, za1.w,
                          zb0.x, zb0.y, zb0.z, zb0.w, zb1.x, zb1.y, zb1.z, zb1.w};
    float y[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const float v = (zz[e] - mu[e >> 2][e & 3]) * al[e >> 2][e & 3] + be[e >> 2][e & 3];
      y[e] = v > 0.f ? v : 0.f;
    }
    if (drop) {  // pair (c, c + 32): low half of the permutation for c, high for c + 32
      const uint32_t rk = dropout_row_key(key, r0 + 16 * w + r);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const uint32_t h = perm32(rk ^ ((uint32_t)(8 * g + e) * 0x9E3779B9u));
        y[e] = (h & 0xFFFFu) >= a.drop_thr ? y[e] * a.drop_scale : 0.f;
        y[8 + e] = (h >> 16) >= a.drop_thr ? y[8 + e] * a.drop_scale : 0.f;
      }
    }
    float x0[8], x1[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      x0[e] = y[e];
      x1[e] = y[8 + e];
    }
    split8x3(x0, xa[0]);
    split8x3(x1, xa[1]);
  }
  TT_STAMP(1, 5);

  // ---- Z4 = A0 W4^T (bf16x3, two K steps per 16-column tile); waves 0 and 1
  // also compute tile w of the shift row with the same MFMA sequence in every
  // block (bitwise one shift for all blocks)
  f32x4 acc[2] = {zero4(), zero4()}, accs = zero4();
  {
    bf16x8 sa[2][3];
    if (a.train && w < 2) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const f32x4* ap = reinterpret_cast<const f32x4*>(a0r + 32 * kk + 8 * g);
        const f32x4 p0 = ap[0], p1 = ap[1];
        const float xs[8] = {p0[0], p0[1], p0[2], p0[3], p1[0], p1[1], p1[2], p1[3]};
        split8x3(xs, sa[kk]);
      }
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bf16x8 wf[3];
#pragma unroll
        for (int p = 0; p < 3; ++p)
          wf[p] = *reinterpret_cast<const bf16x8*>(Wh + p * PL + (16 * j + r) * LDK + 32 * kk + 8 * g);
        mfma_x3(xa[kk], wf, acc[j]);
      }
    }
    if (a.train && w < 2) {  // the shift row's tile w (one uniform branch, not one per tile)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 ws[3];
#pragma unroll
        for (int p = 0; p < 3; ++p)
          ws[p] = *reinterpret_cast<const bf16x8*>(Wh + p * PL + (16 * w + r) * LDK + 32 * kk + 8 * g);
        mfma_x3(sa[kk], ws, accs);
      }
    }
  }
  if (a.train) {
    if (w < 2 && g == 0) {
      const float sh = accs[0] + bias[w];
      shl[16 * w + r] = sh;
      if (blockIdx.x == 0) T.shift1[16 * w + r] = sh;
    }
    __syncthreads();  // shl
  }
  TT_STAMP(1, 6);

  float s1[2], s2[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float sh = a.train ? shl[16 * j + r] : 0.f;
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
    cols_to_lds<2>(s1, red, 2 * H1);
    cols_to_lds<2>(s2, red + H1, 2 * H1);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) store_tile_rm_wt<TT_HANDOFF_AUX>(T.Z4 + r0 * H1, 16 * w * H1 + 16 * j, H1, acc[j]);
  if (a.train) {
    __syncthreads();
    if (threadIdx.x < 2 * H1)
      xblock_add(a.det, T.st1, ST1S, T.dslot, 2 * H1, threadIdx.x, wave_rows_sum<NW>(red, 2 * H1, threadIdx.x));
  }
  TT_STAMP(1, 7);
}

// ---------------------------------------------------------------------------
// k_top : both towers' last layer, cosine score, loss, own-tower backward.
// Grid (tiles, 2): block (x, y) owns rows [x R, x R + R) and the backward of
// tower y; both towers' forward is needed by both blocks of a tile.
//
// All four products run on the bf16x3 MFMA core (fp32-accurate, tt_common.h):
//   forward   U^T[d][row]  = sum_h W8[d][h] A1[row][h]
//             (A = W8 image rows, B = this lane's A1 slice straight from Z4)
//   dA1^T[h][row]          = sum_d W8[d][h] dU[row][d]
//             (A = W8 image via transposed reads, B = dU in the forward's
//              accumulator layout -- no LDS round trip)
//   dW8^T[h][d]            = sum_rows A1[row][h] dU[row][d]
//   db8[d]                 = sum_rows dU[row][d]      (ones x dU, same loop)
//             (A1 and dU images read transposed, rows = K)
// The forward is computed transposed so that each row sits on one lane (its 4
// lane groups split the latent dimension): the cosine's dot products are
// in-lane sums plus one permlane reduction, and dU's registers of latent
// tiles 2t, 2t+1 are exactly the 16x16x32 B operand of K step t of dA1^T.
// dA1^T's hidden index is permuted (h = 8g + 4q + i for accumulator q,
// register i, lane group g), so each lane ends with dY1 for its own row and
// hidden columns 8g..8g+7 -- the columns it holds A1 and Z4 for: the ReLU /
// dropout mask, the BN1-backward partials and the dY1 store (two float4)
// need no data movement.
// ---------------------------------------------------------------------------
template <int NDT, int R>
struct TopLds {
  static constexpr int DP = 16 * NDT;  // latent padded to whole 16-wide tiles
  static constexpr int CH = DP / 4;    // 8-B chunks per dU image row
  // bf16 images, 3 planes each (uint16_t units)
  static constexpr int LDW = H1;       // W8 image row: 64 B, chunk-swizzled (swz_w)
  static constexpr int PW = DP * LDW;  // one plane of a W8 image [DP][LDW]
  static constexpr int PA1 = R * H1;   // one plane of the A1 image [R][32] (chunk-swizzled)
  static constexpr int PU = R * DP;    // one plane of the dU image [R][DP] (chunk-swizzled)
  static constexpr int W8own = 0;
  static constexpr int A1i = W8own + 3 * PW;
  static constexpr int dUi = A1i + 3 * PA1;
  static constexpr int W8oth = dUi;  // the other tower's W8 lives in the dU region during the forward
  static constexpr int hend = dUi + 3 * PU;
  // fp32 region (float units)
  static constexpr int rsc = (dUi + 3 * PW) / 2;  // [4R] replica-sum scratch (phase 0), dU region after W8oth
  static constexpr int b8s = hend / 2;            // [2][DP] b8 of oth | own (0 for d >= D)
  static constexpr int NW = R / 16;
  static constexpr int cf1 = b8s + 2 * DP;        // [2][4][H1] BN1 mean | gamma*inv | beta | inv per tower
  static constexpr int red = cf1 + 8 * H1;        // [NW][2*H1] dgamma1 | dbeta1 partials per wave
  static constexpr int scal = red + NW * 2 * H1;  // [NW][2] (loss, dls) partials per wave
  static constexpr int rst = scal + 2 * NW;       // [2][2*H1] BN1 moment sums S1|S2 per tower
  static constexpr int total = rst + 4 * H1;      // floats
  static_assert(3 * PW + 8 * R <= 3 * PU, "W8oth + rsc inside the dU region");
  static_assert(A1i % 8 == 0 && dUi % 8 == 0 && hend % 8 == 0, "16-B aligned images");
};

// LDS image swizzles: 8-B chunk c of image row rr is stored at chunk
// c ^ swz(rr) (XOR of row bits; stores bank by dword mod 32, reads mod 64).
// dU image (256-B rows): bits 0-3 of swz_u a bijection of rr's bits 0-3, so
// the 8-B accumulator-layout stores (16 rows x 1 chunk per 16-lane group) are
// conflict-free; bits 2-4 a bijection of rr's bits 0, 1, 3, so the transposed
// reads (8 rows x 4 consecutive chunks per half wave) are conflict-free.
template <int CH>
__device__ __forceinline__ int swz_u(int rr) {
  const int b0 = rr & 1, b1 = (rr >> 1) & 1, b2 = (rr >> 2) & 1, b3 = (rr >> 3) & 1;
  return (b3 | (b2 << 1) | (b0 << 2) | (b1 << 3) | (b3 << 4)) & (CH - 1);
}
// A1 image (64-B rows, 16-B stores = chunk pairs, so the XOR is even):
// conflict-free stores and transposed reads
__device__ __forceinline__ int swz_a(int rr) {
  return (((rr >> 1) & 1) << 1) | ((((rr >> 2) ^ (rr >> 3)) & 1) << 2);
}
// W8 image (64-B rows): conflict-free 16-B forward reads, 2-way transposed reads
__device__ __forceinline__ int swz_w(int d) { return ((d >> 2) & 1) << 2; }


// EMB instances serve the tower-embedding entry points (tt_embed_*):
// TOP_EMB_FWD stores the raw tower outputs U, V (model.py:76-77 before the
// normalisation) and stops; TOP_EMB_BWD takes dU / dV from the caller
// instead of the cosine/MSE closed form.  Everything from dU on is shared.
template <int NDT, int R, bool EMB>
__global__ __launch_bounds__(R * 4) TT_WPE(TT_WPE_TOP) void k_top(StepArgs a) {
  using L = TopLds<NDT, R>;
  constexpr int NTH = R * 4, NW = R / 16, DP = L::DP;
  constexpr int WF4 = DP * (H1 / 4);  // float4 of one tower's padded W8
  constexpr int WPT = (WF4 + NTH - 1) / NTH;
  static_assert(NDT % 2 == 0, "a dA1 K step pairs two latent tiles");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  uint16_t* hs = reinterpret_cast<uint16_t*>(smem);
  const bool bwd = a.mode != TOP_FWD && a.mode != TOP_EMB_FWD;
  const int own = bwd ? (int)blockIdx.y : 0;
  const int oth = 1 - own;
  const int64_t step = step_current(a);
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  const int D = a.D;
  const int rl = 16 * w + r;  // this lane's row in the tile (all 4 lane groups)
  const int64_t row = r0 + rl;
  TT_STAMP(2, 0);

  // ---- phase 0: issue every load: both towers' Z4 slices and W8, biases,
  // logit_scale, this row's (target, weight) or dscore
  float4 zo[2], zs[2], wo[WPT], ws[WPT];
  {
    const float4* po = reinterpret_cast<const float4*>(a.tw[oth].Z4 + row * H1 + 8 * g);
    const float4* ps = reinterpret_cast<const float4*>(a.tw[own].Z4 + row * H1 + 8 * g);
    zo[0] = po[0];
    zo[1] = po[1];
    zs[0] = ps[0];
    zs[1] = ps[1];
  }
#pragma unroll
  for (int k = 0; k < WPT; ++k) {
    const int e = min((int)threadIdx.x + k * NTH, D * (H1 / 4) - 1);
    wo[k] = reinterpret_cast<const float4*>(a.tw[oth].W8)[e];
    ws[k] = reinterpret_cast<const float4*>(a.tw[own].W8)[e];
  }
  float bo = 0.f, bs = 0.f;
  if (threadIdx.x < DP) {
    const int d = min((int)threadIdx.x, D - 1);
    bo = a.tw[oth].b8[d];
    bs = a.tw[own].b8[d];
  }
  const float lsc = *a.logit_scale;
  // this row's (target, weight) or dscore: loads from a valid address in
  // every mode, no branch -- a load under one arm of a branch made hipcc
  // drain vmcnt at the join, before the replica loads below were issued
  const bool m_train = a.mode == TOP_TRAIN, m_given = a.mode == TOP_BWD_GIVEN;
  const float* p_tg = m_train ? a.tgw + 2 * row : (m_given ? a.dscore + min(row, a.B - 1) : a.logit_scale);
  const float* p_wt = m_train ? a.tgw + 2 * row + 1 : a.logit_scale;
  const float tg_raw = *p_tg, wt_raw = *p_wt;
  const float tg = (m_train || m_given) ? tg_raw : 0.f, wt = m_train ? wt_raw : 0.f;
  f32x4 dem[EMB ? NDT : 1];  // TOP_EMB_BWD: this lane's dU slice (issued with the other loads)
  if constexpr (EMB) {
    if (bwd) {
      const float* src = a.demb + ((int64_t)own * a.B + min(row, a.B - 1)) * D;
#pragma unroll
      for (int j = 0; j < NDT; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) dem[j][i] = src[min(16 * j + 4 * g + i, D - 1)];
    }
  }
  // BN1 parameters of column bc of tower bt (wave 0: threads < 2 H1), issued
  // with the other loads; the per-lane tower's pointers are selected from
  // both towers' (scalar) kernel arguments -- a.tw[lane-dependent] would be a
  // vector load of the argument block, then a second dependent round trip
  const int bt = ((int)threadIdx.x / H1) & 1, bc = (int)threadIdx.x % H1;
  auto pick = [&](auto p0, auto p1) { return bt ? p1 : p0; };
  float bn_sh = 0.f, bn_rm = 0.f, bn_rv = 0.f, bn_g = 0.f, bn_be = 0.f;
  if (w == 0) {
    // running stats are NULL when the caller passes no buffers (backward):
    // read gamma in their place then (never used: bn_coefs_pre reads them
    // only for eval or a statistics update, which come with buffers)
    const bool have_rs = a.tw[0].rm1 != nullptr;
    const float* g1p = pick(a.tw[0].g1, a.tw[1].g1);
    bn_sh = pick(a.tw[0].shift1, a.tw[1].shift1)[bc];
    bn_rm = (have_rs ? pick(a.tw[0].rm1, a.tw[1].rm1) : g1p)[bc];
    bn_rv = (have_rs ? pick(a.tw[0].rv1, a.tw[1].rv1) : g1p)[bc];
    bn_g = g1p[bc];
    bn_be = pick(a.tw[0].be1, a.tw[1].be1)[bc];
  }
  RepSum2<NTH, 2 * H1> rs;
  if (a.train) rs.issue(a.tw[0].st1, a.tw[1].st1, ST1S);
  // while the replica loads are in flight: biases, zeroed partials, W8 images
  if (threadIdx.x < DP) {
    const bool ok = (int)threadIdx.x < D;
    smem[L::b8s + threadIdx.x] = ok ? bo : 0.f;
    smem[L::b8s + DP + threadIdx.x] = ok ? bs : 0.f;
  }
  // W8 images: 3 bf16 planes of [DP][LDW], rows d >= D zero
#pragma unroll
  for (int k = 0; k < WPT; ++k) {
    const int e = threadIdx.x + k * NTH;
    if (e < WF4) {
      const int d = e >> 3, c = ((e & 7) ^ swz_w(d)) * 4;
      const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
      put_planes4(hs + L::W8oth + d * L::LDW + c, L::PW, d < D ? wo[k] : z);
      put_planes4(hs + L::W8own + d * L::LDW + c, L::PW, d < D ? ws[k] : z);
    }
  }
  if (a.train) rs.finish(smem + L::rsc, smem + L::rst);
  static_assert(2 * H1 <= 64, "BN1 coefficients: wave 0");
  if (threadIdx.x < 2 * H1) {
    const int tau = bt, c = bc;
    const bool upd = a.update_stats && blockIdx.x == 0 && (bwd ? tau == own : true);
    float mean, inv;
    bn_coefs_pre(a, H1, smem + L::rst + tau * 2 * H1, bn_sh, bn_rm, bn_rv, pick(a.tw[0].rm1, a.tw[1].rm1),
                 pick(a.tw[0].rv1, a.tw[1].rv1), pick(a.tw[0].nbt1, a.tw[1].nbt1), pick(a.tw[0].fin1, a.tw[1].fin1),
                 upd, c, &mean, &inv);
    float* cf = smem + L::cf1 + tau * 4 * H1;
    cf[c] = mean;
    cf[H1 + c] = inv * bn_g;
    cf[2 * H1 + c] = bn_be;
    cf[3 * H1 + c] = inv;
  }
  __syncthreads();
  TT_STAMP(2, 1);

  // ---- this lane's A1 slice (row rl, hidden 8g..8g+7) of both towers:
  // BN1 + ReLU + dropout of Z4, split into bf16 planes (the forward's B operand)
  const bool drop = a.train && a.drop_thr > 0;
  float a1s[8], z4s[8];
  bf16x8 po[3], ps[3];
  {
    auto act = [&](int tau, const float4 (&z)[2], float (&y)[8]) {
      const f32x4* cf = reinterpret_cast<const f32x4*>(smem + L::cf1 + tau * 4 * H1 + 8 * g);
      const f32x4 mu[2] = {cf[0], cf[1]}, al[2] = {cf[H1 / 4], cf[H1 / 4 + 1]}, be[2] = {cf[H1 / 2], cf[H1 / 2 + 1]};
      const float zz[8] = {z[0].x, z[0].y, z[0].z, z[0].w, z[1].x, z[1].y, z[1].z, z[1].w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float v = (zz[e] - mu[e >> 2][e & 3]) * al[e >> 2][e & 3] + be[e >> 2][e & 3];
        y[e] = v > 0.f ? v : 0.f;
      }
      if (drop) {
        const uint64_t key = dropout_key(a.seed, (uint64_t)step, tau, 1);
        const uint32_t rk = dropout_row_key(key, row);
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] = dropout_keep_rk<DROP_HB1>(rk, 8 * g + e, a.drop_thr) ? y[e] * a.drop_scale : 0.f;
      }
    };
    float a1o[8];
    act(oth, zo, a1o);
    act(own, zs, a1s);
    split8x3(a1o, po);
    split8x3(a1s, ps);
    const float zz[8] = {zs[0].x, zs[0].y, zs[0].z, zs[0].w, zs[1].x, zs[1].y, zs[1].z, zs[1].w};
#pragma unroll
    for (int e = 0; e < 8; ++e) z4s[e] = zz[e];
  }
  if (bwd) {  // own A1 image (16-B chunk pair 2g, swizzled)
#pragma unroll
    for (int p = 0; p < 3; ++p)
      *reinterpret_cast<bf16x8*>(hs + L::A1i + p * L::PA1 + rl * H1 + ((2 * g) ^ swz_a(rl)) * 4) = ps[p];
  }

  TT_STAMP(2, 2);
  // ---- forward, transposed: lane (r, g) gets U[row rl][16j + 4g + i]
  f32x4 accO[NDT], accS[NDT];
  {
    // W8 fragments of latent tile j+1 are in flight during tile j's MFMAs
    auto ld = [&](int j, bf16x8 (&fo)[3], bf16x8 (&fs)[3]) {
      const int dr = 16 * j + r;
      const int off = dr * L::LDW + ((2 * g) ^ swz_w(dr)) * 4;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        fo[p] = *reinterpret_cast<const bf16x8*>(hs + L::W8oth + p * L::PW + off);
        fs[p] = *reinterpret_cast<const bf16x8*>(hs + L::W8own + p * L::PW + off);
      }
    };
    bf16x8 fo[2][3], fs[2][3];
    if (!(EMB && bwd)) {  // the embedding backward needs no forward recompute
#pragma unroll
      for (int j = 0; j < NDT; ++j) {  // bias first: U = b + sum
        accO[j] = *reinterpret_cast<const f32x4*>(smem + L::b8s + 16 * j + 4 * g);
        accS[j] = *reinterpret_cast<const f32x4*>(smem + L::b8s + DP + 16 * j + 4 * g);
      }
      ld(0, fo[0], fs[0]);
#pragma unroll
      for (int j = 0; j < NDT; ++j) {
        if (j + 1 < NDT) ld(j + 1, fo[(j + 1) & 1], fs[(j + 1) & 1]);
        // keep the next tile's reads above this tile's MFMAs (the scheduler
        // otherwise sinks them next to their use, one LDS latency per step)
        // and interleave the two independent accumulation chains
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < 6; ++q) {
          accO[j] = mfma_bf16(fo[j & 1][PA[q]], po[PB[q]], accO[j]);
          accS[j] = mfma_bf16(fs[j & 1][PA[q]], ps[PB[q]], accS[j]);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  const bool valid = row < a.B;
  if constexpr (EMB) {
    if (!bwd) {  // TOP_EMB_FWD (own = firm): U -> emb[0][row], V -> emb[1][row]
      if (valid) {
#pragma unroll
        for (int j = 0; j < NDT; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int d = 16 * j + 4 * g + i;
            if (d < D) {
              a.emb[row * D + d] = accS[j][i];
              a.emb[(a.B + row) * D + d] = accO[j][i];
            }
          }
      }
      return;
    }
  }
  if (bwd) __syncthreads();  // W8oth (dU region) read by every wave; A1 image complete
  TT_STAMP(2, 3);

  // ---- cosine, one row per lane
  float ka = 0.f, kb = 0.f;
  if constexpr (!EMB) {
  const float s = expf(lsc);
  float uv = 0.f, oo = 0.f, tt2 = 0.f;
#pragma unroll
  for (int j = 0; j < NDT; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uv += accS[j][i] * accO[j][i];
      oo += accS[j][i] * accS[j][i];
      tt2 += accO[j][i] * accO[j][i];
    }
  uv = col_reduce(uv);
  oo = col_reduce(oo);
  tt2 = col_reduce(tt2);
  const float ino = __builtin_amdgcn_rsqf(oo);  // v_rsq_f32 (1 ulp): no IEEE divides
  const float int_ = __builtin_amdgcn_rsqf(tt2);
  const float cs = uv * ino * int_;
  const float sc = cs * s;
  float ds = 0.f, loss_p = 0.f;
  if (a.mode == TOP_TRAIN) {
    const float diff = sc - tg;
    ds = 2.f * diff * (wt * (1.f / (float)a.B));
    loss_p = valid ? wt * diff * diff : 0.f;
  } else if (a.mode == TOP_BWD_GIVEN) {
    ds = tg;
  }
  ds = valid ? ds : 0.f;
  if (a.score && own == 0 && g == 0 && valid) a.score[row] = sc;
  if (!bwd) return;

  if (own == 0) {  // loss + logit_scale grad once per row tile (lane group 0 covers the rows)
    const float lp = row_reduce16(loss_p), dp = row_reduce16(ds * sc);
    if (l == 0) {
      smem[L::scal + 2 * w + 0] = lp;
      smem[L::scal + 2 * w + 1] = dp;
    }
  }

  // ---- own-tower output gradient (SURVEY 3D closed form)
  //   dU = dc (oth/|oth| - own cos/|own|) / |own|,
  // split into planes per K step t (latent tiles 2t, 2t+1): stored into the
  // dU image for dW8 and used at once as the B operand of dA1^T
  const float dc = ds * s;
  ka = valid ? dc * ino * int_ : 0.f;
  kb = valid ? dc * cs * ino * ino : 0.f;
  }  // !EMB
  const int qd = (l & 15) >> 2, pc = l & 3;  // transposed read: row q, chunk p of this lane
  const int su = swz_u<L::CH>(rl);
  uint16_t* dUs = hs + L::dUi;
  f32x4 dA[2] = {zero4(), zero4()};
#pragma unroll
  for (int t = 0; t < NDT / 2; ++t) {
    float x[8];
    if constexpr (EMB) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d0 = 32 * t + 4 * g + i;
        x[i] = (valid && d0 < D) ? dem[2 * t][i] : 0.f;
        x[4 + i] = (valid && d0 + 16 < D) ? dem[2 * t + 1][i] : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x[i] = ka * accO[2 * t][i] - kb * accS[2 * t][i];
        x[4 + i] = ka * accO[2 * t + 1][i] - kb * accS[2 * t + 1][i];
      }
    }
    bf16x8 du[3];
    split8x3(x, du);
#pragma unroll
    for (int p = 0; p < 3; ++p) {
      const u32x4 v = __builtin_bit_cast(u32x4, du[p]);
      uint16_t* base = dUs + p * L::PU + rl * DP;
      *reinterpret_cast<u32x2*>(base + ((8 * t + g) ^ su) * 4) = (u32x2){v[0], v[1]};
      *reinterpret_cast<u32x2*>(base + ((8 * t + 4 + g) ^ su) * 4) = (u32x2){v[2], v[3]};
    }
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      bf16x8 wf[3];
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const int d0 = 32 * t + 4 * g + qd, d1 = d0 + 16;
        const uint16_t* b = hs + L::W8own + p * L::PW;
        wf[p] = tr_frag(b + d0 * L::LDW + ((2 * pc + q) ^ swz_w(d0)) * 4, b + d1 * L::LDW + ((2 * pc + q) ^ swz_w(d1)) * 4);
      }
      mfma_x3(wf, du, dA[q]);
    }
  }
  TT_STAMP(2, 4);

  // ---- dY1 = dA1 * mask * scale (mask = [A1 > 0] covers ReLU and dropout),
  // dgamma1 / dbeta1 partials
  const TowerDev& T = a.tw[own];
  const float* cf = smem + L::cf1 + own * 4 * H1;
  const float scl = (a.drop_thr > 0) ? a.drop_scale : 1.f;
  float dy[8], sg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int h = 8 * g + e;
    dy[e] = a1s[e] > 0.f ? dA[e >> 2][e & 3] * scl : 0.f;  // 0 on rows >= B (dU = 0)
    sg[e] = dy[e] * ((z4s[e] - cf[h]) * cf[3 * H1 + h]);
  }
  {
    const uint32_t off = (uint32_t)((row * H1 + 8 * g) * 4);
    st_wt16<TT_HANDOFF_AUX>(T.dY1, off, f32x4{dy[0], dy[1], dy[2], dy[3]});
    st_wt16<TT_HANDOFF_AUX>(T.dY1, off + 16, f32x4{dy[4], dy[5], dy[6], dy[7]});
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float vg = row_reduce16(sg[e]), vb = row_reduce16(dy[e]);
    if (r == 0) {
      smem[L::red + w * 2 * H1 + 8 * g + e] = vg;
      smem[L::red + w * 2 * H1 + H1 + 8 * g + e] = vb;
    }
  }
  __syncthreads();  // dU image, BN partials
  TT_STAMP(2, 5);

  // ---- dW8 (as dW8^T[h][d]) and db8 over the R rows of the tile: wave w owns
  // latent tiles w, w + NW, ...; K = rows, 32 per step, read transposed
  float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
  const bf16x8 ones = __builtin_bit_cast(bf16x8, (u32x4){0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});
  for (int pt = w; pt < NDT; pt += NW) {
    f32x4 acc[2] = {zero4(), zero4()};
    f32x4 accb = zero4();
    // operands of K step kk+1 are read while step kk's MFMAs run
    auto ld = [&](int kk, bf16x8 (&bu)[3], bf16x8 (&aa)[2][3]) {
      const int ra = 32 * kk + 8 * g + qd, rb = ra + 4;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const uint16_t* u = dUs + p * L::PU;
        bu[p] = tr_frag(u + ra * DP + ((4 * pt + pc) ^ swz_u<L::CH>(ra)) * 4,
                        u + rb * DP + ((4 * pt + pc) ^ swz_u<L::CH>(rb)) * 4);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const uint16_t* v = hs + L::A1i + p * L::PA1;
          aa[q][p] = tr_frag(v + ra * H1 + ((4 * q + pc) ^ swz_a(ra)) * 4, v + rb * H1 + ((4 * q + pc) ^ swz_a(rb)) * 4);
        }
      }
    };
    bf16x8 bu[2][3], aa[2][2][3];
    ld(0, bu[0], aa[0]);
#pragma unroll
    for (int kk = 0; kk < R / 32; ++kk) {
      if (kk + 1 < R / 32) ld(kk + 1, bu[(kk + 1) & 1], aa[(kk + 1) & 1]);
#pragma unroll
      for (int q = 0; q < 2; ++q) mfma_x3(aa[kk & 1][q], bu[kk & 1], acc[q]);
#pragma unroll
      for (int p = 2; p >= 0; --p) accb = mfma_bf16(ones, bu[kk & 1][p], accb);
    }
    // lane (r, g): dW8[d = 16 pt + r][16 q + 4g + i], db8[d] in every element of accb
    const int d = 16 * pt + r;
    if (d < D) {
#pragma unroll
      for (int q = 0; q < 2; ++q) st_wt16(slab, (uint32_t)((T.so_W8 + d * H1 + 16 * q + 4 * g) * 4), acc[q]);
      if (g == 0) slab[T.so_b8 + d] = accb[0];
    }
  }
  TT_STAMP(2, 6);

  // dgamma1 | dbeta1 (adjacent in a replica) and (dls, loss): the waves'
  // partials in wave order, then the cross-block accumulation
  if (threadIdx.x < 2 * H1)
    xblock_add(a.det, T.gg1, BNG, T.dslot, 2 * H1, threadIdx.x, wave_rows_sum<NW>(smem + L::red, 2 * H1, threadIdx.x));
  if (own == 0 && threadIdx.x < 2) {
    const int c = threadIdx.x;  // 0: dL/dlogit_scale, 1: batch-mean loss
    const float v = EMB ? 0.f : wave_rows_sum<NW>(smem + L::scal + 1 - c, 2, 0);  // EMB: no cosine, no scale
    if (c == 0 || a.mode == TOP_TRAIN || a.det)
      xblock_add(a.det, a.lsr, LSR, a.dslot_lsr, 2, c, c == 0 ? v : (a.mode == TOP_TRAIN ? v / (float)a.B : 0.f));
  }
  TT_STAMP(2, 7);
}

// ---------------------------------------------------------------------------
// k_top_pair : the training step's k_top at large batches with BOTH towers'
// backward in one block of 64 rows: waves 0-3 take tower 0, waves 4-7 tower 1,
// 16 rows each.  k_top's tile pair (one block per tower) computes both
// towers' forward in both blocks; here each tower's forward is computed once
// and U / V are exchanged through LDS (fp32, padded rows), which halves the
// forward MFMAs and the BN1 / ReLU / dropout work per row.  Everything else
// follows k_top (same fragment layouts, swizzles and closed-form dU); the
// dW8 partials of a block cover 64 rows of both towers.
// LDS: the W8 images of both towers (phases 0-3) are reused for tower 0's dU
// image and the U / V exchange region for tower 1's, once dA1 has read W8.
// ---------------------------------------------------------------------------
template <int NDT, int R_ = 64>
struct PairLds {
  static constexpr int R = R_;           // rows per block (64, or 32 for small batches)
  static constexpr int WT = R / 16;      // waves per tower
  static constexpr int NW = 2 * WT;      // waves per block
  static constexpr int DP = 16 * NDT;
  static constexpr int CH = DP / 4;      // 8-B chunks per dU image row
  static constexpr int LDW = H1;         // W8 image row (bf16)
  static constexpr int PW = DP * LDW;    // one W8 plane
  static constexpr int PA1 = R * H1;     // one A1 plane
  static constexpr int PU = R * DP;      // one dU plane
  static constexpr int XLD = DP + 4;     // exchange row stride (floats): conflict-free float4 rows
  // bf16 units
  static constexpr int W8i = 0;                     // [tower][3][DP][LDW], phases 0-3
  static constexpr int dU0 = 0;                     // tower 0's dU image [3][R][DP], after dA1
  static constexpr int A1i = W8i + 2 * 3 * PW;      // [tower][3][R][H1]
  static constexpr int XCi = A1i + 2 * 3 * PA1;     // exchange fp32 [tower][R][XLD], phases 2-3
  static constexpr int dU1 = XCi;                   // tower 1's dU image, after dA1
  static constexpr int xc_h = 2 * R * XLD * 2;      // exchange size, bf16 units
  static constexpr int hend = XCi + (xc_h > 3 * PU ? xc_h : 3 * PU);
  static_assert(3 * PU <= 2 * 3 * PW, "tower 0's dU image inside the two W8 images");
  static_assert(A1i % 8 == 0 && XCi % 8 == 0 && hend % 8 == 0, "16-B aligned regions");
  // fp32 region (float units)
  static constexpr int b8s = hend / 2;              // [tower][DP] (0 for d >= D)
  static constexpr int cf1 = b8s + 2 * DP;          // [tower][4][H1] mean | gamma*inv | beta | inv
  static constexpr int red = cf1 + 8 * H1;          // [NW waves][2*H1] dgamma1 | dbeta1 partials (tower = w / WT)
  static constexpr int scal = red + NW * 2 * H1;    // [WT waves][2] (loss, dls) partials of the tower-0 waves
  static constexpr int rsc = scal + 8;              // [8 R] replica-sum scratch
  static constexpr int rst = rsc + 8 * R;           // [tower][2*H1] BN1 moment sums
  static constexpr int total = rst + 4 * H1;
};

// R = 64: both towers of 64 rows (8 waves); R = 32 (batches below the folded
// path: twice the blocks on the same CUs) 4 waves of 16 rows
template <int NDT, int R>
__global__ __launch_bounds__(R * 8) TT_WPE(TT_WPE_TOP) void k_top_pair(StepArgs a) {
  using L = PairLds<NDT, R>;
  constexpr int NTH = R * 8, DP = L::DP, WT = L::WT;
  constexpr int WF4 = DP * (H1 / 4);                // float4 of one tower's padded W8
  constexpr int WPT = (2 * WF4 + NTH - 1) / NTH;    // both towers' W8: float4 per thread
  static_assert(NDT % 2 == 0, "a dA1 K step pairs two latent tiles");
  static_assert(2 * WF4 % NTH == 0, "whole W8 float4 rounds");
  static_assert(2 * DP <= NTH && 4 * H1 <= NTH, "b8 / BN1-affine lanes");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  uint16_t* hs = reinterpret_cast<uint16_t*>(smem);
  const int64_t step = step_current(a);
  const int64_t r0 = (int64_t)tile64(a) * R;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  const int tw = __builtin_amdgcn_readfirstlane(w / WT);  // this wave's tower (uniform: scalar a.tw[tw] reads)
  const int rl = 16 * (w % WT) + r;  // this lane's row in the tile
  const int64_t row = r0 + rl;
  const int D = a.D;
  const TowerDev& T = a.tw[tw];
  auto pick = [&](int t_, auto p0, auto p1) { return t_ ? p1 : p0; };
  TT_STAMP(2, 0);

  // ---- phase 0: every load -- own tower's Z4 slice, both W8 (raw), biases,
  // logit_scale, (target, weight), BN1 inputs, BN1 moment replicas
  float4 zs[2];
  {
    const float4* ps_ = reinterpret_cast<const float4*>(T.Z4 + row * H1 + 8 * g);
    zs[0] = ps_[0];
    zs[1] = ps_[1];
  }
  float4 wv[WPT];
#pragma unroll
  for (int k = 0; k < WPT; ++k) {
    const int e = (int)threadIdx.x + k * NTH, tt = e / WF4;
    const int el = min(e - tt * WF4, D * (H1 / 4) - 1);
    wv[k] = reinterpret_cast<const float4*>(pick(tt, a.tw[0].W8, a.tw[1].W8))[el];
  }
  const int bt8 = (int)threadIdx.x / DP, bd8 = min((int)threadIdx.x % DP, D - 1);
  const float b8v = threadIdx.x < 2 * DP ? pick(bt8 & 1, a.tw[0].b8, a.tw[1].b8)[bd8] : 0.f;
  const float lsc = *a.logit_scale;
  const float tg = a.tgw[2 * row], wt = a.tgw[2 * row + 1];
  const int bt = ((int)threadIdx.x / H1) & 1, bc = (int)threadIdx.x % H1;
  float bn_sh = 0.f, bn_rm = 0.f, bn_rv = 0.f, bn_g = 0.f, bn_be = 0.f;
  if (w == 0) {
    const bool have_rs = a.tw[0].rm1 != nullptr;
    const float* g1p = pick(bt, a.tw[0].g1, a.tw[1].g1);
    bn_sh = pick(bt, a.tw[0].shift1, a.tw[1].shift1)[bc];
    bn_rm = (have_rs ? pick(bt, a.tw[0].rm1, a.tw[1].rm1) : g1p)[bc];
    bn_rv = (have_rs ? pick(bt, a.tw[0].rv1, a.tw[1].rv1) : g1p)[bc];
    bn_g = g1p[bc];
    bn_be = pick(bt, a.tw[0].be1, a.tw[1].be1)[bc];
  }
  RepSum2<NTH, 2 * H1> rs;
  rs.issue(a.tw[0].st1, a.tw[1].st1, ST1S);
  if (threadIdx.x < 2 * DP) smem[L::b8s + threadIdx.x] = (threadIdx.x % DP) < (unsigned)D ? b8v : 0.f;
#pragma unroll
  for (int k = 0; k < WPT; ++k) {
    const int e = (int)threadIdx.x + k * NTH, tt = e / WF4, el = e - tt * WF4;
    const int d = el >> 3, c = ((el & 7) ^ swz_w(d)) * 4;
    const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
    put_planes4(hs + L::W8i + tt * 3 * L::PW + d * L::LDW + c, L::PW, d < D ? wv[k] : z);
  }
  rs.finish(smem + L::rsc, smem + L::rst);
  if (threadIdx.x < 2 * H1) {
    float mean, inv;
    bn_coefs_pre(a, H1, smem + L::rst + bt * 2 * H1, bn_sh, bn_rm, bn_rv, pick(bt, a.tw[0].rm1, a.tw[1].rm1),
                 pick(bt, a.tw[0].rv1, a.tw[1].rv1), pick(bt, a.tw[0].nbt1, a.tw[1].nbt1),
                 pick(bt, a.tw[0].fin1, a.tw[1].fin1), a.update_stats && blockIdx.x == 0, bc, &mean, &inv);
    float* cf = smem + L::cf1 + bt * 4 * H1;
    cf[bc] = mean;
    cf[H1 + bc] = inv * bn_g;
    cf[2 * H1 + bc] = bn_be;
    cf[3 * H1 + bc] = inv;
  }
  __syncthreads();
  TT_STAMP(2, 1);

  // ---- phase 1: own tower's A1 slice (row rl, hidden 8g..8g+7): BN1 + ReLU
  // + dropout of Z4, split into planes (the forward's B operand), A1 image
  const bool drop = a.drop_thr > 0;
  float a1s[8], z4s[8];
  bf16x8 ps[3];
  {
    const f32x4* cf = reinterpret_cast<const f32x4*>(smem + L::cf1 + tw * 4 * H1 + 8 * g);
    const f32x4 mu[2] = {cf[0], cf[1]}, al[2] = {cf[H1 / 4], cf[H1 / 4 + 1]}, be[2] = {cf[H1 / 2], cf[H1 / 2 + 1]};
    const float zz[8] = {zs[0].x, zs[0].y, zs[0].z, zs[0].w, zs[1].x, zs[1].y, zs[1].z, zs[1].w};
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      z4s[e] = zz[e];
      const float v = (zz[e] - mu[e >> 2][e & 3]) * al[e >> 2][e & 3] + be[e >> 2][e & 3];
      a1s[e] = v > 0.f ? v : 0.f;
    }
    if (drop) {
      const uint64_t key = dropout_key(a.seed, (uint64_t)step, tw, 1);
      const uint32_t rk = dropout_row_key(key, row);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        a1s[e] = dropout_keep_rk<DROP_HB1>(rk, 8 * g + e, a.drop_thr) ? a1s[e] * a.drop_scale : 0.f;
    }
    split8x3(a1s, ps);
#pragma unroll
    for (int p = 0; p < 3; ++p)
      *reinterpret_cast<bf16x8*>(hs + L::A1i + (tw * 3 + p) * L::PA1 + rl * H1 + ((2 * g) ^ swz_a(rl)) * 4) = ps[p];
  }
  TT_STAMP(2, 2);

  // ---- phase 2: own tower's forward, transposed (lane (r, g): U[row rl][16j
  // + 4g + i]); tile pairs as two interleaved chains, the next pair's W8
  // fragments read above the current pair's MFMAs
  f32x4 accS[NDT];
  {
    const uint16_t* wb = hs + L::W8i + tw * 3 * L::PW;
    auto ld = [&](int j, bf16x8 (&f)[3]) {
      const int dr = 16 * j + r;
      const int off = dr * L::LDW + ((2 * g) ^ swz_w(dr)) * 4;
#pragma unroll
      for (int p = 0; p < 3; ++p) f[p] = *reinterpret_cast<const bf16x8*>(wb + p * L::PW + off);
    };
#pragma unroll
    for (int j = 0; j < NDT; ++j) accS[j] = *reinterpret_cast<const f32x4*>(smem + L::b8s + tw * DP + 16 * j + 4 * g);
    bf16x8 f[2][2][3];
    ld(0, f[0][0]);
    ld(1, f[0][1]);
#pragma unroll
    for (int jj = 0; jj < NDT / 2; ++jj) {
      if (jj + 1 < NDT / 2) {
        ld(2 * jj + 2, f[(jj + 1) & 1][0]);
        ld(2 * jj + 3, f[(jj + 1) & 1][1]);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        accS[2 * jj] = mfma_bf16(f[jj & 1][0][PA[q]], ps[PB[q]], accS[2 * jj]);
        accS[2 * jj + 1] = mfma_bf16(f[jj & 1][1][PA[q]], ps[PB[q]], accS[2 * jj + 1]);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  // exchange: own U to LDS, the other tower's V back
  float* xc = smem + L::XCi / 2;
#pragma unroll
  for (int j = 0; j < NDT; ++j)
    *reinterpret_cast<f32x4*>(xc + (tw * R + rl) * L::XLD + 16 * j + 4 * g) = accS[j];
  __syncthreads();  // exchange rows written; A1 images complete
  f32x4 accO[NDT];
#pragma unroll
  for (int j = 0; j < NDT; ++j)
    accO[j] = *reinterpret_cast<const f32x4*>(xc + ((1 - tw) * R + rl) * L::XLD + 16 * j + 4 * g);
  TT_STAMP(2, 3);

  // ---- phase 3: cosine (one row per lane), loss and dls (tower-0 waves),
  // closed-form dU, dA1^T = W8^T dU
  const bool valid = row < a.B;
  const float s = expf(lsc);
  float uv = 0.f, oo = 0.f, tt2 = 0.f;
#pragma unroll
  for (int j = 0; j < NDT; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uv += accS[j][i] * accO[j][i];
      oo += accS[j][i] * accS[j][i];
      tt2 += accO[j][i] * accO[j][i];
    }
  uv = col_reduce(uv);
  oo = col_reduce(oo);
  tt2 = col_reduce(tt2);
  const float ino = __builtin_amdgcn_rsqf(oo);
  const float int_ = __builtin_amdgcn_rsqf(tt2);
  const float cs = uv * ino * int_;
  const float sc = cs * s;
  const float diff = sc - tg;
  float ds = 2.f * diff * (wt * (1.f / (float)a.B));
  const float loss_p = valid ? wt * diff * diff : 0.f;
  ds = valid ? ds : 0.f;
  if (tw == 0) {
    if (a.score && g == 0 && valid) a.score[row] = sc;
    const float lp = row_reduce16(loss_p), dp = row_reduce16(ds * sc);
    if (l == 0) {
      smem[L::scal + 2 * w + 0] = lp;
      smem[L::scal + 2 * w + 1] = dp;
    }
  }
  const float dc = ds * s;
  const float ka = valid ? dc * ino * int_ : 0.f;
  const float kb = valid ? dc * cs * ino * ino : 0.f;
  const int qd = (l & 15) >> 2, pc = l & 3;
  f32x4 dA[2] = {zero4(), zero4()};
  bf16x8 du[NDT / 2][3];
  {
    const uint16_t* wb = hs + L::W8i + tw * 3 * L::PW;
#pragma unroll
    for (int t = 0; t < NDT / 2; ++t) {
      float x[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        x[i] = ka * accO[2 * t][i] - kb * accS[2 * t][i];
        x[4 + i] = ka * accO[2 * t + 1][i] - kb * accS[2 * t + 1][i];
      }
      split8x3(x, du[t]);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        bf16x8 wf[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const int d0 = 32 * t + 4 * g + qd, d1 = d0 + 16;
          const uint16_t* b = wb + p * L::PW;
          wf[p] = tr_frag(b + d0 * L::LDW + ((2 * pc + q) ^ swz_w(d0)) * 4, b + d1 * L::LDW + ((2 * pc + q) ^ swz_w(d1)) * 4);
        }
        mfma_x3(wf, du[t], dA[q]);
      }
    }
  }
  TT_STAMP(2, 4);

  // ---- phase 4: dY1 = dA1 * mask * scale, dgamma1 / dbeta1 partials; the dU
  // images once every wave is past the W8 reads and the exchange reads
  const float* cf = smem + L::cf1 + tw * 4 * H1;
  const float scl = drop ? a.drop_scale : 1.f;
  float dy[8], sg[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int h = 8 * g + e;
    dy[e] = a1s[e] > 0.f ? dA[e >> 2][e & 3] * scl : 0.f;
    sg[e] = dy[e] * ((z4s[e] - cf[h]) * cf[3 * H1 + h]);
  }
  {
    const uint32_t off = (uint32_t)((row * H1 + 8 * g) * 4);
    st_wt16<TT_HANDOFF_AUX>(T.dY1, off, f32x4{dy[0], dy[1], dy[2], dy[3]});
    st_wt16<TT_HANDOFF_AUX>(T.dY1, off + 16, f32x4{dy[4], dy[5], dy[6], dy[7]});
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float vg = row_reduce16(sg[e]), vb = row_reduce16(dy[e]);
    if (r == 0) {
      smem[L::red + w * 2 * H1 + 8 * g + e] = vg;
      smem[L::red + w * 2 * H1 + H1 + 8 * g + e] = vb;
    }
  }
  __syncthreads();  // W8 and exchange regions dead
  {
    const int su = swz_u<L::CH>(rl);
    uint16_t* dUs = hs + (tw == 0 ? L::dU0 : L::dU1);
#pragma unroll
    for (int t = 0; t < NDT / 2; ++t)
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        const u32x4 v = __builtin_bit_cast(u32x4, du[t][p]);
        uint16_t* base = dUs + p * L::PU + rl * DP;
        *reinterpret_cast<u32x2*>(base + ((8 * t + g) ^ su) * 4) = (u32x2){v[0], v[1]};
        *reinterpret_cast<u32x2*>(base + ((8 * t + 4 + g) ^ su) * 4) = (u32x2){v[2], v[3]};
      }
  }
  __syncthreads();  // dU images, BN partials
  // BN1 affine and logit_scale / loss partials into the replicas, issued here
  // so their round trip overlaps dW8 instead of ending the kernel
  // (dgamma1 | dbeta1 of a tower: the sum of its 4 waves' rows in wave order;
  // adjacent in a replica)
  if (threadIdx.x < 4 * H1) {
    const int tt = (int)threadIdx.x / (2 * H1), k = (int)threadIdx.x % (2 * H1);
    const float v = wave_rows_sum<WT>(smem + L::red + tt * WT * 2 * H1, 2 * H1, k);
    xblock_add(a.det, pick(tt, a.tw[0].gg1, a.tw[1].gg1), BNG, pick(tt, a.tw[0].dslot, a.tw[1].dslot), 2 * H1, k, v);
  }
  if (threadIdx.x < 2) {
    const int c = threadIdx.x;  // 0: dL/dlogit_scale, 1: batch-mean loss
    const float v = wave_rows_sum<WT>(smem + L::scal + 1 - c, 2, 0);
    xblock_add(a.det, a.lsr, LSR, a.dslot_lsr, 2, c, c == 0 ? v : v / (float)a.B);
  }
  TT_STAMP(2, 5);

  // ---- phase 5: dW8 (as dW8^T[h][d]) and db8 of the wave's tower over the
  // R rows (K = rows, 32-row steps); its WT waves own latent tiles
  // (w % WT), (w % WT) + WT, ...
  {
    float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
    const uint16_t* dUs = hs + (tw == 0 ? L::dU0 : L::dU1);
    const uint16_t* a1b = hs + L::A1i + tw * 3 * L::PA1;
    const bf16x8 ones = __builtin_bit_cast(bf16x8, (u32x4){0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u});
    for (int pt = w % WT; pt < NDT; pt += WT) {
      f32x4 acc[2] = {zero4(), zero4()};
      f32x4 accb = zero4();
#pragma unroll
      for (int kk = 0; kk < R / 32; ++kk) {
        const int ra = 32 * kk + 8 * g + qd, rb = ra + 4;
        bf16x8 bu[3], aa[2][3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
          const uint16_t* u = dUs + p * L::PU;
          bu[p] = tr_frag(u + ra * DP + ((4 * pt + pc) ^ swz_u<L::CH>(ra)) * 4,
                          u + rb * DP + ((4 * pt + pc) ^ swz_u<L::CH>(rb)) * 4);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const uint16_t* v = a1b + p * L::PA1;
            aa[q][p] = tr_frag(v + ra * H1 + ((4 * q + pc) ^ swz_a(ra)) * 4, v + rb * H1 + ((4 * q + pc) ^ swz_a(rb)) * 4);
          }
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) mfma_x3(aa[q], bu, acc[q]);
#pragma unroll
        for (int p = 2; p >= 0; --p) accb = mfma_bf16(ones, bu[p], accb);
      }
      const int d = 16 * pt + r;
      if (d < D) {
#pragma unroll
        for (int q = 0; q < 2; ++q) st_wt16(slab, (uint32_t)((T.so_W8 + d * H1 + 16 * q + 4 * g) * 4), acc[q]);
        if (g == 0) slab[T.so_b8 + d] = accb[0];
      }
    }
  }
  TT_STAMP(2, 6);

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
      sizeof(float) * ((size_t)H1 * LDW + (size_t)(H1 + H0) * LDT + 4 * H1 + 5 * H1 + 4 * H0 + 8 * H0 + 4 * R +
                       2 * H1);
};

template <int R>
__global__ __launch_bounds__(R * 4) void k_bwd_mid(StepArgs a) {
  static_assert(R == 64 || R == 32, "4 (or 2) waves of 16 rows");
  constexpr int NTH = R * 4, NW = R / 16, TPW = 8 / NW;  // dW4 tiles (of 2 x 4) per wave
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
  float* db4 = A0T + H0 * LDT;        // [4 waves][32]
  float* c1 = db4 + 4 * H1;           // k1[32] mb[32] mg[32] mean1[32] inv1[32]
  float* c0 = c1 + 5 * H1;            // mean0[64] alpha0[64] beta0[64] inv0[64]
  float* red = c0 + 4 * H0;           // [4 waves][128]
  float* rsc = red + 8 * H0;          // [NTH] replica-sum scratch
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
  // W4 and the BN coefficients' inputs are issued with the tiles above (one
  // round trip; they used to follow the replica sum, W4 in two dependent
  // load -> store pairs).  Every thread loads (clamped columns): no branch.
  constexpr int W4T = H1 * H0 / 4 / NTH;  // W4 float4 per thread
  static_assert(H1 * H0 / 4 == W4T * NTH, "whole W4 float4 rounds");
  float4 w4v[W4T];
#pragma unroll
  for (int k = 0; k < W4T; ++k) {
    const int we = (int)threadIdx.x + k * NTH;
    w4v[k] = *reinterpret_cast<const float4*>(T.W4 + (we >> 4) * H0 + 4 * (we & 15));
  }
  const int c1i = min((int)threadIdx.x, H1 - 1), c0i = min(max((int)threadIdx.x - H1, 0), H0 - 1);
  const float f1inv = T.fin1[H1 + c1i], f1mean = T.fin1[c1i], g1v = T.g1[c1i];
  const float f0inv = T.fin0[H0 + c0i], f0mean = T.fin0[c0i], g0v = T.g0[c0i], be0v = T.be0[c0i];
  const float invB = 1.f / (float)a.B;
  rep_sum<NTH, 2 * H1>(T.gg1, BNG, rsc, rst);  // gg1|gbe1 are adjacent in a replica
  if (threadIdx.x < H1) {
    const int c = threadIdx.x;
    c1[c] = f1inv * g1v;
    c1[H1 + c] = a.train ? rst[H1 + c] * invB : 0.f;  // eval: BN is affine, no batch-mean terms
    c1[2 * H1 + c] = a.train ? rst[c] * invB : 0.f;
    c1[3 * H1 + c] = f1mean;
    c1[4 * H1 + c] = f1inv;
  } else if (threadIdx.x < H1 + H0) {
    const int c = threadIdx.x - H1;
    c0[c] = f0mean;
    c0[H0 + c] = f0inv * g0v;
    c0[2 * H0 + c] = be0v;
    c0[3 * H0 + c] = f0inv;
  }
#pragma unroll
  for (int k = 0; k < W4T; ++k) {
    const int we = (int)threadIdx.x + k * NTH;
    *reinterpret_cast<float4*>(W4s + (we >> 4) * LDW + 4 * (we & 15)) = w4v[k];
  }
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
    if (g == 0) db4[w * H1 + col] = cb;
  }
  const bool drop = a.drop_thr > 0;
  const uint64_t key = dropout_key(a.seed, (uint64_t)step, t, 0);
  f32x4 a0[4], zh0[4];
  uint32_t rk[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) rk[i] = dropout_row_key(key, r0 + 16 * w + 4 * g + i);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      const float z = zz0[j][i];
      const bool ok = row < a.B;
      const float av = bn_relu_drop(z, c0[col], c0[H0 + col], c0[2 * H0 + col], drop, rk[i], col, a.drop_thr,
                                    a.drop_scale);
      a0[j][i] = ok ? av : 0.f;
      zh0[j][i] = ok ? (z - c0[col]) * c0[3 * H0 + col] : 0.f;
    }
    store_tile_T(A0T, LDT, 16 * j, 16 * w, a0[j]);
  }
  __syncthreads();
  TT_STAMP(3, 2);

  // dW4 = dZ4^T A0 over the tile's rows: wave w owns h1-tile (w&1) x h0-tiles
  // TPW*(w>>1)..+TPW-1 and writes them straight into this tile's slab
  float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
  {
    const int p = w & 1, q0 = TPW * (w >> 1);
    f32x4 acc[TPW];
#pragma unroll
    for (int q = 0; q < TPW; ++q) acc[q] = zero4();
    strip_gemm_nt<TPW>(dZT + 16 * p * LDT, LDT, A0T + 16 * q0 * LDT, LDT, R, acc);
#pragma unroll
    for (int q = 0; q < TPW; ++q) store_tile_rm_wt(slab, (int)T.so_W4 + 16 * p * H0 + 16 * (q0 + q), H0, acc[q]);
  }

  // dA0 = dZ4 W4  (K = 32; A from the transposed image, W4 row-major)
  f32x4 dA[4] = {zero4(), zero4(), zero4(), zero4()};
  strip_gemm_tn<4>(dZT + 16 * w, LDT, W4s, LDW, H1, dA);
  const float scl = drop ? a.drop_scale : 1.f;
  float sg[4], sb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sg[j] = 0.f;
    sb[j] = 0.f;
    f32x4 dyv;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float dy = a0[j][i] > 0.f ? dA[j][i] * scl : 0.f;  // 0 on rows >= B (a0 = 0)
      dyv[i] = dy;
      sg[j] += dy * zh0[j][i];
      sb[j] += dy;
    }
    store_tile_rm_wt(T.dY0 + r0 * H0, 16 * w * H0 + 16 * j, H0, dyv);
  }
  cols_to_lds<4>(sg, red, 2 * H0);
  cols_to_lds<4>(sb, red + H0, 2 * H0);
  __syncthreads();
  TT_STAMP(3, 3);
  if (threadIdx.x < 2 * H0)  // gamma0 | beta0 grads (adjacent in a replica)
    xblock_add(a.det, T.gg0, BNG, T.dslot, 2 * H0, threadIdx.x, wave_rows_sum<NW>(red, 2 * H0, threadIdx.x));
  if (threadIdx.x < H1) slab[T.so_b4 + threadIdx.x] = wave_rows_sum<NW>(db4, H1, threadIdx.x);
  TT_STAMP(3, 4);
}

// ---------------------------------------------------------------------------
// k_bwd_mid_fold : k_bwd_mid with the BN0 backward and dW0 folded in, for
// numeric-only towers with kp <= 64 (k_bwd_first is not launched).
//
// BN0's backward  dZ0 = k0 (dY0 - mb - Zh0 mg)  (k0 = inv0 gamma0,
// mb = mean_B dY0, mg = mean_B dY0 Zh0) needs batch-wide means, but
// dW0 = dZ0^T X is linear in them:
//   dW0 = k0 (P - mb s^T - mg Q) + db0 c^T,   X' = X - c (c: the batch's
//   first row, keeps the subtractions well conditioned),
//   P = dY0^T X', Q = Zh0^T X', s = sum_rows X', db0 = -k0 mg sum_rows Zh0.
// Each 128-row tile writes P and Q as slab partials (the same bytes per
// batch row as k_bwd_first's dW0 partials of 64-row tiles) and s, sum Zh0,
// dgamma0, dbeta0 into replicas; k_reduce_adam combines them with the batch
// means (Seg kinds 3, 4).  dY0 never leaves the block.
// 8 waves, wave w owns tile rows 16w..16w+15 (C layout) as in k_bwd_mid.
// P and Q run on the bf16x3 MFMA core (fp32-accurate, tt_common.h) from
// channel-major bf16 plane images: dY0 / Zh0 written from the accumulator
// layout, X' from a row-coalesced gather (16 lanes per 256-B row, each lane a
// 4-row x 4-column block, so every image write is one 8-B chunk per plane).
// ---------------------------------------------------------------------------
template <int R>
struct FoldLds {
  // bf16x3 images (bf16 units, 3 planes each).  Phases 1-2: A0 channel-major
  // [64][R] (fold_at, as the P | Q images), dZ4 row-major [R][32] and W4^T
  // [64][32] (swz_dz), the operands of dW4 and dA0
  static constexpr int PL = H0 * R;              // one [64][R] plane
  static constexpr int PZ = R * H1;              // one dZ4 plane
  static constexpr int PW4 = H0 * H1;            // one W4^T plane
  static constexpr int A0i = 0;
  static constexpr int dZi = A0i + 3 * PL;
  static constexpr int W4i = dZi + 3 * PZ;
  static constexpr int dead = W4i + 3 * PW4;     // end of the region dead after dW4 / dA0
  // phase 3-4 (over the dead region and beyond): the images of dY0, Zh0 and
  // X', channel / column major ([64][R] per plane, rows along the
  // contraction), 16-B chunks XOR-swizzled by the row's low 4 bits
  static constexpr int img = 3 * PL;             // one image (3 planes)
  static constexpr int IY = 0, IZ = img, IX = 2 * img;
  static constexpr int imgs_f = 3 * img / 2;     // floats
  static_assert(IX >= dead, "X' image clear of the phase-2 operands (written during phase 2)");
  static_assert(dZi % 8 == 0 && W4i % 8 == 0, "16-B aligned images");
  static constexpr int db4 = imgs_f;             // [8 waves][32]
  static constexpr int c1 = db4 + 8 * H1;        // k1 mb mg mean1 inv1 [5][32]
  static constexpr int c0 = c1 + 5 * H1;         // mean0 alpha0 beta0 inv0 [4][64]
  static constexpr int red = c0 + 4 * H0;        // [8 waves][sum dY0 Zh0 | sum dY0 | sum Zh0 | sum X' [4][64]]
  static constexpr int rsc = red + 8 * 4 * H0;   // [4R] replica-sum scratch
  static constexpr int rst = rsc + 4 * R;        // [2][32] sum dgamma1 | sum dbeta1
  static constexpr int total = rst + 2 * H1;
  static constexpr size_t bytes = sizeof(float) * (size_t)total;
  static_assert(R == 128, "16 chunks of 8 rows per image row: the swizzle covers a whole row");
};

// 8-B chunk swizzle of the 64-B-row images (dZ4 [R][32], W4^T [64][32]):
// conflict-free 8-B stores of 4 rows x 4 chunks per 16 lanes, 16-B reads of
// chunk pairs (the XOR is 0 or 4) and transposed reads of 8 rows x 4 chunks
// per half wave
__device__ __forceinline__ int swz_dz(int row) { return (((row >> 1) ^ (row >> 3)) & 1) << 2; }

// bf16 offset of (row c, contraction index k) in a FoldLds image plane; the
// chunk swizzle folds in c >> 4 so the X' writes (rows 4 xc + i for 16 lanes
// xc) land on 16 distinct chunks as well as the fragment reads (16 rows)
__device__ __forceinline__ int fold_at(int c, int k) {
  return c * 128 + ((((k >> 3) ^ c ^ (c >> 4)) & 15) << 3) + (k & 7);
}

template <int R, bool VEC>
__global__ __launch_bounds__(R * 4) TT_WPE(TT_WPE_MID) void k_bwd_mid_fold(StepArgs a) {
  using L = FoldLds<R>;
  static_assert(R == 128, "8 waves: one dW4 tile and one P|Q strip per wave");
  constexpr int NTH = R * 4;
  constexpr int XK = R * (FOLD_MAX_KP / 4) / NTH;  // X' float4 per thread (4)
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int64_t step = step_current(a);
  const int64_t r0 = (int64_t)blockIdx.x * R;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  uint16_t* hs = reinterpret_cast<uint16_t*>(smem);
  float* db4 = smem + L::db4;
  float* c1 = smem + L::c1;
  float* c0 = smem + L::c0;
  float* red = smem + L::red;
  TT_STAMP(3, 0);
  TT_STAMP_T(4, 0, 448);

  // ---- phase 0: issue every load -- dY1, Z4, Z0 of this wave's rows (C
  // layout), W4, BN inputs, then (after the step load they depend on) the
  // dataset rows of this thread's X' gather rows and of the shift row.
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
  // W4^T image: wave w, lane l takes h0 = 16 (w & 3) + (l >> 2) and h1
  // chunk 4 (w >> 2) + (l & 3): four W4 rows (4 scalar loads, lanes along h0)
  static_assert(H1 * H0 / 4 == NTH, "W4: one chunk of 4 per thread");
  const int w4r = 16 * (w & 3) + (l >> 2), w4c = 4 * (w >> 2) + (l & 3);
  float4 w4v;
  w4v.x = T.W4[(4 * w4c + 0) * H0 + w4r];
  w4v.y = T.W4[(4 * w4c + 1) * H0 + w4r];
  w4v.z = T.W4[(4 * w4c + 2) * H0 + w4r];
  w4v.w = T.W4[(4 * w4c + 3) * H0 + w4r];
  const int c1i = min((int)threadIdx.x, H1 - 1), c0i = min(max((int)threadIdx.x - H1, 0), H0 - 1);
  const float f1inv = T.fin1[H1 + c1i], f1mean = T.fin1[c1i], g1v = T.g1[c1i];
  const float f0inv = T.fin0[H0 + c0i], f0mean = T.fin0[c0i], g0v = T.g0[c0i], be0v = T.be0[c0i];
  const float invB = 1.f / (float)a.B;
  // X' gather: thread takes float4 column group xc of rows xr0 .. xr0 + 3
  static_assert(XK == 4, "4 x 4 block per thread");
  const int xc = (int)threadIdx.x & 15, xr0 = 4 * ((int)threadIdx.x >> 4);
  const int64_t base = batch_row0(a, step);
  int64_t xrow[XK];
#pragma unroll
  for (int k = 0; k < XK; ++k) xrow[k] = data_row_nb(a, base, min(r0 + xr0 + k, a.B - 1));
  const int64_t crow = data_row_nb(a, base, 0);
  rep_sum<NTH, 2 * H1>(T.gg1, BNG, smem + L::rsc, smem + L::rst);  // gg1|gbe1 are adjacent in a replica
  {
    const float* rst = smem + L::rst;
    if (threadIdx.x < H1) {
      const int c = threadIdx.x;
      c1[c] = f1inv * g1v;
      c1[H1 + c] = rst[H1 + c] * invB;
      c1[2 * H1 + c] = rst[c] * invB;
      c1[3 * H1 + c] = f1mean;
      c1[4 * H1 + c] = f1inv;
    } else if (threadIdx.x < H1 + H0) {
      const int c = threadIdx.x - H1;
      c0[c] = f0mean;
      c0[H0 + c] = f0inv * g0v;
      c0[2 * H0 + c] = be0v;
      c0[3 * H0 + c] = f0inv;
    }
  }
  put_planes4(hs + L::W4i + w4r * H1 + ((w4c ^ swz_dz(w4r)) * 4), L::PW4, w4v);
  __syncthreads();
  TT_STAMP(3, 1);
  TT_STAMP_T(4, 1, 448);
  TT_SUBSTAMP(6, 0);

  // ---- phase 1: X' gather issued (used in phase 3: its latency hides
  // behind this phase's arithmetic), dZ4, A0 / Zh0 recompute
  // (VEC a template argument: a load under a run-time branch would make hipcc
  // wait for it at the join, exposing the gather here)
  const int n4 = VEC ? (T.n_num >> 2) : 0;
  const int xcl = min(xc, max(n4 - 1, 0));
  float4 xv[XK], cv;
  if constexpr (VEC) {
#pragma unroll
    for (int k = 0; k < XK; ++k) xv[k] = *reinterpret_cast<const float4*>(T.num + xrow[k] * T.num_ld + 4 * xcl);
    cv = *reinterpret_cast<const float4*>(T.num + crow * T.num_ld + 4 * xcl);
  } else {
    const int nn = T.n_num;
    auto ld1 = [&](int64_t drow, int col) { return T.num[drow * T.num_ld + min(col, nn - 1)]; };
#pragma unroll
    for (int k = 0; k < XK; ++k)
      xv[k] = make_float4(ld1(xrow[k], 4 * xc), ld1(xrow[k], 4 * xc + 1), ld1(xrow[k], 4 * xc + 2),
                          ld1(xrow[k], 4 * xc + 3));
    cv = make_float4(ld1(crow, 4 * xc), ld1(crow, 4 * xc + 1), ld1(crow, 4 * xc + 2), ld1(crow, 4 * xc + 3));
  }
  TT_SUBSTAMP(6, 1);

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
    {  // dZ4 image: quad transpose -> row 16w + 4g + (r & 3), columns 16q + (r & ~3) .. +3
      const f32x4 tq = quad_transpose(dz[q]);
      const int zr = 16 * w + 4 * g + (r & 3), zc = 4 * q + (r >> 2);
      put_planes4(hs + L::dZi + zr * H1 + ((zc ^ swz_dz(zr)) * 4), L::PZ, make_float4(tq[0], tq[1], tq[2], tq[3]));
    }
    const float cb = col_reduce(dz[q][0] + dz[q][1] + dz[q][2] + dz[q][3]);
    if (g == 0) db4[w * H1 + col] = cb;
  }
  TT_SUBSTAMP(6, 2);
  const bool drop = a.drop_thr > 0;
  const uint64_t key = dropout_key(a.seed, (uint64_t)step, t, 0);
  f32x4 a0[4], zh0[4];
  uint32_t rk[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) rk[i] = dropout_row_key(key, r0 + 16 * w + 4 * g + i);
  // straight-line A0 / Zh0 (bn_relu_drop's arithmetic, bitwise): the four
  // columns' BN0 coefficients read once, all issued before use; the dropout
  // keep bits of columns c and c + 32 (j and j + 2) come from one hash
  // (DROP_HB0 = 5), computed under one uniform branch -- per-element calls
  // compiled to a branch and an lgkmcnt(0) wait per element
  float cmu[4], cal[4], cbe[4], cin[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
    cmu[j] = c0[col];
    cal[j] = c0[H0 + col];
    cbe[j] = c0[2 * H0 + col];
    cin[j] = c0[3 * H0 + col];
  }
  const float dscl = drop ? a.drop_scale : 1.f;
  uint32_t kb = 0xFFFFu;  // bit 4 j + i: element (row i, column 16 j + r) kept
  if (drop) {
    kb = 0u;
#pragma unroll
    for (int jp = 0; jp < 2; ++jp)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t h = perm32(rk[i] ^ ((uint32_t)(16 * jp + r) * 0x9E3779B9u));
        kb |= ((h & 0xFFFFu) >= a.drop_thr ? 1u : 0u) << (4 * jp + i);
        kb |= ((h >> 16) >= a.drop_thr ? 1u : 0u) << (4 * (jp + 2) + i);
      }
  }
  TT_SUBSTAMP(6, 3);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = 16 * j + r;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int64_t row = r0 + 16 * w + 4 * g + i;
      const float z = zz0[j][i];
      const bool ok = row < a.B;
      float y = (z - cmu[j]) * cal[j] + cbe[j];
      y = y > 0.f ? y : 0.f;
      y = ((kb >> (4 * j + i)) & 1u) ? y * dscl : 0.f;  // dscl = 1 without dropout: y * 1 == y
      a0[j][i] = ok ? y : 0.f;
      zh0[j][i] = ok ? (z - cmu[j]) * cin[j] : 0.f;
    }
    put_planes4(hs + L::A0i + fold_at(col, 16 * w + 4 * g), L::PL, make_float4(a0[j][0], a0[j][1], a0[j][2], a0[j][3]));
  }
  TT_SUBSTAMP(6, 4);
  __syncthreads();
  TT_STAMP(3, 2);
  TT_STAMP_T(4, 2, 448);
  TT_SUBSTAMP(6, 5);

  // ---- phase 2: dW4 = dZ4^T A0 (wave w: h1-tile w & 1, h0-tile w >> 1),
  // dA0 = dZ4 W4 on the wave's rows -> dY0, BN0-backward column partials
  // (bf16x3: dZ4 read transposed as the A operand of dW4, K = the tile's rows)
  float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
  {
    const int p = w & 1, q = w >> 1;
    const int qd = (l & 15) >> 2, pc = l & 3;
    f32x4 acc = zero4();
#pragma unroll
    for (int kk = 0; kk < R / 32; ++kk) {
      const int ra = 32 * kk + 8 * g + qd, rb = ra + 4;
      bf16x8 af[3], bf[3];
#pragma unroll
      for (int p3 = 0; p3 < 3; ++p3) {
        const uint16_t* zb = hs + L::dZi + p3 * L::PZ;
        af[p3] = tr_frag(zb + ra * H1 + (((4 * p + pc) ^ swz_dz(ra)) * 4), zb + rb * H1 + (((4 * p + pc) ^ swz_dz(rb)) * 4));
        bf[p3] = *reinterpret_cast<const bf16x8*>(hs + L::A0i + p3 * L::PL + fold_at(16 * q + r, 32 * kk + 8 * g));
      }
      mfma_x3(af, bf, acc);
    }
    store_tile_rm_wt(slab, (int)T.so_W4 + 16 * p * H0 + 16 * q, H0, acc);
  }
  // dA0 = dZ4 W4 on the wave's rows (one 32-deep K step per h0 tile)
  f32x4 dA[4];
  {
    bf16x8 af[3];
    const int ar = 16 * w + r;
#pragma unroll
    for (int p3 = 0; p3 < 3; ++p3)
      af[p3] = *reinterpret_cast<const bf16x8*>(hs + L::dZi + p3 * L::PZ + ar * H1 + (((2 * g) ^ swz_dz(ar)) * 4));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int wr = 16 * j + r;
      bf16x8 bw[3];
#pragma unroll
      for (int p3 = 0; p3 < 3; ++p3)
        bw[p3] = *reinterpret_cast<const bf16x8*>(hs + L::W4i + p3 * L::PW4 + wr * H1 + (((2 * g) ^ swz_dz(wr)) * 4));
      dA[j] = zero4();
      mfma_x3(af, bw, dA[j]);
    }
  }
  TT_STAMP(3, 3);
  TT_STAMP_T(4, 3, 448);
  const float scl = drop ? a.drop_scale : 1.f;
  float sg[4], sb[4], sz[4];
  f32x4 dyt[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    sg[j] = 0.f;
    sb[j] = 0.f;
    sz[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float dy = a0[j][i] > 0.f ? dA[j][i] * scl : 0.f;  // 0 on rows >= B (a0 = 0)
      dyt[j][i] = dy;
      sg[j] += dy * zh0[j][i];
      sb[j] += dy;
      sz[j] += zh0[j][i];
    }
  }
  // X' image (clear of W4s|dZT|A0T) and its column sums while the GEMMs above drain
  const bool cok = xc < ((T.n_num + 3) >> 2);
  {
    // X' = X - c on valid rows and columns, 0 elsewhere; column partial sums
    float d[XK][4];
#pragma unroll
    for (int k = 0; k < XK; ++k) {
      const bool ok = cok && r0 + xr0 + k < a.B;
      const float x4[4] = {xv[k].x, xv[k].y, xv[k].z, xv[k].w}, c4[4] = {cv.x, cv.y, cv.z, cv.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bool ci = VEC || 4 * xc + i < T.n_num;  // ragged last group of an unaligned width
        d[k][i] = (ok && ci) ? x4[i] - c4[i] : 0.f;
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 4 * xc + i;
      put_planes4(hs + L::IX + fold_at(c, xr0), L::PL, make_float4(d[0][i], d[1][i], d[2][i], d[3][i]));
    }
    // lanes xc, xc + 16, xc + 32, xc + 48 share a column group
    float sx[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) sx[i] = col_reduce(d[0][i] + d[1][i] + d[2][i] + d[3][i]);
    if (g == 0) {
      float* rs = red + w * 4 * H0 + 3 * H0 + 4 * xc;
#pragma unroll
      for (int i = 0; i < 4; ++i) rs[i] = sx[i];
    }
  }
  TT_STAMP(3, 4);
  TT_STAMP_T(4, 4, 448);
  cols_to_lds<4>(sg, red, 4 * H0);
  cols_to_lds<4>(sb, red + H0, 4 * H0);
  cols_to_lds<4>(sz, red + 2 * H0, 4 * H0);
  __syncthreads();  // every wave is past dW4 and dA0 (A0, dZ4, W4^T images)
  TT_STAMP(3, 5);
  TT_STAMP_T(4, 5, 448);

  // ---- phase 3: bf16x3 images of dY0, Zh0 (from the accumulator layout:
  // channel 16j + r, rows 16w + 4g .. +3) over the dead f32 region (X'
  // went in during phase 2: columns 4xc .. +3 of rows xr0 .. +3)
  {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = 16 * j + r, o = fold_at(c, 16 * w + 4 * g);
      put_planes4(hs + L::IY + o, L::PL, make_float4(dyt[j][0], dyt[j][1], dyt[j][2], dyt[j][3]));
      put_planes4(hs + L::IZ + o, L::PL, make_float4(zh0[j][0], zh0[j][1], zh0[j][2], zh0[j][3]));
    }
    if (blockIdx.x == 0) {  // inv0 * gamma0 and the shift row for k_reduce_adam
      if (threadIdx.x < H0) T.k0s[threadIdx.x] = c0[H0 + threadIdx.x];
      if (threadIdx.x < 16) {
        float4 c = cv;
        if (!cok) c = make_float4(0.f, 0.f, 0.f, 0.f);
        *reinterpret_cast<float4*>(T.xsh + 4 * xc) = c;
      }
    }
  }
  __syncthreads();
  TT_STAMP(3, 6);
  TT_STAMP_T(4, 6, 448);
  TT_SUBSTAMP(7, 0);

  // ---- phase 4: P | Q = [dY0 | Zh0]^T X' over the tile's rows (bf16x3,
  // K = rows in 32-row steps): wave w owns channels 16 (w & 3) .. +15 of P
  // (w < 4) or Q, every column tile.  Slab layout [64][kp/16][P 16 | Q 16]:
  // k_reduce_adam's lanes for 16 columns of P and the same 16 of Q read one
  // contiguous 128 B
  {
    const uint16_t* Ai = hs + (w < 4 ? L::IY : L::IZ);
    const uint16_t* Bi = hs + L::IX;
    const int kp = T.kp, KT = kp / 16;
    const int ca = 16 * (w & 3) + r;
    const int so = (int)T.so_W0 + 16 * (w & 3) * 2 * kp + (w < 4 ? 0 : 16);
    f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
    // all four column tiles every time (X' columns >= the input width are
    // zero in the image; tiles j >= kp / 16 are not stored): a branch-free
    // loop whose next K step's reads are pinned above this step's 24 MFMAs
    // (four interleaved accumulation chains)
    bf16x8 af[2][3], bf[2][4][3];
    auto ldk = [&](int kk, bf16x8 (&a_)[3], bf16x8 (&b_)[4][3]) {
      const int k0 = 32 * kk + 8 * g;
#pragma unroll
      for (int p = 0; p < 3; ++p) {
        a_[p] = *reinterpret_cast<const bf16x8*>(Ai + p * L::PL + fold_at(ca, k0));
#pragma unroll
        for (int j = 0; j < 4; ++j) b_[j][p] = *reinterpret_cast<const bf16x8*>(Bi + p * L::PL + fold_at(16 * j + r, k0));
      }
    };
    ldk(0, af[0], bf[0]);
#pragma unroll
    for (int kk = 0; kk < R / 32; ++kk) {
      if (kk + 1 < R / 32) ldk(kk + 1, af[(kk + 1) & 1], bf[(kk + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = mfma_bf16(af[kk & 1][PA[q]], bf[kk & 1][j][PB[q]], acc[j]);
      __builtin_amdgcn_sched_barrier(0);
    }
    TT_SUBSTAMP(7, 1);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < KT) store_tile_rm_wt(slab, so + 32 * j, 2 * kp, acc[j]);
  }
  TT_SUBSTAMP(7, 2);
  static_assert(FRW == 4 * H0, "fold replica: gamma0 grad | beta0 grad | sum Zh0 | sum X'");
  if (threadIdx.x < 4 * H0)
    xblock_add(a.det, T.fr, FRW, T.dslot, FRW, threadIdx.x, wave_rows_sum<8>(red, 4 * H0, threadIdx.x));
  TT_SUBSTAMP(7, 3);
  if (threadIdx.x < H1) slab[T.so_b4 + threadIdx.x] = wave_rows_sum<8>(db4, H1, threadIdx.x);
  TT_SUBSTAMP(7, 4);
  TT_STAMP(3, 7);
  TT_STAMP_T(4, 7, 448);
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
    return sizeof(float) * (xt_floats(kp) + (size_t)H0 * LDT + 4 * H0 + 5 * H0 + 2 * R + 4 * R + 2 * H0);
  }
};

template <int R>
__global__ __launch_bounds__(R * 4) void k_bwd_first(StepArgs a) {
  static_assert(R == 64 || R == 32, "4 (or 2) waves of 16 rows");
  constexpr int NTH = R * 4, NW = R / 16;
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
  float* db0 = dZT + H0 * LDT;                         // [4 waves][64]
  float* c0 = db0 + 4 * H0;                            // k0[64] mb[64] mg[64] mean0[64] inv0[64]
  float* rsc = c0 + 5 * H0;                            // [NTH] replica-sum scratch
  float* rst = rsc + NTH;                              // [2*64] sum dgamma0 | sum dbeta0
  TT_STAMP(4, 0);

  // Phase 0 issues every load before its first wait: this tile's dataset
  // rows (first: the X gather after the barrier depends on them), the dY0 /
  // Z0 tiles, BN0's inputs (every thread, clamped column: no branch) and the
  // replica loads inside rep_sum; the row indices reach LDS after rep_sum's
  // wait (a store right after their load would wait for the tiles too).
  const int64_t my_row = data_row_nb(a, base, min(r0 + (int64_t)(threadIdx.x % R), a.B - 1));
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
  const int cc = (int)threadIdx.x % H0;
  const float f0inv = T.fin0[H0 + cc], f0mean = T.fin0[cc], g0v = T.g0[cc];
  const float invB = 1.f / (float)a.B;
  rep_sum<NTH, 2 * H0>(T.gg0, BNG, rsc, rst);  // gg0|gbe0 are adjacent in a replica
  if (threadIdx.x < R) ridx[threadIdx.x] = my_row;
  if (threadIdx.x < H0) {
    const int c = threadIdx.x;
    c0[c] = f0inv * g0v;
    c0[H0 + c] = a.train ? rst[H0 + c] * invB : 0.f;  // eval: BN is affine, no batch-mean terms
    c0[2 * H0 + c] = a.train ? rst[c] * invB : 0.f;
    c0[3 * H0 + c] = f0mean;
    c0[4 * H0 + c] = f0inv;
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
    if (g == 0) db0[w * H0 + col] = cb;
  }
  __syncthreads();
  TT_STAMP(4, 2);

  // dW0 = dZ0^T X over the tile's rows: wave w owns outputs 16w..16w+15 and
  // every input column tile; results go straight into this tile's slab
  float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
  const int in = T.in_dim;
  const bool w0_vec = (in & 3) == 0 && (T.so_W0 & 3) == 0;
  // wave w owns outputs 16 wo .. 16 wo + 15 for wo = w, w + NW, ...
  auto put_w0 = [&](int wo, int kt, const f32x4& acc) {
    const int k = 16 * kt + r;
    float* dst = slab + T.so_W0 + (16 * wo + 4 * g) * in + k;
    if (w0_vec && 16 * kt + 16 <= in) {  // whole tile: row-major 16-B write-through stores
      store_tile_rm_wt(slab, (int)T.so_W0 + 16 * wo * in + 16 * kt, in, acc);
    } else if (16 * kt + 16 <= in) {
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[i * in] = acc[i];
    } else if (k < in) {
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[i * in] = acc[i];
    }
  };
#pragma unroll
  for (int wo = w; wo < 4; wo += NW) {
    int kt = 0;
    for (; kt + 4 <= KT; kt += 4) {
      f32x4 acc[4] = {zero4(), zero4(), zero4(), zero4()};
      strip_gemm_nt<4>(dZT + 16 * wo * LDT, LDT, XT + 16 * kt * LDT, LDT, R, acc);
#pragma unroll
      for (int q = 0; q < 4; ++q) put_w0(wo, kt + q, acc[q]);
    }
    for (; kt < KT; ++kt) {
      f32x4 acc[1] = {zero4()};
      strip_gemm_nt<1>(dZT + 16 * wo * LDT, LDT, XT + 16 * kt * LDT, LDT, R, acc);
      put_w0(wo, kt, acc[0]);
    }
  }
  float* dxn = T.dxn;
  if (emb || dxn) {
    // dX = dZ0 W0: the embedding columns are scatter-added into the tables,
    // the numeric columns (when the caller asked for input gradients,
    // model.py:67 f_numeric / c_numeric.grad) stored row-major [B, n_num].
    // W0 (row-major [64][ldk]) takes over the X^T image's LDS.
    __syncthreads();
    float* W0s = XT;
    stage_w<NTH>(T.W0, H0, T.in_dim, kp, W0s, ldk);
    __syncthreads();
    for (int ktt = dxn ? 0 : T.n_num / 16; ktt < KT; ++ktt) {
      f32x4 dx[1] = {zero4()};
      strip_gemm_tn<1>(dZT + 16 * w, LDT, W0s + 16 * ktt, ldk, H0, dx);
      const int col = 16 * ktt + r;
      if (col < T.n_num) {
        if (dxn) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int64_t row = r0 + 16 * w + 4 * g + i;
            if (row < a.B) dxn[row * T.n_num + col] = dx[0][i];
          }
        }
      } else if (col < T.in_dim) {
        const int c = col - T.n_num;
        const int jj = c / T.emb_dim, e = c - jj * T.emb_dim;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int rl = 16 * w + 4 * g + i;
          if (r0 + rl >= a.B) continue;
          if (a.det) {  // deterministic: the row's dX, scattered in row order by k_det_scatter
            T.demb[(r0 + rl) * T.emb_w + c] = dx[0][i];
            continue;
          }
          int64_t code = T.cat[ridx[rl] * T.cat_ld + jj];
          code = code < 0 ? 0 : (code >= T.emb_rows[jj] ? T.emb_rows[jj] - 1 : code);
          atomicAdd(T.gemb[jj] + code * T.emb_dim + e, dx[0][i]);
        }
      }
    }
  }
  if (threadIdx.x < H0) slab[T.so_b0 + threadIdx.x] = wave_rows_sum<NW>(db0, H0, threadIdx.x);
  TT_STAMP(4, 3);
}

#define TT_L0(KS) template __global__ void k_l0_fwd<64, KS, true, false>(StepArgs, LateRed); \
  template __global__ void k_l0_fwd<64, KS, false, false>(StepArgs, LateRed);
TT_L0(1)
TT_L0(2)
TT_L0(4)
TT_L0(8)
#undef TT_L0
#define TT_L0(KS) template __global__ void k_l0_fwd<32, KS, true, false>(StepArgs, LateRed); \
  template __global__ void k_l0_fwd<32, KS, false, false>(StepArgs, LateRed);
TT_L0(1)
TT_L0(2)
TT_L0(4)
TT_L0(8)
#undef TT_L0
template __global__ void k_l0_fwd<64, 1, true, true>(StepArgs, LateRed);
template __global__ void k_l0_fwd<64, 2, true, true>(StepArgs, LateRed);
template __global__ void k_l4_fwd<64>(StepArgs);
template __global__ void k_l4_fwd<32>(StepArgs);
template __global__ void k_top_pair<4, 64>(StepArgs);
template __global__ void k_top_pair<8, 64>(StepArgs);
template __global__ void k_top_pair<4, 32>(StepArgs);
template __global__ void k_top_pair<8, 32>(StepArgs);
template __global__ void k_top<4, 64, false>(StepArgs);
template __global__ void k_top<8, 64, false>(StepArgs);
template __global__ void k_top<4, 128, false>(StepArgs);
template __global__ void k_top<8, 128, false>(StepArgs);
template __global__ void k_top<4, 64, true>(StepArgs);
template __global__ void k_top<8, 64, true>(StepArgs);
template __global__ void k_top<4, 128, true>(StepArgs);
template __global__ void k_top<8, 128, true>(StepArgs);
template __global__ void k_bwd_mid<64>(StepArgs);
template __global__ void k_bwd_mid<32>(StepArgs);
template __global__ void k_bwd_mid_fold<128, true>(StepArgs);
template __global__ void k_bwd_mid_fold<128, false>(StepArgs);
template __global__ void k_bwd_first<64>(StepArgs);
template __global__ void k_bwd_first<32>(StepArgs);

}  // namespace tt
