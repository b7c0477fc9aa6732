// Generic top of the towers for LATENT in (128, 512] (gfx950).
//
// The fused k_top / k_top_pair keep both towers' W8 images and a tile's U / V
// rows in LDS, which fits LATENT <= 128.  Wider latent spaces (the
// reference accepts any config.LATENT_DIM, model.py:46,61; the contrastive
// configurations project 256- / 512-wide embeddings, SURVEY 8d cfg 5) run
// the top of the step as three kernels over U / V / dU / dV kept in the
// workspace ([tower][Bpad][Dp] fp32, Dp = LATENT rounded up to 16, padding
// columns zero), products on the exact fp32 MFMA (v_mfma_f32_16x16x4_f32):
//
//   k_top_gen_fwd : A1 = drop(relu(BN1(Z4))) of a 64-row tile of one tower
//                   (BN1 coefficients from the batch moments or the running
//                   statistics; the train forward folds the batch moments
//                   into the running estimates), U = A1 W8^T + b8
//                   model.py:43-46 (firm), :57-61 (ceo)
//   k_cos_gen     : score = exp(ls) <U/|U|, V/|V|> (model.py:79-87); train:
//                   weighted MSE (training.py:52) into the loss replicas,
//                   dL/dlogit_scale, and the closed-form dU, dV;
//                   backward of a given dscore the same without the loss
//   k_top_gen_bwd : dW8 / db8 partials of the tile, dA1 = dU W8,
//                   dY1 = dA1 * [A1 > 0] * dropout scale, dgamma1 / dbeta1
//
// Everything after dY1 (k_bwd_mid*, k_bwd_first, k_reduce_adam) is shared
// with the fused path: the W8 | b8 slab range is [D][32] | [D] for any D.
#include "tt_common.h"

namespace tt {

constexpr int GEN_MAX_D = 512;
constexpr int GEN_R = 64;            // rows per tile (4 waves x 16)
constexpr int GEN_NTH = 256;
constexpr int GEN_LDH = H1 + 4;      // A1 / W8 rows in LDS (floats)
constexpr int GEN_DC = 128;          // latent columns per backward chunk
constexpr int GEN_LDU = GEN_DC + 4;  // dU chunk row stride

__host__ __device__ constexpr int gen_dp(int D) { return (D + 15) / 16 * 16; }

// LDS of k_top_gen_fwd: W8 [Dp][36] | A1 [64][36] | BN1 coefficients | replica scratch
__host__ __device__ constexpr size_t gen_fwd_lds(int D) {
  return sizeof(float) * ((size_t)gen_dp(D) * GEN_LDH + GEN_R * GEN_LDH + 4 * H1 + GEN_NTH + 2 * H1);
}
// LDS of k_top_gen_bwd: W8^T [32][Dp + 4] | A1 [64][36] | dU chunk [64][132] |
// BN1 coefficients | per-wave BN partials [4][64] | replica scratch
__host__ __device__ constexpr size_t gen_bwd_lds(int D) {
  return sizeof(float) * ((size_t)H1 * (gen_dp(D) + 4) + GEN_R * GEN_LDH + GEN_R * GEN_LDU + 4 * H1 + 4 * 2 * H1 +
                          GEN_NTH + 2 * H1);
}

// BN1 coefficients of tower t into cf[mean | gamma*inv | beta | inv] (threads < H1):
// train: the batch moments' replica sums (st1; k_l4_fwd), with the running
// statistics updated by block 0 when `update`; eval: the running statistics.
__device__ __forceinline__ void gen_bn1_coefs(const StepArgs& a, const TowerDev& T, bool update, float* scratch,
                                              float* rst, float* cf) {
  if (a.train) rep_sum<GEN_NTH, 2 * H1>(T.st1, ST1S, scratch, rst);
  if (threadIdx.x < H1) {
    const int c = threadIdx.x;
    const bool have_rs = T.rm1 != nullptr;
    float mean, inv;
    bn_coefs_pre(a, H1, rst, T.shift1[c], have_rs ? T.rm1[c] : 0.f, have_rs ? T.rv1[c] : 1.f, T.rm1, T.rv1, T.nbt1,
                 T.fin1, update && blockIdx.x == 0, c, &mean, &inv);
    cf[c] = mean;
    cf[H1 + c] = inv * T.g1[c];
    cf[2 * H1 + c] = T.be1[c];
    cf[3 * H1 + c] = inv;
  }
  __syncthreads();
}

// A1 of the tile (row-major [64][36] in LDS) from Z4; z4h (nullable) gets the
// normalised Z4 (BN1 backward) in the same layout
__device__ __forceinline__ void gen_a1(const StepArgs& a, const TowerDev& T, int t, int64_t step, int64_t r0,
                                       const float* cf, float* A1s, float* z4h) {
  const bool drop = a.train && a.drop_thr > 0;
  const uint64_t key = dropout_key(a.seed, (uint64_t)step, t, 1);
  // 64 rows x 32 columns = 512 float4, two per thread
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = threadIdx.x + k * GEN_NTH;
    const int rl = e >> 3, c4 = (e & 7) * 4;
    const float4 z = *reinterpret_cast<const float4*>(T.Z4 + (r0 + rl) * H1 + c4);
    const uint32_t rk = dropout_row_key(key, r0 + rl);
    const float zz[4] = {z.x, z.y, z.z, z.w};
    float y[4], zh[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = c4 + q;
      zh[q] = (zz[q] - cf[c]) * cf[3 * H1 + c];
      float v = (zz[q] - cf[c]) * cf[H1 + c] + cf[2 * H1 + c];
      v = v > 0.f ? v : 0.f;
      if (drop) v = dropout_keep_rk<DROP_HB1>(rk, c, a.drop_thr) ? v * a.drop_scale : 0.f;
      y[q] = v;
    }
    *reinterpret_cast<float4*>(A1s + rl * GEN_LDH + c4) = make_float4(y[0], y[1], y[2], y[3]);
    if (z4h) *reinterpret_cast<float4*>(z4h + rl * GEN_LDH + c4) = make_float4(zh[0], zh[1], zh[2], zh[3]);
  }
}

// ---------------------------------------------------------------------------
// k_top_gen_fwd : grid (tiles, 2 towers)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(GEN_NTH) void k_top_gen_fwd(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int D = a.D, Dp = gen_dp(D);
  const int64_t step = step_current(a);
  const int64_t r0 = (int64_t)blockIdx.x * GEN_R;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  float* W8s = smem;                     // [Dp][36]
  float* A1s = W8s + Dp * GEN_LDH;       // [64][36]
  float* cf = A1s + GEN_R * GEN_LDH;     // [4][32]
  float* scr = cf + 4 * H1;              // [256]
  float* rst = scr + GEN_NTH;            // [64]
  // W8 [D][32] row-major (rows >= D zero)
  for (int e = threadIdx.x; e < Dp * (H1 / 4); e += GEN_NTH) {
    const int d = e >> 3, c4 = (e & 7) * 4;
    const float4 v = d < D ? *reinterpret_cast<const float4*>(T.W8 + d * H1 + c4) : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(W8s + d * GEN_LDH + c4) = v;
  }
  gen_bn1_coefs(a, T, a.update_stats != 0, scr, rst, cf);
  gen_a1(a, T, t, step, r0, cf, A1s, nullptr);
  __syncthreads();
  // U[16 rows of wave w][Dp] = A1 W8^T + b8, 8 latent tiles at a time
  const bool emb = a.mode == TOP_EMB_FWD;
  for (int j0 = 0; j0 < Dp / 16; j0 += 8) {
    f32x4 acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = zero4();
    const int nt = min(8, Dp / 16 - j0);
    if (nt == 8) {
      strip_gemm_nt<8>(A1s + 16 * w * GEN_LDH, GEN_LDH, W8s + 16 * j0 * GEN_LDH, GEN_LDH, H1, acc);
    } else {
      for (int j = 0; j < nt; ++j) {
        f32x4 a1[1] = {zero4()};
        strip_gemm_nt<1>(A1s + 16 * w * GEN_LDH, GEN_LDH, W8s + 16 * (j0 + j) * GEN_LDH, GEN_LDH, H1, a1);
        acc[j] = a1[0];
      }
    }
    for (int j = 0; j < nt; ++j) {
      const int d = 16 * (j0 + j) + r;
      const float bias = d < D ? T.b8[d] : 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int64_t row = r0 + 16 * w + 4 * g + i;
        const float u = acc[j][i] + bias;
        if (emb) {
          if (row < a.B && d < D) a.emb[((int64_t)t * a.B + row) * D + d] = u;
        } else {
          T.ug[row * Dp + d] = d < D ? u : 0.f;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// k_cos_gen : 64 rows per block, one row per 16-lane group at a time
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(GEN_NTH) void k_cos_gen(StepArgs a) {
  __shared__ float part[GEN_NTH / 16][2];  // per 16-lane group: (dls, loss) partial
  const int D = a.D, Dp = gen_dp(D);
  const int l = lane_id(), r = l & 15, grp = (int)threadIdx.x >> 4;
  const float s = expf(*a.logit_scale);
  const bool bwd = a.mode != TOP_FWD;
  float dls_p = 0.f, loss_p = 0.f;
  constexpr int NK = GEN_MAX_D / 16;
  for (int q = 0; q < GEN_R / (GEN_NTH / 16); ++q) {
    const int64_t row = (int64_t)blockIdx.x * GEN_R + q * (GEN_NTH / 16) + grp;
    const float* U = a.tw[0].ug + row * Dp;
    const float* V = a.tw[1].ug + row * Dp;
    float u[NK], v[NK];
    float uv = 0.f, uu = 0.f, vv = 0.f;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int d = r + 16 * k;
      u[k] = d < Dp ? U[d] : 0.f;
      v[k] = d < Dp ? V[d] : 0.f;
      uv += u[k] * v[k];
      uu += u[k] * u[k];
      vv += v[k] * v[k];
    }
    uv = row_reduce16(uv);
    uu = row_reduce16(uu);
    vv = row_reduce16(vv);
    const float ino = __builtin_amdgcn_rsqf(uu), inv = __builtin_amdgcn_rsqf(vv);
    const float cs = uv * ino * inv, sc = cs * s;
    const bool valid = row < a.B;
    if (a.score && valid && r == 0) a.score[row] = sc;
    if (!bwd) continue;
    float ds = 0.f;
    if (a.mode == TOP_TRAIN) {
      const float tg = a.tgw[2 * row], wt = a.tgw[2 * row + 1];
      const float diff = sc - tg;
      ds = 2.f * diff * (wt * (1.f / (float)a.B));
      if (valid && r == 0) loss_p += wt * diff * diff;
    } else {
      ds = a.dscore[valid ? row : 0];
    }
    ds = valid ? ds : 0.f;
    if (r == 0) dls_p += ds * sc;
    const float dc = ds * s;
    const float ka = dc * ino * inv, kbu = dc * cs * ino * ino, kbv = dc * cs * inv * inv;
    float* dU = a.tw[0].dug + row * Dp;
    float* dV = a.tw[1].dug + row * Dp;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const int d = r + 16 * k;
      if (d < Dp) {
        dU[d] = ka * v[k] - kbu * u[k];
        dV[d] = ka * u[k] - kbv * v[k];
      }
    }
  }
  if (!bwd) return;
  if (r == 0) {
    part[grp][0] = dls_p;
    part[grp][1] = loss_p;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    const int c = threadIdx.x;  // 0: dL/dlogit_scale, 1: batch-mean loss
    float v = 0.f;
    for (int k = 0; k < GEN_NTH / 16; ++k) v += part[k][c];
    if (c == 1) v = a.mode == TOP_TRAIN ? v / (float)a.B : 0.f;
    if (c == 0 || a.mode == TOP_TRAIN || a.det) xblock_add(a.det, a.lsr, LSR, a.dslot_lsr, 2, c, v);
  }
}

// ---------------------------------------------------------------------------
// k_top_gen_bwd : grid (tiles, 2 towers)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(GEN_NTH) void k_top_gen_bwd(StepArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int t = blockIdx.y;
  const TowerDev& T = a.tw[t];
  const int D = a.D, Dp = gen_dp(D), LDT = Dp + 4;
  const int64_t step = step_current(a);
  const int64_t r0 = (int64_t)blockIdx.x * GEN_R;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  float* W8T = smem;                     // [32][Dp + 4]  W8^T
  float* A1s = W8T + H1 * LDT;           // [64][36]  (then dY1 Zh1 products reuse nothing)
  float* dUs = A1s + GEN_R * GEN_LDH;    // [64][132] dU chunk
  float* cf = dUs + GEN_R * GEN_LDU;     // [4][32]
  float* red = cf + 4 * H1;              // [4 waves][64] dgamma1 | dbeta1 partials
  float* scr = red + 4 * 2 * H1;         // [256]
  float* rst = scr + GEN_NTH;            // [64]
  for (int e = threadIdx.x; e < Dp * H1; e += GEN_NTH) {
    const int d = e / H1, h = e - d * H1;
    W8T[h * LDT + d] = d < D ? T.W8[d * H1 + h] : 0.f;
  }
  gen_bn1_coefs(a, T, false, scr, rst, cf);
  gen_a1(a, T, t, step, r0, cf, A1s, nullptr);
  float* slab = T.slab + (int64_t)blockIdx.x * a.slab_ld;
  const bool emb = a.mode == TOP_EMB_BWD;
  f32x4 dA[2] = {zero4(), zero4()};
  for (int d0 = 0; d0 < Dp; d0 += GEN_DC) {
    const int dc = min(GEN_DC, Dp - d0);
    __syncthreads();  // the previous chunk's readers are done (and A1 / W8^T complete)
    for (int e = threadIdx.x; e < GEN_R * GEN_DC; e += GEN_NTH) {
      const int rl = e / GEN_DC, c = e - rl * GEN_DC;
      const int64_t row = r0 + rl;
      const int d = d0 + c;
      float v = 0.f;
      if (c < dc) {
        if (emb)
          v = (row < a.B && d < D) ? a.demb[((int64_t)t * a.B + row) * D + d] : 0.f;
        else
          v = T.dug[row * Dp + d];
      }
      dUs[rl * GEN_LDU + c] = v;
    }
    __syncthreads();
    // dA1 += dU[rows of wave w][chunk] W8[chunk][32]   (B = W8^T rows h, k = d)
    for (int k0 = 0; k0 < dc; k0 += 16) {
      f32x4 tmp[2] = {zero4(), zero4()};
      strip_gemm_nt<2>(dUs + 16 * w * GEN_LDU + k0, GEN_LDU, W8T + d0 + k0, LDT, 16, tmp);
      dA[0] += tmp[0];
      dA[1] += tmp[1];
    }
    // dW8^T[h][d] = sum_rows A1[row][h] dU[row][d]: wave w owns h tile (w & 1)
    // and the chunk's latent tiles of parity (w >> 1)
    const int ht = w & 1;
    for (int dt = (w >> 1); dt < dc / 16; dt += 2) {
      f32x4 acc[1] = {zero4()};
      strip_gemm_tn<1>(A1s + 16 * ht, GEN_LDH, dUs + 16 * dt, GEN_LDU, GEN_R, acc);
      // lane (r, g): h = 16 ht + 4g + i, d = d0 + 16 dt + r -> slab W8 [d][32]
      const int d = d0 + 16 * dt + r;
      if (d < D)
        *reinterpret_cast<f32x4*>(slab + T.so_W8 + (int64_t)d * H1 + 16 * ht + 4 * g) = acc[0];
    }
    // db8[d] = sum_rows dU[row][d]
    if ((int)threadIdx.x < dc) {
      const int c = threadIdx.x;
      float sum = 0.f;
      for (int rl = 0; rl < GEN_R; ++rl) sum += dUs[rl * GEN_LDU + c];
      if (d0 + c < D) slab[T.so_b8 + d0 + c] = sum;
    }
  }
  // dY1 = dA1 * [A1 > 0] * scale; BN1 partials sum dY1 * Zh1, sum dY1
  const float scl = (a.train && a.drop_thr > 0) ? a.drop_scale : 1.f;
  float sg[2], sb[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int c = 16 * j + r;
    sg[j] = 0.f;
    sb[j] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = 16 * w + 4 * g + i;
      const int64_t row = r0 + rl;
      const float a1 = A1s[rl * GEN_LDH + c];
      const float dy = a1 > 0.f ? dA[j][i] * scl : 0.f;  // 0 on rows >= B (dU = 0)
      const float zh = (T.Z4[row * H1 + c] - cf[c]) * cf[3 * H1 + c];
      T.dY1[row * H1 + c] = dy;
      sg[j] += dy * zh;
      sb[j] += dy;
    }
  }
  cols_to_lds<2>(sg, red, 2 * H1);
  cols_to_lds<2>(sb, red + H1, 2 * H1);
  __syncthreads();
  if (threadIdx.x < 2 * H1)
    xblock_add(a.det, T.gg1, BNG, T.dslot, 2 * H1, threadIdx.x, wave_rows_sum<4>(red, 2 * H1, threadIdx.x));
}

}  // namespace tt
