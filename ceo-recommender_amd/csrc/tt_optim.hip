// Gradient reduction + Adam over the flat parameter arena (gfx950).
//
// k_reduce_adam : for every parameter element, sum its per-row-tile partial
//   slabs (dW/db written by the tower kernels) in a fixed order -- or take the
//   atomically accumulated value (BN affine, embeddings, logit_scale) -- write
//   the full gradient, zero the accumulators for the next step, and optionally
//   apply Adam in the same pass (single-GPU training: one launch for K10+K11);
//   EX: the data-parallel mean over ranks (peer memory) between the two.
// k_adam : Adam alone (data-parallel: after the RCCL all-reduce of `grad`).
//
// Adam arithmetic follows torch 2.10 _single_tensor_adam (optim.Adam.step,
// training.py:55):  m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, 1-b2);
//   denom = sqrt(v) / sqrt(bc2) + eps;  p.addcdiv_(m, denom, -lr/bc1)
// with bias corrections in double precision, element math in fp32.
#include "tt_common.h"
#include "tt_reduce.h"

namespace tt {

// Element space: block b, lane (pg, el) takes virtual element v = b RED_E + el.
// Every segment's virtual range starts on a block boundary, so the segment
// (and its kind) is uniform per block: one scalar lookup, no per-lane
// divergence.  Ranges map one to one onto the parameter arena, except kind 3
// (W0 of the folded BN0 backward, slab partials laid out [64][kp/16][P 16 |
// Q 16]): each 32-element group of its range covers 16 W0 elements twice --
// el < 16 sums their P partials, el >= 16 the Q partials of the same
// elements -- so the owner finds both sums in this block's LDS and every lane
// reads 64 B of one 128-B P|Q row segment.
// PRE: the step's Adam coefficients come from the workspace cache (AdamSlot,
// tt_common.h: a fused train step); otherwise the owner lanes compute them.
template <bool PRE, bool EX>
__global__ __launch_bounds__(RED_E* RED_G, TT_RED_MINW) void k_reduce_adam(RedArgs a) {
  __shared__ float part[RED_G * RED_E];
  __shared__ float xpart[4 * RED_G * RED_E];  // kinds 3, 4: gg0, gbe0, sum Zh0, sum X' replicas
  __shared__ int xok_s;
  reduce_body<RedArgs, RED_G, PRE, EX, false>(a, (int)blockIdx.x, part, xpart, &xok_s);
}

// A deferred late half on its own (tt_train_flush): the same LATE_G body and
// summation order as inside k_l0_fwd, so flushed and in-step late halves
// give the same bits.
__global__ __launch_bounds__(RED_E* LATE_G) void k_reduce_late(LateRed a) {
  __shared__ float part[LATE_G * RED_E];
  __shared__ float xpart[4 * LATE_G * RED_E];
  __shared__ int xok_s;
  reduce_body<LateRed, LATE_G, true, false, true>(a, (int)blockIdx.x, part, xpart, &xok_s);
}
__global__ void k_clear_late(int64_t* late_pending) { *late_pending = 0; }

template __global__ void k_reduce_adam<true, false>(RedArgs);
template __global__ void k_reduce_adam<false, false>(RedArgs);
template __global__ void k_reduce_adam<true, true>(RedArgs);

// ---------------------------------------------------------------------------
// Deterministic mode (TT_FLAG_DETERMINISTIC).  The tower kernels store each
// block's partial of a cross-block accumulator into its own slot instead of
// a float atomic into a replica; k_det_fold sums the slots of every column in
// a fixed order (a fixed summation tree over the slots) into replica 0 -- the
// replicas the consumers then add are that sum and zeros, so every step is
// bitwise repeatable.  Up to 4 arrays per launch (blockIdx.y).
// ---------------------------------------------------------------------------
struct DetFold {
  const float* src[4];
  float* dst[4];
  int n_slots[4], width[4];
};

// Block (x, y): 32 columns of array y; thread (c, q) sums slots q, q + 8,
// q + 16, ... of column c (4 independent chains), then the 8 partials of a
// column are added in q order: a fixed summation tree for any timing.
constexpr int DET_COLS = 32, DET_GROUPS = 8;
__global__ __launch_bounds__(DET_COLS * DET_GROUPS) void k_det_fold(DetFold f) {
  __shared__ float part[DET_GROUPS][DET_COLS];
  const int k = blockIdx.y;
  const int w = f.width[k], n = f.n_slots[k];
  const int cl = (int)threadIdx.x % DET_COLS, q = (int)threadIdx.x / DET_COLS;
  const int c = (int)blockIdx.x * DET_COLS + cl;
  const bool live = c < w;
  const float* s = f.src[k] + (live ? c : 0);
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  // slot i = q + 8 j goes to chain j & 3 (the fixed tree of the original
  // loop); all DET_LOADS slots of a round are loaded before the first add --
  // one memory round trip per 256 slots instead of one per 4 (was 4.9 us per
  // fold launch at 256 slots, 4 launches per deterministic step)
  constexpr int DET_LOADS = 32;
  static_assert((DET_GROUPS * DET_LOADS / DET_GROUPS) % 4 == 0, "rounds keep the chain order");
  for (int base = 0; base < n; base += DET_GROUPS * DET_LOADS) {
    float x[DET_LOADS];
#pragma unroll
    for (int j = 0; j < DET_LOADS; ++j) x[j] = s[(int64_t)min(base + q + DET_GROUPS * j, n - 1) * w];
#pragma unroll
    for (int j = 0; j < DET_LOADS; ++j)
      if (base + q + DET_GROUPS * j < n) acc[j & 3] += x[j];
  }
  part[q][cl] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (q == 0 && live) {
    float v = part[0][cl];
#pragma unroll
    for (int g = 1; g < DET_GROUPS; ++g) v += part[g][cl];
    f.dst[k][c] = v;
  }
}

#ifndef TT_DET_SCATTER_V2
#define TT_DET_SCATTER_V2 1
#endif
#if TT_DET_SCATTER_V2
// Embedding-table gradients in deterministic mode (model.py:69,74 backward,
// EmbeddingBackward): block (x, y) owns 256 consecutive (code, element)
// entries of categorical column y -- the codes c_lo .. c_hi -- and walks the
// batch in row order.  Per chunk of DET_SCAT_CHUNK rows it stages the codes,
// keeps the rows whose code falls in its range (a stable compaction: wave
// ballots, waves in order), and every entry adds its code's kept rows' dX in
// that order -- the batch-row order of the reference's sum, so every entry of
// every table is written (codes absent from the batch get 0) and the gacc
// arena needs no zeroing in between.  A block reads the B codes once and
// then only its own codes' rows: table_rows x E x B compares became
// blocks x B + B x E (large label-encoded vocabularies).
constexpr int DET_SCAT_CHUNK = 2048;
__global__ __launch_bounds__(256) void k_det_scatter(StepArgs a) {
  __shared__ int codes[DET_SCAT_CHUNK];
  __shared__ int sel_row[DET_SCAT_CHUNK];   // chunk-local row of a kept row, in row order
  __shared__ int sel_code[DET_SCAT_CHUNK];
  __shared__ int wcnt[4];
  int j = (int)blockIdx.y, t = 0;
  if (j >= a.tw[0].n_cat) {
    j -= a.tw[0].n_cat;
    t = 1;
  }
  const TowerDev& T = a.tw[t];
  const int E = T.emb_dim, rows = T.emb_rows[j];
  const int64_t q0 = (int64_t)blockIdx.x * blockDim.x;
  if (q0 >= (int64_t)rows * E) return;  // whole block past the table
  const int64_t q = q0 + threadIdx.x;   // entry code * E + e
  const int code = (int)(q / E), e = (int)(q - (int64_t)code * E);
  const bool live = code < rows;
  const int c_lo = (int)(q0 / E), c_hi = (int)min((q0 + (int64_t)blockDim.x - 1) / E, (int64_t)rows - 1);
  const int64_t base = batch_row0(a, step_current(a));
  const float* dx = T.demb + j * E + e;
  const int w = wave_id(), l = lane_id();
  const uint64_t below = l ? (~0ull >> (64 - l)) : 0ull;  // lanes < l
  float acc = 0.f;
  for (int64_t r0 = 0; r0 < a.B; r0 += DET_SCAT_CHUNK) {
    const int n = (int)min((int64_t)DET_SCAT_CHUNK, a.B - r0);
    __syncthreads();  // the previous chunk's lists are consumed
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      int64_t c = T.cat[data_row(a, base, r0 + i) * T.cat_ld + j];
      codes[i] = (int)(c < 0 ? 0 : (c >= rows ? rows - 1 : c));  // the kernels' clamp
    }
    __syncthreads();
    int nsel = 0;
    for (int s0 = 0; s0 < n; s0 += 256) {
      const int i = s0 + (int)threadIdx.x;
      const int c = i < n ? codes[i] : -1;
      const bool keep = c >= c_lo && c <= c_hi;
      const uint64_t bal = __ballot(keep);
      if (l == 0) wcnt[w] = __popcll(bal);
      __syncthreads();
      int woff = 0, tot = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        woff += k < w ? wcnt[k] : 0;
        tot += wcnt[k];
      }
      if (keep) {
        const int at = nsel + woff + __popcll(bal & below);
        sel_row[at] = i;
        sel_code[at] = c;
      }
      nsel += tot;
      __syncthreads();  // wcnt reused; the lists complete
    }
    if (live)
      for (int k = 0; k < nsel; ++k)
        if (sel_code[k] == code) acc += dx[(r0 + sel_row[k]) * T.emb_w];
  }
  if (live) T.gemb[j][q] = acc;
}

#else
constexpr int DET_SCAT_CHUNK = 2048;
// Embedding-table gradients in deterministic mode (model.py:69,74 backward,
// EmbeddingBackward): block (x, y) owns 256 consecutive (code, element)
// entries of categorical column y (towers' columns concatenated); it stages
// the batch's codes in chunks and adds the rows' dX (k_bwd_first, T.demb) in
// batch-row order.  Every entry of every table is written (codes absent from
// the batch get 0), so the gacc arena needs no zeroing in between.
__global__ __launch_bounds__(256) void k_det_scatter(StepArgs a) {  // (round-3 form)
  __shared__ int codes[DET_SCAT_CHUNK];
  int j = (int)blockIdx.y, t = 0;
  if (j >= a.tw[0].n_cat) {
    j -= a.tw[0].n_cat;
    t = 1;
  }
  const TowerDev& T = a.tw[t];
  const int E = T.emb_dim, rows = T.emb_rows[j];
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // entry code * E + e
  if ((int64_t)blockIdx.x * blockDim.x >= (int64_t)rows * E) return;  // whole block past the table
  const int code = (int)(q / E), e = (int)(q - (int64_t)code * E);
  const bool live = code < rows;
  const int64_t base = batch_row0(a, step_current(a));
  const float* dx = T.demb + j * E + e;
  float acc = 0.f;
  for (int64_t r0 = 0; r0 < a.B; r0 += DET_SCAT_CHUNK) {
    const int n = (int)min((int64_t)DET_SCAT_CHUNK, a.B - r0);
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
      int64_t c = T.cat[data_row(a, base, r0 + i) * T.cat_ld + j];
      codes[i] = (int)(c < 0 ? 0 : (c >= rows ? rows - 1 : c));  // the kernels' clamp
    }
    __syncthreads();
    if (live)
      for (int i = 0; i < n; ++i)
        if (codes[i] == code) acc += dx[(r0 + i) * T.emb_w];
  }
  if (live) T.gemb[j][q] = acc;
}

#endif

__global__ __launch_bounds__(256) void k_adam(float* __restrict__ P, const float* __restrict__ G,
                                              float* __restrict__ M, float* __restrict__ V, int64_t n,
                                              double lr, double b1, double b2, double eps, tt_state* state,
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
