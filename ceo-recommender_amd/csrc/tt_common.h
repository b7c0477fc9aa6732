// Shared device helpers for the two-tower (CEOFirmMatcher) training kernels.
//
// gfx950 / CDNA4 only: wave64, v_mfma_f32_16x16x4_f32 (exact fp32 MFMA),
// ds_add_f32 LDS atomics, global_atomic_add_f32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ceo_tt.h"

namespace tt {

constexpr int WAVE = 64;
constexpr int H0 = 64;    // model.py:38  Linear(in, 64)
constexpr int H1 = 32;    // model.py:42  Linear(64, 32)
constexpr int ROWS = 64;  // rows of the batch per row tile (one 16-row strip per wave)
constexpr int WAVES = ROWS / 16;
constexpr int THREADS = WAVES * WAVE;
constexpr int TOP_ROWS_MAX = 128;  // k_top may use 128-row tiles (8 waves)
constexpr int MAX_KP = 256;  // padded tower input width supported by the fused kernels
// Cross-block sums (BN moments, BN-affine grads, logit-scale grad, loss) are
// accumulated into NREP replicas picked by blockIdx.x: 512 blocks adding into
// the same 128 addresses serialise at the memory-side atomic unit (measured:
// +4.5 us on k_l0_fwd); with replicas each address sees 1/NREP of the adds and
// the consumers sum NREP values.  NREP = 8 (round 6; was 16): every block of
// one XCD (blockIdx % 8) adds into that XCD's replica, and every consumer
// block (all of k_l4_fwd's 512, the reduction's replica ranges) loads half
// the bytes.  Two interleaved rounds at cfg 3 (profiles/r06_nrep_ab): step
// 16: 49.6-49.7 us, 8: 49.2, 4: 50.5-50.6, 2: 56.1 (the adds serialise again).
#ifndef TT_NREP
#define TT_NREP 8
#endif
constexpr int NREP = TT_NREP;
// replica strides (floats) of the BN moment sums S1|S2 (st0: 2*64, st1: 2*32
// floats of content); TT_REP_PAD spaces the replicas further apart
#ifndef TT_REP_PAD
#define TT_REP_PAD 0
#endif
constexpr int ST0S = 2 * H0 + TT_REP_PAD;
constexpr int ST1S = 2 * H1 + TT_REP_PAD;
constexpr int BNG = 2 * H0 + 2 * H1;  // one replica of a tower's BN-affine grads: gg0|gbe0|gg1|gbe1
// Folded BN0 backward (k_bwd_mid<R, true>, numeric-only towers with kp <= 64):
// one replica of a tower's fold sums: gg0 | gbe0 | sum Zhat0 | sum (X - shift)
constexpr int FRW = 3 * H0 + 64;
constexpr int FOLD_MAX_KP = 64;
constexpr int FOLD_ROWS = 128;  // k_bwd_mid_fold row tile (8 waves)
// k_reduce_adam's element space heaviest range first (make_red)
#ifndef TT_RED_HEAVY_FIRST
#define TT_RED_HEAVY_FIRST 1
#endif
#ifndef TT_PAIR32_MAX_B
#define TT_PAIR32_MAX_B 8192  // training batches below it (and unfolded) run k_top_pair on 32-row blocks
#endif
#ifndef TT_FWD32_MAX_B
#define TT_FWD32_MAX_B 0  // (off: measured slower) batches below it run k_l0_fwd / k_l4_fwd on 32-row blocks
#endif
#ifndef TT_BWD32_MAX_B
#define TT_BWD32_MAX_B 0  // (off: measured slower) unfolded batches below it run k_bwd_mid / k_bwd_first on 32-row blocks
#endif
#ifndef TT_FOLD_MIN_B
#define TT_FOLD_MIN_B 4096  // smallest batch that runs the folded BN0 backward (round 5: cfg 2 40.0 -> 38.9 us)
#endif
constexpr int LSR = 32;               // replica stride of the (dls, loss) pair
// Replica of a block: (blockIdx.x / 8) % NREP spreads each XCD's blocks
// (dispatched round robin: block b on XCD b % 8) over all NREP replicas;
// blockIdx.x % NREP put all of an XCD's adds on one replica.  Three
// interleaved rounds at cfg 3 (profiles/r06_rep_spread_ab): step 49.3-49.4 ->
// 48.4-48.6 us (k_l0_fwd -0.5, k_l4_fwd -0.5 us); with the spread, 8 replicas
// beat 4 (49.6) and 16 (49.3-49.4).  Placement changes speed only: any block
// may add into any replica.
#ifndef TT_REP_SPREAD
#define TT_REP_SPREAD 1
#endif
__device__ __forceinline__ int rep_of_block() {
  return TT_REP_SPREAD ? (int)((blockIdx.x >> 3) % NREP) : (int)(blockIdx.x % NREP);
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane((int)threadIdx.x >> 6); }  // uniform: SGPR, scalar branches

// ---------------------------------------------------------------------------
// v_mfma_f32_16x16x4_f32, fp32 in / fp32 acc (bitwise an fmaf chain).
//   lane l supplies A[i = l&15][k = l>>4] and B[k = l>>4][j = l&15];
//   C/D: lane l holds C[row = 4*(l>>4) + reg][col = l&15].
// Our K order: MFMA step s of a 16-wide K chunk k0 uses k = k0 + 4*(l>>4) + s,
// so every lane reads 4 consecutive k with ONE ds_read_b128 per operand.
// ---------------------------------------------------------------------------
__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ void mfma_k16(const float4& a, const float4& b, f32x4& c) {
  c = mfma4(a.x, b.x, c);
  c = mfma4(a.y, b.y, c);
  c = mfma4(a.z, b.z, c);
  c = mfma4(a.w, b.w, c);
}

// Row-strip NT GEMM from LDS:  C[16 x 16*NT] = A[16 x K] * B[16*NT x K]^T
//   A: this wave's 16-row strip, row-major, stride lda (floats)
//   B: row-major [n][k], stride ldb;  K a multiple of 16 (zero padded)
template <int NT>
__device__ __forceinline__ void strip_gemm_nt(const float* A, int lda, const float* B, int ldb,
                                              int K, f32x4 (&acc)[NT]) {
  const int l = lane_id(), r = l & 15, g = l >> 4;
  for (int k0 = 0; k0 < K; k0 += 16) {
    const float4 a = *reinterpret_cast<const float4*>(A + r * lda + k0 + 4 * g);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const float4 b = *reinterpret_cast<const float4*>(B + (16 * j + r) * ldb + k0 + 4 * g);
      mfma_k16(a, b, acc[j]);
    }
  }
}

// Strip GEMM with A given TRANSPOSED in LDS (AT[k][m], stride lda) and B given
// row-major [k][n] (stride ldb); both read with 4 ds_read_b32 per operand:
//   C[16 x 16*NT] = A[16 x K] * B[K x 16*NT],  A(r,k) = AT[k][r]
template <int NT>
__device__ __forceinline__ void strip_gemm_tn(const float* AT, int lda, const float* B, int ldb, int K,
                                              f32x4 (&acc)[NT]) {
  const int l = lane_id(), r = l & 15, g = l >> 4;
  for (int k0 = 0; k0 < K; k0 += 16) {
    const float* ap = AT + (k0 + 4 * g) * lda + r;
    const float4 a = make_float4(ap[0], ap[lda], ap[2 * lda], ap[3 * lda]);
    const float* bp = B + (k0 + 4 * g) * ldb + r;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const float4 b = make_float4(bp[16 * j], bp[ldb + 16 * j], bp[2 * ldb + 16 * j], bp[3 * ldb + 16 * j]);
      mfma_k16(a, b, acc[j]);
    }
  }
}

// Store a C-layout 16x16 tile TRANSPOSED into LDS: dst[c][row0 + 4g .. +3]
// (one ds_write_b128 per lane; dst row stride ld, row0 and ld multiples of 4)
__device__ __forceinline__ void store_tile_T(float* dst, int ld, int c0, int row0, const f32x4& v) {
  const int l = lane_id(), r = l & 15, g = l >> 4;
  *reinterpret_cast<f32x4*>(dst + (c0 + r) * ld + row0 + 4 * g) = v;
}

// Rows-contracted product from C-layout registers (no LDS):
//   acc[16 x 16] += P^T Q  over this wave's 16 rows, where P, Q are 16x16 tiles
//   held in C layout (lane (r,g) holds rows 4g..4g+3 of column r).
__device__ __forceinline__ void cl_gemm_tn(const f32x4& P, const f32x4& Q, f32x4& acc) {
  acc = mfma4(P[0], Q[0], acc);
  acc = mfma4(P[1], Q[1], acc);
  acc = mfma4(P[2], Q[2], acc);
  acc = mfma4(P[3], Q[3], acc);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

// ---------------------------------------------------------------------------
// fp32 through the bf16 MFMA (bf16x3 split).  Each fp32 value x is split
// exactly into three bf16 planes x = h + m + l (round-to-nearest-even), and a
// product is the six plane products whose magnitude is >= 2^-16 of h*h:
//     x*y ~= l*h + m*m + h*l + m*h + h*m + h*h
// (the dropped m*l, l*m, l*l terms are <= ~2^-24 relative: fp32's own
// rounding).  Every plane product is exact in the fp32 accumulator, so a
// 32-deep K step costs 6 v_mfma_f32_16x16x32_bf16 (16 cycles each) instead of
// 8 v_mfma_f32_16x16x4_f32 (32 cycles each): 2.7x the fp32 MFMA rate.
//   16x16x32 operand map: lane l holds A[m = l&15][k = 8(l>>4) + e] and
//   B[k = 8(l>>4) + e][n = l&15] in element e; C as the fp32 form.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 16-B write-through store (buffer_store_dwordx4 ... sc1): the line leaves the
// XCD's L2 at once and is dropped there, so the kernel ends with no dirty
// lines for the boundary's L2 write-back (MI355X_MICROARCH.md 'boundary':
// + B / 6 TB/s when a kernel leaves B bytes dirty).  base must be uniform
// across the wave (it becomes the SGPR buffer descriptor); off = per-lane bytes.
template <int AUX = 16>
__device__ __forceinline__ void st_wt16(const float* base, uint32_t off, f32x4 v) {
  const auto rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, 0x7FFFFFFF, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, (int)off, 0, AUX);
}
// Cache policy of the activation hand-offs (Z0, Z4, dY1) that the next
// kernels re-read on the SAME XCD (tile64): 16 = sc1 (write-through, line
// dropped), 0 = plain (kept in L2, written back at the boundary)
#ifndef TT_HANDOFF_AUX
#define TT_HANDOFF_AUX 16
#endif

__device__ __forceinline__ uint16_t bf16_bits(float x) { return __builtin_bit_cast(uint16_t, (__bf16)x); }
__device__ __forceinline__ float bf16_val(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {  // one v_cvt_pk_bf16_f32 (RNE)
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}
// split two values at once: packed planes (lo half = first value)
__device__ __forceinline__ void split3x2(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = pk_bf16(x0, x1);
  const float r0 = x0 - __uint_as_float(h << 16), r1 = x1 - __uint_as_float(h & 0xffff0000u);
  m = pk_bf16(r0, r1);
  l = pk_bf16(r0 - __uint_as_float(m << 16), r1 - __uint_as_float(m & 0xffff0000u));
}
__device__ __forceinline__ void split3(float x, uint16_t& h, uint16_t& m, uint16_t& l) {
  h = bf16_bits(x);
  const float r1 = x - bf16_val(h);  // exact
  m = bf16_bits(r1);
  l = bf16_bits(r1 - bf16_val(m));   // exact residual, rounded to bf16
}
// 8 values -> three bf16x8 planes (element e = x[e])
__device__ __forceinline__ void split8x3(const float (&x)[8], bf16x8 (&pl)[3]) {
  u32x4 h, m, l;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t hh, mm, ll;
    split3x2(x[2 * q], x[2 * q + 1], hh, mm, ll);
    h[q] = hh;
    m[q] = mm;
    l[q] = ll;
  }
  pl[0] = __builtin_bit_cast(bf16x8, h);
  pl[1] = __builtin_bit_cast(bf16x8, m);
  pl[2] = __builtin_bit_cast(bf16x8, l);
}

// 4 floats -> 4 bf16 in each of the 3 planes (8-B stores)
__device__ __forceinline__ void put_planes4(uint16_t* dst, int plane, const float4& v) {
  uint32_t h01, m01, l01, h23, m23, l23;
  split3x2(v.x, v.y, h01, m01, l01);
  split3x2(v.z, v.w, h23, m23, l23);
  *reinterpret_cast<u32x2*>(dst) = (u32x2){h01, h23};
  *reinterpret_cast<u32x2*>(dst + plane) = (u32x2){m01, m23};
  *reinterpret_cast<u32x2*>(dst + 2 * plane) = (u32x2){l01, l23};
}

__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// the six plane products, smallest first (a fixed order: k_nce_diag replays
// exactly this sequence)
constexpr int PA[6] = {2, 1, 0, 1, 0, 0};
constexpr int PB[6] = {0, 1, 2, 0, 1, 0};
__device__ __forceinline__ void mfma_x3(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x4& c) {
#pragma unroll
  for (int q = 0; q < 6; ++q) c = mfma_bf16(a[PA[q]], b[PB[q]], c);
}

// gfx950 ds_read_b64_tr_b16: per 16-lane group, lane 4q+p supplies the
// address of row q, 4 consecutive 16-bit columns (8-B aligned); lane i of the
// group receives column i (chunk i>>2, element i&3) of the 4 rows, row q in
// element q.  EXEC must be all ones.
__device__ __forceinline__ s16x4 lds_tr16(const uint16_t* p) {
  typedef __attribute__((address_space(3))) s16x4 lds_s16x4;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
}
// two transposed reads -> one 16x16x32 operand (elements 0-3, 4-7)
__device__ __forceinline__ bf16x8 tr_frag(const uint16_t* p0, const uint16_t* p1) {
  const s16x4 x = lds_tr16(p0), y = lds_tr16(p1);
  const u32x2 xu = __builtin_bit_cast(u32x2, x), yu = __builtin_bit_cast(u32x2, y);
  return __builtin_bit_cast(bf16x8, (u32x4){xu[0], xu[1], yu[0], yu[1]});
}

// Cross-lane sums without LDS round trips (ds_bpermute costs a full LDS
// latency per step and the compiler serialises dependent ones):
//  * within a 16-lane row: DPP quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
//    row_mirror -- each step pairs disjoint partial sums, so after four steps
//    every lane of the row holds the same total;
//  * across rows: gfx950 v_permlane16_swap / v_permlane32_swap exchange whole
//    rows between two registers in one VALU op.
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float xrow16_add(float v) {  // v[l] + v[l ^ 16]
  const unsigned u = __float_as_uint(v);
  const auto p = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  // copy the elements out first: __builtin_bit_cast(float, p[1]) is folded
  // into p[0] by this hipcc
  const unsigned lo = p[0], hi = p[1];
  return __uint_as_float(lo) + __uint_as_float(hi);
}
__device__ __forceinline__ float xrow32_add(float v) {  // v[l] + v[l ^ 32]
  const unsigned u = __float_as_uint(v);
  const auto p = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  // copy the elements out first: __builtin_bit_cast(float, p[1]) is folded
  // into p[0] by this hipcc
  const unsigned lo = p[0], hi = p[1];
  return __uint_as_float(lo) + __uint_as_float(hi);
}
// 4x4 transpose inside each lane quad (lanes 4c..4c+3): on entry lane k
// holds column k of the quad's 4x4 block (v[i] = M[i][k]), on exit row k
// (M[k][0..3]).  Two DPP exchange stages (xor 2, xor 1), no LDS.
__device__ __forceinline__ f32x4 quad_transpose(f32x4 v) {
  const int k = lane_id() & 3;
  const bool hi = (k & 2) != 0, odd = (k & 1) != 0;
  float a0 = hi ? v[0] : v[2], a1 = hi ? v[1] : v[3];
  float b0 = dpp_mov<0x4E>(a0), b1 = dpp_mov<0x4E>(a1);  // quad_perm [2,3,0,1]
  const f32x4 s = hi ? f32x4{b0, b1, v[2], v[3]} : f32x4{v[0], v[1], b0, b1};
  a0 = odd ? s[0] : s[1];
  a1 = odd ? s[2] : s[3];
  b0 = dpp_mov<0xB1>(a0);  // quad_perm [1,0,3,2]
  b1 = dpp_mov<0xB1>(a1);
  return odd ? f32x4{b0, s[1], b1, s[3]} : f32x4{s[0], b0, s[2], b1};
}
// Store a 16x16 tile held in the MFMA accumulator layout (lane (r, g): rows
// 4g..4g+3 of column r) row-major: quad transpose, then one 16-B
// write-through store per lane (4 consecutive columns of one row).
// base: block-uniform pointer; off: element offset of the tile's (0, 0) from
// base (small); ld: row stride in floats (multiple of 4, base 16-B aligned).
template <int AUX = 16>
__device__ __forceinline__ void store_tile_rm_wt(const float* base, int off, int ld, f32x4 acc) {
  const int l = lane_id(), r = l & 15, g = l >> 4;
  const f32x4 t = quad_transpose(acc);
  st_wt16<AUX>(base, (uint32_t)((off + (4 * g + (r & 3)) * ld + (r & ~3)) * 4), t);
}
// sum over the 4 lane groups (g = l>>4) that share a column r
__device__ __forceinline__ float col_reduce(float v) { return xrow32_add(xrow16_add(v)); }
// sum over the 16 lanes (r) that share a row group g
__device__ __forceinline__ float row_reduce16(float v) {
  v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp_mov<0x141>(v);  // row_half_mirror
  v += dpp_mov<0x140>(v);  // row_mirror
  return v;
}
// full-wave sum (every lane gets the total)
__device__ __forceinline__ float wave_reduce(float v) { return col_reduce(row_reduce16(v)); }

// ---------------------------------------------------------------------------
// Counter-based dropout RNG (restated in oracle/two_tower.py dropout_keep_mask)
// ---------------------------------------------------------------------------
__host__ __device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ uint64_t dropout_key(uint64_t seed, uint64_t step, int tower, int layer) {
  return mix64(seed * 0x9E3779B97F4A7C15ull + step * 0xD1B54A32D192ED03ull +
               (uint64_t)(tower * 2 + layer + 1) * 0x8CB92BA72F3D8DD7ull);
}
// Per element (row, column) of one stream: a 32-bit avalanche permutation
// (lowbias32) keyed per row, rk = P(row ^ key_lo) + key_hi, and per PAIR of
// columns h = P(rk ^ pid * 0x9E3779B9): the pair (c, c ^ 2^HB) shares h, the
// element with bit HB clear takes its low 16 bits, the other the high 16;
// keep iff that 16-bit uniform >= floor(p * 2^16).  HB follows how the
// kernels hold a layer's columns, so both halves of a hash land in one lane:
// layer 0 (A0: k_l4_fwd's A operand holds columns 8g.. and 32 + 8g.., the
// backward kernels' MFMA C layout columns 16j + r, j = 0..3) HB = 5, layer 1
// (A1, k_top: 8 consecutive columns per lane) HB = 0.  Two elements per permutation (two
// quarter-rate multiplies each) halves the cost of recomputing the masks
// wherever the forward or backward needs them.
__host__ __device__ __forceinline__ uint32_t perm32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint32_t dropout_row_key(uint64_t key, int64_t row) {
  return perm32((uint32_t)row ^ (uint32_t)key) + (uint32_t)(key >> 32);
}
template <int HB>
__device__ __forceinline__ bool dropout_keep_rk(uint32_t rk, int col, uint32_t thr) {
  const uint32_t c = (uint32_t)col;
  const uint32_t pid = ((c >> (HB + 1)) << HB) | (c & ((1u << HB) - 1u));
  const uint32_t h = perm32(rk ^ (pid * 0x9E3779B9u));
  return (((c >> HB) & 1u) ? (h >> 16) : (h & 0xFFFFu)) >= thr;
}
constexpr int DROP_HB0 = 5, DROP_HB1 = 0;  // layer 0 (A0), layer 1 (A1)

// ---------------------------------------------------------------------------
// Kernel argument block (passed by value; lives in the kernarg segment).
// ---------------------------------------------------------------------------
struct TowerDev {
  const float* num;  int64_t num_ld;      // numeric features [N, num_ld]
  const int64_t* cat; int64_t cat_ld;     // categorical codes [N, cat_ld]
  int n_num, n_cat, emb_dim, in_dim, kp;  // kp = in_dim rounded up to 16
  int num_vec;                            // numeric rows 16-B aligned, no embeddings: float4 gather
  const float* emb[TT_MAX_CAT];           // embedding tables (param arena)
  int emb_rows[TT_MAX_CAT];               // rows per table (codes are clamped into range)
  float* gemb[TT_MAX_CAT];                // their gradient accumulators (gacc arena)
  const float *W0, *b0, *g0, *be0, *W4, *b4, *g1, *be1, *W8, *b8;
  float *rm0, *rv0, *rm1, *rv1;           // BN running stats
  int64_t *nbt0, *nbt1;                   // num_batches_tracked
  float *gg0, *gbe0, *gg1, *gbe1;         // BN affine grad accumulators: replica r at +r*BNG
  // workspace
  float *Z0, *Z4, *dY0, *dY1;             // [B,64] [B,32] [B,64] [B,32]
  float *st0, *st1;                       // shifted moment sums S1|S2 [NREP][2*64], [NREP][2*32]
  float *shift0, *shift1;                 // shifts used for S1/S2 [64], [32]
  float *fin0, *fin1;                     // finalized mean|invstd [2*64], [2*32]
  float* slab;                            // [n_slabs][slab_ld] partial dW/db sums
  int64_t so_W0, so_b0, so_W4, so_b4, so_W8, so_b8;  // offsets inside one slab
  float* fr;                              // folded: [NREP][FRW] replicas (zeroed by k_l0_fwd)
  float *k0s, *xsh;                       // folded: inv0*gamma0 [64], shift row [64] (block 0 writes)
  float* dxn;                             // backward: dL/d numeric input [B, n_num] (nullable; k_bwd_first)
  // deterministic mode (StepArgs::det): cross-block partial sums go to
  // per-block slots [blocks][width] (plain stores) instead of float atomics
  // into replicas; k_det_fold sums the slots in block order into replica 0
  float* dslot;
  float* demb;                            // det: dX of the embedding columns [Bpad][emb_w] for k_det_scatter
  int emb_w;                              // n_cat * emb_dim
  float *ug, *dug;                        // LATENT > 128 (tt_topgen.hip): U (V) and dU (dV) [Bpad][Dp]
};

enum TopMode : int { TOP_FWD = 0, TOP_TRAIN = 1, TOP_BWD_GIVEN = 2, TOP_EMB_FWD = 3, TOP_EMB_BWD = 4 };

// Adam arithmetic of torch 2.10 _single_tensor_adam (training.py:55) from
// the hyperparameters as Python passes them (double): bias corrections in
// double, each scalar cast to float where torch's kernels cast it (lerp
// weight 1 - beta1, mul_ beta2, addcmul value 1 - beta2, addcdiv value
// -lr / bc1, the divisor sqrt(bc2), eps), element math in fp32
// (k_reduce_adam, k_adam, k_ar_adam and k_bwd_mid_fold's side reduction)
struct AdamCoef {
  float w1, c2, b2, step_size, bc2s, eps;
};

__device__ __forceinline__ AdamCoef adam_coef(double lr, double b1, double b2, double eps, int64_t t) {
  const double bc1 = 1.0 - pow(b1, (double)t);
  const double bc2 = 1.0 - pow(b2, (double)t);
  AdamCoef c;
  c.w1 = (float)(1.0 - b1);
  c.c2 = (float)(1.0 - b2);
  c.b2 = (float)b2;
  c.step_size = (float)(lr / bc1);
  c.bc2s = (float)sqrt(bc2);
  c.eps = (float)eps;
  return c;
}

__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, const AdamCoef& c) {
  m = m + c.w1 * (g - m);           // lerp, weight < 0.5 branch
  v = v * c.b2 + (c.c2 * g) * g;    // mul_ + addcmul_
  const float denom = sqrtf(v) / c.bc2s + c.eps;
  p = p + (-c.step_size) * (m / denom);
}

// Adam coefficients of step t, cached in the workspace at slot t & 1 with
// the step and hyperparameters they were computed for.  k_reduce_adam of
// step t reads slot t & 1 and one of its light blocks (a replica segment:
// no slab loads, slack to spare) computes step t + 1's into the other slot,
// so the double pow chain is off every critical path; k_l0_fwd recomputes a
// slot that does not match (first step, a step counter set by the host,
// changed hyperparameters).  Two slots: the write for t + 1 never races the
// reads of t.
struct AdamSlot {
  int64_t t;
  double lr, b1, b2, eps;
  AdamCoef c;
};
__device__ __forceinline__ bool adam_slot_ok(const AdamSlot& s, int64_t t, double lr, double b1, double b2,
                                             double eps) {
  return s.t == t && s.lr == lr && s.b1 == b1 && s.b2 == b2 && s.eps == eps;
}
__device__ __forceinline__ void adam_slot_fill(AdamSlot& s, int64_t t, double lr, double b1, double b2, double eps) {
  s.c = adam_coef(lr, b1, b2, eps, t);
  s.lr = lr;
  s.b1 = b1;
  s.b2 = b2;
  s.eps = eps;
  s.t = t;
}

struct StepArgs {
  TowerDev tw[2];
  // batch
  const float* target; const float* weight;  // [N] each
  const int64_t* rows;   // row index list (nullable: identity)
  int64_t row0;          // host-mode offset into rows / dataset
  int64_t B;             // rows in this batch
  int64_t cycle;         // >0: device-counter mode, batch k starts at ((t-1-t_base)%cycle)*B
  int64_t t_base;
  tt_state* state;       // device counters (nullable: host mode)
  int64_t step_host;     // host-mode step number (dropout stream / Adam t)
  uint64_t seed;
  uint32_t drop_thr;     // keep iff 16-bit uniform >= drop_thr = floor(p 2^16)  (0: no dropout)
  float drop_scale;      // 1/(1-p) as fp32
  float eps, momentum;
  int train;
  int update_stats;      // fold batch stats into running stats (forward of a train step)
  int D, n_tiles, slab_ld;
  int mode;              // TopMode for the top kernel
  const float* logit_scale;
  float* lsr;            // [NREP][LSR] replicas: [0] dL/dlogit_scale, [1] batch-mean loss
  float* score;          // [B] output scores (nullable)
  const float* dscore;   // [B] upstream grad (TOP_BWD_GIVEN)
  float* tgw;            // [Bpad][2] (target, weight) of each batch row, gathered by k_l0_fwd
  float* emb;            // [2][B][D] raw tower outputs U | V (TOP_EMB_FWD)
  const float* demb;     // [2][B][D] upstream dU | dV (TOP_EMB_BWD)
  float* fr_zero;        // k_l0_fwd zeroes fr_zero[0, fr_zero_len) (both towers' fold replicas)
  int fr_zero_len;
  AdamSlot* adam_slots;  // non-null: k_l0_fwd makes sure slot t & 1 holds step t's coefficients
  double adam_lr, adam_b1, adam_b2, adam_eps;
  int det;               // deterministic reductions (TT_FLAG_DETERMINISTIC): slots + k_det_fold
  float* dslot_lsr;      // det: per-block (dls, loss) partials [blocks][2]
  int xcd_pair;          // folded step: 64-row kernels take XCD-paired tiles (tile64)
  int l0_gx;             // k_l0_fwd's row-tile blocks along x (more blocks: a deferred late half)
};

// Row tile of a 64-row kernel's block (k_l0_fwd, k_l4_fwd, k_top_pair).
// Blocks are dispatched round-robin over the 8 XCDs (block b -> XCD b % 8;
// each XCD has its own L2) and k_bwd_mid_fold's block x -- 128 rows, the
// 64-row tiles 2x and 2x + 1 -- runs on XCD x % 8.  With xcd_pair the 64-row
// kernels take their tiles so that 2x and 2x + 1 run on XCD x % 8 as well:
// the Z0 / Z4 / dY1 tiles and X rows the fold kernel re-reads were last
// touched through its own XCD's L2.  Bijective on every whole group of 16
// tiles, identity on the rest.
#ifndef TT_XCD_PAIR
#define TT_XCD_PAIR 1
#endif
__device__ __forceinline__ int tile64(const StepArgs& a) {
  const int b = blockIdx.x;
  if (!TT_XCD_PAIR || !a.xcd_pair || b >= (a.n_tiles & ~15)) return b;
  return 2 * (b & 7) + 16 * (b >> 4) + ((b >> 3) & 1);
}

// A block's partial sum of cross-block accumulator c: a float atomic into
// replica rep_of_block() (order of arrival decides the rounding), or in
// deterministic mode a plain store into the block's own slot, which
// k_det_fold then sums in block order (bitwise repeatable).
__device__ __forceinline__ void xblock_add(bool det, float* rep, int rep_stride, float* slot, int width, int c,
                                           float v) {
  if (det)
    slot[(int64_t)blockIdx.x * width + c] = v;
  else
    atomicAdd(&rep[rep_of_block() * rep_stride + c], v);
}

// ---------------------------------------------------------------------------
// Diagnostic phase stamps (separate -DTT_STAMPS build only; compiled out of
// the product library).  s_memrealtime (100 MHz, chip-wide) per block/phase.
// ---------------------------------------------------------------------------
// Register budget per kernel as waves per SIMD (amdgpu_waves_per_eu upper
// bound).  The dynamic LDS of the 8-wave kernels allows one block per CU (two
// waves per SIMD), but without this the compiler sizes registers for the
// occupancy __launch_bounds__ alone would allow (4 waves: 128 VGPRs) and
// serialises the bf16x3 MFMA chains to fit.
#define TT_WPE(n) __attribute__((amdgpu_waves_per_eu(1, n)))
#ifndef TT_WPE_TOP
#define TT_WPE_TOP 2
#endif
#ifndef TT_WPE_MID
#define TT_WPE_MID 8
#endif
#ifndef TT_WPE_L0
#define TT_WPE_L0 8
#endif
#ifndef TT_WPE_L4
#define TT_WPE_L4 8
#endif

#ifdef TT_STAMPS
extern __constant__ uint64_t* g_tt_stamps;
#define TT_STAMP_T(kid, slot, thr)                                                                      \
  do {                                                                                                  \
    if (g_tt_stamps && threadIdx.x == (thr))                                                            \
      g_tt_stamps[((uint64_t)(kid) * 2048 + blockIdx.y * gridDim.x + blockIdx.x) * 8 + (slot)] =        \
          __builtin_amdgcn_s_memrealtime();                                                             \
  } while (0)
#define TT_STAMP(kid, slot) TT_STAMP_T(kid, slot, 0)
#else
#define TT_STAMP_T(kid, slot, thr) ((void)0)
#define TT_STAMP(kid, slot) ((void)0)
#endif
// finer stamps inside one kernel's phases (kernel ids 6, 7), a separate
// diagnostic build: -DTT_STAMPS -DTT_SUBSTAMPS
#ifdef TT_SUBSTAMPS
#define TT_SUBSTAMP(kid, slot) TT_STAMP(kid, slot)
#else
#define TT_SUBSTAMP(kid, slot) ((void)0)
#endif

__device__ __forceinline__ int64_t step_for_first_kernel(const StepArgs& a) {
  return a.state ? a.state->step_done + 1 : a.step_host;
}
// The load goes through an explicit global pointer: written as a select
// between a.state->step_cur and the kernel argument a.step_host it became a
// FLAT load (generic address of either), whose wait is vmcnt(0) -- every load
// issued before it then had to land before anything that depends on the step
__device__ __forceinline__ int64_t load_step(const tt_state* st, const int64_t* dummy_global) {
  typedef __attribute__((address_space(1))) const int64_t gi64;
  const int64_t* p = st ? &st->step_cur : dummy_global;
  return *(gi64*)p;
}
__device__ __forceinline__ int64_t step_current(const StepArgs& a) {
  const int64_t v = load_step(a.state, reinterpret_cast<const int64_t*>(a.lsr));
  return a.state ? v : a.step_host;
}
__device__ __forceinline__ int64_t batch_row0(const StepArgs& a, int64_t t) {
  if (a.cycle > 0) return ((t - 1 - a.t_base) % a.cycle) * a.B;
  return a.row0;
}
// dataset row of batch row i
__device__ __forceinline__ int64_t data_row(const StepArgs& a, int64_t base, int64_t i) {
  return a.rows ? a.rows[base + i] : base + i;
}
// the same without a branch around the load (the load goes to a valid dummy
// address when there is no permutation): keeps the issue phase straight-line
__device__ __forceinline__ int64_t data_row_nb(const StepArgs& a, int64_t base, int64_t i) {
  const int64_t* p = a.rows ? a.rows + (base + i) : reinterpret_cast<const int64_t*>(a.lsr);
  const int64_t v = *p;
  return a.rows ? v : base + i;
}

// ---------------------------------------------------------------------------
// Global -> LDS staging.  Every helper issues UNR independent 16-byte loads
// per thread before the first LDS store (no per-iteration latency chain:
// these kernels are latency-, not bandwidth-bound at B = 16K).
// ---------------------------------------------------------------------------
// g[R][C] (row stride gld floats) -> s[R][sld]; C % 4 == 0, 16-B aligned rows.
// When the element count is a multiple of NT*UNR (the usual shapes) the loop
// has no per-element guard: a guarded store per element splits the code into
// small basic blocks at whose joins hipcc drains vmcnt(0), serialising the
// loads.  (Same rule for every hot loop in these kernels.)
template <int NT, int UNR>
__device__ __forceinline__ void g2s_f4(const float* __restrict__ g, int64_t gld, float* s, int sld, int R, int C) {
  const int c4 = C >> 2, n4 = R * c4;
  if (n4 % (NT * UNR) == 0) {
    for (int base = 0; base < n4; base += NT * UNR) {
      float4 v[UNR];
#pragma unroll
      for (int k = 0; k < UNR; ++k) {
        const int e = base + (int)threadIdx.x + k * NT;
        const int r = e / c4, c = e - r * c4;
        v[k] = *reinterpret_cast<const float4*>(g + r * gld + 4 * c);
      }
#pragma unroll
      for (int k = 0; k < UNR; ++k) {
        const int e = base + (int)threadIdx.x + k * NT;
        const int r = e / c4, c = e - r * c4;
        *reinterpret_cast<float4*>(s + r * sld + 4 * c) = v[k];
      }
    }
    return;
  }
  for (int base = 0; base < n4; base += NT * UNR) {
    float4 v[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int e = min(base + (int)threadIdx.x + k * NT, n4 - 1);
      const int r = e / c4, c = e - r * c4;
      v[k] = *reinterpret_cast<const float4*>(g + r * gld + 4 * c);
    }
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int e = base + (int)threadIdx.x + k * NT;
      if (e < n4) {
        const int r = e / c4, c = e - r * c4;
        *reinterpret_cast<float4*>(s + r * sld + 4 * c) = v[k];
      }
    }
  }
}
// transposed: g[R][C] -> s[C][sld] (s[c][r] = g[r][c]); C % 4 == 0.
template <int NT, int UNR>
__device__ __forceinline__ void g2s_f4_T(const float* __restrict__ g, int64_t gld, float* s, int sld, int R, int C) {
  const int c4 = C >> 2, n4 = R * c4;
  if (n4 % (NT * UNR) == 0) {
    for (int base = 0; base < n4; base += NT * UNR) {
      float4 v[UNR];
#pragma unroll
      for (int k = 0; k < UNR; ++k) {
        const int e = base + (int)threadIdx.x + k * NT;
        const int r = e / c4, c = e - r * c4;
        v[k] = *reinterpret_cast<const float4*>(g + r * gld + 4 * c);
      }
#pragma unroll
      for (int k = 0; k < UNR; ++k) {
        const int e = base + (int)threadIdx.x + k * NT;
        const int r = e / c4, c = 4 * (e - r * c4);
        s[(c + 0) * sld + r] = v[k].x;
        s[(c + 1) * sld + r] = v[k].y;
        s[(c + 2) * sld + r] = v[k].z;
        s[(c + 3) * sld + r] = v[k].w;
      }
    }
    return;
  }
  for (int base = 0; base < n4; base += NT * UNR) {
    float4 v[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int e = min(base + (int)threadIdx.x + k * NT, n4 - 1);
      const int r = e / c4, c = e - r * c4;
      v[k] = *reinterpret_cast<const float4*>(g + r * gld + 4 * c);
    }
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int e = base + (int)threadIdx.x + k * NT;
      if (e < n4) {
        const int r = e / c4, c = 4 * (e - r * c4);
        s[(c + 0) * sld + r] = v[k].x;
        s[(c + 1) * sld + r] = v[k].y;
        s[(c + 2) * sld + r] = v[k].z;
        s[(c + 3) * sld + r] = v[k].w;
      }
    }
  }
}
// scalar version for rows that are not 16-B aligned: g[R][C] -> s[R][sld]
template <int NT, int UNR>
__device__ __forceinline__ void g2s_f1(const float* __restrict__ g, int64_t gld, float* s, int sld, int R, int C) {
  const int n = R * C;
  for (int base = 0; base < n; base += NT * UNR) {
    float v[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int e = min(base + (int)threadIdx.x + k * NT, n - 1);
      const int r = e / C, c = e - r * C;
      v[k] = g[r * gld + c];
    }
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int e = base + (int)threadIdx.x + k * NT;
      if (e < n) {
        const int r = e / C, c = e - r * C;
        s[r * sld + c] = v[k];
      }
    }
  }
}
template <int NT, int UNR>
__device__ __forceinline__ void g2s_f1_T(const float* __restrict__ g, int64_t gld, float* s, int sld, int R, int C) {
  const int n = R * C;
  for (int base = 0; base < n; base += NT * UNR) {
    float v[UNR];
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int e = min(base + (int)threadIdx.x + k * NT, n - 1);
      const int r = e / C, c = e - r * C;
      v[k] = g[r * gld + c];
    }
#pragma unroll
    for (int k = 0; k < UNR; ++k) {
      const int e = base + (int)threadIdx.x + k * NT;
      if (e < n) {
        const int r = e / C, c = e - r * C;
        s[c * sld + r] = v[k];
      }
    }
  }
}
// zero s[R][c0..c1) (padding columns)
template <int NT>
__device__ __forceinline__ void zero_cols(float* s, int sld, int R, int c0, int c1) {
  const int w = c1 - c0;
  if (w <= 0) return;
  for (int e = threadIdx.x; e < R * w; e += NT) {
    const int r = e / w, c = e - r * w;
    s[r * sld + c0 + c] = 0.f;
  }
}

// X[row][col] of a tower input (numeric ++ embeddings), col < kp (zero pad)
__device__ __forceinline__ float tower_x(const TowerDev& T, int64_t drow, int col) {
  if (col < T.n_num) return T.num[drow * T.num_ld + col];
  if (col >= T.in_dim) return 0.f;
  const int c = col - T.n_num;
  const int j = c / T.emb_dim, e = c - j * T.emb_dim;
  int64_t code = T.cat[drow * T.cat_ld + j];
  code = code < 0 ? 0 : (code >= T.emb_rows[j] ? T.emb_rows[j] - 1 : code);
  return T.emb[j][code * T.emb_dim + e];
}

// ---------------------------------------------------------------------------
// gradient reduction / Adam arguments (tt_optim.hip)
// ---------------------------------------------------------------------------
#ifndef TT_MAX_SEG
#define TT_MAX_SEG 16  // was 48: 5.2 KB of kernel arguments per k_reduce_adam launch, now 1.9 KB
#endif
// segment capacity of a reduction (make_red adds at most 1 + 2 x 6 + 1 = 14)
constexpr int MAX_SEG = TT_MAX_SEG;
static_assert(MAX_SEG >= 14, "make_red's ranges: embeddings, 6 per tower, logit_scale");
#ifndef TT_RED_MINW
#define TT_RED_MINW 7  // waves per SIMD: <= 73 VGPRs (no spills with 16 loads in flight); 9.4 us vs 10.8 at 8
#endif
#ifndef TT_RED_E
#define TT_RED_E 64  // 64 x 8: 8.1 us vs 9.4 at 32 x 16 (cfg3, folded: every range <= 128 slabs)
#endif
constexpr int RED_E = TT_RED_E;    // elements per k_reduce_adam block
constexpr int RED_G = 512 / RED_E; // slab groups per element (512 threads, 16 slab loads in flight each)
constexpr int RED_UNR = 16;        // slab loads in flight per lane
// Seg kinds: 0 slab partials, 1 gacc, 2 replicas, 3 folded W0 (P | Q), 4
// folded b0, 5 slab partials of 129..256 slabs split in two slab halves:
// lanes el < 32 sum slabs [0, 128) of 32 elements, lanes el >= 32 the rest
// of the same elements (k_top_pair's 64-row W8 partials: every block then
// loads as much as a 128-slab block)

struct Seg {
  int64_t off, len;      // range in the parameter arena
  int64_t voff, vlen;    // range in k_reduce_adam's element space (kind 3: 2 len, 32-aligned)
  int64_t slab_off;      // offset of the range inside a tower slab (kind 0)
  // kind 0: slab partials, 1: atomic accumulator (gacc), 2: NREP replicas,
  // 3: W0 of the folded BN0 backward, 4: b0 of the folded BN0 backward
  int32_t kind, tower;
  int32_t n_slabs, keep; // partial slabs to sum (kinds 0, 3); keep: kind 2 leaves its replicas (no zeroing)
  float* rep;            // kinds 2-4: replica 0 of the range; replica r at + r * rep_stride
  int64_t rep_stride;
  int32_t in, kp;        // kinds 3, 4: tower input width, padded width (P|Q rows: 2 kp floats)
  const float *k0, *xsh; // kinds 3, 4: inv0*gamma0, shift row
};

// Data-parallel gradient exchange inside k_reduce_adam (tt_train_step_dp):
// every rank's exchange region mapped here (tt_ar_*; flags of the fused step
// [TT_AR_MAX_RANKS][blocks] after the standalone exchange's flags).
struct RedExchange {
  float* slot[TT_AR_MAX_RANKS];      // slot 0 of each rank's region (slot 1 at + slot_stride)
  uint64_t* flags[TT_AR_MAX_RANKS];  // each rank's fused-step flag array
  uint64_t* ll[TT_AR_MAX_RANKS];     // each rank's push words [2 parities][TT_AR_MAX_RANKS sources][slot_stride]
  int64_t slot_stride;
  int32_t rank, world, blocks;
  int32_t protocol;                  // TT_AR_PULL / TT_AR_PUSH (tt_ar_peers.protocol)
  int32_t* err;                      // set when a wait times out (sticky)
  uint64_t wait_ticks;               // wait bound in s_memrealtime ticks (100 MHz)
};

// Push protocol (TT_AR_PUSH): each exchanged element travels as ONE 8-byte
// word -- the float's bits in the low half, the epoch (the step, mod 2^32)
// in the high half -- stored by its owner straight into every peer's region
// (row [t & 1][source rank]); a reader polls its OWN region until every
// peer's word carries this epoch.  An aligned 8-byte store is single-copy
// atomic, so a word with the right epoch holds the right value: no separate
// flag, no release fence and no wait for the remote stores' completion
// before signalling (the pull protocol's publish -> flag -> remote read is
// three one-way trips; this is one).  Twice the bytes per element on the
// links.  Row reuse: rank r rewrites row [t & 1][r] of peer q at step t + 2,
// after its step-(t+1) reads saw q's step-(t+1) words, which q stored in a
// launch that began after its step-t reads ended (stream order).
__device__ __forceinline__ uint64_t ll_word(float v, uint32_t ep) {
  return ((uint64_t)ep << 32) | (uint64_t)__float_as_uint(v);
}
// owner lane: this rank's value of element e into every peer's row
__device__ __forceinline__ void ll_publish(uint64_t* const* ll, int world, int rank, int64_t row_stride,
                                           int64_t par, int64_t e, float v, uint32_t ep) {
  const uint64_t w = ll_word(v, ep);
  const int64_t off = (par * TT_AR_MAX_RANKS + rank) * row_stride + e;
  for (int q = 0; q < world; ++q)
    if (q != rank) __hip_atomic_store(ll[q] + off, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// wait (bounded) until every peer's word of this lane's EPT elements e[j]
// (live[j]) in this rank's own region carries epoch ep, then the rank-order
// sums with this rank's own terms from the registers -- the same adds as
// rank_order_sums, so both protocols give every rank bitwise the same mean.
// All EPT x W polls are in flight at once; only the words still stale are
// re-read.  False on timeout (out[] then undefined).
template <int W, int EPT>
__device__ __forceinline__ bool ll_gather_sums(const uint64_t* own_ll, int world, int rank, int64_t row_stride,
                                               int64_t par, const int64_t* e, const bool* live, const float* own,
                                               uint32_t ep, uint64_t t0, uint64_t bound, float* out) {
  uint64_t x[EPT][W];
  auto src = [&](int j, int r) {
    const int q = (r < world && r != rank) ? r : rank;  // inactive: this rank's own (unused) row, a valid address
    return own_ll + (par * TT_AR_MAX_RANKS + q) * row_stride + e[j];
  };
  auto want = [&](int j, int r) { return live[j] && r < world && r != rank; };
#pragma unroll
  for (int j = 0; j < EPT; ++j)
#pragma unroll
    for (int r = 0; r < W; ++r) x[j][r] = __hip_atomic_load(src(j, r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (;;) {
    bool done = true;
#pragma unroll
    for (int j = 0; j < EPT; ++j)
#pragma unroll
      for (int r = 0; r < W; ++r)
        if (want(j, r) && (uint32_t)(x[j][r] >> 32) != ep) done = false;
    if (done) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > bound) return false;
    __builtin_amdgcn_s_sleep(1);
#pragma unroll
    for (int j = 0; j < EPT; ++j)
#pragma unroll
      for (int r = 0; r < W; ++r)
        if (want(j, r) && (uint32_t)(x[j][r] >> 32) != ep)
          x[j][r] = __hip_atomic_load(src(j, r), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < W; ++r)
      if (r < world) s += r == rank ? own[j] : __uint_as_float((uint32_t)x[j][r]);
    out[j] = s;
  }
  return true;
}

// Rank-order sum of one exchanged element: the peers' slot values, this
// rank's own term from the register (the bits its slot holds).  All W loads
// are issued before the first add -- one s_waitcnt covers every peer's
// system-scope read, instead of one round trip per rank over xGMI -- and the
// adds run in rank order, so every rank computes bitwise the same sum.  W is
// a compile-time bound >= world; lanes r >= world (and r == rank) load this
// rank's own slot (a valid address, no branch around the load) and are
// skipped by the uniform select.
template <int W>
__device__ __forceinline__ float rank_order_sum(float* const* slot, int world, int rank, int64_t off, float own) {
  float x[W];
#pragma unroll
  for (int r = 0; r < W; ++r) {
    const int q = (r < world && r != rank) ? r : rank;
    x[r] = __hip_atomic_load(slot[q] + off, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  float s = 0.f;
#pragma unroll
  for (int r = 0; r < W; ++r)
    if (r < world) s += r == rank ? own : x[r];
  return s;
}
// the same for EPT elements per lane (k_ar_adam): EPT x W loads in flight
template <int W, int EPT>
__device__ __forceinline__ void rank_order_sums(float* const* slot, int world, int rank, const int64_t* off,
                                                const float* own, float* out) {
  float x[EPT][W];
#pragma unroll
  for (int j = 0; j < EPT; ++j)
#pragma unroll
    for (int r = 0; r < W; ++r) {
      const int q = (r < world && r != rank) ? r : rank;
      x[j][r] = __hip_atomic_load(slot[q] + off[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
#pragma unroll
  for (int j = 0; j < EPT; ++j) {
    float s = 0.f;
#pragma unroll
    for (int r = 0; r < W; ++r)
      if (r < world) s += r == rank ? own[j] : x[j][r];
    out[j] = s;
  }
}

// NS: segment capacity (the whole arena: MAX_SEG; a deferred late half,
// LateRed below: MAX_LATE_SEG -- it rides in k_l0_fwd's kernel arguments)
template <int NS>
struct RedArgsN {
  Seg seg[NS];
  // the segments in element-space (block) order: entry j covers blocks
  // [blk0[j], blk0[j + 1]) and is seg[blk_seg[j]] -- a block finds its
  // segment from these two compact arrays (one scalar-load round trip and
  // SALU compares) instead of walking seg[] with a dependent kernel-argument
  // load per segment (the last ranges paid ~12 of them: DESIGN 14b)
  int32_t blk0[NS];
  int32_t blk_seg[NS];
  int32_t n_seg;
  int32_t n_slabs;
  int64_t n;
  int64_t vn;            // k_reduce_adam elements (blocks = vn / RED_E)
  const float* slab[2];
  int64_t slab_ld;
  float* gacc;
  float* grad;
  float* zero_buf[4];
  int32_t zero_len[4];
  float* lsr;            // (dls, loss) replicas: loss folded into state->loss_sum
  tt_state* loss_state;
  int32_t apply_adam;
  float* p; float* m; float* v;
  double lr, b1, b2, eps;
  AdamSlot* adam_slots;  // non-null: coefficients from slot t & 1; segment next_seg fills t + 1's
  int32_t next_seg;
  tt_state* state;
  int64_t step_host;
  float inv_b;           // 1 / batch rows (kinds 3, 4)
  RedExchange x;         // k_reduce_adam<PRE, true>: mean over ranks before Adam
  // deferred late half (TT_FLAG_DEFER_LATE): the early half of step t
  // records t + 1 in *late_pending (0: nothing deferred; a zeroed workspace
  // holds 0); a late half runs only when *late_pending == state->step_done + 1,
  // and takes its Adam step from step_done (k_l0_fwd of step t + 1 rewrites
  // step_cur meanwhile)
  int64_t* late_pending;
  int32_t late_mark;     // early half: 1 records t + 1 (deferring), -1 records 0 (not deferring), 0 leaves it
};
using RedArgs = RedArgsN<MAX_SEG>;
constexpr int MAX_LATE_SEG = 8;
using LateRed = RedArgsN<MAX_LATE_SEG>;
constexpr int LATE_G = 4;  // slab groups of a late-half block: 64 elements x 4 = k_l0_fwd's 256 threads

}  // namespace tt
