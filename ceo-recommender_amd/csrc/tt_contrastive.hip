// Contrastive scoring (gfx950): symmetric InfoNCE forward/backward over the
// full firm x CEO similarity matrix, and retrieval ranks.
//
// Reference: contrastive.py:102-138 (info_nce_loss: S = F C^T / tau,
// (CE(S, diag) + CE(S^T, diag)) / 2) and contrastive.py:275-332
// (compute_retrieval_metrics: rank of the diagonal in each row of F C^T).
// SURVEY 8a rows a18/a19, BASELINE cfg 5 (100k x 100k, D = 256).
//
// MFMA-bound: three fp32 GEMMs of 2 M N D flops each (fp32-accurate on the
// bf16x3 core below, v_mfma_f32_16x16x32_bf16), never materialising S as
// logits:
//   k_nce_sim  : S tile = F C^T (K = D) -> E = exp(S/tau - shift) stored in
//                16x16 MFMA-accumulator tiles (one coalesced 1 KB store per
//                tile), deterministic row / column partial sums of E, diag.
//   k_nce_dgrad: dF = E'C and dC = E'^T F with E' = E (1/rowsum_i +
//                1/colsum_j), E streamed from HBM (split-K partials).
//   reduce     : sums, log-sum-exp, loss, diagonal terms, scaling.
// One shared exponent per element serves both softmaxes: with the fixed
// shift = max|f| max|c| / tau >= every S_ij, row sums and column sums are
// plain sums (no running max; column partials of different row blocks and
// different ranks simply add).  L2-normalised inputs give shift = 1/tau and
// every term >= exp(-2/tau); sums that still underflow (far-from-normalised
// inputs) are counted in a status word instead of silently returning inf.
//
// Robust mode (the caller's fallback when that status is set: temperatures
// far below 0.03 on normalised inputs, or unnormalised projections): exact
// per-row and per-column maxima first (k_nce_sim<3>), then row sums of
// exp(s - rowmax_i) and column sums of exp(s - colmax_j) -- two exponentials
// per element -- with the logits s themselves kept for the backward
// (k_nce_sim<4>); the backward stages E' = exp(s - lse_i) + exp(s - lse_j)
// from the row / column log-sum-exps (k_nce_dgrad<SA, true>).
#include "tt_common.h"

namespace tt {
namespace nce {

constexpr int BK = 32, WM = 64, TM = WM / 16;  // K chunk; waves own WM rows = 4 MFMA row tiles
// Block shapes: BM x BN output tiles, 8 waves of WM x WN (TN = WN / 16 column
// tiles per wave), one block per CU.
//  * gradient kernels, Cfg<256, 256, 128>: one 120 KB LDS stage (padded
//    k-major layout); the next chunk's global loads fly during the MFMAs, its
//    split and LDS writes wait for the barrier after them;
//  * similarity kernels: the same (default), or with TT_NCE_SIM_DB=1
//    Cfg<256, 128, 64> with TWO 72 KB stages -- chunk c + 1 is split into
//    planes and written to one stage while chunk c's MFMAs run from fragments
//    already read out of the other, one barrier per chunk.  Measured at
//    N = 100k, D = 256 (tools/gpu_nce_ab.sh): fwd 31.8 vs 29.2 ms, ranks 28.6
//    vs 24.4 ms -- with K = 256 a block runs only 8 chunks, so the halved tile
//    pays its prologue / epilogue twice as often and splits 1.5x the operand
//    floats per output (1.4 VALU per MFMA, beyond the 2 issue slots an MFMA
//    leaves once address math is counted).
// Every element's K order and six-product order are the same in both, so the
// similarity values (and k_nce_diag's replay of them) are bitwise unchanged.
template <int BM_, int BN_, int WN_, int NP_ = 0> struct Cfg {
  static constexpr int BM = BM_, BN = BN_, WN = WN_, TN = WN_ / 16;
  static constexpr int NWM = BM_ / WM, NWN = BN_ / WN_, NW = NWM * NWN;  // MFMA waves
  static constexpr int NP = NP_;                                          // producer waves (warp-specialised)
  static constexpr int NTH = (NW + NP_) * 64;
  static_assert(NW + NP_ == 8, "8 waves");
};
#ifndef TT_NCE_SIM_DB
#define TT_NCE_SIM_DB 0
#endif
// Warp-specialised similarity kernels (round 3): 128 x 256 block tiles,
// waves 0-3 run only MFMAs (64 x 128 each) from one LDS stage while waves 4-7
// load, split into bf16 planes and store the next K chunk into the other
// stage -- two 72 KB stages, one barrier per chunk.  On each SIMD one
// MFMA-only wave sits beside one VALU / memory wave, whose split work fills
// the vector-issue slots the MFMAs leave (MI355X_MICROARCH.md: separate
// pipes, 8 of the 16 cycles of a 16x16x32 MFMA free for vector issue).
#ifndef TT_NCE_WS
#define TT_NCE_WS 0  // measured slower (r03: fwd 34.2 vs 29.6 ms, ranks 31.8 vs 25.5 ms)
#endif
// fp32 operand stages (round 6, measured, not the default): the similarity kernels stage
// raw fp32 tiles in LDS -- 64 KB per 256 x 256 x 32 stage instead of 96 KB of
// bf16 planes -- so TWO stages fit: chunk c + 1 is copied in (global -> VGPR
// -> ds_write_b128, no arithmetic) while chunk c's MFMAs run, one barrier per
// chunk, and each wave splits its own fragments into the three bf16 planes
// right after reading them (3x the split work of splitting at staging, but
// issued between the MFMAs, not in a phase of its own).  Same plane values,
// same K order and six-product order: bitwise the same similarities.
// Measured (tools/gpu_nce_check.sh, two interleaved rounds, N = 100k, D =
// 256; contrastive GPU tests green): forward 28.2 -> 32.2 ms, ranks 23.9 ->
// 27.8 ms -- each wave splits its 4 A and 8 B fragments itself, 3x the VALU
// of the single split at staging (B tiles split by all 4 M-waves), and the A
// fragments' split at the top of each chunk is not hidden.
#ifndef TT_NCE_F32LDS
#define TT_NCE_F32LDS 0  // measured slower (round 6: fwd 28.2 -> 32.2 ms, ranks 23.9 -> 27.8 ms at N = 100k, D = 256)
#endif
#if TT_NCE_WS
using CfgSim = Cfg<128, 256, 128, 4>;
#elif TT_NCE_SIM_DB
using CfgSim = Cfg<256, 128, 64>;
#else
using CfgSim = Cfg<256, 256, 128>;
#endif
using CfgGrad = Cfg<256, 256, 128>;
#ifndef TT_NCE_PIPE
// the similarity kernels' gemm_loop reads B fragments one tile ahead of the
// MFMAs (cfg 5: fwd 28.2 -> 27.9 ms, ranks 23.9 -> 23.6 ms); the gradient
// kernels do not (their dF / dC loop measured 57.2 -> 65.8 ms with it)
#define TT_NCE_PIPE 1
#endif
constexpr int TILE = 256;                                    // floats per 16x16 tile
constexpr float SUM_MIN = 1e-30f;  // row/col sums below this: exp underflow (reported)

// Operand precision: fp32 through the bf16 MFMA.  Each fp32 value x is
// split exactly into three bf16 planes x = h + m + l (8 significand bits
// each, round-to-nearest), and a product is the six plane products whose
// magnitude is >= 2^-16 of h*h:
//     x*y ~= l*h + m*m + h*l + m*h + h*m + h*h
// (the dropped m*l, l*m, l*l terms are <= ~2^-24 relative, i.e. fp32's own
// rounding).  Every plane product is exact in the fp32 accumulator, so the
// GEMM is fp32-accurate while running v_mfma_f32_16x16x32_bf16: 6 MFMAs of
// 16 cycles per 32-deep K step instead of 8 fp32 MFMAs of 32 cycles (2.7x).
// The split happens once per element while staging into LDS.
constexpr int NPL = 3;                // planes h, m, l
// LDS operand images [plane][m][k] bf16, two layouts:
//  * SWZ (both operands row-major along k, the similarity kernels): 64-B rows,
//    16-B granule c of row m stored at c ^ swz(m), swz = [0,2,3,1][(m >> 2) & 3]:
//    every 16-lane group of a ds_read_b128 fragment read (rows r, granule g)
//    hits 16 distinct 16-B slots of the 256-B bank window (MI355X_MICROARCH.md
//    LDS table) -- conflict-free reads and row-contiguous staging writes;
//  * padded (the gradient kernels, whose k-major staging writes 16 rows at one
//    k): 80-B rows.
template <bool SWZ, int ROWS> struct Lay {
  static constexpr int LDK = SWZ ? BK : BK + 8;  // bf16 per LDS row
  static constexpr int PLANE = ROWS * LDK;       // bf16 per plane of one operand
  static constexpr int OPND = NPL * PLANE;       // bf16 per operand
};
__device__ __forceinline__ int lds_swz(int m) { return (0x78 >> (2 * ((m >> 2) & 3))) & 3; }
template <bool SWZ>
__device__ __forceinline__ int lds_off(int m, int k) {  // bf16 offset of (m, k) in a plane
  if constexpr (SWZ) return m * Lay<SWZ, 1>::LDK + ((((k >> 3) ^ lds_swz(m)) << 3) | (k & 7));
  else return m * Lay<SWZ, 1>::LDK + k;
}
// one stage = A (BM rows) + B (BN rows), in bf16 elements
template <class C, bool SWZ>
constexpr int stage_elems() { return Lay<SWZ, C::BM>::OPND + Lay<SWZ, C::BN>::OPND; }
constexpr size_t LDS_SIM = (TT_NCE_F32LDS && !TT_NCE_WS && !TT_NCE_SIM_DB)
    ? sizeof(float) * 2 * (CfgSim::BM + CfgSim::BN) * BK                                       // 128 KB
    : sizeof(uint16_t) * ((TT_NCE_SIM_DB || TT_NCE_WS) ? 2 : 1) * stage_elems<CfgSim, true>();  // 96 / 144 KB
constexpr size_t LDS_GRAD = sizeof(uint16_t) * stage_elems<CfgGrad, false>();                        // 120 KB
static_assert(LDS_SIM <= 160 * 1024 && LDS_GRAD <= 160 * 1024, "LDS per CU");


// Where an operand comes from.  LDS always holds [m][k] bf16 planes.
enum Src : int {
  // every source hands a thread 4 (SRC_KROWS: 8) consecutive k, so the split
  // planes are written along k (8- / 16-byte LDS writes, no transposition)
  SRC_MK = 0,       // row-major G[m][k] (ld): one float4 along k
  SRC_E_AS_MK = 3,  // E tiles, m = E col j, k = E row i: the tile's float4 (4 rows i)  (dC = E'^T F)
  SRC_KROWS = 4,    // row-major G[k][m] (ld): 8 scalar loads down k, lanes along m (coalesced)
  SRC_E_ROWS = 5,   // E tiles, m = E row i, k = E col j: the tile float4, quad-transposed (dF = E' C)
};

// Buffer resources (SGPR base + 32-bit lane offsets; reads outside
// [0, bytes) return 0, which zero-fills every partial tile for free).
constexpr uint32_t BUF_OOB = 0xFFFFFFFFu;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p, int64_t bytes) {
  const int64_t nb = bytes < 0 ? 0 : (bytes > 0x7FFFFFFF ? 0x7FFFFFFF : bytes);
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)nb, 0x00020000);
}
__device__ __forceinline__ float buf_f32(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));  // the builtin returns the bits
}
__device__ __forceinline__ float4 buf_f32x4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

struct Opnd {
  const float* p;
  int64_t ld;      // row stride (SRC_MK / SRC_KROWS)
  int64_t mdim;    // extent along m (rows of the output side)
  int64_t kdim;    // extent along k
  int64_t nti, ntj;  // E tile grid (SRC_E_*)
  const float* a;  // E row scale (1/rowsum_i, padded)  (SRC_E_*); robust mode: row log-sum-exp
  const float* b;  // E col scale (1/colsum_j, padded);  robust mode: column log-sum-exp
};

struct GemmArgs {
  Opnd A, B;
  int64_t M, N;        // output extent
  int64_t k_per_split; // multiple of BK
  int n_blocks_n;      // blocks along N
  // sim epilogue
  float inv_tau;
  const float* shift;  // device scalar
  float* E;            // tiles [nti][ntj][256]
  int64_t e_nti, e_ntj;
  float* rowpart;      // [N / WN parts][M_pad] (WN of CfgSim)
  float* colpart;      // [M / WM parts][N_pad]
  int64_t m_pad, n_pad;
  int64_t row0;        // global index of local row 0 (diagonal j == row0 + i)
  // rank epilogue
  const float* diag;   // [M] raw sim_ii (GEMM-identical arithmetic)
  int* rank_cnt;       // [M]
  // grad epilogue
  float* part;         // [split][M_tiles][N_tiles][256]
  int64_t p_nti, p_ntj;
  // triplet (semi-hard mining) epilogue
  float margin;
  uint64_t* semi_part;  // [N / WN parts][M_pad] min key over semi-hard negatives
  uint64_t* all_part;   // [N / WN parts][M_pad] min key over all negatives
  // robust mode (MODE 4): exact row maxima [M_pad] and column maxima [N_pad] of s
  const float* rmax;
  const float* cmax;
};

// Orderable 64-bit key of a distance and its column: the float bits mapped
// to an unsigned order (negative values flipped), column in the low word --
// the minimum key is the smallest distance, ties to the lowest column.
constexpr uint64_t KEY_NONE = ~0ull;
__device__ __forceinline__ uint32_t ord_f32(float x) {
  const uint32_t u = __float_as_uint(x);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unord_f32(uint32_t k) {
  return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const int lo = __builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, false);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}
// min over the 16 lanes (r) that share a row group g (DPP, no LDS)
__device__ __forceinline__ uint64_t row_min16(uint64_t v) {
  uint64_t o;
  o = dpp_u64<0xB1>(v);  v = o < v ? o : v;   // quad_perm [1,0,3,2]
  o = dpp_u64<0x4E>(v);  v = o < v ? o : v;   // quad_perm [2,3,0,1]
  o = dpp_u64<0x141>(v); v = o < v ? o : v;   // row_half_mirror
  o = dpp_u64<0x140>(v); v = o < v ? o : v;   // row_mirror
  return v;
}

// max over the 16 lanes of a row group / over the 4 row groups of a column
__device__ __forceinline__ float row_max16(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));
  v = fmaxf(v, dpp_mov<0x4E>(v));
  v = fmaxf(v, dpp_mov<0x141>(v));
  v = fmaxf(v, dpp_mov<0x140>(v));
  return v;
}
__device__ __forceinline__ float col_max4(float v) {
  unsigned u = __float_as_uint(v);
  auto p = __builtin_amdgcn_permlane16_swap(u, u, false, false);
  unsigned lo = p[0], hi = p[1];
  v = fmaxf(__uint_as_float(lo), __uint_as_float(hi));
  u = __float_as_uint(v);
  auto p2 = __builtin_amdgcn_permlane32_swap(u, u, false, false);
  lo = p2[0];
  hi = p2[1];
  return fmaxf(__uint_as_float(lo), __uint_as_float(hi));
}

// ---- global -> registers (4 float4 per thread per operand per K chunk) ----
// (ROWS x BK floats per operand tile, NT threads: ROWS * 8 / NT float4 each)
// E' staging: default x (a_i + b_j) with a, b the reciprocal row / column
// sums of E = exp(s - shift); robust (LSE) mode exp(x - a_i) + exp(x - b_j)
// with x = s and a, b the row / column log-sum-exps (0 outside the tiles).
template <bool LSE>
__device__ __forceinline__ float ep(float x, float ai, float bj, bool ok) {
  if constexpr (LSE) return ok ? __expf(x - ai) + __expf(x - bj) : 0.f;
  else return x * (ai + bj);
}

template <int S, int ROWS, int NT, bool LSE = false>
__device__ __forceinline__ void load_opnd(const Opnd& o, int64_t m0, int64_t k0, float4 (&v)[ROWS * 8 / NT]) {
  constexpr int NQ = ROWS * 8 / NT;
  if constexpr (S == SRC_MK) {  // tile ROWS x BK from G[m][k]: 4 k-octets (2 float4) per row
    const auto rs = buf_rsrc(o.p + m0 * o.ld, (o.mdim - m0) * o.ld * 4);
#pragma unroll
    for (int t = 0; t < NQ / 2; ++t) {
      const int e = (int)threadIdx.x + t * NT;
      const int r = e >> 2, k8 = (e & 3) * 8;
      const bool ok0 = k0 + k8 < o.kdim, ok1 = k0 + k8 + 4 < o.kdim;
      v[2 * t] = buf_f32x4(rs, ok0 ? (uint32_t)((r * o.ld + k0 + k8) * 4) : BUF_OOB);
      v[2 * t + 1] = buf_f32x4(rs, ok1 ? (uint32_t)((r * o.ld + k0 + k8 + 4) * 4) : BUF_OOB);
    }
  } else if constexpr (S == SRC_KROWS) {  // G[k][m]: ROWS m (lanes) x 4 k-octets, 8 scalar loads
    // (an item is 8 consecutive k = one 16-B LDS granule per plane, v[2t] | v[2t + 1])
    const auto rs = buf_rsrc(o.p + k0 * o.ld, (o.kdim - k0) * o.ld * 4);
#pragma unroll
    for (int t = 0; t < NQ / 2; ++t) {
      const int e = (int)threadIdx.x + t * NT;
      const int ml = e % ROWS, k8 = (e / ROWS) * 8;
      const bool ok = m0 + ml < o.mdim;
      float x[8];
#pragma unroll
      for (int c = 0; c < 8; ++c)
        x[c] = buf_f32(rs, ok ? (uint32_t)(((k8 + c) * o.ld + m0 + ml) * 4) : BUF_OOB);
      v[2 * t] = make_float4(x[0], x[1], x[2], x[3]);
      v[2 * t + 1] = make_float4(x[4], x[5], x[6], x[7]);
    }
  } else if constexpr (S == SRC_E_ROWS) {  // E tiles as [m = i][k = j]: ROWS/16 i-tiles x 2 j-tiles
    // one coalesced float4 per lane (4 rows i at one column j, the MFMA
    // accumulator layout k_nce_sim stored), quad-transposed in registers to
    // 4 consecutive j of one row i
    const int64_t ti0 = m0 >> 4, tj0 = k0 >> 4;
    const int64_t tiles = (o.nti - ti0) * o.ntj - tj0;  // tiles from (ti0, tj0) to the end of E
    const auto rs = buf_rsrc(o.p + (ti0 * o.ntj + tj0) * TILE, tiles * TILE * 4);
    const auto ra = buf_rsrc(o.a, o.nti * 16 * 4), rb = buf_rsrc(o.b, o.ntj * 16 * 4);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int e = (int)threadIdx.x + q * NT;
      const int t = e >> 6, ln = e & 63;
      const int tm = t >> 1, tk = t & 1;
      const int64_t ti = ti0 + tm, tj = tj0 + tk;
      const bool ok = ti < o.nti && tj < o.ntj;
      const f32x4 x = quad_transpose(__builtin_bit_cast(
          f32x4, buf_f32x4(rs, ok ? (uint32_t)(((tm * o.ntj + tk) * TILE + ln * 4) * 4) : BUF_OOB)));
      const float ai = buf_f32(ra, ok ? (uint32_t)((ti * 16 + 4 * (ln >> 4) + (ln & 3)) * 4) : BUF_OOB);
      const float4 bj = buf_f32x4(rb, ok ? (uint32_t)((tj * 16 + (ln & 12)) * 4) : BUF_OOB);
      v[q] = make_float4(ep<LSE>(x[0], ai, bj.x, ok), ep<LSE>(x[1], ai, bj.y, ok), ep<LSE>(x[2], ai, bj.z, ok),
                         ep<LSE>(x[3], ai, bj.w, ok));
    }
  } else if constexpr (S == SRC_E_AS_MK) {  // E tiles as [m = j][k = i]: ROWS/16 j-tiles x 2 i-tiles
    const int64_t tj0 = m0 >> 4, ti0 = k0 >> 4;
    const int64_t tiles = (o.nti - ti0) * o.ntj - tj0;
    const auto rs = buf_rsrc(o.p + (ti0 * o.ntj + tj0) * TILE, tiles * TILE * 4);
    const auto ra = buf_rsrc(o.a, o.nti * 16 * 4), rb = buf_rsrc(o.b, o.ntj * 16 * 4);
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int e = (int)threadIdx.x + q * NT;
      const int t = e >> 6, ln = e & 63;
      const int tm = t >> 1, tk = t & 1;
      const int64_t tj = tj0 + tm, ti = ti0 + tk;
      const bool ok = ti < o.nti && tj < o.ntj;
      const float4 x = buf_f32x4(rs, ok ? (uint32_t)(((tk * o.ntj + tm) * TILE + ln * 4) * 4) : BUF_OOB);
      const float4 ai = buf_f32x4(ra, ok ? (uint32_t)((ti * 16 + 4 * (ln >> 4)) * 4) : BUF_OOB);
      const float bj = buf_f32(rb, ok ? (uint32_t)((tj * 16 + (ln & 15)) * 4) : BUF_OOB);
      v[q] = make_float4(ep<LSE>(x.x, ai.x, bj, ok), ep<LSE>(x.y, ai.y, bj, ok), ep<LSE>(x.z, ai.z, bj, ok),
                         ep<LSE>(x.w, ai.w, bj, ok));
    }
  }
}

// split the staged float4s into the three bf16 planes of LDS [m][k]
template <int S, bool SWZ, int ROWS, int NT>
__device__ __forceinline__ void store_opnd(uint16_t* L, const float4 (&v)[ROWS * 8 / NT]) {
  constexpr int PLANE = Lay<SWZ, ROWS>::PLANE;
  if constexpr (S == SRC_KROWS || S == SRC_MK) {
    // one k-octet per item: a 16-B granule per plane.  SRC_KROWS: lanes run
    // along m at one octet -- 16-B writes of 80-B rows hit 16 distinct 16-B
    // slots per 16 lanes (8-B writes of 4 k would pair rows m and m + 16 on
    // one bank); SRC_MK: 4 lanes per 64-B swizzled row, 16 lanes = 256 B.
    // Half the write instructions of 8-B plane writes.
#pragma unroll
    for (int t = 0; t < ROWS * 4 / NT; ++t) {
      const int e = (int)threadIdx.x + t * NT;
      const int m = S == SRC_KROWS ? e % ROWS : e >> 2;
      const int k8 = S == SRC_KROWS ? (e / ROWS) * 8 : (e & 3) * 8;
      const float x[8] = {v[2 * t].x,     v[2 * t].y,     v[2 * t].z,     v[2 * t].w,
                          v[2 * t + 1].x, v[2 * t + 1].y, v[2 * t + 1].z, v[2 * t + 1].w};
      bf16x8 pl[NPL];
      split8x3(x, pl);
      uint16_t* d = L + lds_off<SWZ>(m, k8);
      *reinterpret_cast<bf16x8*>(d) = pl[0];
      *reinterpret_cast<bf16x8*>(d + PLANE) = pl[1];
      *reinterpret_cast<bf16x8*>(d + 2 * PLANE) = pl[2];
    }
    return;
  }
#pragma unroll
  for (int q = 0; q < ROWS * 8 / NT; ++q) {
    const int e = (int)threadIdx.x + q * NT;
    int m, k;  // the thread's float4 holds k .. k+3 of row m
    if constexpr (S == SRC_E_ROWS) {  // quad-transposed tile float4: row i, 4 consecutive j
      const int t = e >> 6, ln = e & 63, tm = t >> 1, tk = t & 1;
      m = 16 * tm + 4 * (ln >> 4) + (ln & 3); k = 16 * tk + (ln & 12);
    } else {  // SRC_E_AS_MK: the tile float4 = 4 consecutive E rows i = k
      const int t = e >> 6, ln = e & 63, tm = t >> 1, tk = t & 1;
      m = 16 * tm + (ln & 15); k = 16 * tk + 4 * (ln >> 4);
    }
    uint32_t h01, m01, l01, h23, m23, l23;  // packed bf16 pairs of the three planes
    split3x2(v[q].x, v[q].y, h01, m01, l01);
    split3x2(v[q].z, v[q].w, h23, m23, l23);
    uint16_t* d = L + lds_off<SWZ>(m, k);  // one 8-byte write per plane
    *reinterpret_cast<uint2*>(d) = make_uint2(h01, h23);
    *reinterpret_cast<uint2*>(d + PLANE) = make_uint2(m01, m23);
    *reinterpret_cast<uint2*>(d + 2 * PLANE) = make_uint2(l01, l23);
  }
}

// MFMA operand: 8 consecutive k (k = kk + 8g .. +7) of row m, one plane
template <bool SWZ, int ROWS>
__device__ __forceinline__ bf16x8 frag(const uint16_t* L, int plane, int m, int g) {
  return *reinterpret_cast<const bf16x8*>(L + plane * Lay<SWZ, ROWS>::PLANE + lds_off<SWZ>(m, 8 * g));
}


// Main loop: acc[TM][TN] += A[m0.., k-range] B[n0.., k-range]^T.  One LDS
// stage; the next chunk's global loads are in flight during the MFMAs of the
// current one.
template <int SA, int SB, class C, bool LSE = false, bool PIPE = false>
__device__ __forceinline__ void gemm_loop(const GemmArgs& g_, int64_t m0, int64_t n0, int64_t kb, int64_t ke,
                                          uint16_t* smem, f32x4 (&acc)[TM][C::TN]) {
  constexpr int NT = C::NTH, BM_ = C::BM, BN = C::BN, TN = C::TN, WN = C::WN;
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  const int wm = w / C::NWN, wn = w % C::NWN;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();
  float4 va[BM_ * 8 / NT], vb[BN * 8 / NT];
  const int nch = (int)((ke - kb + BK - 1) / BK);
  if (nch <= 0) return;
  constexpr bool SWZ = SA == SRC_MK && SB == SRC_MK;
  uint16_t* As = smem;
  uint16_t* Bs = smem + Lay<SWZ, BM_>::OPND;
  load_opnd<SA, BM_, NT, LSE>(g_.A, m0, kb, va);
  load_opnd<SB, BN, NT>(g_.B, n0, kb, vb);
  for (int c = 0; c < nch; ++c) {
    __syncthreads();  // the previous chunk's fragments have been read
    store_opnd<SA, SWZ, BM_, NT>(As, va);
    store_opnd<SB, SWZ, BN, NT>(Bs, vb);
    __syncthreads();
    if (c + 1 < nch) {
      load_opnd<SA, BM_, NT, LSE>(g_.A, m0, kb + (int64_t)(c + 1) * BK, va);
      load_opnd<SB, BN, NT>(g_.B, n0, kb + (int64_t)(c + 1) * BK, vb);
    }
    bf16x8 a[TM][NPL];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int p = 0; p < NPL; ++p) a[i][p] = frag<SWZ, BM_>(As, p, wm * WM + 16 * i + r, g);
    if constexpr (PIPE) {
    // B fragments one tile ahead: tile j + 1's LDS reads are issued before
    // tile j's 24 MFMAs (pinned by scheduling barriers), so their latency
    // hides behind them instead of ahead of every tile's first MFMA
    bf16x8 b[2][NPL];
#pragma unroll
    for (int p = 0; p < NPL; ++p) b[0][p] = frag<SWZ, BN>(Bs, p, wn * WN + r, g);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (j + 1 < TN) {
#pragma unroll
        for (int p = 0; p < NPL; ++p) b[(j + 1) & 1][p] = frag<SWZ, BN>(Bs, p, wn * WN + 16 * (j + 1) + r, g);
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][j] = mfma_bf16(a[i][PA[q]], b[j & 1][PB[q]], acc[i][j]);
      __builtin_amdgcn_sched_barrier(0);
    }
    } else {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bf16x8 b[NPL];
#pragma unroll
      for (int p = 0; p < NPL; ++p) b[p] = frag<SWZ, BN>(Bs, p, wn * WN + 16 * j + r, g);
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][j] = mfma_bf16(a[i][PA[q]], b[PB[q]], acc[i][j]);
    }
    }
  }
}

// Double-buffered main loop of the similarity kernels (both operands SRC_MK,
// swizzled LDS): stage c & 1 holds chunk c, the registers chunk c + 1.  Each
// iteration reads all of chunk c's fragments (24 x 16 B per lane), then splits
// and writes chunk c + 1 into the other stage and issues chunk c + 2's loads --
// VALU and LDS writes the scheduler interleaves with chunk c's 96 MFMAs, which
// depend only on registers -- and ends with the one barrier.  Loads past K
// return zeros (buffer range), so the body has no branches.
template <class C>
__device__ __forceinline__ void gemm_loop_db(const GemmArgs& g_, int64_t m0, int64_t n0, uint16_t* smem,
                                             f32x4 (&acc)[TM][C::TN]) {
  constexpr int NT = C::NTH, TN = C::TN;
  constexpr int AOP = Lay<true, C::BM>::OPND, STAGE = stage_elems<C, true>();
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  const int wm = w / C::NWN, wn = w % C::NWN;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();
  const int nch = (int)((g_.A.kdim + BK - 1) / BK);
  if (nch <= 0) return;
  float4 va[C::BM * 8 / NT], vb[C::BN * 8 / NT];
  auto fetch = [&](int c) {
    load_opnd<SRC_MK, C::BM, NT>(g_.A, m0, (int64_t)c * BK, va);
    load_opnd<SRC_MK, C::BN, NT>(g_.B, n0, (int64_t)c * BK, vb);
  };
  auto put = [&](uint16_t* S) {
    store_opnd<SRC_MK, true, C::BM, NT>(S, va);
    store_opnd<SRC_MK, true, C::BN, NT>(S + AOP, vb);
  };
  bf16x8 a[TM][NPL], b[TN][NPL];
  auto frags = [&](const uint16_t* S) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int p = 0; p < NPL; ++p) a[i][p] = frag<true, C::BM>(S, p, wm * WM + 16 * i + r, g);
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int p = 0; p < NPL; ++p) b[j][p] = frag<true, C::BN>(S + AOP, p, wn * C::WN + 16 * j + r, g);
  };
  auto mma = [&]() {
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][j] = mfma_bf16(a[i][PA[q]], b[j][PB[q]], acc[i][j]);
  };
  fetch(0);
  put(smem);
  fetch(1);
  __syncthreads();
  for (int c = 0; c + 1 < nch; ++c) {
    frags(smem + (c & 1) * STAGE);
    put(smem + ((c + 1) & 1) * STAGE);  // its readers (chunk c - 1) passed the last barrier
    fetch(c + 2);
    mma();
    __syncthreads();
  }
  frags(smem + ((nch - 1) & 1) * STAGE);
  mma();
}

// fp32-stage main loop (TT_NCE_F32LDS, both operands SRC_MK).  Stage layout:
// A rows [BM][32 floats] then B rows [BN][32 floats]; 16-B granule q of row m
// sits at q ^ f32_swz(m) -- a table found by search against the gfx950
// ds_read_b128 lane groups (MI355X_MICROARCH.md LDS table): the fragment
// reads (lane (r, g): row 16t + r, granules 2g and 2g + 1) are conflict-free,
// and so are the staging writes (4 lanes per row, one granule each).
__device__ __forceinline__ int f32_swz(int m) {
  // rows 0..15: 7 6 3 3 6 6 4 2 7 3 2 0 2 7 1 5 (3 bits each)
  constexpr uint64_t T = 7ull | 6ull << 3 | 3ull << 6 | 3ull << 9 | 6ull << 12 | 6ull << 15 | 4ull << 18 |
                         2ull << 21 | 7ull << 24 | 3ull << 27 | 2ull << 30 | 0ull << 33 | 2ull << 36 | 7ull << 39 |
                         1ull << 42 | 5ull << 45;
  return (int)((T >> (3 * (m & 15))) & 7);
}
__device__ __forceinline__ int f32_off(int m, int q) { return m * BK + ((q ^ f32_swz(m)) << 2); }

// 8 consecutive k (k-octet g) of row m from an fp32 stage, split into planes
__device__ __forceinline__ void frag32(const float* S, int m, int g, bf16x8 (&pl)[NPL]) {
  const float4 u = *reinterpret_cast<const float4*>(S + f32_off(m, 2 * g));
  const float4 v = *reinterpret_cast<const float4*>(S + f32_off(m, 2 * g + 1));
  const float x[8] = {u.x, u.y, u.z, u.w, v.x, v.y, v.z, v.w};
  split8x3(x, pl);
}

template <class C>
__device__ __forceinline__ void gemm_loop_f32(const GemmArgs& g_, int64_t m0, int64_t n0, float* smem,
                                              f32x4 (&acc)[TM][C::TN]) {
  constexpr int NT = C::NTH, TN = C::TN, BM_ = C::BM, BN = C::BN;
  constexpr int STAGE = (BM_ + BN) * BK;  // floats
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  const int wm = w / C::NWN, wn = w % C::NWN;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();
  const int nch = (int)((g_.A.kdim + BK - 1) / BK);
  if (nch <= 0) return;
  float4 va[BM_ * 8 / NT], vb[BN * 8 / NT];
  auto fetch = [&](int c) {  // loads past K return zeros (buffer range)
    load_opnd<SRC_MK, BM_, NT>(g_.A, m0, (int64_t)c * BK, va);
    load_opnd<SRC_MK, BN, NT>(g_.B, n0, (int64_t)c * BK, vb);
  };
  auto put = [&](float* S) {  // item e: row e >> 2, granules 2 (e & 3) and + 1
#pragma unroll
    for (int t = 0; t < BM_ * 4 / NT; ++t) {
      const int e = (int)threadIdx.x + t * NT, m = e >> 2, q = 2 * (e & 3);
      *reinterpret_cast<float4*>(S + f32_off(m, q)) = va[2 * t];
      *reinterpret_cast<float4*>(S + f32_off(m, q + 1)) = va[2 * t + 1];
    }
    float* SB = S + BM_ * BK;
#pragma unroll
    for (int t = 0; t < BN * 4 / NT; ++t) {
      const int e = (int)threadIdx.x + t * NT, m = e >> 2, q = 2 * (e & 3);
      *reinterpret_cast<float4*>(SB + f32_off(m, q)) = vb[2 * t];
      *reinterpret_cast<float4*>(SB + f32_off(m, q + 1)) = vb[2 * t + 1];
    }
  };
  fetch(0);
  put(smem);
  if (nch > 1) fetch(1);
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const float* S = smem + (c & 1) * STAGE;
    // chunk c + 1 into the other stage (its readers, chunk c - 1, passed the
    // last barrier) and chunk c + 2's loads in flight, beside chunk c's MFMAs
    if (c + 1 < nch) {
      put(smem + ((c + 1) & 1) * STAGE);
      if (c + 2 < nch) fetch(c + 2);
    }
    bf16x8 a[TM][NPL];
#pragma unroll
    for (int i = 0; i < TM; ++i) frag32(S, wm * WM + 16 * i + r, g, a[i]);
    bf16x8 b[2][NPL];
    frag32(S + BM_ * BK, wn * C::WN + r, g, b[0]);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if (j + 1 < TN) frag32(S + BM_ * BK, wn * C::WN + 16 * (j + 1) + r, g, b[(j + 1) & 1]);
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][j] = mfma_bf16(a[i][PA[q]], b[j & 1][PB[q]], acc[i][j]);
    }
    __syncthreads();
  }
}

// Warp-specialised main loop (TT_NCE_WS, both operands SRC_MK, swizzled LDS):
// stage c & 1 holds chunk c.  Producer waves (w >= NW) stored chunk c + 1
// into stage (c + 1) & 1 and issue chunk c + 2's loads while the MFMA waves
// consume stage c & 1; one barrier per chunk separates the two (the stage a
// producer writes in iteration c was last read in iteration c - 1).  The
// MFMA waves' per-element K order and six-product order are the single-stage
// loop's, so every similarity value (and k_nce_diag's replay) is unchanged.
template <int ROWS>
__device__ __forceinline__ void ws_load(const Opnd& o, int64_t m0, int64_t k0, int pt, float4 (&v)[ROWS / 32]) {
  const auto rs = buf_rsrc(o.p + m0 * o.ld, (o.mdim - m0) * o.ld * 4);
#pragma unroll
  for (int t = 0; t < ROWS / 64; ++t) {
    const int e = pt + t * 256;
    const int r = e >> 2, k8 = (e & 3) * 8;
    const bool ok0 = k0 + k8 < o.kdim, ok1 = k0 + k8 + 4 < o.kdim;
    v[2 * t] = buf_f32x4(rs, ok0 ? (uint32_t)((r * o.ld + k0 + k8) * 4) : BUF_OOB);
    v[2 * t + 1] = buf_f32x4(rs, ok1 ? (uint32_t)((r * o.ld + k0 + k8 + 4) * 4) : BUF_OOB);
  }
}
template <int ROWS>
__device__ __forceinline__ void ws_store(uint16_t* L, int pt, const float4 (&v)[ROWS / 32]) {
  constexpr int PLANE = Lay<true, ROWS>::PLANE;
#pragma unroll
  for (int t = 0; t < ROWS / 64; ++t) {
    const int e = pt + t * 256;
    const int m = e >> 2, k8 = (e & 3) * 8;
    const float x[8] = {v[2 * t].x,     v[2 * t].y,     v[2 * t].z,     v[2 * t].w,
                        v[2 * t + 1].x, v[2 * t + 1].y, v[2 * t + 1].z, v[2 * t + 1].w};
    bf16x8 pl[NPL];
    split8x3(x, pl);
    uint16_t* d = L + lds_off<true>(m, k8);
    *reinterpret_cast<bf16x8*>(d) = pl[0];
    *reinterpret_cast<bf16x8*>(d + PLANE) = pl[1];
    *reinterpret_cast<bf16x8*>(d + 2 * PLANE) = pl[2];
  }
}

template <class C>
__device__ __forceinline__ void gemm_loop_ws(const GemmArgs& g_, int64_t m0, int64_t n0, uint16_t* smem,
                                             f32x4 (&acc)[TM][C::TN]) {
  static_assert(C::NP == 4 && C::NW == 4, "4 MFMA + 4 producer waves");
  constexpr int TN = C::TN;
  constexpr int AOP = Lay<true, C::BM>::OPND, STAGE = stage_elems<C, true>();
  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  const int nch = (int)((g_.A.kdim + BK - 1) / BK);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = zero4();
  if (w >= C::NW) {  // ---- producers
    const int pt = (int)threadIdx.x - C::NW * 64;
    float4 va[C::BM / 32], vb[C::BN / 32];
    ws_load<C::BM>(g_.A, m0, 0, pt, va);
    ws_load<C::BN>(g_.B, n0, 0, pt, vb);
    ws_store<C::BM>(smem, pt, va);
    ws_store<C::BN>(smem + AOP, pt, vb);
    if (nch > 1) {
      ws_load<C::BM>(g_.A, m0, BK, pt, va);
      ws_load<C::BN>(g_.B, n0, BK, pt, vb);
    }
    __syncthreads();
    for (int c = 0; c < nch; ++c) {
      if (c + 1 < nch) {
        uint16_t* S = smem + ((c + 1) & 1) * STAGE;
        ws_store<C::BM>(S, pt, va);
        ws_store<C::BN>(S + AOP, pt, vb);
        if (c + 2 < nch) {
          ws_load<C::BM>(g_.A, m0, (int64_t)(c + 2) * BK, pt, va);
          ws_load<C::BN>(g_.B, n0, (int64_t)(c + 2) * BK, pt, vb);
        }
      }
      __syncthreads();
    }
    return;
  }
  // ---- MFMA waves
  const int wm = w / C::NWN, wn = w % C::NWN;
  __syncthreads();
  for (int c = 0; c < nch; ++c) {
    const uint16_t* S = smem + (c & 1) * STAGE;
    bf16x8 a[TM][NPL];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int p = 0; p < NPL; ++p) a[i][p] = frag<true, C::BM>(S, p, wm * WM + 16 * i + r, g);
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      bf16x8 b[NPL];
#pragma unroll
      for (int p = 0; p < NPL; ++p) b[p] = frag<true, C::BN>(S + AOP, p, wn * C::WN + 16 * j + r, g);
#pragma unroll
      for (int q = 0; q < 6; ++q)
#pragma unroll
        for (int i = 0; i < TM; ++i) acc[i][j] = mfma_bf16(a[i][PA[q]], b[PB[q]], acc[i][j]);
    }
    __syncthreads();
  }
}

// XCD-aware block order: consecutive block ids land on different XCDs
// (round robin); remap so each XCD walks a compact run of the tile grid
// (shared A/B panels stay in its L2).
// Bijective: XCD x (= bid % 8) owns logical ids [x*qf + min(x, rem), ...).
__device__ __forceinline__ int64_t xcd_swizzle(int64_t bid, int64_t nblk) {
  const int64_t qf = nblk / 8, rem = nblk % 8;
  const int64_t x = bid % 8, q = bid / 8;
  return x * qf + (x < rem ? x : rem) + q;
}

// ---------------------------------------------------------------------------
// k_nce_sim: S = F C^T (MODE 0: InfoNCE exp/partials; MODE 1: rank counts)
// ---------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(CfgSim::NTH) void k_nce_sim(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  using C = CfgSim;
  constexpr int NWM = C::NWM, NWN = C::NWN, TN = C::TN, WN = C::WN;
  const int64_t nblk = (int64_t)gridDim.x;
  const int64_t bid = xcd_swizzle(blockIdx.x, nblk);
  const int64_t bm = bid / a.n_blocks_n, bn = bid % a.n_blocks_n;
  const int64_t m0 = bm * C::BM, n0 = bn * C::BN;
  f32x4 acc[TM][TN];
#if TT_NCE_WS
  gemm_loop_ws<C>(a, m0, n0, smem, acc);
  if (wave_id() >= C::NW) return;  // producers: no epilogue
#elif TT_NCE_SIM_DB
  gemm_loop_db<C>(a, m0, n0, smem, acc);
#elif TT_NCE_F32LDS
  gemm_loop_f32<C>(a, m0, n0, reinterpret_cast<float*>(smem), acc);
#else
  gemm_loop<SRC_MK, SRC_MK, C, false, (bool)TT_NCE_PIPE>(a, m0, n0, 0, a.A.kdim, smem, acc);
#endif

  const int w = wave_id(), l = lane_id(), r = l & 15, g = l >> 4;
  const int wm = w / NWN, wn = w % NWN;
  if constexpr (MODE == 0) {
    const float shift = *a.shift;
    float rs[TM][4];
    float cs[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) cs[j] = 0.f;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int q = 0; q < 4; ++q) rs[i][q] = 0.f;
      const int64_t ti = (m0 + wm * WM + 16 * i) / 16;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int64_t tj = (n0 + wn * WN + 16 * j) / 16;
        const int64_t gj = tj * 16 + r;
        f32x4 e;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t gi = ti * 16 + 4 * g + q;
          const float s = acc[i][j][q] * a.inv_tau;
          const bool in = gi < a.M && gj < a.N;
          e[q] = in ? __expf(s - shift) : 0.f;
          rs[i][q] += e[q];
          cs[j] += e[q];
        }
        if (ti < a.e_nti && tj < a.e_ntj)
          __builtin_nontemporal_store(e, reinterpret_cast<f32x4*>(a.E + (ti * a.e_ntj + tj) * TILE) + l);
      }
    }
    // row partials (sum over this wave's WN columns) -> rowpart[part][row]
    const int64_t rpart = bn * NWN + wn;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v = row_reduce16(rs[i][q]);
        const int64_t gi = m0 + wm * WM + 16 * i + 4 * g + q;
        if (r == 0 && gi < a.m_pad) a.rowpart[rpart * a.m_pad + gi] = v;
      }
    // column partials (sum over this wave's WM rows) -> colpart[part][col]
    const int64_t cpart = bm * NWM + wm;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const float v = col_reduce(cs[j]);
      const int64_t gj = n0 + wn * WN + 16 * j + r;
      if (g == 0 && gj < a.n_pad) a.colpart[cpart * a.n_pad + gj] = v;
    }
  } else if constexpr (MODE == 3 || MODE == 4) {
    // robust InfoNCE.  MODE 3: per-wave row / column maxima of s -> rowpart /
    // colpart.  MODE 4: row sums of exp(s - rmax_i), column sums of
    // exp(s - cmax_j) -> rowpart / colpart, and s itself (-inf outside the
    // matrix) into the E tiles for the backward.
    constexpr bool MX = MODE == 3;
    const float init = MX ? -INFINITY : 0.f;
    float rs[TM][4];
    float cs[TN];
    float cmx[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      cs[j] = init;
      const int64_t gj = n0 + wn * WN + 16 * j + r;
      cmx[j] = MX ? 0.f : a.cmax[gj < a.n_pad ? gj : 0];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int64_t ti = (m0 + wm * WM + 16 * i) / 16;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        rs[i][q] = init;
        const int64_t gi = ti * 16 + 4 * g + q;
        const float rmx = MX ? 0.f : a.rmax[gi < a.m_pad ? gi : 0];
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int64_t gj = (n0 + wn * WN + 16 * j) + r;
          const bool in = gi < a.M && gj < a.N;
          const float sv = acc[i][j][q] * a.inv_tau;
          if constexpr (MX) {
            rs[i][q] = in ? fmaxf(rs[i][q], sv) : rs[i][q];
            cs[j] = in ? fmaxf(cs[j], sv) : cs[j];
          } else {
            rs[i][q] += in ? __expf(sv - rmx) : 0.f;
            cs[j] += in ? __expf(sv - cmx[j]) : 0.f;
            acc[i][j][q] = in ? sv : -INFINITY;
          }
        }
      }
      if constexpr (!MX) {
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int64_t tj = (n0 + wn * WN + 16 * j) / 16;
          if (ti < a.e_nti && tj < a.e_ntj)
            __builtin_nontemporal_store(acc[i][j], reinterpret_cast<f32x4*>(a.E + (ti * a.e_ntj + tj) * TILE) + l);
        }
      }
    }
    const int64_t rpart = bn * NWN + wn;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float v = MX ? row_max16(rs[i][q]) : row_reduce16(rs[i][q]);
        const int64_t gi = m0 + wm * WM + 16 * i + 4 * g + q;
        if (r == 0 && gi < a.m_pad) a.rowpart[rpart * a.m_pad + gi] = v;
      }
    const int64_t cpart = bm * NWM + wm;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const float v = MX ? col_max4(cs[j]) : col_reduce(cs[j]);
      const int64_t gj = n0 + wn * WN + 16 * j + r;
      if (g == 0 && gj < a.n_pad) a.colpart[cpart * a.n_pad + gj] = v;
    }
  } else if constexpr (MODE == 2) {
    // semi-hard triplet mining (contrastive.py:163-190): dist = 1 - sim in
    // fp32 as the reference rounds it; per row the smallest semi-hard
    // negative (pos < dist < pos + margin) and the smallest negative overall
    const int64_t rpart = bn * NWN + wn;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t gi = m0 + wm * WM + 16 * i + 4 * g + q;
        const float pos = 1.f - a.diag[gi < a.M ? gi : 0];
        const float hi = pos + a.margin;
        uint64_t ks = KEY_NONE, ka = KEY_NONE;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int64_t gj = n0 + wn * WN + 16 * j + r;
          const float dist = 1.f - acc[i][j][q];
          const bool ok = gj < a.N && gj != a.row0 + gi;
          const uint64_t key = ((uint64_t)ord_f32(dist) << 32) | (uint32_t)gj;
          ka = (ok && key < ka) ? key : ka;
          ks = (ok && dist > pos && dist < hi && key < ks) ? key : ks;
        }
        ks = row_min16(ks);
        ka = row_min16(ka);
        if (r == 0 && gi < a.m_pad) {
          a.semi_part[rpart * a.m_pad + gi] = ks;
          a.all_part[rpart * a.m_pad + gi] = ka;
        }
      }
    }
  } else {
    // rank: count j != row0 + i with sim_ij > sim_ii
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t gi = m0 + wm * WM + 16 * i + 4 * g + q;
        const float d = a.diag[gi < a.M ? gi : 0];
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int64_t gj = n0 + wn * WN + 16 * j + r;
          cnt += (gj < a.N && gj != a.row0 + gi && acc[i][j][q] > d) ? 1 : 0;
        }
        const float c = row_reduce16((float)cnt);  // exact for counts < 2^24
        if (r == 0 && gi < a.M && c > 0.f) atomicAdd(a.rank_cnt + gi, (int)c);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// diagonal of F C^T with the GEMM's own arithmetic (same plane split, same
// six-MFMA sequence per 32-deep K step, same K order) -> bitwise the value
// the tiled GEMM produces.  One wave per 16-row tile; C rows row0 + i.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void split8(const float (&x)[8], bf16x8 (&pl)[NPL]) {
#pragma unroll
  for (int s = 0; s < 8; ++s) {
    uint16_t h, m, l;
    split3(x[s], h, m, l);
    pl[0][s] = __builtin_bit_cast(__bf16, h);
    pl[1][s] = __builtin_bit_cast(__bf16, m);
    pl[2][s] = __builtin_bit_cast(__bf16, l);
  }
}

__global__ __launch_bounds__(256) void k_nce_diag(const float* __restrict__ F, const float* __restrict__ C,
                                                  int64_t m, int64_t n, int d, int64_t row0, float scale,
                                                  float* __restrict__ diag) {
  const int l = lane_id(), r = l & 15, g = l >> 4;
  const int64_t t = (int64_t)blockIdx.x * 4 + wave_id();
  const int64_t i = t * 16 + r;  // row of this lane (A operand) and column (B operand)
  const bool okf = i < m, okc = (row0 + i) < n && (row0 + i) >= 0;
  f32x4 acc = zero4();
  for (int k0 = 0; k0 < d; k0 += BK) {
    float xa[8], xb[8];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = k0 + 8 * g + 4 * h;
      const bool kk = k < d;
      float4 av = make_float4(0.f, 0.f, 0.f, 0.f), bv = av;
      if (okf && kk) av = *reinterpret_cast<const float4*>(F + i * d + k);
      if (okc && kk) bv = *reinterpret_cast<const float4*>(C + (row0 + i) * d + k);
      xa[4 * h + 0] = av.x; xa[4 * h + 1] = av.y; xa[4 * h + 2] = av.z; xa[4 * h + 3] = av.w;
      xb[4 * h + 0] = bv.x; xb[4 * h + 1] = bv.y; xb[4 * h + 2] = bv.z; xb[4 * h + 3] = bv.w;
    }
    bf16x8 a[NPL], b[NPL];
    split8(xa, a);
    split8(xb, b);
#pragma unroll
    for (int q = 0; q < 6; ++q) acc = mfma_bf16(a[PA[q]], b[PB[q]], acc);
  }
  // acc[q] = C[row 4g+q][col r]; the diagonal is row == col
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (4 * g + q == r && okf && okc) diag[i] = acc[q] * scale;
}

// ---------------------------------------------------------------------------
// k_nce_dgrad: split-K partial of  E'^(T) X  (dF: E' C, dC: E'^T F) into
// accumulator-layout tiles part[split][ti][tj][256]
// ---------------------------------------------------------------------------
template <int SA, bool LSE>
__global__ __launch_bounds__(CfgGrad::NTH) void k_nce_dgrad(GemmArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  using C = CfgGrad;
  constexpr int NWN = C::NWN, TN = C::TN, WN = C::WN;
  const int64_t nblk = (int64_t)gridDim.x;
  const int64_t bid = xcd_swizzle(blockIdx.x, nblk);
  const int64_t bm = bid / a.n_blocks_n, bn = bid % a.n_blocks_n;
  const int64_t m0 = bm * C::BM, n0 = bn * C::BN;
  const int64_t split = blockIdx.y;
  const int64_t kb = split * a.k_per_split;
  const int64_t ke = min(kb + a.k_per_split, a.A.kdim);
  f32x4 acc[TM][TN];
  gemm_loop<SA, SRC_KROWS, C, LSE>(a, m0, n0, kb, ke, smem, acc);
  const int w = wave_id(), l = lane_id();
  const int wm = w / NWN, wn = w % NWN;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int64_t ti = (m0 + wm * WM + 16 * i) / 16, tj = (n0 + wn * WN + 16 * j) / 16;
      if (ti < a.p_nti && tj < a.p_ntj)
        *(reinterpret_cast<f32x4*>(a.part + ((split * a.p_nti + ti) * a.p_ntj + tj) * TILE) + l) = acc[i][j];
    }
}

// out[row][col] = scale * sum_split part - corr * X[row + xoff][col]  (X row in range)
__global__ __launch_bounds__(256) void k_nce_grad_finish(const float* __restrict__ part, int64_t n_split,
                                                         int64_t p_nti, int64_t p_ntj, int64_t rows, int d,
                                                         float scale, float corr, const float* __restrict__ X,
                                                         int64_t x_rows, int64_t xoff, float* __restrict__ out) {
  const int64_t tile_elems = p_nti * p_ntj * 64;  // float4 per split
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tile_elems;
       e += (int64_t)gridDim.x * blockDim.x) {
    f32x4 s = zero4();
    for (int64_t sp = 0; sp < n_split; ++sp) s += reinterpret_cast<const f32x4*>(part)[sp * tile_elems + e];
    const int64_t t = e >> 6;
    const int ln = (int)(e & 63);
    const int64_t ti = t / p_ntj, tj = t % p_ntj;
    const int64_t col = tj * 16 + (ln & 15);
    if (col >= d) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t row = ti * 16 + 4 * (ln >> 4) + q;
      if (row >= rows) continue;
      const int64_t xr = row + xoff;
      const float xv = (xr >= 0 && xr < x_rows) ? X[xr * d + col] : 0.f;
      out[row * d + col] = s[q] * scale - corr * xv;
    }
  }
}

// max squared row norms of F (m rows) and C (n rows) -> norm2[0], norm2[1]
// (float bit patterns of non-negative values order like the values)
__global__ __launch_bounds__(256) void k_nce_norms(const float* __restrict__ F, const float* __restrict__ C,
                                                   int64_t m, int64_t n, int d, float* norm2) {
  const int r = lane_id() & 15;
  const int64_t groups = (int64_t)gridDim.x * 16;
  float mf = 0.f, mc = 0.f;
  for (int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4); row < m + n; row += groups) {
    const float* p = row < m ? F + row * d : C + (row - m) * d;
    float s = 0.f;
    for (int k = r; k < d; k += 16) s += p[k] * p[k];
    s = row_reduce16(s);
    if (row < m) mf = fmaxf(mf, s); else mc = fmaxf(mc, s);
  }
  if (r == 0) {
    atomicMax(reinterpret_cast<unsigned*>(norm2), __float_as_uint(mf));
    atomicMax(reinterpret_cast<unsigned*>(norm2) + 1, __float_as_uint(mc));
  }
}

__device__ __forceinline__ float nce_shift(const float* norm2, float inv_tau) {
  return sqrtf(norm2[0]) * sqrtf(norm2[1]) * inv_tau;
}

__global__ __launch_bounds__(256) void k_nce_set_shift(const float* norm2, float inv_tau, float* shift) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *shift = nce_shift(norm2, inv_tau);
}

// fixed-order sums of the per-wave partials: rowsum[i] (i < m_pad), colsum[j] (j < n_pad)
__global__ __launch_bounds__(256) void k_nce_sums(const float* __restrict__ rowpart, int64_t n_rp, int64_t m_pad,
                                                  const float* __restrict__ colpart, int64_t n_cp, int64_t n_pad,
                                                  float* __restrict__ rowsum, float* __restrict__ colsum) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m_pad + n_pad;
       e += (int64_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    if (e < m_pad) {
      for (int64_t p = 0; p < n_rp; ++p) s += rowpart[p * m_pad + e];
      rowsum[e] = s;
    } else {
      const int64_t j = e - m_pad;
      for (int64_t p = 0; p < n_cp; ++p) s += colpart[p * n_pad + j];
      colsum[j] = s;
    }
  }
}

// loss contribution of local rows i (row term) and columns j = row0 + i
// (column term), plus the softmax scales a_i = 1/rowsum_i, b_j = 1/colsum_j
// (zero in the padding).  loss += sum / (2 B).
__global__ __launch_bounds__(256) void k_nce_loss(const float* __restrict__ rowsum, const float* __restrict__ colsum,
                                                  const float* __restrict__ diag, int64_t m, int64_t m_pad,
                                                  int64_t n, int64_t n_pad, int64_t row0, float inv_2b,
                                                  const float* __restrict__ shift, float* __restrict__ a,
                                                  float* __restrict__ b, float* loss, int* status) {
  __shared__ float red[4];
  const float sh = *shift;
  float acc = 0.f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m_pad + n_pad;
       e += (int64_t)gridDim.x * blockDim.x) {
    bool bad = false;
    if (e < m_pad) {
      a[e] = e < m ? 1.f / rowsum[e] : 0.f;
      if (e < m) {
        const float dg = diag[e];
        acc += (logf(rowsum[e]) + sh - dg) + (logf(colsum[row0 + e]) + sh - dg);
        bad = !(rowsum[e] >= SUM_MIN);
      }
    } else {
      const int64_t j = e - m_pad;
      b[j] = j < n ? 1.f / colsum[j] : 0.f;
      bad = j < n && !(colsum[j] >= SUM_MIN);
    }
    if (bad && status) atomicAdd(status, 1);
  }
  acc = wave_reduce(acc);
  if (lane_id() == 0) red[wave_id()] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss, (red[0] + red[1] + red[2] + red[3]) * inv_2b);
}

// robust mode: fixed-order max (MX) or sum of the per-wave partials, as k_nce_sums
template <bool MX>
__global__ __launch_bounds__(256) void k_nce_reduce_parts(const float* __restrict__ rowpart, int64_t n_rp,
                                                          int64_t m_pad, const float* __restrict__ colpart,
                                                          int64_t n_cp, int64_t n_pad, float* __restrict__ rowv,
                                                          float* __restrict__ colv) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m_pad + n_pad;
       e += (int64_t)gridDim.x * blockDim.x) {
    float s = MX ? -INFINITY : 0.f;
    if (e < m_pad) {
      for (int64_t p = 0; p < n_rp; ++p) s = MX ? fmaxf(s, rowpart[p * m_pad + e]) : s + rowpart[p * m_pad + e];
      rowv[e] = s;
    } else {
      const int64_t j = e - m_pad;
      for (int64_t p = 0; p < n_cp; ++p) s = MX ? fmaxf(s, colpart[p * n_pad + j]) : s + colpart[p * n_pad + j];
      colv[j] = s;
    }
  }
}

// robust loss: a_i = rmax_i + log rowsum_i, b_j = cmax_j + log colsum_j (the
// log-sum-exps; +inf outside the matrix, where E' must vanish), loss +=
// (a_i - s_ii) + (b_{row0+i} - s_ii) over this shard's rows, / (2 B).  Every
// sum is >= 1 (its max term is exp(0)), so *status counts only non-finite ones.
__global__ __launch_bounds__(256) void k_nce_loss_lse(const float* __restrict__ rowsum, const float* __restrict__ rmax,
                                                      const float* __restrict__ colsum, const float* __restrict__ cmax,
                                                      const float* __restrict__ diag, int64_t m, int64_t m_pad,
                                                      int64_t n, int64_t n_pad, int64_t row0, float inv_2b,
                                                      float* __restrict__ a, float* __restrict__ b, float* loss,
                                                      int* status) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m_pad + n_pad;
       e += (int64_t)gridDim.x * blockDim.x) {
    bool bad = false;
    if (e < m_pad) {
      const float li = e < m ? rmax[e] + logf(rowsum[e]) : INFINITY;
      a[e] = li;
      if (e < m) {
        const float si = diag[e];  // s_ii (k_nce_diag scaled it by 1 / tau)
        const float lj = cmax[row0 + e] + logf(colsum[row0 + e]);
        acc += (li - si) + (lj - si);
        bad = !isfinite(li) || !isfinite(lj);
      }
    } else {
      const int64_t j = e - m_pad;
      b[j] = j < n ? cmax[j] + logf(colsum[j]) : INFINITY;
    }
    if (bad && status) atomicAdd(status, 1);
  }
  acc = wave_reduce(acc);
  if (lane_id() == 0) red[wave_id()] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss, (red[0] + red[1] + red[2] + red[3]) * inv_2b);
}

__global__ __launch_bounds__(256) void k_rank_finish(const int* __restrict__ cnt, int64_t m, int* __restrict__ rank) {
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < m; e += (int64_t)gridDim.x * blockDim.x)
    rank[e] = cnt[e] + 1;
}

// Per row: the hardest semi-hard negative if there is one, else the hardest
// negative overall (contrastive.py:181-188); row_loss = relu(pos - hardest +
// margin) (fp32, the reference's rounding), hardest[i] = its column;
// loss += sum(row_loss) / batch.
__global__ __launch_bounds__(256) void k_triplet_finish(const uint64_t* __restrict__ semi_part,
                                                        const uint64_t* __restrict__ all_part, int64_t n_rp,
                                                        int64_t m_pad, int64_t m, const float* __restrict__ diag,
                                                        float margin, float inv_batch, int* __restrict__ hardest,
                                                        float* __restrict__ row_loss, float* loss) {
  __shared__ float red[4];
  float acc = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t ks = KEY_NONE, ka = KEY_NONE;
    for (int64_t p = 0; p < n_rp; ++p) {
      const uint64_t s = semi_part[p * m_pad + i], x = all_part[p * m_pad + i];
      ks = s < ks ? s : ks;
      ka = x < ka ? x : ka;
    }
    const uint64_t k = ks != KEY_NONE ? ks : ka;
    const float hd = unord_f32((uint32_t)(k >> 32));
    const float pos = 1.f - diag[i];
    float li = (pos - hd) + margin;
    li = li > 0.f ? li : 0.f;
    hardest[i] = (int)(uint32_t)k;
    row_loss[i] = li;
    acc += li;
  }
  acc = wave_reduce(acc);
  if (lane_id() == 0) red[wave_id()] = acc;
  __syncthreads();
  if (threadIdx.x == 0) atomicAdd(loss, ((red[0] + red[1]) + (red[2] + red[3])) * inv_batch);
}

// Backward of the mined triplet loss: for every active row i (row_loss > 0)
// with hardest column j, dL/dloss = g:  dF_i = (g / B) (c_j - c_{row0+i}),
// dC_{row0+i} -= (g / B) f_i,  dC_j += (g / B) f_i.  One wave per row;
// dF rows are owned, dC receives atomics (dc zeroed by the caller).
__global__ __launch_bounds__(256) void k_triplet_bwd(const float* __restrict__ F, const float* __restrict__ C,
                                                     int64_t m, int d, int64_t row0, const int* __restrict__ hardest,
                                                     const float* __restrict__ row_loss, const float* __restrict__ g,
                                                     float inv_batch, float* __restrict__ dF, float* __restrict__ dC) {
  const int64_t i = (int64_t)blockIdx.x * 4 + wave_id();
  if (i >= m) return;
  const float sc = row_loss[i] > 0.f ? *g * inv_batch : 0.f;
  const int64_t j = hardest[i], ip = row0 + i;
  for (int k = lane_id(); k < d; k += 64) {
    const float fk = F[i * d + k];
    dF[i * d + k] = sc * (C[j * d + k] - C[ip * d + k]);
    if (sc != 0.f) {
      atomicAdd(dC + ip * d + k, -sc * fk);
      atomicAdd(dC + j * d + k, sc * fk);
    }
  }
}

}  // namespace nce
}  // namespace tt
