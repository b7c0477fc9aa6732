// Host side of libceo_tt.so: argument checking, arena / workspace layout and
// kernel launch sequences behind the C-ABI declared in include/ceo_tt.h.
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <mutex>
#include <random>

#include <hip/hip_ext.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include "tt_common.h"
#include "tt_tower.hip"
#include "tt_topgen.hip"
#include "tt_optim.hip"
#include "tt_comm.hip"
#include "tt_cosine.hip"
#include "tt_contrastive.hip"

#ifdef TT_STAMPS
namespace tt {
__constant__ uint64_t* g_tt_stamps = nullptr;  // __constant__: read with a scalar load, no vmcnt wait per stamp
}
extern "C" int32_t tt_debug_set_stamps(uint64_t* buf) {
  return (int32_t)hipMemcpyToSymbol(HIP_SYMBOL(tt::g_tt_stamps), &buf, sizeof(buf));
}
#endif

namespace tt {

constexpr size_t LDS_MAX = 160 * 1024;

// roctx range around one host entry (the step and the exchange
// attributed per rank in a rocprofv3 --marker-trace; without a profiler the
// calls return at once).  Host code only: enqueue-side ranges, the kernels'
// own times come from the kernel trace.
struct Range {
  explicit Range(const char* m) { roctxRangePushA(m); }
  ~Range() { roctxRangePop(); }
  Range(const Range&) = delete;
  Range& operator=(const Range&) = delete;
};

// ---------------------------------------------------------------------------
// layouts
// ---------------------------------------------------------------------------
struct Layout {
  int in_dim[2], kp[2], n_num[2];
  int latent;
  int64_t emb_off[2][TT_MAX_CAT];
  int64_t slot[2][TT_SLOTS_PER_TOWER];
  int64_t ls;
  int64_t n;          // parameter count
  int64_t so[2][6];   // slab offsets W0 b0 W4 b4 W8 b8
  int64_t slab_ld;
  bool fold_ok;       // numeric-only towers, widths % 4 == 0 and <= 64: the BN0 backward can be
                      // folded into k_bwd_mid (slab W0 range sized for P | Q); Plan::fold decides
};

static int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

static bool desc_ok(const tt_model_desc* d) {
  if (!d) return false;
  for (int t = 0; t < 2; ++t) {
    if (d->n_num[t] < 0 || d->n_cat[t] < 0 || d->n_cat[t] > TT_MAX_CAT) return false;
    if (d->n_cat[t] > 0 && d->emb_dim[t] <= 0) return false;
    for (int j = 0; j < d->n_cat[t]; ++j)
      if (d->cat_counts[t][j] <= 0) return false;
    if (d->n_num[t] + d->n_cat[t] * d->emb_dim[t] <= 0) return false;
  }
  return d->latent > 0 && d->dropout_p >= 0.f && d->dropout_p < 1.f;
}

static Layout make_layout(const tt_model_desc* d) {
  Layout L;
  std::memset(&L, 0, sizeof(L));
  int64_t off = 0;
  for (int t = 0; t < 2; ++t)
    for (int j = 0; j < TT_MAX_CAT; ++j) L.emb_off[t][j] = -1;
  // every parameter starts on a 16-byte boundary (float4 loads of weights)
  for (int t = 0; t < 2; ++t)
    for (int j = 0; j < d->n_cat[t]; ++j) {
      L.emb_off[t][j] = off;
      off = round_up(off + (int64_t)d->cat_counts[t][j] * d->emb_dim[t], 4);
    }
  const int D = d->latent;
  L.latent = D;
  L.fold_ok = true;
  for (int t = 0; t < 2; ++t) {
    const int in = d->n_num[t] + d->n_cat[t] * d->emb_dim[t];
    L.in_dim[t] = in;
    L.n_num[t] = d->n_num[t];
    L.kp[t] = (int)round_up(in, 16);
    L.fold_ok = L.fold_ok && d->n_cat[t] == 0 && in % 4 == 0 && L.kp[t] <= FOLD_MAX_KP;
  }
#ifdef TT_NO_FOLD
  L.fold_ok = false;
#endif
  for (int t = 0; t < 2; ++t) {
    const int in = L.in_dim[t];
    const int64_t sz[TT_SLOTS_PER_TOWER] = {(int64_t)H0 * in, H0, H0, H0, (int64_t)H1 * H0, H1, H1, H1,
                                            (int64_t)D * H1, D};
    for (int s = 0; s < TT_SLOTS_PER_TOWER; ++s) {
      L.slot[t][s] = off;
      off = round_up(off + sz[s], 4);
    }
    int64_t so = 0;
    // folded: P and Q partials interleaved [64][kp/16][P 16 | Q 16] in the W0 range
    L.so[t][0] = so; so += (int64_t)H0 * (L.fold_ok ? 2 * L.kp[t] : in);
    L.so[t][1] = so; so += H0;
    L.so[t][2] = so; so += (int64_t)H1 * H0;
    L.so[t][3] = so; so += H1;
    L.so[t][4] = so; so += (int64_t)D * H1;
    L.so[t][5] = so; so += D;
    L.slab_ld = std::max<int64_t>(L.slab_ld, round_up(so, 64));
  }
  L.ls = off;
  L.n = off + 1;
  return L;
}

struct WsLayout {
  int64_t Z0[2], Z4[2], dY0[2], dY1[2], st0[2], st1[2], sh0[2], sh1[2], fin0[2], fin1[2], bng[2], lsr;
  int64_t fr, k0s[2], xsh[2];  // folded BN0 backward: replicas (both towers), inv0*gamma0, shift row
  int64_t adam;                // AdamSlot[2]: cached Adam coefficients (k_l0_fwd, k_reduce_adam)
  int64_t late;                // int64: deferred late half pending (step + 1, 0: none)
  int64_t tgw;
  int64_t slab[2];
  int64_t gacc;
  int64_t det[2], det_lsr;     // deterministic mode: per-block partial slots [n_tiles][DET_W] per tower, (dls, loss)
  int64_t demb[2];             // deterministic mode: embedding-column dX per batch row [rows][emb_w] (-1: none)
  int64_t ug[2], dug[2];       // LATENT > 128: U / V and dU / dV [rows][Dp] (-1: none)
  int64_t total;  // floats
  int n_tiles;
};

constexpr int DET_W = 256;     // widest cross-block accumulator of one block (FRW, 2 * H0 .. )

// Per-row workspace arrays hold whole 128-row tiles (the kernels store rows
// beyond B unconditionally into this padding instead of branching per row).
static int64_t padded_rows(int64_t b) { return round_up(std::max<int64_t>(b, 1), TOP_ROWS_MAX); }

// Layout: the accumulators a fused step leaves zeroed for the next one (BN
// moment sums, the atomic gradient arena) come first, at offsets that do not
// depend on the batch size -- consecutive steps of different B (the last
// partial batch of an epoch) must find them where the previous step zeroed
// them.  Per-row arrays and per-tile partial slabs follow.
static WsLayout make_ws(const Layout& L, int64_t max_batch) {
  WsLayout W;
  int64_t off = 0;
  auto take = [&](int64_t n) { const int64_t o = off; off += round_up(n, 64); return o; };
  for (int t = 0; t < 2; ++t) {
    W.st0[t] = take(NREP * ST0S);
    W.st1[t] = take(NREP * ST1S);
    W.bng[t] = take(NREP * BNG);
    W.sh0[t] = take(H0);
    W.sh1[t] = take(H1);
    W.fin0[t] = take(2 * H0);
    W.fin1[t] = take(2 * H1);
  }
  W.lsr = take(NREP * LSR);
  W.fr = take(2 * NREP * FRW);
  for (int t = 0; t < 2; ++t) {
    W.k0s[t] = take(H0);
    W.xsh[t] = take(FOLD_MAX_KP);
  }
  W.adam = take(2 * sizeof(AdamSlot) / sizeof(float));
  W.late = take(2);
  W.gacc = take(L.n);
  const int64_t rows = padded_rows(max_batch);
  W.n_tiles = (int)(rows / ROWS);
  for (int t = 0; t < 2; ++t) {
    W.Z0[t] = take(rows * H0);
    W.Z4[t] = take(rows * H1);
    W.dY0[t] = take(rows * H0);
    W.dY1[t] = take(rows * H1);
  }
  W.tgw = take(rows * 2);
  // slab / deterministic-slot rows: one per 64-row tile, or per 32-row
  // k_top_pair tile of a batch below TT_PAIR32_MAX_B (twice as many)
  static_assert(TT_FWD32_MAX_B <= TT_PAIR32_MAX_B && TT_BWD32_MAX_B <= TT_PAIR32_MAX_B,
                "the 32-row tile counts of k_l0_fwd / k_l4_fwd / k_bwd_mid / k_bwd_first index the slab and "
                "det-slot rows sized from TT_PAIR32_MAX_B");
  const int64_t srows = std::max<int64_t>(W.n_tiles, std::min<int64_t>(2 * W.n_tiles, 2 * (TT_PAIR32_MAX_B / ROWS) + 2));
  for (int t = 0; t < 2; ++t) W.slab[t] = take(srows * L.slab_ld);
  for (int t = 0; t < 2; ++t) W.det[t] = take(srows * DET_W);
  W.det_lsr = take(srows * 2);
  for (int t = 0; t < 2; ++t) {
    const int ew = L.in_dim[t] - L.n_num[t];
    W.demb[t] = ew > 0 ? take(rows * ew) : -1;
  }
  for (int t = 0; t < 2; ++t) {
    const bool gen = L.latent > 128;
    W.ug[t] = gen ? take(rows * gen_dp(L.latent)) : -1;
    W.dug[t] = gen ? take(rows * gen_dp(L.latent)) : -1;
  }
  W.total = off;
  return W;
}

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
static std::once_flag g_attr_once;
static void set_lds_attrs() {
  std::call_once(g_attr_once, [] {
    const int mx = (int)LDS_MAX;
    const void* ks[] = {(const void*)k_l0_fwd<32, 1, true, false>, (const void*)k_l0_fwd<32, 1, false, false>,
                        (const void*)k_l0_fwd<32, 2, true, false>, (const void*)k_l0_fwd<32, 2, false, false>,
                        (const void*)k_l0_fwd<32, 4, true, false>, (const void*)k_l0_fwd<32, 4, false, false>,
                        (const void*)k_l0_fwd<32, 8, true, false>, (const void*)k_l0_fwd<32, 8, false, false>,
                        (const void*)k_l4_fwd<32>, (const void*)k_bwd_mid<32>, (const void*)k_bwd_first<32>,
                        (const void*)k_l0_fwd<ROWS, 1, true, false>, (const void*)k_l0_fwd<ROWS, 1, false, false>,
                        (const void*)k_l0_fwd<ROWS, 2, true, false>, (const void*)k_l0_fwd<ROWS, 2, false, false>,
                        (const void*)k_l0_fwd<ROWS, 4, true, false>, (const void*)k_l0_fwd<ROWS, 4, false, false>,
                        (const void*)k_l0_fwd<ROWS, 8, true, false>, (const void*)k_l0_fwd<ROWS, 8, false, false>,
                        (const void*)k_l0_fwd<ROWS, 1, true, true>, (const void*)k_l0_fwd<ROWS, 2, true, true>,
                        (const void*)k_l4_fwd<ROWS>,
                        (const void*)k_top<4, 64, false>, (const void*)k_top<8, 64, false>,
                        (const void*)k_top<4, 128, false>, (const void*)k_top<8, 128, false>,
                        (const void*)k_top<4, 64, true>,  (const void*)k_top<8, 64, true>,
                        (const void*)k_top<4, 128, true>, (const void*)k_top<8, 128, true>,
                        (const void*)k_top_pair<4, 64>, (const void*)k_top_pair<8, 64>,
                        (const void*)k_top_pair<4, 32>, (const void*)k_top_pair<8, 32>,
                        (const void*)k_bwd_mid<ROWS>, (const void*)k_bwd_mid_fold<FOLD_ROWS, true>,
                        (const void*)k_bwd_mid_fold<FOLD_ROWS, false>, (const void*)k_bwd_first<ROWS>};
    // the dynamic limit is what the kernel's static LDS (e.g. a block vote's
    // word) leaves of the CU's 160 KB; a refused attribute would otherwise
    // stay behind as the thread's last error and fail the next launch check
    auto set = [](const void* k) {
      hipFuncAttributes fa;
      const int st = hipFuncGetAttributes(&fa, k) == hipSuccess ? (int)fa.sharedSizeBytes : 0;
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, mx - st);
    };
    for (const void* k : ks) set(k);
    set((const void*)k_top_gen_fwd);
    set((const void*)k_top_gen_bwd);
    (void)hipGetLastError();
  });
}

struct Plan {
  size_t lds_l0, lds_l4, lds_l4_32, lds_top, lds_mid, lds_first, lds_pair;
  bool top_pair;    // training steps run k_top_pair (both towers per block)
  int pair_rows;    // its rows per block: 64, or 32 below the folded path (twice the blocks)
  int fwd_rows;     // k_l0_fwd / k_l4_fwd rows per block: 64, or 32 below the folded path
  int bwd_rows;     // k_bwd_mid / k_bwd_first rows per block (unfolded): 64, or 32 below the folded path
  int n_tiles_fwd;  // their tiles (deterministic slots of their BN moments)
  int n_tiles_pair; // its tiles (a training step's k_top slab count)
  int ndt;
  int top_rows;     // row tile of k_top (64, or 128 for large batches)
  int n_tiles;      // 64-row tiles
  int n_tiles_top;  // k_top tiles
  int n_tiles_mid;  // k_bwd_mid tiles (FOLD_ROWS rows when the BN0 backward is folded)
  bool fold;        // BN0 backward folded into k_bwd_mid_fold (k_bwd_first not launched)
  bool top_gen;     // LATENT > 128: the generic top (tt_topgen.hip) instead of k_top / k_top_pair
  size_t lds_gen_fwd, lds_gen_bwd;
};

static int make_plan(const tt_model_desc* d, const Layout& L, int64_t B, Plan* P) {
  if (d->latent > GEN_MAX_D) return TT_ERR_UNSUPPORTED;
  P->top_gen = d->latent > 128;
  P->ndt = d->latent <= 64 ? 4 : 8;
  const int kpm = std::max(L.kp[0], L.kp[1]);
  if (kpm > MAX_KP) return TT_ERR_UNSUPPORTED;
  const bool emb = d->n_cat[0] > 0 || d->n_cat[1] > 0;
  // 128-row k_top tiles once the grid still covers every CU twice over
#ifdef TT_TOP_ROWS
  P->top_rows = TT_TOP_ROWS;
  P->top_pair = false;
#else
  // from B = 4096 (64 blocks of 64 rows) the training step's k_top runs
  // k_top_pair (cfg 2: k_top 8.9 -> 8.5 us, step 44.2 -> 43.8 us); its other
  // modes take k_top's 64-row tiles (same slab count)
  P->top_pair = B >= 4096;
  P->top_rows = 64;
#endif
  // the 64-row kernels cover the padded rows, so every workspace row that any
  // kernel reads was written earlier in the same step
  P->n_tiles = (int)(padded_rows(B) / ROWS);
  P->n_tiles_top = (int)((P->n_tiles * ROWS) / P->top_rows);
  // folded from B = 4096 (32 blocks of 128 rows per tower): cfg 2 measured
  // 45.9 us folded vs 42.4 us not (r01), 44.1 vs 43.7 (r03); round 5, with
  // the reduction's segment lookup fixed and k_top_pair on 32-row blocks
  // below 8192 (TT_PAIR32_FOLD): 38.1-38.2 us folded vs 40.0-40.1 not
  // (three interleaved rounds)
  P->fold = L.fold_ok && B >= TT_FOLD_MIN_B;
  P->bwd_rows = !P->fold && B < TT_BWD32_MAX_B ? 32 : ROWS;
  P->n_tiles_mid = (int)((P->n_tiles * ROWS) / (P->fold ? FOLD_ROWS : P->bwd_rows));
  P->lds_l0 = L0Lds<ROWS>::bytes(kpm);
  P->lds_l4 = L4Lds<ROWS>::bytes;
  P->lds_l4_32 = L4Lds<32>::bytes;
  const int tl = P->ndt == 4 ? (P->top_rows == 64 ? TopLds<4, 64>::total : TopLds<4, 128>::total)
                             : (P->top_rows == 64 ? TopLds<8, 64>::total : TopLds<8, 128>::total);
  P->lds_top = sizeof(float) * (size_t)tl;
  // below the folded path the 64-row k_top_pair leaves CUs idle (cfg 2: 64
  // blocks on 256 CUs): 32-row blocks there (TT_PAIR32_MAX_B = 0: never)
#ifndef TT_PAIR32_FOLD
#define TT_PAIR32_FOLD 1  // 32-row k_top_pair on the folded path below TT_PAIR32_MAX_B too (cfg 2: 38.9 -> 38.2 us)
#endif
  P->pair_rows = P->top_pair && (!P->fold || TT_PAIR32_FOLD) && B < TT_PAIR32_MAX_B ? 32 : 64;
  P->fwd_rows = !P->fold && B < TT_FWD32_MAX_B ? 32 : 64;
  P->n_tiles_fwd = (int)((P->n_tiles * ROWS) / P->fwd_rows);
  P->n_tiles_pair = (int)((P->n_tiles * ROWS) / P->pair_rows);
  P->lds_pair = sizeof(float) * (size_t)(P->pair_rows == 32 ? (P->ndt == 4 ? PairLds<4, 32>::total : PairLds<8, 32>::total)
                                                            : (P->ndt == 4 ? PairLds<4>::total : PairLds<8>::total));
  P->lds_mid = P->fold ? FoldLds<FOLD_ROWS>::bytes : P->bwd_rows == 32 ? MidLds<32>::bytes : MidLds<ROWS>::bytes;
  P->lds_first = P->bwd_rows == 32 ? FirstLds<32>::bytes(kpm) : FirstLds<ROWS>::bytes(kpm);
  P->lds_gen_fwd = gen_fwd_lds(d->latent);
  P->lds_gen_bwd = gen_bwd_lds(d->latent);
  if (P->top_gen) {  // 64-row top tiles (the W8 slabs of the generic backward)
    P->top_pair = false;
    P->top_rows = 64;
    P->n_tiles_top = P->n_tiles;
    P->lds_top = P->lds_pair = 0;
  }
  (void)emb;
  for (size_t s : {P->lds_l0, P->lds_l4, P->lds_top, P->lds_mid, P->lds_first, P->lds_pair, P->lds_gen_fwd,
                   P->lds_gen_bwd})
    if (s > LDS_MAX) return TT_ERR_UNSUPPORTED;
  return TT_OK;
}

static bool batch_ok(const tt_model_desc* d, const tt_batch* b) {
  if (!b || b->n_rows < 0) return false;
  for (int t = 0; t < 2; ++t) {
    if (d->n_num[t] > 0 && (!b->num[t] || b->num_ld[t] < d->n_num[t])) return false;
    if (d->n_cat[t] > 0 && (!b->cat[t] || b->cat_ld[t] < d->n_cat[t])) return false;
  }
  return true;
}

static void fill_args(StepArgs& a, const tt_model_desc* d, const Layout& L, const WsLayout& W, bool fold,
                      const float* params,
                      float* buffers, int64_t* nbt, const tt_batch* b, float* ws) {
  std::memset(&a, 0, sizeof(a));
  for (int t = 0; t < 2; ++t) {
    TowerDev& T = a.tw[t];
    T.num = b->num[t];
    T.num_ld = b->num_ld[t];
    T.cat = b->cat[t];
    T.cat_ld = b->cat_ld[t];
    T.n_num = d->n_num[t];
    T.n_cat = d->n_cat[t];
    T.emb_dim = d->n_cat[t] > 0 ? d->emb_dim[t] : 1;
    T.in_dim = L.in_dim[t];
    T.kp = L.kp[t];
    T.num_vec = d->n_cat[t] == 0 && d->n_num[t] % 4 == 0 && b->num_ld[t] % 4 == 0 &&
                (uintptr_t)b->num[t] % 16 == 0;
    float* gacc = ws + W.gacc;
    for (int j = 0; j < d->n_cat[t]; ++j) {
      T.emb[j] = params + L.emb_off[t][j];
      T.gemb[j] = gacc + L.emb_off[t][j];
      T.emb_rows[j] = d->cat_counts[t][j];
    }
    const int64_t* s = L.slot[t];
    T.W0 = params + s[TT_SLOT_W0];
    T.b0 = params + s[TT_SLOT_B0];
    T.g0 = params + s[TT_SLOT_G0];
    T.be0 = params + s[TT_SLOT_BE0];
    T.W4 = params + s[TT_SLOT_W4];
    T.b4 = params + s[TT_SLOT_B4];
    T.g1 = params + s[TT_SLOT_G1];
    T.be1 = params + s[TT_SLOT_BE1];
    T.W8 = params + s[TT_SLOT_W8];
    T.b8 = params + s[TT_SLOT_B8];
    if (buffers) {  // NULL for backward (running stats untouched)
      float* bt = buffers + t * (2 * H0 + 2 * H1);
      T.rm0 = bt;
      T.rv0 = bt + H0;
      T.rm1 = bt + 2 * H0;
      T.rv1 = bt + 2 * H0 + H1;
    }
    if (nbt) {
      T.nbt0 = nbt + 2 * t;
      T.nbt1 = nbt + 2 * t + 1;
    }
    float* bng = ws + W.bng[t];
    T.gg0 = bng;
    T.gbe0 = bng + H0;
    T.gg1 = bng + 2 * H0;
    T.gbe1 = bng + 2 * H0 + H1;
    T.Z0 = ws + W.Z0[t];
    T.Z4 = ws + W.Z4[t];
    T.dY0 = ws + W.dY0[t];
    T.dY1 = ws + W.dY1[t];
    T.st0 = ws + W.st0[t];
    T.st1 = ws + W.st1[t];
    T.shift0 = ws + W.sh0[t];
    T.shift1 = ws + W.sh1[t];
    T.fin0 = ws + W.fin0[t];
    T.fin1 = ws + W.fin1[t];
    T.slab = ws + W.slab[t];
    T.so_W0 = L.so[t][0];
    T.so_b0 = L.so[t][1];
    T.so_W4 = L.so[t][2];
    T.so_b4 = L.so[t][3];
    T.so_W8 = L.so[t][4];
    T.so_b8 = L.so[t][5];
    T.fr = ws + W.fr + (int64_t)t * NREP * FRW;
    T.k0s = ws + W.k0s[t];
    T.xsh = ws + W.xsh[t];
    T.dslot = ws + W.det[t];
    T.demb = W.demb[t] >= 0 ? ws + W.demb[t] : nullptr;
    T.emb_w = L.in_dim[t] - L.n_num[t];
    T.ug = W.ug[t] >= 0 ? ws + W.ug[t] : nullptr;
    T.dug = W.dug[t] >= 0 ? ws + W.dug[t] : nullptr;
    if (fold) {  // the folded k_bwd_mid accumulates gg0 | gbe0 into the fold replicas
      T.gg0 = T.fr;
      T.gbe0 = T.fr + H0;
    }
  }
  if (fold) {
    a.fr_zero = ws + W.fr;
    a.fr_zero_len = 2 * NREP * FRW;
  }
  a.target = b->target;
  a.weight = b->weight;
  a.rows = b->rows;
  a.row0 = b->row0;
  a.B = b->n_rows;
  a.cycle = b->cycle;
  a.t_base = b->t_base;
  a.eps = d->bn_eps;
  a.momentum = d->bn_momentum;
  const double thr = (double)d->dropout_p * 65536.0;  // 16-bit uniforms (tt_common.h dropout_keep_rk)
  a.drop_thr = (uint32_t)thr;
  a.drop_scale = a.drop_thr > 0 ? 1.0f / (1.0f - d->dropout_p) : 1.0f;
  a.D = d->latent;
  a.n_tiles = (int)((b->n_rows + ROWS - 1) / ROWS);
  a.slab_ld = (int)L.slab_ld;
  a.logit_scale = params + L.ls;
  a.lsr = ws + W.lsr;
  a.tgw = ws + W.tgw;
  a.det = (d->flags & TT_FLAG_DETERMINISTIC) ? 1 : 0;
  a.xcd_pair = fold ? 1 : 0;  // 64-row tiles on the XCD of the fold kernel's 128-row tile (tile64)
  a.l0_gx = (int)(padded_rows(b->n_rows) / ROWS);  // k_l0_fwd's row-tile blocks (Plan::n_tiles)
  a.dslot_lsr = ws + W.det_lsr;
}

// Segments of the parameter arena for k_reduce_adam: W/b ranges come from the
// per-tile partial slabs (k_top writes n_tiles_top of them, the 64-row
// kernels n_tiles), BN affine / embeddings / logit_scale from gacc.
// part: RED_ALL (every range, one k_reduce_adam), RED_EARLY / RED_LATE (the
// step's reduction split for TT_FLAG_DEFER_LATE: the late half holds W4, the
// BN1 affine, W8 | b8 and logit_scale -- first read by the NEXT step's
// k_l4_fwd / k_top -- and zeroes the BN1 moment sums and folds the loss; the
// early half everything k_l0_fwd of the next step reads).
enum { RED_ALL = 0, RED_EARLY = 1, RED_LATE = 2 };
static RedArgs make_red(const tt_model_desc* d, const Layout& L, const WsLayout& W, float* ws, const Plan& P,
                        float* grad, int part = RED_ALL) {
  RedArgs r;
  std::memset(&r, 0, sizeof(r));
  int k = 0;
  bool overflow = false;
  bool late_range = false;  // set around the late ranges below
  const int G = part == RED_LATE ? LATE_G : RED_G;
  // returns whether the range went into this part's segment list
  auto add = [&](int64_t off, int64_t len, int kind, int tower, int64_t so, int n_slabs, float* rep = nullptr,
                 int64_t rep_stride = 0) -> bool {
    if (len <= 0) return false;
    if ((part == RED_EARLY && late_range) || (part == RED_LATE && !late_range)) return false;
    if (k >= MAX_SEG) {  // 1 + 2 x 6 + 1 ranges at most (static_assert MAX_SEG >= 14)
      overflow = true;   // reported as n_seg < 0: the caller returns an error before enqueuing
      return false;
    }
    r.seg[k].off = off;
    r.seg[k].len = len;
    r.seg[k].kind = kind;
    r.seg[k].tower = tower;
    r.seg[k].slab_off = so;
    r.seg[k].n_slabs = n_slabs;
    r.seg[k].rep = rep;
    r.seg[k].rep_stride = rep_stride;
    ++k;
    return true;
  };
  int64_t emb_total = L.slot[0][TT_SLOT_W0];
  add(0, emb_total, 1, 0, 0, 0);
  for (int t = 0; t < 2; ++t) {
    const int64_t* s = L.slot[t];
    float* bng = ws + W.bng[t];
    // gamma|beta slots are adjacent and unpadded (H0, H1 multiples of 4): same order as a replica
    if (P.fold) {
      float* fr = ws + W.fr + (int64_t)t * NREP * FRW;
      for (int kind = 3; kind <= 4; ++kind) {
        // only when added: in a late-half list nothing is, and seg[k - 1] is
        // then another range -- or, at k = 0, the caller's stack before the
        // struct (that write corrupted the pending step's kernel arguments:
        // GPU faults at the first deferred step; tests/native/abi_host_check)
        if (!add(s[kind == 3 ? TT_SLOT_W0 : TT_SLOT_B0], kind == 3 ? (int64_t)H0 * L.in_dim[t] : H0, kind, t,
                 L.so[t][0], P.n_tiles_mid, fr, FRW))
          continue;
        Seg& g = r.seg[k - 1];
        g.in = L.in_dim[t];
        g.kp = L.kp[t];
        g.k0 = ws + W.k0s[t];
        g.xsh = ws + W.xsh[t];
      }
      if (add(s[TT_SLOT_G0], 2 * H0, 2, t, 0, 0, fr, FRW))
        r.seg[k - 1].keep = 1;  // zeroed by the next step's k_l0_fwd
    } else {
      // W0 and b0 apart: the slab's W0 range may be sized for the folded P | Q
      add(s[TT_SLOT_W0], (int64_t)H0 * L.in_dim[t], 0, t, L.so[t][0], P.n_tiles_mid);  // k_bwd_first's tiles
      add(s[TT_SLOT_B0], H0, 0, t, L.so[t][1], P.n_tiles_mid);
      add(s[TT_SLOT_G0], 2 * H0, 2, t, 0, 0, bng, BNG);
    }
    late_range = true;
    add(s[TT_SLOT_W4], s[TT_SLOT_G1] - s[TT_SLOT_W4], 0, t, L.so[t][2], P.n_tiles_mid);
    add(s[TT_SLOT_G1], 2 * H1, 2, t, 0, 0, bng + 2 * H0, BNG);
    // k_top_pair's 64-row partials: more than one round of slab loads, split
    const int k8 = RED_E == 64 && P.n_tiles_top > G * RED_UNR && P.n_tiles_top <= 2 * G * RED_UNR ? 5 : 0;
    add(s[TT_SLOT_W8], s[TT_SLOT_B8] + d->latent - s[TT_SLOT_W8], k8, t, L.so[t][4], P.n_tiles_top);
    late_range = false;
  }
  late_range = true;
  add(L.ls, 1, 2, 0, 0, 0, ws + W.lsr, LSR);
  late_range = false;
  if (overflow) {
    r.n_seg = -1;
    return r;
  }
  // element space of k_reduce_adam: every range starts on a block (one
  // segment per block); kind 3 ranges hold every W0 element twice (P and Q
  // halves of one 32-lane group).  Ranges are laid out heaviest first (slab
  // loads per element: W8, then W0 / W4, the replica ranges last) on a grid
  // of ~2.3 blocks per CU: k_reduce_adam 7.6-8.0 -> 7.2-7.7 us at cfg 3 in
  // six interleaved rounds.  No arithmetic changes (each
  // element's sum is its own, in the same slab order).
  int order[sizeof(r.seg) / sizeof(r.seg[0])];
  for (int i = 0; i < k; ++i) order[i] = i;
#if TT_RED_HEAVY_FIRST
  auto cost = [&](int i) -> int {
    const Seg& g = r.seg[i];
    return g.kind == 0 || g.kind == 3 ? g.n_slabs : g.kind == 5 ? 2 * g.n_slabs : 0;
  };
  std::stable_sort(order, order + k, [&](int x, int y) { return cost(x) > cost(y); });
#endif
  int64_t vo = 0;
  for (int j = 0; j < k; ++j) {
    const int i = order[j];
    r.blk0[j] = (int32_t)(vo / RED_E);
    r.blk_seg[j] = i;
    r.seg[i].voff = vo;
    const int64_t len = r.seg[i].len;
    r.seg[i].vlen = r.seg[i].kind == 3 ? 2 * len : r.seg[i].kind == 5 ? (len + 31) / 32 * 64 : len;
    vo = round_up(vo + r.seg[i].vlen, RED_E);
  }
  r.vn = vo;
  // the first replica segment (BN0 affine: no slab loads) fills the next
  // step's Adam-coefficient slot
  r.next_seg = -1;
  for (int i = 0; i < k && r.next_seg < 0 && part != RED_LATE; ++i)
    if (r.seg[i].kind == 2) r.next_seg = i;
  r.lsr = part == RED_EARLY ? nullptr : ws + W.lsr;  // the loss fold rides with logit_scale's replicas
  r.late_pending = reinterpret_cast<int64_t*>(ws + W.late);
  r.n_seg = k;
  r.n_slabs = P.n_tiles;
  r.n = L.n;
  r.slab[0] = ws + W.slab[0];
  r.slab[1] = ws + W.slab[1];
  r.slab_ld = L.slab_ld;
  r.gacc = ws + W.gacc;
  r.grad = grad;
  return r;
}

// The per-step fields of a training step's reduction (part as make_red):
// the BN moment sums it zeroes (BN0's with the early half: k_l0_fwd of the
// next step accumulates them; BN1's with the late half: k_l4_fwd), the loss
// target and the Adam hyperparameters.
template <class A>
static void red_step_fields(A& r, int part, const WsLayout& W, float* w, int64_t n_rows, tt_state* state,
                            int32_t apply_adam, float* params, float* exp_avg, float* exp_avg_sq,
                            const tt_adam_hp* hp, AdamSlot* slots) {
  r.inv_b = 1.f / (float)n_rows;
  for (int t = 0; t < 2; ++t) {
    r.zero_buf[2 * t] = w + W.st0[t];
    r.zero_len[2 * t] = part == RED_LATE ? 0 : NREP * ST0S;
    r.zero_buf[2 * t + 1] = w + W.st1[t];
    r.zero_len[2 * t + 1] = part == RED_EARLY ? 0 : NREP * ST1S;
  }
  r.loss_state = state;
  if (apply_adam) {
    r.apply_adam = 1;
    r.p = params;
    r.m = exp_avg;
    r.v = exp_avg_sq;
    r.lr = hp->lr;
    r.b1 = hp->beta1;
    r.b2 = hp->beta2;
    r.eps = hp->eps;
    r.adam_slots = slots;
    r.state = state;
  }
}

// A late half in the kernel-argument form (LateRed: MAX_LATE_SEG segments)
static LateRed to_late(const RedArgs& r) {
  LateRed q;
  std::memset(&q, 0, sizeof(q));
  for (int i = 0; i < r.n_seg; ++i) {
    q.seg[i] = r.seg[i];
    q.blk0[i] = r.blk0[i];
    q.blk_seg[i] = r.blk_seg[i];
  }
#define TT_CP(f) q.f = r.f;
  TT_CP(n_seg) TT_CP(n_slabs) TT_CP(n) TT_CP(vn) TT_CP(slab_ld) TT_CP(gacc) TT_CP(grad) TT_CP(lsr) TT_CP(loss_state)
  TT_CP(apply_adam) TT_CP(p) TT_CP(m) TT_CP(v) TT_CP(lr) TT_CP(b1) TT_CP(b2) TT_CP(eps) TT_CP(adam_slots)
  TT_CP(next_seg) TT_CP(state) TT_CP(step_host) TT_CP(inv_b) TT_CP(late_pending) TT_CP(late_mark)
#undef TT_CP
  for (int i = 0; i < 2; ++i) q.slab[i] = r.slab[i];
  for (int i = 0; i < 4; ++i) {
    q.zero_buf[i] = r.zero_buf[i];
    q.zero_len[i] = r.zero_len[i];
  }
  return q;
}
// k_l0_fwd blocks per tower row (y) that carry a late half: half of its
// element blocks each, rounded to 8 so the row tiles keep their XCDs
static int late_gx(const LateRed& q) { return (int)round_up((q.vn / RED_E + 1) / 2, 8); }

static int launch_check() {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? TT_OK : (int)e;
}

// A training step's k_top is k_top_pair (from B = 4096): its tiles are the
// W8 / b8 slab count of the step's reduction and deterministic fold
static void pair_plan(Plan* P) {
  if (P->top_pair) P->n_tiles_top = P->n_tiles_pair;
}

struct Ctx {
  Layout L;
  WsLayout W;
  Plan P;
};

// Every argument error is decided here, on the host, before any HIP call.
static int prepare(const tt_model_desc* d, const tt_batch* b, int64_t ws_bytes, int64_t min_rows, Ctx* c) {
  if (!desc_ok(d) || !batch_ok(d, b)) return TT_ERR_ARG;
  if (b->n_rows < min_rows) return TT_ERR_BATCH_TOO_SMALL;
  c->L = make_layout(d);
  int rc = make_plan(d, c->L, std::max<int64_t>(b->n_rows, 1), &c->P);
  if (rc) return rc;
  c->W = make_ws(c->L, std::max<int64_t>(b->n_rows, 1));
  if ((int64_t)(c->W.total * sizeof(float)) > ws_bytes) return TT_ERR_WORKSPACE;
  set_lds_attrs();
  return TT_OK;
}

// Kernel launch with optional profiling events: when (e0, e1) are given the
// kernel goes through hipExtLaunchKernelGGL, which stamps e0/e1 from the
// kernel's own dispatch packet (start / end of the kernel, no gap), so
// bench.py's HIP-event timing is the kernel duration rocprofv3 reports.
struct Evs {
  hipEvent_t e0 = nullptr, e1 = nullptr;
};
template <typename K, typename... A>
static void launch(K kern, dim3 g, dim3 b, size_t lds, hipStream_t s, Evs ev, A... args) {
  if (ev.e0 && ev.e1)
    hipExtLaunchKernelGGL(kern, g, b, (uint32_t)lds, s, ev.e0, ev.e1, 0, args...);
  else
    hipLaunchKernelGGL(kern, g, b, lds, s, args...);
}

// k_l0_fwd's instance for this step, or -1 when a deferred late half rides
// along (late != NULL) and no LATE instance covers the geometry
static int l0_late_ok(const StepArgs& a) {
  return a.tw[0].num_vec && a.tw[1].num_vec && l0_ks(std::max(a.tw[0].kp, a.tw[1].kp)) <= 2;
}
static void launch_l0(const StepArgs& a, const Plan& P, hipStream_t s, Evs ev = {}, const LateRed* late = nullptr) {
  // instance by the widest tower input (32-wide K steps held in registers)
  // and whether both towers take the aligned numeric-only gather
  const int ks = l0_ks(std::max(a.tw[0].kp, a.tw[1].kp));
  const bool vec = a.tw[0].num_vec && a.tw[1].num_vec;
  const dim3 blk(4 * ROWS);
  LateRed none;
  std::memset(&none, 0, sizeof(none));
  if (late) {  // the caller checked l0_late_ok
    const dim3 grid(P.n_tiles + late_gx(*late), 2);
    if (ks == 1)
      launch(k_l0_fwd<ROWS, 1, true, true>, grid, blk, P.lds_l0, s, ev, a, *late);
    else
      launch(k_l0_fwd<ROWS, 2, true, true>, grid, blk, P.lds_l0, s, ev, a, *late);
    return;
  }
  const dim3 grid(P.n_tiles_fwd, 2), blk32(4 * 32);
#define TT_L0(KS)                                                                        \
  if (ks == KS) {                                                                        \
    if (P.fwd_rows == 32) {                                                              \
      if (vec)                                                                           \
        launch(k_l0_fwd<32, KS, true, false>, grid, blk32, P.lds_l0, s, ev, a, none);    \
      else                                                                               \
        launch(k_l0_fwd<32, KS, false, false>, grid, blk32, P.lds_l0, s, ev, a, none);   \
    } else if (vec) {                                                                    \
      launch(k_l0_fwd<ROWS, KS, true, false>, grid, blk, P.lds_l0, s, ev, a, none);      \
    } else {                                                                             \
      launch(k_l0_fwd<ROWS, KS, false, false>, grid, blk, P.lds_l0, s, ev, a, none);     \
    }                                                                                    \
    return;                                                                              \
  }
  TT_L0(1)
  TT_L0(2)
  TT_L0(4)
  TT_L0(8)
#undef TT_L0
}
static void launch_l4(const StepArgs& a, const Plan& P, hipStream_t s, Evs ev = {}) {
  if (P.fwd_rows == 32)
    launch(k_l4_fwd<32>, dim3(P.n_tiles_fwd, 2), dim3(4 * 32), P.lds_l4_32, s, ev, a);
  else
    launch(k_l4_fwd<ROWS>, dim3(P.n_tiles_fwd, 2), dim3(4 * ROWS), P.lds_l4, s, ev, a);
}
static void launch_mid(const StepArgs& a, const Plan& P, hipStream_t s, Evs ev = {}) {
  if (!a.fr_zero) {
    if (P.bwd_rows == 32)
      launch(k_bwd_mid<32>, dim3(P.n_tiles_mid, 2), dim3(4 * 32), P.lds_mid, s, ev, a);
    else
      launch(k_bwd_mid<ROWS>, dim3(P.n_tiles_mid, 2), dim3(4 * ROWS), P.lds_mid, s, ev, a);
    return;
  }
  const dim3 grid(P.n_tiles_mid, 2), blk(4 * FOLD_ROWS);
  if (a.tw[0].num_vec && a.tw[1].num_vec)
    launch(k_bwd_mid_fold<FOLD_ROWS, true>, grid, blk, P.lds_mid, s, ev, a);
  else
    launch(k_bwd_mid_fold<FOLD_ROWS, false>, grid, blk, P.lds_mid, s, ev, a);
}
// folded BN0 backward: nothing to launch (its event pair stays unrecorded:
// tt_step_plan tells the caller which kernels a step runs)
static void launch_first(const StepArgs& a, const Plan& P, hipStream_t s, Evs ev = {}) {
  if (a.fr_zero) return;
  if (P.bwd_rows == 32)
    launch(k_bwd_first<32>, dim3(P.n_tiles_mid, 2), dim3(4 * 32), P.lds_first, s, ev, a);
  else
    launch(k_bwd_first<ROWS>, dim3(P.n_tiles_mid, 2), dim3(4 * ROWS), P.lds_first, s, ev, a);
}
static void launch_reduce(const RedArgs& r, hipStream_t s, Evs ev = {}, bool ex = false) {
  const dim3 grid((unsigned)(r.vn / RED_E)), blk(RED_E * RED_G);
  if (ex)  // data-parallel exchange inside the reduction (tt_train_step_dp: Adam slots set)
    launch(k_reduce_adam<true, true>, grid, blk, 0, s, ev, r);
  else if (r.adam_slots || !r.apply_adam)  // <true> reads no coefficients when there is no Adam
    launch(k_reduce_adam<true, false>, grid, blk, 0, s, ev, r);
  else
    launch(k_reduce_adam<false, false>, grid, blk, 0, s, ev, r);
}

// ---- peer-memory exchange region (tt_ar_*): [flags of the standalone
// exchange: TT_AR_MAX_RANKS x AR_BLOCKS][flags of the fused step:
// TT_AR_MAX_RANKS x ar_red_blocks(n)][slot 0][slot 1][push words:
// 2 parities x TT_AR_MAX_RANKS sources x ar_slot_floats(n), 8 B each] ----
static constexpr int AR_BLOCKS = 32;
static int64_t ar_slot_floats(int64_t n) { return (n + 63) / 64 * 64; }
static int64_t ar_ll_bytes(int64_t n) { return 2 * (int64_t)TT_AR_MAX_RANKS * ar_slot_floats(n) * 8; }
// k_reduce_adam blocks of any model with n parameters: every segment's
// element range is at most 2 len + 64 long and starts on a block
static int64_t ar_red_blocks(int64_t n) { return (2 * n) / RED_E + 2 * MAX_SEG + 1; }
static int64_t ar_flag_bytes(int64_t n) { return (int64_t)TT_AR_MAX_RANKS * (AR_BLOCKS + ar_red_blocks(n)) * 8; }
static uint64_t* ar_ll_base(void* region, int64_t n) {
  return (uint64_t*)((char*)region + ar_flag_bytes(n) + 2 * ar_slot_floats(n) * (int64_t)sizeof(float));
}

// Deterministic mode: fold the per-block partial slots the kernel of stage
// `pt` just stored into replica 0 of each accumulator (k_det_fold), or
// scatter the embedding gradients in batch-row order (k_det_scatter).
enum DetPoint { DET_L0, DET_L4, DET_TOP, DET_MID, DET_FIRST };
static void det_fold(const StepArgs& a, const Plan& P, DetPoint pt, hipStream_t s) {
  if (!a.det) return;
  if (pt == DET_FIRST) {
    if (P.fold) return;
    int tables = 0, maxq = 0;
    for (int t = 0; t < 2; ++t)
      for (int j = 0; j < a.tw[t].n_cat; ++j) {
        ++tables;
        maxq = std::max(maxq, a.tw[t].emb_rows[j] * a.tw[t].emb_dim);
      }
    if (tables)
      hipLaunchKernelGGL(k_det_scatter, dim3((unsigned)((maxq + 255) / 256), (unsigned)tables), dim3(256), 0, s, a);
    return;
  }
  DetFold f;
  std::memset(&f, 0, sizeof(f));
  int n = 0, wmax = 0;
  auto add = [&](const float* src, float* dst, int slots, int width) {
    f.src[n] = src;
    f.dst[n] = dst;
    f.n_slots[n] = slots;
    f.width[n] = width;
    wmax = std::max(wmax, width);
    ++n;
  };
  for (int t = 0; t < 2; ++t) {
    const TowerDev& T = a.tw[t];
    if (pt == DET_L0) add(T.dslot, T.st0, P.n_tiles_fwd, 2 * H0);
    if (pt == DET_L4) add(T.dslot, T.st1, P.n_tiles_fwd, 2 * H1);
    if (pt == DET_TOP) add(T.dslot, T.gg1, P.n_tiles_top, 2 * H1);
    if (pt == DET_MID) {
      if (P.fold)
        add(T.dslot, T.fr, P.n_tiles_mid, FRW);
      else
        add(T.dslot, T.gg0, P.n_tiles_mid, 2 * H0);
    }
  }
  // (the generic top's embedding backward writes no (dls, loss) slots: its
  // replicas stay as the caller zeroed them)
  if (pt == DET_TOP && !(P.top_gen && a.mode == TOP_EMB_BWD)) add(a.dslot_lsr, a.lsr, P.n_tiles_top, 2);
  hipLaunchKernelGGL(k_det_fold, dim3((unsigned)((wmax + DET_COLS - 1) / DET_COLS), (unsigned)n),
                     dim3(DET_COLS * DET_GROUPS), 0, s, f);
}

template <bool EMB>
static void launch_top_t(const StepArgs& a, const Plan& P, int grid_y, hipStream_t s, Evs ev) {
  const dim3 grid(P.n_tiles_top, grid_y), blk(4 * P.top_rows);
  if (P.ndt == 4 && P.top_rows == 64)
    launch(k_top<4, 64, EMB>, grid, blk, P.lds_top, s, ev, a);
  else if (P.ndt == 4)
    launch(k_top<4, 128, EMB>, grid, blk, P.lds_top, s, ev, a);
  else if (P.top_rows == 64)
    launch(k_top<8, 64, EMB>, grid, blk, P.lds_top, s, ev, a);
  else
    launch(k_top<8, 128, EMB>, grid, blk, P.lds_top, s, ev, a);
}
static void launch_top(const StepArgs& a, const Plan& P, int grid_y, hipStream_t s, Evs ev = {}) {
  if (P.top_gen) {  // LATENT > 128 (tt_topgen.hip); no per-kernel events on this path
    const dim3 g2(P.n_tiles, 2), g1(P.n_tiles), blk(GEN_NTH);
    if (a.mode != TOP_EMB_BWD) hipLaunchKernelGGL(k_top_gen_fwd, g2, blk, P.lds_gen_fwd, s, a);
    if (a.mode == TOP_FWD || a.mode == TOP_TRAIN || a.mode == TOP_BWD_GIVEN)
      hipLaunchKernelGGL(k_cos_gen, g1, blk, 0, s, a);
    if (a.mode == TOP_TRAIN || a.mode == TOP_BWD_GIVEN || a.mode == TOP_EMB_BWD)
      hipLaunchKernelGGL(k_top_gen_bwd, g2, blk, P.lds_gen_bwd, s, a);
    (void)grid_y;
    (void)ev;
    return;
  }
  if (a.mode == TOP_TRAIN && P.top_pair) {  // (training steps set n_tiles_top = n_tiles_pair: pair_plan)
    const dim3 g(P.n_tiles_pair), b(8 * P.pair_rows);
    if (P.pair_rows == 32) {
      if (P.ndt == 4)
        launch(k_top_pair<4, 32>, g, b, P.lds_pair, s, ev, a);
      else
        launch(k_top_pair<8, 32>, g, b, P.lds_pair, s, ev, a);
    } else {
      if (P.ndt == 4)
        launch(k_top_pair<4, 64>, g, b, P.lds_pair, s, ev, a);
      else
        launch(k_top_pair<8, 64>, g, b, P.lds_pair, s, ev, a);
    }
    return;
  }
  if (a.mode == TOP_EMB_FWD || a.mode == TOP_EMB_BWD)
    launch_top_t<true>(a, P, grid_y, s, ev);
  else
    launch_top_t<false>(a, P, grid_y, s, ev);
}

}  // namespace tt

using namespace tt;

extern "C" {

int32_t tt_abi_version(void) { return TT_ABI_VERSION; }

void tt_range_push(const char* message) {
  if (message) roctxRangePushA(message);
}
void tt_range_pop(void) { roctxRangePop(); }

int64_t tt_struct_size(int32_t which) {
  switch (which) {
    case TT_STRUCT_MODEL_DESC: return (int64_t)sizeof(tt_model_desc);
    case TT_STRUCT_BATCH: return (int64_t)sizeof(tt_batch);
    case TT_STRUCT_ADAM_HP: return (int64_t)sizeof(tt_adam_hp);
    case TT_STRUCT_STATE: return (int64_t)sizeof(tt_state);
    case TT_STRUCT_AR_PEERS: return (int64_t)sizeof(tt_ar_peers);
    default: return -1;
  }
}

int64_t tt_param_count(const tt_model_desc* d) {
  if (!desc_ok(d)) return TT_ERR_ARG;
  return make_layout(d).n;
}

int32_t tt_param_offsets(const tt_model_desc* d, int64_t* out) {
  if (!desc_ok(d) || !out) return TT_ERR_ARG;
  const Layout L = make_layout(d);
  for (int t = 0; t < 2; ++t)
    for (int j = 0; j < TT_MAX_CAT; ++j) out[t * TT_MAX_CAT + j] = L.emb_off[t][j];
  for (int t = 0; t < 2; ++t)
    for (int s = 0; s < TT_SLOTS_PER_TOWER; ++s) out[2 * TT_MAX_CAT + t * TT_SLOTS_PER_TOWER + s] = L.slot[t][s];
  out[2 * TT_MAX_CAT + 2 * TT_SLOTS_PER_TOWER] = L.ls;
  return TT_OK;
}

int32_t tt_step_plan(const tt_model_desc* d, int64_t batch, int32_t* info, int32_t n_info) {
  if (!desc_ok(d) || batch < 1 || !info || n_info < 4) return TT_ERR_ARG;
  const Layout L = make_layout(d);
  Plan P;
  const int rc = make_plan(d, L, batch, &P);
  if (rc) return rc;
  info[0] = P.fold ? 1 : 0;
  info[1] = P.top_rows;
  info[2] = P.fold ? FOLD_ROWS : P.bwd_rows;
  info[3] = P.fold ? 5 : 6;
  if (n_info >= 5) info[4] = P.top_pair ? 1 : 0;
  if (n_info >= 6) info[5] = P.ndt;
  if (n_info >= 7) info[6] = P.fwd_rows;
  if (n_info >= 8) info[7] = P.top_pair ? P.pair_rows : P.top_rows;
  return TT_OK;
}

int64_t tt_buffer_count(const tt_model_desc* d) {
  if (!desc_ok(d)) return TT_ERR_ARG;
  return 2 * (2 * H0 + 2 * H1);
}

int64_t tt_workspace_bytes(const tt_model_desc* d, int64_t max_batch) {
  if (!desc_ok(d) || max_batch < 1) return TT_ERR_ARG;
  const Layout L = make_layout(d);
  return make_ws(L, max_batch).total * (int64_t)sizeof(float);
}

static int32_t forward_impl(const tt_model_desc* d, const float* params, float* buffers, int64_t* nbt,
                            const tt_batch* b, int32_t train, uint64_t seed, int64_t step, void* ws,
                            int64_t ws_bytes, float* score, float* emb, tt_stream_t stream) {
  if (!params || !buffers || !nbt || !ws || (!score && !emb)) return TT_ERR_ARG;
  Ctx c;
  int rc = prepare(d, b, ws_bytes, train ? 2 : 0, &c);
  if (rc) return rc;
  if (b->n_rows == 0) return TT_OK;
  hipStream_t s = (hipStream_t)stream;
  float* w = (float*)ws;
  StepArgs a;
  fill_args(a, d, c.L, c.W, c.P.fold, params, buffers, nbt, b, w);
  a.train = train ? 1 : 0;
  a.update_stats = a.train;
  a.seed = seed;
  a.step_host = step;
  a.mode = emb ? TOP_EMB_FWD : TOP_FWD;
  a.score = score;
  a.emb = emb;
  if (train) {
    for (int t = 0; t < 2; ++t) {
      (void)hipMemsetAsync(w + c.W.st0[t], 0, sizeof(float) * NREP * ST0S, s);
      (void)hipMemsetAsync(w + c.W.st1[t], 0, sizeof(float) * NREP * ST1S, s);
    }
  }
  launch_l0(a, c.P, s);
  if (train) det_fold(a, c.P, DET_L0, s);
  launch_l4(a, c.P, s);
  if (train) det_fold(a, c.P, DET_L4, s);
  launch_top(a, c.P, 1, s);
  return launch_check();
}

int32_t tt_forward(const tt_model_desc* d, const float* params, float* buffers, int64_t* nbt, const tt_batch* b,
                   int32_t train, uint64_t seed, int64_t step, void* ws, int64_t ws_bytes, float* score,
                   tt_stream_t stream) {
  if (!score) return TT_ERR_ARG;
  return forward_impl(d, params, buffers, nbt, b, train, seed, step, ws, ws_bytes, score, nullptr, stream);
}

int32_t tt_embed_forward(const tt_model_desc* d, const float* params, float* buffers, int64_t* nbt,
                         const tt_batch* b, int32_t train, uint64_t seed, int64_t step, void* ws, int64_t ws_bytes,
                         float* emb, tt_stream_t stream) {
  if (!emb) return TT_ERR_ARG;
  return forward_impl(d, params, buffers, nbt, b, train, seed, step, ws, ws_bytes, nullptr, emb, stream);
}

// The backward without the folded BN0 backward (k_bwd_mid + k_bwd_first):
// eval-mode backward and input gradients need dZ0 per row, which the fold
// never forms.
static void unfold(Plan& P) {
  if (!P.fold) return;  // (already the unfolded plan, possibly on 32-row tiles)
  P.fold = false;
  P.bwd_rows = ROWS;
  P.n_tiles_mid = P.n_tiles;
  P.lds_mid = MidLds<ROWS>::bytes;
}

static int32_t backward_impl(const tt_model_desc* d, const float* params, const float* buffers, const tt_batch* b,
                             const float* dscore, const float* demb, int32_t train, uint64_t seed, int64_t step,
                             void* ws, int64_t ws_bytes, float* grad, float* dx0, float* dx1, tt_stream_t stream) {
  if (!params || (!dscore && !demb) || !ws || !grad) return TT_ERR_ARG;
  if (!train && !buffers) return TT_ERR_ARG;  // eval: running statistics
  Ctx c;
  int rc = prepare(d, b, ws_bytes, train ? 2 : 0, &c);
  if (rc) return rc;
  if ((dx0 && d->n_num[0] <= 0) || (dx1 && d->n_num[1] <= 0)) return TT_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  if (b->n_rows == 0) {  // an empty eval batch: every gradient is zero
    (void)hipMemsetAsync(grad, 0, sizeof(float) * c.L.n, s);
    return launch_check();
  }
  if (!train || dx0 || dx1) unfold(c.P);
  float* w = (float*)ws;
  // running-stat buffers are read (eval) but never updated by a backward
  StepArgs a;
  fill_args(a, d, c.L, c.W, c.P.fold, params, train ? nullptr : const_cast<float*>(buffers), nullptr, b, w);
  a.train = train ? 1 : 0;
  a.update_stats = 0;
  a.seed = seed;
  a.step_host = step;
  a.mode = demb ? TOP_EMB_BWD : TOP_BWD_GIVEN;
  a.dscore = dscore;
  a.demb = demb;
  a.tw[0].dxn = dx0;
  a.tw[1].dxn = dx1;
  if (!train) {  // eval: no dropout, BN affine with the running statistics
    a.drop_thr = 0;
    a.drop_scale = 1.f;
  }
  RedArgs r = make_red(d, c.L, c.W, w, c.P, grad);
  if (r.n_seg < 0) return TT_ERR_UNSUPPORTED;
  (void)hipMemsetAsync(w + c.W.gacc, 0, sizeof(float) * c.L.n, s);
  for (int t = 0; t < 2; ++t) (void)hipMemsetAsync(w + c.W.bng[t], 0, sizeof(float) * NREP * BNG, s);
  (void)hipMemsetAsync(w + c.W.lsr, 0, sizeof(float) * NREP * LSR, s);
  if (c.P.fold) (void)hipMemsetAsync(w + c.W.fr, 0, sizeof(float) * 2 * NREP * FRW, s);
  launch_top(a, c.P, 2, s);
  det_fold(a, c.P, DET_TOP, s);
  launch_mid(a, c.P, s);
  det_fold(a, c.P, DET_MID, s);
  launch_first(a, c.P, s);
  det_fold(a, c.P, DET_FIRST, s);
  r.inv_b = 1.f / (float)b->n_rows;
  launch_reduce(r, s);
  return launch_check();
}

int32_t tt_backward(const tt_model_desc* d, const float* params, const tt_batch* b, const float* dscore,
                    uint64_t seed, int64_t step, void* ws, int64_t ws_bytes, float* grad, tt_stream_t stream) {
  if (!dscore) return TT_ERR_ARG;
  return backward_impl(d, params, nullptr, b, dscore, nullptr, 1, seed, step, ws, ws_bytes, grad, nullptr, nullptr,
                       stream);
}

int32_t tt_backward_ex(const tt_model_desc* d, const float* params, const float* buffers, const tt_batch* b,
                       const float* dscore, int32_t train, uint64_t seed, int64_t step, void* ws, int64_t ws_bytes,
                       float* grad, float* dx_firm, float* dx_ceo, tt_stream_t stream) {
  if (!dscore) return TT_ERR_ARG;
  return backward_impl(d, params, buffers, b, dscore, nullptr, train, seed, step, ws, ws_bytes, grad, dx_firm,
                       dx_ceo, stream);
}

int32_t tt_embed_backward(const tt_model_desc* d, const float* params, const tt_batch* b, const float* demb,
                          uint64_t seed, int64_t step, void* ws, int64_t ws_bytes, float* grad, tt_stream_t stream) {
  if (!demb) return TT_ERR_ARG;
  return backward_impl(d, params, nullptr, b, nullptr, demb, 1, seed, step, ws, ws_bytes, grad, nullptr, nullptr,
                       stream);
}

int32_t tt_embed_backward_ex(const tt_model_desc* d, const float* params, const float* buffers, const tt_batch* b,
                             const float* demb, int32_t train, uint64_t seed, int64_t step, void* ws,
                             int64_t ws_bytes, float* grad, float* dx_firm, float* dx_ceo, tt_stream_t stream) {
  if (!demb) return TT_ERR_ARG;
  return backward_impl(d, params, buffers, b, nullptr, demb, train, seed, step, ws, ws_bytes, grad, dx_firm, dx_ceo,
                       stream);
}

static int32_t train_step_impl(const tt_model_desc* d, float* params, float* buffers, int64_t* nbt,
                               const tt_batch* b, const tt_adam_hp* hp, uint64_t seed, tt_state* state, void* ws,
                               int64_t ws_bytes, float* grad, float* exp_avg, float* exp_avg_sq, int32_t apply_adam,
                               tt_stream_t stream, void* const* events, const RedExchange* x = nullptr,
                               int32_t co_ranks = 1) {
  if (!params || !buffers || !nbt || !state || !ws || !grad) return TT_ERR_ARG;
  if (apply_adam && (!hp || !exp_avg || !exp_avg_sq)) return TT_ERR_ARG;
  if (b && b->cycle > 0 && b->n_rows < 1) return TT_ERR_ARG;
  Ctx c;
  int rc = prepare(d, b, ws_bytes, 2, &c);
  if (rc) return rc;
  pair_plan(&c.P);
  hipStream_t s = (hipStream_t)stream;
  float* w = (float*)ws;
  // TT_FLAG_DEFER_LATE / TT_FLAG_LATE_PENDING: single-GPU Adam steps of the
  // folded plan only (decided here, before anything is enqueued)
  const bool defer = (d->flags & TT_FLAG_DEFER_LATE) != 0, pending = (d->flags & TT_FLAG_LATE_PENDING) != 0;
  if ((defer || pending) && (!apply_adam || x)) return TT_ERR_UNSUPPORTED;
  RedArgs r = make_red(d, c.L, c.W, w, c.P, grad, defer ? RED_EARLY : RED_ALL);
  if (r.n_seg < 0) return TT_ERR_UNSUPPORTED;
  r.late_mark = defer ? 1 : -1;
  if (x) {
    // every block of the reduction waits for its peers' same block: all of
    // them (co_ranks grids when ranks share this device) must be resident at
    // once, else the caller keeps the two-launch exchange
    const int64_t blocks = r.vn / RED_E;
    if (blocks > ar_red_blocks(c.L.n)) return TT_ERR_UNSUPPORTED;
    int dev = 0, cus = 0, per_cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_reduce_adam<true, true>, RED_E * RED_G, 0) !=
            hipSuccess)
      return TT_ERR_UNSUPPORTED;
    if (blocks * std::max(co_ranks, 1) > (int64_t)per_cu * cus) return TT_ERR_UNSUPPORTED;
    r.x = *x;
    r.x.blocks = (int32_t)ar_red_blocks(c.L.n);
  }
  StepArgs a;
  fill_args(a, d, c.L, c.W, c.P.fold, params, buffers, nbt, b, w);
  a.train = 1;
  a.update_stats = 1;
  a.seed = seed;
  a.state = state;
  a.mode = TOP_TRAIN;
  if (apply_adam) {
    a.adam_slots = reinterpret_cast<AdamSlot*>(w + c.W.adam);
    a.adam_lr = hp->lr;
    a.adam_b1 = hp->beta1;
    a.adam_b2 = hp->beta2;
    a.adam_eps = hp->eps;
  }
  auto ev = [&](int k) {
    Evs e;
    if (events) {
      e.e0 = (hipEvent_t)events[2 * k];
      e.e1 = (hipEvent_t)events[2 * k + 1];
    }
    return e;
  };
  if ((defer || pending) && !l0_late_ok(a)) return TT_ERR_UNSUPPORTED;  // (nothing enqueued yet)
  if (defer || pending) {  // the late half rides in the 64-row k_l0_fwd: 64-row forward tiles
    c.P.fwd_rows = ROWS;
    c.P.n_tiles_fwd = c.P.n_tiles;
  }
  LateRed late;
  if (pending) {  // the previous step's late half (same batch size: the caller flushes otherwise)
    RedArgs lr = make_red(d, c.L, c.W, w, c.P, grad, RED_LATE);
    if (lr.n_seg < 0) return TT_ERR_UNSUPPORTED;
    red_step_fields(lr, RED_LATE, c.W, w, b->n_rows, state, 1, params, exp_avg, exp_avg_sq, hp, a.adam_slots);
    late = to_late(lr);
  }
  launch_l0(a, c.P, s, ev(0), pending ? &late : nullptr);
  det_fold(a, c.P, DET_L0, s);
  launch_l4(a, c.P, s, ev(1));
  det_fold(a, c.P, DET_L4, s);
  launch_top(a, c.P, 2, s, ev(2));
  det_fold(a, c.P, DET_TOP, s);
  launch_mid(a, c.P, s, ev(3));
  det_fold(a, c.P, DET_MID, s);
  launch_first(a, c.P, s, ev(4));
  det_fold(a, c.P, DET_FIRST, s);
  red_step_fields(r, defer ? RED_EARLY : RED_ALL, c.W, w, b->n_rows, state, apply_adam, params, exp_avg,
                  exp_avg_sq, hp, a.adam_slots);
  launch_reduce(r, s, ev(5), x != nullptr);
  return launch_check();
}

int32_t tt_train_flush(const tt_model_desc* d, float* params, float* buffers, int64_t* nbt, const tt_batch* b,
                       const tt_adam_hp* hp, tt_state* state, void* ws, int64_t ws_bytes, float* grad,
                       float* exp_avg, float* exp_avg_sq, tt_stream_t stream) {
  if (!params || !buffers || !nbt || !state || !ws || !grad || !hp || !exp_avg || !exp_avg_sq) return TT_ERR_ARG;
  Ctx c;
  int rc = prepare(d, b, ws_bytes, 2, &c);
  if (rc) return rc;
  pair_plan(&c.P);
  hipStream_t s = (hipStream_t)stream;
  float* w = (float*)ws;
  RedArgs lr = make_red(d, c.L, c.W, w, c.P, grad, RED_LATE);
  if (lr.n_seg < 0) return TT_ERR_UNSUPPORTED;
  red_step_fields(lr, RED_LATE, c.W, w, b->n_rows, state, 1, params, exp_avg, exp_avg_sq, hp,
                  reinterpret_cast<AdamSlot*>(w + c.W.adam));
  const LateRed late = to_late(lr);
  Range rg("tt_train_flush");
  hipLaunchKernelGGL(k_reduce_late, dim3((unsigned)(late.vn / RED_E)), dim3(RED_E * LATE_G), 0, s, late);
  hipLaunchKernelGGL(k_clear_late, dim3(1), dim3(1), 0, s, late.late_pending);
  return launch_check();
}

int32_t tt_train_steps(const tt_model_desc* d, float* params, float* buffers, int64_t* nbt, const tt_batch* b,
                       const tt_adam_hp* hp, uint64_t seed, tt_state* state, void* ws, int64_t ws_bytes, float* grad,
                       float* exp_avg, float* exp_avg_sq, int32_t n_steps, tt_stream_t stream) {
  if (!b || b->cycle <= 0 || n_steps < 0) return TT_ERR_ARG;  // the batch must follow the device step counter
  // a deferred late half needs the caller's pending record between steps
  // (TT_FLAG_LATE_PENDING on the next call, tt_train_flush at the end): with
  // the flags passed unchanged to every step, n - 1 late halves would be lost
  if (d && (d->flags & (TT_FLAG_DEFER_LATE | TT_FLAG_LATE_PENDING))) return TT_ERR_UNSUPPORTED;
  Range rg("tt_train_steps");
  for (int32_t k = 0; k < n_steps; ++k) {
    const int32_t rc = train_step_impl(d, params, buffers, nbt, b, hp, seed, state, ws, ws_bytes, grad, exp_avg,
                                       exp_avg_sq, 1, stream, nullptr);
    if (rc) return rc;
  }
  return TT_OK;
}

int32_t tt_train_step(const tt_model_desc* d, float* params, float* buffers, int64_t* nbt, const tt_batch* b,
                      const tt_adam_hp* hp, uint64_t seed, tt_state* state, void* ws, int64_t ws_bytes, float* grad,
                      float* exp_avg, float* exp_avg_sq, int32_t apply_adam, tt_stream_t stream) {
  Range rg("tt_train_step");
  return train_step_impl(d, params, buffers, nbt, b, hp, seed, state, ws, ws_bytes, grad, exp_avg, exp_avg_sq,
                         apply_adam, stream, nullptr);
}

int32_t tt_train_step_ev(const tt_model_desc* d, float* params, float* buffers, int64_t* nbt, const tt_batch* b,
                         const tt_adam_hp* hp, uint64_t seed, tt_state* state, void* ws, int64_t ws_bytes,
                         float* grad, float* exp_avg, float* exp_avg_sq, int32_t apply_adam, tt_stream_t stream,
                         void* const* events) {
  return train_step_impl(d, params, buffers, nbt, b, hp, seed, state, ws, ws_bytes, grad, exp_avg, exp_avg_sq,
                         apply_adam, stream, events);
}

int32_t tt_train_step_dp(const tt_model_desc* d, float* params, float* buffers, int64_t* nbt, const tt_batch* b,
                         const tt_adam_hp* hp, uint64_t seed, tt_state* state, void* ws, int64_t ws_bytes,
                         float* grad, float* exp_avg, float* exp_avg_sq, const tt_ar_peers* peers, int32_t rank,
                         int32_t world, int32_t co_ranks, int32_t* err, int64_t wait_us, tt_stream_t stream) {
  if (!peers || world < 1 || world > TT_AR_MAX_RANKS || rank < 0 || rank >= world || !err || co_ranks < 1 ||
      !hp || !exp_avg || !exp_avg_sq || !desc_ok(d) ||
      (peers->protocol != TT_AR_PULL && peers->protocol != TT_AR_PUSH))
    return TT_ERR_ARG;
  if (peers->protocol == TT_AR_PUSH && world > TT_AR_PUSH_MAX_RANKS) return TT_ERR_UNSUPPORTED;
  const int64_t n = make_layout(d).n;
  RedExchange x;
  std::memset(&x, 0, sizeof(x));
  for (int q = 0; q < world; ++q) {
    if (!peers->region[q]) return TT_ERR_ARG;
    char* base = (char*)peers->region[q];
    x.flags[q] = (uint64_t*)(base + (int64_t)TT_AR_MAX_RANKS * AR_BLOCKS * 8);
    x.slot[q] = (float*)(base + ar_flag_bytes(n));
    x.ll[q] = ar_ll_base(peers->region[q], n);
  }
  x.protocol = peers->protocol;
  x.slot_stride = ar_slot_floats(n);
  x.rank = rank;
  x.world = world;
  x.err = err;
  x.wait_ticks = (uint64_t)(wait_us > 0 ? wait_us : 2000000) * 100ull;  // s_memrealtime: 100 MHz
  Range rg("tt_train_step_dp");
  return train_step_impl(d, params, buffers, nbt, b, hp, seed, state, ws, ws_bytes, grad, exp_avg, exp_avg_sq, 1,
                         stream, nullptr, &x, co_ranks);
}

int32_t tt_adam_apply(float* params, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                      const tt_adam_hp* hp, tt_state* state, int64_t step_host, tt_stream_t stream) {
  if (!params || !grad || !exp_avg || !exp_avg_sq || !hp || n < 0) return TT_ERR_ARG;
  if (!state && step_host < 1) return TT_ERR_ARG;
  if (n == 0) return TT_OK;
  const int nb = (int)std::min<int64_t>((n + 255) / 256, 2048);
  hipLaunchKernelGGL(k_adam, dim3(nb), dim3(256), 0, (hipStream_t)stream, params, grad, exp_avg, exp_avg_sq, n,
                     hp->lr, hp->beta1, hp->beta2, hp->eps, state, step_host);
  return launch_check();
}

static int cosine_launch(const float* u, const float* v, const float* tg, const float* wt, int64_t B, int32_t D,
                         const float* ls, float inv_batch, float* score, float* du, float* dv, float* loss,
                         float* dls, bool bwd, hipStream_t s) {
  if (!u || !v || !ls || !score || B < 0 || D <= 0) return TT_ERR_ARG;
  if (bwd && (!tg || !wt || !du || !dv || !loss || !dls)) return TT_ERR_ARG;
  if (B == 0) return TT_OK;
  const bool vec0 = (D % 4 == 0);
  const int64_t rows_per_block = vec0 ? COS_ROWS_PER_BLOCK : COS_ROWS_PER_BLOCK_ITER;
  // at most 16,384 blocks: at B = 4M, D = 128 each loops 8 times over its
  // rows (the next rows prefetched) and ends with the two loss / dls
  // atomics.  Probed with the two sums in one line, as bench.py and the
  // tests pass them (tools/cosprobe): 1,024-4,096 blocks 5.07-5.26 TB/s
  // (4,096: a partial last wave of blocks), 16,384 5.41, 65,536 4.53 (the
  // atomics on one line serialise)
  const int nb = (int)std::max<int64_t>(1, std::min<int64_t>((B + rows_per_block - 1) / rows_per_block, 16384));
  const dim3 g(nb), t(256);
  const bool vec = (D % 4 == 0) && ((uintptr_t)u % 16 == 0) && ((uintptr_t)v % 16 == 0) &&
                   (!bwd || ((uintptr_t)du % 16 == 0 && (uintptr_t)dv % 16 == 0));
  const int n4 = D / 4;
#define TT_COS(NV)                                                                                             \
  do {                                                                                                         \
    if (bwd)                                                                                                   \
      hipLaunchKernelGGL((k_cosine<NV, true>), g, t, 0, s, u, v, tg, wt, B, D, ls, inv_batch, score, du, dv,  \
                         loss, dls);                                                                           \
    else                                                                                                       \
      hipLaunchKernelGGL((k_cosine<NV, false>), g, t, 0, s, u, v, tg, wt, B, D, ls, inv_batch, score, du, dv, \
                         loss, dls);                                                                           \
  } while (0)
  if (vec && n4 <= 16)
    TT_COS(1);
  else if (vec && n4 <= 32)
    TT_COS(2);
  else if (vec && n4 <= 64)
    TT_COS(4);
  else if (vec && n4 <= 128)
    TT_COS(8);
  else if (bwd)
    hipLaunchKernelGGL((k_cosine_scalar<true>), g, t, 0, s, u, v, tg, wt, B, D, ls, inv_batch, score, du, dv, loss,
                       dls);
  else
    hipLaunchKernelGGL((k_cosine_scalar<false>), g, t, 0, s, u, v, tg, wt, B, D, ls, inv_batch, score, du, dv, loss,
                       dls);
#undef TT_COS
  return launch_check();
}

int32_t tt_cosine_forward(const float* u, const float* v, int64_t B, int32_t D, const float* logit_scale,
                          float* score, tt_stream_t stream) {
  return cosine_launch(u, v, nullptr, nullptr, B, D, logit_scale, 0.f, score, nullptr, nullptr, nullptr, nullptr,
                       false, (hipStream_t)stream);
}

int32_t tt_cosine_mse_fwd_bwd(const float* u, const float* v, const float* target, const float* weight, int64_t B,
                              int32_t D, const float* logit_scale, float inv_batch, float* score, float* du,
                              float* dv, float* loss_sum, float* dls_sum, tt_stream_t stream) {
  return cosine_launch(u, v, target, weight, B, D, logit_scale, inv_batch, score, du, dv, loss_sum, dls_sum, true,
                       (hipStream_t)stream);
}

int32_t tt_stream_copy(const void* src, void* dst, int64_t bytes, tt_stream_t stream) {
  if (!src || !dst || bytes < 0 || bytes % 16 || ((uintptr_t)src | (uintptr_t)dst) % 16) return TT_ERR_ARG;
  const int64_t n4 = bytes / 16;
  if (n4 == 0) return TT_OK;
  // one float4 per thread, contiguous blocks (k_stream_copy); launched in
  // pieces of at most 2^31 - 1 blocks
  const int64_t per = (int64_t)0x7FFFFFFF * COPY_THREADS;
  for (int64_t o = 0; o < n4; o += per) {
    const int64_t m = std::min(per, n4 - o);
    hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)((m + COPY_THREADS - 1) / COPY_THREADS)), dim3(COPY_THREADS), 0,
                       (hipStream_t)stream, (const float4*)src + o, (float4*)dst + o, m);
  }
  return (int32_t)hipGetLastError();
}

// One epoch's sample order of DataLoader(shuffle=True): torch 2.10's CPU
// randperm(n, generator seeded with `seed`) -- the mt19937 stream of the
// generator (32-bit seed, 32-bit outputs) driving the Fisher-Yates swaps
// out[i] <-> out[i + mt() % (n - i)] -- bit for bit.  torch runs the swaps one
// dependent cache miss at a time (23 ns per pair at 10M); here the swap
// targets are drawn AHEAD steps early and their lines prefetched, so the loop
// runs at the memory system's rate.  Host memory, no HIP call.
int32_t tt_randperm(int64_t n, uint64_t seed, int64_t* out) {
  if (n < 0 || (n > 0 && !out)) return TT_ERR_ARG;
  // torch draws 64-bit randoms from n >= 2^32 / 20 on: not restated here
  if (n >= (int64_t)(0xFFFFFFFFu / 20)) return TT_ERR_UNSUPPORTED;
  for (int64_t i = 0; i < n; ++i) out[i] = i;
  if (n < 2) return TT_OK;
  std::mt19937 mt((uint32_t)seed);
  constexpr int AHEAD = 64;  // power of two
  uint32_t zq[AHEAD];
  const int64_t last = n - 1;  // swaps i = 0 .. n - 2
  int64_t drawn = 0;
  for (; drawn < std::min<int64_t>(AHEAD, last); ++drawn) {
    zq[drawn] = (uint32_t)(drawn + (uint32_t)mt() % (uint32_t)(n - drawn));
    __builtin_prefetch(out + zq[drawn], 1, 0);
  }
  for (int64_t i = 0; i < last; ++i) {
    const int64_t z = zq[i & (AHEAD - 1)];
    if (drawn < last) {
      const uint32_t zn = (uint32_t)(drawn + (uint32_t)mt() % (uint32_t)(n - drawn));
      zq[drawn & (AHEAD - 1)] = zn;
      __builtin_prefetch(out + zn, 1, 0);
      ++drawn;
    }
    const int64_t v = out[i];
    out[i] = out[z];
    out[z] = v;
  }
  return TT_OK;
}

// ---------------------------------------------------------------------------
// Contrastive (InfoNCE / retrieval): tt_nce_*, tt_retrieval_ranks
// ---------------------------------------------------------------------------
}  // extern "C"

namespace tt {
namespace nce {

struct NceLayout {
  int64_t m, n, m_pad, n_pad, nti, ntj;
  int64_t n_bm, n_bn;       // sim GEMM blocks
  int64_t n_rp, n_cp;       // row / column partial counts
  int64_t d_pad, pntj;      // grad outputs: columns (D) in 16-tiles
  int64_t split_f, kps_f;   // dF = E' C   (K = n_pad)
  int64_t split_c, kps_c;   // dC = E'^T F (K = m_pad)
  int64_t E, rowpart, colpart, rowsum, diag, a, b, shift, part, rmax, cmax, total;  // float offsets
};

static int64_t rup(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// split-K so a grad GEMM launches >= ~4 blocks per CU; each split >= 8 K chunks
static void pick_split(int64_t out_rows, int64_t d, int64_t K, int64_t* split, int64_t* kps) {
  const int64_t blocks = ((out_rows + CfgGrad::BM - 1) / CfgGrad::BM) * ((d + CfgGrad::BN - 1) / CfgGrad::BN);
  int64_t s = std::max<int64_t>(1, (1024 + blocks - 1) / blocks);
  const int64_t chunks = (K + BK - 1) / BK;
  s = std::min<int64_t>(s, std::max<int64_t>(1, chunks / 8));
  *kps = rup((chunks + s - 1) / s, 1) * BK;
  *split = (K + *kps - 1) / *kps;
}

static NceLayout nce_layout(int64_t m, int64_t n, int d) {
  NceLayout L;
  L.m = m;
  L.n = n;
  L.m_pad = rup(std::max<int64_t>(m, 1), 16);
  L.n_pad = rup(std::max<int64_t>(n, 1), 16);
  L.nti = L.m_pad / 16;
  L.ntj = L.n_pad / 16;
  L.n_bm = (m + CfgSim::BM - 1) / CfgSim::BM;
  L.n_bn = (n + CfgSim::BN - 1) / CfgSim::BN;
  L.n_rp = L.n_bn * CfgSim::NWN;
  L.n_cp = L.n_bm * CfgSim::NWM;
  L.d_pad = rup(d, 16);
  L.pntj = L.d_pad / 16;
  pick_split(m, d, L.n_pad, &L.split_f, &L.kps_f);
  pick_split(n, d, L.m_pad, &L.split_c, &L.kps_c);
  int64_t off = 0;
  auto take = [&](int64_t k) { const int64_t o = off; off += rup(k, 64); return o; };
  L.E = take(L.nti * L.ntj * TILE);
  L.rowpart = take(L.n_rp * L.m_pad);
  L.colpart = take(L.n_cp * L.n_pad);
  L.rowsum = take(L.m_pad);
  L.diag = take(L.m_pad);
  L.a = take(L.m_pad);
  L.b = take(L.n_pad);
  L.shift = take(1);
  L.part = take(std::max(L.split_f * L.nti, L.split_c * L.ntj) * L.pntj * TILE);
  L.rmax = take(L.m_pad);  // robust mode: row / column maxima of s
  L.cmax = take(L.n_pad);
  L.total = off;
  return L;
}

static bool nce_args_ok(const float* f, const float* c, int64_t m, int64_t n, int d, int64_t row0) {
  if (!f || !c || m < 1 || n < 1 || d < 4 || d % 4) return false;
  if ((uintptr_t)f % 16 || (uintptr_t)c % 16) return false;
  return row0 >= 0 && row0 + m <= n;
}

static std::once_flag g_nce_attr;
static void nce_attrs() {
  std::call_once(g_nce_attr, [] {
    const void* sim[] = {(const void*)k_nce_sim<0>, (const void*)k_nce_sim<1>, (const void*)k_nce_sim<2>,
                         (const void*)k_nce_sim<3>, (const void*)k_nce_sim<4>};
    const void* grad[] = {(const void*)k_nce_dgrad<SRC_E_ROWS, false>, (const void*)k_nce_dgrad<SRC_E_AS_MK, false>,
                          (const void*)k_nce_dgrad<SRC_E_ROWS, true>, (const void*)k_nce_dgrad<SRC_E_AS_MK, true>};
    for (const void* k : sim) (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_SIM);
    for (const void* k : grad)
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_GRAD);
    (void)hipGetLastError();  // (see set_lds_attrs)
  });
}

static GemmArgs sim_args(const float* f, const float* c, int64_t m, int64_t n, int d, int64_t row0) {
  GemmArgs g;
  std::memset(&g, 0, sizeof(g));
  g.A = Opnd{f, d, m, d, 0, 0, nullptr, nullptr};
  g.B = Opnd{c, d, n, d, 0, 0, nullptr, nullptr};
  g.M = m;
  g.N = n;
  g.n_blocks_n = (int)((n + CfgSim::BN - 1) / CfgSim::BN);
  g.row0 = row0;
  return g;
}

}  // namespace nce
}  // namespace tt

extern "C" {

int64_t tt_nce_workspace_bytes(int64_t m, int64_t n, int32_t d) {
  if (m < 1 || n < 1 || d < 4 || d % 4) return TT_ERR_ARG;
  return tt::nce::nce_layout(m, n, d).total * (int64_t)sizeof(float);
}

int32_t tt_nce_norms(const float* f, const float* c, int64_t m, int64_t n, int32_t d, float* norm2,
                     tt_stream_t stream) {
  if (!f || !c || !norm2 || m < 1 || n < 1 || d < 1) return TT_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  (void)hipMemsetAsync(norm2, 0, 2 * sizeof(float), s);
  const int64_t groups = (m + n + 15) / 16;
  const int nb = (int)std::min<int64_t>(groups, 4096);
  hipLaunchKernelGGL(tt::nce::k_nce_norms, dim3(nb), dim3(256), 0, s, f, c, m, n, d, norm2);
  return launch_check();
}

int32_t tt_nce_forward(const float* f, const float* c, int64_t m, int64_t n, int32_t d, int64_t row0,
                       float temperature, const float* norm2, void* ws, int64_t ws_bytes, float* col_sum,
                       tt_stream_t stream) {
  using namespace tt::nce;
  if (!nce_args_ok(f, c, m, n, d, row0) || !norm2 || !ws || !col_sum || !(temperature > 0.f)) return TT_ERR_ARG;
  const NceLayout L = nce_layout(m, n, d);
  if (L.total * (int64_t)sizeof(float) > ws_bytes) return TT_ERR_WORKSPACE;
  nce_attrs();
  hipStream_t s = (hipStream_t)stream;
  float* w = (float*)ws;
  const float inv_tau = 1.0f / temperature;
  hipLaunchKernelGGL(k_nce_set_shift, dim3(1), dim3(64), 0, s, norm2, inv_tau, w + L.shift);
  hipLaunchKernelGGL(k_nce_diag, dim3((unsigned)((L.nti + 3) / 4)), dim3(256), 0, s, f, c, m, n, d, row0, inv_tau,
                     w + L.diag);
  GemmArgs g = sim_args(f, c, m, n, d, row0);
  g.inv_tau = inv_tau;
  g.shift = w + L.shift;
  g.E = w + L.E;
  g.e_nti = L.nti;
  g.e_ntj = L.ntj;
  g.rowpart = w + L.rowpart;
  g.colpart = w + L.colpart;
  g.m_pad = L.m_pad;
  g.n_pad = L.n_pad;
  hipLaunchKernelGGL(k_nce_sim<0>, dim3((unsigned)(L.n_bm * L.n_bn)), dim3(CfgSim::NTH), LDS_SIM, s, g);
  const int64_t tot = L.m_pad + L.n_pad;
  const int nb = (int)std::min<int64_t>((tot + 255) / 256, 4096);
  hipLaunchKernelGGL(k_nce_sums, dim3(nb), dim3(256), 0, s, w + L.rowpart, L.n_rp, L.m_pad, w + L.colpart, L.n_cp,
                     L.n_pad, w + L.rowsum, w + L.b);
  // column partial sums of these rows -> caller (n values; all-reduce SUM across row shards)
  (void)hipMemcpyAsync(col_sum, w + L.b, sizeof(float) * n, hipMemcpyDeviceToDevice, s);
  return launch_check();
}

int32_t tt_nce_loss(int64_t m, int64_t n, int32_t d, int64_t row0, int64_t batch, float temperature, void* ws,
                    int64_t ws_bytes, const float* col_sum, float* loss, int32_t* status, tt_stream_t stream) {
  using namespace tt::nce;
  if (m < 1 || n < 1 || d < 4 || !ws || !col_sum || !loss || batch < 2 || row0 < 0 || row0 + m > n)
    return TT_ERR_ARG;
  const NceLayout L = nce_layout(m, n, d);
  if (L.total * (int64_t)sizeof(float) > ws_bytes) return TT_ERR_WORKSPACE;
  (void)temperature;
  hipStream_t s = (hipStream_t)stream;
  float* w = (float*)ws;
  const int64_t tot = L.m_pad + L.n_pad;
  const int nb = (int)std::min<int64_t>((tot + 255) / 256, 4096);
  hipLaunchKernelGGL(k_nce_loss, dim3(nb), dim3(256), 0, s, w + L.rowsum, col_sum, w + L.diag, m, L.m_pad, n,
                     L.n_pad, row0, (float)(0.5 / (double)batch), w + L.shift, w + L.a, w + L.b, loss, status);
  return launch_check();
}

}  // extern "C"

template <bool LSE>
static int32_t nce_backward_impl(const float* f, const float* c, int64_t m, int64_t n, int32_t d, int64_t row0,
                                 int64_t batch, float temperature, void* ws, int64_t ws_bytes, float* df, float* dc,
                                 tt_stream_t stream) {
  using namespace tt::nce;
  if (!nce_args_ok(f, c, m, n, d, row0) || !ws || !df || !dc || batch < 2 || !(temperature > 0.f))
    return TT_ERR_ARG;
  const NceLayout L = nce_layout(m, n, d);
  if (L.total * (int64_t)sizeof(float) > ws_bytes) return TT_ERR_WORKSPACE;
  nce_attrs();
  hipStream_t s = (hipStream_t)stream;
  float* w = (float*)ws;
  const float scale = (float)(1.0 / (2.0 * (double)batch * (double)temperature));
  const float corr = (float)(1.0 / ((double)batch * (double)temperature));
  // dF = E' C  (M = m rows i, N = d, K = n_pad columns j)
  {
    GemmArgs g;
    std::memset(&g, 0, sizeof(g));
    g.A = Opnd{w + L.E, 0, m, L.n_pad, L.nti, L.ntj, w + L.a, w + L.b};
    g.B = Opnd{c, d, d, n, 0, 0, nullptr, nullptr};
    g.M = m;
    g.N = d;
    g.k_per_split = L.kps_f;
    g.n_blocks_n = (int)((d + CfgGrad::BN - 1) / CfgGrad::BN);
    g.part = w + L.part;
    g.p_nti = L.nti;
    g.p_ntj = L.pntj;
    const dim3 grid((unsigned)(((m + CfgGrad::BM - 1) / CfgGrad::BM) * g.n_blocks_n), (unsigned)L.split_f);
    hipLaunchKernelGGL((k_nce_dgrad<SRC_E_ROWS, LSE>), grid, dim3(CfgGrad::NTH), LDS_GRAD, s, g);
    const int64_t el = L.nti * L.pntj * 64;
    hipLaunchKernelGGL(k_nce_grad_finish, dim3((unsigned)std::min<int64_t>((el + 255) / 256, 8192)), dim3(256), 0,
                       s, w + L.part, L.split_f, L.nti, L.pntj, m, d, scale, corr, c, n, row0, df);
  }
  // dC = E'^T F  (M = n columns j, N = d, K = m_pad rows i)
  {
    GemmArgs g;
    std::memset(&g, 0, sizeof(g));
    g.A = Opnd{w + L.E, 0, n, L.m_pad, L.nti, L.ntj, w + L.a, w + L.b};
    g.B = Opnd{f, d, d, m, 0, 0, nullptr, nullptr};
    g.M = n;
    g.N = d;
    g.k_per_split = L.kps_c;
    g.n_blocks_n = (int)((d + CfgGrad::BN - 1) / CfgGrad::BN);
    g.part = w + L.part;
    g.p_nti = L.ntj;
    g.p_ntj = L.pntj;
    const dim3 grid((unsigned)(((n + CfgGrad::BM - 1) / CfgGrad::BM) * g.n_blocks_n), (unsigned)L.split_c);
    hipLaunchKernelGGL((k_nce_dgrad<SRC_E_AS_MK, LSE>), grid, dim3(CfgGrad::NTH), LDS_GRAD, s, g);
    const int64_t el = L.ntj * L.pntj * 64;
    hipLaunchKernelGGL(k_nce_grad_finish, dim3((unsigned)std::min<int64_t>((el + 255) / 256, 8192)), dim3(256), 0,
                       s, w + L.part, L.split_c, L.ntj, L.pntj, n, d, scale, corr, f, m, -row0, dc);
  }
  return launch_check();
}

extern "C" {

int32_t tt_nce_backward(const float* f, const float* c, int64_t m, int64_t n, int32_t d, int64_t row0,
                        int64_t batch, float temperature, void* ws, int64_t ws_bytes, float* df, float* dc,
                        tt_stream_t stream) {
  return nce_backward_impl<false>(f, c, m, n, d, row0, batch, temperature, ws, ws_bytes, df, dc, stream);
}

// ---- robust (two-exponent) InfoNCE: the fallback when tt_nce_loss reports underflow
int32_t tt_nce_maxes(const float* f, const float* c, int64_t m, int64_t n, int32_t d, int64_t row0,
                     float temperature, void* ws, int64_t ws_bytes, float* col_max, tt_stream_t stream) {
  using namespace tt::nce;
  if (!nce_args_ok(f, c, m, n, d, row0) || !ws || !col_max || !(temperature > 0.f)) return TT_ERR_ARG;
  const NceLayout L = nce_layout(m, n, d);
  if (L.total * (int64_t)sizeof(float) > ws_bytes) return TT_ERR_WORKSPACE;
  nce_attrs();
  hipStream_t s = (hipStream_t)stream;
  float* w = (float*)ws;
  GemmArgs g = sim_args(f, c, m, n, d, row0);
  g.inv_tau = 1.0f / temperature;
  g.rowpart = w + L.rowpart;
  g.colpart = w + L.colpart;
  g.m_pad = L.m_pad;
  g.n_pad = L.n_pad;
  hipLaunchKernelGGL(k_nce_sim<3>, dim3((unsigned)(L.n_bm * L.n_bn)), dim3(CfgSim::NTH), LDS_SIM, s, g);
  const int64_t tot = L.m_pad + L.n_pad;
  const int nb = (int)std::min<int64_t>((tot + 255) / 256, 4096);
  hipLaunchKernelGGL(k_nce_reduce_parts<true>, dim3(nb), dim3(256), 0, s, w + L.rowpart, L.n_rp, L.m_pad,
                     w + L.colpart, L.n_cp, L.n_pad, w + L.rmax, w + L.cmax);
  (void)hipMemcpyAsync(col_max, w + L.cmax, sizeof(float) * n, hipMemcpyDeviceToDevice, s);
  return launch_check();
}

int32_t tt_nce_forward_lse(const float* f, const float* c, int64_t m, int64_t n, int32_t d, int64_t row0,
                           float temperature, const float* col_max, void* ws, int64_t ws_bytes, float* col_sum,
                           tt_stream_t stream) {
  using namespace tt::nce;
  if (!nce_args_ok(f, c, m, n, d, row0) || !col_max || !ws || !col_sum || !(temperature > 0.f)) return TT_ERR_ARG;
  const NceLayout L = nce_layout(m, n, d);
  if (L.total * (int64_t)sizeof(float) > ws_bytes) return TT_ERR_WORKSPACE;
  nce_attrs();
  hipStream_t s = (hipStream_t)stream;
  float* w = (float*)ws;
  const float inv_tau = 1.0f / temperature;
  if (col_max != w + L.cmax)  // the caller's (all-reduced) column maxima
    (void)hipMemcpyAsync(w + L.cmax, col_max, sizeof(float) * n, hipMemcpyDeviceToDevice, s);
  hipLaunchKernelGGL(k_nce_diag, dim3((unsigned)((L.nti + 3) / 4)), dim3(256), 0, s, f, c, m, n, d, row0, inv_tau,
                     w + L.diag);
  GemmArgs g = sim_args(f, c, m, n, d, row0);
  g.inv_tau = inv_tau;
  g.E = w + L.E;
  g.e_nti = L.nti;
  g.e_ntj = L.ntj;
  g.rowpart = w + L.rowpart;
  g.colpart = w + L.colpart;
  g.m_pad = L.m_pad;
  g.n_pad = L.n_pad;
  g.rmax = w + L.rmax;
  g.cmax = w + L.cmax;
  hipLaunchKernelGGL(k_nce_sim<4>, dim3((unsigned)(L.n_bm * L.n_bn)), dim3(CfgSim::NTH), LDS_SIM, s, g);
  const int64_t tot = L.m_pad + L.n_pad;
  const int nb = (int)std::min<int64_t>((tot + 255) / 256, 4096);
  hipLaunchKernelGGL(k_nce_reduce_parts<false>, dim3(nb), dim3(256), 0, s, w + L.rowpart, L.n_rp, L.m_pad,
                     w + L.colpart, L.n_cp, L.n_pad, w + L.rowsum, w + L.b);
  (void)hipMemcpyAsync(col_sum, w + L.b, sizeof(float) * n, hipMemcpyDeviceToDevice, s);
  return launch_check();
}

int32_t tt_nce_loss_lse(int64_t m, int64_t n, int32_t d, int64_t row0, int64_t batch, void* ws, int64_t ws_bytes,
                        const float* col_max, const float* col_sum, float* loss, int32_t* status,
                        tt_stream_t stream) {
  using namespace tt::nce;
  if (m < 1 || n < 1 || d < 4 || !ws || !col_max || !col_sum || !loss || batch < 2 || row0 < 0 || row0 + m > n)
    return TT_ERR_ARG;
  const NceLayout L = nce_layout(m, n, d);
  if (L.total * (int64_t)sizeof(float) > ws_bytes) return TT_ERR_WORKSPACE;
  hipStream_t s = (hipStream_t)stream;
  float* w = (float*)ws;
  const int64_t tot = L.m_pad + L.n_pad;
  const int nb = (int)std::min<int64_t>((tot + 255) / 256, 4096);
  hipLaunchKernelGGL(k_nce_loss_lse, dim3(nb), dim3(256), 0, s, w + L.rowsum, w + L.rmax, col_sum, col_max,
                     w + L.diag, m, L.m_pad, n, L.n_pad, row0, (float)(0.5 / (double)batch), w + L.a, w + L.b, loss,
                     status);
  return launch_check();
}

int32_t tt_nce_backward_lse(const float* f, const float* c, int64_t m, int64_t n, int32_t d, int64_t row0,
                            int64_t batch, float temperature, void* ws, int64_t ws_bytes, float* df, float* dc,
                            tt_stream_t stream) {
  return nce_backward_impl<true>(f, c, m, n, d, row0, batch, temperature, ws, ws_bytes, df, dc, stream);
}

int64_t tt_rank_workspace_bytes(int64_t m) {
  if (m < 1) return TT_ERR_ARG;
  return (int64_t)sizeof(float) * 2 * ((m + 63) / 64 * 64);
}

int32_t tt_retrieval_ranks(const float* f, const float* c, int64_t m, int64_t n, int32_t d, int64_t row0, void* ws,
                           int64_t ws_bytes, int32_t* ranks, tt_stream_t stream) {
  using namespace tt::nce;
  if (!nce_args_ok(f, c, m, n, d, row0) || !ws || !ranks) return TT_ERR_ARG;
  if (tt_rank_workspace_bytes(m) > ws_bytes) return TT_ERR_WORKSPACE;
  nce_attrs();
  hipStream_t s = (hipStream_t)stream;
  const int64_t mp = (m + 63) / 64 * 64;
  float* diag = (float*)ws;
  int* cnt = (int*)((float*)ws + mp);
  (void)hipMemsetAsync(cnt, 0, sizeof(int) * m, s);
  hipLaunchKernelGGL(k_nce_diag, dim3((unsigned)(((m + 15) / 16 + 3) / 4)), dim3(256), 0, s, f, c, m, n, d, row0,
                     1.0f, diag);
  GemmArgs g = sim_args(f, c, m, n, d, row0);
  g.diag = diag;
  g.rank_cnt = cnt;
  const int64_t nblk = ((m + CfgSim::BM - 1) / CfgSim::BM) * g.n_blocks_n;
  hipLaunchKernelGGL(k_nce_sim<1>, dim3((unsigned)nblk), dim3(CfgSim::NTH), LDS_SIM, s, g);
  hipLaunchKernelGGL(k_rank_finish, dim3((unsigned)std::min<int64_t>((m + 255) / 256, 4096)), dim3(256), 0, s, cnt,
                     m, ranks);
  return launch_check();
}

// ---- semi_hard_negative_mining (contrastive.py:141-192) ----
static int64_t triplet_ws_floats(int64_t m, int64_t n, int64_t* m_pad, int64_t* n_rp) {
  using namespace tt::nce;
  *m_pad = (m + 63) / 64 * 64;
  *n_rp = ((n + CfgSim::BN - 1) / CfgSim::BN) * CfgSim::NWN;
  return *m_pad + 2 * 2 * (*n_rp) * (*m_pad);  // diag | semi_part (u64) | all_part (u64)
}

int64_t tt_triplet_workspace_bytes(int64_t m, int64_t n, int32_t d) {
  if (m < 1 || n < 1 || d < 4 || d % 4) return TT_ERR_ARG;
  int64_t mp, nrp;
  return triplet_ws_floats(m, n, &mp, &nrp) * (int64_t)sizeof(float);
}

int32_t tt_triplet_forward(const float* f, const float* c, int64_t m, int64_t n, int32_t d, int64_t row0,
                           float margin, int64_t batch, void* ws, int64_t ws_bytes, int32_t* hardest,
                           float* row_loss, float* loss, tt_stream_t stream) {
  using namespace tt::nce;
  if (!nce_args_ok(f, c, m, n, d, row0) || !ws || !hardest || !row_loss || !loss || batch < 2 || n < 2)
    return TT_ERR_ARG;
  int64_t mp, nrp;
  if (triplet_ws_floats(m, n, &mp, &nrp) * (int64_t)sizeof(float) > ws_bytes) return TT_ERR_WORKSPACE;
  nce_attrs();
  hipStream_t s = (hipStream_t)stream;
  float* diag = (float*)ws;
  uint64_t* semi = (uint64_t*)((float*)ws + mp);
  uint64_t* all = semi + nrp * mp;
  hipLaunchKernelGGL(k_nce_diag, dim3((unsigned)(((m + 15) / 16 + 3) / 4)), dim3(256), 0, s, f, c, m, n, d, row0,
                     1.0f, diag);
  GemmArgs g = sim_args(f, c, m, n, d, row0);
  g.diag = diag;
  g.margin = margin;
  g.semi_part = semi;
  g.all_part = all;
  g.m_pad = mp;
  const int64_t nblk = ((m + CfgSim::BM - 1) / CfgSim::BM) * g.n_blocks_n;
  hipLaunchKernelGGL(k_nce_sim<2>, dim3((unsigned)nblk), dim3(CfgSim::NTH), LDS_SIM, s, g);
  hipLaunchKernelGGL(k_triplet_finish, dim3((unsigned)std::min<int64_t>((m + 255) / 256, 4096)), dim3(256), 0, s,
                     semi, all, nrp, mp, m, diag, margin, (float)(1.0 / (double)batch), hardest, row_loss, loss);
  return launch_check();
}

int32_t tt_triplet_backward(const float* f, const float* c, int64_t m, int64_t n, int32_t d, int64_t row0,
                            int64_t batch, const int32_t* hardest, const float* row_loss, const float* grad_loss,
                            float* df, float* dc, tt_stream_t stream) {
  using namespace tt::nce;
  if (!nce_args_ok(f, c, m, n, d, row0) || !hardest || !row_loss || !grad_loss || !df || !dc || batch < 2)
    return TT_ERR_ARG;
  hipStream_t s = (hipStream_t)stream;
  (void)hipMemsetAsync(dc, 0, sizeof(float) * n * d, s);
  hipLaunchKernelGGL(k_triplet_bwd, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, s, f, c, m, d, row0, hardest,
                     row_loss, grad_loss, (float)(1.0 / (double)batch), df, dc);
  return launch_check();
}

// ---- data-parallel gradient exchange over peer memory (region layout at
// ar_flag_bytes above) ----
int64_t tt_ar_region_bytes(int64_t n) {
  if (n < 1) return TT_ERR_ARG;
  return ar_flag_bytes(n) + 2 * ar_slot_floats(n) * (int64_t)sizeof(float) + ar_ll_bytes(n);
}

int32_t tt_ar_alloc(int64_t bytes, void** region, void* ipc_handle) {
  if (bytes < 1 || !region || !ipc_handle) return TT_ERR_ARG;
  static_assert(sizeof(hipIpcMemHandle_t) == TT_AR_HANDLE_BYTES, "IPC handle size");
  void* p = nullptr;
  hipError_t e = hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  e = hipMemset(p, 0, (size_t)bytes);
  if (e == hipSuccess) {
    hipIpcMemHandle_t h;
    e = hipIpcGetMemHandle(&h, p);
    if (e == hipSuccess) std::memcpy(ipc_handle, &h, sizeof(h));
  }
  if (e != hipSuccess) {
    (void)hipFree(p);
    return (int)e;
  }
  *region = p;
  return TT_OK;
}

int32_t tt_ar_open(const void* ipc_handle, void** region) {
  if (!ipc_handle || !region) return TT_ERR_ARG;
  hipIpcMemHandle_t h;
  std::memcpy(&h, ipc_handle, sizeof(h));
  void* p = nullptr;
  const hipError_t e = hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) return (int)e;
  *region = p;
  return TT_OK;
}

int32_t tt_ar_close(void* region) { return region ? (int)hipIpcCloseMemHandle(region) : TT_ERR_ARG; }
int32_t tt_ar_free(void* region) { return region ? (int)hipFree(region) : TT_ERR_ARG; }

int32_t tt_ar_reset(void* region, int64_t n, tt_stream_t stream) {
  if (!region || n < 1) return TT_ERR_ARG;
  return (int)hipMemsetAsync(region, 0, (size_t)tt_ar_region_bytes(n), (hipStream_t)stream);
}

int32_t tt_ar_allreduce_adam(const tt_ar_peers* peers, int32_t rank, int32_t world, int64_t n, const float* grad,
                             float* grad_out, float* params, float* exp_avg, float* exp_avg_sq,
                             const tt_adam_hp* hp, tt_state* state, int64_t step_host, int32_t* err,
                             int64_t wait_us, tt_stream_t stream) {
  if (!peers || world < 1 || world > TT_AR_MAX_RANKS || rank < 0 || rank >= world || n < 1 || !grad || !err ||
      (peers->protocol != TT_AR_PULL && peers->protocol != TT_AR_PUSH))
    return TT_ERR_ARG;
  if (params && (!exp_avg || !exp_avg_sq || !hp)) return TT_ERR_ARG;
  if (!state && step_host < 1) return TT_ERR_ARG;
  ArArgs a;
  std::memset(&a, 0, sizeof(a));
  for (int q = 0; q < world; ++q) {
    if (!peers->region[q]) return TT_ERR_ARG;
    char* base = (char*)peers->region[q];
    a.flags[q] = (uint64_t*)base;
    a.slot[q] = (float*)(base + ar_flag_bytes(n));
    a.ll[q] = ar_ll_base(peers->region[q], n);
  }
  a.slot_stride = ar_slot_floats(n);
  a.rank = rank;
  a.world = world;
  a.blocks = AR_BLOCKS;
  a.n = n;
  a.grad = grad;
  a.grad_out = grad_out;
  a.p = params;
  a.m = exp_avg;
  a.v = exp_avg_sq;
  if (hp) {
    a.lr = hp->lr;
    a.b1 = hp->beta1;
    a.b2 = hp->beta2;
    a.eps = hp->eps;
  }
  a.state = state;
  a.step_host = step_host;
  a.err = err;
  // s_memrealtime runs at 100 MHz; default bound 2 s of polling, then give up (err)
  a.wait_ticks = (uint64_t)(wait_us > 0 ? wait_us : 2000000) * 100ull;
  if (peers->protocol == TT_AR_PUSH && world > TT_AR_PUSH_MAX_RANKS) return TT_ERR_UNSUPPORTED;
  Range rg("tt_ar_exchange");
  if (peers->protocol == TT_AR_PUSH) {
    hipLaunchKernelGGL(k_ar_adam_push, dim3(AR_BLOCKS), dim3(AR_THREADS), 0, (hipStream_t)stream, a);
  } else {
    hipLaunchKernelGGL(k_ar_adam, dim3(AR_BLOCKS), dim3(AR_THREADS), 0, (hipStream_t)stream, a);
  }
  return launch_check();
}

}  // extern "C"
