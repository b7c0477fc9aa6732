/*
 * ceo_tt.h -- C-ABI of the MI355X-native CEOFirmMatcher two-tower training
 * path (libceo_tt.so, HIP / gfx950).
 *
 * The reference (SMaric93/CEO-Recommender) is pure Python: its hot path is
 * ATen ops issued by CEOFirmMatcher.forward, loss.backward() and
 * optim.Adam.step().  It has no FFI of its own, so every entry point below
 * names the reference code it replaces (file:line under the reference's
 * ceo_firm_matching/ package).  The Python mirror that binds them with ctypes
 * is ceo-recommender_amd/ceo_firm_matching/_native.py; INTEGRATION.md shows
 * the binding a maintainer of the reference would add.
 *
 * Conventions
 *   - every pointer argument is a DEVICE pointer owned by the caller (torch
 *     tensors' data_ptr), fp32 row-major unless noted; descriptors
 *     (tt_model_desc, tt_batch, tt_adam_hp) are HOST structs;
 *   - no entry point allocates, synchronises or keeps global state; work is
 *     enqueued on the given hipStream_t (so all of it is graph-capturable);
 *   - return value: TT_OK or a negative TT_ERR_* (argument errors, detected
 *     on the host before anything is enqueued) or a positive hipError_t.
 */
#ifndef CEO_TT_H
#define CEO_TT_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TT_ABI_VERSION 6
#define TT_MAX_CAT 16      /* categorical columns per tower */

/* status codes */
#define TT_OK 0
#define TT_ERR_ARG (-1)            /* bad pointer / size */
#define TT_ERR_BATCH_TOO_SMALL (-2) /* train-mode BatchNorm needs B >= 2 (torch ValueError) */
#define TT_ERR_UNSUPPORTED (-3)    /* shape outside what the fused kernels cover */
#define TT_ERR_WORKSPACE (-4)      /* workspace too small */

typedef struct ihipStream_t* tt_stream_t; /* == hipStream_t */

/* Model geometry: CEOFirmMatcher(metadata, config)  (model.py:19-65).
 * tower 0 = firm, tower 1 = ceo.  Fixed by the reference architecture:
 * Linear(in,64) BN(64) ReLU Dropout Linear(64,32) BN(32) ReLU Dropout
 * Linear(32,latent)  (model.py:37-62).                                       */
typedef struct tt_model_desc {
  int32_t n_num[2];                    /* metadata n_firm_numeric / n_ceo_numeric */
  int32_t n_cat[2];                    /* len(firm_cat_counts) / len(ceo_cat_counts) */
  int32_t emb_dim[2];                  /* EMBEDDING_DIM_LARGE (48) / _MEDIUM (8) */
  int32_t latent;                      /* config.LATENT_DIM */
  int32_t cat_counts[2][TT_MAX_CAT];   /* embedding rows per categorical column */
  float dropout_p;                     /* nn.Dropout(0.1) */
  float bn_eps;                        /* 1e-5 */
  float bn_momentum;                   /* 0.1 */
  int32_t flags;                       /* TT_FLAG_* execution options */
} tt_model_desc;

/* tt_model_desc.flags
 * TT_FLAG_DETERMINISTIC: bitwise repeatable steps.  Cross-block sums (BN
 *   moments, BN-affine grads, the loss / logit_scale partials, the folded BN0
 *   sums, embedding gradients) are accumulated by float atomics in arrival
 *   order by default; with the flag every block stores its partial in a slot
 *   of its own and a fold kernel adds the slots in block order (one extra
 *   launch per reduction point).  The reference's CPU loop is repeatable
 *   under torch.manual_seed (training.py:36-57); so is a fused step with
 *   this flag.  The workspace layout does not depend on the flags.       */
#define TT_FLAG_DETERMINISTIC 1
/* TT_FLAG_DEFER_LATE (ABI v4): tt_train_step* runs only the EARLY half of the
 *   step's gradient reduction + Adam (embeddings, W0 / b0, BN0 affine: what
 *   the next step's first kernel reads); the LATE half (W4 / b4, BN1 affine,
 *   W8 / b8, logit_scale, and the step's loss into state->loss_sum) stays
 *   pending on the workspace.  Until it runs those parameters, their Adam
 *   moments and loss_sum hold the previous step's values.
 * TT_FLAG_LATE_PENDING: the previous step on this workspace deferred its late
 *   half (same batch size): run it inside this step's first kernel, as extra
 *   workgroups beside the row tiles -- the step keeps five launches and the
 *   late half leaves the critical path.
 * tt_train_flush runs a pending late half on its own (before parameters,
 *   moments or the loss are read, or a step of another batch size).  A late
 *   half runs only if the workspace records one (the step counter makes a
 *   stale LATE_PENDING a no-op on the device).  Both flags: single-GPU Adam
 *   steps (apply_adam = 1) of numeric-only towers with 16-B aligned rows and
 *   inputs up to 64 wide; otherwise TT_ERR_UNSUPPORTED, nothing enqueued.   */
#define TT_FLAG_DEFER_LATE 2
#define TT_FLAG_LATE_PENDING 4

/* One batch, described over dataset-resident arrays.  Row i of the batch is
 * dataset row rows[row0 + i] (or row0 + i when rows == NULL).  With cycle > 0
 * the offset comes from the device step counter instead (graph replay):
 * row0 = ((t - 1 - t_base) % cycle) * n_rows.  Replaces the per-sample
 * CEOFirmDataset.__getitem__ + collate + .to(DEVICE) (data.py:190-198,
 * training.py:40-42).                                                        */
typedef struct tt_batch {
  const float* num[2];     int64_t num_ld[2];   /* firm_numeric / ceo_numeric [N, ld] */
  const int64_t* cat[2];   int64_t cat_ld[2];   /* firm_cat / ceo_cat [N, ld] int64 */
  const float* target;                          /* match_means [N] */
  const float* weight;                          /* 1/(sd^2+1e-6) [N] */
  const int64_t* rows;                          /* permutation / index list or NULL */
  int64_t row0;
  int64_t n_rows;                               /* B */
  int64_t cycle;
  int64_t t_base;
} tt_batch;

/* torch.optim.Adam hyperparameters of train_model (training.py:32), as the
 * reference passes them: Python floats (double).  The coefficients follow
 * torch's _single_tensor_adam from these doubles (bias corrections in
 * double, each scalar cast to float where torch casts it), so a fused step
 * equals torch.optim.Adam applied to the same fp32 gradient. */
typedef struct tt_adam_hp {
  double lr, beta1, beta2, eps;
} tt_adam_hp;

/* Device-resident step counters (so a captured hipGraph can be replayed). */
typedef struct tt_state {
  int64_t step_done;   /* completed optimizer steps */
  int64_t step_cur;    /* step being executed (written by the first kernel) */
  float loss_sum;      /* += batch-mean weighted MSE of every step */
  float pad0;
  int64_t pad1;
} tt_state;

/* Slot ids for tt_param_offsets (float offsets into the flat parameter
 * arena, which is laid out in CEOFirmMatcher.parameters() order). */
enum {
  TT_SLOT_W0 = 0, TT_SLOT_B0, TT_SLOT_G0, TT_SLOT_BE0,
  TT_SLOT_W4, TT_SLOT_B4, TT_SLOT_G1, TT_SLOT_BE1, TT_SLOT_W8, TT_SLOT_B8,
  TT_SLOTS_PER_TOWER
};
#define TT_NUM_OFFSETS (2 * TT_MAX_CAT + 2 * TT_SLOTS_PER_TOWER + 1)
/* out[0..15]   firm embedding tables,  out[16..31] ceo embedding tables,
 * out[32..41]  firm tower slots,       out[42..51] ceo tower slots,
 * out[52]      logit_scale.            (-1 for absent tables)            */

int32_t tt_abi_version(void);

/* roctx ranges (rocprofiler-sdk-roctx) for callers that want their own host
 * regions in a rocprofv3 --marker-trace beside the library's: every
 * tt_train_step / tt_train_steps / tt_train_step_dp / tt_train_flush /
 * tt_ar_allreduce_adam call already opens one named after the entry point.
 * No-ops without a profiler.  (step and exchange attributed per
 * rank; the reference has no tracing of its own.)                          */
void tt_range_push(const char* message);
void tt_range_pop(void);

/* sizeof of the host descriptors as this library was compiled (ABI v4): a
 * binding checks its own struct definitions against them before the first
 * call (a struct a field short makes the library read past the caller's
 * object).  which = TT_STRUCT_*; -1 for an unknown id.                      */
#define TT_STRUCT_MODEL_DESC 0
#define TT_STRUCT_BATCH 1
#define TT_STRUCT_ADAM_HP 2
#define TT_STRUCT_STATE 3
#define TT_STRUCT_AR_PEERS 4
int64_t tt_struct_size(int32_t which);

/* Flat parameter arena size (floats) and per-parameter offsets. */
int64_t tt_param_count(const tt_model_desc* d);
int32_t tt_param_offsets(const tt_model_desc* d, int64_t* out /* TT_NUM_OFFSETS */);
/* BN running stats arena (floats): per tower running_mean0[64] running_var0[64]
 * running_mean1[32] running_var1[32]; num_batches_tracked lives in a separate
 * int64[4] array (firm bn1, firm bn5, ceo bn1, ceo bn5). */
/* How a training step of this model at this batch size runs (no GPU work):
 * info[0] = 1 when the BN0 backward is folded into k_bwd_mid (numeric-only
 * towers, widths % 4 == 0 and <= 64: k_bwd_first is not launched),
 * info[1] = k_top row tile, info[2] = k_bwd_mid (and k_bwd_first) row tile,
 * info[3] = kernels per tt_train_step (5 or 6; the event slots of
 * tt_train_step_ev are fixed: l0, l4, top, mid, first, reduce -- slot 4
 * stays unrecorded when folded),
 * info[4] (n_info >= 5) = 1 when the step's k_top is k_top_pair (both
 * towers' backward per block; from B = 4096),
 * info[5] (n_info >= 6) = latent tiles of 16 the top kernels are
 * instantiated for (4: LATENT <= 64, 8: LATENT <= 128),
 * info[6] (n_info >= 7) = k_l0_fwd / k_l4_fwd row tile,
 * info[7] (n_info >= 8) = the training step's top row tile (k_top_pair's
 * when info[4]).  Below the folded path (B < 8192) the tower kernels run
 * 32-row tiles: twice the blocks of a batch that leaves CUs idle at 64.
 * Replaces nothing in the reference (training.py:44-57 is one autograd
 * pass); a query for callers that time or trace the step.             */
int32_t tt_step_plan(const tt_model_desc* d, int64_t batch, int32_t* info, int32_t n_info);
int64_t tt_buffer_count(const tt_model_desc* d);
/* Bytes of the workspace for batches of up to max_batch.  Zero it once and
 * keep it with its trainer: its leading region (offsets independent of the
 * batch size) holds accumulators every fused step leaves zeroed for the next
 * one, so steps of different B may share it.                                */
int64_t tt_workspace_bytes(const tt_model_desc* d, int64_t max_batch);

/* Forward of CEOFirmMatcher (model.py:67-89).  train=1: batch-statistics
 * BatchNorm (+ running-stat update, model.py:39,43) and dropout drawn from the
 * counter RNG stream (seed, step); train=0: running stats, no dropout.
 * Writes score[B]; keeps what backward needs in ws.                        */
int32_t tt_forward(const tt_model_desc* d, const float* params, float* buffers, int64_t* nbt,
                   const tt_batch* b, int32_t train, uint64_t seed, int64_t step,
                   void* ws, int64_t ws_bytes, float* score, tt_stream_t stream);

/* Backward of the preceding train-mode tt_forward on the same ws/batch/seed/
 * step: autograd reverse of model.py:67-89 given dL/dscore (training.py:54).
 * Writes the full flat gradient grad[param_count] (overwrites).             */
int32_t tt_backward(const tt_model_desc* d, const float* params, const tt_batch* b,
                    const float* dscore, uint64_t seed, int64_t step,
                    void* ws, int64_t ws_bytes, float* grad, tt_stream_t stream);

/* tt_backward for a forward of either mode, with optional input gradients
 * (autograd of model.py:67-89 w.r.t. f_numeric / c_numeric as well as the
 * parameters: run_deep_extensions.py:564-590 integrated gradients calls
 * model.eval(), requires_grad_ on the numeric inputs and score.backward()).
 *   train=1: as tt_backward (batch statistics, the forward's dropout stream);
 *   train=0: the backward of an eval-mode tt_forward -- BatchNorm is the
 *            affine map of the running statistics in `buffers` (no batch
 *            coupling, B = 1 allowed), no dropout.
 * dx_firm [B, n_num[0]], dx_ceo [B, n_num[1]]: dL/d(numeric input), row-major
 * fp32 (nullable each).  grad[param_count] is overwritten.                   */
int32_t tt_backward_ex(const tt_model_desc* d, const float* params, const float* buffers,
                       const tt_batch* b, const float* dscore, int32_t train, uint64_t seed,
                       int64_t step, void* ws, int64_t ws_bytes, float* grad,
                       float* dx_firm, float* dx_ceo, tt_stream_t stream);

/* Tower embeddings: the raw tower outputs U = firm_tower(x_f), V =
 * ceo_tower(x_c) before the L2 normalisation (contrastive.py:52-72
 * get_embeddings; model.py:69-77).  emb is [2][B][latent]: U rows then V
 * rows.  Same BatchNorm / dropout semantics and workspace contract as
 * tt_forward; tt_embed_backward takes demb = dL/d(emb) [2][B][latent] and
 * writes the full flat gradient (logit_scale's entry is 0).               */
int32_t tt_embed_forward(const tt_model_desc* d, const float* params, float* buffers, int64_t* nbt,
                         const tt_batch* b, int32_t train, uint64_t seed, int64_t step,
                         void* ws, int64_t ws_bytes, float* emb, tt_stream_t stream);
int32_t tt_embed_backward(const tt_model_desc* d, const float* params, const tt_batch* b,
                          const float* demb, uint64_t seed, int64_t step,
                          void* ws, int64_t ws_bytes, float* grad, tt_stream_t stream);
/* ... of either mode with optional input gradients (as tt_backward_ex) */
int32_t tt_embed_backward_ex(const tt_model_desc* d, const float* params, const float* buffers,
                             const tt_batch* b, const float* demb, int32_t train, uint64_t seed,
                             int64_t step, void* ws, int64_t ws_bytes, float* grad,
                             float* dx_firm, float* dx_ceo, tt_stream_t stream);

/* One fused training step = training.py:44-57: forward, weighted MSE,
 * backward, and (apply_adam=1) the Adam update.  With apply_adam=0 only grad
 * is produced (data-parallel: all-reduce grad, then tt_adam_apply).
 * Dropout stream and Adam step t come from state (t = step_done + 1).       */
int32_t tt_train_step(const tt_model_desc* d, float* params, float* buffers, int64_t* nbt,
                      const tt_batch* b, const tt_adam_hp* hp, uint64_t seed, tt_state* state,
                      void* ws, int64_t ws_bytes, float* grad, float* exp_avg, float* exp_avg_sq,
                      int32_t apply_adam, tt_stream_t stream);

/* The pending late half of the last TT_FLAG_DEFER_LATE step on this
 * workspace (b: that step's batch; only n_rows and the geometry are used),
 * then the workspace records none.  A no-op on the device when nothing is
 * pending.  Replaces the remainder of optim.Adam.step (training.py:55).     */
int32_t tt_train_flush(const tt_model_desc* d, float* params, float* buffers, int64_t* nbt,
                       const tt_batch* b, const tt_adam_hp* hp, tt_state* state, void* ws,
                       int64_t ws_bytes, float* grad, float* exp_avg, float* exp_avg_sq,
                       tt_stream_t stream);

/* n_steps consecutive tt_train_step launches in one call (cycle-mode
 * batches: b->cycle > 0, each step's batch taken from the device step
 * counter, so the arguments do not change between steps): the epoch loop of
 * training.py:36-57 without a host round trip per step.  Same semantics as
 * n_steps calls of tt_train_step; returns the first error.  Not with
 * TT_FLAG_DEFER_LATE / TT_FLAG_LATE_PENDING in d->flags (TT_ERR_UNSUPPORTED,
 * nothing launched): a deferred chain needs the caller's pending record
 * between steps -- call tt_train_step per step, then tt_train_flush.       */
int32_t tt_train_steps(const tt_model_desc* d, float* params, float* buffers, int64_t* nbt,
                       const tt_batch* b, const tt_adam_hp* hp, uint64_t seed, tt_state* state,
                       void* ws, int64_t ws_bytes, float* grad, float* exp_avg, float* exp_avg_sq,
                       int32_t n_steps, tt_stream_t stream);

/* tt_train_step with per-kernel timing: when events != NULL, kernel k of the
 * step (k = 0..5: l0_fwd, l4_fwd, top, bwd_mid, bwd_first, reduce_adam) is
 * launched with hipExtLaunchKernelGGL(..., events[2k], events[2k+1]) (two
 * hipEvent_t, or NULL to launch it plainly): the events are stamped from the
 * kernel's own dispatch, i.e. they bracket exactly its execution (what
 * rocprofv3 --kernel-trace reports).  Used by bench.py's roofline leg.      */
int32_t tt_train_step_ev(const tt_model_desc* d, float* params, float* buffers, int64_t* nbt,
                         const tt_batch* b, const tt_adam_hp* hp, uint64_t seed, tt_state* state,
                         void* ws, int64_t ws_bytes, float* grad, float* exp_avg, float* exp_avg_sq,
                         int32_t apply_adam, tt_stream_t stream, void* const* events);

/* Adam over a flat arena (optim.Adam.step, training.py:55; torch 2.10
 * _single_tensor_adam arithmetic).  step t = state->step_cur when state is
 * not NULL (then state->step_done := t), else step_host.                    */
int32_t tt_adam_apply(float* params, const float* grad, float* exp_avg, float* exp_avg_sq,
                      int64_t n, const tt_adam_hp* hp, tt_state* state, int64_t step_host,
                      tt_stream_t stream);

/* Standalone fused L2-normalise + scaled cosine (+ weighted MSE fwd/bwd)
 * over precomputed tower outputs u, v [B, D] (model.py:79-87,
 * training.py:52).  score = exp(logit_scale) * <u/|u|, v/|v|>.
 *   tt_cosine_forward : score only.
 *   tt_cosine_mse_fwd_bwd : also loss_sum += sum w (s-t)^2 * inv_batch,
 *     dls_sum += sum ds*score, du, dv  with ds = 2 w (s-t) * inv_batch.      */
int32_t tt_cosine_forward(const float* u, const float* v, int64_t B, int32_t D,
                          const float* logit_scale, float* score, tt_stream_t stream);
int32_t tt_cosine_mse_fwd_bwd(const float* u, const float* v, const float* target,
                              const float* weight, int64_t B, int32_t D,
                              const float* logit_scale, float inv_batch, float* score,
                              float* du, float* dv, float* loss_sum, float* dls_sum,
                              tt_stream_t stream);

/* Device-to-device copy of `bytes` (a multiple of 16; 16-B aligned pointers)
 * with 16-B vector loads and stores: the HBM stream ceiling of this box,
 * measured with the same kind of kernel as the bandwidth-bound paths above
 * (bench.py's cosine roofline quotes it beside the 8 TB/s spec).  Replaces
 * nothing in the reference (a measurement probe).                           */
int32_t tt_stream_copy(const void* src, void* dst, int64_t bytes, tt_stream_t stream);

/* One epoch's batch order of DataLoader(dataset of n, shuffle=True): out[n]
 * (host memory) = torch 2.10 CPU torch.randperm(n, generator) for a
 * generator after manual_seed(seed) -- what RandomSampler.__iter__ draws
 * (reference training.py:36-44 via data.py's DataLoader), bit for bit, with
 * the Fisher-Yates swap targets prefetched ahead (no HIP call).
 * TT_ERR_UNSUPPORTED for n >= 2^32 / 20 (torch's 64-bit draw path): the
 * caller then uses torch.randperm.                                          */
int32_t tt_randperm(int64_t n, uint64_t seed, int64_t* out);

/* ---------------------------------------------------------------------------
 * Contrastive scoring (BASELINE cfg 5).
 *
 * info_nce_loss (contrastive.py:102-138) over firm rows F [m, d] (a shard
 * starting at global row row0) against ALL ceo rows C [n, d]:
 *   S = F C^T / temperature,  loss = (CE(S, diag) + CE(S^T, diag)) / 2,
 * with batch = the global B (n).  Data-parallel use: each rank passes its F
 * shard and the all-gathered C; all-reduce MAX of norm2, SUM of col_sum and
 * loss; the dc of every rank are summed (reduce-scatter) for the C shard.
 *   1. tt_nce_norms    : norm2 = {max_i |f_i|^2, max_j |c_j|^2}; the shared
 *      exponent shift sqrt(norm2[0] norm2[1]) / temperature bounds every
 *      logit, so one exp per element serves both softmaxes.
 *   2. tt_nce_forward  : E = exp(S - shift) kept in ws, row sums, diag;
 *      col_sum[n] = column sums of E over these m rows.
 *   3. tt_nce_loss     : loss += this shard's share (col_sum complete);
 *      *status += number of row / column sums below 1e-30 (exp underflow,
 *      inputs far from L2-normalised): the result is invalid if > 0.
 *   4. tt_nce_backward : df [m, d] (complete), dc [n, d] (this shard's
 *      contribution).  ws must hold the forward's E.
 * ws: tt_nce_workspace_bytes(m, n, d) bytes (E alone is 4 m n bytes).     */
int64_t tt_nce_workspace_bytes(int64_t m, int64_t n, int32_t d);
int32_t tt_nce_norms(const float* f, const float* c, int64_t m, int64_t n, int32_t d,
                     float* norm2, tt_stream_t stream);
int32_t tt_nce_forward(const float* f, const float* c, int64_t m, int64_t n, int32_t d,
                       int64_t row0, float temperature, const float* norm2, void* ws,
                       int64_t ws_bytes, float* col_sum, tt_stream_t stream);
int32_t tt_nce_loss(int64_t m, int64_t n, int32_t d, int64_t row0, int64_t batch,
                    float temperature, void* ws, int64_t ws_bytes, const float* col_sum,
                    float* loss, int32_t* status, tt_stream_t stream);
int32_t tt_nce_backward(const float* f, const float* c, int64_t m, int64_t n, int32_t d,
                        int64_t row0, int64_t batch, float temperature, void* ws,
                        int64_t ws_bytes, float* df, float* dc, tt_stream_t stream);

/* Robust InfoNCE -- the same loss and gradients when tt_nce_loss reports
 * underflow (temperature far below 0.03 on L2-normalised rows, or
 * unnormalised projections: contrastive.py:102-138 computes those too).
 * Exact per-row / per-column maxima replace the shared shift, so every sum
 * holds its exp(0) term and cannot underflow; two exponentials per element.
 *   5. tt_nce_maxes      : row maxima of S (ws) and col_max[n] over these m
 *      rows (all-reduce MAX across row shards);
 *   6. tt_nce_forward_lse: with the global col_max: row sums of
 *      exp(s - rowmax), col_sum[n] of exp(s - colmax) over these rows
 *      (all-reduce SUM), S kept in ws for the backward;
 *   7. tt_nce_loss_lse   : loss += this shard's share; *status counts
 *      non-finite log-sum-exps (inf / nan inputs);
 *   8. tt_nce_backward_lse: df, dc as tt_nce_backward.
 * Same workspace as the default path (tt_nce_workspace_bytes).            */
int32_t tt_nce_maxes(const float* f, const float* c, int64_t m, int64_t n, int32_t d, int64_t row0,
                     float temperature, void* ws, int64_t ws_bytes, float* col_max, tt_stream_t stream);
int32_t tt_nce_forward_lse(const float* f, const float* c, int64_t m, int64_t n, int32_t d,
                           int64_t row0, float temperature, const float* col_max, void* ws,
                           int64_t ws_bytes, float* col_sum, tt_stream_t stream);
int32_t tt_nce_loss_lse(int64_t m, int64_t n, int32_t d, int64_t row0, int64_t batch, void* ws,
                        int64_t ws_bytes, const float* col_max, const float* col_sum, float* loss,
                        int32_t* status, tt_stream_t stream);
int32_t tt_nce_backward_lse(const float* f, const float* c, int64_t m, int64_t n, int32_t d,
                            int64_t row0, int64_t batch, float temperature, void* ws,
                            int64_t ws_bytes, float* df, float* dc, tt_stream_t stream);

/* compute_retrieval_metrics (contrastive.py:275-332): for firm rows F [m, d]
 * (global rows row0..) against all n ceo rows C, ranks[i] = 1 + #{j != row0+i :
 * f_i.c_j > f_i.c_{row0+i}} -- the rank of the true match under a descending
 * sort (identical to torch.sort's whenever the row has no exact ties).
 * ws: tt_rank_workspace_bytes(m) bytes.                                     */
int64_t tt_rank_workspace_bytes(int64_t m);
int32_t tt_retrieval_ranks(const float* f, const float* c, int64_t m, int64_t n, int32_t d,
                           int64_t row0, void* ws, int64_t ws_bytes, int32_t* ranks,
                           tt_stream_t stream);

/* semi_hard_negative_mining (contrastive.py:141-192): dist = 1 - F C^T
 * (fp32), pos_i = dist[i][row0+i]; per firm row i the hardest semi-hard
 * negative (smallest dist with pos < dist < pos + margin over j != row0+i),
 * else the hardest negative overall; row_loss[i] = relu(pos - hardest +
 * margin), hardest[i] = its column (ties: lowest column),
 * *loss += sum_i row_loss[i] / batch (caller zeroes it).  One fused
 * similarity GEMM + masked-min epilogue replaces the reference's per-row
 * Python loop.  Backward (autograd of the same expression): with
 * g = *grad_loss, for each row with row_loss > 0:
 *   df_i = (g/B)(c_j - c_{row0+i}),  dc_{row0+i} -= (g/B) f_i,  dc_j += (g/B) f_i;
 * df [m, d] and dc [n, d] are overwritten.  ws: tt_triplet_workspace_bytes. */
int64_t tt_triplet_workspace_bytes(int64_t m, int64_t n, int32_t d);
int32_t tt_triplet_forward(const float* f, const float* c, int64_t m, int64_t n, int32_t d,
                           int64_t row0, float margin, int64_t batch, void* ws, int64_t ws_bytes,
                           int32_t* hardest, float* row_loss, float* loss, tt_stream_t stream);
int32_t tt_triplet_backward(const float* f, const float* c, int64_t m, int64_t n, int32_t d,
                            int64_t row0, int64_t batch, const int32_t* hardest,
                            const float* row_loss, const float* grad_loss, float* df, float* dc,
                            tt_stream_t stream);

/* ---- data-parallel gradient exchange over peer memory (xGMI) ------------
 * Replaces the DistributedDataParallel gradient all-reduce + optim.Adam.step
 * of a data-parallel training step (training.py:54-55 under DDP)
 * with ONE launch: every rank publishes its flat gradient into its exchange
 * region (uncached device memory shared through IPC handles), signals every
 * peer, waits (bounded) for theirs, sums all ranks' gradients in rank order
 * (every rank computes bitwise the same mean) and applies Adam.  Setup entry
 * points allocate / map memory (unlike the compute entries); the caller
 * exchanges the TT_AR_HANDLE_BYTES handles between ranks (e.g. an all-gather)
 * and passes every rank's mapped region in tt_ar_peers.  A wait that exceeds
 * its bound (wait_us; <= 0: 2 s) increments *err instead of hanging: that
 * block's slice of params / exp_avg / exp_avg_sq / grad_out is left
 * untouched, and every later call with *err != 0 returns on the device
 * without publishing or updating anything (the peers then time out too).
 * The caller checks *err and fails the step; *err is cleared only by
 * re-creating the exchange (tt_ar_reset on every rank).                   */
#define TT_AR_MAX_RANKS 16
#define TT_AR_HANDLE_BYTES 64
/* exchange protocols (tt_ar_peers.protocol; zero-initialised = pull):
 * TT_AR_PULL: each rank stores its slice into its OWN region, raises a flag
 *   in every peer's region, waits for the peers' flags and reads their slices
 *   remotely.
 * TT_AR_PUSH: each rank stores every element as one 8-byte word (value |
 *   epoch) straight into every PEER's region and polls its own region until
 *   all peers' words carry this step's epoch: no flags, no remote reads.
 * Both sum in rank order: bitwise the same mean.  (ABI 6)                   */
#define TT_AR_PULL 0
#define TT_AR_PUSH 1
#define TT_AR_PUSH_MAX_RANKS 8  /* push: world <= 8 (one node), else TT_ERR_UNSUPPORTED */
typedef struct tt_ar_peers {
  void* region[TT_AR_MAX_RANKS];   /* every rank's region, mapped in this process */
  int32_t protocol;                /* TT_AR_PULL or TT_AR_PUSH; the same on every rank */
  int32_t reserved;
} tt_ar_peers;
int64_t tt_ar_region_bytes(int64_t n);
int32_t tt_ar_alloc(int64_t bytes, void** region, void* ipc_handle);
int32_t tt_ar_open(const void* ipc_handle, void** region);
int32_t tt_ar_close(void* region);
int32_t tt_ar_free(void* region);
/* zero the region's flags and slots (all ranks, then a host barrier) */
int32_t tt_ar_reset(void* region, int64_t n, tt_stream_t stream);
/* grad_out (nullable, may alias grad) = mean over ranks; params/exp_avg/
 * exp_avg_sq (nullable params: no Adam) updated with hp at step t =
 * state->step_cur (state non-NULL) or step_host, which is also the epoch the
 * flags carry (strictly increasing per region).                             */
int32_t tt_ar_allreduce_adam(const tt_ar_peers* peers, int32_t rank, int32_t world, int64_t n,
                             const float* grad, float* grad_out, float* params, float* exp_avg,
                             float* exp_avg_sq, const tt_adam_hp* hp, tt_state* state,
                             int64_t step_host, int32_t* err, int64_t wait_us, tt_stream_t stream);

/* One data-parallel training step with the exchange inside the gradient
 * reduction (training.py:44-57 under DDP): tt_train_step's
 * kernels, whose last one (k_reduce_adam) publishes each block's reduced
 * gradient slice into this rank's region, signals the peers, waits (bounded)
 * for theirs, takes the mean in rank order and applies Adam -- the launch and
 * the boundary of tt_ar_allreduce_adam disappear.  Same peers / err / wait_us
 * semantics as tt_ar_allreduce_adam (epoch = the device step counter), grad =
 * the mean gradient.  co_ranks = ranks of this job sharing this device (1 for
 * one process per GPU).  Returns TT_ERR_UNSUPPORTED with nothing launched
 * when the reduction's blocks (co_ranks grids of them) cannot all be resident
 * at once: the caller keeps tt_train_step(apply_adam=0) + tt_ar_allreduce_adam. */
int32_t tt_train_step_dp(const tt_model_desc* d, float* params, float* buffers, int64_t* nbt,
                         const tt_batch* b, const tt_adam_hp* hp, uint64_t seed, tt_state* state,
                         void* ws, int64_t ws_bytes, float* grad, float* exp_avg, float* exp_avg_sq,
                         const tt_ar_peers* peers, int32_t rank, int32_t world, int32_t co_ranks,
                         int32_t* err, int64_t wait_us, tt_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* CEO_TT_H */
