// Host-side checks of libceo_tt's C-ABI under AddressSanitizer (SURVEY 5:
// sanitizer variant for the host code).  Built by `make -C
// ceo-recommender_amd/csrc asan` with the whole C-ABI translation unit
// (tt_abi.hip) instrumented on the host side only (-Xarch_host
// -fsanitize=address); run on a CPU: every call below is decided on the host
// (layout, plan, workspace sizes, argument errors) before anything would be
// enqueued, so no GPU is needed.  Prints "abi_host_check: ALL OK" on success.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/ceo_tt.h"

static int failures = 0;
#define CHECK(cond)                                                      \
  do {                                                                   \
    if (!(cond)) {                                                       \
      std::fprintf(stderr, "FAILED %s:%d  %s\n", __FILE__, __LINE__, #cond); \
      ++failures;                                                        \
    }                                                                    \
  } while (0)

static tt_model_desc desc(int nf, int nc, std::vector<int> fc, std::vector<int> cc, int latent) {
  tt_model_desc d;
  std::memset(&d, 0, sizeof(d));
  d.n_num[0] = nf;
  d.n_num[1] = nc;
  d.n_cat[0] = (int)fc.size();
  d.n_cat[1] = (int)cc.size();
  d.emb_dim[0] = 48;
  d.emb_dim[1] = 8;
  d.latent = latent;
  for (size_t j = 0; j < fc.size(); ++j) d.cat_counts[0][j] = fc[j];
  for (size_t j = 0; j < cc.size(); ++j) d.cat_counts[1][j] = cc[j];
  d.dropout_p = 0.1f;
  d.bn_eps = 1e-5f;
  d.bn_momentum = 0.1f;
  return d;
}

int main() {
  CHECK(tt_abi_version() == TT_ABI_VERSION);
  const tt_model_desc geoms[] = {
      desc(12, 2, {4, 4, 2, 2}, {2, 4, 2, 2, 2, 2, 2}, 60),  // the reference test metadata
      desc(32, 32, {}, {}, 64),                              // cfg 2
      desc(64, 64, {}, {}, 128),                             // cfg 3
      desc(1, 5, {3}, {}, 8),
      desc(200, 3, {}, {9, 9, 9}, 128),
  };
  for (const tt_model_desc& d : geoms) {
    const int64_t n = tt_param_count(&d);
    CHECK(n > 0);
    int64_t offs[TT_NUM_OFFSETS];
    CHECK(tt_param_offsets(&d, offs) == TT_OK);
    for (int i = 0; i < TT_NUM_OFFSETS; ++i) CHECK(offs[i] == -1 || (offs[i] >= 0 && offs[i] < n && offs[i] % 4 == 0));
    CHECK(tt_buffer_count(&d) == 2 * (2 * 64 + 2 * 32));
    int64_t prev = 0;
    for (int64_t b : {1, 2, 63, 64, 65, 4096, 8192, 16384, 20000}) {
      const int64_t ws = tt_workspace_bytes(&d, b);
      CHECK(ws > 0 && ws >= prev);
      prev = ws;
      int32_t info[6] = {-7, -7, -7, -7, -7, -7};
      CHECK(tt_step_plan(&d, b, info, 6) == TT_OK);
      CHECK(info[3] == 5 || info[3] == 6);
      CHECK(info[5] == 4 || info[5] == 8);
    }
    // argument errors: decided before any HIP call
    std::vector<float> dummy(16);
    tt_batch bt;
    std::memset(&bt, 0, sizeof(bt));
    bt.n_rows = 1;
    float* p = dummy.data();
    int64_t nbt[4] = {0, 0, 0, 0};
    // train-mode B = 1: BatchNorm's ValueError
    if (d.n_num[0] > 0) bt.num[0] = p, bt.num_ld[0] = d.n_num[0];
    if (d.n_num[1] > 0) bt.num[1] = p, bt.num_ld[1] = d.n_num[1];
    int64_t cat[64] = {0};
    if (d.n_cat[0]) bt.cat[0] = cat, bt.cat_ld[0] = d.n_cat[0];
    if (d.n_cat[1]) bt.cat[1] = cat, bt.cat_ld[1] = d.n_cat[1];
    CHECK(tt_forward(&d, p, p, nbt, &bt, 1, 0, 1, p, 1 << 30, p, nullptr) == TT_ERR_BATCH_TOO_SMALL);
    // short workspace
    bt.n_rows = 64;
    CHECK(tt_forward(&d, p, p, nbt, &bt, 1, 0, 1, p, 16, p, nullptr) == TT_ERR_WORKSPACE);
    // null pointers / missing inputs
    CHECK(tt_forward(&d, nullptr, p, nbt, &bt, 1, 0, 1, p, 1 << 30, p, nullptr) == TT_ERR_ARG);
    CHECK(tt_forward(&d, p, p, nbt, nullptr, 1, 0, 1, p, 1 << 30, p, nullptr) == TT_ERR_ARG);
    CHECK(tt_backward_ex(&d, p, nullptr, &bt, p, 0, 0, 1, p, 1 << 30, p, nullptr, nullptr, nullptr) == TT_ERR_ARG);
    tt_adam_hp hp = {4e-4, 0.9, 0.999, 1e-8};
    CHECK(tt_train_step(&d, p, p, nbt, &bt, &hp, 0, nullptr, p, 1 << 30, p, p, p, 1, nullptr) == TT_ERR_ARG);
    CHECK(tt_adam_apply(p, p, p, p, -1, &hp, nullptr, 1, nullptr) == TT_ERR_ARG);
    tt_batch nob = bt;
    nob.num[0] = nullptr;
    if (d.n_num[0] > 0) CHECK(tt_forward(&d, p, p, nbt, &nob, 0, 0, 1, p, 1 << 30, p, nullptr) == TT_ERR_ARG);
  }
  // the deferred late half's host planning (make_red for the late part of the
  // reduction, tt_train_flush / TT_FLAG_LATE_PENDING) on the cfg-3 geometry:
  // everything up to the launch is host code (without a GPU the launches
  // themselves fail, which is all right here); ASan checks the segment lists
  {
    tt_model_desc d = desc(64, 64, {}, {}, 128);
    std::vector<float> big(64 * 16384);
    float* p = big.data();
    tt_batch bt;
    std::memset(&bt, 0, sizeof(bt));
    bt.n_rows = 16384;
    bt.num[0] = bt.num[1] = p;
    bt.num_ld[0] = bt.num_ld[1] = 64;
    int64_t nbt[4] = {0, 0, 0, 0};
    tt_adam_hp hp = {4e-4, 0.9, 0.999, 1e-8};
    const int64_t ws = tt_workspace_bytes(&d, 16384);
    (void)tt_train_flush(&d, p, p, nbt, &bt, &hp, reinterpret_cast<tt_state*>(p), p, ws, p, p, p, nullptr);
    d.flags |= TT_FLAG_DEFER_LATE | TT_FLAG_LATE_PENDING;
    (void)tt_train_step(&d, p, p, nbt, &bt, &hp, 0, reinterpret_cast<tt_state*>(p), p, ws, p, p, p, 1, nullptr);
  }
  // unsupported shapes
  tt_model_desc big = desc(64, 64, {}, {}, 1024);
  int32_t info[6];
  CHECK(tt_step_plan(&big, 16384, info, 6) == TT_ERR_UNSUPPORTED);
  tt_model_desc bad = desc(-1, 4, {}, {}, 8);
  CHECK(tt_param_count(&bad) == TT_ERR_ARG);
  CHECK(tt_param_count(nullptr) == TT_ERR_ARG);
  // contrastive / exchange sizes
  CHECK(tt_nce_workspace_bytes(100000, 100000, 256) > (int64_t)4 * 100000 * 100000);
  CHECK(tt_nce_workspace_bytes(0, 10, 256) == TT_ERR_ARG);
  CHECK(tt_rank_workspace_bytes(5000) > 0);
  CHECK(tt_triplet_workspace_bytes(128, 256, 32) > 0);
  CHECK(tt_ar_region_bytes(21313) > 21313 * 4);
  CHECK(tt_ar_region_bytes(0) == TT_ERR_ARG);
  if (failures) {
    std::fprintf(stderr, "abi_host_check: %d FAILED\n", failures);
    return 1;
  }
  std::printf("abi_host_check: ALL OK\n");
  return 0;
}
