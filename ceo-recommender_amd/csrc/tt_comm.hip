// Data-parallel gradient exchange over peer memory (xGMI), gfx950.
//
// The only exchange of the data-parallel step is the mean over
// ranks of the 85 KB flat gradient, followed by Adam (training.py:55).  At
// this size an all-reduce is pure latency; this is a one-shot exchange in ONE
// launch that also applies Adam:
//
//   every rank owns an exchange region (uncached device memory, shared with the
//   other ranks through IPC handles): two gradient slots (step parity) and a
//   flag word per (source rank, block).  Block b of rank r
//     1. copies slice b of its gradient into its own slot[t & 1],
//     2. waits for those stores, then writes epoch t into flag[r][b] of every
//        rank (remote stores over xGMI),
//     3. waits (bounded) until flag[p][b] == t for every rank p,
//     4. reads slice b of every rank's slot[t & 1] -- in rank order, so every
//        rank computes bitwise the same mean -- scales by 1/world and applies
//        Adam (the k_adam arithmetic) to its parameters.
//   Slot reuse is safe: rank r rewrites slot[t & 1] at step t + 2, after its
//   step-(t+1) exchange saw every peer's step-(t+1) flags, which each peer
//   wrote after finishing its step-t reads (stream order).
//   The epoch is the device step counter (tt_state.step_cur), so the launch
//   replays unchanged inside a captured hipGraph.
//   A wait that exceeds its bound sets *err and gives up (no hang).  The
//   failure is never papered over with local data: a block that timed out
//   leaves its slice of p / m / v / grad_out untouched, and every later launch
//   on this rank sees *err != 0 at entry and does nothing at all -- it neither
//   applies Adam nor publishes, so the peers time out in turn and stop
//   updating too, and no slot is rewritten while a slow peer may still read
//   it.  The host checks err (FusedTrainer.check_exchange) and raises.
#include "tt_common.h"

namespace tt {

constexpr int AR_THREADS = 256;

struct ArArgs {
  float* slot[TT_AR_MAX_RANKS];          // slot 0 of each rank's region (slot 1 at + slot_stride)
  uint64_t* flags[TT_AR_MAX_RANKS];      // each rank's flag array [TT_AR_MAX_RANKS][blocks]
  uint64_t* ll[TT_AR_MAX_RANKS];         // each rank's push words [2][TT_AR_MAX_RANKS][slot_stride] (TT_AR_PUSH)
  int64_t slot_stride;                   // floats between slot 0 and slot 1
  int rank, world, blocks;
  int64_t n;                             // gradient floats
  const float* grad;                     // this rank's gradient (k_reduce_adam output)
  float* grad_out;                       // mean gradient (nullable)
  float *p, *m, *v;                      // Adam (nullable p: no Adam)
  double lr, b1, b2, eps;
  tt_state* state;
  int64_t step_host;
  int32_t* err;                          // set when a wait times out
  uint64_t wait_ticks;                   // wait bound in s_memrealtime ticks (100 MHz)
};

__device__ __forceinline__ uint64_t ld_flag(const uint64_t* f) {
  return __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Step 4 for slice [lo, hi): per lane AR_EPT elements at a time, the W peer
// slot loads of all of them (and their Adam state) issued before the first
// wait; the own term comes from this rank's gradient (the bits its slot holds),
// the adds run in rank order (rank_order_sums).  W >= world.
constexpr int AR_EPT = 4;  // cfg 3: 21,313 floats / 32 blocks / 256 lanes = 2.6 per lane: one round
template <int W>
__device__ __forceinline__ void ar_mean_adam(const ArArgs& a, int64_t lo, int64_t hi, int64_t par,
                                             const AdamCoef& c) {
  const float inv_w = 1.0f / (float)a.world;
  for (int64_t e0 = lo + threadIdx.x; e0 < hi; e0 += AR_EPT * AR_THREADS) {
    int64_t off[AR_EPT], ec[AR_EPT];
    float own[AR_EPT], s[AR_EPT], p[AR_EPT], m[AR_EPT], v[AR_EPT];
#pragma unroll
    for (int j = 0; j < AR_EPT; ++j) {  // clamped: no branch around a load
      ec[j] = min(e0 + (int64_t)j * AR_THREADS, hi - 1);
      off[j] = par + ec[j];
      own[j] = a.grad[ec[j]];
    }
    if (a.p) {
#pragma unroll
      for (int j = 0; j < AR_EPT; ++j) {
        p[j] = a.p[ec[j]];
        m[j] = a.m[ec[j]];
        v[j] = a.v[ec[j]];
      }
    }
    rank_order_sums<W, AR_EPT>(a.slot, a.world, a.rank, off, own, s);
#pragma unroll
    for (int j = 0; j < AR_EPT; ++j) {
      const int64_t e = e0 + (int64_t)j * AR_THREADS;
      if (e >= hi) break;
      const float g = s[j] * inv_w;
      if (a.grad_out) a.grad_out[e] = g;
      if (a.p) {
        adam_elem(p[j], m[j], v[j], g, c);
        a.p[e] = p[j];
        a.m[e] = m[j];
        a.v[e] = v[j];
      }
    }
  }
}

__global__ __launch_bounds__(AR_THREADS) void k_ar_adam(ArArgs a) {
  // sticky failure: an earlier exchange on this rank timed out (one read per
  // block, so the whole block takes the same branch)
  __shared__ int ok_s;
  if (threadIdx.x == 0) ok_s = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
  __syncthreads();
  if (ok_s == 0) return;
  const int64_t t = a.state ? load_step(a.state, reinterpret_cast<const int64_t*>(a.grad)) : a.step_host;
  const uint64_t epoch = (uint64_t)t;
  const int b = blockIdx.x;
  const int64_t per = (a.n + a.blocks - 1) / a.blocks;
  const int64_t lo = b * per, hi = min(a.n, lo + per);
  const int64_t par = (t & 1) ? a.slot_stride : 0;
  float* mine = a.slot[a.rank] + par;
  // 1. publish this block's slice (system-coherent stores), every thread's
  // stores performed before the barrier that precedes the flags
  for (int64_t e = lo + threadIdx.x; e < hi; e += AR_THREADS)
    __hip_atomic_store(mine + e, a.grad[e], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  // explicit wait after the release: ROCm 7.2 may drop the s_waitcnt that
  // follows the fence's write-back when it believes the counter is already
  // empty (MI355X_MICROARCH.md, compiler hazard) -- the asm is opaque to that
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  // 2. signal every rank (one lane per destination), behind every wave's wait
  if (threadIdx.x < a.world) {
    uint64_t* f = a.flags[threadIdx.x] + (int64_t)a.rank * a.blocks + b;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(f, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // Adam's bias corrections (double pow, a long dependent chain) while the
  // peers' flags are in flight, not after the wait
  AdamCoef c{};
  if (a.p) c = adam_coef(a.lr, a.b1, a.b2, a.eps, t);
  // 3. wait for every rank's slice b (bounded)
  if (threadIdx.x < a.world) {
    const uint64_t* f = a.flags[a.rank] + (int64_t)threadIdx.x * a.blocks + b;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz, chip-wide
    while (ld_flag(f) < epoch) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > a.wait_ticks) {
        ok_s = 0;
        atomicAdd(a.err, 1);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (ok_s == 0) return;  // this slice keeps its parameters (err reports it)
  // 4. mean over ranks in rank order + Adam
  if (a.world <= 2)
    ar_mean_adam<2>(a, lo, hi, par, c);
  else if (a.world <= 4)
    ar_mean_adam<4>(a, lo, hi, par, c);
  else if (a.world <= 8)
    ar_mean_adam<8>(a, lo, hi, par, c);
  else
    ar_mean_adam<TT_AR_MAX_RANKS>(a, lo, hi, par, c);
  if (a.p && a.state && b == 0 && threadIdx.x == 0) a.state->step_done = t;
}

// TT_AR_PUSH form of k_ar_adam (tt_common.h, ll_publish / ll_gather_sums),
// the same AR_BLOCKS grid as the pull form (every block of a rank must be
// resident while it waits for its peers: a grid sized by n could exceed what
// the GPU holds at once and wait on itself).  Block b owns [lo, hi): every
// lane stores its elements' words into every peer's region, then polls its
// own region until all peers' words carry this step's epoch, and only then --
// after a barrier that makes the outcome block-uniform -- applies the mean
// and Adam: a block that timed out leaves its whole slice untouched, as the
// pull form does.  A slice of one round (<= AR_EPT x AR_THREADS elements,
// cfg 3) keeps the sums of the poll; a longer one polls every round first and
// re-reads the (then settled) words for the sums.  No flags, no remote reads.
template <int W>
__device__ __forceinline__ void ar_push_block(const ArArgs& a, int64_t lo, int64_t hi, int64_t t, int* ok_s) {
  const int64_t par = t & 1;
  const uint32_t ep = (uint32_t)t;
  constexpr int64_t RND = (int64_t)AR_EPT * AR_THREADS;
  auto lanes = [&](int64_t e0, int64_t (&ec)[AR_EPT], bool (&live)[AR_EPT], float (&own)[AR_EPT]) {
#pragma unroll
    for (int j = 0; j < AR_EPT; ++j) {  // clamped: no branch around a load
      const int64_t e = e0 + threadIdx.x + (int64_t)j * AR_THREADS;
      live[j] = e < hi;
      ec[j] = min(e, hi - 1);
      own[j] = a.grad[ec[j]];
    }
  };
  int64_t ec[AR_EPT];
  bool live[AR_EPT];
  float own[AR_EPT], s[AR_EPT];
  for (int64_t e0 = lo; e0 < hi; e0 += RND) {  // publish the whole slice
    lanes(e0, ec, live, own);
#pragma unroll
    for (int j = 0; j < AR_EPT; ++j)
      if (live[j]) ll_publish(a.ll, a.world, a.rank, a.slot_stride, par, ec[j], own[j], ep);
  }
  AdamCoef c{};
  if (a.p) c = adam_coef(a.lr, a.b1, a.b2, a.eps, t);
  const bool one = hi - lo <= RND;  // (block-uniform)
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  bool fine = true;
  for (int64_t e0 = lo; e0 < hi && fine; e0 += RND) {  // wait for every peer word of the slice
    lanes(e0, ec, live, own);
    fine = ll_gather_sums<W, AR_EPT>(a.ll[a.rank], a.world, a.rank, a.slot_stride, par, ec, live, own, ep, t0,
                                     a.wait_ticks, s);
  }
  if (!fine) *ok_s = 0;
  __syncthreads();
  if (*ok_s == 0) {
    if (threadIdx.x == 0) atomicAdd(a.err, 1);
    return;
  }
  const float inv_w = 1.0f / (float)a.world;
  for (int64_t e0 = lo; e0 < hi; e0 += RND) {
    if (!one) {  // the words are settled: the sums of this round
      lanes(e0, ec, live, own);
      (void)ll_gather_sums<W, AR_EPT>(a.ll[a.rank], a.world, a.rank, a.slot_stride, par, ec, live, own, ep, t0,
                                      ~0ull, s);
    }
    float p[AR_EPT], m[AR_EPT], v[AR_EPT];
    if (a.p) {
#pragma unroll
      for (int j = 0; j < AR_EPT; ++j) {
        p[j] = a.p[ec[j]];
        m[j] = a.m[ec[j]];
        v[j] = a.v[ec[j]];
      }
    }
#pragma unroll
    for (int j = 0; j < AR_EPT; ++j) {
      if (!live[j]) continue;
      const float g = s[j] * inv_w;
      if (a.grad_out) a.grad_out[ec[j]] = g;
      if (a.p) {
        adam_elem(p[j], m[j], v[j], g, c);
        a.p[ec[j]] = p[j];
        a.m[ec[j]] = m[j];
        a.v[ec[j]] = v[j];
      }
    }
  }
}

__global__ __launch_bounds__(AR_THREADS) void k_ar_adam_push(ArArgs a) {
  __shared__ int ok_s;
  if (threadIdx.x == 0) ok_s = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
  __syncthreads();
  if (ok_s == 0) return;
  const int64_t t = a.state ? load_step(a.state, reinterpret_cast<const int64_t*>(a.grad)) : a.step_host;
  const int64_t per = (a.n + a.blocks - 1) / a.blocks;
  const int64_t lo = (int64_t)blockIdx.x * per, hi = min(a.n, lo + per);
  if (lo >= hi) return;  // (block-uniform)
  if (a.world <= 2)
    ar_push_block<2>(a, lo, hi, t, &ok_s);
  else if (a.world <= 4)
    ar_push_block<4>(a, lo, hi, t, &ok_s);
  else
    ar_push_block<8>(a, lo, hi, t, &ok_s);  // (the host allows the push protocol up to TT_AR_PUSH_MAX_RANKS = 8)
  if (ok_s && a.p && a.state && blockIdx.x == 0 && threadIdx.x == 0) a.state->step_done = t;
}

}  // namespace tt
