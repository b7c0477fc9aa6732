// Grid-barrier microbenchmark (review r05 item 7: is a persistent cfg-2 step
// worth building?).  K back-to-back grid barriers in one launch of NB
// workgroups (256 threads, one per CU up to 256), two forms:
//   flat: one arrival counter for the whole grid, the last arriver bumps the
//         generation word, everyone polls it;
//   xcd:  hierarchical, blocks grouped by blockIdx % 8 (the dispatcher's XCD
//         round robin -- placement matters for speed only, the protocol is
//         correct for any placement): per-group counters, each group's last
//         arriver bumps the top counter, the last group bumps the generation.
// Release fence (agent) before arriving, acquire fence after the wait, as a
// persistent kernel needs to hand data across the barrier.  `pub` floats per
// block are stored (plain stores) before each arrival: the release then has
// dirty lines to write back, as after a phase that produced a partial.
// Every spin is bounded (s_memrealtime, 100 MHz): a stranded block sets err
// and leaves, so the grid always drains.  Counters are monotonic (epoch e
// expects e * n arrivals): no reset between barriers.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

struct Bar {
  unsigned grp[8][32];  // one 128-B line per group counter
  unsigned top[32];
  unsigned gen[32];
  int err[32];
};

__device__ __forceinline__ unsigned ld_relaxed(const unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned add_relaxed(unsigned* p) {
  return __hip_atomic_fetch_add(p, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool XCD>
__global__ __launch_bounds__(256) void k_bar(Bar* b, float* pub, int pub_per_thread, int iters, uint64_t bound) {
  const int nb = (int)gridDim.x;
  const int ngrp = nb < 8 ? nb : 8;
  const int g = (int)blockIdx.x % ngrp;
  const unsigned in_g = (unsigned)((nb - g + ngrp - 1) / ngrp);
  __shared__ int ok;
  if (threadIdx.x == 0) ok = 1;
  __syncthreads();
  float* mine = pub + (int64_t)blockIdx.x * 256 * pub_per_thread;
  for (int e = 1; e <= iters; ++e) {
    for (int i = 0; i < pub_per_thread; ++i) mine[i * 256 + threadIdx.x] = (float)e;
    __syncthreads();
    if (threadIdx.x == 0 && ok) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      if (XCD) {
        if (add_relaxed(&b->grp[g][0]) == (unsigned)e * in_g - 1u)
          if (add_relaxed(&b->top[0]) == (unsigned)e * (unsigned)ngrp - 1u)
            __hip_atomic_store(&b->gen[0], (unsigned)e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        if (add_relaxed(&b->top[0]) == (unsigned)e * (unsigned)nb - 1u)
          __hip_atomic_store(&b->gen[0], (unsigned)e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (ld_relaxed(&b->gen[0]) < (unsigned)e) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > bound) {
          atomicAdd(&b->err[0], 1);
          ok = 0;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
    if (!ok) return;
  }
}

}  // namespace

extern "C" int grid_barrier_probe(void* bar, float* pub, int pub_per_thread, int nb, int iters, int xcd,
                                  uint64_t bound_ticks, hipStream_t s) {
  if (xcd)
    hipLaunchKernelGGL(k_bar<true>, dim3(nb), dim3(256), 0, s, (Bar*)bar, pub, pub_per_thread, iters, bound_ticks);
  else
    hipLaunchKernelGGL(k_bar<false>, dim3(nb), dim3(256), 0, s, (Bar*)bar, pub, pub_per_thread, iters, bound_ticks);
  return (int)hipGetLastError();
}
extern "C" int grid_barrier_bytes() { return (int)sizeof(Bar); }
