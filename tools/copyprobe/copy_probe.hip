// HBM stream-copy variants (probe for tt_stream_copy): U float4 per thread,
// contiguous per block or grid-stride, plain or nontemporal.
#include <hip/hip_runtime.h>
#include <cstdint>
typedef float v4f __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy_blk(const v4f* __restrict__ s, v4f* __restrict__ d, int64_t n4) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  v4f v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n4) v[u] = NT ? __builtin_nontemporal_load(s + i) : s[i];
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n4) {
      if (NT) __builtin_nontemporal_store(v[u], d + i); else d[i] = v[u];
    }
  }
}

// read-only stream (the cosine kernel's traffic is 99 % reads): each block
// sums its U float4 per thread and writes one float
template <int U>
__global__ __launch_bounds__(256) void k_read_blk(const v4f* __restrict__ s, float* __restrict__ d, int64_t n4) {
  const int64_t base = (int64_t)blockIdx.x * 256 * U + threadIdx.x;
  v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = base + u * 256;
    if (i < n4) acc += __builtin_nontemporal_load(s + i);
  }
  float x = acc.x + acc.y + acc.z + acc.w;
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o);
  if ((threadIdx.x & 63) == 0) d[blockIdx.x * 4 + (threadIdx.x >> 6)] = x;
}

template <int U>
static int run_read(const void* s, void* d, int64_t n4, hipStream_t st) {
  const int64_t g = (n4 + 256 * U - 1) / (256 * U);
  hipLaunchKernelGGL((k_read_blk<U>), dim3((unsigned)g), dim3(256), 0, st, (const v4f*)s, (float*)d, n4);
  return (int)hipGetLastError();
}

template <int U, bool NT>
static int run(const void* s, void* d, int64_t n4, hipStream_t st) {
  const int64_t g = (n4 + 256 * U - 1) / (256 * U);
  hipLaunchKernelGGL((k_copy_blk<U, NT>), dim3((unsigned)g), dim3(256), 0, st, (const v4f*)s, (v4f*)d, n4);
  return (int)hipGetLastError();
}

extern "C" int copy_probe(const void* s, void* d, int64_t bytes, int variant, void* stream) {
  const int64_t n4 = bytes / 16;
  hipStream_t st = (hipStream_t)stream;
  switch (variant) {
    case 0: return run<1, false>(s, d, n4, st);
    case 1: return run<2, false>(s, d, n4, st);
    case 2: return run<4, false>(s, d, n4, st);
    case 3: return run<8, false>(s, d, n4, st);
    case 4: return run<1, true>(s, d, n4, st);
    case 5: return run<2, true>(s, d, n4, st);
    case 6: return run<4, true>(s, d, n4, st);
    case 7: return run<8, true>(s, d, n4, st);
    case 8: return run_read<4>(s, d, n4, st);
    case 9: return run_read<8>(s, d, n4, st);
    default: return -1;
  }
}
