// randread.hip — random 64-byte-line read throughput vs table size and
// cache policy on MI355X (guides the node-table / solid-table designs).
//   hipcc --offload-arch=gfx950 -O3 -o randread randread.hip && ./randread
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}

template <int MODE>
__global__ void k_rand(const uint64_t* __restrict__ t, uint64_t nlines, uint64_t n, unsigned long long* out) {
  uint64_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t line = __umul64hi(mix(i), nlines);
    const uint64_t* p = t + line * 8;
    if (MODE == 0) {
      acc += p[0] + p[1] + p[2];
    } else {
      acc += __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
             __hip_atomic_load(p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) +
             __hip_atomic_load(p + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if (acc == 42) atomicAdd(out, 1ull);
}

int main() {
  const uint64_t maxb = 16ull << 30;
  uint64_t* t;
  unsigned long long* out;
  if (hipMalloc(&t, maxb) != hipSuccess) return 1;
  hipMalloc(&out, 8);
  hipMemset(t, 1, maxb);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  int ncu = 256;
  const uint64_t n = 1ull << 28;  // 268M random line reads
  for (uint64_t mb : {64ull, 256ull, 1024ull, 4096ull, 8192ull, 16384ull}) {
    const uint64_t nlines = (mb << 20) / 64;
    for (int mode = 0; mode < 2; ++mode)
      for (int occ : {16, 32}) {
        const int grid = ncu * occ;
        for (int rep = 0; rep < 2; ++rep) {
          hipEventRecord(a);
          if (mode == 0)
            k_rand<0><<<grid, 256>>>(t, nlines, n, out);
          else
            k_rand<1><<<grid, 256>>>(t, nlines, n, out);
          hipEventRecord(b);
          hipEventSynchronize(b);
          float ms;
          hipEventElapsedTime(&ms, a, b);
          if (rep == 1)
            printf("table %6llu MB  %s  blocks/CU %2d  %7.2f ms  %6.2f G lines/s\n", (unsigned long long)mb,
                   mode ? "agent-coherent" : "plain         ", occ, ms, n / (ms * 1e-3) / 1e9);
        }
      }
  }
  hipFree(t);
  return 0;
}
