// Round trip of a small count read back by the host between two kernels
// (the unipath / count stages do ~100 per step): tiny kernel -> 8-byte
// D2H -> stream sync -> next launch.  Variants: pageable destination,
// pinned destination, and the kernel writing the count straight into pinned
// host memory (no copy).  Prints microseconds per round trip.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

__global__ void k_inc(unsigned long long* c, unsigned long long* host_out) {
  if (threadIdx.x == 0) {
    const unsigned long long v = atomicAdd(c, 1ull) + 1;
    if (host_out) *host_out = v;
  }
}

#define CK(x)                                                         \
  do {                                                                \
    hipError_t e_ = (x);                                              \
    if (e_ != hipSuccess) {                                           \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  unsigned long long* d = nullptr;
  CK(hipMalloc(&d, 64));
  CK(hipMemset(d, 0, 64));
  unsigned long long* pin = nullptr;
  CK(hipHostMalloc(&pin, 64, hipHostMallocDefault));
  unsigned long long* pin_c = nullptr;  // coherent, for direct kernel writes
  CK(hipHostMalloc(&pin_c, 64, hipHostMallocCoherent | hipHostMallocMapped));
  const int iters = 3000;
  for (int mode = 0; mode < 3; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      unsigned long long stack_v = 0, last = 0;
      auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < iters; ++i) {
        if (mode == 2) {
          k_inc<<<1, 64, 0, s>>>(d, pin_c);
          CK(hipStreamSynchronize(s));
          last = *(volatile unsigned long long*)pin_c;
        } else {
          k_inc<<<1, 64, 0, s>>>(d, nullptr);
          unsigned long long* dst = mode == 0 ? &stack_v : pin;
          CK(hipMemcpyAsync(dst, d, 8, hipMemcpyDeviceToHost, s));
          CK(hipStreamSynchronize(s));
          last = *dst;
        }
      }
      auto t1 = std::chrono::steady_clock::now();
      const double us = std::chrono::duration<double, std::micro>(t1 - t0).count() / iters;
      printf("%s: %.2f us per round trip (last %llu)\n",
             mode == 0 ? "pageable D2H" : mode == 1 ? "pinned D2H" : "kernel -> pinned host", us, last);
    }
  }
  // launch-only reference: back-to-back tiny kernels, one sync at the end
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < iters; ++i) k_inc<<<1, 64, 0, s>>>(d, nullptr);
  CK(hipStreamSynchronize(s));
  auto t1 = std::chrono::steady_clock::now();
  printf("queued tiny kernels: %.2f us each\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / iters);
  return 0;
}
