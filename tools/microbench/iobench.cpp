// iobench.cpp — where the file -> HBM time goes (apg_reads_load_dev's
// staging): a file on /dev/shm read by T threads into pinned chunks (pread
// only), pinned chunks copied to the device by T streams (H2D only), and both
// overlapped as the loader does, for T in {4, 8, 16} and chunk sizes 4 / 16 /
// 64 MiB.  Prints GB/s per configuration.  Microbenchmark, not product code.
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const uint64_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 10) : (4ull << 30);
  const char* path = "/dev/shm/apg_iobench.bin";
  {
    FILE* f = fopen(path, "wb");
    std::vector<char> blk(64 << 20, 7);
    for (uint64_t w = 0; w < bytes; w += blk.size()) fwrite(blk.data(), 1, std::min<uint64_t>(blk.size(), bytes - w), f);
    fclose(f);
  }
  uint8_t* dev = nullptr;
  if (hipMalloc(&dev, bytes) != hipSuccess) return 1;
  for (uint64_t chunk : {4ull << 20, 16ull << 20, 64ull << 20})
    for (int T : {4, 8, 16}) {
      std::vector<uint8_t*> buf(2 * T);
      std::vector<hipStream_t> st(T);
      std::vector<hipEvent_t> ev(2 * T);
      for (int i = 0; i < 2 * T; ++i) {
        (void)hipHostMalloc((void**)&buf[i], chunk, 0);
        (void)hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
      }
      for (int i = 0; i < T; ++i) (void)hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking);
      const uint64_t nch = (bytes + chunk - 1) / chunk;
      double r[3];
      for (int mode = 0; mode < 3; ++mode) {  // 0 pread only, 1 H2D only, 2 both
        std::atomic<uint64_t> next{0};
        const double t0 = now();
        std::vector<std::thread> ts;
        for (int w = 0; w < T; ++w)
          ts.emplace_back([&, w] {
            (void)hipSetDevice(0);
            const int fd = open(path, O_RDONLY);
            int k = 0;
            bool used[2] = {false, false};
            for (uint64_t c; (c = next.fetch_add(1)) < nch; k ^= 1) {
              const uint64_t o = c * chunk, n = std::min(chunk, bytes - o);
              uint8_t* b = buf[2 * w + k];
              if (used[k]) (void)hipEventSynchronize(ev[2 * w + k]);
              if (mode != 1)
                for (uint64_t got = 0; got < n;) got += (uint64_t)pread(fd, b + got, n - got, (off_t)(o + got));
              if (mode != 0) {
                (void)hipMemcpyAsync(dev + o, b, n, hipMemcpyHostToDevice, st[w]);
                (void)hipEventRecord(ev[2 * w + k], st[w]);
                used[k] = true;
              }
            }
            (void)hipStreamSynchronize(st[w]);
            close(fd);
          });
        for (auto& t : ts) t.join();
        r[mode] = bytes / (now() - t0) / 1e9;
      }
      printf("chunk %3llu MiB  T=%2d  pread %6.1f GB/s  H2D %6.1f GB/s  both %6.1f GB/s\n",
             (unsigned long long)(chunk >> 20), T, r[0], r[1], r[2]);
      fflush(stdout);
      for (auto b : buf) (void)hipHostFree(b);
      for (auto e : ev) (void)hipEventDestroy(e);
      for (auto s : st) (void)hipStreamDestroy(s);
    }
  unlink(path);
  return 0;
}
