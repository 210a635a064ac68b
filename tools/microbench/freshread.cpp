// freshread.cpp — is the first read of a just-written /dev/shm file slower
// than later reads of it?  Writes a file with fwrite (as apg_fastb_write
// does), then reads it three times with 16 pread threads (16 MiB chunks);
// then writes a second file and reads it after posix_fadvise(WILLNEED).
// Microbenchmark, not product code.
#include <fcntl.h>
#include <sys/mman.h>
#include <cstring>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static void write_file(const char* path, uint64_t bytes) {
  FILE* f = fopen(path, "wb");
  std::vector<char> blk(1 << 20, 3);
  for (uint64_t w = 0; w < bytes; w += blk.size()) fwrite(blk.data(), 1, blk.size(), f);
  fclose(f);
}
static double read_file(const char* path, uint64_t bytes, int T) {
  const uint64_t chunk = 16ull << 20, nch = bytes / chunk;
  std::atomic<uint64_t> next{0};
  const double t0 = now();
  std::vector<std::thread> ts;
  for (int w = 0; w < T; ++w)
    ts.emplace_back([&] {
      std::vector<char> buf(chunk);
      const int fd = open(path, O_RDONLY);
      for (uint64_t c; (c = next.fetch_add(1)) < nch;)
        for (uint64_t got = 0; got < chunk;) got += (uint64_t)pread(fd, buf.data() + got, chunk - got, (off_t)(c * chunk + got));
      close(fd);
    });
  for (auto& t : ts) t.join();
  return bytes / (now() - t0) / 1e9;
}
static double mmap_read(const char* path, uint64_t bytes, int T, bool populate) {
  const uint64_t chunk = 16ull << 20, nch = bytes / chunk;
  const double t0 = now();
  const int fd = open(path, O_RDONLY);
  const uint8_t* m = (const uint8_t*)mmap(nullptr, bytes, PROT_READ, MAP_SHARED | (populate ? MAP_POPULATE : 0), fd, 0);
  close(fd);
  const double t1 = now();
  std::atomic<uint64_t> next{0};
  std::vector<std::thread> ts;
  for (int w = 0; w < T; ++w)
    ts.emplace_back([&] {
      std::vector<char> buf(chunk);
      for (uint64_t c; (c = next.fetch_add(1)) < nch;) memcpy(buf.data(), m + c * chunk, chunk);
    });
  for (auto& t : ts) t.join();
  const double t2 = now();
  munmap((void*)m, bytes);
  printf("  mmap%s: map %.1f ms, copy %.1f ms\n", populate ? "+populate" : "", (t1 - t0) * 1e3, (t2 - t1) * 1e3);
  return bytes / (t2 - t0) / 1e9;
}
int main() {
  const uint64_t bytes = 4ull << 30;
  const char* a = "/dev/shm/apg_fresh_a";
  const char* b = "/dev/shm/apg_fresh_b";
  double t0 = now();
  write_file(a, bytes);
  printf("write %.1f GB/s\n", bytes / (now() - t0) / 1e9);
  for (int r = 0; r < 3; ++r) printf("read %d: %.1f GB/s\n", r, read_file(a, bytes, 16));
  write_file(b, bytes);
  const int fd = open(b, O_RDONLY);
  t0 = now();
  posix_fadvise(fd, 0, (off_t)bytes, POSIX_FADV_WILLNEED);
  printf("fadvise WILLNEED %.1f ms\n", (now() - t0) * 1e3);
  close(fd);
  for (int r = 0; r < 2; ++r) printf("read b %d: %.1f GB/s\n", r, read_file(b, bytes, 16));
  const char* c = "/dev/shm/apg_fresh_c";
  write_file(c, bytes);
  printf("mmap c 0: %.1f GB/s\n", mmap_read(c, bytes, 16, false));
  printf("mmap c 1: %.1f GB/s\n", mmap_read(c, bytes, 16, false));
  const char* d = "/dev/shm/apg_fresh_d";
  write_file(d, bytes);
  printf("mmap d 0: %.1f GB/s\n", mmap_read(d, bytes, 16, true));
  unlink(c);
  unlink(d);
  const char* e = "/dev/shm/apg_fresh_e";
  write_file(e, bytes);
  printf("pread e 1 thread: %.1f GB/s\n", read_file(e, bytes, 1));
  printf("pread e again 16: %.1f GB/s\n", read_file(e, bytes, 16));
  unlink(e);
  unlink(a);
  unlink(b);
  return 0;
}
