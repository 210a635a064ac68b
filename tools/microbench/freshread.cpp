// freshread.cpp — what makes the first pread of a /dev/shm file slow on the
// MI355X hosts?  Candidates: the file's page-cache pages being fresh (just
// written), or the reader's destination buffers being fresh anonymous pages.
// Per-thread 16 MiB buffers are either reused (allocated and touched once,
// outside the timed region) or allocated fresh inside it.  Microbenchmark,
// not product code.
#include <fcntl.h>
#include <sched.h>
#include <sys/syscall.h>
#include <sys/mman.h>
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
static void write_file(const char* path, uint64_t bytes) {
  FILE* f = fopen(path, "wb");
  std::vector<char> blk(1 << 20, 3);
  for (uint64_t w = 0; w < bytes; w += blk.size()) fwrite(blk.data(), 1, blk.size(), f);
  fclose(f);
}
constexpr uint64_t kChunk = 16ull << 20;
constexpr int kT = 16;
static char* g_buf[kT];
// fresh: each thread mmaps (and unmaps) its own buffer inside the timed region
static std::vector<int> g_cpus;  // when non-empty: reader threads pinned round-robin to these CPUs
static std::vector<int> node_cpus(int node) {
  std::vector<int> out;
  char fn[128];
  snprintf(fn, sizeof fn, "/sys/devices/system/node/node%d/cpulist", node);
  FILE* f = fopen(fn, "r");
  if (!f) return out;
  int a, b;
  char sep;
  while (fscanf(f, "%d", &a) == 1) {
    b = a;
    if (fscanf(f, "%c", &sep) == 1 && sep == '-') {
      if (fscanf(f, "%d", &b) != 1) break;
      if (fscanf(f, "%c", &sep) != 1) sep = 0;
    }
    for (int c = a; c <= b; ++c) out.push_back(c);
    if (sep != ',') break;
  }
  fclose(f);
  return out;
}
// NUMA node of the page holding byte `off` of the file (move_pages without moving)
static int page_node(const char* path, uint64_t off) {
  const int fd = open(path, O_RDONLY);
  void* m = mmap(nullptr, 4096, PROT_READ, MAP_SHARED, fd, (off_t)(off & ~4095ull));
  close(fd);
  volatile char c = *(char*)m;
  (void)c;
  void* pages[1] = {m};
  int status[1] = {-1};
  syscall(SYS_move_pages, 0, 1, pages, nullptr, status, 0);
  munmap(m, 4096);
  return status[0];
}
static double read_file(const char* path, uint64_t bytes, bool fresh) {
  const uint64_t nch = bytes / kChunk;
  std::atomic<uint64_t> next{0};
  const double t0 = now();
  std::vector<std::thread> ts;
  for (int w = 0; w < kT; ++w)
    ts.emplace_back([&, w] {
      if (!g_cpus.empty()) {
        cpu_set_t cs;
        CPU_ZERO(&cs);
        CPU_SET(g_cpus[w % g_cpus.size()], &cs);
        sched_setaffinity(0, sizeof cs, &cs);
      }
      char* buf = fresh ? (char*)mmap(nullptr, kChunk, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0)
                        : g_buf[w];
      const int fd = open(path, O_RDONLY);
      for (uint64_t c; (c = next.fetch_add(1)) < nch;)
        for (uint64_t got = 0; got < kChunk;) got += (uint64_t)pread(fd, buf + got, kChunk - got, (off_t)(c * kChunk + got));
      close(fd);
      if (fresh) munmap(buf, kChunk);
    });
  for (auto& t : ts) t.join();
  return bytes / (now() - t0) / 1e9;
}
int main() {
  const uint64_t bytes = 4ull << 30;
  for (int w = 0; w < kT; ++w) {
    g_buf[w] = (char*)malloc(kChunk);
    memset(g_buf[w], 1, kChunk);
  }
  const char* a = "/dev/shm/apg_fresh_a";
  double t0 = now();
  write_file(a, bytes);
  printf("fwrite %.1f GB/s; file pages on nodes %d %d %d\n", bytes / (now() - t0) / 1e9, page_node(a, 0),
         page_node(a, bytes / 2), page_node(a, bytes - 4096));
  for (int node = 0; node < 8; ++node) {
    g_cpus = node_cpus(node);
    if (g_cpus.empty()) break;
    printf("readers on node %d (%zu cpus, first %d): %.1f, %.1f, %.1f GB/s\n", node, g_cpus.size(), g_cpus[0],
           read_file(a, bytes, false), read_file(a, bytes, false), read_file(a, bytes, false));
  }
  g_cpus.clear();
  printf("unpinned: %.1f, %.1f, %.1f GB/s\n", read_file(a, bytes, false), read_file(a, bytes, false),
         read_file(a, bytes, false));
  // fresh anonymous memory: first touch rate
  t0 = now();
  char* m = (char*)mmap(nullptr, 1ull << 30, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  memset(m, 1, 1ull << 30);
  printf("first touch of 1 GiB anonymous memory, 1 thread: %.2f GB/s\n", (1ull << 30) / (now() - t0) / 1e9);
  t0 = now();
  memset(m, 2, 1ull << 30);
  printf("second touch: %.2f GB/s\n", (1ull << 30) / (now() - t0) / 1e9);
  munmap(m, 1ull << 30);
  unlink(a);
  return 0;
}
