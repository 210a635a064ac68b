// san_host.cpp — libapg's host-side code under the sanitizers (SURVEY §5
// "race detection / sanitizers").  Built by
// tests/sanitize/Makefile from the library's own host sources (the .cpp files
// of allpathslg_amd/csrc, compiled here with -fsanitize=address,undefined or
// -fsanitize=thread) and run in this container, no GPU:
//   * APG-fastb / APG-qualb round trips and every rejected header (bad magic,
//     implausible or file-exceeding read count, offsets not starting at 0,
//     non-monotone offsets, truncated payload);
//   * unipath-stage files (apg_graph_write / read, KmerPath containers);
//   * the synthetic read simulator's worker threads (1 vs 8 threads: same
//     bytes);
//   * the TCP communicator (exchange.cpp) at world 1, 2 and 4 with the ranks
//     as threads of this process — alltoallv / allgatherv with irregular and
//     empty segments, sums and maxima, barriers — and a send/receive size
//     mismatch that must fail on the receiver instead of hanging.
// The device paths (apg_reads_load_dev's pinned-buffer workers, RCCL) need a
// GPU and run in the -m gpu suite; GPU ASan is not available on the pool.
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <functional>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "apg.h"

namespace {

int fails = 0;
#define CHECK(c)                                                                  \
  do {                                                                            \
    if (!(c)) {                                                                   \
      std::fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #c, apg_last_error()); \
      ++fails;                                                                    \
    }                                                                             \
  } while (0)

uint64_t rng_state = 0x9E3779B97F4A7C15ull;
uint64_t rnd() {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return rng_state;
}

std::string tmpdir;

struct HostReads {
  std::vector<uint64_t> bo, yo;
  std::vector<uint8_t> packed, quals;
  apg_reads r{};
  void make(uint64_t n) {
    bo.assign(n + 1, 0);
    yo.assign(n + 1, 0);
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t len = (i % 17 == 0) ? 0 : rnd() % 151;
      bo[i + 1] = bo[i] + len;
    }
    CHECK(apg_byte_offsets(bo.data(), n, yo.data()) == APG_OK);
    packed.resize(yo[n] + 64);
    quals.resize(bo[n] + 1);
    for (auto& b : packed) b = (uint8_t)rnd();
    for (uint64_t i = 0; i < n; ++i) {  // bits past a read's end are zero
      const uint64_t len = bo[i + 1] - bo[i];
      if (len % 4) packed[yo[i] + len / 4] &= (uint8_t)((1u << (2 * (len % 4))) - 1);
    }
    for (auto& q : quals) q = (uint8_t)(2 + rnd() % 39);
    r.n_reads = n;
    r.base_off = bo.data();
    r.byte_off = yo.data();
    r.packed = packed.data();
    r.quals = quals.data();
  }
};

void write_bytes(const std::string& path, const std::vector<uint8_t>& b) {
  FILE* f = std::fopen(path.c_str(), "wb");
  std::fwrite(b.data(), 1, b.size(), f);
  std::fclose(f);
}

std::vector<uint8_t> read_bytes(const std::string& path) {
  std::vector<uint8_t> b;
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return b;
  int c;
  while ((c = std::fgetc(f)) != EOF) b.push_back((uint8_t)c);
  std::fclose(f);
  return b;
}

void test_formats() {
  HostReads h;
  h.make(5000);
  const std::string fb = tmpdir + "/r.fastb", qb = tmpdir + "/r.qualb";
  CHECK(apg_fastb_write(fb.c_str(), &h.r) == APG_OK);
  CHECK(apg_qualb_write(qb.c_str(), &h.r) == APG_OK);
  apg_reads in{};
  CHECK(apg_fastb_read(fb.c_str(), &in) == APG_OK);
  CHECK(apg_qualb_read(qb.c_str(), &in) == APG_OK);
  CHECK(in.n_reads == h.r.n_reads);
  CHECK(std::memcmp(in.base_off, h.bo.data(), 8 * (h.r.n_reads + 1)) == 0);
  CHECK(std::memcmp(in.packed, h.packed.data(), h.yo.back()) == 0);
  CHECK(std::memcmp(in.quals, h.quals.data(), h.bo.back()) == 0);
  apg_reads_release(&in);
  // rejected headers: each must fail with APG_E_IO, never crash or allocate wildly
  const std::vector<uint8_t> good = read_bytes(fb);
  auto expect_bad = [&](std::vector<uint8_t> b, const char* what) {
    const std::string p = tmpdir + "/bad.fastb";
    write_bytes(p, b);
    apg_reads x{};
    const int rc = apg_fastb_read(p.c_str(), &x);
    if (rc != APG_E_IO) std::fprintf(stderr, "FAIL: %s accepted (rc %d)\n", what, rc), ++fails;
    apg_reads_release(&x);
  };
  {
    auto b = good;
    b[0] = 'X';
    expect_bad(b, "bad magic");
  }
  {
    auto b = good;
    const uint64_t n = 1ull << 39;  // plausible count, far beyond the file
    std::memcpy(&b[16], &n, 8);
    expect_bad(b, "read count beyond the file");
  }
  {
    auto b = good;
    const uint64_t n = ~0ull;
    std::memcpy(&b[16], &n, 8);
    expect_bad(b, "implausible read count");
  }
  {
    auto b = good;
    const uint64_t one = 1;  // base_off[0] = 1
    std::memcpy(&b[32], &one, 8);
    expect_bad(b, "offsets not starting at 0");
  }
  {
    auto b = good;
    uint64_t v;
    std::memcpy(&v, &b[32 + 8 * 10], 8);
    v += 1000;  // base_off[10] past base_off[11]
    std::memcpy(&b[32 + 8 * 10], &v, 8);
    expect_bad(b, "non-monotone offsets");
  }
  {
    auto b = good;
    b.resize(b.size() - 100);
    expect_bad(b, "truncated payload");
  }
  // an empty set round-trips
  apg_reads e{};
  uint64_t zero = 0;
  e.base_off = &zero;
  e.byte_off = &zero;
  const std::string ep = tmpdir + "/e.fastb";
  CHECK(apg_fastb_write(ep.c_str(), &e) == APG_OK);
  apg_reads ein{};
  CHECK(apg_fastb_read(ep.c_str(), &ein) == APG_OK && ein.n_reads == 0);
  apg_reads_release(&ein);
}

void test_graphio() {
  const uint64_t U = 6, NR = 3;
  std::vector<uint64_t> len = {5, 5, 1, 1, 9, 9}, idb = {0, 5, 10, 11, 12, 21}, rc = {1, 0, 3, 2, 5, 4};
  std::vector<uint64_t> ub_off(U + 1, 0);
  const int K = 4;
  for (uint64_t u = 0; u < U; ++u) ub_off[u + 1] = ub_off[u] + len[u] + K - 1;
  std::vector<uint8_t> ub(ub_off[U]);
  for (auto& b : ub) b = (uint8_t)(rnd() & 3);
  std::vector<uint64_t> from = {0, 1, 2, 3, 4, 5}, to = {1, 2, 3, 4, 5, 0};
  std::vector<uint64_t> po = {0, 1, 3, 3}, ps = {2, 7, 12}, pl = {3, 1, 4};
  apg_unipath_graph g{};
  g.K = K;
  g.n_nodes = 30;
  g.n_unipaths = U;
  g.len = len.data();
  g.id_base = idb.data();
  g.rc = rc.data();
  g.ub_off = ub_off.data();
  g.unibases = ub.data();
  g.n_vertices = 6;
  g.from = from.data();
  g.to = to.data();
  g.n_reads = NR;
  g.path_off = po.data();
  g.n_intervals = 3;
  g.path_start = ps.data();
  g.path_len = pl.data();
  const std::string head = tmpdir + "/all_reads";
  CHECK(apg_graph_write(head.c_str(), &g) == APG_OK);
  apg_unipath_graph r{};
  CHECK(apg_graph_read(head.c_str(), K, &r) == APG_OK);
  CHECK(r.n_unipaths == U && r.n_vertices == 6 && r.n_reads == NR && r.n_intervals == 3);
  CHECK(r.len && std::memcmp(r.len, len.data(), 8 * U) == 0);
  CHECK(r.unibases && std::memcmp(r.unibases, ub.data(), ub.size()) == 0);
  CHECK(r.path_start && std::memcmp(r.path_start, ps.data(), 24) == 0);
  apg_unipath_graph_free(&r);
  const std::string kp = tmpdir + "/x.paths.k4";
  CHECK(apg_kmerpaths_write(kp.c_str(), K, NR, po.data(), ps.data(), pl.data()) == APG_OK);
  int k2 = 0;
  uint64_t n2 = 0, ni = 0, *o2 = nullptr, *s2 = nullptr, *l2 = nullptr;
  CHECK(apg_kmerpaths_read(kp.c_str(), &k2, &n2, &o2, &ni, &s2, &l2) == APG_OK);
  CHECK(k2 == K && n2 == NR && ni == 3 && o2 && std::memcmp(l2, pl.data(), 24) == 0);
  apg_free(o2);
  apg_free(s2);
  apg_free(l2);
}

void test_synth_threads() {
  const uint64_t G = 200000;
  std::vector<uint8_t> genome(G);
  CHECK(apg_synth_genome(G, 7, genome.data()) == APG_OK);
  apg_synth_params p{};
  p.genome_len = G;
  p.seed = 11;
  p.n_pairs = 30000;
  p.read_len = 100;
  p.insert_mean = 180;
  p.insert_sd = 18;
  p.err_lo = 0.002;
  p.err_hi = 0.02;
  uint64_t n = 0, nb = 0, ny = 0;
  CHECK(apg_synth_sizes(&p, &n, &nb, &ny) == APG_OK);
  std::vector<uint8_t> out[2];
  std::vector<uint8_t> q[2];
  for (int t = 0; t < 2; ++t) {
    p.threads = t ? 8 : 1;
    std::vector<uint64_t> bo(n + 1), yo(n + 1);
    out[t].assign(ny + 64, 0);
    q[t].assign(nb, 0);
    CHECK(apg_synth_reads(&p, genome.data(), bo.data(), yo.data(), out[t].data(), q[t].data()) == APG_OK);
  }
  CHECK(out[0] == out[1] && q[0] == q[1]);
}

int free_port() {
  // a port the kernel hands out for bind(0); the communicator's rank 0 then
  // binds it again (SO_REUSEADDR)
  const int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in sa{};
  sa.sin_family = AF_INET;
  sa.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  socklen_t len = sizeof sa;
  if (fd < 0 || ::bind(fd, reinterpret_cast<sockaddr*>(&sa), sizeof sa) != 0 ||
      ::getsockname(fd, reinterpret_cast<sockaddr*>(&sa), &len) != 0)
    std::abort();
  const int port = ntohs(sa.sin_port);
  ::close(fd);
  return port;
}

// world ranks as threads of this process
void run_ranks(int world, const std::function<void(int, apg_comm*)>& body) {
  const int port = free_port();
  std::vector<std::thread> ts;
  for (int r = 0; r < world; ++r)
    ts.emplace_back([&, r] {
      apg_comm* c = nullptr;
      const int rc = apg_comm_init_tcp(nullptr, "127.0.0.1", port, r, world, 60000, &c);
      if (rc != APG_OK) {
        std::fprintf(stderr, "FAIL: comm init rank %d/%d: %s\n", r, world, apg_last_error());
        ++fails;
        return;
      }
      body(r, c);
      apg_comm_destroy(c);
    });
  for (auto& t : ts) t.join();
}

uint8_t seg_byte(int src, int dst, uint64_t i) { return (uint8_t)(src * 31 + dst * 7 + i * 13 + (i >> 9)); }

void test_comm(int world) {
  std::vector<std::vector<uint64_t>> sz(world, std::vector<uint64_t>(world));
  for (int s = 0; s < world; ++s)
    for (int d = 0; d < world; ++d) sz[s][d] = ((s + 2 * d) % 3 == 0) ? 0 : 1000 + rnd() % 300000;
  sz[0][world - 1] = 5u << 20;  // one larger segment (several poll rounds)
  std::atomic<int> bad{0};
  run_ranks(world, [&](int r, apg_comm* c) {
    // alltoallv
    std::vector<uint64_t> sb(world), rb(world);
    uint64_t ts = 0, tr = 0;
    for (int q = 0; q < world; ++q) {
      sb[q] = sz[r][q];
      rb[q] = sz[q][r];
      ts += sb[q];
      tr += rb[q];
    }
    std::vector<uint8_t> send(ts + 1), recv(tr + 1, 0xEE);
    uint64_t o = 0;
    for (int q = 0; q < world; ++q)
      for (uint64_t i = 0; i < sb[q]; ++i) send[o++] = seg_byte(r, q, i);
    if (apg_comm_alltoallv(c, send.data(), sb.data(), recv.data(), rb.data()) != APG_OK) ++bad;
    o = 0;
    for (int q = 0; q < world; ++q)
      for (uint64_t i = 0; i < rb[q]; ++i)
        if (recv[o++] != seg_byte(q, r, i)) {
          ++bad;
          break;
        }
    // allgatherv
    std::vector<uint64_t> gb(world);
    uint64_t gt = 0;
    for (int q = 0; q < world; ++q) gt += (gb[q] = 100 + 977 * q);
    std::vector<uint8_t> mine(gb[r]), all(gt);
    for (uint64_t i = 0; i < gb[r]; ++i) mine[i] = seg_byte(r, 99, i);
    if (apg_comm_allgatherv(c, mine.data(), gb[r], all.data(), gb.data()) != APG_OK) ++bad;
    o = 0;
    for (int q = 0; q < world; ++q)
      for (uint64_t i = 0; i < gb[q]; ++i)
        if (all[o++] != seg_byte(q, 99, i)) {
          ++bad;
          break;
        }
    // sums and maxima
    uint64_t v[3] = {(uint64_t)r + 1, 1000u * (uint64_t)r, 7};
    if (apg_comm_allreduce_u64(c, v, 3, APG_COMM_SUM) != APG_OK) ++bad;
    if (v[0] != (uint64_t)world * (world + 1) / 2 || v[2] != 7u * world) ++bad;
    uint64_t m = (uint64_t)r * 5;
    if (apg_comm_allreduce_u64(c, &m, 1, APG_COMM_MAX) != APG_OK || m != 5u * (world - 1)) ++bad;
    if (apg_comm_barrier(c) != APG_OK) ++bad;
  });
  if (bad) std::fprintf(stderr, "FAIL: comm world %d: %d bad checks\n", world, bad.load()), ++fails;
}

void test_comm_mismatch() {
  std::atomic<int> errs{0};
  run_ranks(2, [&](int r, apg_comm* c) {
    // rank 1 sends 64 bytes to rank 0, which expects 32: rank 0 must get an error
    std::vector<uint64_t> sb = {r == 1 ? 64u : 0u, 0}, rb = {0, r == 0 ? 32u : 0u};
    if (r == 0) sb = {0, 16};
    if (r == 1) rb = {16, 0};
    std::vector<uint8_t> send(128, 1), recv(128, 0);
    const int rc = apg_comm_alltoallv(c, send.data(), sb.data(), recv.data(), rb.data());
    if (rc != APG_OK) ++errs;
  });
  CHECK(errs.load() >= 1);
}

}  // namespace

int main() {
  char tmpl[] = "/tmp/apg_san_XXXXXX";
  if (!mkdtemp(tmpl)) return 2;
  tmpdir = tmpl;
  test_formats();
  test_graphio();
  test_synth_threads();
  for (int w : {1, 2, 4}) test_comm(w);
  test_comm_mismatch();
  std::string rm = "rm -rf " + tmpdir;
  if (std::system(rm.c_str()) != 0) std::fprintf(stderr, "warning: could not remove %s\n", tmpdir.c_str());
  std::printf("san_host: %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}
