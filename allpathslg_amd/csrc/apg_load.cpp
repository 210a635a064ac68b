// apg_load.cpp — .fastb / .qualb straight into a device read set.
//
// The module boundary of a drop-in ALLPATHS-LG stage is a pair of files in the
// RUN directory ([R:M] src/feudal/, every module's `frag_reads_*.fastb`
// inputs).  apg_fastb_read + apg_reads_upload parse the files
// into host arrays and then copy them (two passes over 5 GB for 40 M reads,
// one thread); here the payload goes from the file to HBM once: worker
// threads pread fixed-size chunks into their own pinned buffers and issue the
// H2D copy on their own stream, double-buffered, so file reads and PCIe
// transfers overlap across chunks and threads.  Offsets are read and
// validated as in apg_fastb_read (monotone; qualb offsets equal fastb's).
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "apg_core.hpp"

namespace apg {
int fmt_read_head(const char* path, bool qual, uint64_t* n, std::vector<uint64_t>* base_off, uint64_t* payload);
}

using namespace apg;

namespace {

constexpr uint64_t kLoadChunk = 16ull << 20;  // bytes per pread / H2D copy

struct Fd {
  int fd = -1;
  ~Fd() {
    if (fd >= 0) close(fd);
  }
};

// bytes [off, off + len) of the file -> dst (device), by `threads` workers.
int stream_to_device(int device, const char* path, uint64_t off, uint64_t len, uint8_t* dst, int threads) {
  if (!len) return APG_OK;
  Fd f;
  f.fd = open(path, O_RDONLY);
  if (f.fd < 0) {
    set_error(std::string("cannot open ") + path);
    return APG_E_IO;
  }
  const uint64_t nch = (len + kLoadChunk - 1) / kLoadChunk;
  const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)threads, nch));
  std::atomic<int> err{APG_OK};
  std::vector<std::string> msg(T);
  auto worker = [&](int w) {
    auto fail = [&](int code, const std::string& m) {
      int ok = APG_OK;
      if (err.compare_exchange_strong(ok, code)) msg[w] = m;
    };
    if (hipSetDevice(device) != hipSuccess) return fail(APG_E_HIP, "hipSetDevice failed");
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) return fail(APG_E_HIP, "hipStreamCreate");
    uint8_t* buf[2] = {nullptr, nullptr};
    hipEvent_t ev[2] = {nullptr, nullptr};
    bool used[2] = {false, false};
    bool ok = true;
    for (int b = 0; b < 2 && ok; ++b)
      ok = hipHostMalloc(reinterpret_cast<void**>(&buf[b]), kLoadChunk, 0) == hipSuccess &&
           hipEventCreateWithFlags(&ev[b], hipEventDisableTiming) == hipSuccess;
    if (!ok) fail(APG_E_NOMEM, "pinned staging buffers");
    int k = 0;
    for (uint64_t c = (uint64_t)w; ok && c < nch && err.load() == APG_OK; c += (uint64_t)T, k ^= 1) {
      if (used[k] && hipEventSynchronize(ev[k]) != hipSuccess) {  // this buffer's previous copy
        fail(APG_E_HIP, "hipEventSynchronize");
        break;
      }
      const uint64_t o = c * kLoadChunk, n = std::min(kLoadChunk, len - o);
      for (uint64_t got = 0; got < n;) {
        const ssize_t r = pread(f.fd, buf[k] + got, n - got, (off_t)(off + o + got));
        if (r <= 0) {
          fail(APG_E_IO, std::string("short read from ") + path);
          ok = false;
          break;
        }
        got += (uint64_t)r;
      }
      if (!ok) break;
      if (hipMemcpyAsync(dst + o, buf[k], n, hipMemcpyHostToDevice, st) != hipSuccess ||
          hipEventRecord(ev[k], st) != hipSuccess) {
        fail(APG_E_HIP, "hipMemcpyAsync");
        break;
      }
      used[k] = true;
    }
    (void)hipStreamSynchronize(st);
    for (int b = 0; b < 2; ++b) {
      if (ev[b]) (void)hipEventDestroy(ev[b]);
      if (buf[b]) (void)hipHostFree(buf[b]);
    }
    (void)hipStreamDestroy(st);
  };
  std::vector<std::thread> ts;
  for (int w = 0; w < T; ++w) ts.emplace_back(worker, w);
  for (auto& t : ts) t.join();
  if (err.load() != APG_OK) {
    for (auto& m : msg)
      if (!m.empty()) set_error("apg_reads_load_dev: " + m);
    return err.load();
  }
  return APG_OK;
}

}  // namespace

extern "C" {

int apg_reads_load_dev(apg_ctx* ctx, const char* fastb, const char* qualb, int threads, apg_dreads** out) {
  APG_REQUIRE(ctx && fastb && out, "apg_reads_load_dev: NULL argument");
  *out = nullptr;
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  auto ms = [&](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  uint64_t n = 0, pay = 0;
  std::vector<uint64_t> bo;
  APG_TRY(fmt_read_head(fastb, false, &n, &bo, &pay));
  // the qualb header and offsets are read while the fastb's are turned into a device read set
  uint64_t qpay = 0, nq = 0;
  std::vector<uint64_t> qo;
  int qrc = APG_OK;
  std::string qerr;
  std::thread qt;
  if (qualb)
    qt = std::thread([&] {
      try {  // nothing may escape a worker thread (std::terminate)
        qrc = fmt_read_head(qualb, true, &nq, &qo, &qpay);
        if (qrc) qerr = apg_last_error();
      } catch (const std::exception& e) {
        qrc = APG_E_NOMEM;
        qerr = std::string("reading ") + qualb + ": " + e.what();
      }
    });
  std::vector<uint64_t> yo(n + 1);
  int rc0 = apg_byte_offsets(bo.data(), n, yo.data());
  if (threads <= 0) threads = (int)std::min<unsigned>(4, std::max(1u, std::thread::hardware_concurrency()));
  apg_dreads* d = nullptr;
  if (rc0 == APG_OK) rc0 = dreads_create(ctx, n, bo.data(), yo.data(), qualb != nullptr, &d);
  if (qt.joinable()) qt.join();
  if (rc0 == APG_OK && qualb) {
    if (qrc) {
      set_error(qerr);  // the worker thread's error text (thread-local)
      rc0 = qrc;
    } else if (nq != n || std::memcmp(qo.data(), bo.data(), (n + 1) * 8) != 0) {
      set_error(std::string("qualb/fastb length mismatch: ") + qualb);
      rc0 = APG_E_IO;
    }
  }
  if (rc0 != APG_OK) {
    if (d) apg_reads_free(d);
    return rc0;
  }
  // the packed zero-fill and the offsets' H2D are on ctx->stream: done before the workers write
  if (hipStreamSynchronize(ctx->stream) != hipSuccess) {
    apg_reads_free(d);
    set_error("apg_reads_load_dev: hipStreamSynchronize");
    return APG_E_HIP;
  }
  const double t_meta = ms(t0);
  const auto t1 = clk::now();
  int rc = stream_to_device(ctx->device, fastb, pay, d->n_bytes, d->d_packed, threads);
  const double t_bases = ms(t1);
  const auto t2 = clk::now();
  if (rc == APG_OK && qualb && n) rc = stream_to_device(ctx->device, qualb, qpay, d->n_bases, d->d_quals, threads);
  vlog(ctx, "load_dev: %llu reads, offsets + checks %.1f ms, bases %.1f ms (%.2f GB/s), quals %.1f ms, %d threads",
       (unsigned long long)n, t_meta, t_bases, d->n_bytes / std::max(t_bases, 1e-3) / 1e6, ms(t2), threads);
  if (rc != APG_OK) {
    apg_reads_free(d);
    return rc;
  }
  *out = d;
  return APG_OK;
}

}  // extern "C"
