// apg_load.cpp — .fastb / .qualb straight into a device read set.
//
// The module boundary of a drop-in ALLPATHS-LG stage is a pair of files in the
// RUN directory ([R:M] src/feudal/, every module's `frag_reads_*.fastb`
// inputs).  apg_fastb_read + apg_reads_upload parse the files
// into host arrays and then copy them (two passes over 5 GB for 40 M reads,
// one thread); here the payload goes from the file to HBM once: worker
// threads pread fixed-size chunks into their own pinned buffers and issue the
// H2D copy on their own stream, double-buffered, so file reads and PCIe
// transfers overlap across chunks and threads.  Measured on the MI355X pool
// (40 M reads, 5 GB): 35-48 GB/s re-reading files already loaded once in the
// process, 10-14 GB/s on the first load of files written just before
// (bench.py file_to_graph, scripts/diag/load_rate.py); the host's own pread of
// /dev/shm files varies ~13-150 GB/s from read to read with no GPU involved
// (tools/microbench/freshread.cpp), so that first-load figure is not the
// loader's alone.  Copying out of a mapping instead (APG_LOAD_IO=mmap)
// measured the same first load and a slower re-read (24-27 GB/s: page faults
// on every fresh mapping).  The offset tables take the
// same path and are validated on the device (apg_fastb_read's rules:
// monotone, from 0 to the header's total; qualb offsets equal fastb's; file
// sizes exact), where the byte offsets are also derived.
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <new>
#include <vector>

#include "apg_core.hpp"

using namespace apg;

namespace {

struct Fd {
  int fd = -1;
  ~Fd() {
    if (fd >= 0) close(fd);
  }
};

// bytes [off, off + len) of the file -> dst (device), by `threads` workers,
// each double-buffering its copy out of the mapping into its pinned staging chunk against the H2D
// copy of its previous chunk on its own stream (the context's staging pool).
// The caller has checked the file's size against [off, off + len); a file
// truncated while it is being loaded faults the copy (SIGBUS), as any mapped
// read would.
struct Map {
  void* base = MAP_FAILED;
  uint64_t bytes = 0;
  ~Map() {
    if (base != MAP_FAILED) munmap(base, bytes);
  }
};

// w0: the first staging worker used (a load streaming two files at once gives
// each its own workers; the caller has made the pool large enough).
int stream_to_device(apg_ctx* ctx, const char* path, uint64_t off, uint64_t len, uint8_t* dst, int threads,
                     int w0 = 0) {
  if (!len) return APG_OK;
  Fd f;
  f.fd = open(path, O_RDONLY);
  if (f.fd < 0) {
    set_error(std::string("cannot open ") + path);
    return APG_E_IO;
  }
  // APG_LOAD_IO=mmap copies out of a read-only mapping instead (A/B knob)
  static const bool use_pread = [] {
    const char* e = std::getenv("APG_LOAD_IO");
    return !(e && std::strcmp(e, "mmap") == 0);
  }();
  const uint64_t page = (uint64_t)sysconf(_SC_PAGESIZE), moff = off & ~(page - 1);
  Map m;
  const uint8_t* src = nullptr;
  if (!use_pread) {
    m.bytes = off + len - moff;
    m.base = mmap(nullptr, m.bytes, PROT_READ, MAP_SHARED, f.fd, (off_t)moff);
    if (m.base == MAP_FAILED) {
      set_error(std::string("cannot map ") + path);
      return APG_E_IO;
    }
    src = static_cast<const uint8_t*>(m.base) + (off - moff);
  }
  const uint64_t nch = (len + kStageChunk - 1) / kStageChunk;
  const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)threads, nch));
  if (w0 == 0) APG_TRY(staging_get(ctx, T));
  std::atomic<int> err{APG_OK};
  std::atomic<uint64_t> next{0};
  std::vector<std::string> msg(T);
  const int device = ctx->device;
  auto worker = [&](int w) {
    auto fail = [&](int code, const std::string& m) {
      int ok = APG_OK;
      if (err.compare_exchange_strong(ok, code)) msg[w] = m;
    };
    if (hipSetDevice(device) != hipSuccess) return fail(APG_E_HIP, "hipSetDevice failed");
    const int sw = w0 + w;
    uint8_t* buf[2] = {ctx->staging.buf[2 * sw], ctx->staging.buf[2 * sw + 1]};
    hipEvent_t ev[2] = {ctx->staging.ev[2 * sw], ctx->staging.ev[2 * sw + 1]};
    hipStream_t st = ctx->staging.st[sw];
    bool used[2] = {false, false};
    int k = 0;
    for (uint64_t c; (c = next.fetch_add(1)) < nch && err.load() == APG_OK; k ^= 1) {
      if (used[k] && hipEventSynchronize(ev[k]) != hipSuccess) {  // this buffer's previous copy
        fail(APG_E_HIP, "hipEventSynchronize");
        break;
      }
      const uint64_t o = c * kStageChunk, n = std::min(kStageChunk, len - o);
      if (src) {
        std::memcpy(buf[k], src + o, n);
      } else {
        bool ok = true;
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
      }
      if (hipMemcpyAsync(dst + o, buf[k], n, hipMemcpyHostToDevice, st) != hipSuccess ||
          hipEventRecord(ev[k], st) != hipSuccess) {
        fail(APG_E_HIP, "hipMemcpyAsync");
        break;
      }
      used[k] = true;
    }
    (void)hipStreamSynchronize(st);
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

// Header of an APG-fastb / APG-qualb file (apg_formats.cpp layout): read count,
// base total and the file size.
struct Head {
  uint64_t n = 0, total = 0, size = 0;
};
int read_head(const char* path, const char* magic, Head* h) {
  Fd f;
  f.fd = open(path, O_RDONLY);
  if (f.fd < 0) {
    set_error(std::string("cannot open ") + path);
    return APG_E_IO;
  }
  uint8_t b[32];
  if (pread(f.fd, b, 32, 0) != 32 || std::memcmp(b, magic, 8) != 0) {
    set_error(std::string("bad magic in ") + path);
    return APG_E_IO;
  }
  uint32_t ver = 0;
  std::memcpy(&ver, b + 8, 4);
  if (ver != 0) {
    set_error(std::string("unsupported version in ") + path);
    return APG_E_IO;
  }
  std::memcpy(&h->n, b + 16, 8);
  std::memcpy(&h->total, b + 24, 8);
  const off_t end = lseek(f.fd, 0, SEEK_END);
  h->size = end < 0 ? 0 : (uint64_t)end;
  if (h->n > (1ull << 40) || 32 + 8 * (h->n + 1) > h->size) {
    set_error(std::string("truncated offsets in ") + path);
    return APG_E_IO;
  }
  return APG_OK;
}

// The offset tables of a .fastb and its .qualb (both at byte 32, n + 1 u64)
// are identical: compared chunk by chunk from the files (apg_qualb_read's
// rule: the qualities follow the bases read by read).
int qualb_offsets_match(const char* fastb, const char* qualb, uint64_t n) {
  Fd a, b;
  a.fd = open(fastb, O_RDONLY);
  b.fd = open(qualb, O_RDONLY);
  if (a.fd < 0 || b.fd < 0) {
    set_error(std::string("cannot open ") + (a.fd < 0 ? fastb : qualb));
    return APG_E_IO;
  }
  constexpr uint64_t kChunk = 8ull << 20;
  std::vector<uint8_t> x(kChunk), y(kChunk);
  const uint64_t len = 8 * (n + 1);
  for (uint64_t o = 0; o < len; o += kChunk) {
    const uint64_t m = std::min(kChunk, len - o);
    if (pread(a.fd, x.data(), m, (off_t)(32 + o)) != (ssize_t)m || pread(b.fd, y.data(), m, (off_t)(32 + o)) != (ssize_t)m) {
      set_error(std::string("short read of the offset tables of ") + qualb);
      return APG_E_IO;
    }
    if (std::memcmp(x.data(), y.data(), m) != 0) {
      set_error(std::string("qualb/fastb length mismatch: ") + qualb);
      return APG_E_IO;
    }
  }
  return APG_OK;
}

}  // namespace

namespace apg {
struct DreadsPending {
  std::thread th;
  int rc = APG_OK;
  std::string err;
  apg_ctx* ctx = nullptr;
  double ms = 0;
};

void dreads_join(const apg_dreads* cd) {
  apg_dreads* d = const_cast<apg_dreads*>(cd);
  if (!d || !d->pending) return;
  DreadsPending* p = d->pending;
  p->th.join();
  d->pending = nullptr;
  if (p->ctx && p->ctx->bg_load == d) p->ctx->bg_load = nullptr;
  d->quals_rc = p->rc;
  if (p->rc != APG_OK) d->quals_err = p->err;
  vlog(p->ctx, "load_dev: qualities landed in the background (%.1f ms of streaming)", p->ms);
  delete p;
}

int dreads_quals_ready(const apg_dreads* cd) {
  if (!cd) return APG_OK;
  dreads_join(cd);
  if (cd->quals_rc != APG_OK) set_error(cd->quals_err);
  return cd->quals_rc;
}
}  // namespace apg

extern "C" {

// Files -> HBM with no host pass over the reads: the offset tables stream to
// the device like the payloads (pinned chunks, worker threads), are validated
// there (dreads_device_shape: monotone, starting at 0, ending at the header's
// total, qualb offsets equal to fastb's) and the byte offsets are derived there
// by a scan; the host only checks the file sizes against the device's byte
// total.  Round 2 read and checked the two 320 MB tables of 40 M reads on the
// host (≈0.35 s of a 0.72 s load).
int apg_reads_load_dev(apg_ctx* ctx, const char* fastb, const char* qualb, int threads, apg_dreads** out) {
  APG_REQUIRE(ctx && fastb && out, "apg_reads_load_dev: NULL argument");
  *out = nullptr;
  if (ctx->bg_load) dreads_join(ctx->bg_load);  // one load at a time through the staging buffers
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  auto ms = [&](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
  static const char kFb[8] = {'A', 'P', 'G', 'F', 'B', 0, 0, 0}, kQb[8] = {'A', 'P', 'G', 'Q', 'B', 0, 0, 0};
  Head hf, hq;
  APG_TRY(read_head(fastb, kFb, &hf));
  if (qualb) {
    APG_TRY(read_head(qualb, kQb, &hq));
    if (hq.n != hf.n || hq.total != hf.total) {
      set_error(std::string("qualb/fastb length mismatch: ") + qualb);
      return APG_E_IO;
    }
    if (hq.size != 32 + 8 * (hq.n + 1) + hq.total) {
      set_error(std::string("truncated or oversized payload in ") + qualb);
      return APG_E_IO;
    }
  }
  const uint64_t n = hf.n;
  if (threads <= 0) threads = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  apg_dreads* d = nullptr;
  APG_TRY(dreads_alloc(ctx, n, &d));
  auto fail = [&](int rc) {
    apg_reads_free(d);
    return rc;
  };
  // the qualb's offset table only has to equal the fastb's: compared on the
  // host beside the qualities' load (qualb_offsets_match), off the path to
  // the bases
  int rc = stream_to_device(ctx, fastb, 32, 8 * (n + 1), reinterpret_cast<uint8_t*>(d->d_base_off), threads);
  if (rc == APG_OK) {
    rc = dreads_device_shape(ctx, d, nullptr, true, fastb);
    if (rc == APG_E_ARG) rc = APG_E_IO;  // a bad table is a bad file
  }
  if (rc == APG_OK && d->n_bases != hf.total) {
    set_error(std::string("offset table/total mismatch in ") + fastb);
    rc = APG_E_IO;
  }
  if (rc == APG_OK && hf.size != 32 + 8 * (n + 1) + d->n_bytes) {
    set_error(std::string("truncated or oversized payload in ") + fastb);
    rc = APG_E_IO;
  }
  if (rc == APG_OK) rc = dreads_alloc_payload(ctx, d, qualb != nullptr);
  // the packed zero-fill is on ctx->stream: done before the workers write
  if (rc == APG_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) {
    set_error("apg_reads_load_dev: hipStreamSynchronize");
    rc = APG_E_HIP;
  }
  if (rc != APG_OK) return fail(rc);
  const double t_meta = ms(t0);
  // The qualities (4/5 of the bytes) are first read by PreCorrect's
  // candidate scan, after the whole K-mer count: they stream in on a host
  // thread while the caller's next module counts the bases, and every
  // reader of d_quals joins the load first (dreads_quals_ready).
  // APG_LOAD_SYNC=1: loaded before the call returns (the round-4 form).
  // APG_LOAD_EARLY=1: the qualities' thread starts beside the bases' load,
  // on staging workers of its own, instead of after it.
  static const bool sync_load = std::getenv("APG_LOAD_SYNC") && !std::strcmp(std::getenv("APG_LOAD_SYNC"), "1");
  static const bool early = std::getenv("APG_LOAD_EARLY") && !std::strcmp(std::getenv("APG_LOAD_EARLY"), "1");
  auto start_quals = [&](int w0) -> int {
    auto* pend = new (std::nothrow) DreadsPending();
    if (!pend) return APG_E_NOMEM;
    pend->ctx = ctx;
    const std::string qpath(qualb);
    const uint64_t qo = 32 + 8 * (n + 1), qn = d->n_bases;
    uint8_t* qdst = d->d_quals;
    const std::string fpath(fastb);
    pend->th = std::thread([pend, ctx, qpath, fpath, n, qo, qn, qdst, threads, w0]() {
      const auto tq = std::chrono::steady_clock::now();
      pend->rc = stream_to_device(ctx, qpath.c_str(), qo, qn, qdst, threads, w0);
      if (pend->rc == APG_OK) pend->rc = qualb_offsets_match(fpath.c_str(), qpath.c_str(), n);
      if (pend->rc != APG_OK) pend->err = get_error();
      pend->ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tq).count();
    });
    d->pending = pend;
    ctx->bg_load = d;
    return APG_OK;
  };
  const bool bg = qualb && n && !sync_load;
  if (bg && early) {
    rc = staging_get(ctx, 2 * threads);  // workers [threads, 2 threads) for the qualities
    if (rc != APG_OK) return fail(rc);
    rc = start_quals(threads);
    if (rc != APG_OK) return fail(rc);
  }
  const auto t1 = clk::now();
  rc = stream_to_device(ctx, fastb, 32 + 8 * (n + 1), d->n_bytes, d->d_packed, threads);
  const double t_bases = ms(t1);
  const auto t2 = clk::now();
  if (rc == APG_OK && qualb && n) {
    if (sync_load) {
      rc = stream_to_device(ctx, qualb, 32 + 8 * (n + 1), d->n_bases, d->d_quals, threads);
      if (rc == APG_OK) rc = qualb_offsets_match(fastb, qualb, n);
    } else if (!early) {
      rc = start_quals(0);
    }
  }
  vlog(ctx, "load_dev: %llu reads, offsets -> HBM + device checks %.1f ms, bases %.1f ms (%.2f GB/s), quals %.1f ms%s, "
       "%d threads", (unsigned long long)n, t_meta, t_bases, d->n_bytes / std::max(t_bases, 1e-3) / 1e6, ms(t2),
       d->pending ? " (streaming on)" : "", threads);
  if (rc != APG_OK) return fail(rc);
  *out = d;
  return APG_OK;
}

}  // extern "C"
