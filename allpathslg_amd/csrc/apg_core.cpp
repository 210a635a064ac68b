// apg_core.cpp — context lifecycle, errors, workspaces, kernel timing, uploads.
#include "apg_core.hpp"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <new>
#include <thread>

namespace apg {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
const char* get_error() { return g_err.c_str(); }

static int ws_release_list(apg_ctx* ctx, const char* const* names, size_t n, uint64_t* freed,
                           const char* keep = nullptr);
static const char* const kCorrectWs[] = {"pc_ext", "fill_ext", "ecj_ext", "fill_solid", "x_solid", "pc_solid"};

// An allocation that fails while the correction stage's tables are dead
// (ctx->ws_dead, set by the unipath stage): they are released and the
// allocation retried once.  ws_make_room's estimate before the unipath stage
// counts its records, not its node tables and graph arrays, which at a
// C5-rank's 0.4 G nodes need ~180 GB (the rehearsal ran out of memory there
// holding 112 GB of dead correction tables).
static int release_dead_for(apg_ctx* ctx, const char* name) {
  if (!(ctx->ws_dead & kRoomCorrection)) return 0;
  uint64_t freed = 0;
  if (ws_release_list(ctx, kCorrectWs, sizeof kCorrectWs / sizeof kCorrectWs[0], &freed, name) != APG_OK) return 0;
  ctx->ws_dead &= ~kRoomCorrection;
  ctx->pc_ext_valid = false;
  ctx->pc_list_valid = false;
  ctx->solid_valid = false;
  ++ctx->mem_releases;
  vlog(ctx, "memory: %.2f GB of dead correction tables released after a failed allocation of '%s'", freed / 1e9,
       name);
  return freed > 0;
}

int workspace(apg_ctx* ctx, const char* name, size_t bytes, void** out) {
  auto& b = ctx->ws[name];
  if (b.bytes < bytes) {
    if (b.p && ctx->side_finish) APG_TRY(side_join(ctx));  // the side work may read it
    if (b.p) APG_CHECK_HIP(hipFree(b.p));
    ctx->ws_bytes -= b.bytes;
    b.p = nullptr;
    b.bytes = 0;
    // Grow by 1/8 headroom so steadily growing calls do not realloc each time.
    size_t want = bytes + bytes / 8;
    // APG_DEVICE_MEM_LIMIT with APG_DEVICE_MEM_HARD=1 (tests): an allocation
    // past the emulated device fails as a real one would, so the
    // failed-allocation release runs on a small input
    static const uint64_t hard = getenv("APG_DEVICE_MEM_HARD") && getenv("APG_DEVICE_MEM_LIMIT")
                                     ? strtoull(getenv("APG_DEVICE_MEM_LIMIT"), nullptr, 10)
                                     : 0;
    auto alloc = [&](size_t n) -> hipError_t {
      if (hard && ctx->ws_bytes + n > hard) return hipErrorOutOfMemory;
      return hipMalloc(&b.p, n);
    };
    hipError_t e = alloc(want);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      want = bytes;
      e = alloc(want);
    }
    if (e != hipSuccess) {
      (void)hipGetLastError();
      if (release_dead_for(ctx, name)) e = alloc(want);
    }
    if (e != hipSuccess) {
      b.p = nullptr;
      set_error(std::string("hipMalloc(") + std::to_string(bytes) + ") for workspace '" + name +
                "' failed: " + hipGetErrorString(e));
      return APG_E_HIP;
    }
    b.bytes = want;
    ctx->ws_bytes += want;
    ctx->ws_peak = std::max(ctx->ws_peak, ctx->ws_bytes);
    if (ctx->verbose) {
      size_t tot = 0;
      for (auto& kv : ctx->ws) tot += kv.second.bytes;
      vlog(ctx, "workspace %s -> %.3f GB (all workspaces %.3f GB)", name, want / 1e9, tot / 1e9);
    }
  }
  *out = b.p;
  return APG_OK;
}

// Memory pressure (C5-scale inputs, DESIGN.md §7 "Memory model"): the
// counting stages' record and partition buffers are dead once a count has
// produced its spectrum, solid list and weak bitmap, but as grow-only named
// workspaces they would stay allocated under the tables the next stage
// builds.  When the device lacks `need` bytes (plus a 2 GiB margin) they are
// released; the next count allocates them again.  Releasing a table some
// later call may reuse (the extension table, the solid list) invalidates that
// reuse.  Nothing is freed while memory suffices (the single-GPU bench never
// releases).
static const char* const kStageWs[] = {"big0",    "big1",    "big2",    "x_send",  "x_recv",  "x_pos",  "x_rmask",
                                       "x_smask", "x_local", "sk_gtab", "sk_cmat", "sk_omat",
                                       "sk_solid_sparse", "sk_dcount", "ext_e0", "ext_e1", "sk_ovf_e0", "sk_ovf_e1"};
// record descriptors of a count pass: live from the count to its scatter
static const char* const kDescWs[] = {"sk_desc", "usk_desc"};
// The name of the releasable workspace (a stage buffer, a descriptor buffer
// or a correction table: the lists above) whose allocation holds p, or null.
const char* ws_releasable(apg_ctx* ctx, const void* p) {
  if (!p) return nullptr;
  const char* const* lists[] = {kStageWs, kDescWs, kCorrectWs};
  const size_t lens[] = {sizeof kStageWs / sizeof kStageWs[0], sizeof kDescWs / sizeof kDescWs[0],
                         sizeof kCorrectWs / sizeof kCorrectWs[0]};
  for (int l = 0; l < 3; ++l)
    for (size_t i = 0; i < lens[l]; ++i) {
      auto it = ctx->ws.find(lists[l][i]);
      if (it == ctx->ws.end() || !it->second.p) continue;
      const char* b = static_cast<const char*>(it->second.p);
      if (static_cast<const char*>(p) >= b && static_cast<const char*>(p) < b + it->second.bytes) return lists[l][i];
    }
  return nullptr;
}

// APG_DEVICE_MEM_LIMIT=<bytes>: act as if the device held only that much for
// this context's workspaces (tests of the release path on a 288 GB device).
uint64_t device_free_bytes(apg_ctx* ctx) {
  size_t fr = 0, tot = 0;
  if (hipMemGetInfo(&fr, &tot) != hipSuccess) {
    (void)hipGetLastError();
    fr = ~(size_t)0;
  }
  static const uint64_t limit = getenv("APG_DEVICE_MEM_LIMIT") ? strtoull(getenv("APG_DEVICE_MEM_LIMIT"), nullptr, 10) : 0;
  if (limit) {
    uint64_t used = 0;
    for (auto& kv : ctx->ws) used += kv.second.bytes;
    const uint64_t emu = used >= limit ? 0 : limit - used;
    if (emu < fr) fr = emu;
  }
  return fr;
}

static int ws_release_list(apg_ctx* ctx, const char* const* names, size_t n, uint64_t* freed, const char* keep) {
  APG_TRY(side_join(ctx));
  // every stream of the context: a release may be asked for from the
  // auxiliary stream (StreamSwap) while the main stream's kernels read the
  // buffers (hipFree does not wait for them)
  APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->home && ctx->home != ctx->stream) APG_CHECK_HIP(hipStreamSynchronize(ctx->home));
  if (ctx->aux && ctx->aux != ctx->stream) APG_CHECK_HIP(hipStreamSynchronize(ctx->aux));
  if (ctx->side) APG_CHECK_HIP(hipStreamSynchronize(ctx->side));
  for (size_t i = 0; i < n; ++i) {
    if (keep && !std::strcmp(keep, names[i])) continue;  // the caller holds a reference to it
    auto it = ctx->ws.find(names[i]);
    if (it == ctx->ws.end() || !it->second.p) continue;
    *freed += it->second.bytes;
    ctx->ws_bytes -= it->second.bytes;
    APG_CHECK_HIP(hipFree(it->second.p));
    ctx->ws.erase(it);
  }
  return APG_OK;
}

int ws_make_room(apg_ctx* ctx, uint64_t need, unsigned what) {
  const uint64_t margin = 2ull << 30;
  if (device_free_bytes(ctx) >= need + margin) return APG_OK;
  uint64_t freed = 0;
  APG_TRY(ws_release_list(ctx, kStageWs, sizeof kStageWs / sizeof kStageWs[0], &freed));
  if (what & kRoomDescriptors) {
    APG_TRY(ws_release_list(ctx, kDescWs, sizeof kDescWs / sizeof kDescWs[0], &freed));
    ctx->skstate.desc = false;  // a scatter of the last count must walk again
    ctx->urstate.desc = false;
  }
  if ((what & kRoomCorrection) && device_free_bytes(ctx) < need + margin) {
    APG_TRY(ws_release_list(ctx, kCorrectWs, sizeof kCorrectWs / sizeof kCorrectWs[0], &freed));
    ctx->pc_ext_valid = false;  // FillFragments / ErrorCorrectJump rebuild their tables
    ctx->pc_list_valid = false;
    ctx->solid_valid = false;
  }
  ++ctx->mem_releases;
  vlog(ctx, "memory: %.2f GB of dead stage buffers released for a %.2f GB allocation", freed / 1e9, need / 1e9);
  return APG_OK;
}

// After a unipath build the graph stage's temporaries (record buffers,
// overflow node tables, ranking and stitch arrays) are dead: only what the
// graph state (and the sharded build's urstate) points at is read again —
// by UnipathLocs, apg_unibases_dev, consensus.  Under memory pressure they
// are released before such a call allocates: every "u_" / "g_" / "usk" /
// "big" workspace that holds none of those pointers (descriptor buffers
// stay, for a scatter replay).  A C5-rank's placement stage: ~90 GB.
int ws_release_graph_temps(apg_ctx* ctx, uint64_t need) {
  const uint64_t margin = 2ull << 30;
  if (device_free_bytes(ctx) >= need + margin) return APG_OK;
  const auto& g = ctx->gstate;
  const auto& u = ctx->urstate;
  const void* keep[] = {g.nodes, g.idx, g.head, g.rank, g.uoh, g.ulen, g.urc, g.ub_off, g.ub, g.uloc, g.vu, g.vr,
                        u.lsucc, u.idx};
  auto holds = [&](const apg_ctx::Buf& w) {
    const char* b = static_cast<const char*>(w.p);
    for (const void* k : keep)
      if (k && static_cast<const char*>(k) >= b && static_cast<const char*>(k) < b + w.bytes) return true;
    return false;
  };
  APG_TRY(side_join(ctx));
  APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  if (ctx->aux && ctx->aux != ctx->stream) APG_CHECK_HIP(hipStreamSynchronize(ctx->aux));
  if (ctx->side) APG_CHECK_HIP(hipStreamSynchronize(ctx->side));
  uint64_t freed = 0;
  for (auto it = ctx->ws.begin(); it != ctx->ws.end();) {
    const std::string& n = it->first;
    const bool graph = !n.compare(0, 2, "u_") || !n.compare(0, 2, "g_") || !n.compare(0, 3, "usk") ||
                       !n.compare(0, 3, "big");
    if (!graph || n.find("desc") != std::string::npos || !it->second.p || holds(it->second)) {
      ++it;
      continue;
    }
    freed += it->second.bytes;
    ctx->ws_bytes -= it->second.bytes;
    APG_CHECK_HIP(hipFree(it->second.p));
    it = ctx->ws.erase(it);
  }
  // plans whose buffers may be gone: made again on their next use
  ctx->urstate.valid = false;
  ctx->urstate.desc = false;
  ctx->urstate.lsucc = nullptr;
  ctx->urstate.idx = nullptr;
  ctx->ustate.valid = false;
  ctx->ustate.local_ready = false;
  ++ctx->mem_releases;
  vlog(ctx, "memory: %.2f GB of dead graph-stage workspaces released for a %.2f GB allocation", freed / 1e9,
       need / 1e9);
  return APG_OK;
}

int staging_get(apg_ctx* ctx, int workers) {
  auto& S = ctx->staging;
  while (S.workers < workers) {
    uint8_t* b[2] = {nullptr, nullptr};
    hipStream_t st = nullptr;
    hipEvent_t ev[2] = {nullptr, nullptr};
    APG_CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&b[0]), kStageChunk, 0));
    APG_CHECK_HIP(hipHostMalloc(reinterpret_cast<void**>(&b[1]), kStageChunk, 0));
    APG_CHECK_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    APG_CHECK_HIP(hipEventCreateWithFlags(&ev[0], hipEventDisableTiming));
    APG_CHECK_HIP(hipEventCreateWithFlags(&ev[1], hipEventDisableTiming));
    S.buf.push_back(b[0]);
    S.buf.push_back(b[1]);
    S.st.push_back(st);
    S.ev.push_back(ev[0]);
    S.ev.push_back(ev[1]);
    ++S.workers;
  }
  return APG_OK;
}

static void staging_free(apg_ctx* ctx) {
  auto& S = ctx->staging;
  for (auto* b : S.buf) (void)hipHostFree(b);
  for (auto s : S.st) (void)hipStreamDestroy(s);
  for (auto e : S.ev) (void)hipEventDestroy(e);
  S = apg_ctx::Staging{};
}

int d2h_bulk(apg_ctx* ctx, const std::vector<D2HJob>& jobs, int workers) {
  if (ctx->bg_load) dreads_join(ctx->bg_load);  // it holds the staging buffers
  struct Chunk {
    uint8_t* dst;
    const uint8_t* src;
    uint64_t n;
  };
  std::vector<Chunk> ch;
  for (const auto& j : jobs)
    for (uint64_t o = 0; o < j.bytes; o += kStageChunk)
      ch.push_back(Chunk{static_cast<uint8_t*>(j.dst) + o, static_cast<const uint8_t*>(j.src) + o,
                         std::min<uint64_t>(kStageChunk, j.bytes - o)});
  if (ch.empty()) return APG_OK;
  // small copies: straight (a worker thread costs more than they do)
  if (ch.size() == 1 && ch[0].n < (1u << 20)) {
    APG_CHECK_HIP(hipMemcpy(ch[0].dst, ch[0].src, ch[0].n, hipMemcpyDeviceToHost));
    return APG_OK;
  }
  if (const char* e = std::getenv("APG_D2H_WORKERS"))
    if (std::atoi(e) > 0) workers = std::atoi(e);
  const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)workers, ch.size()));
  APG_TRY(staging_get(ctx, T));
  std::atomic<uint64_t> next{0};
  std::atomic<int> err{0};
  const int dev = ctx->device;
  auto worker = [&](int w) {
    if (hipSetDevice(dev) != hipSuccess) {
      err = 1;
      return;
    }
    uint8_t* buf[2] = {ctx->staging.buf[2 * w], ctx->staging.buf[2 * w + 1]};
    hipEvent_t ev[2] = {ctx->staging.ev[2 * w], ctx->staging.ev[2 * w + 1]};
    hipStream_t st = ctx->staging.st[w];
    const Chunk* pend[2] = {nullptr, nullptr};
    int k = 0;
    auto drain = [&](int b) {
      if (!pend[b]) return;
      if (hipEventSynchronize(ev[b]) != hipSuccess) err = 1;
      std::memcpy(pend[b]->dst, buf[b], pend[b]->n);  // also first-touches the destination pages, in parallel
      pend[b] = nullptr;
    };
    for (uint64_t c; (c = next.fetch_add(1)) < ch.size() && !err.load(); k ^= 1) {
      drain(k);
      if (hipMemcpyAsync(buf[k], ch[c].src, ch[c].n, hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipEventRecord(ev[k], st) != hipSuccess) {
        err = 1;
        break;
      }
      pend[k] = &ch[c];
    }
    drain(k);
    drain(k ^ 1);
  };
  std::vector<std::thread> ts;
  for (int w = 0; w < T; ++w) ts.emplace_back(worker, w);
  for (auto& t : ts) t.join();
  if (err.load()) {
    set_error("device-to-host copy through the staging buffers failed");
    return APG_E_HIP;
  }
  return APG_OK;
}

static hipEvent_t take_event(apg_ctx* ctx) {
  if (!ctx->event_pool.empty()) {
    hipEvent_t e = ctx->event_pool.back();
    ctx->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  (void)hipEventCreate(&e);
  return e;
}

void kbegin(apg_ctx* ctx, const char* name, uint64_t bytes) {
  if (!ctx->timing) return;
  apg_ctx::Pending p;
  p.name = name;
  p.bytes = bytes;
  p.a = take_event(ctx);
  p.b = take_event(ctx);
  p.closed = false;
  p.s = ctx->stream;
  p.overlapped = ctx->stream != ctx->home;
  (void)hipEventRecord(p.a, ctx->stream);
  ctx->pending.push_back(p);
}

void kend(apg_ctx* ctx) {
  if (!ctx->timing) return;
  for (auto it = ctx->pending.rbegin(); it != ctx->pending.rend(); ++it)
    if (!it->closed) {  // innermost open bracket
      (void)hipEventRecord(it->b, ctx->stream);
      it->closed = true;
      return;
    }
}

void kbytes_add(apg_ctx* ctx, const char* name, uint64_t bytes) {
  if (!ctx->timing) return;
  auto it = ctx->kstats.find(name);
  if (it != ctx->kstats.end()) it->second.bytes += bytes;
}

int kflush(apg_ctx* ctx) {
  std::vector<apg_ctx::Pending> open;
  for (auto& p : ctx->pending) {
    // still bracketing work, or another stream's still running: a later flush
    bool later = !p.closed;
    if (!later && p.s != ctx->stream && hipEventQuery(p.b) != hipSuccess) {
      (void)hipGetLastError();  // hipErrorNotReady is not an error here
      later = true;
    }
    if (later) {
      open.push_back(p);
      continue;
    }
    float ms = 0;
    APG_CHECK_HIP(hipEventSynchronize(p.b));
    APG_CHECK_HIP(hipEventElapsedTime(&ms, p.a, p.b));
    auto it = ctx->kstats.find(p.name);
    if (it == ctx->kstats.end()) {
      ctx->korder.push_back(p.name);
      it = ctx->kstats.emplace(p.name, KernelStat{}).first;
    }
    it->second.ms += ms;
    it->second.launches += 1;
    it->second.bytes += p.bytes;
    it->second.overlapped += p.overlapped ? 1 : 0;
    ctx->event_pool.push_back(p.a);
    ctx->event_pool.push_back(p.b);
  }
  ctx->pending.swap(open);
  return APG_OK;
}

int sync(apg_ctx* ctx) {
  APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  APG_CHECK_HIP(hipGetLastError());
  return kflush(ctx);
}

int d2h_sync(apg_ctx* ctx, void* dst, const void* src, size_t bytes) {
  static const bool pageable = getenv("APG_D2H_PAGEABLE") && !strcmp(getenv("APG_D2H_PAGEABLE"), "1");  // A/B
  if (!pageable && bytes && bytes <= kPinBytes && !ctx->pin &&
      hipHostMalloc(&ctx->pin, kPinBytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    ctx->pin = nullptr;
  }
  if (!pageable && ctx->pin && bytes <= kPinBytes) {
    if (bytes) APG_CHECK_HIP(hipMemcpyAsync(ctx->pin, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    APG_TRY(sync(ctx));
    if (bytes) std::memcpy(dst, ctx->pin, bytes);
    return APG_OK;
  }
  if (bytes) APG_CHECK_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  return sync(ctx);
}

int side_kick(apg_ctx* ctx, int stage) {
  if (!ctx->side_kick || (stage >= 0 && stage != ctx->side_kick_at)) return APG_OK;
  std::function<int()> k;
  k.swap(ctx->side_kick);
  return k();
}

int side_join(apg_ctx* ctx) {
  APG_TRY(side_kick(ctx, -1));  // a pass still waiting for its kick runs now
  if (!ctx->side_finish) return APG_OK;
  std::function<int()> f;
  f.swap(ctx->side_finish);  // cleared first: the finish may allocate workspaces
  return f();
}

// APG_{MAIN,SIDE,AUX}_PRIO=high|low: that stream's queue priority (A/B knob;
// unset = normal).  The CP prefers a high-priority queue's workgroups when
// kernels of several streams wait for CUs.
static hipError_t make_stream(hipStream_t* s, const char* env) {
  const char* e = getenv(env);
  if (e && (!strcmp(e, "high") || !strcmp(e, "low"))) {
    int least = 0, greatest = 0;
    if (hipDeviceGetStreamPriorityRange(&least, &greatest) == hipSuccess)
      return hipStreamCreateWithPriority(s, hipStreamNonBlocking, !strcmp(e, "high") ? greatest : least);
    (void)hipGetLastError();
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}
static hipStream_t lazy_stream(hipStream_t* s, const char* env) {
  if (!*s && make_stream(s, env) != hipSuccess) {
    (void)hipGetLastError();
    *s = nullptr;
  }
  return *s;
}
hipStream_t side_stream(apg_ctx* ctx) { return lazy_stream(&ctx->side, "APG_SIDE_PRIO"); }
hipStream_t aux_stream(apg_ctx* ctx) { return lazy_stream(&ctx->aux, "APG_AUX_PRIO"); }

}  // namespace apg

using namespace apg;

extern "C" {

int apg_abi_version(void) { return APG_ABI_VERSION; }
const char* apg_last_error(void) { return get_error(); }

int apg_create(const apg_config* cfg, apg_ctx** out) {
  APG_REQUIRE(out != nullptr, "apg_create: out is NULL");
  *out = nullptr;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0) {
    set_error(std::string("apg_create: no HIP device available (") +
              (e != hipSuccess ? hipGetErrorString(e) : "0 devices") + ")");
    return APG_E_HIP;
  }
  const int dev = cfg ? cfg->device : 0;
  APG_REQUIRE(dev >= 0 && dev < ndev, "apg_create: device ordinal out of range");
  APG_CHECK_HIP(hipSetDevice(dev));
  apg_ctx* ctx = new (std::nothrow) apg_ctx();
  if (!ctx) return APG_E_NOMEM;
  ctx->device = dev;
  ctx->timing = cfg && cfg->timing;
  ctx->verbose = cfg && cfg->verbose;
  ctx->kmer_dedup = cfg ? cfg->kmer_dedup : 0;
  if (ctx->kmer_dedup < 0 || ctx->kmer_dedup > 2) {
    delete ctx;
    set_error("apg_create: kmer_dedup must be 0, 1 or 2");
    return APG_E_ARG;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess) ctx->n_cu = prop.multiProcessorCount;
  if (ctx->n_cu <= 0) ctx->n_cu = 256;
  if (make_stream(&ctx->stream, "APG_MAIN_PRIO") != hipSuccess) {
    delete ctx;
    set_error("apg_create: hipStreamCreate failed");
    return APG_E_HIP;
  }
  ctx->home = ctx->stream;
  *out = ctx;
  return APG_OK;
}

int apg_trim(apg_ctx* ctx) {
  APG_REQUIRE(ctx, "apg_trim: ctx is NULL");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  if (ctx->bg_load) dreads_join(ctx->bg_load);
  APG_TRY(side_join(ctx));
  APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  for (auto& kv : ctx->ws)
    if (kv.second.p) (void)hipFree(kv.second.p);
  ctx->ws.clear();
  ctx->ws_bytes = 0;
  ctx->pc_list_valid = false;
  ctx->pc_ext_valid = false;
  ctx->clean_valid = false;
  ctx->solid_valid = false;
  ctx->gstate.valid = false;
  return APG_OK;
}

void apg_destroy(apg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->device);
  if (ctx->bg_load) dreads_join(ctx->bg_load);
  (void)side_join(ctx);
  if (ctx->side) (void)hipStreamSynchronize(ctx->side);
  if (ctx->aux) (void)hipStreamSynchronize(ctx->aux);
  (void)hipStreamSynchronize(ctx->stream);
  for (auto& kv : ctx->ws)
    if (kv.second.p) (void)hipFree(kv.second.p);
  for (auto& p : ctx->pending) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  for (auto e : ctx->event_pool) (void)hipEventDestroy(e);
  staging_free(ctx);
  if (ctx->pin) (void)hipHostFree(ctx->pin);
  ctx->pin = nullptr;
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  if (ctx->aux) (void)hipStreamDestroy(ctx->aux);
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
}

int apg_timing_get(apg_ctx* ctx, int idx, char* name, size_t name_len, double* total_ms,
                   uint64_t* launches, uint64_t* bytes) {
  APG_REQUIRE(ctx, "apg_timing_get: ctx is NULL");
  APG_TRY(kflush(ctx));
  if (idx < 0 || idx >= (int)ctx->korder.size()) return APG_E_ARG;
  const std::string& n = ctx->korder[idx];
  const KernelStat& s = ctx->kstats[n];
  if (name && name_len) {
    std::strncpy(name, n.c_str(), name_len - 1);
    name[name_len - 1] = 0;
  }
  if (total_ms) *total_ms = s.ms;
  if (launches) *launches = s.launches;
  if (bytes) *bytes = s.bytes;
  return APG_OK;
}

int apg_mem_stats_get(apg_ctx* ctx, int reset_peak, apg_mem_stats* out) {
  APG_REQUIRE(ctx && out, "apg_mem_stats_get: NULL argument");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  std::memset(out, 0, sizeof *out);
  out->workspace_bytes = ctx->ws_bytes;
  out->workspace_peak = ctx->ws_peak;
  out->releases = ctx->mem_releases;
  size_t fr = 0, tot = 0;
  APG_CHECK_HIP(hipMemGetInfo(&fr, &tot));
  out->device_used = tot - fr;
  out->device_total = tot;
  if (reset_peak) ctx->ws_peak = ctx->ws_bytes;
  return APG_OK;
}

int apg_timing_overlapped(apg_ctx* ctx, int idx, uint64_t* overlapped) {
  APG_REQUIRE(ctx, "apg_timing_overlapped: ctx is NULL");
  APG_TRY(kflush(ctx));
  if (idx < 0 || idx >= (int)ctx->korder.size()) return APG_E_ARG;
  if (overlapped) *overlapped = ctx->kstats[ctx->korder[idx]].overlapped;
  return APG_OK;
}

int apg_timing_reset(apg_ctx* ctx) {
  APG_REQUIRE(ctx, "apg_timing_reset: ctx is NULL");
  APG_TRY(kflush(ctx));
  ctx->korder.clear();
  ctx->kstats.clear();
  return APG_OK;
}

int apg_byte_offsets(const uint64_t* base_off, uint64_t n_reads, uint64_t* byte_off) {
  APG_REQUIRE(base_off && byte_off, "apg_byte_offsets: NULL pointer");
  byte_off[0] = 0;
  for (uint64_t i = 0; i < n_reads; ++i) {
    APG_REQUIRE(base_off[i + 1] >= base_off[i], "apg_byte_offsets: base_off not monotone");
    byte_off[i + 1] = byte_off[i] + (base_off[i + 1] - base_off[i] + 3) / 4;
  }
  return APG_OK;
}

}  // extern "C"

namespace apg {
// A device read set with room for its offset tables (n + 1 each); the shape
// fields are filled by dreads_device_shape (readset.hip) once the tables are
// on the device.
int dreads_alloc(apg_ctx* ctx, uint64_t n, apg_dreads** out) {
  *out = nullptr;
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  auto* d = new (std::nothrow) apg_dreads();
  if (!d) return APG_E_NOMEM;
  d->ctx = ctx;
  d->device = ctx->device;
  static std::atomic<uint64_t> g_gen{1};
  d->gen = g_gen.fetch_add(1);
  d->n_reads = n;
  hipError_t e;
  if ((e = hipMalloc(&d->d_base_off, (n + 1) * 8)) != hipSuccess || (e = hipMalloc(&d->d_byte_off, (n + 1) * 8)) != hipSuccess) {
    set_error(std::string("read set: ") + hipGetErrorString(e));
    apg_reads_free(d);
    return APG_E_HIP;
  }
  *out = d;
  return APG_OK;
}

// Payload buffers of a read set whose shape is known: packed bases zeroed, +64
// bytes of slack (kernels may issue aligned 4/16-byte loads past the end),
// qualities if asked.
int dreads_alloc_payload(apg_ctx* ctx, apg_dreads* d, bool with_quals) {
  hipError_t e;
  if ((e = hipMalloc(&d->d_packed, d->n_bytes + 64)) != hipSuccess ||
      (e = hipMemsetAsync(d->d_packed, 0, d->n_bytes + 64, ctx->stream)) != hipSuccess ||
      (with_quals && d->n_reads && (e = hipMalloc(&d->d_quals, d->n_bases + 64)) != hipSuccess)) {
    set_error(std::string("read set: ") + hipGetErrorString(e));
    return APG_E_HIP;
  }
  return APG_OK;
}

// Host offset tables -> a device read set with its offsets uploaded, its
// shape checked on the device and its payload buffers allocated (packed
// zeroed): the caller fills packed / quals on the context's stream.
int dreads_create(apg_ctx* ctx, uint64_t n, const uint64_t* base_off, const uint64_t* byte_off, bool with_quals,
                  apg_dreads** out) {
  *out = nullptr;
  apg_dreads* d = nullptr;
  APG_TRY(dreads_alloc(ctx, n, &d));
  auto fail = [&](int rc) {
    apg_reads_free(d);
    return rc;
  };
  hipError_t e;
  const uint64_t z = 0;
  if ((e = hipMemcpyAsync(d->d_base_off, n ? base_off : &z, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess ||
      (e = hipMemcpyAsync(d->d_byte_off, n ? byte_off : &z, (n + 1) * 8, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess) {
    set_error(std::string("read set: ") + hipGetErrorString(e));
    return fail(APG_E_HIP);
  }
  int rc = dreads_device_shape(ctx, d, nullptr, false, "read set");  // syncs: &z may be released after
  if (rc == APG_OK) rc = dreads_alloc_payload(ctx, d, with_quals);
  if (rc != APG_OK) return fail(rc);
  *out = d;
  return APG_OK;
}
}  // namespace apg

extern "C" {

int apg_reads_upload(apg_ctx* ctx, const apg_reads* r, apg_dreads** out) {
  APG_REQUIRE(ctx && r && out, "apg_reads_upload: NULL argument");
  APG_REQUIRE(r->n_reads == 0 || (r->base_off && r->byte_off && r->packed),
              "apg_reads_upload: missing base_off/byte_off/packed");
  APG_REQUIRE(r->n_reads == 0 || (r->base_off[0] == 0 && r->byte_off[0] == 0),
              "apg_reads_upload: base_off[0] and byte_off[0] must be 0");
  *out = nullptr;
  const uint64_t n = r->n_reads;
  apg_dreads* d = nullptr;
  APG_TRY(dreads_create(ctx, n, r->base_off, r->byte_off, r->quals != nullptr, &d));
  auto fail = [&](hipError_t e) {
    set_error(std::string("apg_reads_upload: ") + hipGetErrorString(e));
    apg_reads_free(d);
    return APG_E_HIP;
  };
  hipError_t e;
  if (n && (e = hipMemcpyAsync(d->d_packed, r->packed, d->n_bytes, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess)
    return fail(e);
  if (r->quals && n &&
      (e = hipMemcpyAsync(d->d_quals, r->quals, d->n_bases, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess)
    return fail(e);
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return fail(e);
  *out = d;
  return APG_OK;
}

void apg_reads_free(apg_dreads* d) {
  if (!d) return;
  dreads_join(d);  // no load may still write into it
  (void)hipSetDevice(d->device);
  if (d->d_base_off) (void)hipFree(d->d_base_off);
  if (d->d_byte_off) (void)hipFree(d->d_byte_off);
  if (d->d_packed) (void)hipFree(d->d_packed);
  if (d->d_quals) (void)hipFree(d->d_quals);
  delete d;
}

uint64_t apg_dreads_count(const apg_dreads* d) { return d ? d->n_reads : 0; }

int apg_dreads_shape(apg_ctx* ctx, const apg_dreads* d, uint64_t* n_reads, uint64_t* n_bases, uint64_t* n_bytes,
                     uint64_t* base_off, uint64_t* byte_off) {
  APG_REQUIRE(ctx && d, "apg_dreads_shape: NULL argument");
  if (n_reads) *n_reads = d->n_reads;
  if (n_bases) *n_bases = d->n_bases;
  if (n_bytes) *n_bytes = d->n_bytes;
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  if (base_off)
    APG_CHECK_HIP(hipMemcpyAsync(base_off, d->d_base_off, (d->n_reads + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (byte_off)
    APG_CHECK_HIP(hipMemcpyAsync(byte_off, d->d_byte_off, (d->n_reads + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  return APG_OK;
}

int apg_reads_copy_dev(apg_ctx* ctx, apg_dreads* dst, const apg_dreads* src) {
  APG_REQUIRE(ctx && dst && src, "apg_reads_copy_dev: NULL argument");
  // Shape identity: the sets' length hashes (an element-wise compare of two
  // 40 M-entry offset vectors cost 13 ms of host time per bench step); a set
  // produced on the device (fill, concat, unibases) gets its hash computed
  // here, once.
  for (apg_dreads* x : {dst, const_cast<apg_dreads*>(src)})
    if (!x->shape_hash) {
      const uint64_t nb = x->n_bases, ny = x->n_bytes, ml = x->max_len;
      APG_TRY(dreads_device_shape(ctx, x, nullptr, false, "apg_reads_copy_dev"));
      APG_REQUIRE(x->n_bases == nb && x->n_bytes == ny && x->max_len == ml,
                  "apg_reads_copy_dev: device read set shape inconsistent (internal error)");
    }
  const bool same = dst->shape_hash == src->shape_hash;
  APG_REQUIRE(dst->n_reads == src->n_reads && dst->n_bases == src->n_bases && dst->n_bytes == src->n_bytes && same,
              "apg_reads_copy_dev: read sets differ in shape");
  APG_REQUIRE(!src->d_quals || dst->d_quals, "apg_reads_copy_dev: destination has no qualities");
  APG_TRY(dreads_quals_ready(src));
  dreads_join(dst);  // its own load's outcome is overwritten below when src has qualities
  if (!src->d_quals) APG_TRY(dreads_quals_ready(dst));
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  if (src->n_bytes)
    APG_CHECK_HIP(hipMemcpyAsync(dst->d_packed, src->d_packed, src->n_bytes, hipMemcpyDeviceToDevice, ctx->stream));
  if (src->d_quals && src->n_bases)
    APG_CHECK_HIP(hipMemcpyAsync(dst->d_quals, src->d_quals, src->n_bases, hipMemcpyDeviceToDevice, ctx->stream));
  if (src->d_quals) {  // dst's qualities are src's now
    dst->quals_rc = APG_OK;
    dst->quals_err.clear();
  }
  dst->gen = src->gen;  // same bases: plans made for src are valid for dst's contents
  return APG_OK;
}

int apg_device_copy(apg_ctx* ctx, void* d_dst, const void* d_src, uint64_t bytes) {
  APG_REQUIRE(ctx, "apg_device_copy: NULL ctx");
  if (!bytes) return APG_OK;
  APG_REQUIRE(d_dst && d_src, "apg_device_copy: NULL pointer");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  APG_CHECK_HIP(hipMemcpyAsync(d_dst, d_src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  return APG_OK;
}

int apg_device_alloc(apg_ctx* ctx, uint64_t bytes, void** d_out) {
  APG_REQUIRE(ctx && d_out, "apg_device_alloc: NULL argument");
  *d_out = nullptr;
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  void* p = nullptr;
  APG_CHECK_HIP(hipMalloc(&p, std::max<uint64_t>(bytes, 1)));
  const hipError_t e = hipMemsetAsync(p, 0, std::max<uint64_t>(bytes, 1), ctx->stream);
  if (e == hipSuccess && hipStreamSynchronize(ctx->stream) == hipSuccess) {
    *d_out = p;
    return APG_OK;
  }
  (void)hipFree(p);
  set_error("apg_device_alloc: zero fill failed");
  return APG_E_HIP;
}

void apg_device_free(apg_ctx* ctx, void* d) {
  if (!d) return;
  if (ctx) (void)hipSetDevice(ctx->device);
  (void)hipFree(d);
}

int apg_device_to_host(apg_ctx* ctx, void* h_dst, const void* d_src, uint64_t bytes) {
  APG_REQUIRE(ctx, "apg_device_to_host: NULL ctx");
  if (!bytes) return APG_OK;
  APG_REQUIRE(h_dst && d_src, "apg_device_to_host: NULL pointer");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  APG_CHECK_HIP(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, ctx->stream));
  APG_CHECK_HIP(hipStreamSynchronize(ctx->stream));
  return APG_OK;
}

void apg_free(void* p) { std::free(p); }

}  // extern "C"
