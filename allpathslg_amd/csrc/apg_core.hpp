// apg_core.hpp — internal context, error and workspace plumbing of libapg.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <functional>
#include <map>
#include <string>
#include <vector>

#include "../../include/apg.h"

namespace apg {

// Thread-local last-error message behind apg_last_error().
void set_error(const std::string& msg);
// apg_core.cpp: a device read set with offsets uploaded and payload buffers
// allocated, for the caller to fill on ctx->stream.
int dreads_create(apg_ctx* ctx, uint64_t n, const uint64_t* base_off, const uint64_t* byte_off, bool with_quals,
                  apg_dreads** out);
// apg_core.cpp: room for the offset tables only / the payload of a set whose
// shape is known.
int dreads_alloc(apg_ctx* ctx, uint64_t n, apg_dreads** out);
int dreads_alloc_payload(apg_ctx* ctx, apg_dreads* d, bool with_quals);
// readset.hip: validate the device offset tables of d (byte_off derived from
// base_off when compute_bytes; d_qoff, if given, must equal base_off) and
// fill n_bases, n_bytes, max_len, shape_hash.  Synchronous.
int dreads_device_shape(apg_ctx* ctx, apg_dreads* d, const uint64_t* d_qoff, bool compute_bytes, const char* who);
const char* get_error();

struct Status {
  int code;
};

#define APG_CHECK_HIP(expr)                                                       \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      ::apg::set_error(std::string(#expr " failed: ") + hipGetErrorString(_e) +   \
                       " (" __FILE__ ":" + std::to_string(__LINE__) + ")");     \
      return APG_E_HIP;                                                           \
    }                                                                             \
  } while (0)

#define APG_TRY(expr)            \
  do {                           \
    int _rc = (expr);            \
    if (_rc != APG_OK) return _rc; \
  } while (0)

#define APG_REQUIRE(cond, msg)              \
  do {                                      \
    if (!(cond)) {                          \
      ::apg::set_error(std::string(msg));   \
      return APG_E_ARG;                     \
    }                                       \
  } while (0)

struct KernelStat {
  double ms = 0;
  uint64_t launches = 0;
  uint64_t bytes = 0;
  uint64_t overlapped = 0;  // launches on the side / auxiliary stream (beside the main stream's kernels)
};

}  // namespace apg

namespace apg {
// A read set's qualities still streaming in from a .qualb file
// (apg_reads_load_dev): the host thread that loads them, and its outcome.
struct DreadsPending;
// Result of a minimizer-partitioned count (superkmer.hip; device pointers
// into ctx workspaces, valid until the next counting call on the context).
struct SkResult {
  uint64_t* solid = nullptr;  // solid mode: hashes with count >= min_solid ("pc_solid" workspace)
  uint64_t n_solid = 0;
  uint64_t n_distinct = 0;
  uint64_t n_overflow_buckets = 0;  // buckets counted by the global-table fallback
  uint64_t n_redo_buckets = 0;      // buckets the record-dedup kernel handed back to k_sk_bucket
  uint64_t nbuckets = 0;
  uint64_t n_kmers = 0;
  uint64_t n_records = 0;
};
}  // namespace apg

// Device-resident read set.
struct apg_dreads {
  apg_ctx* ctx = nullptr;  // producing context: identity only, never dereferenced (it may be destroyed first)
  int device = 0;          // device ordinal of the buffers (apg_reads_free needs no live context)
  uint64_t gen = 0;  // unique per upload (cache key for per-read-set plans)
  uint64_t n_reads = 0;
  uint64_t n_bases = 0;
  uint64_t n_bytes = 0;
  uint64_t max_len = 0;
  uint64_t* d_base_off = nullptr;  // n+1
  uint64_t* d_byte_off = nullptr;  // n+1
  uint8_t* d_packed = nullptr;
  uint8_t* d_quals = nullptr;      // optional
  uint64_t shape_hash = 0;  // hash of the read lengths and byte strides (dreads_device_shape; 0 = not yet known)
  // device-produced sets (apg_fill_fragments_dev): buffer capacities, reused
  // when the same object is passed back in
  bool fill_owned = false;
  bool concat_owned = false;  // apg_reads_concat_dev output
  uint64_t cap_reads = 0, cap_bytes = 0, cap_quals = 0;
  // qualities still loading in the background (apg_reads_load_dev): every
  // reader of d_quals calls apg::dreads_quals_ready first
  apg::DreadsPending* pending = nullptr;
  // the background load's outcome, kept once joined: every later reader of
  // the qualities gets the same error
  int quals_rc = 0;
  std::string quals_err;
};

struct apg_ctx {
  int device = 0;
  bool timing = false;
  bool verbose = false;
  int kmer_dedup = 0;  // apg_config.kmer_dedup
  hipStream_t stream = nullptr;
  hipStream_t home = nullptr;  // the main stream (ctx->stream while no StreamSwap is active)
  int n_cu = 0;
  // Side stream: work that runs beside the main stream inside one module call
  // (the fused K+1 spectrum pass beside PreCorrect's correction kernels).
  // side_finish completes it (host syncs of the side stream, outputs); it is
  // run by apg::side_join before the call returns, and before any workspace
  // is freed or grown.
  hipStream_t side = nullptr;
  std::function<int()> side_finish;
  // a side launch deferred to a later point of the same call (side_kick_at:
  // the caller's stage number that kicks it); side_join kicks it first
  std::function<int()> side_kick;
  int side_kick_at = 0;
  // the stage a fused K+1 pass is kicked at when APG_SK_UP_AT is not set
  // (1; apg_spectrum_precorrect_fill_dev: APG_SK_UP_AT_FILL's or its own)
  int side_kick_default = 1;
  // apg_spectrum_precorrect_dev's K+1 count result, written by the side
  // pass's finish; kstats filled from it once joined (spectrum_precorrect_impl)
  apg::SkResult up_res_pending;
  apg_kstats* up_kstats = nullptr;
  // Auxiliary stream: a producer that overlaps the main stream's next
  // kernels and is joined by an event wait (PreCorrect's extension table
  // built beside its candidate scan).
  hipStream_t aux = nullptr;
  // Pinned host scratch for the small device-to-host reads between kernels
  // (d2h_sync): a pageable destination costs ~27 us per round trip against
  // ~16 us pinned (tools/microbench/d2h_latency.hip).
  void* pin = nullptr;

  // Grow-only named device workspaces.
  struct Buf {
    void* p = nullptr;
    size_t bytes = 0;
  };
  std::map<std::string, Buf> ws;
  // the read set whose qualities a background load is streaming through this
  // context's staging buffers (apg_load.cpp); any other staging user joins it
  apg_dreads* bg_load = nullptr;

  // Per-kernel timing.
  std::vector<std::string> korder;
  std::map<std::string, apg::KernelStat> kstats;
  struct Pending {
    std::string name;
    hipEvent_t a, b;
    uint64_t bytes;
    bool closed;
    hipStream_t s;  // the stream the events bracket (kflush resolves only ctx->stream's)
    bool overlapped;  // s is not the main stream
  };
  std::vector<Pending> pending;
  std::vector<hipEvent_t> event_pool;

  // Stage-A plan of the last extract_count (reused by extract_scatter).
  struct XState {
    bool valid = false;
    uint64_t gen = 0;
    int K = 0, P = 0, dshift = 0;
    uint32_t G = 0, ndig = 0;
    uint64_t total = 0;
  } xstate;

  // Unipath-stage plan of the last apg_ushard_count / apg_ushard_nodes.
  struct UState {
    bool valid = false;
    uint64_t gen = 0;
    int K = 0;
    uint32_t G = 0;
    uint64_t n = 0;        // instances extracted
    uint64_t n_local = 0;  // distinct local nodes of the last apg_ushard_count
    bool local_ready = false;  // "u_nodes" holds those local nodes
    uint64_t n_nodes = 0;  // nodes of the last apg_ushard_nodes
    uint64_t n_recv = 0;
  } ustate;

  // K <= 96 super-k-mer plan of the last usk_plan (reused by usk_scatter).
  struct UrState {
    bool valid = false;
    uint64_t gen = 0;
    int K = 0, P = 0;
    uint32_t G = 0;
    uint64_t n = 0;  // records
    uint64_t n_nodes = 0;  // nodes of the last apg_urec_nodes ("usk_nodes")
    bool desc = false;  // the count pass kept record descriptors ("usk_desc*")
    // what the last apg_urec_nodes' buckets built beside the nodes, for the
    // sharded graph over the exported (same-order) node array: each node's
    // bucket-resolved links ("usk_lsucc", uint2 per node; null: none) and the
    // node index ("u_idx" of idx_T slots; null: none)
    const void* lsucc = nullptr;
    unsigned long long* idx = nullptr;
    uint64_t idx_T = 0;
  } urstate;

  // Super-k-mer plan of the last sk_count (reused by sk_scatter).
  struct SkState {
    bool valid = false;
    uint64_t gen = 0;
    int K = 0, P = 0;
    uint32_t G = 0;
    uint64_t total = 0;
    bool desc = false;  // the count pass kept record descriptors ("sk_desc*")
    uint32_t split = 0;  // records counted as pieces of <= split K-mers (SkP::split)
  } skstate;

  // Device graph of the last unipath build ("u_*" workspaces + the node
  // array it indexed), for apg_unipath_locs / apg_unibases_dev.
  struct GState {
    bool valid = false;
    int K = 0;
    uint64_t n_nodes = 0, n_unipaths = 0, tmask = 0;
    const void* nodes = nullptr;  // KRec[n_nodes]
    const unsigned long long* idx = nullptr;  // node index (unipath.hip NodeIdx)
    const uint32_t *head = nullptr, *rank = nullptr, *uoh = nullptr;
    const uint64_t *ulen = nullptr, *urc = nullptr, *ub_off = nullptr;
    const uint8_t* ub = nullptr;  // unibases, one base per byte
    const uint64_t* uloc = nullptr;  // apg_unipath_locs' (unipath, rank) table of this graph, once built
    // sharded compaction (apg_sharded_unipaths): nodes / idx / n_nodes are this
    // rank's shard only; vu / vr give each local directed node its (unipath,
    // rank); unipath arrays and unibases are the replicated global ones
    bool sharded = false;
    const uint32_t *vu = nullptr, *vr = nullptr;
    const void* comm = nullptr;  // the communicator of the sharded build (identity only)
    int n_shards = 1;
  } gstate;

  // Solid K-mer list of the last apg_shard_solid ("pc_solid" workspace).
  uint64_t n_solid = 0;
  bool solid_valid = false;

  // Solid list the last correction pass corrected against ("pc_solid", or
  // the caller's gathered list in the sharded flow); APG_FILL_LAST_SOLID.
  const uint64_t* pc_list = nullptr;
  uint64_t pc_n = 0;
  int pc_K = 0;
  bool pc_list_valid = false;
  // pc_self: pc_list was counted (min_solid pc_min_solid) from the very reads
  // that pass corrected, whose generation after the pass is pc_self_gen.  A
  // pass leaves its reads' solid set unchanged (a suspect's covering K-mers
  // are all weak, an accepted alternative's all solid, and accepted
  // corrections lie >= K apart: removed instances are of weak K-mers, added
  // ones of solid K-mers), so pc_list IS the corrected reads' solid set —
  // ErrorCorrectJump's fragment count reuses it (ecj_run).
  bool pc_self = false;
  uint64_t pc_self_gen = 0;
  uint32_t pc_min_solid = 0;
  // the list and size pc_self was recorded for (any later install of another
  // list — apg_solid_upload, a sharded pass — no longer matches)
  const uint64_t* pc_self_list = nullptr;
  uint64_t pc_self_n = 0;
  // pc_shard: pc_list is the replicated solid set a sharded correction pass
  // over `pc_shard_comm` gathered — the global solid set of every rank's
  // corrected reads; this rank's part of them has generation pc_shard_gen
  // (apg_sharded_error_correct_jump reuses it, as ecj_run does pc_self)
  bool pc_shard = false;
  const void* pc_shard_comm = nullptr;
  uint64_t pc_shard_gen = 0;
  const uint64_t* pc_shard_list = nullptr;
  uint64_t pc_shard_n = 0;
  uint32_t pc_shard_min_solid = 0;
  // Per-read clean flags of that pass (1: every K-mer solid after correction,
  // 0: not, 2: not derived), valid for the read set while its gen is clean_gen.
  const uint8_t* pc_clean = nullptr;
  // (K-1)-mer extension table of pc_list (ext_table.hpp; "pc_ext" workspace),
  // built by the pass when 2 <= K <= 29: FillFragments reuses it.
  unsigned long long* pc_ext_slot = nullptr;
  uint64_t pc_ext_mask = 0;
  bool pc_ext_valid = false;
  uint64_t clean_gen = 0;
  bool clean_valid = false;
  // record form of the last solid-set count (apg_pc_stats.record_form)
  uint64_t sk_record_form = 0;
  // Capacity for the next single-pass candidate write (last count + 25 %).
  uint64_t pc_cand_hint = 0;
  uint64_t pc_cand_hint_lk = 0;  // the same for the passes without a weak bitmap (every low-quality position)
  // ws_make_room calls that released buffers (memory pressure; logged with
  // cfg.verbose)
  uint64_t mem_releases = 0;
  // bytes held by the workspaces now, and the most held at once since the
  // context was made or apg_mem_stats_get reset it
  uint64_t ws_bytes = 0, ws_peak = 0;
  // workspace classes the running stage no longer needs (kRoomCorrection: the
  // unipath stage runs after the correction stage's last reader): a
  // workspace allocation that fails releases them and retries (apg_core.cpp)
  unsigned ws_dead = 0;
  // Host <-> device staging of the module boundary (apg_reads_load_dev,
  // graph egress): per worker two pinned chunks, a stream and two events,
  // allocated once per context (pinning 256 MB per call cost more than the
  // copies it staged).
  struct Staging {
    int workers = 0;
    std::vector<uint8_t*> buf;  // 2 per worker, kStageChunk bytes each
    std::vector<hipStream_t> st;
    std::vector<hipEvent_t> ev;  // 2 per worker
  } staging;
};

namespace apg {

// The large record buffers are shared by name across modules, so a context
// holds max(module sizes) instead of their sum (spectrum: 8-byte records,
// unipaths: 32-byte records).  Nothing in them outlives the call that fills
// them, except a CountResult, which is consumed before the next module runs:
//   kBig0: spectrum stage-A records / count ping-pong B; unipath extraction /
//          partition ping-pong B
//   kBig1: spectrum / unipath partition ping-pong A
//   kBig2: spectrum table-mode counts
constexpr const char* kBig0 = "big0";
constexpr const char* kBig1 = "big1";
constexpr const char* kBig2 = "big2";

// Grid of a grid-stride kernel over `work` items: exactly the blocks that
// are resident at once (CUs x the kernel's occupancy), so every block gets
// the same share and no second, partial round of blocks trails the first.
template <typename Kern>
inline uint32_t resident_grid(apg_ctx* ctx, Kern kernel, int threads, uint64_t work) {
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, threads, 0) != hipSuccess || per_cu < 1)
    per_cu = 1;
  const uint64_t g = (uint64_t)ctx->n_cu * (uint64_t)per_cu;
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(work, g));
}

// Grid of a grid-stride kernel over n items, `per` items per block, capped at
// 16 blocks per CU.
inline uint32_t grid_for(apg_ctx* ctx, uint64_t n, int per = 256) {
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + per - 1) / per, (uint64_t)ctx->n_cu * 16));
}

// Device workspace `name` of at least `bytes`; contents are undefined.
int workspace(apg_ctx* ctx, const char* name, size_t bytes, void** out);
template <typename T>
int workspace_t(apg_ctx* ctx, const char* name, size_t count, T** out) {
  void* p = nullptr;
  int rc = workspace(ctx, name, count * sizeof(T) + 16, &p);
  *out = static_cast<T*>(p);
  return rc;
}

// Module-boundary copies through the context's pinned staging (apg_core.cpp):
// chunks of kStageChunk bytes spread over `workers` host threads, each
// double-buffering its copies on its own stream.
constexpr uint64_t kStageChunk = 16ull << 20;
int staging_get(apg_ctx* ctx, int workers);
struct D2HJob {
  void* dst;        // host (pageable)
  const void* src;  // device
  uint64_t bytes;
};
// Device arrays -> host arrays (the device data must be complete: call after a
// sync of ctx->stream).  Synchronous.
int d2h_bulk(apg_ctx* ctx, const std::vector<D2HJob>& jobs, int workers = 4);

// Wait for a background load of the read set's qualities (apg_reads_load_dev)
// to land in HBM; APG_OK at once when none is running.  Every reader of
// d_quals calls it first (apg_load.cpp).
int dreads_quals_ready(const apg_dreads* dr);
// Joins a background load without taking on its error (context-level joins:
// another load, a bulk D2H, trim, destroy); the set's readers still get it.
void dreads_join(const apg_dreads* dr);

// Free device memory (hipMemGetInfo; ~0 if unknown).
uint64_t device_free_bytes(apg_ctx* ctx);
// Name of the workspace ws_make_room / a failed allocation may release that
// holds device pointer p (nullptr: none does).
const char* ws_releasable(apg_ctx* ctx, const void* p);
// Under memory pressure (device free < need + 2 GiB): the last unipath
// build's dead temporaries released (everything but what the graph state
// points at); placement / consensus call it before they allocate.
int ws_release_graph_temps(apg_ctx* ctx, uint64_t need);
// Before a large allocation of `need` bytes: when the device lacks it, release
// the counting stages' dead record / partition workspaces, plus (flags) the
// count passes' record descriptors (dead once scattered) and the correction
// stage's extension tables / solid lists (dead once FillFragments ran) —
// apg_core.cpp.
constexpr unsigned kRoomDescriptors = 1, kRoomCorrection = 2;
int ws_make_room(apg_ctx* ctx, uint64_t need, unsigned what = 0);

// Bracket a launch with timing events when ctx->timing.
void kbegin(apg_ctx* ctx, const char* name, uint64_t bytes);
void kend(apg_ctx* ctx);
// Add algorithmic bytes to a timed kernel known only after it ran (e.g. 64 B
// per random touch counted by the kernel itself); call after a sync.
void kbytes_add(apg_ctx* ctx, const char* name, uint64_t bytes);
// Resolve pending events into kstats (call after a stream sync).
int kflush(apg_ctx* ctx);
int sync(apg_ctx* ctx);
// Copy `bytes` from device `src` to host `dst` on ctx->stream and sync(ctx),
// through the context's pinned scratch when it fits (kPinBytes).
constexpr size_t kPinBytes = 1u << 20;
int d2h_sync(apg_ctx* ctx, void* dst, const void* src, size_t bytes);
// Complete the side-stream work, if any (runs ctx->side_finish once).
int side_join(apg_ctx* ctx);
// Launch a deferred side-stream pass whose kick point is `stage`.
int side_kick(apg_ctx* ctx, int stage);
// The side / auxiliary stream (created on first use); 0 on failure.
hipStream_t side_stream(apg_ctx* ctx);
hipStream_t aux_stream(apg_ctx* ctx);
// Launches between construction and destruction go to `s` (kbegin / kend /
// sync included).
struct StreamSwap {
  apg_ctx* ctx;
  hipStream_t saved;
  StreamSwap(apg_ctx* c, hipStream_t s) : ctx(c), saved(c->stream) { c->stream = s; }
  ~StreamSwap() { ctx->stream = saved; }
};

inline void vlog(apg_ctx* ctx, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

}  // namespace apg

#include <cstdarg>
inline void apg::vlog(apg_ctx* ctx, const char* fmt, ...) {
  if (!ctx || !ctx->verbose) return;
  va_list ap;
  va_start(ap, fmt);
  std::fputs("[apg] ", stderr);
  std::vfprintf(stderr, fmt, ap);
  std::fputc('\n', stderr);
  va_end(ap);
}
