// sharded.cpp — the sharded (multi-GPU) forms of the module entry points:
// spectrum, PreCorrect / FindErrors, FillFragments and the K=96 unipath
// build over every rank's reads, one process per GPU, every exchange through
// the rank's communicator (exchange.cpp).  Each rank holds whole
// read pairs; K-mers are owned by the shard their minimizer key selects, so
// shards never share a K-mer.
//
//   spectrum     local reads -> 16-byte super-k-mer records by owner shard
//                -> alltoallv -> owner counts its shard -> allreduce of the
//                spectrum and the counters
//   PreCorrect   per pass: records out (their positions stay home) -> owner
//                counts, keeps its solid K-mers and returns each record's
//                weak-K-mer mask (alltoallv back) -> allgatherv of the solid
//                sets -> every rank corrects its own reads through the weak
//                bitmap its masks rebuild (no weak-test lookups) and keeps the
//                pass's extension table + clean flags for FillFragments
//   Fill         pairs are local: no exchange but the counters' sum
//   unipaths     48-byte K=96 super-k-mer records by owner shard -> alltoallv
//                -> owner's distinct nodes (OR of extension bits) -> sharded
//                compaction (ushard_graph.inc: local chain fragments, their
//                ends gathered and stitched; no rank holds every node) ->
//                the graph (same on every rank) + KmerPaths of this rank's
//                reads.  APG_UNIPATH_GATHER_NODES: allgatherv of the node
//                sets and the whole graph built on every rank instead.
// Results equal the single-GPU entry points on the union of the ranks' reads
// (tests/test_distributed.py).
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "apg_core.hpp"
#include "exchange.hpp"
#include "kmer_internal.hpp"

namespace apg {
namespace {

int check_comm(apg_ctx* ctx, apg_comm* comm, Comm** out) {
  Comm* c = comm_of(comm);
  APG_REQUIRE(ctx && c, "apg_sharded: NULL context or communicator");
  APG_REQUIRE(c->ctx == ctx, "apg_sharded: the communicator belongs to another context");
  const int P = c->world;
  APG_REQUIRE(P >= 1 && (P & (P - 1)) == 0 && P <= 32, "apg_sharded: world size must be a power of two <= 32");
  *out = c;
  return APG_OK;
}

// Per-peer byte sizes of B-group count rows (counts[q * B + g] records of
// rec_bytes each).
std::vector<uint64_t> seg_bytes(const std::vector<uint64_t>& counts, int P, int B, uint64_t rec_bytes) {
  std::vector<uint64_t> b(P, 0);
  for (int q = 0; q < P; ++q)
    for (int g = 0; g < B; ++g) b[q] += counts[(size_t)q * B + g] * rec_bytes;
  return b;
}

uint64_t total(const std::vector<uint64_t>& v) { return std::accumulate(v.begin(), v.end(), 0ull); }

// counts -> send (scatter callback) -> records exchanged; returns the receive
// buffer, receive counts and both sides' per-peer byte sizes.
struct Exchanged {
  void* recv = nullptr;
  std::vector<uint64_t> recv_counts, sb, rb;
  uint64_t n_in = 0, n_out = 0;
};

template <typename Scatter>
int exchange_records(apg_ctx* ctx, Comm* c, const std::vector<uint64_t>& counts, int B, uint64_t rec_bytes,
                     const char* send_ws, const char* recv_ws, Scatter scatter, Exchanged* x) {
  const int P = c->world;
  x->sb = seg_bytes(counts, P, B, rec_bytes);
  x->n_in = total(x->sb) / rec_bytes;
  void* send = nullptr;
  APG_TRY(workspace(ctx, send_ws, std::max<uint64_t>(x->n_in * rec_bytes, 64), &send));
  APG_TRY(scatter(send));
  if (P == 1) {  // a single rank receives what it sends: the scatter wrote the receive buffer
    x->recv_counts = counts;
    x->rb = x->sb;
    x->n_out = x->n_in;
    x->recv = send;
    return APG_OK;
  }
  x->recv_counts.assign((size_t)P * B, 0);
  APG_TRY(c->alltoall_u64(counts.data(), x->recv_counts.data(), (uint64_t)B));  // counts[dest * B + g] -> [src * B + g]
  x->rb = seg_bytes(x->recv_counts, P, B, rec_bytes);
  x->n_out = total(x->rb) / rec_bytes;
  APG_TRY(workspace(ctx, recv_ws, std::max<uint64_t>(x->n_out * rec_bytes, 64), &x->recv));
  return c->alltoallv(send, x->sb.data(), x->recv, x->rb.data());
}

// allgatherv of n_local elements of `bytes` each from every rank into ws.
int gather_all(apg_ctx* ctx, Comm* c, const void* local, uint64_t n_local, uint64_t bytes, const char* ws,
               void** out, uint64_t* n_all) {
  if (c->world == 1) {  // the gathered set is this rank's
    // handed back as is only when no memory-pressure release can free it
    // under the caller (the C5 rehearsal's fault was a
    // world-1 solid list in the stage buffer "x_local"); a releasable buffer
    // other than `ws` itself is copied into `ws`
    const char* rel = ws_releasable(ctx, local);
    if (!rel || !std::strcmp(rel, ws)) {
      *out = const_cast<void*>(local);
      *n_all = n_local;
      return APG_OK;
    }
    APG_TRY(workspace(ctx, ws, std::max<uint64_t>(n_local * bytes, 64), out));
    if (n_local)
      APG_CHECK_HIP(hipMemcpyAsync(*out, local, n_local * bytes, hipMemcpyDeviceToDevice, ctx->stream));
    *n_all = n_local;
    return APG_OK;
  }
  std::vector<uint64_t> sizes;
  APG_TRY(c->allgather_u64(n_local, &sizes));
  std::vector<uint64_t> rb(sizes.size());
  for (size_t q = 0; q < sizes.size(); ++q) rb[q] = sizes[q] * bytes;
  *n_all = total(sizes);
  APG_TRY(workspace(ctx, ws, std::max<uint64_t>(*n_all * bytes, 64), out));
  return c->allgatherv(local, n_local * bytes, *out, rb.data());
}

}  // namespace
}  // namespace apg

using namespace apg;

extern "C" {

int apg_sharded_spectrum(apg_ctx* ctx, apg_comm* comm, const apg_dreads* reads, int K, uint64_t* hist,
                         size_t hist_len, apg_kstats* stats) {
  Comm* c = nullptr;
  APG_TRY(check_comm(ctx, comm, &c));
  APG_REQUIRE(reads && hist && hist_len >= 2, "apg_sharded_spectrum: NULL argument or hist_len < 2");
  const int P = c->world, B = apg_shard_bins(K, P);
  APG_REQUIRE(B > 0, "apg_sharded_spectrum: K / world size unsupported (K <= 32, world <= 8)");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  std::vector<uint64_t> counts((size_t)P * B);
  APG_TRY(apg_shard_count(ctx, reads, K, P, counts.data()));
  Exchanged x;
  APG_TRY(exchange_records(ctx, c, counts, B, 16, "x_send", "x_recv",
                           [&](void* send) { return apg_shard_scatter(ctx, reads, K, P, send); }, &x));
  apg_kstats st;
  APG_TRY(apg_shard_spectrum(ctx, x.recv, x.recv_counts.data(), K, P, hist, hist_len, &st));
  APG_TRY(c->allreduce_u64(hist, hist_len, APG_COMM_SUM));
  uint64_t v[4] = {st.n_kmers, st.n_distinct, st.n_overflow, st.n_redo};
  APG_TRY(c->allreduce_u64(v, 4, APG_COMM_SUM));
  uint64_t mb = st.max_bucket;
  APG_TRY(c->allreduce_u64(&mb, 1, APG_COMM_MAX));
  st.n_kmers = v[0];
  st.n_distinct = v[1];
  st.n_overflow = v[2];
  st.n_redo = v[3];
  st.max_bucket = mb;
  if (stats) *stats = st;
  return APG_OK;
}

}  // extern "C"

namespace apg {
namespace {
// apg_sharded_precorrect; with up_hist, the first cycle's owner count also
// yields the K+1 spectrum of the uncorrected reads (the fused
// apg_sharded_spectrum_precorrect: one exchange of K-records instead of two)
int sharded_pc(apg_ctx* ctx, apg_comm* comm, apg_dreads* reads, const apg_pc_params* pp, apg_pc_stats* stats,
               uint64_t* up_hist, size_t up_hist_len, apg_kstats* up_stats) {
  Comm* c = nullptr;
  APG_TRY(check_comm(ctx, comm, &c));
  APG_REQUIRE(reads, "apg_sharded_precorrect: NULL reads");
  apg_pc_params p;
  if (pp)
    p = *pp;
  else
    apg_pc_defaults(&p);
  const int P = c->world, K = p.K, B = apg_shard_bins(K, P);
  APG_REQUIRE(B > 0, "apg_sharded_precorrect: K / world size unsupported (K <= 32, world <= 8)");
  APG_REQUIRE(p.n_cycles >= 1, "apg_sharded_precorrect: n_cycles must be >= 1");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const bool weak = K >= 9 && K <= 29;  // the weak-mask return (apg_shard_solid_weak)
  SkResult up_res;
  bool up_pending = false;
  apg_pc_stats tot;
  std::memset(&tot, 0, sizeof tot);
  // weak mode: records cut to <= 32 bases (sk_pack_split), so the owner's
  // partition levels carry them packed (16 bytes with the receive index)
  const uint32_t split = weak ? sk_pack_split(K) : 0u;
  for (uint32_t cyc = 0; cyc < p.n_cycles; ++cyc) {
    std::vector<uint64_t> counts((size_t)P * B), kc;
    uint64_t n_kmers_in = ~0ull;  // K-mer instances this rank receives (the owner count's sizing)
    if (weak) {
      APG_TRY(sk_count(ctx, reads, K, P, &counts, &kc, split));
      std::vector<uint64_t> kin((size_t)P * B);
      APG_TRY(c->alltoall_u64(kc.data(), kin.data(), (uint64_t)B));
      n_kmers_in = total(kin);
    } else {
      APG_TRY(apg_shard_count(ctx, reads, K, P, counts.data()));
    }
    void* pos = nullptr;
    Exchanged x;
    uint64_t n_local = 0;
    void* smask = nullptr;
    unsigned long long* wbits = nullptr;  // the bitmap the owner count built (all records or the self-owned ones)
    uint64_t self_send = 0, self_n = 0;
    if (weak) {
      APG_TRY(exchange_records(ctx, c, counts, B, 16, "x_send", "x_recv",
                               [&](void* send) {
                                 const uint64_t n = total(seg_bytes(counts, P, B, 1));
                                 APG_TRY(workspace(ctx, "x_pos", std::max<uint64_t>(n * 8, 64), &pos));
                                 return sk_scatter_pos(ctx, reads, K, P, static_cast<SK16*>(send),
                                                       static_cast<uint64_t*>(pos), split);
                               },
                               &x));
      void* rmask = nullptr;
      // P == 1: the owner is this rank and the receive order the send order:
      // the count ORs the weak bits straight into the reads' bitmap at
      // x_pos[receive index] (no masks, no return, no apply pass).  P > 1: the
      // same for the 1/P of the records this rank sent to itself (SkSelf);
      // only the other ranks' records travel back as masks (APG_SHARD_SELF=0:
      // every record's mask travels, the round-4 form)
      static const bool self_on = !(getenv("APG_SHARD_SELF") && !strcmp(getenv("APG_SHARD_SELF"), "0"));
      const bool direct = P == 1 || self_on;
      SkSelf self;
      if (P > 1 && direct) {
        for (int q = 0; q < c->rank; ++q) {
          self.lo += x.rb[q] / 16;
          self.send += x.sb[q] / 16;
        }
        self.n = x.rb[c->rank] / 16;
      }
      if (direct) {
        void* wb = nullptr;
        APG_TRY(workspace(ctx, "pc_weak", (reads->n_bases / 64 + 2) * 8, &wb));
        APG_CHECK_HIP(hipMemsetAsync(wb, 0, (reads->n_bases / 64 + 2) * 8, ctx->stream));
        wbits = static_cast<unsigned long long*>(wb);
      }
      if (P > 1) APG_TRY(workspace(ctx, "x_rmask", std::max<uint64_t>((x.n_out - self.n) * 4, 64), &rmask));
      const uint64_t* wpos = wbits ? static_cast<const uint64_t*>(pos) : nullptr;
      if (up_hist && cyc == 0) {
        // the K+1 pass runs on the side stream beside the mask return, the
        // solid-set gather and the correction below; joined after them
        APG_TRY(shard_solid_weak_fused(ctx, x.recv, x.recv_counts.data(), K, P, p.min_solid, rmask, &n_local, up_hist,
                                       up_hist_len, &up_res, true, n_kmers_in, wbits, wpos, self));
        up_pending = true;
      } else {
        APG_TRY(shard_solid_weak_fused(ctx, x.recv, x.recv_counts.data(), K, P, p.min_solid, rmask, &n_local, nullptr,
                                       0, nullptr, true, n_kmers_in, wbits, wpos, self));
      }
      // masks travel back: the splits reversed, 4 bytes per record (none for
      // the self segment when its bits are in the bitmap already)
      std::vector<uint64_t> mb_out(P), mb_in(P);
      for (int q = 0; q < P; ++q) {
        const bool own = direct && q == c->rank;
        mb_out[q] = own ? 0 : x.rb[q] / 16 * 4;
        mb_in[q] = own ? 0 : x.sb[q] / 16 * 4;
      }
      if (P == 1) {  // the weak bits are in the reads' bitmap already
        smask = nullptr;
      } else {
        APG_TRY(workspace(ctx, "x_smask", std::max<uint64_t>((x.n_in - self.n) * 4, 64), &smask));
        APG_TRY(c->alltoallv(rmask, mb_out.data(), smask, mb_in.data()));
      }
      self_send = self.send;
      self_n = self.n;
    } else {
      APG_TRY(exchange_records(ctx, c, counts, B, 16, "x_send", "x_recv",
                               [&](void* send) { return apg_shard_scatter(ctx, reads, K, P, send); }, &x));
      APG_TRY(apg_shard_solid(ctx, x.recv, x.recv_counts.data(), K, P, p.min_solid, &n_local));
    }
    // at world size 1 the gathered set IS this rank's list (gather_all
    // returns it as is), so it goes straight into "x_solid": the pass's list
    // must survive the release of the counting buffers under memory pressure
    // (ws_make_room frees "x_local" as a stage buffer before the extension
    // table is built — the C5-rank rehearsal faulted on exactly that)
    void* local = nullptr;
    APG_TRY(workspace(ctx, P == 1 ? "x_solid" : "x_local", std::max<uint64_t>(n_local * 8, 64), &local));
    APG_TRY(apg_solid_export(ctx, local));
    // the replicated solid set; it stays in "x_solid" as the pass's list
    // (APG_FILL_LAST_SOLID) until the next sharded pass
    void* solid = nullptr;
    uint64_t n_solid = 0;
    APG_TRY(gather_all(ctx, c, local, n_local, 8, "x_solid", &solid, &n_solid));
    apg_pc_stats st;
    if (wbits && P > 1)
      APG_TRY(precorrect_weak_masks(ctx, reads, p, solid, n_solid, wbits, static_cast<const uint64_t*>(pos),
                                    static_cast<const uint32_t*>(smask), x.n_in, self_send, self_n, &st));
    else if (wbits)
      APG_TRY(precorrect_weak_built(ctx, reads, p, solid, n_solid, wbits, &st));
    else if (weak)
      APG_TRY(apg_precorrect_weak(ctx, reads, &p, solid, n_solid, pos, smask, x.n_in, &st));
    else
      APG_TRY(apg_precorrect_solid(ctx, reads, &p, solid, n_solid, &st));
    tot.n_suspect += st.n_suspect;
    tot.n_corrected += st.n_corrected;
    tot.n_ambiguous += st.n_ambiguous;
    tot.n_uncorrectable += st.n_uncorrectable;
    tot.n_solid = n_solid;
    tot.record_form = st.record_form;
    if (up_pending) {  // the first cycle's K+1 spectrum: side pass complete, summed over ranks
      up_pending = false;
      APG_TRY(side_join(ctx));
      APG_TRY(c->allreduce_u64(up_hist, up_hist_len, APG_COMM_SUM));
      uint64_t v[5] = {up_res.n_kmers, up_res.n_distinct, up_res.nbuckets, up_res.n_overflow_buckets,
                       up_res.n_redo_buckets};
      APG_TRY(c->allreduce_u64(v, 5, APG_COMM_SUM));
      if (up_stats) {
        std::memset(up_stats, 0, sizeof(*up_stats));
        up_stats->n_kmers = v[0];
        up_stats->n_distinct = v[1];
        up_stats->n_buckets = v[2];
        up_stats->n_overflow = v[3];
        up_stats->n_redo = v[4];
      }
    }
  }
  uint64_t v[4] = {tot.n_suspect, tot.n_corrected, tot.n_ambiguous, tot.n_uncorrectable};
  APG_TRY(c->allreduce_u64(v, 4, APG_COMM_SUM));
  tot.n_suspect = v[0];
  tot.n_corrected = v[1];
  tot.n_ambiguous = v[2];
  tot.n_uncorrectable = v[3];
  if (stats) *stats = tot;
  // the replicated list the last cycle corrected against is the global solid
  // set of the corrected reads (a pass leaves it unchanged): recorded for
  // apg_sharded_error_correct_jump
  ctx->pc_shard = ctx->pc_list_valid;
  ctx->pc_shard_comm = comm;
  ctx->pc_shard_gen = reads->gen;
  ctx->pc_shard_list = ctx->pc_list;
  ctx->pc_shard_n = ctx->pc_n;
  ctx->pc_shard_min_solid = p.min_solid;
  return APG_OK;
}

// The global solid set of every rank's reads, replicated on every rank
// ("x_solid"): owner counts of the exchanged records, then all-gathered.
int sharded_solid(apg_ctx* ctx, Comm* c, const apg_dreads* reads, int K, uint32_t min_solid, const uint64_t** solid,
                  uint64_t* n_solid) {
  const int P = c->world, B = apg_shard_bins(K, P);
  APG_REQUIRE(B > 0, "sharded solid set: K / world size unsupported (K <= 32, world <= 8)");
  std::vector<uint64_t> counts((size_t)P * B);
  APG_TRY(apg_shard_count(ctx, reads, K, P, counts.data()));
  Exchanged x;
  APG_TRY(exchange_records(ctx, c, counts, B, 16, "x_send", "x_recv",
                           [&](void* send) { return apg_shard_scatter(ctx, reads, K, P, send); }, &x));
  uint64_t n_local = 0;
  APG_TRY(apg_shard_solid(ctx, x.recv, x.recv_counts.data(), K, P, min_solid, &n_local));
  void* local = nullptr;
  APG_TRY(workspace(ctx, P == 1 ? "x_solid" : "x_local", std::max<uint64_t>(n_local * 8, 64), &local));
  APG_TRY(apg_solid_export(ctx, local));
  void* all = nullptr;
  APG_TRY(gather_all(ctx, c, local, n_local, 8, "x_solid", &all, n_solid));
  *solid = static_cast<const uint64_t*>(all);
  return APG_OK;
}
}  // namespace
}  // namespace apg

extern "C" {

int apg_sharded_precorrect(apg_ctx* ctx, apg_comm* comm, apg_dreads* reads, const apg_pc_params* pp,
                           apg_pc_stats* stats) {
  return sharded_pc(ctx, comm, reads, pp, stats, nullptr, 0, nullptr);
}

int apg_sharded_spectrum_precorrect(apg_ctx* ctx, apg_comm* comm, apg_dreads* reads, int K_spec, uint64_t* hist,
                                    size_t hist_len, apg_kstats* kstats, const apg_pc_params* pp,
                                    apg_pc_stats* pstats) {
  APG_REQUIRE(ctx && reads && hist && hist_len >= 2, "apg_sharded_spectrum_precorrect: NULL argument or hist_len < 2");
  apg_pc_params p;
  if (pp)
    p = *pp;
  else
    apg_pc_defaults(&p);
  if (K_spec != p.K + 1 || p.K < 9 || p.K > 29 || !sk_can_fuse_up(p.K)) {  // not fusable: the two entry points
    APG_TRY(apg_sharded_spectrum(ctx, comm, reads, K_spec, hist, hist_len, kstats));
    return apg_sharded_precorrect(ctx, comm, reads, &p, pstats);
  }
  return sharded_pc(ctx, comm, reads, &p, pstats, hist, hist_len, kstats);
}

int apg_sharded_fill(apg_ctx* ctx, apg_comm* comm, const apg_dreads* pairs, const apg_fill_params* pp,
                     const void* d_solid, uint64_t n_solid, apg_dreads** filled, uint8_t* d_status,
                     apg_fill_stats* stats) {
  Comm* c = nullptr;
  APG_TRY(check_comm(ctx, comm, &c));
  apg_fill_stats st;
  APG_TRY(apg_fill_fragments_dev(ctx, pairs, pp, d_solid, n_solid, filled, d_status, &st));
  uint64_t v[8] = {st.n_pairs, st.n_filled, st.n_none, st.n_ambiguous, st.n_budget, st.n_skip, st.filled_bases,
                   st.lookups};
  APG_TRY(c->allreduce_u64(v, 8, APG_COMM_SUM));
  st.n_pairs = v[0];
  st.n_filled = v[1];
  st.n_none = v[2];
  st.n_ambiguous = v[3];
  st.n_budget = v[4];
  st.n_skip = v[5];
  st.filled_bases = v[6];
  st.lookups = v[7];
  if (stats) *stats = st;
  return APG_OK;
}

int apg_sharded_unipaths(apg_ctx* ctx, apg_comm* comm, const apg_dreads* reads, const apg_unipath_params* pp,
                         apg_unipath_graph* out, apg_unipath_stats* stats) {
  // before anything can fail: the error path below frees *out, which must
  // then hold nothing but what this call allocated
  if (out) std::memset(out, 0, sizeof(*out));
  Comm* c = nullptr;
  APG_TRY(check_comm(ctx, comm, &c));
  APG_REQUIRE(reads, "apg_sharded_unipaths: NULL reads");
  apg_unipath_params p;
  if (pp)
    p = *pp;
  else
    apg_unipath_defaults(&p);
  const int P = c->world, K = p.K;
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  // minimizer-partition records (48-byte super-k-mers) up to 8 shards, else
  // distinct local nodes (32-byte records, 32 / P digit groups per shard)
  const bool rec = P <= 8;
  const int B = rec ? 32 : 32 / P;
  const uint64_t W = rec ? 48 : 32;
  std::vector<uint64_t> counts((size_t)P * B);
  uint64_t n_inst = 0;
  if (rec)
    APG_TRY(apg_urec_count(ctx, reads, K, P, counts.data(), &n_inst));
  else
    APG_TRY(apg_ushard_count(ctx, reads, K, P, counts.data(), &n_inst));
  Exchanged x;
  APG_TRY(exchange_records(ctx, c, counts, B, W, "x_send", "x_recv",
                           [&](void* send) {
                             return rec ? apg_urec_scatter(ctx, reads, K, P, send)
                                        : apg_ushard_scatter(ctx, reads, K, P, send);
                           },
                           &x));
  uint64_t n_local = 0;
  if (rec)
    APG_TRY(apg_urec_nodes(ctx, x.recv, x.recv_counts.data(), K, P, &n_local));
  else
    APG_TRY(apg_ushard_nodes(ctx, x.recv, x.recv_counts.data(), K, P, &n_local));
  // the graph stage's per-node arrays to come (a copy of the nodes, index,
  // directed state, ranking and stitch arrays: ~256 bytes per node measured
  // on the C5-rank rehearsal): the dead record buffers and correction tables
  // go now if they would not fit beside them, instead of on a failed
  // allocation later
  APG_TRY(ws_make_room(ctx, n_local * 256, kRoomCorrection));
  // this rank's nodes outlive the call (the sharded graph's node array, for
  // apg_sharded_unipath_locs): a workspace no other stage writes
  void* local = nullptr;
  APG_TRY(workspace(ctx, "x_unodes", std::max<uint64_t>(n_local * 32, 64), &local));
  if (rec)
    APG_TRY(apg_urec_export(ctx, local));
  else
    APG_TRY(apg_ushard_export(ctx, local));
  apg_unipath_stats st;
  std::memset(&st, 0, sizeof st);
  if (rec && !(p.flags & APG_UNIPATH_GATHER_NODES)) {
    // sharded compaction: local chains, fragment ends gathered and stitched
    const auto& us = ctx->urstate;  // the buckets' links and node index over the same node order
    const int rc = u_sharded_graph(ctx, c, local, n_local, reads, p, out, &st, us.lsucc, us.idx, us.idx_T);
    if (rc != APG_OK) {
      if (out) apg_unipath_graph_free(out);
      return rc;
    }
  } else {
    void* nodes = nullptr;
    uint64_t n_nodes = 0;
    APG_TRY(gather_all(ctx, c, local, n_local, 32, "x_nodes", &nodes, &n_nodes));
    APG_TRY(apg_unipaths_from_nodes(ctx, nodes, n_nodes, reads, &p, out, &st));
  }
  APG_TRY(c->allreduce_u64(&n_inst, 1, APG_COMM_SUM));
  st.n_instances = n_inst;
  if (stats) *stats = st;
  return APG_OK;
}

int apg_sharded_error_correct_jump(apg_ctx* ctx, apg_comm* comm, const apg_dreads* frags, apg_dreads* jumps,
                                   const apg_ecj_params* pp, uint32_t* d_keep_len, apg_ecj_stats* stats) {
  Comm* c = nullptr;
  APG_TRY(check_comm(ctx, comm, &c));
  APG_REQUIRE(frags && jumps, "apg_sharded_error_correct_jump: NULL argument");
  apg_ecj_params e;
  if (pp)
    e = *pp;
  else
    apg_ecj_defaults(&e);
  APG_REQUIRE(e.K >= 2 && e.K <= 29 && e.min_solid >= 1,
              "apg_sharded_error_correct_jump: K must be in [2, 29], min_solid >= 1");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  ctx->ws_dead &= ~kRoomCorrection;  // the fragments' solid set and table are read again
  // the global solid set of the fragment reads: the replicated list of their
  // sharded correction pass over this communicator when it is still the
  // context's list, else counted across the ranks
  const uint64_t* solid = nullptr;
  uint64_t n_solid = 0;
  if (ctx->pc_shard && ctx->pc_list_valid && ctx->pc_shard_comm == comm && ctx->pc_shard_gen == frags->gen &&
      ctx->pc_list == ctx->pc_shard_list && ctx->pc_n == ctx->pc_shard_n && ctx->pc_K == e.K &&
      ctx->pc_shard_min_solid == e.min_solid) {
    solid = ctx->pc_list;
    n_solid = ctx->pc_n;
    vlog(ctx, "sharded error_correct_jump: the fragments' replicated solid set (%llu K-mers)",
         (unsigned long long)n_solid);
  } else {
    APG_TRY(sharded_solid(ctx, c, frags, e.K, e.min_solid, &solid, &n_solid));
  }
  apg_ecj_stats st;
  APG_TRY(ecj_with_solid(ctx, jumps, e, solid, n_solid, d_keep_len, &st));
  uint64_t v[9] = {st.pc.n_suspect, st.pc.n_corrected, st.pc.n_ambiguous, st.pc.n_uncorrectable, st.n_reads,
                   st.n_full, st.n_trimmed, st.n_dropped, st.bases_kept};
  APG_TRY(c->allreduce_u64(v, 9, APG_COMM_SUM));
  st.pc.n_suspect = v[0];
  st.pc.n_corrected = v[1];
  st.pc.n_ambiguous = v[2];
  st.pc.n_uncorrectable = v[3];
  st.pc.n_solid = n_solid;
  st.n_reads = v[4];
  st.n_full = v[5];
  st.n_trimmed = v[6];
  st.n_dropped = v[7];
  st.bases_kept = v[8];
  if (stats) *stats = st;
  return APG_OK;
}

int apg_sharded_unipath_locs(apg_ctx* ctx, apg_comm* comm, const apg_dreads* reads, uint32_t flags,
                             const apg_aln_pair** d_locs, uint64_t* n_locs, apg_uloc_stats* stats) {
  Comm* c = nullptr;
  APG_TRY(check_comm(ctx, comm, &c));
  APG_REQUIRE(reads && d_locs && n_locs, "apg_sharded_unipath_locs: NULL argument");
  *d_locs = nullptr;
  *n_locs = 0;
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  return u_sharded_locs(ctx, c, reads, flags, d_locs, n_locs, stats);
}

}  // extern "C"
