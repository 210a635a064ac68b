// kmer_internal.hpp — counting-pipeline internals shared by the modules built
// on the counted k-mer table (PreCorrect / FindErrors).
#pragma once

#include <cstdint>
#include <vector>

#include "apg_core.hpp"

namespace apg {

// Counting modes of the hash-record pipeline: spectrum only, or the full
// table (every distinct hash + count, in hash order; apg_kmer_count).
constexpr int kCountSpectrum = 0, kCountTable = 1;

// Result of the counting pipeline (device pointers into ctx workspaces; valid
// until the next counting call on the same context).
struct CountResult {
  uint64_t* rec = nullptr;        // final records; in table mode rec[boff[b] + i] = i-th distinct hash of bucket b
  uint32_t* tab_cnt = nullptr;    // table mode: count of rec[...] (same index)
  uint32_t* bucket_nd = nullptr;  // table mode: distinct hashes per bucket
  uint64_t* boff = nullptr;       // bucket offsets (nbuckets + 1)
  uint64_t nbuckets = 0;
  uint64_t n_records = 0;
  apg_kstats st{};
};

// Count canonical K-mers (K <= 32) of a device read set.  table = true also
// materialises the sparse (hash, count) table described in CountResult.
int spectrum_impl(apg_ctx* ctx, const apg_dreads* dr, int K, int mode, uint64_t* hist, size_t hist_len,
                  CountResult* res);

// Minimizer-partitioned counting (superkmer.hip), K <= 32.
struct SK16;
// (SkResult: apg_core.hpp, the context holds a pending one)
int sk_count(apg_ctx* ctx, const apg_dreads* dr, int K, int P, std::vector<uint64_t>* rec_counts,
             std::vector<uint64_t>* kmer_counts, uint32_t split = 0);
int sk_scatter(apg_ctx* ctx, const apg_dreads* dr, int K, int P, SK16* out);
// sk_scatter + pos[i] = global base position of record i's first K-mer;
// split > 0: records cut into pieces of <= split K-mers (sk_count with the
// same split first), so that every record fits the packed form (<= 32 bases)
int sk_scatter_pos(apg_ctx* ctx, const apg_dreads* dr, int K, int P, SK16* out, uint64_t* pos, uint32_t split = 0);
// the piece length that keeps a K-mer's records within the packed form
uint32_t sk_pack_split(int K);
// The records a multi-GPU owner received from its own rank (P > 1): receive
// indices [lo, lo + n), sent at send indices [send, send + n).  Their weak
// bits go straight into the reads' bitmap at wpos[send + (b - lo)] (no mask
// for them in the return exchange); the other records' masks are written to
// wrec packed without the self segment (index b, or b - n past it).
struct SkSelf {
  uint64_t lo = 0, n = 0, send = 0;
};
// solid set of received records + per-record weak masks (receive order).
// split_recs: the records were cut by sk_pack_split (<= 32 bases), so the
// owner's partition levels may carry them packed (16 bytes, the receive
// index in the position field) instead of as 24-byte records.  weak + wpos
// (the owner is the reads' own rank): the weak bits ORed straight into the
// per-base bitmap `weak` at wpos[receive index] + t, wrec unused.
int sk_shard_solid_weak(apg_ctx* ctx, const SK16* recv, const std::vector<uint64_t>& rec_counts, uint64_t n_kmers,
                        int K, int P, uint32_t min_solid, uint32_t* wrec, SkResult* res,
                        int up_K = 0, uint64_t* up_hist = nullptr, size_t up_hist_len = 0,
                        SkResult* up_res = nullptr, bool split_recs = false, unsigned long long* weak = nullptr,
                        const uint64_t* wpos = nullptr, SkSelf self = SkSelf{});
bool sk_can_fuse_up(int K);
// Owner side of the sharded fused spectrum + PreCorrect (precorrect.hip): as
// apg_shard_solid_weak, plus this shard's K+1 spectrum (up_hist) from the
// same records (on the side stream: side_join before reading up_hist).
int shard_solid_weak_fused(apg_ctx* ctx, const void* d_recv, const uint64_t* recv_counts, int K, int n_shards,
                           uint32_t min_solid, void* d_mask, uint64_t* n_solid, uint64_t* up_hist, size_t up_hist_len,
                           SkResult* up_res, bool split_recs = false, uint64_t n_kmers = ~0ull,
                           unsigned long long* weak = nullptr, const uint64_t* wpos = nullptr,
                           SkSelf self = SkSelf{});
// apg_spectrum_precorrect_dev; join = false leaves the fused K+1 pass on the
// side stream (its stats land at up_kstats_fill after the caller's side_join)
int spectrum_precorrect_impl(apg_ctx* ctx, apg_dreads* dr, int K_spec, uint64_t* hist, size_t hist_len,
                             apg_kstats* kstats, const apg_pc_params* pp, apg_pc_stats* pstats, bool join);
int up_kstats_fill(apg_ctx* ctx);
// ErrorCorrectJump's correction pass and trim of the jump reads against a
// given solid list of the fragment reads (precorrect.hip)
int ecj_with_solid(apg_ctx* ctx, apg_dreads* jr, const apg_ecj_params& e, const uint64_t* solid, uint64_t n_solid,
                   uint32_t* d_keep, apg_ecj_stats* st);
// PreCorrect's correction pass over reads whose weak bitmap ("pc_weak") the
// owner count already built (sk_shard_solid_weak with weak + wpos)
int precorrect_weak_built(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params& p, const void* d_solid,
                          uint64_t n_solid, unsigned long long* weak, apg_pc_stats* st);
// The same when the owner count built the self-owned records' bits (SkSelf)
// and the returned masks of the other n_in - n_self sent records are still to
// be ORed in: mask[0, self_send) for pos[0, self_send), mask[self_send, ...)
// for pos[self_send + n_self, n_in)
int precorrect_weak_masks(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params& p, const void* d_solid,
                          uint64_t n_solid, unsigned long long* weak, const uint64_t* pos, const uint32_t* mask,
                          uint64_t n_in, uint64_t self_send, uint64_t n_self, apg_pc_stats* st);
int sk_stage_count(apg_ctx* ctx, const SK16* src, SK16* spare, const std::vector<uint64_t>& rec_counts,
                   uint64_t n_kmers, int K, int P, bool solid, uint32_t min_solid, uint64_t* hist, size_t hist_len,
                   SkResult* res);
int sk_spectrum(apg_ctx* ctx, const apg_dreads* dr, int K, bool solid, uint32_t min_solid, uint64_t* hist,
                size_t hist_len, SkResult* res);
// up_res != null: also the K+1 spectrum of the same reads from the K records
// (sk_can_fuse_up(K)), into up_hist (host, may be null) and up_res
int sk_solid_weak(apg_ctx* ctx, const apg_dreads* dr, int K, uint32_t min_solid, unsigned long long* weak,
                  SkResult* res, uint64_t* up_hist = nullptr, size_t up_hist_len = 0, SkResult* up_res = nullptr);
bool sk_can_fuse_up(int K);
uint64_t sk_sum_kmers(apg_ctx* ctx, const SK16* recs, uint64_t n, int* rc);
constexpr int kSkShardBins = 32;  // per-shard digit groups of the exchange (2^kSkDigitBits)

}  // namespace apg
