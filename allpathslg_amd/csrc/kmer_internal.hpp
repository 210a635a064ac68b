// kmer_internal.hpp — counting-pipeline internals shared by the modules built
// on the counted k-mer table (PreCorrect / FindErrors).
#pragma once

#include <cstdint>

#include "apg_core.hpp"

namespace apg {

// Counting modes: spectrum only; full table (every distinct hash + count, in
// hash order); solid (only hashes with count >= min_solid, + count,
// unordered — buckets counted by the global fallback still list every
// distinct hash, so consumers filter on the count).
constexpr int kCountSpectrum = 0, kCountTable = 1, kCountSolid = 2;

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
int spectrum_impl(apg_ctx* ctx, const apg_dreads* dr, int K, int mode, uint32_t min_solid, uint64_t* hist,
                  size_t hist_len, CountResult* res);

// Table-mode count of records received by shard `P`-way exchange
// (apg_shard_scatter layout, recv_counts[src * B1 + l1]).
int shard_table_impl(apg_ctx* ctx, const uint64_t* d_recv, const uint64_t* recv_counts, int K, int P, int mode,
                     uint32_t min_solid, CountResult* res);

}  // namespace apg
