// exchange.hpp — internal interface of libapg's communicators (exchange.cpp).
#pragma once

#include <cstdint>
#include <vector>

#include "../../include/apg.h"

struct apg_ctx;

namespace apg {

// One rank of a sharded run.  Device-memory buffers when ctx is set (the
// stage entry points), host memory otherwise.  Segments of a send / receive
// buffer are contiguous in peer order; sizes are bytes per peer.
struct Comm {
  static constexpr uint64_t kPiece = 1ull << 30;  // largest single transfer (bytes)
  apg_ctx* ctx = nullptr;
  int rank = 0, world = 1;
  virtual ~Comm() = default;
  virtual int alltoallv(const void* send, const uint64_t* send_bytes, void* recv, const uint64_t* recv_bytes) = 0;
  virtual int allgatherv(const void* send, uint64_t bytes, void* recv, const uint64_t* recv_bytes) = 0;
  // in place on host memory (small arrays: spectra, counters)
  virtual int allreduce_u64(uint64_t* data, uint64_t n, int op) = 0;
  // host-memory forms (counts, sizes), whatever the communicator's memory kind
  virtual int alltoallv_host(const void* send, const uint64_t* send_bytes, void* recv, const uint64_t* recv_bytes) = 0;
  virtual int allgatherv_host(const void* send, uint64_t bytes, void* recv, const uint64_t* recv_bytes) = 0;
  virtual int barrier() = 0;
  // in place on a device array of the context (e.g. consensus vote planes): element-wise sum
  virtual int allreduce_dev_u32(uint32_t* d, uint64_t n) = 0;
  // after a local failure: peers blocked on this rank error out (apg_comm_abort)
  virtual void abort() = 0;
  bool aborted = false;
  uint64_t piece_bytes() const;
  // m u64 to every peer (host arrays [peer * m + i])
  int alltoall_u64(const uint64_t* send, uint64_t* recv, uint64_t m);
  int allgather_u64(uint64_t v, std::vector<uint64_t>* all);
};

Comm* comm_of(apg_comm* c);

// Sharded unipath compaction (unipath.hip / ushard_graph.inc): this rank's
// distinct nodes (KRec[n_nodes], its minimizer shard) -> the global graph on
// every rank + KmerPaths of this rank's reads.
// lsucc / idx (may be null): the node buckets' links and node index over
// d_nodes (ctx->urstate after apg_urec_nodes + apg_urec_export).
int u_sharded_graph(apg_ctx* ctx, Comm* c, const void* d_nodes, uint64_t n_nodes, const apg_dreads* reads,
                    const apg_unipath_params& p, apg_unipath_graph* out, apg_unipath_stats* st,
                    const void* lsucc = nullptr, unsigned long long* idx = nullptr, uint64_t idx_T = 0);

// UnipathLocs of this rank's reads on the context's last sharded unipath
// build (unipath.hip / ushard_graph.inc); stats summed over the ranks.
int u_sharded_locs(apg_ctx* ctx, Comm* c, const apg_dreads* reads, uint32_t flags, const apg_aln_pair** d_locs,
                   uint64_t* n_locs, apg_uloc_stats* st);

}  // namespace apg
