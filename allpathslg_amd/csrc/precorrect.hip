// precorrect.hip — k-mer-spectrum read correction (PreCorrect / FindErrors)
// on MI355X.  Spec: SURVEY §A.4 as restated in include/apg.h (semantics
// unpinned: reference snapshot empty); CPU restatement in
// oracle/precorrect_oracle.c.
//
//   1. count canonical K-mers (the spectrum pipeline in table mode)
//   2. k_solid_insert: every distinct hash with count >= min_solid goes into
//      a global open-addressing table (linear probing, load <= 0.5; hashes
//      are already uniformly mixed, so the slot is the hash's low bits)
//   3. k_precorrect: one thread per read walks its positions left to right,
//      probing the table only around low-quality bases (lazy solidity), and
//      edits bases/quals in place.
#include <algorithm>
#include <atomic>
#include <cstring>
#include <vector>

#include "apg_core.hpp"
#include "kmer_common.hpp"
#include "kmer_internal.hpp"

namespace apg {

constexpr uint64_t kSolidEmpty = ~0ull;

__global__ void k_count_solid(const uint32_t* __restrict__ tab_cnt, const uint64_t* __restrict__ boff,
                              const uint32_t* __restrict__ bucket_nd, uint64_t nbuckets, uint32_t min_solid,
                              unsigned long long* __restrict__ n_solid) {
  unsigned long long local = 0;
  for (uint64_t b = blockIdx.x; b < nbuckets; b += gridDim.x) {
    const uint64_t off = boff[b];
    const uint32_t nd = bucket_nd[b];
    for (uint32_t i = threadIdx.x; i < nd; i += blockDim.x) local += tab_cnt[off + i] >= min_solid;
  }
  for (int o = 32; o > 0; o >>= 1) local += __shfl_down(local, o, 64);
  if ((threadIdx.x & 63) == 0 && local) atomicAdd(n_solid, local);
}

__global__ void k_solid_insert(const uint64_t* __restrict__ tab_hash, const uint32_t* __restrict__ tab_cnt,
                               const uint64_t* __restrict__ boff, const uint32_t* __restrict__ bucket_nd,
                               uint64_t nbuckets, uint32_t min_solid, unsigned long long* __restrict__ table,
                               uint64_t tmask) {
  for (uint64_t b = blockIdx.x; b < nbuckets; b += gridDim.x) {
    const uint64_t off = boff[b];
    const uint32_t nd = bucket_nd[b];
    for (uint32_t i = threadIdx.x; i < nd; i += blockDim.x) {
      if (tab_cnt[off + i] < min_solid) continue;
      const unsigned long long h = tab_hash[off + i];
      uint64_t s = h & tmask;
      while (atomicCAS(&table[s], (unsigned long long)kSolidEmpty, h) != kSolidEmpty) s = (s + 1) & tmask;
    }
  }
}

__device__ __forceinline__ bool is_solid(const unsigned long long* __restrict__ table, uint64_t tmask, uint64_t h) {
  uint64_t s = h & tmask;
  for (;;) {
    const unsigned long long x = table[s];
    if (x == h) return true;
    if (x == kSolidEmpty) return false;
    s = (s + 1) & tmask;
  }
}

__device__ __forceinline__ uint32_t get_base(const uint8_t* rd, uint32_t i) { return (rd[i >> 2] >> (2 * (i & 3))) & 3; }

// Hash of the canonical K-mer at [j, j+K) of the read, with base p replaced
// by alt (pass p = 0xffffffff for no override).
__device__ __forceinline__ uint64_t kmer_hash_at(const uint8_t* rd, uint32_t j, int K, const HashP& hp, uint32_t p,
                                                 uint32_t alt) {
  uint64_t fw = 0, rc = 0;
  const int rsh = 2 * K - 2;
  for (int t = 0; t < K; ++t) {
    const uint32_t i = j + t;
    const uint64_t b = i == p ? alt : get_base(rd, i);
    fw = ((fw << 2) | b) & hp.mask;
    rc = (rc >> 2) | ((3 - b) << rsh);
  }
  return khash(hp, fw < rc ? fw : rc);
}

struct PcCounters {
  unsigned long long suspect, corrected, ambiguous, uncorrectable;
};

__global__ void __launch_bounds__(256) k_precorrect(const uint64_t* __restrict__ base_off,
                                                    const uint64_t* __restrict__ byte_off, uint8_t* __restrict__ packed,
                                                    uint8_t* __restrict__ quals, uint64_t n_reads, int K, HashP hp,
                                                    uint32_t maxq, const unsigned long long* __restrict__ table,
                                                    uint64_t tmask, PcCounters* __restrict__ cnt) {
  unsigned long long n_sus = 0, n_cor = 0, n_amb = 0, n_unc = 0;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_reads;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t q0 = base_off[r];
    const uint32_t L = (uint32_t)(base_off[r + 1] - q0);
    if (L < (uint32_t)K) continue;
    uint8_t* rd = packed + byte_off[r];
    uint8_t* q = quals + q0;
    for (uint32_t p = 0; p < L; ++p) {
      if (q[p] >= maxq) continue;
      const uint32_t jlo = p + 1 >= (uint32_t)K ? p + 1 - K : 0;
      const uint32_t jhi = min(p, L - (uint32_t)K);
      bool weak = true;
      for (uint32_t j = jlo; j <= jhi && weak; ++j)
        if (is_solid(table, tmask, kmer_hash_at(rd, j, K, hp, 0xffffffffu, 0))) weak = false;
      if (!weak) continue;
      ++n_sus;
      const uint32_t orig = get_base(rd, p);
      uint32_t ncand = 0, cand = 0;
      for (uint32_t alt = 0; alt < 4; ++alt) {
        if (alt == orig) continue;
        bool ok = true;
        for (uint32_t j = jlo; j <= jhi && ok; ++j)
          if (!is_solid(table, tmask, kmer_hash_at(rd, j, K, hp, p, alt))) ok = false;
        if (ok) {
          ++ncand;
          cand = alt;
        }
      }
      if (ncand == 1) {
        const uint32_t sh = 2 * (p & 3);
        rd[p >> 2] = (uint8_t)((rd[p >> 2] & ~(3u << sh)) | (cand << sh));
        uint32_t nq = 255;
        if (p > 0) nq = min(nq, (uint32_t)q[p - 1]);
        if (p + 1 < L) nq = min(nq, (uint32_t)q[p + 1]);
        q[p] = (uint8_t)nq;
        ++n_cor;
      } else if (ncand > 1) {
        ++n_amb;
      } else {
        ++n_unc;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    n_sus += __shfl_down(n_sus, o, 64);
    n_cor += __shfl_down(n_cor, o, 64);
    n_amb += __shfl_down(n_amb, o, 64);
    n_unc += __shfl_down(n_unc, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (n_sus) atomicAdd(&cnt->suspect, n_sus);
    if (n_cor) atomicAdd(&cnt->corrected, n_cor);
    if (n_amb) atomicAdd(&cnt->ambiguous, n_amb);
    if (n_unc) atomicAdd(&cnt->uncorrectable, n_unc);
  }
}

static int precorrect_pass(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params& p, apg_pc_stats* st) {
  CountResult cr;
  APG_TRY(spectrum_impl(ctx, dr, p.K, true, nullptr, 0, &cr));
  unsigned long long* dcnt = nullptr;
  APG_TRY(workspace_t(ctx, "pc_counters", 8, &dcnt));
  APG_CHECK_HIP(hipMemsetAsync(dcnt, 0, 8 * 8, ctx->stream));
  const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>(cr.nbuckets, (uint64_t)ctx->n_cu * 16));
  k_count_solid<<<grid, 256, 0, ctx->stream>>>(cr.tab_cnt, cr.boff, cr.bucket_nd, cr.nbuckets, p.min_solid, dcnt + 4);
  APG_CHECK_HIP(hipGetLastError());
  unsigned long long n_solid = 0;
  APG_CHECK_HIP(hipMemcpyAsync(&n_solid, dcnt + 4, 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(sync(ctx));
  uint64_t T = 1024;
  while (T < 2 * n_solid) T <<= 1;
  unsigned long long* table = nullptr;
  APG_TRY(workspace_t(ctx, "pc_table", T, &table));
  APG_CHECK_HIP(hipMemsetAsync(table, 0xff, T * 8, ctx->stream));
  kbegin(ctx, "solid_insert", n_solid * 8 * 2);
  k_solid_insert<<<grid, 256, 0, ctx->stream>>>(cr.rec, cr.tab_cnt, cr.boff, cr.bucket_nd, cr.nbuckets, p.min_solid,
                                                table, T - 1);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  const uint64_t rgrid =
      std::max<uint64_t>(1, std::min<uint64_t>((dr->n_reads + 255) / 256, (uint64_t)ctx->n_cu * 32));
  kbegin(ctx, "precorrect", dr->n_bytes * 2 + dr->n_bases * 2);
  k_precorrect<<<rgrid, 256, 0, ctx->stream>>>(dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->d_quals,
                                               dr->n_reads, p.K, make_hashp(p.K), p.max_q_suspect, table, T - 1,
                                               reinterpret_cast<PcCounters*>(dcnt));
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  unsigned long long h[4];
  APG_CHECK_HIP(hipMemcpyAsync(h, dcnt, sizeof h, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(sync(ctx));
  st->n_suspect += h[0];
  st->n_corrected += h[1];
  st->n_ambiguous += h[2];
  st->n_uncorrectable += h[3];
  st->n_solid = n_solid;
  vlog(ctx, "precorrect pass: solid=%llu suspect=%llu corrected=%llu ambiguous=%llu none=%llu", n_solid, h[0], h[1],
       h[2], h[3]);
  return APG_OK;
}

}  // namespace apg

using namespace apg;

extern "C" {

void apg_pc_defaults(apg_pc_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->K = 24;
  p->min_solid = 3;
  p->max_q_suspect = 20;
  p->n_cycles = 1;
}

int apg_precorrect_dev(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params* pp, apg_pc_stats* stats) {
  APG_REQUIRE(ctx && dr, "apg_precorrect_dev: NULL argument");
  apg_pc_params p;
  if (pp)
    p = *pp;
  else
    apg_pc_defaults(&p);
  APG_REQUIRE(p.K >= 1 && p.K <= 32, "apg_precorrect: K must be in [1, 32]");
  APG_REQUIRE(p.min_solid >= 1, "apg_precorrect: min_solid must be >= 1");
  APG_REQUIRE(p.n_cycles >= 1 && p.n_cycles <= 16, "apg_precorrect: n_cycles must be in [1, 16]");
  APG_REQUIRE(dr->n_reads == 0 || dr->d_quals, "apg_precorrect: read set has no qualities");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  apg_pc_stats st;
  std::memset(&st, 0, sizeof st);
  for (uint32_t c = 0; c < p.n_cycles; ++c) {
    APG_TRY(precorrect_pass(ctx, dr, p, &st));
    static std::atomic<uint64_t> g_edit{1ull << 62};
    dr->gen = g_edit.fetch_add(1);  // bases changed: invalidate per-read-set plans
  }
  if (stats) *stats = st;
  return APG_OK;
}

int apg_reads_download(apg_ctx* ctx, const apg_dreads* dr, uint8_t* packed, uint8_t* quals) {
  APG_REQUIRE(ctx && dr, "apg_reads_download: NULL argument");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  if (packed && dr->n_bytes)
    APG_CHECK_HIP(hipMemcpyAsync(packed, dr->d_packed, dr->n_bytes, hipMemcpyDeviceToHost, ctx->stream));
  if (quals && dr->d_quals && dr->n_bases)
    APG_CHECK_HIP(hipMemcpyAsync(quals, dr->d_quals, dr->n_bases, hipMemcpyDeviceToHost, ctx->stream));
  return sync(ctx);
}

int apg_precorrect(apg_ctx* ctx, const apg_reads* reads, const apg_pc_params* p, uint8_t* out_packed,
                   uint8_t* out_quals, apg_pc_stats* stats) {
  APG_REQUIRE(ctx && reads && out_packed && out_quals, "apg_precorrect: NULL argument");
  APG_REQUIRE(reads->n_reads == 0 || reads->quals, "apg_precorrect: reads->quals is required");
  apg_dreads* dr = nullptr;
  APG_TRY(apg_reads_upload(ctx, reads, &dr));
  int rc = apg_precorrect_dev(ctx, dr, p, stats);
  if (rc == APG_OK) rc = apg_reads_download(ctx, dr, out_packed, out_quals);
  apg_reads_free(dr);
  return rc;
}

}  // extern "C"
