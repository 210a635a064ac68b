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
#include "partition.hpp"

namespace apg {

constexpr uint64_t kSolidEmpty = ~0ull;

// Open-addressing table of a solid hash list (linear probing, load <= 0.5;
// hashes are uniformly mixed, so the home slot is the hash's low bits).
__global__ void k_solid_insert(const uint64_t* __restrict__ list, uint64_t n, unsigned long long* __restrict__ table,
                               uint64_t tmask) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long h = list[i];
    uint64_t s = h & tmask;
    while (atomicCAS(&table[s], (unsigned long long)kSolidEmpty, h) != kSolidEmpty) s = (s + 1) & tmask;
  }
}

// The solid set: the exact open-addressing table behind a prefix bitmap —
// bit i set iff some solid K-mer's hash has top bits i — sized at ~16 bits
// per solid K-mer (2^30 bits = 128 MiB for the bench's 66 M solid K-mers), so
// it stays in the 256 MiB Infinity Cache while the exact table (16 B per key)
// does not.  The hash is a bijective mixer, so prefixes are uniform: a weak
// K-mer passes with probability ~1/16.  Most queries of the correction are
// weak K-mers (every K-mer covering a real error, every wrong alternative);
// the bitmap answers those without touching HBM, and only bitmap hits probe
// the table.  The bitmap never changes an answer.
struct SolidSet {
  const unsigned long long* table;
  uint64_t tmask;
  const uint32_t* bitmap;
  int shift;  // bit index = hash >> shift
};

__global__ void k_bitmap_insert(const uint64_t* __restrict__ list, uint64_t n, uint32_t* __restrict__ bm, int shift) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = list[i] >> shift;
    atomicOr(&bm[b >> 5], 1u << (b & 31));
  }
}

__device__ __forceinline__ bool bitmap_maybe(const SolidSet& ss, uint64_t h) {
  const uint64_t b = h >> ss.shift;
  return (ss.bitmap[b >> 5] >> (b & 31)) & 1;
}

__device__ __forceinline__ bool table_has(const unsigned long long* __restrict__ table, uint64_t tmask, uint64_t h) {
  uint64_t s = h & tmask;
  for (;;) {
    const unsigned long long x = table[s];
    if (x == h) return true;
    if (x == kSolidEmpty) return false;
    s = (s + 1) & tmask;
  }
}

// n_tab counts the table probes (filter hits) of the calling lane.
__device__ __forceinline__ bool is_solid(const SolidSet& ss, uint64_t h, uint32_t* n_tab) {
  if (!bitmap_maybe(ss, h)) return false;
  ++*n_tab;
  return table_has(ss.table, ss.tmask, h);
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
  unsigned long long lookups;       // solid-set queries (one bitmap line each)
  unsigned long long table_probes;  // filter hits that probed the exact table (one 64-byte line each)
};

__global__ void __launch_bounds__(256) k_precorrect(const uint64_t* __restrict__ base_off,
                                                    const uint64_t* __restrict__ byte_off, uint8_t* __restrict__ packed,
                                                    uint8_t* __restrict__ quals, uint64_t n_reads, int K, HashP hp,
                                                    uint32_t maxq, SolidSet ss, uint32_t min_len,
                                                    uint8_t* __restrict__ clean, PcCounters* __restrict__ cnt) {
  uint32_t n_tab = 0;
  unsigned long long n_sus = 0, n_cor = 0, n_amb = 0, n_unc = 0;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_reads;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t q0 = base_off[r];
    const uint32_t L = (uint32_t)(base_off[r + 1] - q0);
    if (L < (uint32_t)K || L < min_len) continue;
    if (clean) clean[r] = 2;  // not derived for long reads: FillFragments checks them itself
    uint8_t* rd = packed + byte_off[r];
    uint8_t* q = quals + q0;
    for (uint32_t p = 0; p < L; ++p) {
      if (q[p] >= maxq) continue;
      const uint32_t jlo = p + 1 >= (uint32_t)K ? p + 1 - K : 0;
      const uint32_t jhi = min(p, L - (uint32_t)K);
      bool weak = true;
      for (uint32_t j = jlo; j <= jhi && weak; ++j)
        if (is_solid(ss, kmer_hash_at(rd, j, K, hp, 0xffffffffu, 0), &n_tab)) weak = false;
      if (!weak) continue;
      ++n_sus;
      const uint32_t orig = get_base(rd, p);
      uint32_t ncand = 0, cand = 0;
      for (uint32_t alt = 0; alt < 4; ++alt) {
        if (alt == orig) continue;
        bool ok = true;
        for (uint32_t j = jlo; j <= jhi && ok; ++j)
          if (!is_solid(ss, kmer_hash_at(rd, j, K, hp, p, alt), &n_tab)) ok = false;
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
  wave_add(&cnt->table_probes, n_tab);
}

// ---------------------------------------------------------------------------
// Wave-per-read correction (reads of <= kPcMaxL bases).  Same rule and order
// as k_precorrect (which still handles longer reads), restructured for
// memory-level parallelism: the read's bases live in the wave's registers
// (lane i holds packed bases [16i, 16i+16) as one u32), suspects are found
// 64 positions at a time by ballot, and for each suspect in left-to-right
// order the <= K covering K-mers (weak test) and then the <= 3K
// (alternative, K-mer) pairs are looked up ONE PER LANE in parallel instead
// of one dependent probe at a time.  A K-mer window is cut from the packed
// words (LSB-first: window value W = sum b[j+t] 4^t), so
//   fw = rev2(W) >> (64 - 2K),   rc = W ^ mask(2K).
// ---------------------------------------------------------------------------
constexpr uint32_t kPcMaxL = 1024;  // 64 lanes x 16 bases

__device__ __forceinline__ uint64_t rev2(uint64_t x) {
  x = __builtin_bitreverse64(x);
  return ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
}

// 2K-bit window starting at base j of the read whose packed u32 words are
// spread one per lane (word i in lane i's `word`).
__device__ __forceinline__ uint64_t window_at(uint32_t word, uint32_t j, uint64_t mask) {
  const uint32_t bit = 2 * j, wi = bit >> 5, sh = bit & 31;
  const uint32_t w0 = (uint32_t)__shfl((int)word, (int)min(wi, 63u), 64);
  const uint32_t w1 = (uint32_t)__shfl((int)word, (int)min(wi + 1, 63u), 64);
  const uint32_t w2 = (uint32_t)__shfl((int)word, (int)min(wi + 2, 63u), 64);
  const uint64_t lo = (uint64_t)w0 | ((uint64_t)w1 << 32);
  uint64_t W = lo >> sh;
  if (sh) W |= (uint64_t)w2 << (64 - sh);
  return W & mask;
}

__device__ __forceinline__ uint64_t canon_hash(uint64_t W, int K, const HashP& hp) {
  const uint64_t fw = rev2(W) >> (64 - 2 * K);
  const uint64_t rc = W ^ hp.mask;
  return khash(hp, fw < rc ? fw : rc);
}

__global__ void __launch_bounds__(256) k_precorrect_wave(const uint64_t* __restrict__ base_off,
                                                         const uint64_t* __restrict__ byte_off,
                                                         uint8_t* __restrict__ packed, uint8_t* __restrict__ quals,
                                                         uint64_t n_reads, int K, HashP hp, uint32_t maxq,
                                                         SolidSet ss, const unsigned long long* __restrict__ weak,
                                                         uint8_t* __restrict__ clean, PcCounters* __restrict__ cnt) {
  uint32_t n_tab = 0;
  const int lane = lane_id();
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  unsigned long long n_sus = 0, n_cor = 0, n_amb = 0, n_unc = 0;  // lane 0's
  unsigned long long n_look = 0;
  for (uint64_t r = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave_id(); r < n_reads; r += nwaves) {
    const uint64_t q0 = base_off[r];
    const uint32_t L = (uint32_t)(base_off[r + 1] - q0);
    if (L < (uint32_t)K) {  // wave-uniform; no K-mer, nothing weak
      if (clean && lane == 0) clean[r] = 1;
      continue;
    }
    if (L > kPcMaxL) continue;  // the thread-per-read kernel's
    uint8_t* rd = packed + byte_off[r];
    uint8_t* q = quals + q0;
    const uint32_t nbytes = (L + 3) >> 2;
    uint32_t word = 0;
    if (4u * lane < nbytes) {
      const uint32_t b = 4u * lane;
      word = (uint32_t)rd[b] | (b + 1 < nbytes ? (uint32_t)rd[b + 1] << 8 : 0u) |
             (b + 2 < nbytes ? (uint32_t)rd[b + 2] << 16 : 0u) | (b + 3 < nbytes ? (uint32_t)rd[b + 3] << 24 : 0u);
    }
    // Weak-bitmap mode: lane i holds the weak bits of K-mers [16i, 16i+16) as
    // counted (W16) and the corrected positions [16i, 16i+16) so far (C16).
    uint32_t W16 = 0, C16 = 0;
    const uint32_t nK = L - (uint32_t)K + 1;
    if (weak && 16u * lane < nK) {
      const uint64_t b = q0 + 16u * lane;
      const uint32_t sh = (uint32_t)(b & 63);
      uint64_t x = weak[b >> 6] >> sh;
      if (sh > 48) x |= weak[(b >> 6) + 1] << (64 - sh);
      W16 = (uint32_t)x & 0xffffu;
      if (nK - 16u * lane < 16) W16 &= (1u << (nK - 16u * lane)) - 1;
    }
    int last_corr = -1;  // wave-uniform: latest corrected position
    for (uint32_t c = 0; c < L; c += 64) {
      const uint32_t pl = c + lane;
      uint64_t m = __ballot(pl < L && q[pl] < maxq);
      while (m) {
        const uint32_t p = c + (uint32_t)(__ffsll((long long)m) - 1);
        m &= m - 1;
        const uint32_t jlo = p + 1 >= (uint32_t)K ? p + 1 - K : 0;
        const uint32_t jhi = min(p, L - (uint32_t)K);
        const uint32_t nk = jhi - jlo + 1;  // <= K <= 32
        if (weak) {
          // A covering K-mer holding an earlier correction is solid (it was
          // checked when that base was corrected); the others are unchanged
          // since counting, so their weakness is the counted bit.
          if (last_corr >= 0 && p - (uint32_t)last_corr < (uint32_t)K) continue;
          const uint32_t li = jlo >> 4;
          uint64_t x = 0;
#pragma unroll
          for (uint32_t k = 0; k < 3; ++k) {
            const uint32_t v = (uint32_t)__shfl((int)W16, (int)min(li + k, 63u), 64);
            if (li + k < 64) x |= (uint64_t)v << (16 * k);
          }
          const uint64_t need = (1ull << nk) - 1;
          if (((x >> (jlo & 15)) & need) != need) continue;
        } else {
          // every lane takes part in the shuffles; lanes >= nk repeat the last K-mer
          const uint64_t Wk = window_at(word, jlo + min((uint32_t)lane, nk - 1), hp.mask);
          bool solid = false;
          if ((uint32_t)lane < nk) solid = is_solid(ss, canon_hash(Wk, K, hp), &n_tab);
          n_look += nk;
          if (__ballot(solid)) continue;
        }
        ++n_sus;
        const uint32_t orig = (__shfl((int)word, (int)(p >> 4), 64) >> (2 * (p & 15))) & 3;
        // Alternatives in two rounds of lookups: (A) the first covering K-mer
        // of each of the 3 alternatives (lanes 0..2); (B) the remaining nk-1
        // K-mers of each survivor of (A) — usually one — one per lane.
        const uint64_t W0 = window_at(word, jlo, hp.mask);
        const uint32_t sh0 = 2 * (p - jlo);
        bool badA = false;
        if (lane < 3) {
          const uint32_t alt = (uint32_t)lane + ((uint32_t)lane >= orig ? 1u : 0u);
          badA = !is_solid(ss, canon_hash((W0 & ~(3ull << sh0)) | ((uint64_t)alt << sh0), K, hp), &n_tab);
        }
        uint32_t surv = (uint32_t)(~__ballot(badA)) & 7u;
        n_look += 3 + (uint64_t)__popc(surv) * (nk - 1);
        uint32_t ncand = 0, cand = 0;
        const uint32_t t1 = jlo + 1 + min((uint32_t)lane, nk > 1 ? nk - 2 : 0u);
        const uint64_t W1 = window_at(word, t1, hp.mask);  // every lane joins the shuffles
        const uint32_t sh1 = 2 * (p - t1);
        while (surv) {
          const uint32_t a = (uint32_t)(__ffs((int)surv) - 1);
          surv &= surv - 1;
          const uint32_t alt = a + (a >= orig ? 1u : 0u);
          bool bad = false;
          if ((uint32_t)lane + 1 < nk)
            bad = !is_solid(ss, canon_hash((W1 & ~(3ull << sh1)) | ((uint64_t)alt << sh1), K, hp), &n_tab);
          if (!__ballot(bad)) {
            ++ncand;
            cand = alt;
          }
        }
        if (ncand == 1) {
          if ((uint32_t)lane == (p >> 4)) {
            const uint32_t sh = 2 * (p & 15);
            word = (word & ~(3u << sh)) | (cand << sh);
            C16 |= 1u << (p & 15);
          }
          last_corr = (int)p;
          const uint32_t nw = (uint32_t)__shfl((int)word, (int)(p >> 4), 64);
          if (lane == 0) {
            rd[p >> 2] = (uint8_t)(nw >> (8 * ((p >> 2) & 3)));
            uint32_t nq = 255;
            if (p > 0) nq = min(nq, (uint32_t)q[p - 1]);
            if (p + 1 < L) nq = min(nq, (uint32_t)q[p + 1]);
            q[p] = (uint8_t)nq;
            ++n_cor;
          }
        } else if (ncand > 1) {
          ++n_amb;
        } else {
          ++n_unc;
        }
      }
    }
    if (clean) {
      // Clean read (every K-mer solid after correction, the FillFragments
      // precondition): each counted-weak K-mer holds a corrected base —
      // K-mer j is covered iff a C bit lies in [j, j+K-1].
      uint32_t unc = 0;
      if (weak) {
        uint64_t X = 0;
#pragma unroll
        for (uint32_t k = 0; k < 3; ++k) {
          const uint32_t v = (uint32_t)__shfl((int)C16, (int)min((uint32_t)lane + k, 63u), 64);
          if ((uint32_t)lane + k < 64) X |= (uint64_t)v << (16 * k);
        }
        uint64_t D = 0;
        for (int s = 0; s < K; ++s) D |= X >> s;
        unc = W16 & ~(uint32_t)D & 0xffffu;
      }
      const bool any = __ballot(unc != 0) != 0;
      if (lane == 0) clean[r] = weak ? (any ? 0 : 1) : 2;
    }
  }
  wave_add(&cnt->table_probes, n_tab);
  if (lane == 0) {
    if (n_look) atomicAdd(&cnt->lookups, n_look);
    if (n_sus) atomicAdd(&cnt->suspect, n_sus);
    if (n_cor) atomicAdd(&cnt->corrected, n_cor);
    if (n_amb) atomicAdd(&cnt->ambiguous, n_amb);
    if (n_unc) atomicAdd(&cnt->uncorrectable, n_unc);
  }
}

// One correction pass of every read of `dr` against the solid hash list.
// weak: the pass's weak-instance bitmap (sk_solid_weak) or null (weak tests
// by lookups); with it, the pass also leaves per-read clean flags ("pc_clean":
// 1 every K-mer solid after correction, 0 not, 2 not derived) for
// FillFragments.
static int correct_pass(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params& p, const uint64_t* list, uint64_t n_solid,
                        apg_pc_stats* st, const unsigned long long* weak = nullptr) {
  ctx->clean_valid = false;
  uint8_t* clean = nullptr;
  if (weak) APG_TRY(workspace_t(ctx, "pc_clean", std::max<uint64_t>(dr->n_reads, 1), &clean));
  unsigned long long* dcnt = nullptr;
  APG_TRY(workspace_t(ctx, "pc_counters", 8, &dcnt));
  APG_CHECK_HIP(hipMemsetAsync(dcnt, 0, 8 * 8, ctx->stream));
  uint64_t T = 1024;
  while (T < 2 * n_solid) T <<= 1;
  unsigned long long* table = nullptr;
  APG_TRY(workspace_t(ctx, "pc_table", T, &table));
  APG_CHECK_HIP(hipMemsetAsync(table, 0xff, T * 8, ctx->stream));
  // prefix bitmap: 2^mb bits, ~16 bits per solid K-mer, at most one bit per K-mer
  int mb = 10;
  while ((1ull << mb) < 16 * n_solid && mb < 2 * p.K) ++mb;
  if (mb > 2 * p.K) mb = 2 * p.K;
  uint32_t* bitmap = nullptr;
  const uint64_t words = std::max<uint64_t>(1, (1ull << mb) / 32);
  APG_TRY(workspace_t(ctx, "pc_bitmap", words, &bitmap));
  APG_CHECK_HIP(hipMemsetAsync(bitmap, 0, words * 4, ctx->stream));
  kbegin(ctx, "solid_insert", n_solid * (8 + 64 + 64));
  if (n_solid) {
    k_solid_insert<<<grid_for(ctx, n_solid), 256, 0, ctx->stream>>>(list, n_solid, table, T - 1);
    k_bitmap_insert<<<grid_for(ctx, n_solid), 256, 0, ctx->stream>>>(list, n_solid, bitmap, 2 * p.K - mb);
  }
  kend(ctx);
  const SolidSet ss{table, T - 1, bitmap, 2 * p.K - mb};
  APG_CHECK_HIP(hipGetLastError());
  const HashP hp = make_hashp(p.K);
  // reads + quals (+ the weak bitmap and the clean flags)
  kbegin(ctx, "precorrect", dr->n_bytes + dr->n_bases + (weak ? dr->n_bases / 8 + dr->n_reads : 0));
  if (dr->n_reads)
    k_precorrect_wave<<<grid_for(ctx, dr->n_reads, 4), 256, 0, ctx->stream>>>(
        dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->d_quals, dr->n_reads, p.K, hp, p.max_q_suspect, ss, weak,
        clean, reinterpret_cast<PcCounters*>(dcnt));
  kend(ctx);
  if (dr->max_len > kPcMaxL) {  // reads longer than one wave's registers: thread per read
    const uint64_t rgrid =
        std::max<uint64_t>(1, std::min<uint64_t>((dr->n_reads + 255) / 256, (uint64_t)ctx->n_cu * 32));
    k_precorrect<<<rgrid, 256, 0, ctx->stream>>>(dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->d_quals,
                                                 dr->n_reads, p.K, hp, p.max_q_suspect, ss, kPcMaxL + 1, clean,
                                                 reinterpret_cast<PcCounters*>(dcnt));
  }
  APG_CHECK_HIP(hipGetLastError());
  unsigned long long h[6];
  APG_CHECK_HIP(hipMemcpyAsync(h, dcnt, sizeof h, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(sync(ctx));
  // a bitmap query reads one word of an L3-resident bitmap (counted 4 B); a
  // table probe is a random 64-byte HBM line
  kbytes_add(ctx, "precorrect", h[4] * 4 + h[5] * 64);
  vlog(ctx, "precorrect: %llu solid-set queries, %llu table probes", h[4], h[5]);
  st->n_suspect += h[0];
  st->n_corrected += h[1];
  st->n_ambiguous += h[2];
  st->n_uncorrectable += h[3];
  st->n_solid = n_solid;
  ctx->pc_list = list;  // APG_FILL_LAST_SOLID (FillFragments after correction)
  ctx->pc_n = n_solid;
  ctx->pc_K = p.K;
  ctx->pc_list_valid = true;
  vlog(ctx, "precorrect pass: solid=%llu suspect=%llu corrected=%llu ambiguous=%llu none=%llu",
       (unsigned long long)n_solid, h[0], h[1], h[2], h[3]);
  static std::atomic<uint64_t> g_edit{1ull << 62};
  dr->gen = g_edit.fetch_add(1);  // bases changed: invalidate per-read-set plans
  if (clean) {
    ctx->pc_clean = clean;
    ctx->clean_gen = dr->gen;
    ctx->clean_valid = true;
  }
  return APG_OK;
}

static int precorrect_pass(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params& p, apg_pc_stats* st) {
  SkResult sr;
  if (p.K >= 9) {  // count + the weak-instance bitmap (no lookups for the weak tests)
    unsigned long long* weak = nullptr;
    APG_TRY(workspace_t(ctx, "pc_weak", dr->n_bases / 64 + 2, &weak));
    APG_TRY(sk_solid_weak(ctx, dr, p.K, p.min_solid, weak, &sr));
    ctx->solid_valid = false;  // "pc_solid" now holds this pass's list
    return correct_pass(ctx, dr, p, sr.solid, sr.n_solid, st, weak);
  }
  APG_TRY(sk_spectrum(ctx, dr, p.K, true, p.min_solid, nullptr, 0, &sr));
  ctx->solid_valid = false;
  return correct_pass(ctx, dr, p, sr.solid, sr.n_solid, st);
}

static int check_pc(const apg_pc_params& p) {
  APG_REQUIRE(p.K >= 1 && p.K <= 32, "apg_precorrect: K must be in [1, 32]");
  APG_REQUIRE(p.min_solid >= 1, "apg_precorrect: min_solid must be >= 1");
  APG_REQUIRE(p.n_cycles >= 1 && p.n_cycles <= 16, "apg_precorrect: n_cycles must be in [1, 16]");
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
  APG_TRY(check_pc(p));
  APG_REQUIRE(dr->n_reads == 0 || dr->d_quals, "apg_precorrect: read set has no qualities");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  apg_pc_stats st;
  std::memset(&st, 0, sizeof st);
  for (uint32_t c = 0; c < p.n_cycles; ++c) APG_TRY(precorrect_pass(ctx, dr, p, &st));
  if (stats) *stats = st;
  return APG_OK;
}

int apg_shard_solid(apg_ctx* ctx, const void* d_recv, const uint64_t* recv_counts, int K, int n_shards,
                    uint32_t min_solid, uint64_t* n_solid) {
  APG_REQUIRE(ctx && recv_counts && n_solid, "apg_shard_solid: NULL argument");
  APG_REQUIRE(min_solid >= 1, "apg_shard_solid: min_solid must be >= 1");
  ctx->solid_valid = false;
  APG_REQUIRE(K >= 1 && K <= 32 && n_shards >= 1 && n_shards <= 8 && (n_shards & (n_shards - 1)) == 0,
              "apg_shard_solid: K must be in [1, 32], n_shards a power of two <= 8");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  std::vector<uint64_t> rc(recv_counts, recv_counts + (size_t)n_shards * kSkShardBins);
  uint64_t n = 0;
  for (auto c : rc) n += c;
  APG_REQUIRE(n == 0 || d_recv, "apg_shard_solid: d_recv is NULL");
  const SK16* recs = static_cast<const SK16*>(d_recv);
  int err = APG_OK;
  const uint64_t nk = sk_sum_kmers(ctx, recs, n, &err);
  APG_TRY(err);
  SkResult sr;
  APG_TRY(sk_stage_count(ctx, recs, nullptr, rc, nk, K, n_shards, true, min_solid, nullptr, 0, &sr));
  APG_TRY(sync(ctx));
  const uint64_t ns = sr.n_solid;
  ctx->n_solid = ns;
  ctx->solid_valid = true;
  *n_solid = ns;
  return APG_OK;
}

int apg_solid_export(apg_ctx* ctx, void* d_out) {
  APG_REQUIRE(ctx, "apg_solid_export: NULL ctx");
  APG_REQUIRE(ctx->solid_valid, "apg_solid_export: no apg_shard_solid result on this context");
  if (ctx->n_solid == 0) return APG_OK;
  APG_REQUIRE(d_out, "apg_solid_export: d_out is NULL");
  uint64_t* list = nullptr;
  APG_TRY(workspace_t(ctx, "pc_solid", ctx->n_solid, &list));
  APG_CHECK_HIP(hipMemcpyAsync(d_out, list, ctx->n_solid * 8, hipMemcpyDeviceToDevice, ctx->stream));
  return sync(ctx);
}

int apg_solid_copy(apg_ctx* ctx, void* d_out, uint64_t* n_solid) {
  APG_REQUIRE(ctx && n_solid, "apg_solid_copy: NULL argument");
  APG_REQUIRE(ctx->pc_list_valid, "apg_solid_copy: no correction pass has run on this context");
  *n_solid = ctx->pc_n;
  if (!d_out || ctx->pc_n == 0) return APG_OK;
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  APG_CHECK_HIP(hipMemcpyAsync(d_out, ctx->pc_list, ctx->pc_n * 8, hipMemcpyDeviceToDevice, ctx->stream));
  return sync(ctx);
}

int apg_precorrect_solid(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params* pp, const void* d_solid,
                         uint64_t n_solid, apg_pc_stats* stats) {
  APG_REQUIRE(ctx && dr, "apg_precorrect_solid: NULL argument");
  APG_REQUIRE(n_solid == 0 || d_solid, "apg_precorrect_solid: d_solid is NULL");
  apg_pc_params p;
  if (pp)
    p = *pp;
  else
    apg_pc_defaults(&p);
  APG_TRY(check_pc(p));
  APG_REQUIRE(dr->n_reads == 0 || dr->d_quals, "apg_precorrect_solid: read set has no qualities");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  apg_pc_stats st;
  std::memset(&st, 0, sizeof st);
  APG_TRY(correct_pass(ctx, dr, p, static_cast<const uint64_t*>(d_solid), n_solid, &st));
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
