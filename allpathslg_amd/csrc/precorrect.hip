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
#include "ext_table.hpp"
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

__device__ __forceinline__ uint64_t rev2(uint64_t x) { return f_rev2(x); }

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

// K+1 bases [i-1, i+K) of the read as an LSB-first value (base i-1 at bits
// 0-1; for i == 0 there is no base i-1 and bits 0-1 are 0), with base p
// replaced by alt (p = ~0u: no replacement).  Every lane joins the shuffles.
__device__ __forceinline__ uint64_t ext_window(uint32_t word, uint32_t i, int K, uint32_t p, uint32_t alt) {
  const uint64_t m = (1ull << (2 * (K + 1))) - 1;  // K <= 29
  uint64_t W = window_at(word, i ? i - 1 : 0, m);
  if (!i) W = (W << 2) & m;
  if (p + 1 >= i && p + 1 <= i + (uint32_t)K) {  // p in [i-1, i+K-1]
    const uint32_t sh = 2 * (p + 1 - i);
    W = (W & ~(3ull << sh)) | ((uint64_t)alt << sh);
  }
  return W;
}

// K-mers i-1 (a read K-mer iff i >= 1) and i of the window W = ext_window(i):
// bit 0 = K-mer i-1 solid (pred of (K-1)-mer i holds base i-1), bit 1 = K-mer
// i solid (succ holds base i+K-1).  One extension-table lookup.
__device__ __forceinline__ uint32_t ext_pair(const ExtTab& t, uint64_t W, int K) {
  const uint32_t e = ext_masks_lsb(t, (W >> 2) & t.m1);
  const uint32_t pb = (uint32_t)W & 3, sb = (uint32_t)(W >> (2 * K)) & 3;
  return ((e >> pb) & 1) | (((e >> (4 + sb)) & 1) << 1);
}

// Offsets of read r (L = 0 past the end) and its register-resident data.
struct PcMeta {
  uint64_t q0, bo;
  uint32_t L;
};
struct PcData {
  uint32_t word, qa, qb, W16;
};

__device__ __forceinline__ PcMeta pc_meta(const uint64_t* __restrict__ base_off, const uint64_t* __restrict__ byte_off,
                                          uint64_t n_reads, uint64_t r) {
  PcMeta m{0, 0, 0};
  if (r < n_reads) {
    m.q0 = base_off[r];
    m.L = (uint32_t)(base_off[r + 1] - m.q0);
    m.bo = byte_off[r];
  }
  return m;
}

// Lane i: packed bases [16i, 16i+16) (one aligned u32 load per lane, funnel-
// shifted with the next lane's; the read sets carry 64 bytes of slack), quals
// i and 64 + i, weak bits of K-mers [16i, 16i+16).  Wave-uniform branches.
__device__ __forceinline__ PcData pc_data(const PcMeta& m, const uint8_t* __restrict__ packed,
                                          const uint8_t* __restrict__ quals,
                                          const unsigned long long* __restrict__ weak, int K) {
  PcData d{0, 255, 255, 0};
  if (m.L < (uint32_t)K || m.L > kPcMaxL) return d;
  const uint32_t lane = (uint32_t)lane_id();
  const uint32_t nbytes = (m.L + 3) >> 2;
  const uint32_t s = (uint32_t)(m.bo & 3);
  const uint32_t* aw = reinterpret_cast<const uint32_t*>(packed + (m.bo - s));
  const uint32_t naw = (nbytes + s + 3) >> 2;
  const uint32_t w = lane < naw ? aw[lane] : 0u;
  const uint32_t wx = (lane == 63 && naw > 64) ? aw[64] : 0u;
  uint32_t nx = (uint32_t)__shfl((int)w, (int)min(lane + 1, 63u), 64);
  if (lane == 63) nx = wx;
  uint32_t word = s ? (w >> (8 * s)) | (nx << (32 - 8 * s)) : w;
  if (4 * lane >= nbytes)
    word = 0;
  else if (nbytes - 4 * lane < 4)
    word &= (1u << (8 * (nbytes - 4 * lane))) - 1;
  d.word = word;
  const uint8_t* q = quals + m.q0;
  if (lane < m.L) d.qa = q[lane];
  if (lane + 64 < m.L) d.qb = q[lane + 64];
  const uint32_t nK = m.L - (uint32_t)K + 1;
  if (weak && 16u * lane < nK) {
    const uint64_t b = m.q0 + 16u * lane;
    const uint32_t sh = (uint32_t)(b & 63);
    uint64_t x = weak[b >> 6] >> sh;
    if (sh > 48) x |= weak[(b >> 6) + 1] << (64 - sh);
    uint32_t W16 = (uint32_t)x & 0xffffu;
    if (nK - 16u * lane < 16) W16 &= (1u << (nK - 16u * lane)) - 1;
    d.W16 = W16;
  }
  return d;
}

// EXT = false: solidity by K-mer lookups in the SolidSet (any K <= 32).
// EXT = true (2 <= K <= 29): by (K-1)-mer extension lookups, each answering
// two adjacent K-mers — the weak test and an alternative's covering K-mers
// take half the lookups, and the first and last covering K-mers of a suspect
// (the (K-1)-mers beside p do not contain p) are answered for all 4 bases at
// p by two lookups, before any alternative is tried.
template <bool EXT>
__global__ void __launch_bounds__(256) k_precorrect_wave(const uint64_t* __restrict__ base_off,
                                                         const uint64_t* __restrict__ byte_off,
                                                         uint8_t* __restrict__ packed, uint8_t* __restrict__ quals,
                                                         uint64_t n_reads, int K, HashP hp, uint32_t maxq,
                                                         SolidSet ss, ExtTab et,
                                                         const unsigned long long* __restrict__ weak,
                                                         uint8_t* __restrict__ clean, PcCounters* __restrict__ cnt) {
  uint32_t n_tab = 0;
  const int lane = lane_id();
  const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  unsigned long long n_sus = 0, n_cor = 0, n_amb = 0, n_unc = 0;  // lane 0's
  unsigned long long n_look = 0;
  // Software pipeline over the wave's reads r, r + nwaves, ...: the next
  // read's bases, first 128 quals and weak bits are loaded while this read is
  // corrected, the offsets of the read after it one step earlier still, so a
  // read costs the round trips of its suspects' lookups and no more.
  uint64_t r = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave_id();
  PcMeta m0 = pc_meta(base_off, byte_off, n_reads, r);
  PcData d0 = pc_data(m0, packed, quals, weak, K);
  PcMeta m1 = pc_meta(base_off, byte_off, n_reads, r + nwaves);
  for (; r < n_reads; r += nwaves) {
    const PcMeta mc = m0;
    const PcData dc = d0;
    m0 = m1;
    d0 = pc_data(m1, packed, quals, weak, K);
    m1 = pc_meta(base_off, byte_off, n_reads, r + 2 * nwaves);
    const uint64_t q0 = mc.q0;
    const uint32_t L = mc.L;
    if (L < (uint32_t)K) {  // wave-uniform; no K-mer, nothing weak
      if (clean && lane == 0) clean[r] = 1;
      continue;
    }
    if (L > kPcMaxL) continue;  // the thread-per-read kernel's
    uint8_t* rd = packed + mc.bo;
    uint8_t* q = quals + q0;
    // lane i: packed bases [16i, 16i+16) (word), quals of positions i and
    // 64 + i (qa, qb; 255 past the read); weak-bitmap mode: the weak bits of
    // K-mers [16i, 16i+16) as counted (W16) and the positions [16i, 16i+16)
    // corrected so far (C16).
    uint32_t word = dc.word, qa = dc.qa, qb = dc.qb;
    const uint32_t W16 = dc.W16;
    uint32_t C16 = 0;
    int last_corr = -1;  // wave-uniform: latest corrected position
    for (uint32_t c = 0; c < L; c += 64) {
      const uint32_t pl = c + lane;
      const uint32_t qv = c == 0 ? qa : c == 64 ? qb : (pl < L ? (uint32_t)q[pl] : 255u);
      uint64_t m = __ballot(qv < maxq);
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
        } else if constexpr (EXT) {
          // K-mers jlo..jhi in pairs: lane l looks up (K-1)-mer jlo + 1 + 2l
          const uint32_t G = (nk + 1) >> 1;
          const uint32_t i = jlo + 1 + 2 * min((uint32_t)lane, G - 1);
          const uint64_t Wk = ext_window(word, i, K, ~0u, 0);
          bool solid = false;
          if ((uint32_t)lane < G) {
            const uint32_t r2 = ext_pair(et, Wk, K);
            solid = (r2 & 1) || (i <= jhi && (r2 & 2));
          }
          n_look += G;
          if (__ballot(solid)) continue;
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
        uint32_t ncand = 0, cand = 0;
        if constexpr (EXT) {
          // (A) the (K-1)-mers beside p: lane 0 the one ending at p - 1 (its
          // successors answer K-mer p-K+1 for every base at p), lane 1 the one
          // starting at p + 1 (predecessors: K-mer p).
          const bool hasA = p + 1 >= (uint32_t)K, hasB = p + (uint32_t)K <= L;
          const uint32_t iA = lane == 0 ? (hasA ? p + 1 - K : 0) : (hasB ? p + 1 : 0);
          const uint64_t WA = ext_window(word, iA, K, ~0u, 0);
          uint32_t mA = 15;
          if ((lane == 0 && hasA) || (lane == 1 && hasB)) {
            const uint32_t e = ext_masks_lsb(et, (WA >> 2) & et.m1);
            mA = lane == 0 ? e >> 4 : e & 15;
          }
          const uint32_t allowed = (uint32_t)__shfl((int)mA, 0, 64) & (uint32_t)__shfl((int)mA, 1, 64);
          const uint32_t surv = allowed & ~(1u << orig) & 15u;
          const uint32_t ns = __popc(surv);
          n_look += (hasA ? 1 : 0) + (hasB ? 1 : 0);
          // (B) the other covering K-mers a..b of every survivor at once: survivor
          // s on lanes [sG, sG + G), lane sG + l looking up (K-1)-mer a + 1 + 2l.
          const int ia = (int)jlo + (hasA ? 1 : 0), ib = (int)jhi - (hasB ? 1 : 0);
          if (ib < ia || ns == 0) {
            ncand = ns;
            cand = ns ? (uint32_t)(__ffs((int)surv) - 1) : 0;
          } else {
            const uint32_t G = (uint32_t)(ib - ia + 2) >> 1;
            const uint32_t sidx = min((uint32_t)lane / G, 2u);
            uint32_t sm = surv;
            for (uint32_t k = 0; k < sidx && sm; ++k) sm &= sm - 1;
            const uint32_t alt = sm ? (uint32_t)(__ffs((int)sm) - 1) : orig;
            const bool act = (uint32_t)lane < ns * G;
            const uint32_t i = (uint32_t)ia + 1 + 2 * (act ? (uint32_t)lane - sidx * G : 0);
            const uint64_t WB = ext_window(word, i, K, p, alt);
            bool bad = false;
            if (act) {
              const uint32_t r2 = ext_pair(et, WB, K);
              bad = !(r2 & 1) || ((int)i <= ib && !(r2 & 2));
            }
            const uint64_t badm = __ballot(bad);
            sm = surv;
            for (uint32_t s2 = 0; s2 < ns; ++s2) {
              const uint32_t a2 = (uint32_t)(__ffs((int)sm) - 1);
              sm &= sm - 1;
              if (!((badm >> (s2 * G)) & ((1ull << G) - 1))) {
                ++ncand;
                cand = a2;
              }
            }
            n_look += (uint64_t)ns * G;
          }
        } else {
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
        }
        if (ncand == 1) {
          if ((uint32_t)lane == (p >> 4)) {
            const uint32_t sh = 2 * (p & 15);
            word = (word & ~(3u << sh)) | (cand << sh);
            C16 |= 1u << (p & 15);
          }
          last_corr = (int)p;
          const uint32_t nw = (uint32_t)__shfl((int)word, (int)(p >> 4), 64);
          // current quals of the neighbours (registers below 128, then memory)
          auto qat = [&](uint32_t i) -> uint32_t {
            if (i < 64) return (uint32_t)__shfl((int)qa, (int)i, 64);
            if (i < 128) return (uint32_t)__shfl((int)qb, (int)(i - 64), 64);
            return (uint32_t)q[i];
          };
          uint32_t nq = 255;
          if (p > 0) nq = min(nq, qat(p - 1));
          if (p + 1 < L) nq = min(nq, qat(p + 1));
          if ((uint32_t)lane == p) qa = nq;
          if ((uint32_t)lane + 64 == p) qb = nq;
          if (lane == 0) {
            rd[p >> 2] = (uint8_t)(nw >> (8 * ((p >> 2) & 3)));
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

// ---------------------------------------------------------------------------
// Weak-bitmap + extension-table mode (the bench path: K in [9, 29], reads of
// <= kPcMaxL bases) in three kernels, so that the random lookups run with one
// independent work item per lane instead of a wave's dependent chain per read:
//
//   k_pc_candidates (thread per read, quals staged through LDS): the
//     candidates — positions with Q < maxq whose covering K-mers were all
//     counted weak — each with the 2K+1 bases around it, one contiguous run
//     per read.
//   k_pc_decide (thread per candidate): the candidate's decision as if it were
//     a suspect: its base is unchanged since counting and so are the other
//     bases of every covering K-mer (corrections go left to right and a
//     correction within K before it makes it no suspect), so decisions are
//     independent of each other.
//   k_pc_apply (thread per read): the sequential rule — a candidate is a
//     suspect unless a correction lies within K before it — applied in read
//     order, corrections written, counters and clean flags.
// ---------------------------------------------------------------------------
struct PcCand {
  uint64_t wlo, whi;  // bases [p-K, p+K] LSB-first: base p-K+t at bits 2t (0 outside the read)
  uint32_t r;
  uint16_t p, L;
};
constexpr uint8_t kPcAmbiguous = 4, kPcNone = 5, kPcNotSuspect = 6;

// Covering K-mers [jlo, jhi] of read position p all counted weak: bits
// q0 + jlo .. q0 + jhi of the weak-instance bitmap (nk <= K <= 32 bits).
__device__ __forceinline__ bool pc_all_weak(const unsigned long long* __restrict__ weak, uint64_t q0, uint32_t p,
                                            uint32_t L, int K) {
  const uint32_t jlo = p + 1 >= (uint32_t)K ? p + 1 - K : 0;
  const uint32_t jhi = min(p, L - (uint32_t)K);
  const uint32_t nk = jhi - jlo + 1;
  const uint64_t b = q0 + jlo;
  const uint32_t sh = (uint32_t)(b & 63);
  uint64_t x = weak[b >> 6] >> sh;
  if (sh + nk > 64) x |= weak[(b >> 6) + 1] << (64 - sh);
  const uint64_t need = (1ull << nk) - 1;
  return (x & need) == need;
}

// Bases [p-K, p+K] of a packed read (LSB-first, base p-K+t at bits 2t; bases
// before the read 0, after it whatever the slack holds): aligned u32 loads.
__device__ __forceinline__ unsigned __int128 pc_window(const uint8_t* __restrict__ rd, uint32_t p, int K) {
  const int st = (int)p - K;
  const uint32_t s0 = st < 0 ? 0u : (uint32_t)st;  // first base loaded
  const uintptr_t a = (uintptr_t)rd + (s0 >> 2);
  const uint32_t* w = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
  const uint32_t sh = 8 * (uint32_t)(a & 3) + 2 * (s0 & 3);
  // 160 bits >= sh + 118: four words as one 128-bit value, the fifth above it
  unsigned __int128 v = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) v |= (unsigned __int128)w[i] << (32 * i);
  v >>= sh;
  if (sh) v |= (unsigned __int128)w[4] << (128 - sh);
  if (st < 0) v <<= 2 * (uint32_t)(-st);
  return v;
}

// Candidates of reads [r0, r0 + 256) — one thread per read, quals staged
// through LDS.  The tile's quals are one contiguous range of the flat quals
// array: the block copies it with coalesced 16-byte loads (tiles longer than
// kPcTileQ read global memory instead) and each thread scans its read's quals
// from LDS as aligned u32 words for positions with Q < maxq whose covering
// K-mers were all counted weak.  WRITE = false: tcnt[tile] = the tile's
// candidates.  WRITE = true (toff = exclusive scan of tcnt): a block scan of
// the per-read counts places read r's run at [cstart[r], cstart[r] + ccnt[r]),
// in read order, and a second scan from LDS writes the records.
constexpr uint32_t kPcTileReads = 256;
// 28 KiB of staged quals (256 reads of <= 112 bases; longer tiles read global
// memory) and a 1024-entry candidate list keep the block under 40 KiB of LDS:
// four blocks per CU instead of three
constexpr uint32_t kPcTileQ = 28672;

template <typename F>
__device__ __forceinline__ void pc_scan_read(const uint8_t* qb, uint64_t qbase, uint64_t q0, uint32_t L,
                                             uint32_t maxq, F&& f) {
  const uint64_t a0 = q0 & ~3ull;
  for (uint64_t a = a0; a < q0 + L; a += 4) {
    const uint32_t x = *reinterpret_cast<const uint32_t*>(qb + (a - qbase));
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint64_t g = a + k;
      if (g < q0 || g >= q0 + L || ((x >> (8 * k)) & 0xff) >= maxq) continue;
      f((uint32_t)(g - q0));
    }
  }
}

// weak bits of a staged tile: words [wbase, ...) of the bitmap at wb
__device__ __forceinline__ bool pc_all_weak_at(const unsigned long long* wb, uint64_t wbase, uint64_t q0, uint32_t p,
                                               uint32_t L, int K) {
  const uint32_t jlo = p + 1 >= (uint32_t)K ? p + 1 - K : 0;
  const uint32_t jhi = min(p, L - (uint32_t)K);
  const uint32_t nk = jhi - jlo + 1;
  const uint64_t b = q0 + jlo;
  const uint32_t sh = (uint32_t)(b & 63);
  const uint64_t w = (b >> 6) - wbase;
  uint64_t x = wb[w] >> sh;
  if (sh + nk > 64) x |= wb[w + 1] << (64 - sh);
  const uint64_t need = (1ull << nk) - 1;
  return (x & need) == need;
}

constexpr uint32_t kPcTileW = kPcTileQ / 64 + 2;  // weak words of a staged tile
constexpr uint32_t kPcKeep = 4;                   // candidate positions a thread keeps from its first scan
constexpr uint32_t kPcTileList = 1024;            // candidates of a tile written through LDS

constexpr uint32_t kPcQv = kPcTileQ / 16 / kPcTileReads;  // 16-byte quals chunks a thread stages
static_assert(kPcQv * 16 * kPcTileReads == kPcTileQ && kPcTileW <= 2 * kPcTileReads, "staging shape");

// A tile's staged quals chunks (kPcQv = 7 per thread) and weak words (2),
// loaded ahead into named registers: a register array, captured by a lambda
// or returned in a struct, was kept in scratch.  Loads and stores past the end
// are clamped to the last chunk / word rather than predicated.
static_assert(kPcQv == 7, "PC_STAGE names seven chunks");
#define PC_STAGE_CHUNKS(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6)

// Each block walks its tiles r0, r0 + grid, ... (grid = one resident round)
// with the next tile's inputs — the reads' offsets, then its quals and weak
// words — loaded into registers while the current tile is scanned and its
// candidates written, so a tile costs about the candidate window round trip
// and not a chain of dependent loads (8.7 ms on the bench step when each
// tile's staging, offset and window loads waited in turn).
template <bool WRITE>
__global__ void __launch_bounds__(kPcTileReads) k_pc_candidates(
    const uint64_t* __restrict__ base_off, const uint64_t* __restrict__ byte_off, const uint8_t* __restrict__ packed,
    const uint8_t* __restrict__ quals, uint64_t n_reads, int K, uint32_t maxq,
    const unsigned long long* __restrict__ weak, uint32_t* __restrict__ tcnt, const uint64_t* __restrict__ toff,
    PcCand* __restrict__ cand, uint64_t* __restrict__ cstart, uint32_t* __restrict__ ccnt,
    unsigned long long* __restrict__ tctr = nullptr, uint64_t cap = 0) {
  // tctr (WRITE only): single-pass mode — each tile reserves its run of the
  // candidate array with one atomic instead of a counted, scanned offset; a
  // run past `cap` is not written and tctr ends > cap (the host reruns).
  __shared__ unsigned long long tbase_sm;
  __shared__ __attribute__((aligned(16))) uint8_t qs[kPcTileQ + 16];
  __shared__ unsigned long long ws[kPcTileW];
  __shared__ uint64_t bo_s[kPcTileReads + 1], yo_s[kPcTileReads];  // the tile's base / byte offsets
  __shared__ uint32_t list[WRITE ? kPcTileList : 1];  // read in tile << 16 | position
  __shared__ uint32_t scan_sm[64];
  const uint32_t tid = threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * kPcTileReads;
  // staged inputs of the next tile
  uint64_t nbo = 0, nbo_hi = 0, nyo = 0, nQ0 = 0, nQ1 = 0;
  uint4 ng0, ng1, ng2, ng3, ng4, ng5, ng6;
  unsigned long long ngw0, ngw1;
  // the next tile's quals chunks and weak words (after load_offsets)
  auto stage_load = [&]() {
    if (nQ1 - nQ0 > kPcTileQ || nQ1 == nQ0) return;  // a long tile reads global memory directly
    const uint32_t nch = (uint32_t)((nQ1 - nQ0 + 15) >> 4);
    const uint4* src = reinterpret_cast<const uint4*>(quals + nQ0);
#define PC_LD(k) ng##k = src[min(tid + (k) * kPcTileReads, nch - 1)];
    PC_STAGE_CHUNKS(PC_LD)
#undef PC_LD
    if (!weak) return;  // every low-quality position is a candidate
    const uint64_t W0 = nQ0 >> 6;
    const uint32_t nwd = (uint32_t)(((nQ1 + 63) >> 6) - W0 + 1);  // K-mer bits of the tile lie in [Q0, Q1)
    ngw0 = weak[W0 + min(tid, nwd - 1)];
    ngw1 = weak[W0 + min(tid + kPcTileReads, nwd - 1)];
  };
  auto load_offsets = [&](uint64_t t0) {
    const uint64_t te = min(t0 + kPcTileReads, n_reads);
    nQ0 = base_off[t0] & ~15ull;  // block-uniform: scalar loads
    nQ1 = base_off[te];
    nbo = base_off[min(t0 + tid, n_reads)];
    nbo_hi = base_off[te];
    nyo = t0 + tid < n_reads ? byte_off[t0 + tid] : 0;
  };
  uint64_t r0 = (uint64_t)blockIdx.x * kPcTileReads;
  if (r0 < n_reads) {
    load_offsets(r0);
    stage_load();
  }
  for (; r0 < n_reads; r0 += stride) {
    const uint64_t r = r0 + tid;
    const uint64_t Q0 = nQ0, Q1 = nQ1;
    const bool staged = Q1 - Q0 <= kPcTileQ;
    const uint64_t W0 = Q0 >> 6;
    bo_s[tid] = nbo;
    if (tid == 0) bo_s[kPcTileReads] = nbo_hi;
    yo_s[tid] = nyo;
    if (staged && Q1 > Q0) {
      const uint32_t nch = (uint32_t)((Q1 - Q0 + 15) >> 4);
      uint4* dst = reinterpret_cast<uint4*>(qs);
      // past the end every lane rewrites the last chunk / word with the value
      // its clamped load read
#define PC_ST(k) dst[min(tid + (k) * kPcTileReads, nch - 1)] = ng##k;
      PC_STAGE_CHUNKS(PC_ST)
#undef PC_ST
      if (weak) {
        const uint32_t nwd = (uint32_t)(((Q1 + 63) >> 6) - W0 + 1);
        ws[min(tid, nwd - 1)] = ngw0;
        ws[min(tid + kPcTileReads, nwd - 1)] = ngw1;
      }
    }
    __syncthreads();
    const uint64_t nr0 = r0 + stride;
    if (nr0 < n_reads) load_offsets(nr0);  // in flight during the scan
    const uint8_t* qb = staged ? qs : quals;
    const uint64_t qbase = staged ? Q0 : 0;
    const unsigned long long* wb = staged ? ws : weak;
    const uint64_t wbase = staged ? W0 : 0;
    uint64_t q0 = 0;
    uint32_t L = 0;
    if (r < n_reads) {
      q0 = bo_s[tid];
      L = (uint32_t)(bo_s[tid + 1] - q0);
    }
    const bool scan = r < n_reads && L >= (uint32_t)K && L <= kPcMaxL;
    uint32_t n = 0;
    // the first kPcKeep candidates' positions, kept for the list pass (a read
    // with more scans its quals again)
    uint32_t keep[kPcKeep / 2] = {};
    if (scan)
      pc_scan_read(qb, qbase, q0, L, maxq, [&](uint32_t p) {
        if (weak && !pc_all_weak_at(wb, wbase, q0, p, L, K)) return;
#pragma unroll
        for (uint32_t k = 0; k < kPcKeep; ++k)
          if (n == k) keep[k >> 1] |= p << (16 * (k & 1));
        ++n;
      });
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan<uint32_t>(n, scan_sm, &tot);
    if constexpr (!WRITE) {
      if (tid == 0) tcnt[r0 / kPcTileReads] = tot;
      if (nr0 < n_reads) stage_load();
    } else {
      uint64_t tb;
      bool skip = false;
      if (tctr) {
        if (tid == 0) tbase_sm = tot ? atomicAdd(tctr, (unsigned long long)tot) : 0ull;
        __syncthreads();
        tb = tbase_sm;
        skip = tb + tot > cap;  // over capacity: nothing of this tile is written
      } else {
        tb = toff[r0 / kPcTileReads];
      }
      if (nr0 < n_reads) stage_load();  // in flight with the candidate windows
      if (!skip) {
        if (r < n_reads) {
          cstart[r] = tb + ex;
          ccnt[r] = n;
        }
        if (tot <= kPcTileList) {
          // positions into LDS, then one candidate per thread: independent
          // window loads, consecutive records from consecutive threads
          uint32_t at = ex;
          if (n > kPcKeep) {
            pc_scan_read(qb, qbase, q0, L, maxq, [&](uint32_t p) {
              if (!weak || pc_all_weak_at(wb, wbase, q0, p, L, K)) list[at++] = tid << 16 | p;
            });
          } else {
#pragma unroll
            for (uint32_t k = 0; k < kPcKeep; ++k)
              if (k < n) list[at + k] = tid << 16 | ((keep[k >> 1] >> (16 * (k & 1))) & 0xffffu);
          }
          __syncthreads();
          for (uint32_t i = tid; i < tot; i += kPcTileReads) {
            const uint32_t e = list[i];
            const uint32_t rl = e >> 16, pp = e & 0xffff;
            const uint32_t LL = (uint32_t)(bo_s[rl + 1] - bo_s[rl]);
            const unsigned __int128 v = pc_window(packed + yo_s[rl], pp, K);
            cand[tb + i] = PcCand{(uint64_t)v, (uint64_t)(v >> 64), (uint32_t)(r0 + rl), (uint16_t)pp, (uint16_t)LL};
          }
        } else if (n) {
          uint64_t at = tb + ex;
          const uint8_t* rd = packed + yo_s[tid];
          pc_scan_read(qb, qbase, q0, L, maxq, [&](uint32_t p) {
            if (weak && !pc_all_weak_at(wb, wbase, q0, p, L, K)) return;
            const unsigned __int128 v = pc_window(rd, p, K);
            cand[at++] = PcCand{(uint64_t)v, (uint64_t)(v >> 64), (uint32_t)r, (uint16_t)p, (uint16_t)L};
          });
        }
      }
    }
    __syncthreads();  // the LDS tiles are rewritten by the next tile
  }
}

// dec[i] = the candidate's position << 8 | its decision (a base, kPcAmbiguous
// or kPcNone): k_pc_apply reads these 4 bytes, not the 32-byte record.
// wtest (no weak bitmap: ErrorCorrectJump, K < 9, a given solid list): the
// candidates are all low-quality positions, and one whose covering K-mers are
// not all weak — by extension lookups on the read as it was, the state the
// sequential rule sees unless a correction lies within K before it — is
// kPcNotSuspect.
// Covering K-mers a..b of an alternative's window wa (bases [p-K, p+K],
// LSB-first) all solid, through two-level slots: the (K-1)-mer at c answers
// K-mers c-1 and c by its pred / succ bits, c+1 by its successor's successors
// and c-2 by its predecessor's predecessors where those apply (a lookup of
// c-1 of its own where they do not) — as k_ecj_trim.  Needs a linked table.
__device__ __forceinline__ bool pc_all_solid2(const ExtTab& et, unsigned __int128 wa, uint32_t p, int K, int a, int b,
                                              uint32_t* nl) {
  const int o = K - (int)p;  // window index of base q: q + o
  auto bs = [&](int q) { return (uint32_t)(wa >> (2 * (uint32_t)(q + o))) & 3u; };
  auto y1 = [&](int c) { return (uint64_t)(wa >> (2 * (uint32_t)(c + o))) & et.m1; };
  int u = a;
  while (u <= b) {
    const int c = min(u + 2, b + 1);
    ++*nl;
    const uint32_t e = ext_masks2_lsb(et, y1(c));
    const bool sp = (e >> bs(c - 1)) & 1;  // K-mer c-1 (>= u)
    if (c == u + 2) {                      // K-mer u = c-2 first
      bool s2;
      if (sp && ((e >> 17) & 1)) {
        s2 = (e >> (12 + bs(u))) & 1;
      } else {
        ++*nl;
        s2 = (ext_masks_lsb(et, y1(c - 1)) >> bs(u)) & 1;
      }
      if (!s2) return false;
    }
    if (!sp) return false;
    if (c > b) return true;  // c-1 = b was the last
    if (!((e >> (4 + bs(c + K - 1))) & 1)) return false;
    u = c + 1;
    if (u <= b && ((e >> 16) & 1)) {  // K-mer c+1 from the successor's successors
      if (!((e >> (8 + bs(c + K))) & 1)) return false;
      u = c + 2;
    }
  }
  return true;
}

// two: the table carries linked two-level bits (pc_all_solid2 for the
// alternatives)
__global__ void __launch_bounds__(256) k_pc_decide(const PcCand* __restrict__ cand, uint64_t n, int K, ExtTab et,
                                                   uint32_t* __restrict__ dec, unsigned long long* __restrict__ looks,
                                                   bool wtest, bool two) {
  uint32_t nl = 0;
  const unsigned __int128 km = ((unsigned __int128)1 << (2 * (K + 1))) - 1;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const PcCand c = cand[i];
    const unsigned __int128 win = ((unsigned __int128)c.whi << 64) | c.wlo;
    const uint32_t p = c.p, L = c.L;
    const uint32_t orig = (uint32_t)(win >> (2 * K)) & 3;
    const bool hasA = p + 1 >= (uint32_t)K, hasB = p + (uint32_t)K <= L;
    // (A) the (K-1)-mers beside p answer the first and last covering K-mers
    // for all 4 bases at p: succ of bases [p-K+1, p) and pred of [p+1, p+K)
    uint32_t mA = 15, mB = 15;
    if (hasA) {
      mA = ext_masks_lsb(et, (uint64_t)(win >> 2) & et.m1) >> 4;
      ++nl;
    }
    if (hasB) {
      mB = ext_masks_lsb(et, (uint64_t)(win >> (2 * K + 2)) & et.m1) & 15;
      ++nl;
    }
    const uint32_t allowed = mA & mB;
    uint32_t surv = allowed & ~(1u << orig) & 15u;
    // (B) the other covering K-mers a..b, two per (K-1)-mer lookup
    const uint32_t jlo = p + 1 >= (uint32_t)K ? p + 1 - K : 0;
    const uint32_t jhi = min(p, L - (uint32_t)K);
    const int ia = (int)jlo + (hasA ? 1 : 0), ib = (int)jhi - (hasB ? 1 : 0);
    if (wtest) {
      // the weak test: (A) answered the first and last covering K-mers as
      // read (the original base's bits), the others in pairs as in (B)
      bool solid = (hasA && ((mA >> orig) & 1)) || (hasB && ((mB >> orig) & 1));
      for (int t = ia + 1; t <= ib + 1 && !solid; t += 2) {
        const uint64_t W = (uint64_t)((win >> (2 * (uint32_t)(t - 1 - (int)p + K))) & km);
        const uint32_t r2 = ext_pair(et, W, K);
        ++nl;
        solid = (r2 & 1) || (t <= ib && (r2 & 2));
      }
      if (solid) {
        dec[i] = p << 8 | kPcNotSuspect;
        continue;
      }
    }
    uint32_t ncand = 0, cb = 0;
    while (surv) {
      const uint32_t alt = (uint32_t)(__ffs((int)surv) - 1);
      surv &= surv - 1;
      const unsigned __int128 wa = (win & ~((unsigned __int128)3 << (2 * K))) | ((unsigned __int128)alt << (2 * K));
      bool ok = true;
      if (two) ok = pc_all_solid2(et, wa, p, K, ia, ib, &nl);
      for (int j = ia + 1; !two && j <= ib + 1 && ok; j += 2) {
        // (K-1)-mer j with its pred base j-1 and succ base j+K-1: window bits
        // from base j-1 = p-K + (j-1-p+K)
        const uint64_t W = (uint64_t)((wa >> (2 * (uint32_t)(j - 1 - (int)p + K))) & km);
        const uint32_t r2 = ext_pair(et, W, K);
        ++nl;
        ok = (r2 & 1) && (j > ib || (r2 & 2));
      }
      if (ok) {
        ++ncand;
        cb = alt;
      }
    }
    dec[i] = p << 8 | (ncand == 1 ? cb : ncand > 1 ? kPcAmbiguous : kPcNone);
  }
  wave_add(looks, nl);
}

__global__ void __launch_bounds__(256) k_pc_apply(const uint64_t* __restrict__ base_off,
                                                  const uint64_t* __restrict__ byte_off, uint8_t* __restrict__ packed,
                                                  uint8_t* __restrict__ quals, uint64_t n_reads, int K,
                                                  const unsigned long long* __restrict__ weak,
                                                  const uint32_t* __restrict__ dec,
                                                  const uint64_t* __restrict__ cstart,
                                                  const uint32_t* __restrict__ ccnt, uint8_t* __restrict__ clean,
                                                  PcCounters* __restrict__ cnt) {
  uint32_t n_sus = 0, n_cor = 0, n_amb = 0, n_unc = 0;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_reads;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t q0 = base_off[r];
    const uint32_t L = (uint32_t)(base_off[r + 1] - q0);
    if (L < (uint32_t)K) {  // no K-mer, nothing weak
      if (clean) clean[r] = 1;
      continue;
    }
    const uint64_t s0 = cstart[r];
    const uint32_t n = ccnt[r];
    uint8_t* rd = packed + byte_off[r];
    uint8_t* q = quals + q0;
    int last = -(int)kPcMaxL - 64;  // latest correction
    for (uint32_t i = 0; i < n; ++i) {
      const uint32_t pd = dec[s0 + i];
      const uint32_t p = pd >> 8;
      if ((int)p - last < K) continue;  // a covering K-mer holds a correction: solid
      const uint8_t d = (uint8_t)pd;
      if (d == kPcNotSuspect) continue;  // a covering K-mer was solid as read
      ++n_sus;
      if (d < 4) {
        const uint32_t sh = 2 * (p & 3);
        rd[p >> 2] = (uint8_t)((rd[p >> 2] & ~(3u << sh)) | ((uint32_t)d << sh));
        uint32_t nq = 255;
        if (p > 0) nq = min(nq, (uint32_t)q[p - 1]);
        if (p + 1 < L) nq = min(nq, (uint32_t)q[p + 1]);
        q[p] = (uint8_t)nq;
        ++n_cor;
        last = (int)p;
      } else if (d == kPcAmbiguous) {
        ++n_amb;
      } else {
        ++n_unc;
      }
    }
    if (!clean) continue;
    // clean: every counted-weak K-mer j holds a correction c (j <= c < j+K)
    const uint64_t e = q0 + (L - (uint32_t)K + 1);
    bool ok = true;
    for (uint64_t b = q0; b < e && ok; b = (b | 63) + 1) {
      const uint64_t hi = min(e, (b | 63) + 1);
      uint64_t W = weak[b >> 6] >> (b & 63);
      if (hi - b < 64) W &= (1ull << (hi - b)) - 1;
      if (!W) continue;
      // K-mers b .. hi-1 (global bit index) covered by the corrections
      uint64_t D = 0;
      int lc = -(int)kPcMaxL - 64;
      for (uint32_t i = 0; i < n; ++i) {
        const uint32_t pd = dec[s0 + i];
        const uint32_t p = pd >> 8;
        if ((int)p - lc < K) continue;
        if ((pd & 0xff) >= 4) continue;
        lc = (int)p;
        // covered K-mers [p-K+1, p] relative to b - q0
        const int64_t lo = (int64_t)p - K + 1 - (int64_t)(b - q0), up = (int64_t)p - (int64_t)(b - q0);
        if (up < 0 || lo >= 64) continue;
        const int a = lo < 0 ? 0 : (int)lo, z = up > 63 ? 63 : (int)up;
        D |= (z - a == 63 ? ~0ull : ((1ull << (z - a + 1)) - 1)) << a;
      }
      ok = (W & ~D) == 0;
    }
    clean[r] = ok ? 1 : 0;
  }
  wave_add(&cnt->suspect, n_sus);
  wave_add(&cnt->corrected, n_cor);
  wave_add(&cnt->ambiguous, n_amb);
  wave_add(&cnt->uncorrectable, n_unc);
}

// One correction pass of every read of `dr` against the solid hash list.
// weak: the pass's weak-instance bitmap (sk_solid_weak) or null (weak tests
// by lookups); with it, the pass also leaves per-read clean flags ("pc_clean":
// 1 every K-mer solid after correction, 0 not, 2 not derived) for
// FillFragments.
static int correct_pass(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params& p, const uint64_t* list, uint64_t n_solid,
                        apg_pc_stats* st, const unsigned long long* weak = nullptr, bool self_count = false) {
  ctx->clean_valid = false;
  ctx->ws_dead &= ~kRoomCorrection;  // the correction tables are live again
  APG_TRY(dreads_quals_ready(dr));  // the candidate scan reads them (a load may still stream them in)
  // the previous pass's extension table is this very list's (the jump reads'
  // pass of ErrorCorrectJump against the fragments' reused solid set)
  const bool ext_reuse = ctx->pc_ext_valid && ctx->pc_list_valid && ctx->pc_list == list && ctx->pc_n == n_solid &&
                         ctx->pc_K == p.K && !weak;
  ctx->pc_self = false;
  uint8_t* clean = nullptr;
  if (weak) APG_TRY(workspace_t(ctx, "pc_clean", std::max<uint64_t>(dr->n_reads, 1), &clean));
  unsigned long long* dcnt = nullptr;
  APG_TRY(workspace_t(ctx, "pc_counters", 8, &dcnt));
  APG_CHECK_HIP(hipMemsetAsync(dcnt, 0, 8 * 8, ctx->stream));
  const HashP hp = make_hashp(p.K);
  // (K-1)-mer extension lookups (2 <= K <= 29, reads that fit one wave's
  // registers), else K-mer lookups in a hash set behind a prefix bitmap
  const bool ext = p.K >= 2 && p.K <= 29 && dr->max_len <= kPcMaxL;
  SolidSet ss{};
  ExtTab et{};
  ctx->pc_ext_valid = false;
  // With the weak bitmap the candidate scan needs no table: the extension
  // table is built on the auxiliary stream beside it (random atomics beside
  // a streaming scan), the decisions waiting for it by an event
  // (APG_PC_EXT_AUX=0: in line).  Same box: 152.3 -> 150.8 ms per bench step
  // once the fused K+1 pass moved after the scan; with the K+1 pass beside
  // the scan as well it gained nothing (172.4 vs 171.9 ms).
  hipEvent_t ext_done = nullptr, link_done = nullptr;
  // Where the two-level link pass runs (APG_PC_LINK_AT): 3 (default) right
  // behind the inserts, the decisions behind it reading the two-level bits
  // (4.1 ms instead of 10.5: an alternative's covering K-mers at up to four
  // per lookup); 1 after the decisions, beside the edits; 0 behind the
  // inserts beside one-level decisions; 2 as 0 on APG_PC_LINK_FRAC (0.25) of
  // its grid.  Same box, ms per bench step: 3: 145.95 / 146.0, 1: 146.85 /
  // 146.94; earlier, 1: 144.5 vs 0: 145.4-146.0 (decisions 10.6 vs 15.1 ms);
  // the K+1 pass kicked after the decisions (APG_SK_UP_AT=3) exposes it.
  static const int link_at = [] {
    const char* e = getenv("APG_PC_LINK_AT");
    return e ? atoi(e) : 3;
  }();
  static const double link_frac = [] {
    const char* e = getenv("APG_PC_LINK_FRAC");
    return e ? std::min(1.0, std::max(0.01, atof(e))) : 0.25;
  }();
  // APG_PC_LINK_AT=3: the link pass right behind the inserts and the
  // decisions behind it, so they read the two-level bits too
  const bool link_late = link_at == 1;
  bool link_pending = false;  // the table's link pass still to launch (link_late)
  bool linked_first = false;  // the decisions wait for the link pass (link_at 3)
  if (ext && weak) {
    const char* ae = getenv("APG_PC_EXT_AUX");
    const hipStream_t ax = (ae && !strcmp(ae, "0")) ? nullptr : aux_stream(ctx);
    if (ax) {
      hipEvent_t ready = nullptr;
      APG_CHECK_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
      APG_CHECK_HIP(hipEventCreateWithFlags(&ext_done, hipEventDisableTiming));
      APG_CHECK_HIP(hipEventRecord(ready, ctx->stream));  // the solid list is complete
      APG_CHECK_HIP(hipStreamWaitEvent(ax, ready, 0));
      APG_CHECK_HIP(hipEventDestroy(ready));
      // The decisions read only the pred / succ bits: they wait for the
      // inserts, and the two-level link pass (FillFragments' bits) runs on
      // behind them; the pass joins the main stream before PreCorrect returns.
      int rc;
      {
        StreamSwap sw(ctx, ax);
        rc = ext_build(ctx, list, n_solid, p.K, "pc_ext", "solid_insert", &et, false);
        if (rc == APG_OK && link_at == 3) {
          rc = ext_link(ctx, et, n_solid);
          linked_first = rc == APG_OK && et.ks == 16;
        }
        if (rc == APG_OK && hipEventRecord(ext_done, ax) != hipSuccess) rc = APG_E_HIP;
        if (rc == APG_OK && !link_late && link_at != 3) rc = ext_link(ctx, et, n_solid, link_at == 2 ? link_frac : 1.0);
        link_pending = rc == APG_OK && link_late && et.ks == 16;
        if (rc == APG_OK && et.ks == 16 && !link_late && link_at != 3) {
          if (hipEventCreateWithFlags(&link_done, hipEventDisableTiming) != hipSuccess ||
              hipEventRecord(link_done, ax) != hipSuccess)
            rc = APG_E_HIP;
        }
      }
      if (rc != APG_OK) {
        (void)hipStreamSynchronize(ax);
        (void)hipEventDestroy(ext_done);
        if (link_done) (void)hipEventDestroy(link_done);
        return rc;
      }
    }
  }
  // an early return leaves no table build running behind it
  struct ExtGuard {
    hipEvent_t *ev, *lk;
    hipStream_t ax;
    ~ExtGuard() {
      if (*ev || *lk) (void)hipStreamSynchronize(ax);
      if (*ev) (void)hipEventDestroy(*ev);
      if (*lk) (void)hipEventDestroy(*lk);
    }
  } ext_guard{&ext_done, &link_done, ctx->aux};
  // the main stream's wait for the table (no host sync); idempotent
  auto ext_wait = [&]() -> int {
    if (!ext_done) return APG_OK;
    APG_CHECK_HIP(hipStreamWaitEvent(ctx->stream, ext_done, 0));
    APG_CHECK_HIP(hipEventDestroy(ext_done));
    ext_done = nullptr;
    return APG_OK;
  };
  if (ext && !weak && ext_reuse) {
    et = ext_tab(ctx->pc_ext_slot, ctx->pc_ext_mask, p.K);
  } else if (ext && !weak) {
    APG_TRY(ext_build(ctx, list, n_solid, p.K, "pc_ext", "solid_insert", &et));
  } else if (ext) {
    if (!ext_done) APG_TRY(ext_build(ctx, list, n_solid, p.K, "pc_ext", "solid_insert", &et));
    APG_TRY(side_kick(ctx, 1));  // a deferred side pass (the fused K+1 count) starts here
  } else {
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
    ss = SolidSet{table, T - 1, bitmap, 2 * p.K - mb};
  }
  APG_CHECK_HIP(hipGetLastError());
  PcCounters* pcnt = reinterpret_cast<PcCounters*>(dcnt);
  // Without a weak bitmap (ErrorCorrectJump's jump reads, K < 9, a given
  // solid list) the same three kernels run with every low-quality position a
  // candidate and the weak test by lookups in the decisions; APG_PC_WAVE=1:
  // the wave-per-read kernel instead (A/B; C3's 20 M jump reads took 29 ms
  // there, a dependent chain of lookups per read).
  const char* pwe = getenv("APG_PC_WAVE");
  const bool cand3 = ext && (weak || !(pwe && !strcmp(pwe, "1")));
  if (cand3) {
    // candidates -> independent decisions -> sequential rule per read
    uint32_t* ccnt = nullptr;
    uint64_t* cstart = nullptr;
    const uint64_t nr1 = std::max<uint64_t>(dr->n_reads, 1);
    APG_TRY(workspace_t(ctx, "pc_ccnt", nr1, &ccnt));
    APG_TRY(workspace_t(ctx, "pc_cstart", nr1, &cstart));
    const uint64_t ntiles = (dr->n_reads + kPcTileReads - 1) / kPcTileReads;
    uint32_t* tcnt = nullptr;
    uint64_t* toff = nullptr;
    APG_TRY(workspace_t(ctx, "pc_tcnt", std::max<uint64_t>(ntiles, 1), &tcnt));
    APG_TRY(workspace_t(ctx, "pc_toff", ntiles + 1, &toff));
    // one resident round: each block pipelines its tiles
    const uint32_t cgrid = std::min<uint32_t>(resident_grid(ctx, k_pc_candidates<true>, kPcTileReads, ntiles),
                                              resident_grid(ctx, k_pc_candidates<false>, kPcTileReads, ntiles));
    // Single pass when the previous call's candidate count gives a capacity:
    // tiles reserve their runs with one atomic each (no counting pass, no
    // scan); an overflow falls back to count + scan + write.
    uint64_t ncand = 0;
    PcCand* cand = nullptr;
    bool have = false;
    uint64_t& hint = weak ? ctx->pc_cand_hint : ctx->pc_cand_hint_lk;
    const uint64_t cap = hint;
    if (cap && dr->n_reads) {
      unsigned long long* ctr = nullptr;
      APG_TRY(workspace_t(ctx, "pc_cand_ctr", 1, &ctr));
      APG_CHECK_HIP(hipMemsetAsync(ctr, 0, 8, ctx->stream));
      APG_TRY(workspace_t(ctx, "pc_cand", cap, &cand));
      kbegin(ctx, "pc_cand_write",
             dr->n_bases + (weak ? dr->n_bases / 8 : 0) + 8 * dr->n_reads + 12 * dr->n_reads);
      k_pc_candidates<true><<<cgrid, kPcTileReads, 0, ctx->stream>>>(
          dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->d_quals, dr->n_reads, p.K, p.max_q_suspect, weak, nullptr,
          nullptr, cand, cstart, ccnt, ctr, cap);
      kend(ctx);
      APG_CHECK_HIP(hipGetLastError());
      unsigned long long hn = 0;
      APG_TRY(d2h_sync(ctx, &hn, ctr, 8));
      ncand = hn;
      have = ncand <= cap;
      if (have) kbytes_add(ctx, "pc_cand_write", ncand * sizeof(PcCand));
    }
    if (!have) {
      // reads' offsets + quals + weak bits in; tile counts out
      kbegin(ctx, "pc_candidates", dr->n_bases + (weak ? dr->n_bases / 8 : 0) + 8 * dr->n_reads);
      if (dr->n_reads)
        k_pc_candidates<false><<<cgrid, kPcTileReads, 0, ctx->stream>>>(
            dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->d_quals, dr->n_reads, p.K, p.max_q_suspect, weak, tcnt,
            nullptr, nullptr, nullptr, nullptr);
      kend(ctx);
      APG_CHECK_HIP(hipGetLastError());
      APG_TRY(scan_u32_u64(ctx, tcnt, ntiles, toff, "pct"));
      APG_TRY(d2h_sync(ctx, &ncand, toff + ntiles, 8));
      APG_TRY(workspace_t(ctx, "pc_cand", std::max<uint64_t>(ncand, 1), &cand));
      // reads' offsets + quals + weak bits in; runs and records out
      kbegin(ctx, "pc_cand_write", dr->n_bases + (weak ? dr->n_bases / 8 : 0) + 8 * dr->n_reads + 12 * dr->n_reads +
                                       ncand * sizeof(PcCand));
      if (dr->n_reads)
        k_pc_candidates<true><<<cgrid, kPcTileReads, 0, ctx->stream>>>(
            dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->d_quals, dr->n_reads, p.K, p.max_q_suspect, weak,
            nullptr, toff, cand, cstart, ccnt);
      kend(ctx);
      APG_CHECK_HIP(hipGetLastError());
    }
    APG_TRY(side_kick(ctx, 2));
    hint = ncand + ncand / 4 + 4096;
    uint32_t* dec = nullptr;
    APG_TRY(workspace_t(ctx, "pc_dec", std::max<uint64_t>(ncand, 1), &dec));
    // candidate records in, decisions out (+ 64 B per extension lookup, after the sync)
    APG_TRY(ext_wait());
    // the alternatives through the two-level bits when the table is linked
    // by now: the pass's own inline build or a reused one (ErrorCorrectJump's
    // jump reads), not the weak path's, whose link pass runs after the
    // decisions (APG_PC_TWO=0: pairs as before)
    static const bool two_env = !(getenv("APG_PC_TWO") && !strcmp(getenv("APG_PC_TWO"), "0"));
    const bool pc_two = two_env && et.ks == 16 && (!weak || linked_first);
    kbegin(ctx, "precorrect", ncand * (sizeof(PcCand) + 4));
    if (ncand)
      k_pc_decide<<<grid_for(ctx, ncand), 256, 0, ctx->stream>>>(cand, ncand, p.K, et, dec, &pcnt->lookups, !weak,
                                                                  pc_two);
    kend(ctx);
    APG_TRY(side_kick(ctx, 3));  // APG_SK_UP_AT=3: the K+1 pass behind the decisions' dispatch
    if (link_pending) {
      link_pending = false;
      // the table is complete (the decisions waited for it): the link pass on
      // the auxiliary stream from here, joined before PreCorrect returns
      hipEvent_t go = nullptr;
      APG_CHECK_HIP(hipEventCreateWithFlags(&go, hipEventDisableTiming));
      APG_CHECK_HIP(hipEventRecord(go, ctx->stream));
      APG_CHECK_HIP(hipStreamWaitEvent(ctx->aux, go, 0));
      APG_CHECK_HIP(hipEventDestroy(go));
      APG_CHECK_HIP(hipEventCreateWithFlags(&link_done, hipEventDisableTiming));
      {
        StreamSwap sw(ctx, ctx->aux);
        APG_TRY(ext_link(ctx, et, n_solid));
      }
      APG_CHECK_HIP(hipEventRecord(link_done, ctx->aux));
    }
    // offsets, runs, the candidates' positions and decisions, weak bits in;
    // corrected bases and quals, clean flags out
    kbegin(ctx, "pc_apply",
           16 * dr->n_reads + 8 * dr->n_reads + ncand * 4 + (weak ? dr->n_bases / 8 + dr->n_reads : 0));
    if (dr->n_reads)
      k_pc_apply<<<grid_for(ctx, dr->n_reads), 256, 0, ctx->stream>>>(
          dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->d_quals, dr->n_reads, p.K, weak, dec, cstart, ccnt, clean,
          pcnt);
    kend(ctx);
  } else {
    // reads + quals (+ the weak bitmap and the clean flags)
    kbegin(ctx, "precorrect", dr->n_bytes + dr->n_bases + (weak ? dr->n_bases / 8 + dr->n_reads : 0));
    if (dr->n_reads) {
      if (ext)
        k_precorrect_wave<true><<<grid_for(ctx, dr->n_reads, 4), 256, 0, ctx->stream>>>(
            dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->d_quals, dr->n_reads, p.K, hp, p.max_q_suspect, ss, et,
            weak, clean, reinterpret_cast<PcCounters*>(dcnt));
      else
        k_precorrect_wave<false><<<grid_for(ctx, dr->n_reads, 4), 256, 0, ctx->stream>>>(
            dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->d_quals, dr->n_reads, p.K, hp, p.max_q_suspect, ss, et,
            weak, clean, reinterpret_cast<PcCounters*>(dcnt));
    }
    kend(ctx);
    if (dr->max_len > kPcMaxL) {  // reads longer than one wave's registers: thread per read
      const uint64_t rgrid =
          std::max<uint64_t>(1, std::min<uint64_t>((dr->n_reads + 255) / 256, (uint64_t)ctx->n_cu * 32));
      k_precorrect<<<rgrid, 256, 0, ctx->stream>>>(dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->d_quals,
                                                   dr->n_reads, p.K, hp, p.max_q_suspect, ss, kPcMaxL + 1, clean,
                                                   reinterpret_cast<PcCounters*>(dcnt));
    }
  }
  APG_CHECK_HIP(hipGetLastError());
  if (link_done) {  // the two-level bits complete before the table is handed on
    APG_CHECK_HIP(hipStreamWaitEvent(ctx->stream, link_done, 0));
    APG_CHECK_HIP(hipEventDestroy(link_done));
    link_done = nullptr;
  }
  unsigned long long h[6];
  APG_TRY(d2h_sync(ctx, h, dcnt, sizeof h));
  // extension lookup: a random 64-byte HBM line; K-mer set: a bitmap query
  // reads one word of an L3-resident bitmap (counted 4 B), a table probe a
  // random 64-byte line
  kbytes_add(ctx, "precorrect", ext ? h[4] * 64 : h[4] * 4 + h[5] * 64);
  vlog(ctx, "precorrect: %llu solid-set queries, %llu table probes", h[4], h[5]);
  st->n_suspect += h[0];
  st->n_corrected += h[1];
  st->n_ambiguous += h[2];
  st->n_uncorrectable += h[3];
  st->n_solid = n_solid;
  st->record_form = ctx->sk_record_form;
  ctx->pc_list = list;  // APG_FILL_LAST_SOLID (FillFragments after correction)
  ctx->pc_n = n_solid;
  ctx->pc_K = p.K;
  ctx->pc_list_valid = true;
  if (ext) {
    ctx->pc_ext_slot = et.slot;
    ctx->pc_ext_mask = et.mask;
    ctx->pc_ext_valid = true;
  }
  vlog(ctx, "precorrect pass: solid=%llu suspect=%llu corrected=%llu ambiguous=%llu none=%llu",
       (unsigned long long)n_solid, h[0], h[1], h[2], h[3]);
  static std::atomic<uint64_t> g_edit{1ull << 62};
  dr->gen = g_edit.fetch_add(1);  // bases changed: invalidate per-read-set plans
  ctx->pc_self = self_count;
  ctx->pc_self_gen = dr->gen;
  ctx->pc_self_list = list;
  ctx->pc_self_n = n_solid;
  ctx->pc_min_solid = p.min_solid;
  if (clean) {
    ctx->pc_clean = clean;
    ctx->clean_gen = dr->gen;
    ctx->clean_valid = true;
  }
  return APG_OK;
}

// up_res: the fused K+1 spectrum of the uncorrected reads rides on the count
// (apg_spectrum_precorrect_dev; sk_can_fuse_up(p.K))
static int precorrect_pass(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params& p, apg_pc_stats* st,
                           uint64_t* up_hist = nullptr, size_t up_hist_len = 0, SkResult* up_res = nullptr,
                           bool join = true) {
  SkResult sr;
  if (p.K >= 9) {  // count + the weak-instance bitmap (no lookups for the weak tests)
    unsigned long long* weak = nullptr;
    APG_TRY(workspace_t(ctx, "pc_weak", dr->n_bases / 64 + 2, &weak));
    APG_TRY(sk_solid_weak(ctx, dr, p.K, p.min_solid, weak, &sr, up_hist, up_hist_len, up_res));
    ctx->solid_valid = false;  // "pc_solid" now holds this pass's list
    // the fused K+1 pass may still run on the side stream: joined here, after
    // the correction kernels it overlaps (join = false: by the caller, after
    // FillFragments — apg_spectrum_precorrect_fill_dev)
    const int rc = correct_pass(ctx, dr, p, sr.solid, sr.n_solid, st, weak, true);
    if (!join && rc == APG_OK) return APG_OK;
    const int rj = side_join(ctx);
    return rc != APG_OK ? rc : rj;
  }
  APG_TRY(sk_spectrum(ctx, dr, p.K, true, p.min_solid, nullptr, 0, &sr));
  ctx->solid_valid = false;
  return correct_pass(ctx, dr, p, sr.solid, sr.n_solid, st, nullptr, true);
}

static int check_pc(const apg_pc_params& p) {
  APG_REQUIRE(p.K >= 1 && p.K <= 32, "apg_precorrect: K must be in [1, 32]");
  APG_REQUIRE(p.min_solid >= 1, "apg_precorrect: min_solid must be >= 1");
  APG_REQUIRE(p.n_cycles >= 1 && p.n_cycles <= 16, "apg_precorrect: n_cycles must be in [1, 16]");
  return APG_OK;
}

// Multi-GPU weak-mask return, source side: every sent record whose owner
// reported weak K-mers ORs its mask into the per-base weak bitmap at the
// record's position (masks come back in send order).
__global__ void k_weak_apply(const uint64_t* __restrict__ pos, const uint32_t* __restrict__ mask, uint64_t n,
                             unsigned long long* __restrict__ weak) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t m = mask[i];
    if (!m) continue;
    const uint64_t b = pos[i];
    const uint32_t sh = (uint32_t)(b & 63);
    atomicOr(&weak[b >> 6], (unsigned long long)(m << sh));
    if (sh && (m >> (64 - sh))) atomicOr(&weak[(b >> 6) + 1], (unsigned long long)(m >> (64 - sh)));
  }
}

// ---------------------------------------------------------------------------
// ErrorCorrectJump (spec in include/apg.h; CPU restatement oracle/ecj_oracle.c
// + the PreCorrect restatement).  After the correction pass, k_ecj_trim finds
// each read's first non-solid K-mer through the pass's (K-1)-mer extension
// table: K-mer i is solid <=> the successor mask of the (K-1)-mer at i holds
// base i+K-1, one table line per K-mer, stopping at the first miss.
// ---------------------------------------------------------------------------
struct EcjReads {
  const uint64_t* base_off;
  const uint64_t* byte_off;
  const uint8_t* packed;
  uint64_t n_reads;
};

__global__ void __launch_bounds__(256) k_ecj_trim(EcjReads rv, ExtTab et, int K, uint32_t min_keep,
                                                  uint32_t* __restrict__ keep, unsigned long long* __restrict__ cnt) {
  uint64_t n_full = 0, n_trim = 0, n_drop = 0, kept = 0, looks = 0;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rv.n_reads;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t L = (uint32_t)(rv.base_off[r + 1] - rv.base_off[r]);
    const uint8_t* rd = rv.packed + rv.byte_off[r];
    uint32_t k = 0;
    if (L >= (uint32_t)K) {
      // One lookup per two K-mers: the (K-1)-mer at i+1 answers K-mer i by
      // its predecessor bit for base i and K-mer i+1 by its successor bit for
      // base i+K (ext_table.hpp).  i = the first non-solid K-mer, or nk.
      const int n1 = K - 1;
      auto base = [&](uint32_t x) -> uint32_t { return (rd[x >> 2] >> (2 * (x & 3))) & 3; };
      const uint32_t nk = L - K + 1;
      uint32_t i = nk;
      if (et.ks == 16) {
        // Two-level slots: the (K-1)-mer at c also answers K-mer c+1 by its
        // successor's successor mask (when it has one successor) and K-mer
        // c-2 by its predecessor's predecessor mask (when it has one
        // predecessor): one lookup per four K-mers along a solid read, in
        // order, with a lookup of c-1 of its own where the pp bits do not
        // apply.  u = the first K-mer not yet known solid.
        uint64_t y = 0;  // (K-1)-mer at c, LSB-first: base c+t at bits 2t
        for (int t = 0; t < n1; ++t) y |= (uint64_t)base(t) << (2 * t);
        uint32_t u = 0, c = 0;
        while (u < nk) {
          const uint32_t cn = min(u + 2, nk);
          for (; c < cn; ++c) y = (y >> 2) | ((uint64_t)base(c + (uint32_t)n1) << (2 * (n1 - 1)));
          ++looks;
          const uint32_t e = ext_masks2_lsb(et, y);
          const bool sp = (e >> base(c - 1)) & 1;  // K-mer c-1 (>= u)
          if (c == u + 2) {                        // K-mer u = c-2 first
            bool s2;
            if (sp && ((e >> 17) & 1)) {
              s2 = (e >> (12 + base(u))) & 1;
            } else {
              ++looks;
              s2 = (ext_masks_lsb(et, ((y << 2) & et.m1) | base(c - 1)) >> base(u)) & 1;
            }
            if (!s2) {
              i = u;
              break;
            }
          }
          if (!sp) {
            i = c - 1;
            break;
          }
          if (c == nk) break;  // K-mers [0, nk) all solid
          if (!((e >> (4 + base(c + (uint32_t)n1))) & 1)) {
            i = c;
            break;
          }
          u = c + 1;
          if (u < nk && ((e >> 16) & 1)) {  // K-mer c+1 from the successor's successors
            if (!((e >> (8 + base(c + (uint32_t)n1 + 1))) & 1)) {
              i = u;
              break;
            }
            u = c + 2;
          }
        }
      } else {
      uint64_t y = 0;  // (K-1)-mer at i+1, LSB-first: base i+1+t at bits 2t
      for (int t = 0; t < n1; ++t) y |= (uint64_t)base(1 + t) << (2 * t);
      // kEcjBatch lookups in flight per lane: the (K-1)-mers of a batch
      // follow from the bases alone, so they are issued together and checked
      // in order (a read is almost always solid to its end after correction:
      // the lookups past its first non-solid K-mer are few)
      constexpr uint32_t kEcjBatch = 4;
      for (uint32_t i0 = 0; i0 < nk && i == nk; i0 += 2 * kEcjBatch) {
        ExtProbe pr[kEcjBatch];
#pragma unroll
        for (uint32_t b = 0; b < kEcjBatch; ++b) {
          const uint32_t ib = i0 + 2 * b;
          if (ib < nk) pr[b] = ext_issue_lsb(et, y);
          if (ib + 2 < nk) {
            y = (y >> 2) | ((uint64_t)base(ib + (uint32_t)K) << (2 * (n1 - 1)));
            y = (y >> 2) | ((uint64_t)base(ib + (uint32_t)K + 1) << (2 * (n1 - 1)));
          }
        }
#pragma unroll
        for (uint32_t b = 0; b < kEcjBatch; ++b) {
          const uint32_t ib = i0 + 2 * b;
          if (i != nk || ib >= nk) continue;
          ++looks;
          const uint32_t m = ext_finish(et, pr[b]);
          if (!(m & (1u << base(ib)))) {
            i = ib;
          } else if (ib + 1 < nk && !((m >> 4) & (1u << base(ib + (uint32_t)K)))) {
            i = ib + 1;
          }
        }
      }
      }
      k = i == nk ? L : i + (uint32_t)n1;
      if (k < min_keep) k = 0;
    }
    keep[r] = k;
    n_full += k == L && L > 0;
    n_trim += k && k < L;
    n_drop += k == 0;
    kept += k;
  }
  wave_add(&cnt[0], n_full);
  wave_add(&cnt[1], n_trim);
  wave_add(&cnt[2], n_drop);
  wave_add(&cnt[3], kept);
  wave_add(&cnt[4], looks);
}

static int ecj_run(apg_ctx* ctx, const apg_dreads* fr, apg_dreads* jr, const apg_ecj_params& e, uint32_t* d_keep,
                   apg_ecj_stats* st) {
  APG_REQUIRE(e.K >= 2 && e.K <= 29, "apg_error_correct_jump: K must be in [2, 29]");
  APG_REQUIRE(e.min_solid >= 1, "apg_error_correct_jump: min_solid must be >= 1");
  APG_REQUIRE(jr->n_reads == 0 || jr->d_quals, "apg_error_correct_jump: jump reads have no qualities");
  APG_REQUIRE(jr->n_reads == 0 || d_keep, "apg_error_correct_jump: keep_len is NULL");
  ctx->ws_dead &= ~kRoomCorrection;  // the fragments' solid set and table may be reused
  // solid set of the fragment reads: when they are the output of this
  // context's last counting correction pass (same K, same min_solid), that
  // pass's list is their solid set exactly (apg_core.hpp pc_self: a pass
  // leaves the solid set unchanged) — C3's recount of the 40 M corrected
  // fragment reads is skipped; else counted here
  SkResult sr;
  if (ctx->pc_list_valid && ctx->pc_self && ctx->pc_self_gen == fr->gen && ctx->pc_K == e.K &&
      ctx->pc_min_solid == e.min_solid && ctx->pc_self_list == ctx->pc_list && ctx->pc_self_n == ctx->pc_n) {
    sr.solid = const_cast<uint64_t*>(ctx->pc_list);
    sr.n_solid = ctx->pc_n;
    vlog(ctx, "error_correct_jump: the fragments' solid set from their correction pass (%llu K-mers)",
         (unsigned long long)sr.n_solid);
  } else {
    APG_TRY(sk_spectrum(ctx, fr, e.K, true, e.min_solid, nullptr, 0, &sr));
    ctx->solid_valid = false;  // "pc_solid" now holds the fragments' list
  }
  return ecj_with_solid(ctx, jr, e, sr.solid, sr.n_solid, d_keep, st);
}

}  // namespace apg

namespace apg {
// ErrorCorrectJump's correction pass and trim of the jump reads against a
// given solid list of the fragment reads (ecj_run's count, or the replicated
// list of a sharded pass: apg_sharded_error_correct_jump)
int ecj_with_solid(apg_ctx* ctx, apg_dreads* jr, const apg_ecj_params& e, const uint64_t* solid, uint64_t n_solid,
                   uint32_t* d_keep, apg_ecj_stats* st) {
  APG_REQUIRE(e.K >= 2 && e.K <= 29, "apg_error_correct_jump: K must be in [2, 29]");
  APG_REQUIRE(jr->n_reads == 0 || jr->d_quals, "apg_error_correct_jump: jump reads have no qualities");
  APG_REQUIRE(jr->n_reads == 0 || d_keep, "apg_error_correct_jump: keep_len is NULL");
  apg_pc_params p;
  std::memset(&p, 0, sizeof p);
  p.K = e.K;
  p.min_solid = e.min_solid;
  p.max_q_suspect = e.max_q_suspect;
  p.n_cycles = 1;
  struct {
    uint64_t* solid;
    uint64_t n_solid;
  } sr{const_cast<uint64_t*>(solid), n_solid};
  // one correction pass of the jump reads against it
  std::memset(st, 0, sizeof *st);
  APG_TRY(correct_pass(ctx, jr, p, sr.solid, sr.n_solid, &st->pc));
  ExtTab et{};
  if (ctx->pc_ext_valid && ctx->pc_list == sr.solid && ctx->pc_K == e.K)
    et = ext_tab(ctx->pc_ext_slot, ctx->pc_ext_mask, e.K);
  else
    APG_TRY(ext_build(ctx, sr.solid, sr.n_solid, e.K, "ecj_ext", "ecj_ext", &et));
  unsigned long long* cnt = nullptr;
  APG_TRY(workspace_t(ctx, "ecj_cnt", 5, &cnt));
  APG_CHECK_HIP(hipMemsetAsync(cnt, 0, 5 * 8, ctx->stream));
  kbegin(ctx, "ecj_trim", jr->n_bytes + 20 * jr->n_reads);
  if (jr->n_reads)
    k_ecj_trim<<<grid_for(ctx, jr->n_reads), 256, 0, ctx->stream>>>(
        EcjReads{jr->d_base_off, jr->d_byte_off, jr->d_packed, jr->n_reads}, et, e.K, e.min_keep, d_keep, cnt);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  unsigned long long h[5];
  APG_TRY(d2h_sync(ctx, h, cnt, sizeof h));
  kbytes_add(ctx, "ecj_trim", h[4] * 64);
  st->n_reads = jr->n_reads;
  st->n_full = h[0];
  st->n_trimmed = h[1];
  st->n_dropped = h[2];
  st->bases_kept = h[3];
  return APG_OK;
}

}  // namespace apg

using namespace apg;

extern "C" {

void apg_ecj_defaults(apg_ecj_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->K = 24;
  p->min_solid = 3;
  p->max_q_suspect = 20;
  p->min_keep = 40;
}

int apg_error_correct_jump_dev(apg_ctx* ctx, const apg_dreads* frags, apg_dreads* jumps, const apg_ecj_params* pp,
                               uint32_t* d_keep_len, apg_ecj_stats* stats) {
  APG_REQUIRE(ctx && frags && jumps, "apg_error_correct_jump_dev: NULL argument");
  apg_ecj_params e;
  if (pp)
    e = *pp;
  else
    apg_ecj_defaults(&e);
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  apg_ecj_stats st;
  APG_TRY(ecj_run(ctx, frags, jumps, e, d_keep_len, &st));
  if (stats) *stats = st;
  return APG_OK;
}

int apg_error_correct_jump(apg_ctx* ctx, const apg_reads* frags, const apg_reads* jumps, const apg_ecj_params* p,
                           uint8_t* out_packed, uint8_t* out_quals, uint32_t* keep_len, apg_ecj_stats* stats) {
  APG_REQUIRE(ctx && frags && jumps, "apg_error_correct_jump: NULL argument");
  APG_REQUIRE(jumps->n_reads == 0 || (out_packed && out_quals && keep_len && jumps->quals),
              "apg_error_correct_jump: NULL output or jump qualities");
  apg_dreads *dF = nullptr, *dJ = nullptr;
  APG_TRY(apg_reads_upload(ctx, frags, &dF));
  int rc = apg_reads_upload(ctx, jumps, &dJ);
  uint32_t* dk = nullptr;
  if (rc == APG_OK) rc = workspace_t(ctx, "ecj_keep", std::max<uint64_t>(jumps->n_reads, 1), &dk);
  if (rc == APG_OK) rc = apg_error_correct_jump_dev(ctx, dF, dJ, p, dk, stats);
  if (rc == APG_OK) rc = apg_reads_download(ctx, dJ, out_packed, out_quals);
  if (rc == APG_OK && jumps->n_reads &&
      hipMemcpy(keep_len, dk, jumps->n_reads * 4, hipMemcpyDeviceToHost) != hipSuccess) {
    set_error("apg_error_correct_jump: D2H failed");
    rc = APG_E_HIP;
  }
  apg_reads_free(dF);
  apg_reads_free(dJ);
  return rc;
}

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

int apg_spectrum_precorrect_dev(apg_ctx* ctx, apg_dreads* dr, int K_spec, uint64_t* hist, size_t hist_len,
                                apg_kstats* kstats, const apg_pc_params* pp, apg_pc_stats* pstats) {
  return spectrum_precorrect_impl(ctx, dr, K_spec, hist, hist_len, kstats, pp, pstats, true);
}
}  // extern "C"

namespace apg {
// apg_spectrum_precorrect_dev; join = false (one cycle only) leaves the fused
// K+1 pass on the side stream for the caller to join (side_join) — its
// records and buckets must stay untouched until then, and hist / kstats are
// filled by that join
int spectrum_precorrect_impl(apg_ctx* ctx, apg_dreads* dr, int K_spec, uint64_t* hist, size_t hist_len,
                             apg_kstats* kstats, const apg_pc_params* pp, apg_pc_stats* pstats, bool join) {
  APG_REQUIRE(ctx && dr, "apg_spectrum_precorrect_dev: NULL argument");
  apg_pc_params p;
  if (pp)
    p = *pp;
  else
    apg_pc_defaults(&p);
  APG_TRY(check_pc(p));
  if (K_spec != p.K + 1 || !sk_can_fuse_up(p.K)) {  // not fusable: the two modules in turn
    APG_TRY(apg_kmer_spectrum_dev(ctx, dr, K_spec, hist, hist_len, kstats));
    return apg_precorrect_dev(ctx, dr, &p, pstats);
  }
  APG_REQUIRE(hist_len == 0 || hist_len >= 2, "spectrum: hist_len must be 0 or >= 2");
  APG_REQUIRE(dr->n_reads == 0 || dr->d_quals, "apg_precorrect: read set has no qualities");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  apg_pc_stats st;
  std::memset(&st, 0, sizeof st);
  // the K+1 result lands at the join: held by the context until then
  ctx->up_res_pending = SkResult{};
  SkResult& ur = ctx->up_res_pending;
  const bool defer = !join && p.n_cycles == 1;
  APG_TRY(precorrect_pass(ctx, dr, p, &st, hist, hist_len, &ur, !defer));
  for (uint32_t c = 1; c < p.n_cycles; ++c) APG_TRY(precorrect_pass(ctx, dr, p, &st));
  ctx->up_kstats = kstats;
  if (!defer) APG_TRY(up_kstats_fill(ctx));
  if (pstats) *pstats = st;
  return APG_OK;
}

// the fused K+1 count's stats, once its pass is joined
int up_kstats_fill(apg_ctx* ctx) {
  apg_kstats* kstats = ctx->up_kstats;
  ctx->up_kstats = nullptr;
  if (!kstats) return APG_OK;
  const SkResult& ur = ctx->up_res_pending;
  std::memset(kstats, 0, sizeof(*kstats));
  kstats->n_kmers = ur.n_kmers;
  kstats->n_distinct = ur.n_distinct;
  kstats->n_buckets = ur.nbuckets;
  kstats->n_overflow = ur.n_overflow_buckets;
  kstats->n_redo = ur.n_redo_buckets;
  return APG_OK;
}
}  // namespace apg

extern "C" {

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

int apg_shard_solid_weak(apg_ctx* ctx, const void* d_recv, const uint64_t* recv_counts, int K, int n_shards,
                         uint32_t min_solid, void* d_mask, uint64_t* n_solid) {
  return shard_solid_weak_fused(ctx, d_recv, recv_counts, K, n_shards, min_solid, d_mask, n_solid, nullptr, 0, nullptr);
}
}  // extern "C"

namespace apg {
int shard_solid_weak_fused(apg_ctx* ctx, const void* d_recv, const uint64_t* recv_counts, int K, int n_shards,
                           uint32_t min_solid, void* d_mask, uint64_t* n_solid, uint64_t* up_hist, size_t up_hist_len,
                           SkResult* up_res, bool split_recs, uint64_t n_kmers, unsigned long long* weak,
                           const uint64_t* wpos, SkSelf self) {
  APG_REQUIRE(ctx && recv_counts && n_solid, "apg_shard_solid_weak: NULL argument");
  APG_REQUIRE(!up_res || sk_can_fuse_up(K), "apg_shard_solid_weak: the K+1 spectrum cannot ride on this K");
  APG_REQUIRE(min_solid >= 1, "apg_shard_solid_weak: min_solid must be >= 1");
  ctx->solid_valid = false;
  APG_REQUIRE(K >= 9 && K <= 29 && n_shards >= 1 && n_shards <= 8 && (n_shards & (n_shards - 1)) == 0,
              "apg_shard_solid_weak: K must be in [9, 29], n_shards a power of two <= 8");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  std::vector<uint64_t> rc(recv_counts, recv_counts + (size_t)n_shards * kSkShardBins);
  uint64_t n = 0;
  for (auto c : rc) n += c;
  APG_REQUIRE(n == 0 || (d_recv && (d_mask || (weak && wpos))), "apg_shard_solid_weak: d_recv or d_mask is NULL");
  const SK16* recs = static_cast<const SK16*>(d_recv);
  int err = APG_OK;
  // the received K-mer instances: given by the caller (the senders' counts,
  // exchanged beside the record counts), else summed over the records here
  const uint64_t nk = n_kmers != ~0ull ? n_kmers : sk_sum_kmers(ctx, recs, n, &err);
  APG_TRY(err);
  SkResult sr;
  APG_TRY(sk_shard_solid_weak(ctx, recs, rc, nk, K, n_shards, min_solid, static_cast<uint32_t*>(d_mask), &sr,
                              up_res ? K + 1 : 0, up_hist, up_hist_len, up_res, split_recs, weak, wpos, self));
  // The K+1 pass (side stream, kicked at the correction's stage as on one
  // GPU) reads only this count's record buffers: the caller's mask return,
  // solid-set gather and correction run beside it, and the caller joins it
  // (side_join) before it reads up_hist / up_res.
  APG_TRY(sync(ctx));
  ctx->n_solid = sr.n_solid;
  ctx->solid_valid = true;
  *n_solid = sr.n_solid;
  return APG_OK;
}

int precorrect_weak_built(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params& p, const void* d_solid,
                          uint64_t n_solid, unsigned long long* weak, apg_pc_stats* st) {
  APG_TRY(check_pc(p));
  APG_REQUIRE(p.K >= 9 && p.K <= 29, "apg_precorrect_weak: K must be in [9, 29]");
  APG_REQUIRE(dr->n_reads == 0 || dr->d_quals, "apg_precorrect_weak: read set has no qualities");
  APG_REQUIRE(n_solid == 0 || d_solid, "apg_precorrect_weak: d_solid is NULL");
  std::memset(st, 0, sizeof *st);
  return correct_pass(ctx, dr, p, static_cast<const uint64_t*>(d_solid), n_solid, st, weak);
}

int precorrect_weak_masks(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params& p, const void* d_solid,
                          uint64_t n_solid, unsigned long long* weak, const uint64_t* pos, const uint32_t* mask,
                          uint64_t n_in, uint64_t self_send, uint64_t n_self, apg_pc_stats* st) {
  APG_REQUIRE(self_send + n_self <= n_in, "precorrect_weak_masks: self segment out of range");
  // the returned masks of the records other ranks owned, around the self
  // segment whose bits the owner count wrote already
  const uint64_t n_a = self_send, n_b = n_in - self_send - n_self;
  kbegin(ctx, "weak_apply", (n_a + n_b) * 12);
  if (n_a) k_weak_apply<<<grid_for(ctx, n_a), 256, 0, ctx->stream>>>(pos, mask, n_a, weak);
  if (n_b)
    k_weak_apply<<<grid_for(ctx, n_b), 256, 0, ctx->stream>>>(pos + self_send + n_self, mask + self_send, n_b, weak);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return precorrect_weak_built(ctx, dr, p, d_solid, n_solid, weak, st);
}
}  // namespace apg

extern "C" {

int apg_precorrect_weak(apg_ctx* ctx, apg_dreads* dr, const apg_pc_params* pp, const void* d_solid, uint64_t n_solid,
                        const void* d_pos, const void* d_mask, uint64_t n_rec, apg_pc_stats* stats) {
  APG_REQUIRE(ctx && dr, "apg_precorrect_weak: NULL argument");
  APG_REQUIRE(n_solid == 0 || d_solid, "apg_precorrect_weak: d_solid is NULL");
  APG_REQUIRE(n_rec == 0 || (d_pos && d_mask), "apg_precorrect_weak: d_pos or d_mask is NULL");
  apg_pc_params p;
  if (pp)
    p = *pp;
  else
    apg_pc_defaults(&p);
  APG_TRY(check_pc(p));
  APG_REQUIRE(p.K >= 9 && p.K <= 29, "apg_precorrect_weak: K must be in [9, 29]");
  APG_REQUIRE(dr->n_reads == 0 || dr->d_quals, "apg_precorrect_weak: read set has no qualities");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  unsigned long long* weak = nullptr;
  const uint64_t words = dr->n_bases / 64 + 2;
  APG_TRY(workspace_t(ctx, "pc_weak", words, &weak));
  APG_CHECK_HIP(hipMemsetAsync(weak, 0, words * 8, ctx->stream));
  kbegin(ctx, "weak_apply", n_rec * 12);
  if (n_rec)
    k_weak_apply<<<grid_for(ctx, n_rec), 256, 0, ctx->stream>>>(static_cast<const uint64_t*>(d_pos),
                                                                static_cast<const uint32_t*>(d_mask), n_rec, weak);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  apg_pc_stats st;
  std::memset(&st, 0, sizeof st);
  APG_TRY(correct_pass(ctx, dr, p, static_cast<const uint64_t*>(d_solid), n_solid, &st, weak));
  if (stats) *stats = st;
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

int apg_solid_download(apg_ctx* ctx, uint64_t* out, uint64_t* n_solid) {
  APG_REQUIRE(ctx && n_solid, "apg_solid_download: NULL argument");
  APG_REQUIRE(ctx->pc_list_valid, "apg_solid_download: no correction pass has run on this context");
  *n_solid = ctx->pc_n;
  if (!out || ctx->pc_n == 0) return APG_OK;
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  APG_CHECK_HIP(hipMemcpyAsync(out, ctx->pc_list, ctx->pc_n * 8, hipMemcpyDeviceToHost, ctx->stream));
  return sync(ctx);
}

int apg_solid_upload(apg_ctx* ctx, int K, const uint64_t* hashes, uint64_t n) {
  APG_REQUIRE(ctx && (n == 0 || hashes), "apg_solid_upload: NULL argument");
  APG_REQUIRE(K >= 2 && K <= 32, "apg_solid_upload: K must be in [2, 32]");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  ctx->pc_list_valid = false;  // "x_solid" may hold the current list
  ctx->pc_ext_valid = false;
  ctx->clean_valid = false;
  ctx->pc_self = false;  // an uploaded list is no read set's own count (ecj_run's reuse test)
  ctx->ws_dead &= ~kRoomCorrection;
  uint64_t* list = nullptr;
  APG_TRY(workspace_t(ctx, "x_solid", std::max<uint64_t>(n, 1), &list));
  if (n) APG_CHECK_HIP(hipMemcpyAsync(list, hashes, n * 8, hipMemcpyHostToDevice, ctx->stream));
  APG_TRY(sync(ctx));
  ctx->pc_list = list;
  ctx->pc_n = n;
  ctx->pc_K = K;
  ctx->pc_list_valid = true;
  return APG_OK;
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
  if (quals)
    APG_TRY(dreads_quals_ready(dr));
  else
    dreads_join(dr);  // the bases are loaded; only a failed qualities load fails a download of them
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
