// kmer_spectrum.hip — MI355X-native k-mer counting and spectrum (K <= 32).
//
// Replaces ALLPATHS-LG's naif_kmerize + KernelKmerStorer + KmerSpectrum
// ([R:M] src/kmers/naif_kmer/, src/kmers/KmerSpectra.h; reference snapshot is
// empty).  Semantics restated in oracle/kmer_oracle.c.
//
// Pipeline (all records are w-bit hashes, w = 2K, of canonical k-mers; the
// hash is a bijection so grouping by hash == grouping by k-mer):
//   A  extract_count / extract_scatter: one thread per read rolls the k-mer,
//      hashes it and scatters the hash into 2^D groups, D = top bits of the
//      hash = [shard bits | 5 - shard bits L1 bits].  Per-(digit, block)
//      counts form a count matrix whose exclusive scan places every block's
//      records: no global atomics, and with 32 digits the per-block write
//      frontier stays L2-resident.
//   (multi-GPU: each shard's contiguous range travels by all_to_all)
//   B  part_count / part_scatter levels (<= 8 bits each): chunks of a parent
//      group are counted into a [digit][chunk] matrix, scanned, and scattered
//      through an LDS-staged 4096-record tile sorted by digit, so waves write
//      contiguous runs.  Levels stop when mean bucket size ~ kBucketTarget.
//   C  bucket_count: one workgroup per bucket counts it in an LDS
//      open-addressing table keyed on the hash bits below the bucket prefix,
//      bins counts into the spectrum and (table mode) writes distinct
//      (hash, count) in hash order via rank-by-broadcast.  Buckets over kCap
//      records (very repeated k-mers) take the global-scratch radix fallback.
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "apg_core.hpp"
#include "kmer_common.hpp"
#include "kmer_internal.hpp"
#include "partition.hpp"

namespace apg {

constexpr int kExtractThreads = 256;
constexpr int kMaxExtractBlocks = 2048;
constexpr uint32_t kBucketTarget = 1536;   // mean bucket size the planner aims for
constexpr int kLdsHistBins = 1024;         // spectrum bins kept in LDS

// ------------------------------------------------------------------------
// Stage A: reads -> hash records grouped by top-D-bit digit
// ------------------------------------------------------------------------
struct ReadsView {
  const uint64_t* base_off;
  const uint64_t* byte_off;
  const uint8_t* packed;
  uint64_t n_reads;
};

__device__ __forceinline__ void block_read_range(uint64_t n, uint32_t G, uint32_t b, uint64_t* r0, uint64_t* r1) {
  *r0 = (n * b) / G;
  *r1 = (n * (b + 1)) / G;
}

// cmat[digit * G + block] = #records of `block` whose hash has top-D digit `digit`.
__global__ void __launch_bounds__(kExtractThreads) k_extract_count(ReadsView rv, int K, HashP hp, int dshift,
                                                                   uint32_t ndig, uint32_t* __restrict__ cmat) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  const uint32_t G = gridDim.x, b = blockIdx.x;
  for (uint32_t i = threadIdx.x; i < ndig; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  uint64_t r0, r1;
  block_read_range(rv.n_reads, G, b, &r0, &r1);
  const uint64_t dmask = ndig - 1;
  for (uint64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    const uint64_t s = rv.base_off[r];
    const uint32_t len = (uint32_t)(rv.base_off[r + 1] - s);
    for_each_kmer_hash(rv.packed + rv.byte_off[r], len, K, hp,
                       [&](uint64_t h) { atomicAdd(&hist[(h >> dshift) & dmask], 1u); });
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < ndig; i += blockDim.x) cmat[(uint64_t)i * G + b] = hist[i];
}

// Staged scatter: each thread rolls its read 16 k-mers per round; the
// block's round (<= 4096 records) is counting-sorted by digit in LDS and
// written as contiguous per-digit runs.
constexpr int kXItems = 16;

__global__ void __launch_bounds__(kExtractThreads) k_extract_scatter(ReadsView rv, int K, HashP hp, int dshift,
                                                                     uint32_t ndig,
                                                                     const uint64_t* __restrict__ omat,
                                                                     uint64_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint64_t stage[kExtractThreads * kXItems];
  __shared__ unsigned long long cur[256];
  __shared__ uint32_t lcnt[256];
  __shared__ uint32_t lstart[256];
  __shared__ uint32_t scan_sm[64];
  const uint32_t G = gridDim.x, b = blockIdx.x, tid = threadIdx.x;
  const uint64_t dmask = ndig - 1;
  for (uint32_t d = tid; d < ndig; d += blockDim.x) cur[d] = omat[(uint64_t)d * G + b];
  uint64_t r0, r1;
  block_read_range(rv.n_reads, G, b, &r0, &r1);
  for (uint64_t rb = r0; rb < r1; rb += kExtractThreads) {
    const uint64_t r = rb + tid;
    KmerRoller kr;
    kr.i = 0;
    kr.len = 0;
    if (r < r1) {
      const uint64_t s = rv.base_off[r];
      kr.init(rv.packed + rv.byte_off[r], (uint32_t)(rv.base_off[r + 1] - s), K, hp);
    }
    while (__syncthreads_or(kr.more())) {
      lcnt[tid] = 0;
      __syncthreads();
      uint64_t v[kXItems];
      uint32_t pos[kXItems];
      uint32_t nv = 0;
#pragma unroll
      for (int j = 0; j < kXItems; ++j) {
        if (kr.more()) {
          v[j] = kr.next(hp);
          pos[j] = atomicAdd(&lcnt[(v[j] >> dshift) & dmask], 1u);
          nv = j + 1;
        }
      }
      __syncthreads();
      uint32_t tot;
      const uint32_t ex = block_exclusive_scan<uint32_t>(lcnt[tid], scan_sm, &tot);
      lstart[tid] = ex;
      __syncthreads();
#pragma unroll
      for (int j = 0; j < kXItems; ++j)
        if ((uint32_t)j < nv) stage[lstart[(v[j] >> dshift) & dmask] + pos[j]] = v[j];
      __syncthreads();
      for (uint32_t i = tid; i < tot; i += kExtractThreads) {
        const uint64_t x = stage[i];
        const uint32_t d = (uint32_t)((x >> dshift) & dmask);
        out[cur[d] + (i - lstart[d])] = x;
      }
      __syncthreads();
      if (tid < ndig) cur[tid] += lcnt[tid];
    }
  }
}

// digit_start[d] = omat[d * G], d in [0, ndig]; digit_start[ndig] = total.
__global__ void k_digit_starts(const uint64_t* __restrict__ omat, uint32_t ndig, uint32_t G,
                               uint64_t* __restrict__ ds) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d <= ndig) ds[d] = omat[(uint64_t)d * G];
}

// ------------------------------------------------------------------------
// Stage C: per-bucket counting in LDS.  All records of a bucket share the
// hash bits above `remb`, so a bucket is counted on the low remb bits
// (rem) in an LDS open-addressing table (linear probing, CAS insert, atomic
// count).  Distinct entries are compacted in place, then (table mode) each one's
// rank among the bucket's distinct keys — computed with broadcast LDS reads —
// places it at off + rank, i.e. in ascending-hash order, independent of the
// insertion order.  Counts are binned into the spectrum.
// ------------------------------------------------------------------------
constexpr int kCountThreads = 512;
constexpr uint32_t kCap = 4095;            // max records of an LDS-counted bucket
constexpr uint32_t kTabMax = 4096;         // table slots: > n >= distinct, so a bucket always fits
constexpr int kCapItems = (kCap + kCountThreads - 1) / kCountThreads;
constexpr int kSlotItems = kTabMax / kCountThreads;

template <typename KT>
struct KeyTraits;
template <>
struct KeyTraits<uint32_t> {
  static constexpr uint32_t empty = 0xffffffffu;
};
template <>
struct KeyTraits<unsigned long long> {
  static constexpr unsigned long long empty = ~0ull;
};

struct CountOut {
  uint64_t* tab_hash;            // in place over rec (table / solid modes)
  uint32_t* tab_cnt;             // parallel to rec (table / solid modes)
  uint32_t* bucket_nd;           // distinct per bucket
  unsigned long long* ghist;     // spectrum
  uint64_t hist_len;
  unsigned long long* gstats;    // [0] n_distinct, [1] overflow count, [2] max bucket
  uint32_t* ovf_list;
};

__device__ __forceinline__ void spectrum_add(uint32_t c, uint32_t* lhist, unsigned long long* ghist,
                                             uint64_t hist_len) {
  uint64_t m = c;
  if (m >= hist_len - 1) m = hist_len - 1;
  if (m < (uint64_t)kLdsHistBins)
    atomicAdd(&lhist[m], 1u);
  else
    atomicAdd(&ghist[m], 1ull);
}

// MODE: kCountSpectrum (histogram only) or kCountTable (every distinct hash +
// count, hash order inside the bucket).
template <typename KT, int MODE>
__global__ void __launch_bounds__(kCountThreads) k_bucket_count(uint64_t* __restrict__ rec,
                                                                const uint64_t* __restrict__ boff, uint64_t nbuckets,
                                                                int remb, CountOut o) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  KT* tkey = reinterpret_cast<KT*>(smem_raw);                              // kTabMax
  uint32_t* tcnt = reinterpret_cast<uint32_t*>(tkey + kTabMax);            // kTabMax
  uint32_t* lhist = tcnt + kTabMax;                                        // kLdsHistBins
  uint32_t* scan_sm = lhist + kLdsHistBins;                                // 64
  constexpr KT EMPTY = KeyTraits<KT>::empty;
  const uint32_t tid = threadIdx.x;
  const uint64_t remmask = remb >= 64 ? ~0ull : ((1ull << remb) - 1);
  for (uint32_t i = tid; i < kLdsHistBins; i += kCountThreads) lhist[i] = 0;
  unsigned long long nd_sum = 0, maxb = 0;

  // Records of bucket `b` (offsets off/n already known) into registers
  // (n <= kCap; larger buckets are not loaded).
  auto load = [&](uint64_t off, uint32_t n, uint64_t (&v)[kCapItems]) {
    const uint32_t nl = n <= kCap ? n : 0;
#pragma unroll
    for (int i = 0; i < kCapItems; ++i) {
      const uint32_t idx = i * kCountThreads + tid;
      v[i] = idx < nl ? rec[off + idx] : 0;
    }
  };

  auto bounds = [&](uint64_t b, uint64_t& off, uint32_t& n) {
    off = 0;
    n = 0;
    if (b < nbuckets) {
      off = boff[b];
      n = (uint32_t)(boff[b + 1] - off);
    }
  };
  uint64_t v[kCapItems], vn[kCapItems];
  uint64_t off, offn, off2;
  uint32_t n, nn, n2;
  uint64_t bkt = blockIdx.x;
  bounds(bkt, off, n);
  bounds(bkt + gridDim.x, offn, nn);
  load(off, n, v);
  __syncthreads();
  for (; bkt < nbuckets; bkt += gridDim.x) {
    // pipeline: records of the next bucket and offsets of the one after are
    // in flight while this bucket is counted
    load(offn, nn, vn);
    bounds(bkt + 2 * (uint64_t)gridDim.x, off2, n2);
    if (n > maxb) maxb = n;
    if (n > kCap) {
      if (tid == 0) {
        const unsigned long long k = atomicAdd(&o.gstats[1], 1ull);
        o.ovf_list[k] = (uint32_t)bkt;
      }
    } else if (n == 0) {
      if (MODE != kCountSpectrum && tid == 0) o.bucket_nd[bkt] = 0;
    } else {
      // table size: power of two > n (>= 2 slots per thread); the load factor
      // is distinct/T, typically ~0.2 at genomic coverage
      uint32_t T = 2 * kCountThreads;
      while (T <= n) T <<= 1;
      const uint32_t tmask = T - 1;
      for (uint32_t s = tid; s < T; s += kCountThreads) {
        tkey[s] = EMPTY;
        tcnt[s] = 0;
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < kCapItems; ++i) {
        const uint32_t idx = i * kCountThreads + tid;
        if (idx < n) {
          const KT key = (KT)(v[i] & remmask);
          uint32_t s = (uint32_t)key & tmask;
          for (;;) {
            const KT old = atomicCAS(&tkey[s], EMPTY, key);
            if (old == EMPTY || old == key) {
              atomicAdd(&tcnt[s], 1u);
              break;
            }
            s = (s + 1) & tmask;
          }
        }
      }
      __syncthreads();
      if (MODE == kCountSpectrum) {
        // spectrum only: every occupied slot is one distinct k-mer
        for (uint32_t s = tid; s < T; s += kCountThreads) {
          if (tkey[s] != EMPTY) {
            spectrum_add(tcnt[s], lhist, o.ghist, o.hist_len);
            ++nd_sum;
          }
        }
      } else {
        // compact occupied slots to the front of the table (in place)
        const uint32_t spt = T / kCountThreads;
        KT ks[kSlotItems];
        uint32_t cs[kSlotItems];
        uint32_t occ = 0;
#pragma unroll
        for (int i = 0; i < kSlotItems; ++i) {
          if ((uint32_t)i < spt) {
            const uint32_t s = tid * spt + i;
            ks[i] = tkey[s];
            cs[i] = tcnt[s];
            occ += ks[i] != EMPTY;
          }
        }
        uint32_t d;
        uint32_t j = block_exclusive_scan<uint32_t>(occ, scan_sm, &d);  // ends with a barrier
#pragma unroll
        for (int i = 0; i < kSlotItems; ++i) {
          if ((uint32_t)i < spt && ks[i] != EMPTY) {
            tkey[j] = ks[i];
            tcnt[j] = cs[i];
            ++j;
          }
        }
        __syncthreads();
        const uint64_t prefix = v[0] & ~remmask;  // valid for tid < n; only such threads emit
        for (uint32_t e = tid; e < d; e += kCountThreads) {
          const KT key = tkey[e];
          const uint32_t c = tcnt[e];
          uint32_t r = 0;
          for (uint32_t i = 0; i < d; ++i) r += tkey[i] < key;
          o.tab_hash[off + r] = prefix | (uint64_t)key;
          o.tab_cnt[off + r] = c;
          spectrum_add(c, lhist, o.ghist, o.hist_len);
        }
        if (tid == 0) {
          o.bucket_nd[bkt] = d;
          nd_sum += d;
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < kCapItems; ++i) v[i] = vn[i];
    off = offn;
    n = nn;
    offn = off2;
    nn = n2;
  }
  __syncthreads();
  const uint64_t lim = o.hist_len < (uint64_t)kLdsHistBins ? o.hist_len : (uint64_t)kLdsHistBins;
  for (uint32_t i = tid; i < lim; i += kCountThreads)
    if (lhist[i]) atomicAdd(&o.ghist[i], (unsigned long long)lhist[i]);
  // distinct counts: per-thread partials (spectrum path) or thread 0 (table path)
  for (int o2 = 32; o2 > 0; o2 >>= 1) nd_sum += __shfl_down(nd_sum, o2, 64);
  if ((tid & 63) == 0 && nd_sum) atomicAdd(&o.gstats[0], nd_sum);
  if (tid == 0) atomicMax(&o.gstats[2], maxb);
}

template <typename KT>
constexpr size_t bucket_count_lds() {
  return kTabMax * sizeof(KT) + kTabMax * 4 + kLdsHistBins * 4 + 64 * 4;
}

// ------------------------------------------------------------------------
// Stage C fallback: buckets over kCap records (highly repeated k-mers) are
// radix-sorted in global scratch by one workgroup each, then run-length counted.
// ------------------------------------------------------------------------

// LSD radix sort of A[0..n) on bits [0, sortbits), 8 bits a pass, stable,
// ping-ponging with B.  whist: LDS [nwaves][256] u32.  Works on LDS or global
// buffers.  Returns the buffer holding the result.
__device__ uint64_t* block_radix_sort(uint64_t* A, uint64_t* B, uint32_t n, int sortbits, uint32_t* whist,
                                      uint32_t* scan_sm) {
  const int lane = lane_id(), wave = wave_id(), nw = blockDim.x >> 6;
  const uint32_t rows = (n + 63) >> 6;
  const uint32_t rpw = (rows + nw - 1) / nw;
  const uint32_t r0 = min(rows, wave * rpw), r1 = min(rows, r0 + rpw);
  const uint64_t lt = lanemask_lt();
  uint32_t* wh = whist + wave * 256;
  for (int shift = 0; shift < sortbits; shift += 8) {
    const int nb = min(8, sortbits - shift);
    const uint32_t ndig = 1u << nb, dmask = ndig - 1;
    for (uint32_t i = lane; i < 256; i += 64) wh[i] = 0;
    // (1) per-wave digit histogram over the wave's rows
    for (uint32_t r = r0; r < r1; ++r) {
      const uint32_t idx = (r << 6) + lane;
      const bool valid = idx < n;
      const uint32_t d = valid ? (uint32_t)(A[idx] >> shift) & dmask : 0;
      const uint64_t peers = wave_match(d, valid, nb);
      if (valid && (peers & lt) == 0) wh[d] += __popcll(peers);
    }
    __syncthreads();
    // (2) exclusive offsets in (digit, wave) order -> stable placement
    {
      const uint32_t t = threadIdx.x;
      uint32_t tot = 0;
      if (t < ndig)
        for (int w = 0; w < nw; ++w) tot += whist[w * 256 + t];
      uint32_t all;
      uint32_t base = block_exclusive_scan<uint32_t>(t < ndig ? tot : 0u, scan_sm, &all);
      if (t < ndig)
        for (int w = 0; w < nw; ++w) {
          const uint32_t c = whist[w * 256 + t];
          whist[w * 256 + t] = base;
          base += c;
        }
    }
    __syncthreads();
    // (3) scatter
    for (uint32_t r = r0; r < r1; ++r) {
      const uint32_t idx = (r << 6) + lane;
      const bool valid = idx < n;
      const uint64_t key = valid ? A[idx] : 0;
      const uint32_t d = (uint32_t)(key >> shift) & dmask;
      const uint64_t peers = wave_match(d, valid, nb);
      if (valid) {
        const uint32_t pos = wh[d] + __popcll(peers & lt);
        B[pos] = key;
      }
      __builtin_amdgcn_wave_barrier();
      if (valid && (peers & lt) == 0) wh[d] += __popcll(peers);
      __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    uint64_t* t = A;
    A = B;
    B = t;
  }
  return A;
}

// Oversized buckets: one workgroup each, same algorithm on global scratch.
// scratch: u64 region parallel to rec (free after stage B); heads: u32 region
// parallel to rec.
__global__ void __launch_bounds__(kCountThreads) k_sort_count_global(uint64_t* __restrict__ rec,
                                                                    const uint64_t* __restrict__ boff,
                                                                    uint64_t* __restrict__ scratch,
                                                                    uint32_t* __restrict__ heads, int sortbits,
                                                                    CountOut o) {
  __shared__ uint32_t whist[(kCountThreads / 64) * 256];
  __shared__ uint32_t lhist[kLdsHistBins];
  __shared__ uint32_t scan_sm[64];
  for (int i = threadIdx.x; i < kLdsHistBins; i += blockDim.x) lhist[i] = 0;
  const uint32_t bkt = o.ovf_list[blockIdx.x];
  const uint64_t off = boff[bkt];
  const uint32_t n = (uint32_t)(boff[bkt + 1] - off);
  __syncthreads();
  uint64_t* A = rec + off;
  uint64_t* B = scratch + off;
  uint64_t* S = block_radix_sort(A, B, n, sortbits, whist, scan_sm);
  if (S == A) {  // result must not alias the in-place output below
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) B[i] = A[i];
    __syncthreads();
    S = B;
  }
  uint32_t* H = heads + off;
  const uint32_t ipt = (n + blockDim.x - 1) / blockDim.x;
  const uint32_t i0 = min(n, threadIdx.x * ipt), i1 = min(n, i0 + ipt);
  uint32_t cnt = 0;
  for (uint32_t i = i0; i < i1; ++i) cnt += (i == 0 || S[i] != S[i - 1]);
  uint32_t nd;
  uint32_t j = block_exclusive_scan<uint32_t>(cnt, scan_sm, &nd);
  for (uint32_t i = i0; i < i1; ++i)
    if (i == 0 || S[i] != S[i - 1]) H[j++] = i;
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < nd; k += blockDim.x) {
    const uint32_t s = H[k], e = k + 1 < nd ? H[k + 1] : n;
    o.tab_hash[off + k] = S[s];
    o.tab_cnt[off + k] = e - s;
    spectrum_add(e - s, lhist, o.ghist, o.hist_len);
  }
  __syncthreads();
  const uint64_t lim = o.hist_len < (uint64_t)kLdsHistBins ? o.hist_len : (uint64_t)kLdsHistBins;
  for (uint32_t i = threadIdx.x; i < lim; i += blockDim.x)
    if (lhist[i]) atomicAdd(&o.ghist[i], (unsigned long long)lhist[i]);
  if (threadIdx.x == 0) {
    o.bucket_nd[bkt] = nd;
    atomicAdd(&o.gstats[0], (unsigned long long)nd);
  }
}

// Dense table: keys (un-hashed) and counts in hash order.
__global__ void k_compact_table(const uint64_t* __restrict__ tab_hash, const uint32_t* __restrict__ tab_cnt,
                                const uint64_t* __restrict__ boff, const uint32_t* __restrict__ bucket_nd,
                                const uint64_t* __restrict__ dense_off, uint64_t nbuckets, HashP hp,
                                uint64_t* __restrict__ keys, uint32_t* __restrict__ counts) {
  for (uint64_t b = blockIdx.x; b < nbuckets; b += gridDim.x) {
    const uint64_t s = boff[b], d = dense_off[b];
    const uint32_t nd = bucket_nd[b];
    for (uint32_t i = threadIdx.x; i < nd; i += blockDim.x) {
      keys[d + i] = kunhash(hp, tab_hash[s + i]);
      counts[d + i] = tab_cnt[s + i];
    }
  }
}

// [lower_bound(lo), lower_bound(hi)) of the hash-ordered dense table: two
// binary searches on khash(key), one lane each.
__global__ void k_hash_bounds(const uint64_t* __restrict__ keys, uint64_t n, HashP hp, uint64_t lo, uint64_t hi,
                              unsigned long long* __restrict__ out) {
  if (threadIdx.x >= 2) return;
  if (threadIdx.x == 1 && hi == 0) {  // no upper bound
    out[1] = n;
    return;
  }
  const uint64_t target = threadIdx.x ? hi : lo;
  uint64_t a = 0, b = n;
  while (a < b) {
    const uint64_t m = a + (b - a) / 2;
    if (khash(hp, keys[m]) < target)
      a = m + 1;
    else
      b = m;
  }
  out[threadIdx.x] = a;
}

// ------------------------------------------------------------------------
// Host orchestration
// ------------------------------------------------------------------------
static int ceil_log2(uint64_t x) {
  int b = 0;
  while ((1ull << b) < x) ++b;
  return b;
}

// Stage-A fanout below the shard bits: small, so the LDS-cursor scatter's
// write frontier (digits x blocks x one 128-B line) stays L2-resident.
constexpr int kExtractDigitBits = 5;
static int l1_bits(int K, int P) {
  const int w = 2 * K, pbits = ceil_log2((uint64_t)P);
  return std::max(0, std::min(kExtractDigitBits - pbits, w - pbits));
}

// Stage A.  Digit = top (pbits + l1) bits.  extract_count returns per-digit
// record counts (host, 2^D) and leaves the scanned count matrix in the "x_omat"
// workspace; extract_scatter reuses it when called for the same (reads, K, P).
static int check_shards(int K, int n_shards) {
  APG_REQUIRE(K >= 1 && K <= 32, "K must be in [1, 32]");
  APG_REQUIRE(n_shards >= 1 && n_shards <= 8 && (n_shards & (n_shards - 1)) == 0,
              "n_shards must be a power of two in [1, 8]");  // 2^(3 + kSkDigitBits) <= 256 LDS digits
  APG_REQUIRE(2 * K >= ceil_log2((uint64_t)n_shards), "K too small for n_shards");
  return APG_OK;
}


static int extract_count(apg_ctx* ctx, const apg_dreads* dr, int K, int P, std::vector<uint64_t>* digit_counts) {
  const int w = 2 * K, pbits = ceil_log2((uint64_t)P), D = pbits + l1_bits(K, P);
  const uint32_t ndig = 1u << D;
  const HashP hp = make_hashp(K);
  const int dshift = w - D;
  const uint32_t G =
      (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(kMaxExtractBlocks, (dr->n_reads + 255) / 256));
  uint32_t* cmat = nullptr;
  uint64_t* omat = nullptr;
  uint64_t* dstart = nullptr;
  APG_TRY(workspace_t(ctx, "x_cmat", (uint64_t)ndig * G, &cmat));
  APG_TRY(workspace_t(ctx, "x_omat", (uint64_t)ndig * G + 1, &omat));
  APG_TRY(workspace_t(ctx, "x_dstart", ndig + 1, &dstart));
  ReadsView rv{dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->n_reads};
  ctx->xstate.valid = false;
  kbegin(ctx, "extract_count", dr->n_bytes + 16 * dr->n_reads);
  k_extract_count<<<G, kExtractThreads, ndig * 4, ctx->stream>>>(rv, K, hp, dshift, ndig, cmat);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  APG_TRY(scan_u32_u64(ctx, cmat, (uint64_t)ndig * G, omat, "x"));
  k_digit_starts<<<(ndig + 1 + 255) / 256, 256, 0, ctx->stream>>>(omat, ndig, G, dstart);
  APG_CHECK_HIP(hipGetLastError());
  std::vector<uint64_t> ds(ndig + 1);
  APG_TRY(d2h_sync(ctx, ds.data(), dstart, (ndig + 1) * 8));
  digit_counts->resize(ndig);
  for (uint32_t d = 0; d < ndig; ++d) (*digit_counts)[d] = ds[d + 1] - ds[d];
  auto& xs = ctx->xstate;
  xs.gen = dr->gen;
  xs.K = K;
  xs.P = P;
  xs.G = G;
  xs.ndig = ndig;
  xs.dshift = dshift;
  xs.total = ds[ndig];
  xs.valid = true;
  return APG_OK;
}

static int extract_scatter(apg_ctx* ctx, const apg_dreads* dr, int K, int P, uint64_t* d_out) {
  auto& xs = ctx->xstate;
  if (!xs.valid || xs.gen != dr->gen || xs.K != K || xs.P != P) {
    std::vector<uint64_t> dc;
    APG_TRY(extract_count(ctx, dr, K, P, &dc));
  }
  uint64_t* omat = nullptr;
  APG_TRY(workspace_t(ctx, "x_omat", (uint64_t)xs.ndig * xs.G + 1, &omat));
  ReadsView rv{dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->n_reads};
  kbegin(ctx, "extract_scatter", dr->n_bytes + 16 * dr->n_reads + xs.total * 8);
  k_extract_scatter<<<xs.G, kExtractThreads, 0, ctx->stream>>>(rv, K, make_hashp(K), xs.dshift, xs.ndig,
                                                                        omat, d_out);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return APG_OK;
}

// Stages B + C on records held in `src`, laid out as P source blocks, each
// grouped by L1 group: recv_counts[src * B1 + l1].  `spare` (may be null) is
// a library buffer of >= n records that may be overwritten (ping-pong).
static int stage_count(apg_ctx* ctx, const uint64_t* src, uint64_t* spare, const std::vector<uint64_t>& recv_counts,
                       int K, int P, int mode, uint64_t* hist, size_t hist_len,
                       CountResult* res) {
  const bool table = mode != kCountSpectrum;
  const int w = 2 * K, pbits = ceil_log2((uint64_t)P), l1 = l1_bits(K, P);
  const uint32_t B1 = 1u << l1;
  if (recv_counts.size() != (size_t)P * B1) {
    set_error("stage_count: recv_counts has wrong size");
    return APG_E_ARG;
  }
  uint64_t n = 0;
  for (auto c : recv_counts) n += c;
  const uint64_t need = (n + kBucketTarget - 1) / kBucketTarget;
  const int bb = std::min(w - pbits, std::max(l1, ceil_log2(std::max<uint64_t>(1, need))));
  const int rem = bb - l1;
  int nlev = (rem + kMaxLevelBits - 1) / kMaxLevelBits;
  if (nlev == 0 && P > 1) nlev = 1;  // regroup the P source segments of each L1 group
  std::vector<int> lbits(nlev, 0);
  for (int i = 0; i < nlev; ++i) lbits[i] = rem / nlev + (i < rem % nlev ? 1 : 0);
  const int remb = w - pbits - bb;
  res->n_records = n;
  vlog(ctx, "count: K=%d P=%d records=%llu l1=%d levels=%d bucket_bits=%d remb=%d table=%d", K, P,
       (unsigned long long)n, l1, nlev, bb, remb, mode);

  // parents = L1 groups, each with its P source segments
  std::vector<std::vector<Seg>> parents(B1);
  {
    uint64_t pos = 0;
    for (int s = 0; s < P; ++s)
      for (uint32_t l = 0; l < B1; ++l) {
        const uint64_t c = recv_counts[(size_t)s * B1 + l];
        parents[l].push_back(Seg{pos, c});
        pos += c;
      }
  }
  uint64_t *bufA = nullptr, *bufB = nullptr;
  APG_TRY(workspace_t(ctx, kBig1, std::max<uint64_t>(n, 1), &bufA));
  if (spare) {
    bufB = spare;
  } else {
    APG_TRY(workspace_t(ctx, kBig0, std::max<uint64_t>(n, 1), &bufB));
  }
  uint64_t nb = B1;
  uint64_t* boff = nullptr;
  APG_TRY(workspace_t(ctx, "c_boff", (1ull << bb) + 1, &boff));
  const uint64_t* cur = src;
  uint64_t* other = nullptr;  // buffer not holding `cur`
  int consumed = pbits + l1;
  if (nlev == 0) {
    // P == 1 and no further split: stage-A groups are the buckets.
    std::vector<uint64_t> hb(B1 + 1, 0);
    for (uint32_t l = 0; l < B1; ++l) hb[l + 1] = hb[l] + recv_counts[l];
    APG_CHECK_HIP(hipMemcpyAsync(boff, hb.data(), (B1 + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
    other = bufA;
  }
  for (int lev = 0; lev < nlev; ++lev) {
    consumed += lbits[lev];
    const int shift = w - consumed;
    uint64_t* dst = (lev % 2 == 0) ? bufA : bufB;
    std::vector<uint64_t> hb;
    const bool last = lev + 1 == nlev;
    APG_TRY(part_level<uint64_t>(ctx, cur, dst, parents, shift, lbits[lev], n, boff, last ? nullptr : &hb, "p"));
    nb = parents.size() << lbits[lev];
    if (!last) {
      parents.assign(nb, {});
      for (uint64_t q = 0; q < nb; ++q) parents[q].push_back(Seg{hb[q], hb[q + 1] - hb[q]});
    }
    other = (dst == bufA) ? bufB : bufA;
    cur = dst;
  }
  uint64_t* rec = const_cast<uint64_t*>(cur);  // library-owned here unless nlev == 0 (P == 1, src = spare)

  uint32_t *tab_cnt = nullptr, *bucket_nd = nullptr, *ovf_list = nullptr;
  unsigned long long *ghist = nullptr, *gstats = nullptr;
  const uint64_t hl = std::max<uint64_t>(hist_len, 2);
  APG_TRY(workspace_t(ctx, kBig2, table ? std::max<uint64_t>(n, 1) : 1, &tab_cnt));
  APG_TRY(workspace_t(ctx, "c_bnd", nb, &bucket_nd));
  APG_TRY(workspace_t(ctx, "c_ovf", nb, &ovf_list));
  APG_TRY(workspace_t(ctx, "c_hist", hl, &ghist));
  APG_TRY(workspace_t(ctx, "c_gstats", 4, &gstats));
  APG_CHECK_HIP(hipMemsetAsync(ghist, 0, hl * 8, ctx->stream));
  APG_CHECK_HIP(hipMemsetAsync(gstats, 0, 4 * 8, ctx->stream));

  CountOut co{rec, tab_cnt, bucket_nd, ghist, hl, gstats, ovf_list};
  const bool narrow = remb <= 31;
  const size_t lds = narrow ? bucket_count_lds<uint32_t>() : bucket_count_lds<unsigned long long>();
  const int per_cu = std::max<int>(1, (int)((160 * 1024) / lds));
  const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>(nb, (uint64_t)ctx->n_cu * per_cu * 2));
  kbegin(ctx, mode == kCountTable ? "bucket_count_table" : "bucket_count",
         n * 8 + (mode == kCountTable ? n * 12 : 0) + (nb + 1) * 8 + nb * 4);
#define APG_COUNT_LAUNCH(KT, M) \
  k_bucket_count<KT, M><<<grid, kCountThreads, lds, ctx->stream>>>(rec, boff, nb, remb, co)
  if (narrow) {
    if (mode == kCountTable)
      APG_COUNT_LAUNCH(uint32_t, kCountTable);
    else
      APG_COUNT_LAUNCH(uint32_t, kCountSpectrum);
  } else {
    if (mode == kCountTable)
      APG_COUNT_LAUNCH(unsigned long long, kCountTable);
    else
      APG_COUNT_LAUNCH(unsigned long long, kCountSpectrum);
  }
#undef APG_COUNT_LAUNCH
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  unsigned long long hs[4];
  APG_TRY(d2h_sync(ctx, hs, gstats, sizeof hs));
  if (hs[1]) {
    // Oversized buckets: radix sort in global scratch (the ping-pong buffer not
    // holding rec is free now).
    uint64_t* scratch = other;
    if (scratch == nullptr || scratch == rec) APG_TRY(workspace_t(ctx, "c_scratch", std::max<uint64_t>(n, 1), &scratch));
    uint32_t* heads = nullptr;
    APG_TRY(workspace_t(ctx, "c_heads", std::max<uint64_t>(n, 1), &heads));
    uint32_t* tcnt_full = tab_cnt;
    if (!table) {
      APG_TRY(workspace_t(ctx, kBig2, std::max<uint64_t>(n, 1), &tcnt_full));
      co.tab_cnt = tcnt_full;
    }
    vlog(ctx, "count: %llu oversized buckets -> global radix path", hs[1]);
    kbegin(ctx, "bucket_count_global", 0);
    k_sort_count_global<<<(uint32_t)hs[1], kCountThreads, 0, ctx->stream>>>(rec, boff, scratch, heads, remb, co);
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
    APG_CHECK_HIP(hipMemcpyAsync(hs, gstats, sizeof hs, hipMemcpyDeviceToHost, ctx->stream));
    tab_cnt = co.tab_cnt;
  }
  if (hist && hist_len) APG_CHECK_HIP(hipMemcpyAsync(hist, ghist, hist_len * 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(sync(ctx));
  if (hist && hist_len) hist[0] = 0;
  res->rec = rec;
  res->tab_cnt = tab_cnt;
  res->bucket_nd = bucket_nd;
  res->boff = boff;
  res->nbuckets = nb;
  res->st.n_kmers = n;
  res->st.n_distinct = hs[0];
  res->st.n_buckets = nb;
  res->st.n_overflow = hs[1];
  res->st.max_bucket = hs[2];
  return APG_OK;
}

int spectrum_impl(apg_ctx* ctx, const apg_dreads* dr, int K, int mode, uint64_t* hist, size_t hist_len,
                  CountResult* res) {
  APG_REQUIRE(ctx && dr, "spectrum: NULL ctx/reads");
  APG_REQUIRE(K >= 1 && K <= 32, "spectrum: K must be in [1, 32] for the 64-bit path");
  APG_REQUIRE(hist_len == 0 || hist_len >= 2, "spectrum: hist_len must be 0 or >= 2");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  std::vector<uint64_t> counts;
  APG_TRY(extract_count(ctx, dr, K, 1, &counts));
  uint64_t* buf = nullptr;
  APG_TRY(workspace_t(ctx, kBig0, std::max<uint64_t>(ctx->xstate.total, 1), &buf));
  APG_TRY(extract_scatter(ctx, dr, K, 1, buf));
  return stage_count(ctx, buf, buf, counts, K, 1, mode, hist, hist_len, res);
}

}  // namespace apg

using namespace apg;

extern "C" {

uint64_t apg_kmer_hash(int K, uint64_t canonical) {
  if (K < 1 || K > 32) return 0;
  return khash(make_hashp(K), canonical);
}

uint64_t apg_kmer_unhash(int K, uint64_t hash) {
  if (K < 1 || K > 32) return 0;
  return kunhash(make_hashp(K), hash);
}

static void sk_stats(const SkResult& r, apg_kstats* st) {
  std::memset(st, 0, sizeof(*st));
  st->n_kmers = r.n_kmers;
  st->n_distinct = r.n_distinct;
  st->n_buckets = r.nbuckets;
  st->n_overflow = r.n_overflow_buckets;
  st->n_redo = r.n_redo_buckets;
}

// Spectrum: the minimizer-partitioned super-k-mer pipeline (superkmer.hip).
int apg_kmer_spectrum_dev(apg_ctx* ctx, const apg_dreads* reads, int K, uint64_t* hist, size_t hist_len,
                          apg_kstats* stats) {
  SkResult r;
  APG_TRY(sk_spectrum(ctx, reads, K, false, 0, hist, hist_len, &r));
  if (stats) sk_stats(r, stats);
  return APG_OK;
}

int apg_kmer_spectrum(apg_ctx* ctx, const apg_reads* reads, int K, uint64_t* hist, size_t hist_len,
                      apg_kstats* stats) {
  apg_dreads* dr = nullptr;
  APG_TRY(apg_reads_upload(ctx, reads, &dr));
  const int rc = apg_kmer_spectrum_dev(ctx, dr, K, hist, hist_len, stats);
  apg_reads_free(dr);
  return rc;
}

int apg_kmer_count(apg_ctx* ctx, const apg_reads* reads, int K, uint64_t** keys, uint32_t** counts,
                   uint64_t* n_distinct, apg_kstats* stats) {
  APG_REQUIRE(ctx && reads, "apg_kmer_count: NULL argument");
  apg_dreads* dr = nullptr;
  APG_TRY(apg_reads_upload(ctx, reads, &dr));
  const int rc = apg_kmer_count_dev(ctx, dr, K, 0, 0, keys, counts, n_distinct, stats);
  apg_reads_free(dr);
  return rc;
}

int apg_kmer_count_dev(apg_ctx* ctx, const apg_dreads* dr, int K, uint64_t hash_lo, uint64_t hash_hi,
                       uint64_t** keys, uint32_t** counts, uint64_t* n_out, apg_kstats* stats) {
  APG_REQUIRE(ctx && dr && keys && counts && n_out, "apg_kmer_count_dev: NULL argument");
  *keys = nullptr;
  *counts = nullptr;
  *n_out = 0;
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  CountResult r;
  APG_TRY(spectrum_impl(ctx, dr, K, kCountTable, nullptr, 0, &r));
  const uint64_t nd = r.st.n_distinct;
  uint64_t* dense_off = nullptr;
  uint64_t* d_keys = nullptr;
  uint32_t* d_cnt = nullptr;
  unsigned long long* d_bounds = nullptr;
  APG_TRY(workspace_t(ctx, "t_dense_off", r.nbuckets + 1, &dense_off));
  APG_TRY(workspace_t(ctx, "t_keys", std::max<uint64_t>(nd, 1), &d_keys));
  APG_TRY(workspace_t(ctx, "t_cnt", std::max<uint64_t>(nd, 1), &d_cnt));
  APG_TRY(workspace_t(ctx, "t_bounds", 2, &d_bounds));
  APG_TRY(scan_u32_u64(ctx, r.bucket_nd, r.nbuckets, dense_off, "t"));
  const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>(r.nbuckets, (uint64_t)ctx->n_cu * 16));
  const HashP hp = make_hashp(K);
  kbegin(ctx, "compact_table", nd * 24);
  k_compact_table<<<grid, 256, 0, ctx->stream>>>(r.rec, r.tab_cnt, r.boff, r.bucket_nd, dense_off, r.nbuckets, hp,
                                                  d_keys, d_cnt);
  kend(ctx);
  // the parcel [hash_lo, hash_hi) is a contiguous range of the hash-ordered table
  k_hash_bounds<<<1, 64, 0, ctx->stream>>>(d_keys, nd, hp, hash_lo, hash_hi, d_bounds);
  APG_CHECK_HIP(hipGetLastError());
  unsigned long long hb[2];
  APG_TRY(d2h_sync(ctx, hb, d_bounds, sizeof hb));
  const uint64_t a = hb[0], n = hb[1] > hb[0] ? hb[1] - hb[0] : 0;
  auto* hk = (uint64_t*)std::malloc(std::max<uint64_t>(n, 1) * 8);
  auto* hc = (uint32_t*)std::malloc(std::max<uint64_t>(n, 1) * 4);
  if (!hk || !hc) {
    std::free(hk);
    std::free(hc);
    return APG_E_NOMEM;
  }
  int rc = APG_OK;
  if (n && (hipMemcpyAsync(hk, d_keys + a, n * 8, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess ||
            hipMemcpyAsync(hc, d_cnt + a, n * 4, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess)) {
    set_error("apg_kmer_count_dev: D2H failed");
    rc = APG_E_HIP;
  }
  if (rc == APG_OK) rc = sync(ctx);
  if (rc) {
    std::free(hk);
    std::free(hc);
    return rc;
  }
  *keys = hk;
  *counts = hc;
  *n_out = n;
  if (stats) *stats = r.st;
  return APG_OK;
}

int apg_shard_bins(int K, int n_shards) {
  if (check_shards(K, n_shards) != APG_OK) return APG_E_ARG;
  return kSkShardBins;
}

int apg_shard_count(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards, uint64_t* send_counts) {
  APG_REQUIRE(ctx && reads && send_counts, "apg_shard_count: NULL argument");
  APG_TRY(check_shards(K, n_shards));
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  std::vector<uint64_t> rc, kc;
  APG_TRY(sk_count(ctx, reads, K, n_shards, &rc, &kc));
  std::memcpy(send_counts, rc.data(), rc.size() * 8);
  return APG_OK;
}

int apg_shard_scatter(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards, void* d_send) {
  APG_REQUIRE(ctx && reads, "apg_shard_scatter: NULL argument");
  APG_TRY(check_shards(K, n_shards));
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  APG_TRY(sk_scatter(ctx, reads, K, n_shards, static_cast<SK16*>(d_send)));
  return sync(ctx);
}

int apg_shard_scatter_pos(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards, void* d_send, void* d_pos) {
  APG_REQUIRE(ctx && reads, "apg_shard_scatter_pos: NULL argument");
  APG_TRY(check_shards(K, n_shards));
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  APG_TRY(sk_scatter_pos(ctx, reads, K, n_shards, static_cast<SK16*>(d_send), static_cast<uint64_t*>(d_pos)));
  return sync(ctx);
}

int apg_shard_spectrum(apg_ctx* ctx, const void* d_recv, const uint64_t* recv_counts, int K, int n_shards,
                       uint64_t* hist, size_t hist_len, apg_kstats* stats) {
  APG_REQUIRE(ctx && recv_counts, "apg_shard_spectrum: NULL argument");
  APG_TRY(check_shards(K, n_shards));
  APG_REQUIRE(hist_len == 0 || hist_len >= 2, "apg_shard_spectrum: hist_len must be 0 or >= 2");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  std::vector<uint64_t> rc(recv_counts, recv_counts + (size_t)n_shards * kSkShardBins);
  uint64_t n = 0;
  for (auto c : rc) n += c;
  APG_REQUIRE(n == 0 || d_recv, "apg_shard_spectrum: d_recv is NULL");
  const SK16* recs = static_cast<const SK16*>(d_recv);
  int err = APG_OK;
  const uint64_t nk = sk_sum_kmers(ctx, recs, n, &err);
  APG_TRY(err);
  SkResult r;
  APG_TRY(sk_stage_count(ctx, recs, nullptr, rc, nk, K, n_shards, false, 0, hist, hist_len, &r));
  if (stats) sk_stats(r, stats);
  return APG_OK;
}

}  // extern "C"
