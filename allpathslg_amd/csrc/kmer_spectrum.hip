// kmer_spectrum.hip — MI355X-native k-mer counting and spectrum (K <= 32).
//
// Replaces ALLPATHS-LG's naif_kmerize + KernelKmerStorer + KmerSpectrum
// ([R:M] src/kmers/naif_kmer/, src/kmers/KmerSpectra.h; reference snapshot is
// empty).  Semantics restated in oracle/kmer_oracle.c.
//
// Pipeline (all records are w-bit hashes, w = 2K, of canonical k-mers; the
// hash is a bijection so grouping by hash == grouping by k-mer):
//   A  extract_count / extract_scatter: one thread per read rolls the k-mer,
//      hashes it and scatters the hash into 2^D "digit" groups, D = top bits
//      of the hash = [shard bits | L1 bits].  Per-(digit, block) counts form
//      a count matrix whose exclusive scan places every block's records
//      deterministically: no global atomics.
//   (multi-GPU: each shard's contiguous range travels by all_to_all)
//   B  rec_count / rec_scatter: the next b2 hash bits split every L1 group
//      into LDS-sized buckets (same count-matrix scheme over chunks).
//   C  sort_count: one workgroup per bucket loads it into LDS, LSD-radix-sorts
//      the low bits with a wave64 ballot multisplit, run-length counts equal
//      hashes and bins the counts into the spectrum.  Oversized buckets go to
//      sort_count_global (same algorithm on global scratch).
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "apg_core.hpp"
#include "kmer_common.hpp"

namespace apg {

constexpr int kExtractThreads = 256;
constexpr int kMaxExtractBlocks = 2048;
constexpr int kSortThreads = 512;
constexpr uint32_t kSortCap = 4096;        // records per LDS-resident bucket
constexpr uint32_t kBucketTarget = 1536;   // mean bucket size the planner aims for
constexpr int kLdsHistBins = 1024;         // spectrum bins kept in LDS
constexpr int kMaxL1Bits = 10;
constexpr int kMaxL2Bits = 11;

// ------------------------------------------------------------------------
// scan: u32 counts[n] -> u64 exclusive offsets[n+1] (offsets[n] = total)
// ------------------------------------------------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;

__global__ void __launch_bounds__(kScanThreads) k_scan_tiles(const uint32_t* __restrict__ in, uint64_t n,
                                                             uint64_t* __restrict__ tsum) {
  __shared__ uint64_t sm[32];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i)
    if (base + i < n) s += in[base + i];
  uint64_t tot;
  block_exclusive_scan<uint64_t>(s, sm, &tot);
  if (threadIdx.x == 0) tsum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(1024) k_scan_tsum(uint64_t* __restrict__ tsum, uint64_t nt) {
  __shared__ uint64_t sm[32];
  uint64_t carry = 0;
  for (uint64_t b = 0; b < nt; b += blockDim.x) {
    const uint64_t i = b + threadIdx.x;
    const uint64_t v = i < nt ? tsum[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_exclusive_scan<uint64_t>(v, sm, &tot);
    if (i < nt) tsum[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) tsum[nt] = carry;
}

__global__ void __launch_bounds__(kScanThreads) k_scan_apply(const uint32_t* __restrict__ in, uint64_t n,
                                                             const uint64_t* __restrict__ tsum,
                                                             uint64_t* __restrict__ out, uint64_t nt) {
  __shared__ uint64_t sm[32];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = base + i < n ? in[base + i] : 0;
    s += v[i];
  }
  uint64_t tot;
  uint64_t run = block_exclusive_scan<uint64_t>(s, sm, &tot) + tsum[blockIdx.x];
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = tsum[nt];
}

static int scan_u32_u64(apg_ctx* ctx, const uint32_t* d_in, uint64_t n, uint64_t* d_out, const char* tag) {
  const uint64_t nt = std::max<uint64_t>(1, (n + kScanTile - 1) / kScanTile);
  uint64_t* tsum = nullptr;
  APG_TRY(workspace_t(ctx, (std::string("scan_tsum_") + tag).c_str(), nt + 1, &tsum));
  kbegin(ctx, "scan", n * 4 * 2 + (n + 1) * 8);
  k_scan_tiles<<<nt, kScanThreads, 0, ctx->stream>>>(d_in, n, tsum);
  k_scan_tsum<<<1, 1024, 0, ctx->stream>>>(tsum, nt);
  k_scan_apply<<<nt, kScanThreads, 0, ctx->stream>>>(d_in, n, tsum, d_out, nt);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return APG_OK;
}

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

__global__ void __launch_bounds__(kExtractThreads) k_extract_scatter(ReadsView rv, int K, HashP hp, int dshift,
                                                                     uint32_t ndig,
                                                                     const uint64_t* __restrict__ omat,
                                                                     uint64_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long cur[];
  const uint32_t G = gridDim.x, b = blockIdx.x;
  for (uint32_t i = threadIdx.x; i < ndig; i += blockDim.x) cur[i] = omat[(uint64_t)i * G + b];
  __syncthreads();
  uint64_t r0, r1;
  block_read_range(rv.n_reads, G, b, &r0, &r1);
  const uint64_t dmask = ndig - 1;
  for (uint64_t r = r0 + threadIdx.x; r < r1; r += blockDim.x) {
    const uint64_t s = rv.base_off[r];
    const uint32_t len = (uint32_t)(rv.base_off[r + 1] - s);
    for_each_kmer_hash(rv.packed + rv.byte_off[r], len, K, hp, [&](uint64_t h) {
      const unsigned long long pos = atomicAdd(&cur[(h >> dshift) & dmask], 1ull);
      out[pos] = h;
    });
  }
}

// digit_start[d] = omat[d * G], d in [0, ndig]; digit_start[ndig] = total.
__global__ void k_digit_starts(const uint64_t* __restrict__ omat, uint32_t ndig, uint32_t G,
                               uint64_t* __restrict__ ds) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d <= ndig) ds[d] = omat[(uint64_t)d * G];
}

// ------------------------------------------------------------------------
// Stage B: record chunks -> buckets (count matrix over chunks)
// ------------------------------------------------------------------------
struct Chunk {
  uint64_t start;   // first record
  uint64_t mat;     // count-matrix index of (l1, digit 0, this chunk)
  uint32_t len;     // records
  uint32_t stride;  // chunks of this l1 (matrix stride between digits)
};

__global__ void __launch_bounds__(256) k_rec_count(const uint64_t* __restrict__ rec, const Chunk* __restrict__ ch,
                                                   int dshift, uint32_t ndig, uint32_t* __restrict__ cmat) {
  extern __shared__ __attribute__((aligned(16))) uint32_t hist[];
  const Chunk c = ch[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < ndig; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  const uint64_t dmask = ndig - 1;
  const uint64_t* p = rec + c.start;
  for (uint32_t i = threadIdx.x; i < c.len; i += blockDim.x) atomicAdd(&hist[(p[i] >> dshift) & dmask], 1u);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < ndig; i += blockDim.x) cmat[c.mat + (uint64_t)i * c.stride] = hist[i];
}

__global__ void __launch_bounds__(256) k_rec_scatter(const uint64_t* __restrict__ rec, const Chunk* __restrict__ ch,
                                                     int dshift, uint32_t ndig, const uint64_t* __restrict__ omat,
                                                     uint64_t* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) unsigned long long cur[];
  const Chunk c = ch[blockIdx.x];
  for (uint32_t i = threadIdx.x; i < ndig; i += blockDim.x) cur[i] = omat[c.mat + (uint64_t)i * c.stride];
  __syncthreads();
  const uint64_t dmask = ndig - 1;
  const uint64_t* p = rec + c.start;
  for (uint32_t i = threadIdx.x; i < c.len; i += blockDim.x) {
    const uint64_t h = p[i];
    out[atomicAdd(&cur[(h >> dshift) & dmask], 1ull)] = h;
  }
}

// boff[l1 * B2 + l2] = omat[l1_base[l1] + l2 * nch[l1]];  boff[B1*B2] = total.
__global__ void k_bucket_offsets(const uint64_t* __restrict__ omat, const uint64_t* __restrict__ l1_base,
                                 const uint32_t* __restrict__ nch, uint32_t B1, uint32_t B2, uint64_t total,
                                 uint64_t* __restrict__ boff) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nb = (uint64_t)B1 * B2;
  if (i < nb) {
    const uint32_t l1 = (uint32_t)(i / B2), l2 = (uint32_t)(i % B2);
    boff[i] = omat[l1_base[l1] + (uint64_t)l2 * nch[l1]];
  } else if (i == nb) {
    boff[nb] = total;
  }
}

// ------------------------------------------------------------------------
// Stage C: per-bucket radix sort + run-length count + spectrum
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

__device__ __forceinline__ void spectrum_add(uint32_t c, uint32_t* lhist, unsigned long long* ghist,
                                             uint64_t hist_len) {
  uint64_t m = c;
  if (m >= hist_len - 1) m = hist_len - 1;
  if (m < (uint64_t)kLdsHistBins)
    atomicAdd(&lhist[m], 1u);
  else
    atomicAdd(&ghist[m], 1ull);
}

struct SortOut {
  uint64_t* tab_hash;            // in place over rec
  uint32_t* tab_cnt;             // parallel to rec
  uint32_t* bucket_nd;           // distinct per bucket
  unsigned long long* ghist;     // spectrum
  uint64_t hist_len;
  unsigned long long* gstats;    // [0] n_distinct, [1] overflow count, [2] max bucket
  uint32_t* ovf_list;
};

__global__ void __launch_bounds__(kSortThreads) k_sort_count(uint64_t* __restrict__ rec,
                                                             const uint64_t* __restrict__ boff, uint64_t nbuckets,
                                                             int sortbits, SortOut o) {
  extern __shared__ __attribute__((aligned(16))) uint64_t smem[];
  uint64_t* A = smem;
  uint64_t* B = smem + kSortCap;
  uint32_t* whist = reinterpret_cast<uint32_t*>(smem + 2 * kSortCap);          // 8 waves x 256
  uint32_t* lhist = whist + (kSortThreads / 64) * 256;                         // kLdsHistBins
  uint32_t* scan_sm = lhist + kLdsHistBins;                                    // 64
  for (int i = threadIdx.x; i < kLdsHistBins; i += blockDim.x) lhist[i] = 0;
  unsigned long long nd_sum = 0, maxb = 0;
  __syncthreads();
  for (uint64_t bkt = blockIdx.x; bkt < nbuckets; bkt += gridDim.x) {
    const uint64_t off = boff[bkt];
    const uint32_t n = (uint32_t)(boff[bkt + 1] - off);
    if (n > maxb) maxb = n;
    if (n == 0) {
      if (threadIdx.x == 0) o.bucket_nd[bkt] = 0;
      continue;
    }
    if (n > kSortCap) {
      if (threadIdx.x == 0) {
        const unsigned long long k = atomicAdd(&o.gstats[1], 1ull);
        o.ovf_list[k] = (uint32_t)bkt;
      }
      continue;
    }
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) A[i] = rec[off + i];
    __syncthreads();
    uint64_t* S = block_radix_sort(A, B, n, sortbits, whist, scan_sm);
    uint32_t* H = reinterpret_cast<uint32_t*>(S == A ? B : A);
    // run heads -> distinct index
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
    if (threadIdx.x == 0) {
      o.bucket_nd[bkt] = nd;
      nd_sum += nd;
    }
    __syncthreads();
  }
  __syncthreads();
  const uint64_t lim = o.hist_len < (uint64_t)kLdsHistBins ? o.hist_len : (uint64_t)kLdsHistBins;
  for (uint32_t i = threadIdx.x; i < lim; i += blockDim.x)
    if (lhist[i]) atomicAdd(&o.ghist[i], (unsigned long long)lhist[i]);
  if (threadIdx.x == 0) {
    atomicAdd(&o.gstats[0], nd_sum);
    atomicMax(&o.gstats[2], maxb);
  }
}

// Oversized buckets: one workgroup each, same algorithm on global scratch.
// scratch: u64 region parallel to rec (free after stage B); heads: u32 region
// parallel to rec.
__global__ void __launch_bounds__(kSortThreads) k_sort_count_global(uint64_t* __restrict__ rec,
                                                                    const uint64_t* __restrict__ boff,
                                                                    uint64_t* __restrict__ scratch,
                                                                    uint32_t* __restrict__ heads, int sortbits,
                                                                    SortOut o) {
  __shared__ uint32_t whist[(kSortThreads / 64) * 256];
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

// ------------------------------------------------------------------------
// Host orchestration
// ------------------------------------------------------------------------
static int ceil_log2(uint64_t x) {
  int b = 0;
  while ((1ull << b) < x) ++b;
  return b;
}

struct Plan {
  int K = 0, w = 0, P = 1, pbits = 0, b1 = 0, b2 = 0;
  uint32_t B1 = 1, B2 = 1;
  int shift2 = 0, sortbits = 0;
};

// L1 bits after the shard bits; the stage-A digit (shard | L1) is capped at
// kMaxDigitBits so its LDS histogram / cursor array stays small.
constexpr int kMaxDigitBits = 12;
static int l1_bits(int K, int P) {
  const int w = 2 * K, pbits = ceil_log2((uint64_t)P);
  return std::max(0, std::min({kMaxL1Bits, kMaxDigitBits - pbits, w - pbits}));
}

// Stage A.  Digit = top (pbits + b1) bits.  extract_count returns per-digit
// record counts (host, 2^D) and leaves the scanned count matrix in the "x_omat"
// workspace; extract_scatter reuses it when called for the same (reads, K, P).
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
  APG_CHECK_HIP(hipMemcpyAsync(ds.data(), dstart, (ndig + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(sync(ctx));
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
  k_extract_scatter<<<xs.G, kExtractThreads, xs.ndig * 8, ctx->stream>>>(rv, K, make_hashp(K), xs.dshift, xs.ndig,
                                                                        omat, d_out);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return APG_OK;
}

struct CountResult {
  uint64_t* rec = nullptr;        // tab_hash (in place)
  uint32_t* tab_cnt = nullptr;
  uint32_t* bucket_nd = nullptr;
  uint64_t* boff = nullptr;
  uint64_t nbuckets = 0;
  uint64_t n_records = 0;
  apg_kstats st{};
};

// Stages B + C on records held in `src`, laid out as P source blocks, each
// grouped by l1: recv_counts[src * B1 + l1].
static int stage_count(apg_ctx* ctx, const uint64_t* src, const std::vector<uint64_t>& recv_counts, int K, int P,
                       uint64_t* hist, size_t hist_len, CountResult* res) {
  Plan pl;
  pl.K = K;
  pl.w = 2 * K;
  pl.P = P;
  pl.pbits = ceil_log2((uint64_t)P);
  pl.b1 = l1_bits(K, P);
  pl.B1 = 1u << pl.b1;
  if (recv_counts.size() != (size_t)P * pl.B1) {
    set_error("stage_count: recv_counts has wrong size");
    return APG_E_ARG;
  }
  uint64_t n = 0;
  for (auto c : recv_counts) n += c;
  const int room = pl.w - pl.pbits - pl.b1;
  const uint64_t want = (n + (uint64_t)pl.B1 * kBucketTarget - 1) / ((uint64_t)pl.B1 * kBucketTarget);
  pl.b2 = std::max(0, std::min({kMaxL2Bits, room, ceil_log2(std::max<uint64_t>(1, want))}));
  pl.B2 = 1u << pl.b2;
  pl.shift2 = room - pl.b2;
  pl.sortbits = pl.shift2;
  res->n_records = n;
  vlog(ctx, "count: K=%d P=%d records=%llu b1=%d b2=%d sortbits=%d", K, P, (unsigned long long)n, pl.b1, pl.b2,
       pl.sortbits);

  // Segments of each l1 in source order -> chunks.
  std::vector<uint64_t> src_base(P + 1, 0);
  for (int s = 0; s < P; ++s) {
    uint64_t t = 0;
    for (uint32_t l = 0; l < pl.B1; ++l) t += recv_counts[(size_t)s * pl.B1 + l];
    src_base[s + 1] = src_base[s] + t;
  }
  std::vector<uint64_t> seg_start((size_t)P * pl.B1);
  for (int s = 0; s < P; ++s) {
    uint64_t pos = src_base[s];
    for (uint32_t l = 0; l < pl.B1; ++l) {
      seg_start[(size_t)s * pl.B1 + l] = pos;
      pos += recv_counts[(size_t)s * pl.B1 + l];
    }
  }
  const uint64_t max_chunks = 32768;
  uint64_t C = std::max<uint64_t>(8192, (n + max_chunks - 1) / max_chunks);
  C = std::min<uint64_t>(C, 1u << 30);
  std::vector<Chunk> chunks;
  std::vector<uint64_t> l1_base(pl.B1);
  std::vector<uint32_t> nch(pl.B1);
  uint64_t mat_base = 0;
  for (uint32_t l = 0; l < pl.B1; ++l) {
    const size_t first = chunks.size();
    for (int s = 0; s < P; ++s) {
      const uint64_t st = seg_start[(size_t)s * pl.B1 + l], len = recv_counts[(size_t)s * pl.B1 + l];
      for (uint64_t o = 0; o < len; o += C) chunks.push_back(Chunk{st + o, 0, (uint32_t)std::min(C, len - o), 0});
    }
    if (chunks.size() == first) chunks.push_back(Chunk{0, 0, 0, 0});  // every l1 gets a matrix column
    const uint32_t k = (uint32_t)(chunks.size() - first);
    for (uint32_t i = 0; i < k; ++i) {
      chunks[first + i].mat = mat_base + i;
      chunks[first + i].stride = k;
    }
    l1_base[l] = mat_base;
    nch[l] = k;
    mat_base += (uint64_t)k * pl.B2;
  }
  const uint64_t nmat = mat_base;

  uint64_t *rec = nullptr, *boff = nullptr, *omat = nullptr, *d_l1_base = nullptr;
  uint32_t *cmat = nullptr, *d_nch = nullptr, *tab_cnt = nullptr, *bucket_nd = nullptr, *ovf_list = nullptr;
  Chunk* d_chunks = nullptr;
  const uint64_t nb = (uint64_t)pl.B1 * pl.B2;
  APG_TRY(workspace_t(ctx, "c_rec", std::max<uint64_t>(n, 1), &rec));
  APG_TRY(workspace_t(ctx, "c_tabcnt", std::max<uint64_t>(n, 1), &tab_cnt));
  APG_TRY(workspace_t(ctx, "c_cmat", nmat, &cmat));
  APG_TRY(workspace_t(ctx, "c_omat", nmat + 1, &omat));
  APG_TRY(workspace_t(ctx, "c_chunks", chunks.size(), &d_chunks));
  APG_TRY(workspace_t(ctx, "c_l1base", pl.B1, &d_l1_base));
  APG_TRY(workspace_t(ctx, "c_nch", pl.B1, &d_nch));
  APG_TRY(workspace_t(ctx, "c_boff", nb + 1, &boff));
  APG_TRY(workspace_t(ctx, "c_bnd", nb, &bucket_nd));
  APG_TRY(workspace_t(ctx, "c_ovf", nb, &ovf_list));
  unsigned long long *ghist = nullptr, *gstats = nullptr;
  const uint64_t hl = std::max<uint64_t>(hist_len, 2);
  APG_TRY(workspace_t(ctx, "c_hist", hl, &ghist));
  APG_TRY(workspace_t(ctx, "c_gstats", 4, &gstats));
  APG_CHECK_HIP(hipMemcpyAsync(d_chunks, chunks.data(), chunks.size() * sizeof(Chunk), hipMemcpyHostToDevice,
                               ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(d_l1_base, l1_base.data(), pl.B1 * 8, hipMemcpyHostToDevice, ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(d_nch, nch.data(), pl.B1 * 4, hipMemcpyHostToDevice, ctx->stream));
  APG_CHECK_HIP(hipMemsetAsync(ghist, 0, hl * 8, ctx->stream));
  APG_CHECK_HIP(hipMemsetAsync(gstats, 0, 4 * 8, ctx->stream));

  // Stage B
  const uint32_t nchunks = (uint32_t)chunks.size();
  kbegin(ctx, "rec_count", n * 8 + nmat * 4);
  k_rec_count<<<nchunks, 256, pl.B2 * 4, ctx->stream>>>(src, d_chunks, pl.shift2, pl.B2, cmat);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  APG_TRY(scan_u32_u64(ctx, cmat, nmat, omat, "c"));
  kbegin(ctx, "rec_scatter", n * 16 + nmat * 8);
  k_rec_scatter<<<nchunks, 256, pl.B2 * 8, ctx->stream>>>(src, d_chunks, pl.shift2, pl.B2, omat, rec);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  k_bucket_offsets<<<(nb + 1 + 255) / 256, 256, 0, ctx->stream>>>(omat, d_l1_base, d_nch, pl.B1, pl.B2, n, boff);
  APG_CHECK_HIP(hipGetLastError());

  // Stage C
  SortOut so{rec, tab_cnt, bucket_nd, ghist, hl, gstats, ovf_list};
  const size_t lds = 2 * kSortCap * 8 + (kSortThreads / 64) * 256 * 4 + kLdsHistBins * 4 + 64 * 4;
  const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>(nb, (uint64_t)ctx->n_cu * 8));
  kbegin(ctx, "sort_count", n * 8 + n * 12 + (nb + 1) * 8 + nb * 4);
  k_sort_count<<<grid, kSortThreads, lds, ctx->stream>>>(rec, boff, nb, pl.sortbits, so);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  unsigned long long hs[4];
  APG_CHECK_HIP(hipMemcpyAsync(hs, gstats, sizeof hs, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(sync(ctx));
  if (hs[1]) {
    // Oversized buckets: scratch = a u64 region parallel to rec.
    uint64_t* scratch = nullptr;
    uint32_t* heads = nullptr;
    APG_TRY(workspace_t(ctx, "c_scratch", n, &scratch));
    APG_TRY(workspace_t(ctx, "c_heads", n, &heads));
    vlog(ctx, "count: %llu oversized buckets -> global sort", hs[1]);
    kbegin(ctx, "sort_count_global", 0);
    k_sort_count_global<<<(uint32_t)hs[1], kSortThreads, 0, ctx->stream>>>(rec, boff, scratch, heads, pl.sortbits,
                                                                          so);
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
    APG_CHECK_HIP(hipMemcpyAsync(hs, gstats, sizeof hs, hipMemcpyDeviceToHost, ctx->stream));
  }
  if (hist && hist_len) {
    APG_CHECK_HIP(hipMemcpyAsync(hist, ghist, hist_len * 8, hipMemcpyDeviceToHost, ctx->stream));
  }
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

static int spectrum_impl(apg_ctx* ctx, const apg_dreads* dr, int K, uint64_t* hist, size_t hist_len,
                         CountResult* res) {
  APG_REQUIRE(ctx && dr, "spectrum: NULL ctx/reads");
  APG_REQUIRE(K >= 1 && K <= 32, "spectrum: K must be in [1, 32] for the 64-bit path");
  APG_REQUIRE(hist_len == 0 || hist_len >= 2, "spectrum: hist_len must be 0 or >= 2");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  std::vector<uint64_t> counts;
  APG_TRY(extract_count(ctx, dr, K, 1, &counts));
  uint64_t* buf = nullptr;
  APG_TRY(workspace_t(ctx, "x_records", std::max<uint64_t>(ctx->xstate.total, 1), &buf));
  APG_TRY(extract_scatter(ctx, dr, K, 1, buf));
  return stage_count(ctx, buf, counts, K, 1, hist, hist_len, res);
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

int apg_kmer_spectrum_dev(apg_ctx* ctx, const apg_dreads* reads, int K, uint64_t* hist, size_t hist_len,
                          apg_kstats* stats) {
  CountResult r;
  APG_TRY(spectrum_impl(ctx, reads, K, hist, hist_len, &r));
  if (stats) *stats = r.st;
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
  APG_REQUIRE(keys && counts && n_distinct, "apg_kmer_count: NULL output");
  *keys = nullptr;
  *counts = nullptr;
  *n_distinct = 0;
  apg_dreads* dr = nullptr;
  APG_TRY(apg_reads_upload(ctx, reads, &dr));
  CountResult r;
  int rc = spectrum_impl(ctx, dr, K, nullptr, 0, &r);
  apg_reads_free(dr);
  if (rc) return rc;
  const uint64_t nd = r.st.n_distinct;
  uint64_t* dense_off = nullptr;
  uint64_t* d_keys = nullptr;
  uint32_t* d_cnt = nullptr;
  APG_TRY(workspace_t(ctx, "t_dense_off", r.nbuckets + 1, &dense_off));
  APG_TRY(workspace_t(ctx, "t_keys", std::max<uint64_t>(nd, 1), &d_keys));
  APG_TRY(workspace_t(ctx, "t_cnt", std::max<uint64_t>(nd, 1), &d_cnt));
  APG_TRY(scan_u32_u64(ctx, r.bucket_nd, r.nbuckets, dense_off, "t"));
  const uint64_t grid = std::max<uint64_t>(1, std::min<uint64_t>(r.nbuckets, (uint64_t)ctx->n_cu * 16));
  kbegin(ctx, "compact_table", nd * 24);
  k_compact_table<<<grid, 256, 0, ctx->stream>>>(r.rec, r.tab_cnt, r.boff, r.bucket_nd, dense_off, r.nbuckets,
                                                  make_hashp(K), d_keys, d_cnt);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  auto* hk = (uint64_t*)std::malloc(std::max<uint64_t>(nd, 1) * 8);
  auto* hc = (uint32_t*)std::malloc(std::max<uint64_t>(nd, 1) * 4);
  if (!hk || !hc) {
    std::free(hk);
    std::free(hc);
    return APG_E_NOMEM;
  }
  APG_CHECK_HIP(hipMemcpyAsync(hk, d_keys, nd * 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(hc, d_cnt, nd * 4, hipMemcpyDeviceToHost, ctx->stream));
  rc = sync(ctx);
  if (rc) {
    std::free(hk);
    std::free(hc);
    return rc;
  }
  *keys = hk;
  *counts = hc;
  *n_distinct = nd;
  if (stats) *stats = r.st;
  return APG_OK;
}

int apg_shard_count(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards, uint64_t* send_counts) {
  APG_REQUIRE(ctx && reads && send_counts, "apg_shard_count: NULL argument");
  APG_REQUIRE(K >= 1 && K <= 32, "apg_shard_count: K must be in [1, 32]");
  APG_REQUIRE(n_shards >= 1 && n_shards <= 64 && (n_shards & (n_shards - 1)) == 0,
              "apg_shard_count: n_shards must be a power of two in [1, 64]");
  APG_REQUIRE(2 * K >= ceil_log2((uint64_t)n_shards), "apg_shard_count: K too small for n_shards");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  std::vector<uint64_t> dc;
  APG_TRY(extract_count(ctx, reads, K, n_shards, &dc));
  std::memcpy(send_counts, dc.data(), dc.size() * 8);
  return APG_OK;
}

int apg_shard_scatter(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards, uint64_t* d_send) {
  APG_REQUIRE(ctx && reads, "apg_shard_scatter: NULL argument");
  APG_REQUIRE(K >= 1 && K <= 32, "apg_shard_scatter: K must be in [1, 32]");
  APG_REQUIRE(n_shards >= 1 && n_shards <= 64 && (n_shards & (n_shards - 1)) == 0,
              "apg_shard_scatter: n_shards must be a power of two in [1, 64]");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  APG_TRY(extract_scatter(ctx, reads, K, n_shards, d_send));
  return sync(ctx);
}

int apg_shard_spectrum(apg_ctx* ctx, const uint64_t* d_recv, const uint64_t* recv_counts, int K, int n_shards,
                       uint64_t* hist, size_t hist_len, apg_kstats* stats) {
  APG_REQUIRE(ctx && recv_counts, "apg_shard_spectrum: NULL argument");
  APG_REQUIRE(K >= 1 && K <= 32, "apg_shard_spectrum: K must be in [1, 32]");
  APG_REQUIRE(n_shards >= 1 && n_shards <= 64 && (n_shards & (n_shards - 1)) == 0,
              "apg_shard_spectrum: n_shards must be a power of two in [1, 64]");
  APG_REQUIRE(hist_len == 0 || hist_len >= 2, "apg_shard_spectrum: hist_len must be 0 or >= 2");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const uint32_t B1 = 1u << l1_bits(K, n_shards);
  std::vector<uint64_t> rc(recv_counts, recv_counts + (size_t)n_shards * B1);
  uint64_t n = 0;
  for (auto c : rc) n += c;
  APG_REQUIRE(n == 0 || d_recv, "apg_shard_spectrum: d_recv is NULL");
  CountResult r;
  APG_TRY(stage_count(ctx, d_recv, rc, K, n_shards, hist, hist_len, &r));
  if (stats) *stats = r.st;
  return APG_OK;
}

int apg_shard_bins(int K, int n_shards) {
  if (K < 1 || K > 32 || n_shards < 1) return APG_E_ARG;
  return 1 << l1_bits(K, n_shards);
}

}  // extern "C"
