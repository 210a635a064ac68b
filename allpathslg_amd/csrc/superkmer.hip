// superkmer.hip — minimizer-partitioned k-mer counting for K <= 32 (spectrum
// and solid-set modes).
//
// Same result as the hash-record pipeline of kmer_spectrum.hip (which keeps
// serving the hash-ordered table of apg_kmer_count), with a fraction of its
// HBM traffic: instead of one 8-byte hash per K-mer instance, a read is cut
// into super-k-mers — maximal runs of consecutive K-mers whose minimizer (the
// smallest hashed canonical m-mer of the K-mer, m = min(K, max(10, min(16, K-8)));
// m = 16 for K >= 24 keeps a minimizer's genome occurrences near one, since a
// bucket must hold every distinct K-mer of its minimizers)
// is the same — and each run travels as ONE 16-byte record holding its bases.
// Every K-mer has exactly one minimizer, and a K-mer and its reverse
// complement contain the same canonical m-mers, so all instances of a
// canonical K-mer land in the partition of its minimizer key.
//
//   sk_count / sk_scatter  tiles of reads staged in LDS, one thread per read
//                          rolling m-mers with a van Herk / Gil-Werman
//                          window minimum, and the records scattered into 2^D groups of the key's top bits via
//                          an LDS-staged round (count matrix + scan, no global
//                          atomics), D = shard bits + kSkDigitBits
//   part_level<SK16>       LDS-staged partition levels on the key's next bits
//                          until a bucket holds ~kSkBucketKmers K-mers
//   sk_bucket              one workgroup per bucket expands its records'
//                          K-mers into an LDS open-addressing table (full
//                          64-bit hash keys, CAS insert, atomic count), bins
//                          the counts into the spectrum and, in solid mode,
//                          appends hashes with count >= min_solid (one global
//                          atomic per bucket)
//   sk_big                 buckets whose distinct K-mers overflow the LDS
//                          table are counted together in one global table
// A record's bases: for K-mers [a, a+n) of the read, bases [a, a+n+K-1),
// n <= 41 - K.  Algorithmic bytes per 100-bp read at K = 25: ~12 records of
// 16 B (vs 76 x 8 B hash records).
#include <algorithm>
#include <functional>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <type_traits>
#include <vector>

#include "apg_core.hpp"
#include "kmer_common.hpp"
#include "kmer_internal.hpp"
#include "partition.hpp"
#include "superkmer.hpp"

namespace apg {

constexpr int kSkThreads = 256;
constexpr int kSkMaxBlocks = 8192;
constexpr int kSkBases = 40;
constexpr int kSkDigitBits = 5;
constexpr uint64_t kSkBucketKmers = 4096;  // K-mer instances per bucket the planner aims for
constexpr uint32_t kSkTab = 2048;          // LDS table slots (u64 canonical K-mer + u32 count)
constexpr int kSkHistBins = 128;  // LDS spectrum bins (counts above go to global atomics); keeps k_sk_bucket<false> under 40 KiB LDS = 4 blocks/CU
constexpr uint32_t kSkSlotCap = 6144;  // weak pass: instances per bucket with a recorded slot (LDS: 3 blocks/CU)
constexpr uint32_t kSkWaveSlots = kSkSlotCap / (kSkThreads / 64);  // recorded slots per wave
constexpr int kSkListCap = 1024;  // parked records per tile (8 KiB of LDS)
// A table this full is given up on: an insert that finds no room within
// kSkProbeMax slots marks the bucket for the global table (a full 2048-slot
// table otherwise costs every further insert a scan of all of it).
constexpr uint32_t kSkProbeMax = 256;
// Buckets of more records than this go to the global table without an LDS
// attempt (repeat-rich genomes: one minimizer shared by thousands of copies).
constexpr uint32_t kSkHeavyRecords = 8192;

struct SkP {
  using U = uint32_t;  // m <= 16
  int K, m, w, maxnk;
  uint64_t mmask;  // 2m bits
  HashP hp;
  // > 0: records of more than `split` K-mers leave as pieces of <= split
  // (the packed SKP form holds <= 32 bases); the count pass counts pieces
  uint32_t split = 0;
  // SKP records in the 34-bit-position form (skp_unpack's `wide`)
  bool wide = false;
  // the count walk keeps its column in registers (w == kSkRegW or kSkRegW + 1; APG_SK_REG=0: off)
  bool reg = false;
};
constexpr int kSkRegW = 9;  // the windows of the K = 24 and K = 25 walks (m = kSkRegM)
constexpr int kSkRegM = 16;
// the record queues live in the count pass's p.w x kSkThreads column words
static_assert(kSkRegW * kSkThreads >= (int)sk_regq_words(kSkThreads, kSkRegW) &&
                  (kSkRegW + 1) * kSkThreads >= (int)sk_regq_words(kSkThreads, kSkRegW + 1),
              "register walk queues exceed the count pass's LDS");
__host__ __device__ inline uint32_t sk_pieces(uint32_t n, uint32_t split) {
  return split && n > split ? (n + split - 1) / split : 1u;
}

static SkP make_skp(int K) {
  SkP p;
  p.K = K;
  p.m = std::min(K, std::max(10, std::min(16, K - 8)));
  // APG_SK_M=m (10 <= m <= 16, m < K - 1): the minimizer length of every
  // K <= 32 walk (A/B of records per read against bucket skew)
  static const int m_env = getenv("APG_SK_M") ? atoi(getenv("APG_SK_M")) : 0;
  if (m_env >= 10 && m_env <= 16 && m_env < K - 1) p.m = m_env;
  p.w = K - p.m + 1;
  p.maxnk = std::min(kSkBases - K + 1, 255);
  p.mmask = p.m >= 32 ? ~0ull : ((1ull << (2 * p.m)) - 1);
  p.hp = make_hashp(K);
  static const bool reg = [] {
    const char* e = getenv("APG_SK_REG");
    return !(e && !strcmp(e, "0"));
  }();
  p.reg = reg && p.m == kSkRegM && (p.w == kSkRegW || p.w == kSkRegW + 1);
  return p;
}


// Record flanks (bits 40..45 of w0): the read's bases just before and just
// after the record's bases, with presence bits.  The K-mer counts ignore them;
// the fused K / K+1 count (k_sk_bucket<.., UP>) needs them for the K+1-mers
// that straddle two records.  Record dedup fingerprints and compares a record
// without them (kSkFlankMask).
constexpr uint64_t kSkFlankMask = 0x3full << 40;
__device__ __forceinline__ uint64_t sk_flank_bits(uint32_t lb, uint32_t rb, bool hl, bool hr) {
  return ((uint64_t)(lb | (rb << 2) | ((uint32_t)hl << 4) | ((uint32_t)hr << 5))) << 40;
}

__device__ __forceinline__ SK16 make_rec(const uint8_t* rd, uint32_t L, uint32_t a, uint32_t n, uint32_t key, int K) {
  const uint32_t nb = n + (uint32_t)K - 1;  // <= 40
  uint64_t lo = sk_lsb64(rd, a);
  uint64_t hi = nb > 32 ? sk_lsb64(rd, a + 32) : 0;
  if (nb < 32)
    lo &= (1ull << (2 * nb)) - 1;
  else
    hi &= nb == 32 ? 0ull : ((1ull << (2 * (nb - 32))) - 1);
  const bool hl = a > 0, hr = a + nb < L;
  const uint32_t lb = hl ? (rd[(a - 1) >> 2] >> (2 * ((a - 1) & 3))) & 3 : 0;
  const uint32_t rb = hr ? (rd[(a + nb) >> 2] >> (2 * ((a + nb) & 3))) & 3 : 0;
  SK16 r;
  r.w0 = (uint64_t)part_key(key) | ((uint64_t)n << 32) | sk_flank_bits(lb, rb, hl, hr) | ((lo & 0xffffull) << 48);
  r.w1 = (lo >> 16) | (hi << 48);
  return r;
}


// cmat[digit * G + block] = records of `block` with key digit `digit`;
// kdig[digit] += K-mers of those records.  k_sk_scatter walks the same tiles
// and reads in the same way, so its per-(digit, block) counts match.
__global__ void __launch_bounds__(kSkThreads) k_sk_count(SkReads rv, SkP p, int D, uint32_t* __restrict__ cmat,
                                                         unsigned long long* __restrict__ kdig, SkDesc dd) {
  __shared__ SkTile<kSkThreads> T;
  __shared__ uint32_t hist[256], khist[256];
  __shared__ SkList<1> lst;  // f runs in place
  __shared__ uint32_t dpos, dovf;
  extern __shared__ uint32_t sbuf[];  // p.w x kSkThreads van Herk columns
  const uint32_t ndig = 1u << D;
  const uint32_t G = gridDim.x, b = blockIdx.x;
  for (uint32_t i = threadIdx.x; i < ndig; i += blockDim.x) hist[i] = khist[i] = 0;
  if (threadIdx.x == 0) dpos = dovf = 0;
  uint64_t r0, r1;
  sk_read_range(rv.n_reads, G, b, &r0, &r1);
  SkDescWriter W(dd, rv, r0, r1, &dpos, &dovf);
  auto f = [&](const uint8_t*, uint32_t, uint32_t a, uint32_t n, uint32_t key, uint32_t q) {
    const uint32_t d = D ? part_key(key) >> (32 - D) : 0;
    atomicAdd(&hist[d], sk_pieces(n, p.split));
    atomicAdd(&khist[d], n);
    W.put(a, n, key, q);
  };
  for (uint64_t t0 = r0; t0 < r1;) {
    const uint32_t n = sk_load_tile(rv, t0, r1, T);
    if (n && p.reg && p.w == kSkRegW)
      sk_walk_tile<kSkThreads, false, false, kSkRegW, kSkRegM>(p, T, n, sbuf + threadIdx.x, lst, f);
    else if (n && p.reg)
      sk_walk_tile<kSkThreads, false, false, kSkRegW + 1, kSkRegM>(p, T, n, sbuf + threadIdx.x, lst, f);
    else if (n)
      sk_walk_tile<kSkThreads, false, false>(p, T, n, sbuf + threadIdx.x, lst, f);
    else
      sk_walk_global<kSkThreads, false>(rv, p, T, t0, sbuf + threadIdx.x, f);
    __syncthreads();
    W.tile_done(t0);
    t0 += n ? n : 1;
  }
  W.block_done();
  for (uint32_t i = threadIdx.x; i < ndig; i += blockDim.x) {
    cmat[(uint64_t)i * G + b] = hist[i];
    if (khist[i]) atomicAdd(&kdig[i], (unsigned long long)khist[i]);
  }
}

// Scatter outputs: plain 16-byte records, 24-byte records with the position
// of their first K-mer, or 16-byte records + the positions in a parallel
// array (the multi-GPU weak-mask return: records travel, positions stay).
struct SplitOut {
  SK16* rec;
  uint64_t* pos;
};
template <typename O> struct OutWantsPos { static constexpr bool value = false; };
template <> struct OutWantsPos<SK24*> { static constexpr bool value = true; };
template <> struct OutWantsPos<SplitOut> { static constexpr bool value = true; };
// packed partition records: 32-bit positions, or (wide) 34-bit positions
// with records of <= 31 bases, position bits 32..33 in w1's top two bits
struct SkpOut {
  SKP* rec;
  bool wide;
};
template <> struct OutWantsPos<SkpOut> { static constexpr bool value = true; };
// SK16 layout (<= 32 bases) + position -> the packed partition record
__device__ __forceinline__ void rec_put(SkpOut out, uint64_t i, const SK16& x, uint64_t pos) {
  uint64_t o[2];
  skp_pack(x.w0, x.w1, pos, 0, o);
  if (out.wide) o[1] = (o[1] & ((1ull << 62) - 1)) | ((pos >> 32) << 62);
  out.rec[i] = SKP{o[0], o[1]};
}
__device__ __forceinline__ void rec_put(SplitOut out, uint64_t i, const SK16& x, uint64_t pos) {
  out.rec[i] = x;
  out.pos[i] = pos;
}
__device__ __forceinline__ void rec_put(SK16* out, uint64_t i, const SK16& x, uint64_t) { out[i] = x; }
__device__ __forceinline__ void rec_put(SK24* out, uint64_t i, const SK16& x, uint64_t pos) {
  out[i] = SK24{x.w0, x.w1, pos};
}
__device__ __forceinline__ SK16 rec_head(const SK16& r) { return r; }
__device__ __forceinline__ SK16 rec_head(const SK24& r) { return SK16{r.w0, r.w1}; }

// The bucket kernels' record accessors: SK16 / SK24 (the head is the 16-byte
// super-k-mer form) and the packed SKP the partition levels carry, unpacked
// in registers (no unpacking level: 16 bytes per record written by the last
// level and read by the bucket kernels instead of 24).  RecPos: the record
// carries a position (a base position, a receive index, or — a distinct
// record of the fused K+1 pass — its multiplicity).
template <typename R> struct RecPos { static constexpr bool value = false; };
template <> struct RecPos<SK24> { static constexpr bool value = true; };
template <> struct RecPos<SKP> { static constexpr bool value = true; };
__device__ __forceinline__ SK16 rec_head(const SK16& r, const SkP&) { return r; }
__device__ __forceinline__ SK16 rec_head(const SK24& r, const SkP&) { return SK16{r.w0, r.w1}; }
__device__ __forceinline__ SK16 rec_head(const SKP& r, const SkP& p) {
  uint64_t o[3];
  skp_unpack(r.w0, r.w1, o, p.wide);
  return SK16{o[0], o[1]};
}
__device__ __forceinline__ uint64_t rec_pos(const SK16&, const SkP&) { return 0; }
__device__ __forceinline__ uint64_t rec_pos(const SK24& r, const SkP&) { return r.pos; }
__device__ __forceinline__ uint64_t rec_pos(const SKP& r, const SkP& p) {
  return ((r.w0 >> 10) & 0xffffffffull) | (p.wide ? (r.w1 >> 62) << 32 : 0ull);
}
__device__ __forceinline__ uint32_t rec_nk(const SK16& r) { return (uint32_t)(r.w0 >> 32) & 0xff; }
__device__ __forceinline__ uint32_t rec_nk(const SK24& r) { return (uint32_t)(r.w0 >> 32) & 0xff; }
__device__ __forceinline__ uint32_t rec_nk(const SKP& r) { return (uint32_t)(r.w0 >> 6) & 15; }
// a distinct record of the solid-set count (dout: its multiplicity in the key
// bits) as a record of type R whose position is that multiplicity
template <typename R> __device__ __forceinline__ R rec_from_drec(const SK16& d);
template <> __device__ __forceinline__ SK24 rec_from_drec<SK24>(const SK16& d) {
  return SK24{d.w0, d.w1, d.w0 & 0xffffffffull};
}
template <> __device__ __forceinline__ SKP rec_from_drec<SKP>(const SK16& d) {
  uint64_t o[2];
  skp_pack(d.w0, d.w1, d.w0 & 0xffffffffull, 0, o);  // <= 32 bases: it came from a packed record
  return SKP{o[0], o[1]};
}

// Each record goes straight to the next slot of its digit's run for this
// block (omat, LDS cursor): the run's size is fixed by k_sk_count, the order
// inside a run is immaterial to counting.  SK24 records also carry the global
// base position of their first K-mer.
template <typename O>
__global__ void __launch_bounds__(kSkThreads) k_sk_scatter(SkReads rv, SkP p, int D,
                                                           const uint64_t* __restrict__ omat, O out, SkDesc dd) {
  __shared__ SkTile<kSkThreads> T;
  __shared__ unsigned long long cur[256];
  __shared__ SkList<kSkListCap> lst;
  extern __shared__ uint32_t sbuf[];  // p.w x kSkThreads van Herk columns
  const uint32_t ndig = 1u << D;
  const uint32_t G = gridDim.x, b = blockIdx.x;
  for (uint32_t d = threadIdx.x; d < ndig; d += blockDim.x) cur[d] = omat[(uint64_t)d * G + b];
  if (threadIdx.x == 0) lst.cnt = 0;
  uint64_t r0, r1;
  sk_read_range(rv.n_reads, G, b, &r0, &r1);
  uint64_t t0 = r0;
  auto f = [&](const uint8_t* rd, uint32_t L, uint32_t a, uint32_t n, uint32_t key, uint32_t q) {
    const uint32_t np = sk_pieces(n, p.split);
    for (uint32_t j = 0; j < np; ++j) {  // pieces of <= p.split K-mers (one piece unless split)
      const uint32_t aj = a + j * p.split, nj = np == 1 ? n : min(p.split, n - j * p.split);
      const SK16 x = make_rec(rd, L, aj, nj, key, p.K);
      const uint32_t d = D ? (uint32_t)x.w0 >> (32 - D) : 0;
      const uint64_t pos = OutWantsPos<O>::value ? rv.base_off[t0 + q] + aj : 0;  // the read's first base + aj
      rec_put(out, atomicAdd(&cur[d], 1ull), x, pos);
    }
  };
  if (dd.desc && !dd.flag[b]) return;  // k_sk_replay wrote this block's records
  while (t0 < r1) {
    const uint32_t n = sk_load_tile(rv, t0, r1, T);
    if (n)
      sk_walk_tile<kSkThreads, false, true>(p, T, n, sbuf + threadIdx.x, lst, f);
    else
      sk_walk_global<kSkThreads, false>(rv, p, T, t0, sbuf + threadIdx.x, f);
    __syncthreads();
    t0 += n ? n : 1;
  }
}

// The scatter of the blocks whose count pass kept descriptors (the walk
// kernel above takes the flagged rest): no van Herk column or record list, so
// 14 KiB of LDS per block instead of ~30.  Per tile, the descriptor count,
// the reads' first-base positions and the first batch of descriptors are
// loaded while the tile streams in; each lane then builds its records from
// the LDS tile (ds_read, no generic-pointer loads), positions from LDS, with
// kSkReplayBatch descriptor loads in flight (8: 13.2 -> 12.7 ms against 4) instead of one dependent chain
// per record.
constexpr uint32_t kSkReplayBatch = 8;
template <typename O>
__global__ void __launch_bounds__(kSkThreads) k_sk_replay(SkReads rv, SkP p, int D, const uint64_t* __restrict__ omat,
                                                          O out, SkDesc dd) {
  constexpr bool WP = OutWantsPos<O>::value;
  constexpr uint32_t NT = kSkThreads;
  __shared__ SkTile<kSkThreads> T;
  __shared__ unsigned long long cur[256];
  __shared__ uint64_t tpos[WP ? NT : 1];
  const uint32_t ndig = 1u << D;
  const uint32_t G = gridDim.x, b = blockIdx.x, tid = threadIdx.x;
  if (!dd.desc || dd.flag[b]) return;  // block-uniform: k_sk_scatter walks this block
  for (uint32_t d = tid; d < ndig; d += NT) cur[d] = omat[(uint64_t)d * G + b];
  uint64_t r0, r1;
  sk_read_range(rv.n_reads, G, b, &r0, &r1);
  uint64_t off = dd.lo(rv, r0);
  uint64_t dq[kSkReplayBatch];
  auto load_batch = [&](uint64_t i0) {
#pragma unroll
    for (uint32_t u = 0; u < kSkReplayBatch; ++u) {
      const uint64_t i = off + i0 + u * NT + tid;
      dq[u] = i < dd.slots ? dd.desc[i] : 0;  // past the tile's count: unused
    }
  };
  // one record from its descriptor; bases from the LDS tile at bit `bit0`,
  // or (tile of one over-long read) from HBM
  auto build = [&](uint32_t q, uint32_t a, uint32_t nk, uint32_t key, uint32_t n_tile, const uint8_t* g) {
    SK16 x;
    if (n_tile) {
      const uint32_t nb = nk + (uint32_t)p.K - 1;  // <= 40
      const uint32_t bo = T.rbo[q] * 8 + 2 * a;
      const uint32_t i = bo >> 5, s = bo & 31;
      const uint32_t w0 = T.words[i], w1 = T.words[i + 1], w2 = T.words[i + 2], w3 = T.words[i + 3];
      uint64_t lo = (uint64_t)__builtin_amdgcn_alignbit(w1, w0, s) | ((uint64_t)__builtin_amdgcn_alignbit(w2, w1, s) << 32);
      uint64_t hi = __builtin_amdgcn_alignbit(w3, w2, s);
      if (nb < 32) lo &= (1ull << (2 * nb)) - 1;
      hi = nb > 32 ? hi & ((1ull << (2 * (nb - 32))) - 1) : 0;
      // flanks from the tile: the base before bit bo, the base at bit bo + 2 nb
      const bool hl = a > 0, hr = a + nb < T.rlen[q];
      const uint32_t bl = bo - 2, br = bo + 2 * nb;
      const uint32_t lb = hl ? (T.words[bl >> 5] >> (bl & 31)) & 3 : 0;
      const uint32_t rb = hr ? (T.words[br >> 5] >> (br & 31)) & 3 : 0;
      x.w0 = (uint64_t)part_key(key) | ((uint64_t)nk << 32) | sk_flank_bits(lb, rb, hl, hr) |
             ((lo & 0xffffull) << 48);
      x.w1 = (lo >> 16) | (hi << 48);
    } else {
      x = make_rec(g, T.rlen[q], a, nk, key, p.K);
    }
    return x;
  };
  auto emit = [&](uint64_t d, uint32_t n_tile, const uint8_t* g) {
    const uint32_t q = (uint32_t)(d >> 56), a = (uint32_t)(d >> 32) & 0xffffu, nk = (uint32_t)(d >> 48) & 0xffu;
    // a record longer than p.split K-mers leaves as pieces through its own
    // cursor add (rare: runs longer than the window need a repeated minimizer)
    const bool piecewise = p.split && nk > p.split;
    const uint32_t dg = D ? part_key((uint32_t)d) >> (32 - D) : 0;
    if (piecewise) {
      const uint32_t np = sk_pieces(nk, p.split);
      const unsigned long long b0 = atomicAdd(&cur[dg], (unsigned long long)np);
      for (uint32_t j = 0; j < np; ++j) {
        const uint32_t aj = a + j * p.split, nj = min(p.split, nk - j * p.split);
        uint64_t pj = 0;
        if constexpr (WP) pj = tpos[q] + aj;
        rec_put(out, b0 + j, build(q, aj, nj, (uint32_t)d, n_tile, g), pj);
      }
    }
    SK16 x{0, 0};
    if (!piecewise) x = build(q, a, nk, (uint32_t)d, n_tile, g);
    uint64_t pos = 0;
    if constexpr (WP) pos = tpos[q] + a;
    // the wave's lanes of one digit take consecutive slots through one
    // cursor add by the lowest of them (D ballots find the peers): ~2^D
    // distinct-address atomics per wave instead of 64 on 2^D addresses
    uint64_t peers = __ballot(!piecewise);
    for (int k = 0; k < D; ++k) {
      const uint64_t bk = __ballot((dg >> k) & 1u);
      peers &= ((dg >> k) & 1u) ? bk : ~bk;
    }
    const uint32_t ln = __lane_id();
    const uint32_t rank = (uint32_t)__popcll(peers & ((1ull << ln) - 1));
    const int leader = peers ? __ffsll((long long)peers) - 1 : 0;
    unsigned long long base = 0;
    if (!piecewise && rank == 0) base = atomicAdd(&cur[dg], (unsigned long long)__popcll(peers));
    const uint32_t blo = (uint32_t)__shfl((int)(uint32_t)base, leader, 64);
    const uint32_t bhi = (uint32_t)__shfl((int)(uint32_t)(base >> 32), leader, 64);
    if (!piecewise) rec_put(out, (((uint64_t)bhi << 32) | blo) + rank, x, pos);
  };
  for (uint64_t t0 = r0; t0 < r1;) {
    const uint32_t c = dd.tcnt[t0];
    uint64_t pb = 0;
    if constexpr (WP) {
      if (t0 + tid < r1) pb = rv.base_off[t0 + tid];
    }
    load_batch(0);
    const uint32_t n = sk_load_tile(rv, t0, r1, T);  // ends with a barrier
    if constexpr (WP) {
      if (tid < (n ? n : 1u)) tpos[tid] = pb;
      __syncthreads();
    }
    const uint8_t* g = n ? nullptr : rv.packed + rv.byte_off[t0];  // a read too long for a tile: from HBM
    for (uint32_t i0 = 0; i0 < c; i0 += kSkReplayBatch * NT) {  // block-uniform
      if (i0) load_batch(i0);
#pragma unroll
      for (uint32_t u = 0; u < kSkReplayBatch; ++u)
        if (i0 + u * NT + tid < c) emit(dq[u], n, g);
    }
    off += c;
    __syncthreads();  // the next tile overwrites T and tpos
    t0 += n ? n : 1;
  }
}

__global__ void k_sk_digit_starts(const uint64_t* __restrict__ omat, uint32_t ndig, uint32_t G,
                                  uint64_t* __restrict__ ds) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d <= ndig) ds[d] = omat[(uint64_t)d * G];
}

// ---------------------------------------------------------------------------
// Bucket counting
// ---------------------------------------------------------------------------
// Canonical K-mer t (t + K <= 40) of a record: the record's bases as an
// 80-bit LSB-first string, a 64-bit window at base t, fw = rev2 >> (64 - 2K),
// rc = complement (already most-significant-first).
// Branch-free: the 80-bit string is three 32-bit limbs a0..a2 (a2 holds
// bases 32..39); t <= 31, so the window is a funnel shift by 2t < 64 —
// one limb select for 2t >= 32, then two v_alignbit.
__device__ __forceinline__ uint64_t limb_kmer(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t t, const SkP& p) {
  const uint32_t sh = 2 * t;
  const bool up = sh >= 32;
  const uint32_t b0 = up ? a1 : a0, b1 = up ? a2 : a1, b2 = up ? 0u : a2;
  const uint32_t s5 = sh & 31;
  const uint32_t w0 = __builtin_amdgcn_alignbit(b1, b0, s5), w1 = __builtin_amdgcn_alignbit(b2, b1, s5);
  const uint64_t W = (uint64_t)w0 | ((uint64_t)w1 << 32);
  const uint64_t fw = sk_rev2(W) >> (64 - 2 * p.K);
  const uint64_t rc = ~W & p.hp.mask;
  return fw < rc ? fw : rc;
}
__device__ __forceinline__ uint64_t rec_kmer(const SK16& r, uint32_t t, const SkP& p) {
  return limb_kmer((uint32_t)(r.w0 >> 48) | ((uint32_t)r.w1 << 16), (uint32_t)(r.w1 >> 16), (uint32_t)(r.w1 >> 48), t, p);
}

// The K+1-mers of a K-record (the fused count, k_sk_bucket<.., UP>): slot
// t in [-1, n-1] is the K+1-mer starting at record base t (t = -1 takes the
// left flank, t = n-1 the right flank).  Every K+1-mer of a read lies on two
// consecutive K-mers, and the record that holds the first K-mer of its
// CANONICAL form counts it: that record's minimizer is the minimizer of that
// K-mer, a function of the canonical K+1-mer alone, so every instance lands
// in one bucket.  So the n-1 K+1-mers inside the record count here, the one
// over the left flank counts here iff its reverse complement is canonical (its
// canonical form starts with this record's first K-mer, reversed), the one
// over the right flank iff it is canonical as read.  An odd K+1 has no
// palindromes; for even K+1 a palindrome counts on its left K-mer.
// p: the K+1 parameters (p.K = K + 1, p.hp.mask its 2(K+1)-bit mask).
__device__ __forceinline__ uint64_t rec_kmer_up(const SK16& r, int t, const SkP& p, bool* own) {
  const uint32_t n = (uint32_t)(r.w0 >> 32) & 0xff, fl = (uint32_t)(r.w0 >> 40) & 0x3f;
  const uint32_t nb = n + (uint32_t)p.K - 2;  // record bases (K-mers of K = p.K - 1)
  uint32_t a0 = (uint32_t)(r.w0 >> 48) | ((uint32_t)r.w1 << 16);
  uint32_t a1 = (uint32_t)(r.w1 >> 16);
  uint32_t a2 = (uint32_t)(r.w1 >> 48);
  if (fl & 32) {  // right flank at base nb (<= 40: bits <= 81)
    const uint32_t rb = (fl >> 2) & 3, bit = 2 * nb;
    if (bit < 32)
      a0 |= rb << bit;
    else if (bit < 64)
      a1 |= rb << (bit - 32);
    else
      a2 |= rb << (bit - 64);
  }
  const uint32_t tt = t < 0 ? 0u : (uint32_t)t;
  const uint32_t sh = 2 * tt;
  const bool up = sh >= 32;
  const uint32_t b0 = up ? a1 : a0, b1 = up ? a2 : a1, b2 = up ? 0u : a2;
  const uint32_t s5 = sh & 31;
  uint64_t W = (uint64_t)__builtin_amdgcn_alignbit(b1, b0, s5) | ((uint64_t)__builtin_amdgcn_alignbit(b2, b1, s5) << 32);
  if (t < 0) W = (W << 2) | (fl & 3);  // the left flank first
  const uint64_t fw = sk_rev2(W) >> (64 - 2 * p.K);
  const uint64_t rc = ~W & p.hp.mask;
  if (t < 0)
    *own = (fl & 16) && rc < fw;
  else if ((uint32_t)t + 1 == n)
    *own = (fl & 32) && fw <= rc;
  else
    *own = true;
  return fw < rc ? fw : rc;
}

// The K+1-mer string of a record as the bucket kernel keeps it in LDS: the
// record's bases with the owned flanks attached — the left flank as base 0
// when the record owns that K+1-mer, the right flank after the last base —
// as three 32-bit limbs (<= 42 bases), so that owned slot f is the K+1-mer at
// string base f (limb_kmer) with no per-instance flank work.
__device__ __forceinline__ uint4 rec_up_string(const SK16& r, const SkP& p, bool ol, bool orr) {
  const uint32_t n = (uint32_t)(r.w0 >> 32) & 0xff, fl = (uint32_t)(r.w0 >> 40) & 0x3f;
  uint32_t a0 = (uint32_t)(r.w0 >> 48) | ((uint32_t)r.w1 << 16);
  uint32_t a1 = (uint32_t)(r.w1 >> 16);
  uint32_t a2 = (uint32_t)(r.w1 >> 48);
  if (orr) {
    const uint32_t rb = (fl >> 2) & 3, bit = 2 * (n + (uint32_t)p.K - 2);
    if (bit < 32)
      a0 |= rb << bit;
    else if (bit < 64)
      a1 |= rb << (bit - 32);
    else
      a2 |= rb << (bit - 64);
  }
  if (ol) {
    a2 = (a2 << 2) | (a1 >> 30);
    a1 = (a1 << 2) | (a0 >> 30);
    a0 = (a0 << 2) | (fl & 3);
  }
  return make_uint4(a0, a1, a2, 0u);
}

// Home of a canonical K-mer in a 2^bits table: the first slot of its aligned
// group of kSkGrp slots.  The probe order is linear from there (group by
// group), so a key sits before any empty slot of its probe sequence.
constexpr uint32_t kSkGrp = 4;
__device__ __forceinline__ uint32_t sk_slot(uint64_t c, int bits) {
  return (sk_fmix32((uint32_t)c ^ ((uint32_t)(c >> 32) * 0x9e3779b1u)) >> (32 - bits)) & ~(kSkGrp - 1);
}

// Find-or-claim the slot of key c in the LDS table: one 32-byte group read
// (two ds_read_b128) answers most instances — a hit, or the first empty slot
// to claim with one CAS.  Returns the slot, or kSkTab when the table is full.
template <uint32_t TAB = kSkTab>
__device__ __forceinline__ uint32_t sk_tab_claim(unsigned long long* tkey, uint64_t c, uint32_t g) {
  constexpr unsigned long long EMPTY = ~0ull;
  for (uint32_t n = 0; n < kSkProbeMax;) {
    const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(&tkey[g]);
    const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(&tkey[g + 2]);
    const unsigned long long k[kSkGrp] = {a.x, a.y, b.x, b.y};
    uint32_t j = kSkGrp;
#pragma unroll
    for (uint32_t q = kSkGrp; q-- > 0;)
      if (k[q] == c || k[q] == EMPTY) j = q;  // the first in probe order
    if (j == kSkGrp) {  // group full of other keys: the next group
      g = (g + kSkGrp) & (TAB - 1);
      n += kSkGrp;
      continue;
    }
    if (k[j] == c) return g + j;
    const unsigned long long old = atomicCAS(&tkey[g + j], EMPTY, (unsigned long long)c);
    if (old == EMPTY || old == c) return g + j;
    ++n;  // another key took that slot: look at the group again
  }
  return TAB;
}

struct SkOut {
  unsigned long long* ghist;  // spectrum
  uint64_t hist_len;
  unsigned long long* gstats;  // [0] distinct, [1] overflow buckets, [2] solid written, [3] scratch
  uint32_t* ovf_list;
  uint64_t* solid;             // solid mode output: khash of the canonical K-mer
  uint64_t solid_cap;
  uint32_t min_solid;
  unsigned long long* weak;    // SK24 solid mode: per-base bitmap of weak K-mer instances (or null)
  uint32_t* wrec;              // SK24 solid mode, instead of `weak`: mask of weak K-mers per record, at
                               // index record.pos (the multi-GPU owner side: pos = receive index)
  unsigned long long* prof;    // diagnostics (APG_SK_PROF): k_sk_bucket_dd's per-phase clock64 sums, or null
  uint32_t want_hist;          // k_sk_bucket_dd: bin the spectrum (a solid-set count may not need it)
  unsigned long long* inst;    // k_sk_bucket<.., UP>: K+1-mer instances counted (or null)
  uint32_t* sused;             // solid mode: entries written in each kSolidChunk-slot chunk of `solid`
  uint64_t n_sused;
  // with `weak`: record.pos is a receive index and the record's first base is
  // at wpos[record.pos] (the sharded count at world size 1, where the owner is
  // the reads' own rank: no mask return, no separate apply pass)
  const uint64_t* wpos = nullptr;
  // with `weak` AND `wrec` (P > 1, SkSelf): the records received from this
  // rank itself, receive indices [self_lo, self_lo + self_n), write their bits
  // into `weak` at wpos[self_send + (b - self_lo)]; the others their masks
  // into `wrec`, packed without that segment
  uint64_t self_lo = 0, self_n = 0, self_send = 0;
  uint32_t skip_heavy = 0;  // k_sk_bucket_dd: buckets over kSkHeavyRecords are counted elsewhere (not listed)
};

// A record's weak-K-mer mask m (bit t: K-mer t) at record position b: into the
// per-record mask array, or ORed into the per-base bitmap (one or two words).
__device__ __forceinline__ void sk_weak_write(const SkOut& o, uint64_t b, uint32_t m) {
  if (o.wrec) {
    if (!o.weak) {
      o.wrec[b] = m;
      return;
    }
    if (b - o.self_lo >= o.self_n) {  // another rank's record: its mask travels back
      o.wrec[b < o.self_lo ? b : b - o.self_n] = m;
      return;
    }
    b = o.self_send + (b - o.self_lo);  // a self-owned record: its send index
  }
  if (o.wpos) b = o.wpos[b];
  const uint32_t sh = (uint32_t)(b & 63);
  atomicOr(&o.weak[b >> 6], (unsigned long long)m << sh);
  if (sh && ((uint64_t)m >> (64 - sh))) atomicOr(&o.weak[(b >> 6) + 1], (unsigned long long)m >> (64 - sh));
}

// Solid-list reservations: a block takes whole chunks of kSolidChunk slots
// from gstats[2] and fills them bucket by bucket (a same-address atomic per
// bucket — a million of them per pass — serialised at the L2: a per-bucket
// counter add in k_sk_bucket_dd cost 4.3 ms); o.solid holds the chunks
// sparse, o.sused[c] how much of chunk c is used, and sk_solid_compact makes
// the list dense.  A bucket never has more than kSolidChunk solid K-mers (its
// LDS table has <= 2048 slots).
constexpr uint32_t kSolidChunk = 4096;
struct SolidRes {
  unsigned long long cs;  // current chunk's first slot (~0: none)
  uint32_t cu;            // slots of it used
};
__device__ __forceinline__ void solid_close(const SolidRes& r, const SkOut& o) {
  if (r.cs == ~0ull) return;
  const uint64_t c = r.cs / kSolidChunk;
  if (c < o.n_sused) o.sused[c] = r.cu;
}
// thread 0: first slot for n more solid K-mers of this block (n <= kSolidChunk)
__device__ __forceinline__ unsigned long long solid_take(SolidRes& r, uint32_t n, const SkOut& o) {
  if (n == 0) return 0;
  if (r.cs == ~0ull || r.cu + n > kSolidChunk) {
    solid_close(r, o);
    r.cs = atomicAdd(&o.gstats[2], (unsigned long long)kSolidChunk);
    r.cu = 0;
  }
  const unsigned long long b = r.cs + r.cu;
  r.cu += n;
  return b;
}

__device__ __forceinline__ void sk_spectrum_add(uint32_t c, uint32_t* lhist, const SkOut& o) {
  uint64_t m = c;
  if (m >= o.hist_len - 1) m = o.hist_len - 1;
  if (m < (uint64_t)kSkHistBins)
    atomicAdd(&lhist[m], 1u);
  else
    atomicAdd(&o.ghist[m], 1ull);
}

// One workgroup per bucket (grid-stride).  Records come in chunks of
// kSkThreads; a block scan of their K-mer counts and an LDS owner map
// flatten the chunk to one K-mer per thread, inserted into the LDS table
// keyed by the canonical K-mer (CAS, then count).  The occupied slots feed
// the spectrum; solid mode appends khash of those with count >= min_solid.
// blist (may be null): count only the buckets blist[0 .. *bcount) — the
// buckets k_sk_bucket_dd handed back.
// TAB: LDS table slots (buckets of ~2 TAB instances); OWN: owner-map bytes per
// record slot = the most K-mers a record holds (41 - K; 20 covers K >= 21).
// UP (R = SK24, not SOLID): count the K+1-mers of K-records (rec_kmer_up;
// p = the K+1 parameters): a record offers n + 1 slots, the ones it does not
// own are skipped.  With dcount (UP): bucket b's records are the solid-set
// count's distinct records (16-byte records at drec + boff[b], dcount[b] of
// them, the multiplicity in place of the partition key) unless dcount[b] ==
// ~0u (that bucket was not deduplicated: its records as partitioned,
// multiplicity 1).
template <bool SOLID, typename R, int NT, uint32_t TAB = kSkTab, int OWN = kSkBases, bool UP = false>
__global__ void __launch_bounds__(NT) k_sk_bucket(const R* __restrict__ rec,
                                                          const uint64_t* __restrict__ boff, uint64_t nbuckets, SkP p,
                                                          SkOut o, const uint32_t* __restrict__ blist = nullptr,
                                                          const unsigned long long* __restrict__ bcount = nullptr,
                                                          const SK16* __restrict__ drec = nullptr,
                                                          const uint32_t* __restrict__ dcount = nullptr) {
  constexpr bool WEAK = SOLID && RecPos<R>::value;
  static_assert(!UP || !SOLID, "the K+1 count is a spectrum count");
  unsigned long long n_up = 0;  // UP: owned K+1-mer instances inserted by this thread
  // recorded slots: kSkWaveSlots per wave (NT = 512: each wave sees ~1/8 of a bucket)
  constexpr uint32_t kWaveSlots = NT >= 512 ? 1024 : kSkWaveSlots;
  constexpr uint32_t kSlotCap = kWaveSlots * (NT / 64);
  __shared__ __attribute__((aligned(16))) unsigned long long tkey[TAB];
  __shared__ uint32_t tcnt[TAB];
  __shared__ uint32_t lhist[kSkHistBins];
  __shared__ __attribute__((aligned(16))) SK16 crec[NT];
  __shared__ uint32_t koff[NT];
  __shared__ __attribute__((aligned(16))) uint8_t owner[NT * OWN];
  static_assert(64 * OWN >= kWaveSlots / 8 + 8, "a wave's weak bit array must fit in its owner-map slice");
  __shared__ uint32_t scan_sm[32];
  __shared__ int ovf;
  __shared__ unsigned long long sbase;
  __shared__ SolidRes sres;
  // weak pass: table slot of each of the bucket's first kSlotCap K-mer
  // instances (in record order), recorded while counting — slots never move
  // once claimed, so the weak pass reads final counts without probing.  A
  // bucket with more instances takes the probing fallback, whose per-chunk
  // record positions and weak masks reuse the same LDS.
  __shared__ __attribute__((aligned(16))) uint16_t islot[WEAK ? kSlotCap : 4];
  static_assert(!WEAK || kSlotCap * 2 >= NT * 4, "fallback scratch must fit in islot");
  const uint32_t wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  uint8_t* wown = owner + wv * (64 * OWN);  // this wave's owner-map slice
  uint16_t* wslot = islot + (WEAK ? wv * kWaveSlots : 0);  // this wave's recorded slots
  uint32_t* wmask = reinterpret_cast<uint32_t*>(islot);  // [NT] (probing fallback)
  constexpr unsigned long long EMPTY = ~0ull;
  constexpr int TB = __builtin_ctz(TAB);
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < kSkHistBins; i += NT) lhist[i] = 0;
  if (tid == 0) sres = SolidRes{~0ull, 0};
  unsigned long long nd = 0;
  // The block's buckets bkt, bkt + grid, ... are one record stream: the next
  // chunk's record (this bucket's or the next bucket's first) and the next
  // bucket's bounds are loaded while the current chunk is counted.
  if (blist) nbuckets = *bcount;
  auto bid = [&](uint64_t q) -> uint64_t { return blist ? blist[q] : q; };
  // a bucket's record source: its own records, or (UP with dcount; src =
  // nullptr) its distinct ones, the multiplicity moved to .pos
  auto bounds = [&](uint64_t q, const R*& src_, uint64_t& off_, uint32_t& nr_) {
    const uint64_t b = bid(q);
    off_ = boff[b];
    uint32_t dc = ~0u;
    if constexpr (UP) {
      if (dcount) dc = dcount[b];
    }
    src_ = dc != ~0u ? nullptr : rec;
    nr_ = dc != ~0u ? dc : (uint32_t)(boff[b + 1] - off_);
  };
  auto ld = [&](const R* src_, uint64_t i) -> R {
    if constexpr (UP && RecPos<R>::value) {
      if (!src_) return rec_from_drec<R>(drec[i]);
    }
    return src_[i];
  };
  uint64_t bkt = blockIdx.x, off = 0;
  uint32_t nr = 0;
  const R* src = rec;
  if (bkt < nbuckets) bounds(bkt, src, off, nr);
  R pre{};
  if (tid < nr) pre = ld(src, off + tid);
  for (; bkt < nbuckets;) {
    const uint64_t nbk = bkt + gridDim.x;
    uint64_t noff = 0;
    uint32_t nnr = 0;
    const R* nsrc = rec;
    if (nbk < nbuckets) bounds(nbk, nsrc, noff, nnr);
    if (nr == 0 || nr > kSkHeavyRecords) {  // block-uniform
      if (nr && tid == 0) o.ovf_list[atomicAdd(&o.gstats[1], 1ull)] = (uint32_t)bid(bkt);
      if (tid < nnr) pre = ld(nsrc, noff + tid);
      bkt = nbk;
      off = noff;
      nr = nnr;
      src = nsrc;
      continue;
    }
    const bool mult = UP && !src;  // records carry their multiplicity (block-uniform)
    for (uint32_t s = tid; s < TAB; s += NT) {
      tkey[s] = EMPTY;
      tcnt[s] = 0;
    }
    if (tid == 0) ovf = 0;
    __syncthreads();
    // Each wave flattens and inserts its own 64 records of every chunk with a
    // wave scan and its own slice of the owner map: no block barriers until
    // the bucket's counts are final.
    uint32_t ibw = 0;  // this wave's K-mer instances before this chunk (wave-uniform)
    unsigned long long n_up_b = 0;  // UP: this bucket's owned instances (dropped if it overflows)
    for (uint32_t c0 = 0; c0 < nr; c0 += NT) {
      if (__builtin_amdgcn_readfirstlane(*(volatile int*)&ovf)) {  // the table filled: stop, load the next bucket
        if (tid < nnr) pre = ld(nsrc, noff + tid);
        break;
      }
      uint32_t nk = 0;
      if (c0 + tid < nr) {
        SK16 h = rec_head(pre, p);
        nk = (uint32_t)(h.w0 >> 32) & 0xff;
        if constexpr (UP) {  // the boundary K+1-mers this record owns, decided once per record
          bool ol, orr;
          (void)rec_kmer_up(h, -1, p, &ol);
          (void)rec_kmer_up(h, (int)nk - 1, p, &orr);
          nk = nk - 1 + (ol ? 1u : 0u) + (orr ? 1u : 0u);
          uint4 str = rec_up_string(h, p, ol, orr);  // slot f at string base f
          if constexpr (RecPos<R>::value) str.w = mult ? (uint32_t)rec_pos(pre, p) : 1u;
          *reinterpret_cast<uint4*>(&crec[tid]) = str;
        } else {
          crec[tid] = h;
        }
      }
      if (c0 + NT < nr) {
        if (c0 + NT + tid < nr) pre = ld(src, off + c0 + NT + tid);
      } else if (tid < nnr) {
        pre = ld(nsrc, noff + tid);
      }
      const uint32_t incl = wave_inclusive_scan<uint32_t>(nk);
      const uint32_t ex = incl - nk;
      const uint32_t tot = (uint32_t)__shfl((int)incl, 63, 64);
      koff[tid] = ex;
      for (uint32_t u = 0; u < nk; ++u) wown[ex + u] = (uint8_t)ln;
      wave_lds_sync();
      for (uint32_t f = ln; f < tot; f += 64) {
        const uint32_t i = (wv << 6) + wown[f];
        uint64_t c;
        uint32_t add = 1;
        if constexpr (UP) {  // every slot is owned (decided at the chunk load)
          const uint4 a = *reinterpret_cast<const uint4*>(&crec[i]);
          c = limb_kmer(a.x, a.y, a.z, f - koff[i], p);
          add = a.w;
          n_up_b += add;
        } else {
          c = rec_kmer(crec[i], f - koff[i], p);
        }
        const uint32_t s = sk_tab_claim<TAB>(tkey, c, sk_slot(c, TB));
        const bool ok = s < TAB;
        if (!ok) ovf = 1;  // table full: the bucket goes to the global path
        if (ok) {
          atomicAdd(&tcnt[s], add);
          if constexpr (WEAK) {
            if (ibw + f < kWaveSlots) wslot[ibw + f] = (uint16_t)s;
          }
        }
      }
      ibw += tot;
      wave_lds_sync();  // the next chunk overwrites this wave's crec / koff / owner slices
    }
    // counts final; a wave past its recorded-slot capacity sends the whole
    // bucket's weak pass to the probing fallback
    const bool unrecorded = __syncthreads_or(WEAK && ibw > kWaveSlots);
    if (UP && !ovf) n_up += n_up_b;
    if (ovf) {
      if (tid == 0) o.ovf_list[atomicAdd(&o.gstats[1], 1ull)] = (uint32_t)bid(bkt);
      __syncthreads();
      bkt = nbk;
      off = noff;
      nr = nnr;
      src = nsrc;
      continue;
    }
    if constexpr (WEAK) {
      // Weak pass: each K-mer instance finds its final count in the table,
      // weak ones (count < min_solid) set their bit at the instance's base
      // position — one 64-bit atomic OR (two when the run straddles a word)
      // per record holding a weak K-mer.
      if ((o.weak || o.wrec) && !unrecorded) {
        // (1) lane per K-mer instance of the wave: its recorded slot's final
        // count -> one weak bit; 64 bits land as one ballot word (instances
        // in record order, so a record's K-mers are consecutive bits).  The
        // wave's owner-map slice is free by now and holds the bit array.
        unsigned long long* wbits = reinterpret_cast<unsigned long long*>(wown);
        for (uint32_t f0 = 0; f0 < ibw; f0 += 64) {
          const uint32_t f = f0 + ln;
          const bool wk = f < ibw && tcnt[wslot[f]] < o.min_solid;
          const unsigned long long bal = __ballot(wk);
          if (ln == 0) wbits[f0 >> 6] = bal;
        }
        wave_lds_sync();
        // (2) thread per record (the same records the wave inserted): bits
        // [ex, ex + nk) of the wave's array are its mask; the records are
        // re-read from L2 for their positions
        uint32_t ib = 0;
        for (uint32_t c0 = 0; c0 < nr; c0 += NT) {
          uint32_t nk = 0;
          uint64_t b = 0;
          if (c0 + tid < nr) {
            const R r = rec[off + c0 + tid];
            nk = rec_nk(r);
            b = rec_pos(r, p);
          }
          const uint32_t incl = wave_inclusive_scan<uint32_t>(nk);
          const uint32_t ex = ib + incl - nk;
          const uint32_t tot = (uint32_t)__shfl((int)incl, 63, 64);
          uint32_t m = 0;
          if (nk) {
            const uint32_t w = ex >> 6, sh = ex & 63;
            unsigned long long x = wbits[w] >> sh;
            if (sh + nk > 64) x |= wbits[w + 1] << (64 - sh);
            m = (uint32_t)x & (nk >= 32 ? ~0u : ((1u << nk) - 1));
          }
          if (m) sk_weak_write(o, b, m);  // wrec is zeroed beforehand: only records with weak K-mers write
          ib += tot;
        }
        __syncthreads();
      } else if (o.weak || o.wrec) {
        // probing fallback (a wave outgrew its recorded slots), wave-local
        // like the insert loop: each instance looks its key up again
        for (uint32_t c0 = 0; c0 < nr; c0 += NT) {
          uint32_t nk = 0;
          uint64_t b = 0;
          if (c0 + tid < nr) {
            const R r = rec[off + c0 + tid];
            crec[tid] = rec_head(r, p);
            b = rec_pos(r, p);
            nk = rec_nk(r);
          }
          wmask[tid] = 0;
          const uint32_t incl = wave_inclusive_scan<uint32_t>(nk);
          const uint32_t ex = incl - nk;
          const uint32_t tot = (uint32_t)__shfl((int)incl, 63, 64);
          koff[tid] = ex;
          for (uint32_t u = 0; u < nk; ++u) wown[ex + u] = (uint8_t)ln;
          wave_lds_sync();
          for (uint32_t f = ln; f < tot; f += 64) {
            const uint32_t i = (wv << 6) + wown[f];
            const uint32_t t = f - koff[i];
            const uint64_t c = rec_kmer(crec[i], t, p);
            uint32_t s = sk_slot(c, TB);
            while (tkey[s] != c) s = (s + 1) & (TAB - 1);  // inserted above: present
            if (tcnt[s] < o.min_solid) atomicOr(&wmask[i], 1u << t);
          }
          wave_lds_sync();
          const uint32_t m = wmask[tid];
          if (c0 + tid < nr && m) sk_weak_write(o, b, m);
          wave_lds_sync();
        }
        __syncthreads();
      }
    }
    uint32_t ns = 0;
    for (uint32_t s = tid; s < TAB; s += NT)
      if (tkey[s] != EMPTY) {
        sk_spectrum_add(tcnt[s], lhist, o);
        ++nd;
        if (SOLID) ns += tcnt[s] >= o.min_solid;
      }
    if (SOLID) {
      uint32_t tot;
      uint32_t j = block_exclusive_scan<uint32_t>(ns, scan_sm, &tot);
      if (tid == 0) sbase = solid_take(sres, tot, o);
      __syncthreads();
      const unsigned long long b = sbase;
      for (uint32_t s = tid; s < TAB; s += NT)
        if (tkey[s] != EMPTY && tcnt[s] >= o.min_solid) {
          const unsigned long long at = b + j++;
          if (at < o.solid_cap) o.solid[at] = khash(p.hp, tkey[s]);
        }
    }
    __syncthreads();
    bkt = nbk;
    off = noff;
    nr = nnr;
    src = nsrc;
  }
  __syncthreads();
  const uint64_t lim = o.hist_len < (uint64_t)kSkHistBins ? o.hist_len : (uint64_t)kSkHistBins;
  for (uint32_t i = tid; i < lim; i += NT)
    if (lhist[i]) atomicAdd(&o.ghist[i], (unsigned long long)lhist[i]);
  wave_add(&o.gstats[0], nd);
  if constexpr (UP) wave_add(o.inst, n_up);
  if (SOLID && tid == 0) solid_close(sres, o);
}

// ---------------------------------------------------------------------------
// The K+1 count by an LDS counting sort (A/B of VERDICT r03 #3, APG_SK_UP_SORT=1)
// ---------------------------------------------------------------------------
// The alternative to the hash table that DESIGN.md §4 had only sized: per
// bucket, every owned K+1-mer instance (key, multiplicity) is flattened into
// LDS, counting-sorted on the top 12 bits of its khash (4096 bins: a
// histogram, a block scan, a scatter of the instance indices), and each bin
// is grouped by full-key equality by one thread (bins hold ~0.4 instances on
// average, so the grouping is a short scan) — equal keys always share a bin.
// Same outputs as k_sk_bucket<.., UP>: the spectrum, the distinct count, the
// instance count, and the buckets of more than kSortCap instances sent to the
// global table.
constexpr uint32_t kSortCap = 4096;
constexpr int kSortDigitBits = 12;
template <typename R>
__global__ void __launch_bounds__(256) k_sk_up_sort(const R* __restrict__ rec, const uint64_t* __restrict__ boff,
                                                    uint64_t nbuckets, SkP p, SkOut o,
                                                    const SK16* __restrict__ drec,
                                                    const uint32_t* __restrict__ dcount) {
  constexpr int NT = 256;
  constexpr uint32_t NB = 1u << kSortDigitBits;
  __shared__ unsigned long long key[kSortCap];
  __shared__ uint32_t wt[kSortCap];
  __shared__ uint16_t sidx[kSortCap];
  __shared__ uint32_t cnt[NB];
  __shared__ uint32_t lhist[kSkHistBins];
  __shared__ uint32_t scan_sm[32];
  __shared__ uint32_t ni_sh;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < kSkHistBins; i += NT) lhist[i] = 0;
  unsigned long long nd = 0, n_up = 0;
  const int dsh = 2 * p.K - kSortDigitBits;
  for (uint64_t bkt = blockIdx.x; bkt < nbuckets; bkt += gridDim.x) {
    const uint64_t off = boff[bkt];
    const uint32_t dc = dcount ? dcount[bkt] : ~0u;
    const bool mult = dc != ~0u;  // the solid-set count's distinct records, multiplicity in the key bits
    const uint32_t nr = mult ? dc : (uint32_t)(boff[bkt + 1] - off);
    if (tid == 0) ni_sh = 0;
    __syncthreads();
    // 1. flatten: each record's owned K+1-mers (as k_sk_bucket<.., UP>)
    for (uint32_t r = tid; r < nr; r += NT) {
      R x;
      if constexpr (RecPos<R>::value) {
        x = mult ? rec_from_drec<R>(drec[off + r]) : rec[off + r];
      } else {
        x = rec[off + r];
      }
      const SK16 h = rec_head(x, p);
      const uint32_t nk = (uint32_t)(h.w0 >> 32) & 0xff;
      bool ol, orr;
      (void)rec_kmer_up(h, -1, p, &ol);
      (void)rec_kmer_up(h, (int)nk - 1, p, &orr);
      const uint32_t no = nk - 1 + (ol ? 1u : 0u) + (orr ? 1u : 0u);
      const uint4 str = rec_up_string(h, p, ol, orr);
      const uint32_t w = mult ? (uint32_t)rec_pos(x, p) : 1u;
      const uint32_t at = atomicAdd(&ni_sh, no);
      for (uint32_t f = 0; f < no && at + f < kSortCap; ++f) {
        key[at + f] = limb_kmer(str.x, str.y, str.z, f, p);
        wt[at + f] = w;
      }
    }
    __syncthreads();
    const uint32_t ni = ni_sh;
    if (ni > kSortCap) {  // block-uniform: the global table counts this bucket
      if (tid == 0) o.ovf_list[atomicAdd(&o.gstats[1], 1ull)] = (uint32_t)bkt;
      __syncthreads();
      continue;
    }
    // 2. counting sort of the instance indices on 12 hash bits
    for (uint32_t b = tid; b < NB; b += NT) cnt[b] = 0;
    __syncthreads();
    for (uint32_t i = tid; i < ni; i += NT) atomicAdd(&cnt[(uint32_t)(khash(p.hp, key[i]) >> dsh)], 1u);
    __syncthreads();
    constexpr uint32_t PER = NB / NT;
    uint32_t loc[PER], tsum = 0;
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
      loc[q] = cnt[tid * PER + q];
      tsum += loc[q];
    }
    uint32_t tot;
    uint32_t run = block_exclusive_scan<uint32_t>(tsum, scan_sm, &tot);
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
      cnt[tid * PER + q] = run;
      run += loc[q];
    }
    __syncthreads();
    unsigned long long wsum = 0;
    for (uint32_t i = tid; i < ni; i += NT) {
      sidx[atomicAdd(&cnt[(uint32_t)(khash(p.hp, key[i]) >> dsh)], 1u)] = (uint16_t)i;
      wsum += wt[i];
    }
    n_up += wsum;
    __syncthreads();
    // 3. per bin: group equal keys (cnt[b] is now the bin's end)
    for (uint32_t b = tid; b < NB; b += NT) {
      const uint32_t e = cnt[b], s0 = b ? cnt[b - 1] : 0u;
      for (uint32_t j = s0; j < e; ++j) {
        const unsigned long long kj = key[sidx[j]];
        bool lead = true;
        for (uint32_t q = s0; q < j && lead; ++q) lead = key[sidx[q]] != kj;
        if (!lead) continue;
        uint32_t c = wt[sidx[j]];
        for (uint32_t q = j + 1; q < e; ++q)
          if (key[sidx[q]] == kj) c += wt[sidx[q]];
        sk_spectrum_add(c, lhist, o);
        ++nd;
      }
    }
    __syncthreads();
  }
  __syncthreads();
  const uint64_t lim = o.hist_len < (uint64_t)kSkHistBins ? o.hist_len : (uint64_t)kSkHistBins;
  for (uint32_t i = tid; i < lim; i += NT)
    if (lhist[i]) atomicAdd(&o.ghist[i], (unsigned long long)lhist[i]);
  wave_add(&o.gstats[0], nd);
  wave_add(o.inst, n_up);
}

// ---------------------------------------------------------------------------
// Record-deduplicating bucket count (K >= 21)
// ---------------------------------------------------------------------------
// At genome coverage c most super-k-mer records of a bucket are exact copies:
// interior super-k-mers are fixed by the genome (their ends are minimizer
// changes), so every read covering one error-free emits the same record.  On
// the bench's reads (62x) 36 % of the records are distinct and they carry
// 36.5 % of the K-mer instances.  A bucket (~kDdBucketKmers instances) is
// counted by one 256-thread block in two levels:
//   1. records -> LDS record table keyed by a 64-bit fingerprint of the
//      record's 96 significant bits (n, 40 bases), counting multiplicity; the
//      claiming lane stores the record, and after the chunk's barrier every
//      lane compares its record with the stored one (exact: a fingerprint
//      collision hands the bucket back);
//   2. one block scan over the record-table slots gives each distinct record
//      its first instance index; an LDS owner map (instance -> record slot)
//      spreads the distinct records' K-mer instances over all lanes, two per
//      lane per step, into the LDS K-mer table with count += multiplicity.
// Weak pass (solid mode, SK24): each distinct record's weak mask from the
// K-mer slots its instances recorded (in place of the owner map), then every
// record — its position and record slot kept in registers since phase 1 —
// ORs its mask into the bitmap (or stores it, multi-GPU): no record re-read.
// A bucket this kernel cannot finish in LDS — record table full, fingerprint
// collision, more than kDdRecCap records (weak mode), more than kDdInstCap
// distinct-record instances — is appended to `redo` for k_sk_bucket; a full
// K-mer table sends it to the global-table path as there.
// dout / dcount (SK24, the fused K+1 spectrum): records are folded with their
// flank bases (so a distinct record fixes its K+1-mers too), and each bucket's
// distinct records leave as 16-byte records, the multiplicity in place of
// the partition key, at dout[boff[b] .. + dcount[b]) once its record table is
// complete (dcount[b] = ~0u for a bucket whose record table could not be
// completed): the K+1 count then inserts each distinct record's K+1-mers
// once, with that multiplicity.
constexpr int kDdThreads = 512;
constexpr uint64_t kDdBucketKmers = 4096;  // instances per bucket the planner aims for with this kernel
constexpr uint32_t kDdKTab = 2048;         // K-mer table slots
// Table sizes keep the block at 51 KiB of LDS and <= 80 VGPRs, so three
// 512-thread blocks share a CU (at 1024 record slots and 4096 instances, 70 KiB
// held it to two: 25.5 -> 22.7 ms for the C2 solid count; ~220 distinct
// records per bucket there, the rest go back through `redo`)
constexpr uint32_t kDdTab = 512;           // record table slots
constexpr uint32_t kDdChunks = 4;          // weak mode: records per bucket <= kDdChunks * kDdThreads
constexpr uint32_t kDdRecCap = kDdChunks * kDdThreads;
constexpr uint32_t kDdInstCap = 3072;      // distinct-record K-mer instances per bucket
constexpr int kDdMinK = kSkBases + 1 - 20;  // records hold <= 20 K-mers (owner-map loop bound)

__device__ __forceinline__ uint64_t rec_fp(const SK16& h, uint64_t keep = ~kSkFlankMask) {
  const uint64_t x = sk_fmix(h.w1 ^ (((h.w0 & keep) >> 32) * 0x9e3779b97f4a7c15ull));
  return x == ~0ull ? 0ull : x;  // ~0 marks an empty slot
}

// Find-or-claim in a TS-slot LDS table (as sk_tab_claim); *fresh = this
// lane's CAS created the entry.  Returns TS when the table is full.
template <uint32_t TS>
__device__ __forceinline__ uint32_t lds_claim(unsigned long long* tk, uint64_t c, uint32_t g, bool* fresh) {
  constexpr unsigned long long EMPTY = ~0ull;
  *fresh = false;
  for (uint32_t n = 0; n < (TS < kSkProbeMax ? TS : kSkProbeMax);) {
    const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(&tk[g]);
    const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(&tk[g + 2]);
    const unsigned long long k[kSkGrp] = {a.x, a.y, b.x, b.y};
    uint32_t j = kSkGrp;
#pragma unroll
    for (uint32_t q = kSkGrp; q-- > 0;)
      if (k[q] == c || k[q] == EMPTY) j = q;
    if (j == kSkGrp) {
      g = (g + kSkGrp) & (TS - 1);
      n += kSkGrp;
      continue;
    }
    if (k[j] == c) return g + j;
    const unsigned long long old = atomicCAS(&tk[g + j], EMPTY, (unsigned long long)c);
    if (old == EMPTY) {
      *fresh = true;
      return g + j;
    }
    if (old == c) return g + j;
    ++n;
  }
  return TS;
}

template <bool SOLID, typename R>
__global__ void __launch_bounds__(kDdThreads) __attribute__((amdgpu_waves_per_eu(6))) k_sk_bucket_dd(const R* __restrict__ rec,
                                                             const uint64_t* __restrict__ boff, uint64_t nbuckets,
                                                             SkP p, SkOut o, uint32_t* __restrict__ redo,
                                                             SK16* __restrict__ dout = nullptr,
                                                             uint32_t* __restrict__ dcount = nullptr) {
  constexpr bool WEAK = SOLID && RecPos<R>::value;
  const uint64_t keep = dout ? ~0ull : ~kSkFlankMask;  // record identity: with the flanks for the K+1 count
  constexpr int NT = kDdThreads;
  constexpr unsigned long long EMPTY = ~0ull;
  constexpr int KB = __builtin_ctz(kDdKTab), RB = __builtin_ctz(kDdTab);
  __shared__ __attribute__((aligned(16))) unsigned long long tkey[kDdKTab];
  __shared__ uint32_t tcnt[kDdKTab];
  __shared__ uint16_t klist[kDdKTab];  // claimed K-mer slots (claim order)
  __shared__ __attribute__((aligned(16))) unsigned long long rkey[kDdTab];
  __shared__ uint32_t rcnt[kDdTab];  // multiplicity; weak mode: then the record's weak mask
  __shared__ __attribute__((aligned(16))) SK16 rrec[kDdTab];
  __shared__ uint16_t rlist[kDdTab];  // claimed record slots (claim order)
  __shared__ uint16_t doff[kDdTab];   // first instance of distinct record rlist[j], at j
  __shared__ uint16_t own[kDdInstCap];  // instance -> j; weak mode: then -> its K-mer slot; emit: solid slots
  __shared__ uint32_t lhist[kSkHistBins];
  __shared__ uint32_t scan_sm[32];
  __shared__ uint32_t nk_sh, nr_sh, ns_sh;  // claimed K-mer slots, claimed record slots, solid K-mers
  __shared__ int flag;  // 1: K-mer table full (global path); 2: hand the bucket back (redo)
  __shared__ unsigned long long sbase;
  __shared__ SolidRes sres;
  const uint32_t tid = threadIdx.x;
  const bool want_hist = o.want_hist != 0;
  for (uint32_t i = tid; i < kSkHistBins; i += NT) lhist[i] = 0;
  for (uint32_t s = tid; s < kDdKTab; s += NT) {  // afterwards each bucket clears the slots it claimed
    tkey[s] = EMPTY;
    tcnt[s] = 0;
  }
  for (uint32_t s = tid; s < kDdTab; s += NT) {
    rkey[s] = EMPTY;
    rcnt[s] = 0;
  }
  if (tid == 0) {
    nk_sh = nr_sh = ns_sh = 0;
    flag = 0;
    sres = SolidRes{~0ull, 0};
  }
  __syncthreads();
  unsigned long long nd = 0, n_dout = 0;  // n_dout: distinct records written (thread 0)
  // diagnostics: thread 0's clock64 between the phase barriers
  unsigned long long pt[6] = {0, 0, 0, 0, 0, 0}, t0 = 0;
  const bool prof = o.prof != nullptr && tid == 0;
  auto mark = [&](int ph) {
    if (prof) {
      const unsigned long long t1 = clock64();
      if (ph > 0) pt[ph - 1] += t1 - t0;
      t0 = t1;
    }
  };
  uint64_t bkt = blockIdx.x, off = 0;
  uint32_t nr = 0;
  if (bkt < nbuckets) {
    off = boff[bkt];
    nr = (uint32_t)(boff[bkt + 1] - off);
  }
  R pre{};
  if (tid < nr) pre = rec[off + tid];
  while (bkt < nbuckets) {
    mark(0);
    const uint64_t nbk = bkt + gridDim.x;
    uint64_t noff = 0;
    uint32_t nnr = 0;
    if (nbk < nbuckets) {
      noff = boff[nbk];
      nnr = (uint32_t)(boff[nbk + 1] - noff);
    }
    // ends a bucket: the claimed slots back to empty, counters reset
    auto finish = [&]() {
      const uint32_t nks = nk_sh, nrs = nr_sh;
      __syncthreads();  // every thread has read the counters (and flag)
      if (tid == 0) {
        nk_sh = nr_sh = ns_sh = 0;
        flag = 0;
      }
      for (uint32_t j = tid; j < nks; j += NT) {
        tkey[klist[j]] = EMPTY;
        tcnt[klist[j]] = 0;
      }
      for (uint32_t j = tid; j < nrs; j += NT) {
        rkey[rlist[j]] = EMPTY;
        rcnt[rlist[j]] = 0;
      }
      __syncthreads();
      bkt = nbk;
      off = noff;
      nr = nnr;
    };
    auto hand_back = [&](bool global_table) {
      if (tid == 0) {
        if (global_table)
          o.ovf_list[atomicAdd(&o.gstats[1], 1ull)] = (uint32_t)bkt;
        else
          redo[atomicAdd(&o.gstats[4], 1ull)] = (uint32_t)bkt;
      }
      finish();
    };
    if (nr == 0 || nr > kSkHeavyRecords || (WEAK && nr > kDdRecCap)) {  // block-uniform
      if (dout && tid == 0) dcount[bkt] = nr ? ~0u : 0u;
      if (nr && tid == 0) {
        if (nr > kSkHeavyRecords) {
          if (!o.skip_heavy) o.ovf_list[atomicAdd(&o.gstats[1], 1ull)] = (uint32_t)bkt;
        } else {
          redo[atomicAdd(&o.gstats[4], 1ull)] = (uint32_t)bkt;
        }
      }
      if (tid < nnr) pre = rec[noff + tid];
      bkt = nbk;
      off = noff;
      nr = nnr;
      continue;
    }
    // 1. records -> record table (multiplicity), verified against the
    // claimer's copy after each chunk's barrier.  Weak mode keeps each
    // record's slot and position in registers for the weak pass.
    uint64_t rp_[kDdChunks];  // record slot << 52 | position; slot kDdTab = no record
#pragma unroll
    for (uint32_t c = 0; c < kDdChunks; ++c) rp_[c] = (uint64_t)kDdTab << 52;
    for (uint32_t c = 0, c0 = 0; c0 < nr; ++c, c0 += NT) {
      const bool valid = c0 + tid < nr;
      SK16 hd{0, 0};
      uint64_t ps = 0;
      if (valid) {
        hd = rec_head(pre, p);
        if constexpr (WEAK) ps = rec_pos(pre, p);
      }
      if (c0 + NT < nr) {
        if (c0 + NT + tid < nr) pre = rec[off + c0 + NT + tid];
      } else if (tid < nnr) {
        pre = rec[noff + tid];
      }
      uint32_t s = kDdTab;
      bool fresh = false;
      if (valid) {
        const uint64_t fp = rec_fp(hd, keep);
        s = lds_claim<kDdTab>(rkey, fp, (uint32_t)(fp >> (64 - RB)) & ~(kSkGrp - 1), &fresh);
        if (s < kDdTab) {
          if (fresh) rrec[s] = hd;
          atomicAdd(&rcnt[s], 1u);
        } else {
          atomicOr(&flag, 2);
        }
      }
      if (fresh) rlist[atomicAdd(&nr_sh, 1u)] = (uint16_t)s;
      if constexpr (WEAK) {
#pragma unroll
        for (uint32_t q = 0; q < kDdChunks; ++q)
          if (q == c) rp_[q] = ((uint64_t)(valid ? s : kDdTab) << 52) | ps;
      }
      __syncthreads();
      if (s < kDdTab) {
        const SK16 q = rrec[s];
        if (((q.w0 ^ hd.w0) & keep) || q.w1 != hd.w1) atomicOr(&flag, 2);  // fingerprint collision
      }
    }
    __syncthreads();
    mark(1);
    if (flag) {  // block-uniform
      if (dout && tid == 0) dcount[bkt] = ~0u;
      hand_back(false);
      continue;
    }
    if constexpr (RecPos<R>::value) {
      if (dout) {  // the distinct records with their multiplicity, for the K+1 count
        const uint32_t nD = nr_sh;
        for (uint32_t j = tid; j < nD; j += NT) {
          const uint32_t s = rlist[j];
          const SK16 h = rrec[s];
          dout[off + j] = SK16{(h.w0 & ~0xffffffffull) | rcnt[s], h.w1};
        }
        if (tid == 0) {
          dcount[bkt] = nD;
          n_dout += nD;
        }
      }
    }
    // 2. distinct records' first instance indices (one block scan; <= NT
    // distinct records per thread round), owner map
    const uint32_t nD = nr_sh;
    uint32_t ni = 0;
    for (uint32_t j0 = 0; j0 < nD; j0 += NT) {  // block-uniform
      const uint32_t j = j0 + tid;
      const uint32_t nk = j < nD ? (uint32_t)(rrec[rlist[j]].w0 >> 32) & 0xff : 0;
      uint32_t tot;
      const uint32_t at = ni + block_exclusive_scan<uint32_t>(nk, scan_sm, &tot);
      if (j < nD) {
        doff[j] = (uint16_t)min(at, 0xffffu);
        if (at + nk <= kDdInstCap)
          for (uint32_t u = 0; u < nk; ++u) own[at + u] = (uint16_t)j;
      }
      ni += tot;
    }
    __syncthreads();
    mark(2);
    if (ni > kDdInstCap) {  // block-uniform
      hand_back(false);
      continue;
    }
    // 3. instances -> K-mer table (count += multiplicity), two per lane per step
    auto insert = [&](uint32_t f, bool ok) {
      bool fresh = false;
      uint32_t ts = kDdKTab;
      if (ok) {
        const uint32_t j = own[f];
        const uint32_t s = rlist[j];
        const uint64_t c = rec_kmer(rrec[s], f - doff[j], p);
        ts = lds_claim<kDdKTab>(tkey, c, sk_slot(c, KB), &fresh);
        if (ts < kDdKTab) {
          atomicAdd(&tcnt[ts], rcnt[s]);
          if constexpr (WEAK) own[f] = (uint16_t)ts;
        } else {
          atomicOr(&flag, 1);
        }
      }
      if (fresh) klist[atomicAdd(&nk_sh, 1u)] = (uint16_t)ts;
    };
    for (uint32_t f0 = 0; f0 < ni; f0 += 2 * NT) {
      if (__builtin_amdgcn_readfirstlane(*(volatile int*)&flag)) break;  // the table filled (no barrier inside)
      insert(f0 + tid, f0 + tid < ni);
      if (f0 + NT < ni) insert(f0 + NT + tid, f0 + NT + tid < ni);
    }
    __syncthreads();
    mark(3);
    if (flag) {  // block-uniform: only the K-mer table can have filled here
      hand_back(true);
      continue;
    }
    if constexpr (WEAK) {
      if (o.weak || o.wrec) {
        // (a) distinct record -> weak mask (replaces its multiplicity)
        for (uint32_t j = tid; j < nD; j += NT) {
          const uint32_t s = rlist[j];
          const uint32_t nk = (uint32_t)(rrec[s].w0 >> 32) & 0xff;
          const uint32_t b0 = doff[j];
          uint32_t m = 0;
          for (uint32_t t = 0; t < nk; ++t) m |= (uint32_t)(tcnt[own[b0 + t]] < o.min_solid) << t;
          rcnt[s] = m;
        }
        __syncthreads();
        // (b) each record (registers) -> its record's mask
#pragma unroll
        for (uint32_t c = 0; c < kDdChunks; ++c) {
          const uint32_t rs = (uint32_t)(rp_[c] >> 52);
          if (rs >= kDdTab) continue;
          const uint32_t m = rcnt[rs];
          if (!m) continue;
          sk_weak_write(o, rp_[c] & ((1ull << 52) - 1), m);
        }
      }
    }
    mark(4);
    // 4. the claimed K-mers: spectrum bins, solid slots (into `own`, free now)
    const uint32_t nK = nk_sh;
    nd += tid == 0 ? nK : 0;
    for (uint32_t j0 = 0; j0 < nK; j0 += NT) {  // block-uniform trip count
      const uint32_t j = j0 + tid;
      const uint32_t cn = j < nK ? tcnt[klist[j]] : 0;
      if (want_hist && j < nK) sk_spectrum_add(cn, lhist, o);
      if (SOLID && j < nK && cn >= o.min_solid) own[atomicAdd(&ns_sh, 1u)] = klist[j];
    }
    if (SOLID) {
      __syncthreads();
      const uint32_t ns = ns_sh;
      if (tid == 0) sbase = solid_take(sres, ns, o);
      __syncthreads();
      const unsigned long long b = sbase;
      for (uint32_t j = tid; j < ns; j += NT)
        if (b + j < o.solid_cap) o.solid[b + j] = khash(p.hp, tkey[own[j]]);
    }
    __syncthreads();
    mark(5);
    finish();
    mark(6);
  }
  if (prof)
    for (int i = 0; i < 6; ++i) atomicAdd(&o.prof[i], pt[i]);
  __syncthreads();
  const uint64_t lim = o.hist_len < (uint64_t)kSkHistBins ? o.hist_len : (uint64_t)kSkHistBins;
  for (uint32_t i = tid; i < lim; i += NT)
    if (lhist[i]) atomicAdd(&o.ghist[i], (unsigned long long)lhist[i]);
  wave_add(&o.gstats[0], nd);
  if (dout && tid == 0 && n_dout) atomicAdd(&o.gstats[5], n_dout);  // one same-address atomic per block, not per bucket
  if (SOLID && tid == 0) solid_close(sres, o);
}

// Overflowed buckets: every K-mer of every overflowed bucket into one global
// open-addressing table keyed by canonical K-mer (distinct buckets never
// share a K-mer).  Their records are processed as one flattened list (opre =
// exclusive prefix of the listed buckets' record counts), not a workgroup
// per bucket: the overflowing buckets of a repeat-rich genome are few and
// huge (one minimizer shared by thousands of copies), and a workgroup per
// bucket left one CU crunching the largest while the rest idled.
// The buckets over kSkHeavyRecords records (known from the bucket bounds
// before any counting): their overflow path can start beside the bucket pass.
__global__ void k_sk_heavy(const uint64_t* __restrict__ boff, uint64_t nb, uint32_t* __restrict__ list,
                           unsigned long long* __restrict__ n) {
  for (uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x; b0 < nb; b0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t b = b0 + threadIdx.x;
    const bool h = b < nb && boff[b + 1] - boff[b] > kSkHeavyRecords;
    const unsigned long long at = wave_append(n, h);
    if (h) list[at] = (uint32_t)b;
  }
}
__global__ void k_sk_ovf_sizes(const uint64_t* __restrict__ boff, const uint32_t* __restrict__ ovf, uint32_t n_ovf,
                               uint32_t* __restrict__ sz) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q < n_ovf) sz[q] = (uint32_t)(boff[ovf[q] + 1] - boff[ovf[q]]);
}

// index of the k-th record of the flattened overflow list, for k >= k0 where
// k0 is wave-uniform: the binary search runs on k0 (uniform loads, scalar
// when the compiler sees it), and each lane steps forward from there — the
// overflowed buckets hold thousands of records, so rarely more than once.  A
// per-lane search was a dozen dependent loads per record.
__device__ __forceinline__ uint64_t sk_ovf_record(const uint64_t* __restrict__ boff, const uint32_t* __restrict__ ovf,
                                                  const uint64_t* __restrict__ opre, uint32_t n_ovf, uint64_t k0,
                                                  uint64_t k) {
  uint32_t lo = 0, hi = n_ovf;  // last q with opre[q] <= k0
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (opre[mid] <= k0)
      lo = mid;
    else
      hi = mid;
  }
  while (lo + 1 < n_ovf && opre[lo + 1] <= k) ++lo;
  return boff[ovf[lo]] + (k - opre[lo]);
}

// UP: the K+1-mer slots of K-records (n + 1 each, an upper bound for sizing)
template <typename R, bool UP = false>
__global__ void k_sk_big_kmers(const R* __restrict__ rec, const uint64_t* __restrict__ boff,
                               const uint32_t* __restrict__ ovf, const uint64_t* __restrict__ opre, uint32_t n_ovf,
                               unsigned long long* __restrict__ n_kmers) {
  unsigned long long c = 0;
  const uint64_t tot = opre[n_ovf];
  for (uint64_t k0 = (uint64_t)blockIdx.x * blockDim.x; k0 < tot; k0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = k0 + threadIdx.x;
    if (k < tot) c += rec_nk(rec[sk_ovf_record(boff, ovf, opre, n_ovf, k0, k)]) + (UP ? 1u : 0u);
  }
  wave_add(n_kmers, c);
}

// The global table of the overflowed buckets: key and count side by side in
// one 16-byte slot, so a claim and its count add touch one line (separate key
// and count arrays made every insert and every weak-pass lookup two random
// lines).  It is sized for the distinct K-mers the instances suggest (a
// quarter of them, load <= 1/2 at 8 instances per distinct K-mer), not for
// every instance; a claim that probes kBigProbe slots without finding its key
// or an empty slot gives up and flags the table, and the host redoes the
// pass with the table sized for every instance.
struct BigSlot {
  unsigned long long key;  // ~0: empty
  unsigned long long cnt;
};
constexpr uint32_t kBigProbe = 1024;
struct BigTab {
  BigSlot* s;
  uint64_t mask;
  unsigned long long* full;  // set when a claim gave up
  // probes before a claim gives up: kBigProbe on the first, small table; no
  // limit on the full-size retry (more slots than instances: it cannot fill,
  // so a long linear-probe cluster of repetitive keys costs time, not the pass)
  uint32_t max_probe = kBigProbe;
};

__device__ __forceinline__ void sk_big_add(const BigTab& g, uint64_t c, uint64_t s, uint32_t add) {
  for (uint32_t n = 0; n < g.max_probe; ++n) {
    const unsigned long long old = atomicCAS(&g.s[s].key, ~0ull, (unsigned long long)c);
    if (old == ~0ull || old == c) {
      atomicAdd(&g.s[s].cnt, (unsigned long long)add);
      return;
    }
    s = (s + 1) & g.mask;
  }
  *g.full = 1;  // crowded: the pass is redone on a larger table
}

// Instances are first summed in a per-workgroup LDS table, flushed once per
// kBigFlush chunks of kBigChunk records: a K-mer repeated thousands of times
// (tandem arrays) costs one global atomic per flush, not one per instance.
// Flushing every 4 chunks took the repeats line's global pass 19.4 -> 36.4 ms:
// a chunk's K-mers are mostly distinct, so the fuller table sent more
// instances through 64 failed probes to the global fallback.
constexpr uint32_t kBigChunk = 256;
constexpr uint32_t kBigLds = 4096;
constexpr uint32_t kBigFlush = 1;
template <typename R, bool UP = false>
__global__ void __launch_bounds__(kBigChunk) k_sk_big_insert(const R* __restrict__ rec, const uint64_t* __restrict__ boff,
                                                             const uint32_t* __restrict__ ovf,
                                                             const uint64_t* __restrict__ opre, uint32_t n_ovf, SkP p,
                                                             BigTab g, unsigned long long* __restrict__ inst = nullptr) {
  unsigned long long n_up = 0;
  constexpr unsigned long long EMPTY = ~0ull;
  __shared__ unsigned long long lkey[kBigLds];
  __shared__ uint32_t lcnt[kBigLds];
  const uint32_t tid = threadIdx.x;
  for (uint32_t s = tid; s < kBigLds; s += kBigChunk) {
    lkey[s] = EMPTY;
    lcnt[s] = 0;
  }
  __syncthreads();
  const uint64_t tot = opre[n_ovf];
  uint32_t since = 0;  // chunks since the last flush
  for (uint64_t k0 = (uint64_t)blockIdx.x * kBigChunk; k0 < tot; k0 += (uint64_t)gridDim.x * kBigChunk) {
    const uint64_t k = k0 + tid;
    if (k < tot) {
      const SK16 r = rec_head(rec[sk_ovf_record(boff, ovf, opre, n_ovf, k0, k)], p);
      const uint32_t n = ((uint32_t)(r.w0 >> 32) & 0xff) + (UP ? 1u : 0u);
      for (uint32_t t = 0; t < n; ++t) {
        uint64_t c;
        if constexpr (UP) {
          bool own;
          c = rec_kmer_up(r, (int)t - 1, p, &own);
          if (!own) continue;
          ++n_up;
        } else {
          c = rec_kmer(r, t, p);
        }
        const uint64_t h = khash(p.hp, c);
        uint32_t s = (uint32_t)(h >> 40) & (kBigLds - 1);
        bool done = false;
        for (uint32_t pr = 0; pr < 64; ++pr, s = (s + 1) & (kBigLds - 1)) {
          unsigned long long v = lkey[s];
          if (v == EMPTY) v = atomicCAS(&lkey[s], EMPTY, (unsigned long long)c);
          if (v == EMPTY || v == c) {
            atomicAdd(&lcnt[s], 1u);
            done = true;
            break;
          }
        }
        if (!done) sk_big_add(g, c, h & g.mask, 1u);  // the chunk's LDS table is crowded
      }
    }
    __syncthreads();
    if (++since < kBigFlush && k0 + (uint64_t)gridDim.x * kBigChunk < tot) continue;  // block-uniform
    since = 0;
    for (uint32_t s = tid; s < kBigLds; s += kBigChunk) {
      const unsigned long long c = lkey[s];
      if (c != EMPTY) {
        sk_big_add(g, c, khash(p.hp, c) & g.mask, lcnt[s]);
        lkey[s] = EMPTY;
        lcnt[s] = 0;
      }
    }
    __syncthreads();
  }
  if constexpr (UP) wave_add(inst, n_up);
}

// Weak bits of the overflowed buckets' K-mer instances (counts from the
// global table built by k_sk_big_insert).
template <typename R>
__global__ void k_sk_big_weak(const R* __restrict__ rec, const uint64_t* __restrict__ boff,
                              const uint32_t* __restrict__ ovf, const uint64_t* __restrict__ opre, uint32_t n_ovf,
                              SkP p, BigTab g, uint32_t min_solid, SkOut o) {
  const uint64_t tot = opre[n_ovf];
  for (uint64_t k0 = (uint64_t)blockIdx.x * blockDim.x; k0 < tot; k0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = k0 + threadIdx.x;
    if (k >= tot) continue;
    const R r = rec[sk_ovf_record(boff, ovf, opre, n_ovf, k0, k)];
    const SK16 h = rec_head(r, p);
    const uint32_t n = rec_nk(r);
    uint32_t m = 0;
    for (uint32_t t = 0; t < n; ++t) {
      const uint64_t c = rec_kmer(h, t, p);
      uint64_t s = khash(p.hp, c) & g.mask;
      BigSlot x = g.s[s];
      while (x.key != c) {
        s = (s + 1) & g.mask;
        x = g.s[s];
      }
      if (x.cnt < min_solid) m |= 1u << t;
    }
    if (m) sk_weak_write(o, rec_pos(r, p), m);  // wrec is zeroed beforehand: only records with weak K-mers write
  }
}

// Solid K-mers leave through an LDS buffer: one global reservation per
// kEmitBuf of them (a same-address atomic per wave over half a billion slots
// serialised: 14.7 ms of the repeats line's solid pass).
constexpr uint32_t kEmitBuf = 2048;
template <bool SOLID>
__global__ void __launch_bounds__(256) k_sk_big_emit(const BigSlot* __restrict__ gs, uint64_t T, SkP p, SkOut o) {
  __shared__ uint32_t lhist[kSkHistBins];
  __shared__ unsigned long long sbuf[SOLID ? kEmitBuf : 1];
  __shared__ uint32_t scnt;
  __shared__ unsigned long long sbase;
  __shared__ SolidRes sres;
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < kSkHistBins; i += blockDim.x) lhist[i] = 0;
  if (tid == 0) {
    scnt = 0;
    sres = SolidRes{~0ull, 0};
  }
  __syncthreads();
  auto flush = [&]() {  // block-uniform
    const uint32_t n = scnt;
    if (tid == 0) sbase = solid_take(sres, n, o);
    __syncthreads();
    const unsigned long long b = sbase;
    for (uint32_t i = tid; i < n; i += blockDim.x)
      if (b + i < o.solid_cap) o.solid[b + i] = sbuf[i];
    __syncthreads();
    if (tid == 0) scnt = 0;
    __syncthreads();
  };
  unsigned long long nd = 0;
  for (uint64_t s0 = (uint64_t)blockIdx.x * blockDim.x; s0 < T; s0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t s = s0 + tid;  // block-uniform trip count (the flushes below have barriers)
    const BigSlot x = s < T ? gs[s] : BigSlot{~0ull, 0};
    if (x.key != ~0ull) {
      const uint32_t c = (uint32_t)x.cnt;
      sk_spectrum_add(c, lhist, o);
      ++nd;
      if (SOLID && c >= o.min_solid) sbuf[atomicAdd(&scnt, 1u)] = khash(p.hp, x.key);
    }
    if constexpr (SOLID) {
      __syncthreads();
      if (scnt > kEmitBuf - blockDim.x) flush();
    }
  }
  if constexpr (SOLID) {
    __syncthreads();
    flush();
    if (tid == 0) solid_close(sres, o);
  }
  __syncthreads();
  const uint64_t lim = o.hist_len < (uint64_t)kSkHistBins ? o.hist_len : (uint64_t)kSkHistBins;
  for (uint32_t i = tid; i < lim; i += blockDim.x)
    if (lhist[i]) atomicAdd(&o.ghist[i], (unsigned long long)lhist[i]);
  wave_add(&o.gstats[0], nd);
}

// ---------------------------------------------------------------------------
// Overflowed buckets by sub-bucket counting (default; APG_SK_OVF=global: the
// global-table path above).  Distinct overflowed buckets never share a K-mer
// (their minimizers differ), and inside one the K-mers split by a hash of the
// canonical K-mer, so each (bucket, hash digit) sub-bucket counts alone in an
// LDS table: every K-mer instance of the overflowed buckets leaves as a
// 16-byte entry (k_ovf_expand), one partition level groups each bucket's
// entries by the top 8 bits of the hash, and a workgroup per sub-bucket
// counts it, re-reads it for the weak bits and emits the spectrum bins and
// solid K-mers.  A sub-bucket whose distinct K-mers fill the LDS table (the
// one K-mer of a tandem array seen 10^5 times is one slot; what fills it is
// ~2000 different K-mers of one minimizer and hash digit) goes through a
// global table, listed in `bad`.  The repeat-rich genome's 3.2 K overflowed
// buckets (162 M instances) took 17.6 ms in the global table per pass.
//   entry: w1 = the canonical K-mer; w0 = record position bits 0..23 | hash
//   digit << 24 | position bits 24..33 << 32 | K-mer index in the record << 48
__device__ __forceinline__ uint32_t ovf_digit(uint64_t c) {
  return sk_fmix32((uint32_t)c ^ ((uint32_t)(c >> 32) * 0x85ebca6bu) ^ 0x5bd1e995u) >> 24;
}
__device__ __forceinline__ uint64_t ovf_w0(uint64_t rpos, uint32_t t, uint32_t dig) {
  return (rpos & 0xffffffull) | ((uint64_t)dig << 24) | ((rpos >> 24) << 32) | ((uint64_t)t << 48);
}
__device__ __forceinline__ uint64_t ovf_pos(uint64_t w0) { return (w0 & 0xffffffull) | (((w0 >> 32) & 0xffffull) << 24); }
__device__ __forceinline__ uint32_t ovf_t(uint64_t w0) { return (uint32_t)(w0 >> 48) & 63; }

// the weak bit of one instance: ORed (several sub-buckets may write one
// record's mask)
__device__ __forceinline__ void sk_weak_or(const SkOut& o, uint64_t b, uint32_t t) {
  if (o.wrec) {
    if (!o.weak) {
      atomicOr(&o.wrec[b], 1u << t);
      return;
    }
    if (b - o.self_lo >= o.self_n) {
      atomicOr(&o.wrec[b < o.self_lo ? b : b - o.self_n], 1u << t);
      return;
    }
    b = o.self_send + (b - o.self_lo);
  }
  if (o.wpos) b = o.wpos[b];
  b += t;
  atomicOr(&o.weak[b >> 6], 1ull << (b & 63));
}

// UP (the K+1 pass; p = the K+1 parameters): a record's owned K+1-mers
// (rec_kmer_up over its n + 1 slots) instead of its K-mers.
template <typename R, bool UP>
__device__ __forceinline__ uint32_t ovf_rec_n(const R& x, const SkP& p) {
  if constexpr (!UP) {
    return rec_nk(x);
  } else {
    const SK16 r = rec_head(x, p);
    const uint32_t n = ((uint32_t)(r.w0 >> 32) & 0xff) + 1u;
    uint32_t c = 0;
    for (uint32_t t = 0; t < n; ++t) {
      bool own;
      rec_kmer_up(r, (int)t - 1, p, &own);
      c += own;
    }
    return c;
  }
}
template <typename R, bool UP>
__global__ void k_ovf_nk(const R* __restrict__ rec, const uint64_t* __restrict__ boff, const uint32_t* __restrict__ ovf,
                         const uint64_t* __restrict__ opre, uint32_t n_ovf, SkP p, uint32_t* __restrict__ nk) {
  const uint64_t tot = opre[n_ovf];
  for (uint64_t k0 = (uint64_t)blockIdx.x * blockDim.x; k0 < tot; k0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = k0 + threadIdx.x;
    if (k < tot) nk[k] = ovf_rec_n<R, UP>(rec[sk_ovf_record(boff, ovf, opre, n_ovf, k0, k)], p);
  }
}
// each overflowed bucket's first entry: ipre at its first flattened record
__global__ void k_ovf_starts(const uint64_t* __restrict__ opre, const uint64_t* __restrict__ ipre, uint32_t n_ovf,
                             uint64_t* __restrict__ out) {
  const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q <= n_ovf) out[q] = ipre[opre[q]];
}
template <typename R, bool UP>
__global__ void k_ovf_expand(const R* __restrict__ rec, const uint64_t* __restrict__ boff,
                             const uint32_t* __restrict__ ovf, const uint64_t* __restrict__ opre, uint32_t n_ovf,
                             const uint64_t* __restrict__ ipre, SkP p, SK16* __restrict__ out) {
  const uint64_t tot = opre[n_ovf];
  for (uint64_t k0 = (uint64_t)blockIdx.x * blockDim.x; k0 < tot; k0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = k0 + threadIdx.x;
    if (k >= tot) continue;
    const R r = rec[sk_ovf_record(boff, ovf, opre, n_ovf, k0, k)];
    const SK16 h = rec_head(r, p);
    const uint64_t at = ipre[k];
    if constexpr (UP) {  // owned K+1-mers only; no weak bits, so no position
      const uint32_t n = ((uint32_t)(h.w0 >> 32) & 0xff) + 1u;
      uint32_t j = 0;
      for (uint32_t t = 0; t < n; ++t) {
        bool own;
        const uint64_t c = rec_kmer_up(h, (int)t - 1, p, &own);
        if (own) out[at + j++] = SK16{ovf_w0(0, 0, ovf_digit(c)), c};
      }
    } else {
      const uint32_t n = rec_nk(r);
      const uint64_t pos = RecPos<R>::value ? rec_pos(r, p) : 0;
      for (uint32_t t = 0; t < n; ++t) {
        const uint64_t c = rec_kmer(h, t, p);
        out[at + t] = SK16{ovf_w0(pos, t, ovf_digit(c)), c};
      }
    }
  }
}

// the slot of a key the table holds (probe without claiming)
template <uint32_t TS>
__device__ __forceinline__ uint32_t lds_find(const unsigned long long* tk, uint64_t c, uint32_t g) {
  for (uint32_t n = 0; n < TS; n += kSkGrp) {
    const ulonglong2 a = *reinterpret_cast<const ulonglong2*>(&tk[g]);
    const ulonglong2 b = *reinterpret_cast<const ulonglong2*>(&tk[g + 2]);
    if (a.x == c) return g;
    if (a.y == c) return g + 1;
    if (b.x == c) return g + 2;
    if (b.y == c) return g + 3;
    g = (g + kSkGrp) & (TS - 1);
  }
  return TS;
}

// One workgroup per sub-bucket (grid-stride over the n_sb = n_ovf x 256
// children of the partition level, child[] their entry offsets).  A
// sub-bucket holds ~200 entries, so its chain of dependent global loads
// (bounds, entries, the entries again for the weak bits) was what the
// kernel waited on: the next sub-bucket's bounds and first entries are
// loaded while the current one counts, and a thread keeps its first-chunk
// entry in registers for the weak pass.
constexpr uint32_t kOvfTab = 2048;
constexpr int kOvfThreads = 256;
template <bool SOLID>
__global__ void __launch_bounds__(kOvfThreads) k_ovf_count(const SK16* __restrict__ e, const uint64_t* __restrict__ child,
                                                           uint64_t n_sb, SkP p, SkOut o, uint32_t* __restrict__ bad,
                                                           unsigned long long* __restrict__ n_bad, bool force_bad) {
  constexpr unsigned long long EMPTY = ~0ull;
  constexpr int KB = __builtin_ctz(kOvfTab);
  __shared__ __attribute__((aligned(16))) unsigned long long tk[kOvfTab];
  __shared__ uint32_t tc[kOvfTab];
  __shared__ uint16_t klist[kOvfTab];
  __shared__ uint16_t slist[kOvfTab];
  __shared__ uint32_t lhist[kSkHistBins];
  __shared__ uint32_t nk_sh, ns_sh;
  __shared__ int flag;
  __shared__ unsigned long long sbase;
  __shared__ SolidRes sres;
  const uint32_t tid = threadIdx.x;
  const bool want_hist = o.want_hist != 0;
  const bool want_weak = SOLID && (o.weak || o.wrec);
  for (uint32_t i = tid; i < kSkHistBins; i += kOvfThreads) lhist[i] = 0;
  for (uint32_t s = tid; s < kOvfTab; s += kOvfThreads) {
    tk[s] = EMPTY;
    tc[s] = 0;
  }
  if (tid == 0) {
    nk_sh = ns_sh = 0;
    flag = 0;
    sres = SolidRes{~0ull, 0};
  }
  unsigned long long nd = 0;
  uint64_t sb = blockIdx.x, a = 0, b = 0;
  if (sb < n_sb) {
    a = child[sb];
    b = child[sb + 1];
  }
  SK16 x0{0, EMPTY};  // this thread's entry of the sub-bucket's first chunk
  if (a + tid < b) x0 = e[a + tid];
  __syncthreads();
  while (sb < n_sb) {  // block-uniform
    const uint64_t nsb = sb + gridDim.x;
    uint64_t na = 0, nb = 0;
    if (nsb < n_sb) {  // in flight while this sub-bucket counts
      na = child[nsb];
      nb = child[nsb + 1];
    }
    const bool any = a != b;
    bool full = false;
    if (any) {
      // 1. count
      for (uint64_t i0 = a; i0 < b; i0 += kOvfThreads) {
        if (__builtin_amdgcn_readfirstlane(*(volatile int*)&flag)) break;
        const uint64_t i = i0 + tid;
        bool fresh = false;
        uint32_t sl = kOvfTab;
        if (i < b) {
          const uint64_t c = i0 == a ? x0.w1 : e[i].w1;
          sl = lds_claim<kOvfTab>(tk, c, sk_slot(c, KB), &fresh);
          if (sl < kOvfTab)
            atomicAdd(&tc[sl], 1u);
          else
            atomicOr(&flag, 1);
        }
        if (fresh) klist[atomicAdd(&nk_sh, 1u)] = (uint16_t)sl;
      }
      __syncthreads();
      full = flag != 0 || force_bad;  // force_bad: tests of the global fallback
      // 2. the weak bits, instance by instance (the first chunk from registers)
      if (!full && want_weak) {
        for (uint64_t i = a + tid; i < b; i += kOvfThreads) {
          const SK16 x = i < a + kOvfThreads ? x0 : e[i];
          const uint32_t sl = lds_find<kOvfTab>(tk, x.w1, sk_slot(x.w1, KB));
          if (tc[sl] < o.min_solid) sk_weak_or(o, ovf_pos(x.w0), ovf_t(x.w0));
        }
      }
    }
    // the next sub-bucket's first chunk: in flight during the emission
    x0 = SK16{0, EMPTY};
    if (na + tid < nb) x0 = e[na + tid];
    if (any) {
      if (!full) {
        // 3. spectrum bins, solid K-mers
        const uint32_t nK = nk_sh;
        nd += tid == 0 ? nK : 0;
        for (uint32_t j = tid; j < nK; j += kOvfThreads) {
          const uint32_t cn = tc[klist[j]];
          if (want_hist) sk_spectrum_add(cn, lhist, o);
          if (SOLID && cn >= o.min_solid) slist[atomicAdd(&ns_sh, 1u)] = klist[j];
        }
        if (SOLID) {
          __syncthreads();
          const uint32_t ns = ns_sh;
          if (tid == 0) sbase = solid_take(sres, ns, o);
          __syncthreads();
          const unsigned long long sbs = sbase;
          for (uint32_t j = tid; j < ns; j += kOvfThreads)
            if (sbs + j < o.solid_cap) o.solid[sbs + j] = khash(p.hp, tk[slist[j]]);
        }
      } else if (tid == 0) {
        bad[atomicAdd(n_bad, 1ull)] = (uint32_t)sb;  // a global table counts it
      }
      // clear the claimed slots
      __syncthreads();
      const uint32_t nks = nk_sh;
      for (uint32_t j = tid; j < nks; j += kOvfThreads) {
        tk[klist[j]] = EMPTY;
        tc[klist[j]] = 0;
      }
      __syncthreads();
      if (tid == 0) {
        nk_sh = ns_sh = 0;
        flag = 0;
      }
      __syncthreads();
    }
    sb = nsb;
    a = na;
    b = nb;
  }
  const uint64_t lim = o.hist_len < (uint64_t)kSkHistBins ? o.hist_len : (uint64_t)kSkHistBins;
  for (uint32_t i = tid; i < lim; i += kOvfThreads)
    if (lhist[i]) atomicAdd(&o.ghist[i], (unsigned long long)lhist[i]);
  wave_add(&o.gstats[0], nd);
  if (SOLID && tid == 0) solid_close(sres, o);
}

// the sub-buckets the LDS table could not hold: their entries into a global
// table (as k_sk_big_insert, one entry per instance), then their weak bits
__global__ void k_ovf_big_insert(const SK16* __restrict__ e, const uint64_t* __restrict__ child,
                                 const uint32_t* __restrict__ bad, uint32_t n_bad, SkP p, BigTab g) {
  for (uint32_t q = blockIdx.x; q < n_bad; q += gridDim.x) {
    const uint64_t a = child[bad[q]], b = child[bad[q] + 1];
    for (uint64_t i = a + threadIdx.x; i < b; i += blockDim.x) {
      const uint64_t c = e[i].w1;
      sk_big_add(g, c, khash(p.hp, c) & g.mask, 1u);
    }
  }
}
__global__ void k_ovf_big_weak(const SK16* __restrict__ e, const uint64_t* __restrict__ child,
                               const uint32_t* __restrict__ bad, uint32_t n_bad, SkP p, BigTab g, SkOut o) {
  for (uint32_t q = blockIdx.x; q < n_bad; q += gridDim.x) {
    const uint64_t a = child[bad[q]], b = child[bad[q] + 1];
    for (uint64_t i = a + threadIdx.x; i < b; i += blockDim.x) {
      const SK16 x = e[i];
      uint64_t s = khash(p.hp, x.w1) & g.mask;
      BigSlot y = g.s[s];
      while (y.key != x.w1) {
        s = (s + 1) & g.mask;
        y = g.s[s];
      }
      if (y.cnt < o.min_solid) sk_weak_or(o, ovf_pos(x.w0), ovf_t(x.w0));
    }
  }
}

// The solid list dense again: chunk c's used[c] entries to offs[c].
__global__ void k_solid_compact(const uint64_t* __restrict__ sparse, const uint32_t* __restrict__ used,
                                const uint64_t* __restrict__ offs, uint64_t n_chunks, uint64_t* __restrict__ out) {
  for (uint64_t c = blockIdx.x; c < n_chunks; c += gridDim.x) {
    const uint32_t u = used[c];
    const uint64_t o = offs[c];
    for (uint32_t i = threadIdx.x; i < u; i += blockDim.x) out[o + i] = sparse[c * kSolidChunk + i];
  }
}

__global__ void k_big_init(BigSlot* __restrict__ g, uint64_t T) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < T; i += (uint64_t)gridDim.x * blockDim.x)
    g[i] = BigSlot{~0ull, 0ull};
}
__global__ void k_add_u64(unsigned long long* __restrict__ dst, const unsigned long long* __restrict__ src) {
  atomicAdd(dst, *src);
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------

// The overflowed buckets' K-mers (or owned K+1-mers, UP) counted into the
// global table: first on a table for nbk / 8 distinct K-mers at load <= 1/2,
// redone on one for every instance if a claim gave up.  inst (UP): the owned
// instances counted, added once the pass stands.
template <typename RB, bool UP>
static int big_count(apg_ctx* ctx, const RB* cur, const uint64_t* boff, const uint32_t* ovf, const uint64_t* opre,
                     uint32_t n_ovf, const SkP& p, uint64_t nbk, uint32_t g2, unsigned long long* inst, BigTab* out,
                     uint64_t* T_out) {
  unsigned long long *full = nullptr, *binst = nullptr;
  APG_TRY(workspace_t(ctx, "sk_gfull", 2, &full));
  binst = full + 1;
  for (int attempt = 0; attempt < 2; ++attempt) {
    uint64_t T = 1024;
    const uint64_t want = attempt ? 2 * nbk : nbk / 4;
    while (T < want) T <<= 1;
    BigSlot* gs = nullptr;
    APG_TRY(workspace_t(ctx, "sk_gtab", T, &gs));
    k_big_init<<<grid_for(ctx, T), 256, 0, ctx->stream>>>(gs, T);
    APG_CHECK_HIP(hipMemsetAsync(full, 0, 16, ctx->stream));
    const BigTab g{gs, T - 1, full, attempt ? ~0u : (getenv("APG_SK_BIG_PROBE") ? (uint32_t)atoi(getenv("APG_SK_BIG_PROBE")) : kBigProbe)};
    k_sk_big_insert<RB, UP><<<g2, kBigChunk, 0, ctx->stream>>>(cur, boff, ovf, opre, n_ovf, p, g, UP ? binst : nullptr);
    APG_CHECK_HIP(hipGetLastError());
    unsigned long long hf = 0;
    APG_TRY(d2h_sync(ctx, &hf, full, 8));
    if (!hf) {
      if (UP && inst) k_add_u64<<<1, 1, 0, ctx->stream>>>(inst, binst);
      *out = g;
      *T_out = T;
      return APG_OK;
    }
    vlog(ctx, "sk count: the overflow table of %llu slots is crowded (%llu instances): redone at full size",
         (unsigned long long)T, (unsigned long long)nbk);
  }
  set_error("sk count: overflow table full at one slot per two instances (internal error)");
  return APG_E_STATE;
}
// The overflowed buckets by sub-bucket counting (k_ovf_*): entries out, one
// partition level by hash digit within each bucket, an LDS count per
// sub-bucket; the ones that fill the LDS table through a global table.
// UP: the K+1 pass's overflowed buckets (owned K+1-mers; nbk an upper bound
// of them); *n_inst (may be null) receives the instances counted.
template <typename RB, bool UP = false>
static int ovf_lds_count(apg_ctx* ctx, const RB* cur, const uint64_t* boff, const uint32_t* ovf, const uint64_t* opre,
                         uint32_t n_ovf, const SkP& p, uint64_t nbk, bool solid, const SkOut& o, uint32_t g2,
                         uint64_t* n_inst = nullptr) {
  uint64_t tot = 0;  // flattened records
  APG_TRY(d2h_sync(ctx, &tot, opre + n_ovf, 8));
  uint32_t* nk = nullptr;
  uint64_t *ipre = nullptr, *qs = nullptr, *child = nullptr;
  APG_TRY(workspace_t(ctx, "sk_ovf_nk", std::max<uint64_t>(tot, 1), &nk));
  APG_TRY(workspace_t(ctx, "sk_ovf_ipre", tot + 1, &ipre));
  APG_TRY(workspace_t(ctx, "sk_ovf_qs", (uint64_t)n_ovf + 1, &qs));
  k_ovf_nk<RB, UP><<<g2, 256, 0, ctx->stream>>>(cur, boff, ovf, opre, n_ovf, p, nk);
  APG_CHECK_HIP(hipGetLastError());
  APG_TRY(scan_u32_u64(ctx, nk, tot, ipre, "skoi"));
  k_ovf_starts<<<(n_ovf + 256) / 256, 256, 0, ctx->stream>>>(opre, ipre, n_ovf, qs);
  std::vector<uint64_t> hq((size_t)n_ovf + 1);
  APG_TRY(d2h_sync(ctx, hq.data(), qs, ((size_t)n_ovf + 1) * 8));
  if (UP ? hq[n_ovf] > nbk : hq[n_ovf] != nbk) {
    set_error("sk count: overflowed buckets' instances disagree (internal error)");
    return APG_E_STATE;
  }
  nbk = hq[n_ovf];
  if (n_inst) *n_inst = nbk;
  SK16 *e0 = nullptr, *e1 = nullptr;
  APG_TRY(workspace_t(ctx, "sk_ovf_e0", std::max<uint64_t>(nbk, 1), &e0));
  APG_TRY(workspace_t(ctx, "sk_ovf_e1", std::max<uint64_t>(nbk, 1), &e1));
  k_ovf_expand<RB, UP><<<g2, 256, 0, ctx->stream>>>(cur, boff, ovf, opre, n_ovf, ipre, p, e0);
  APG_CHECK_HIP(hipGetLastError());
  std::vector<std::vector<Seg>> parents(n_ovf);
  for (uint32_t q = 0; q < n_ovf; ++q) parents[q].push_back(Seg{hq[q], hq[q + 1] - hq[q]});
  constexpr int kOvfBits = 8;
  const uint64_t n_sb = (uint64_t)n_ovf << kOvfBits;
  APG_TRY(workspace_t(ctx, "sk_ovf_child", n_sb + 1, &child));
  APG_TRY(part_level<SK16>(ctx, e0, e1, parents, 64 - kOvfBits, kOvfBits, nbk, child, nullptr, "ovf"));
  uint32_t* bad = nullptr;
  unsigned long long* nbad = nullptr;
  APG_TRY(workspace_t(ctx, "sk_ovf_bad", n_sb, &bad));
  APG_TRY(workspace_t(ctx, "sk_ovf_nbad", 1, &nbad));
  APG_CHECK_HIP(hipMemsetAsync(nbad, 0, 8, ctx->stream));
  const uint64_t grid = solid ? resident_grid(ctx, k_ovf_count<true>, kOvfThreads, n_sb)
                              : resident_grid(ctx, k_ovf_count<false>, kOvfThreads, n_sb);
  // APG_SK_OVF=bad (tests): every sub-bucket through the global fallback
  const bool force_bad = getenv("APG_SK_OVF") && !strcmp(getenv("APG_SK_OVF"), "bad");
  if (solid)
    k_ovf_count<true><<<grid, kOvfThreads, 0, ctx->stream>>>(e1, child, n_sb, p, o, bad, nbad, force_bad);
  else
    k_ovf_count<false><<<grid, kOvfThreads, 0, ctx->stream>>>(e1, child, n_sb, p, o, bad, nbad, force_bad);
  APG_CHECK_HIP(hipGetLastError());
  unsigned long long hb = 0;
  APG_TRY(d2h_sync(ctx, &hb, nbad, 8));
  if (hb) {  // sub-buckets past the LDS table: a global table over their entries
    std::vector<uint32_t> hbad(hb);
    std::vector<uint64_t> hc(n_sb + 1);
    APG_CHECK_HIP(hipMemcpyAsync(hbad.data(), bad, hb * 4, hipMemcpyDeviceToHost, ctx->stream));
    APG_TRY(d2h_sync(ctx, hc.data(), child, (n_sb + 1) * 8));
    uint64_t inst = 0;
    for (uint32_t sb : hbad) inst += hc[sb + 1] - hc[sb];
    uint64_t T = 1024;
    while (T < 2 * inst) T <<= 1;  // more slots than instances: a claim always ends
    BigSlot* gs = nullptr;
    unsigned long long* full = nullptr;
    APG_TRY(workspace_t(ctx, "sk_gtab", T, &gs));
    APG_TRY(workspace_t(ctx, "sk_gfull", 2, &full));
    k_big_init<<<grid_for(ctx, T), 256, 0, ctx->stream>>>(gs, T);
    const BigTab g{gs, T - 1, full, ~0u};
    const uint32_t gb = (uint32_t)std::min<uint64_t>(hb, (uint64_t)ctx->n_cu * 8);
    k_ovf_big_insert<<<gb, 256, 0, ctx->stream>>>(e1, child, bad, (uint32_t)hb, p, g);
    if (solid)
      k_sk_big_emit<true><<<grid_for(ctx, T), 256, 0, ctx->stream>>>(gs, T, p, o);
    else
      k_sk_big_emit<false><<<grid_for(ctx, T), 256, 0, ctx->stream>>>(gs, T, p, o);
    if (solid && (o.weak || o.wrec)) k_ovf_big_weak<<<gb, 256, 0, ctx->stream>>>(e1, child, bad, (uint32_t)hb, p, g, o);
    APG_CHECK_HIP(hipGetLastError());
    vlog(ctx, "sk count: %llu of %llu overflow sub-buckets (%llu instances) past the LDS table -> global table",
         hb, (unsigned long long)n_sb, (unsigned long long)inst);
  }
  return APG_OK;
}

static int sk_ceil_log2(uint64_t x) {
  int b = 0;
  while ((1ull << b) < x) ++b;
  return b;
}

// Walk grid: two full rounds of the resident k_sk_scatter blocks (the
// costlier of the pair; k_sk_count must use the same grid for the offsets),
// so the last round is not a partial one.
static uint32_t sk_blocks(const apg_ctx* ctx, uint64_t n_reads, const SkP& p) {
  // two full rounds of the count kernel's resident blocks (7 per CU at K=24-25;
  // sized by the walk kernel's 5 the count ran 1.4 rounds: 13.0 -> 12.1 ms;
  // the descriptor replay that follows is lighter per block)
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_sk_count, kSkThreads, (size_t)p.w * kSkThreads * 4) !=
          hipSuccess ||
      occ < 1)
    occ = 4;
  const uint64_t cap = std::min<uint64_t>(kSkMaxBlocks, (uint64_t)std::max(ctx->n_cu, 1) * occ * 2);
  return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(cap, (n_reads + 255) / 256));
}

// Descriptor buffers of a read set's walk (SkDesc): one 8-byte slot per
// kSkDescDiv bases (records average one per ~6.5 bases of 100-bp reads at
// K = 24-25), per-tile counts by first read, per-block flags.  Off (the
// scatter pass walks) with APG_SK_DESC=0 or a read set of unknown size.
constexpr uint32_t kSkDescDiv = 4;
static int sk_desc_bufs(apg_ctx* ctx, const apg_dreads* dr, uint32_t G, SkDesc* out) {
  const char* env = getenv("APG_SK_DESC");  // "0": off; a number: bases per slot (tests force overflow)
  const uint32_t div = env && atoi(env) > 0 ? (uint32_t)atoi(env) : kSkDescDiv;
  *out = SkDesc{nullptr, nullptr, nullptr, div, 0};
  if ((env && !strcmp(env, "0")) || !dr->n_reads || !dr->n_bases) return APG_OK;
  out->slots = dr->n_bases / div + 1;
  APG_TRY(workspace_t(ctx, "sk_desc", out->slots, &out->desc));
  APG_TRY(workspace_t(ctx, "sk_dtcnt", dr->n_reads, &out->tcnt));
  APG_TRY(workspace_t(ctx, "sk_dflag", G, &out->flag));
  return APG_OK;
}

// Pass 1 over reads: per-digit record counts (host) and K-mer counts; leaves
// the scanned [digit][block] matrix in "sk_omat" and the records'
// descriptors in "sk_desc" for sk_scatter.
int sk_count(apg_ctx* ctx, const apg_dreads* dr, int K, int P, std::vector<uint64_t>* rec_counts,
             std::vector<uint64_t>* kmer_counts, uint32_t split) {
  SkP p = make_skp(K);
  p.split = split;
  const int D = sk_ceil_log2((uint64_t)P) + kSkDigitBits;
  const uint32_t ndig = 1u << D;
  const uint32_t G = sk_blocks(ctx, dr->n_reads, p);
  SkReads rv{dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->n_reads};
  uint32_t* cmat = nullptr;
  uint64_t *omat = nullptr, *ds = nullptr;
  unsigned long long* kdig = nullptr;
  APG_TRY(workspace_t(ctx, "sk_cmat", (uint64_t)ndig * G, &cmat));
  APG_TRY(workspace_t(ctx, "sk_omat", (uint64_t)ndig * G + 1, &omat));
  APG_TRY(workspace_t(ctx, "sk_ds", ndig + 1, &ds));
  APG_TRY(workspace_t(ctx, "sk_kdig", ndig, &kdig));
  APG_CHECK_HIP(hipMemsetAsync(kdig, 0, ndig * 8, ctx->stream));
  if (!dr->n_reads) APG_CHECK_HIP(hipMemsetAsync(cmat, 0, (uint64_t)ndig * G * 4, ctx->stream));
  SkDesc dd;
  APG_TRY(sk_desc_bufs(ctx, dr, G, &dd));
  kbegin(ctx, "sk_count", dr->n_bytes + 16 * dr->n_reads);
  if (dr->n_reads)
    k_sk_count<<<G, kSkThreads, (size_t)p.w * kSkThreads * 4, ctx->stream>>>(rv, p, D, cmat, kdig, dd);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  APG_TRY(scan_u32_u64(ctx, cmat, (uint64_t)ndig * G, omat, "sk"));
  k_sk_digit_starts<<<(ndig + 256) / 256, 256, 0, ctx->stream>>>(omat, ndig, G, ds);
  std::vector<uint64_t> h(ndig + 1), kd(ndig);
  APG_CHECK_HIP(hipMemcpyAsync(h.data(), ds, (ndig + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(d2h_sync(ctx, kd.data(), kdig, ndig * 8));
  rec_counts->resize(ndig);
  for (uint32_t d = 0; d < ndig; ++d) (*rec_counts)[d] = h[d + 1] - h[d];
  *kmer_counts = kd;
  auto& s = ctx->skstate;
  s.valid = true;
  s.gen = dr->gen;
  s.K = K;
  s.P = P;
  s.G = G;
  s.total = h[ndig];
  s.desc = dd.desc != nullptr;
  s.split = split;
  if (s.desc) kbytes_add(ctx, "sk_count", s.total * 8);  // the records' descriptors, written
  return APG_OK;
}

template <typename O>
static int sk_scatter_o(apg_ctx* ctx, const apg_dreads* dr, int K, int P, O out, size_t out_bytes,
                        uint32_t split = 0) {
  auto& s = ctx->skstate;
  if (!s.valid || s.gen != dr->gen || s.K != K || s.P != P || s.split != split) {
    std::vector<uint64_t> rc, kc;
    APG_TRY(sk_count(ctx, dr, K, P, &rc, &kc, split));
  }
  SkP p = make_skp(K);
  p.split = split;
  const int D = sk_ceil_log2((uint64_t)P) + kSkDigitBits;
  SkReads rv{dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->n_reads};
  uint64_t* omat = nullptr;
  APG_TRY(workspace_t(ctx, "sk_omat", (uint64_t)(1u << D) * s.G + 1, &omat));
  SkDesc dd{nullptr, nullptr, nullptr, kSkDescDiv, 0};
  if (s.desc) APG_TRY(sk_desc_bufs(ctx, dr, s.G, &dd));
  kbegin(ctx, "sk_scatter", dr->n_bytes + 16 * dr->n_reads + s.total * (out_bytes + (dd.desc ? 8 : 0)));
  if (dr->n_reads) {
    // k_sk_replay: the blocks with descriptors (15.7 -> 13.3 ms for the two
    // scatters of the C2 step against the walk kernel's replay); k_sk_scatter
    // walks the flagged rest (all blocks when descriptors are off)
    if (dd.desc) k_sk_replay<O><<<s.G, kSkThreads, 0, ctx->stream>>>(rv, p, D, omat, out, dd);
    k_sk_scatter<O><<<s.G, kSkThreads, (size_t)p.w * kSkThreads * 4, ctx->stream>>>(rv, p, D, omat, out, dd);
  }
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return APG_OK;
}

template <typename R>
static int sk_scatter_t(apg_ctx* ctx, const apg_dreads* dr, int K, int P, R* out) {
  return sk_scatter_o<R*>(ctx, dr, K, P, out, sizeof(R));
}

int sk_scatter(apg_ctx* ctx, const apg_dreads* dr, int K, int P, SK16* out) {
  return sk_scatter_t<SK16>(ctx, dr, K, P, out);
}

int sk_scatter_pos(apg_ctx* ctx, const apg_dreads* dr, int K, int P, SK16* out, uint64_t* pos, uint32_t split) {
  return sk_scatter_o<SplitOut>(ctx, dr, K, P, SplitOut{out, pos}, sizeof(SK16) + 8, split);
}

// Records of <= 33 - K K-mers span <= 32 bases (the packed SKP's base word),
// and <= 15 K-mers fit its 4-bit count.
uint32_t sk_pack_split(int K) { return (uint32_t)std::min(33 - K, 15); }

// Partition levels + bucket counting of records laid out as P source blocks,
// each grouped by the kSkDigitBits digit below the shard bits:
// rec_counts[src * B1 + l1].  `spare` (may be null) is a buffer of >= n
// records that may be overwritten.  Spectrum into hist (may be null); solid
// mode leaves the solid hashes in "pc_solid" (res->solid, res->n_solid).
// weak (SK24 records, solid mode only): per-base bitmap of weak K-mer
// instances, zeroed by the caller.
__global__ void k_sk_index24(const SK16* __restrict__ in, uint64_t n, SK24* __restrict__ out);
__global__ void k_skp_unpack(const SKP* __restrict__ in, uint64_t n, SK24* __restrict__ out, bool wide) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t o[3];
    skp_unpack(in[i].w0, in[i].w1, o, wide);
    out[i] = SK24{o[0], o[1], o[2]};
  }
}

// The fused K+1 spectrum (sk_solid_weak with up_K = K + 1): the K-records'
// buckets, partitioned for the K count, counted again for their K+1-mers
// (rec_kmer_up): the K+1 pass needs no walk, scatter or partition of its own.
// Valid when K and K + 1 walk with the same m-mers (make_skp(K).m ==
// make_skp(K + 1).m), so the records' minimizers are those of both K-mer
// sizes' definition.  Overflowing buckets go through the global table.
static int sk_up_alloc(apg_ctx* ctx, uint64_t nb, size_t hist_len, SkOut* u) {
  const uint64_t hl = std::max<uint64_t>(hist_len, 2);
  unsigned long long *ghist = nullptr, *gstats = nullptr, *inst = nullptr;
  uint32_t* ovf = nullptr;
  APG_TRY(workspace_t(ctx, "sku_hist", hl, &ghist));
  APG_TRY(workspace_t(ctx, "sku_gstats", 5, &gstats));
  APG_TRY(workspace_t(ctx, "sku_inst", 1, &inst));
  APG_TRY(workspace_t(ctx, "sku_ovf", std::max<uint64_t>(nb, 1), &ovf));
  *u = SkOut{ghist, hl, gstats, ovf, nullptr, 0, 0, nullptr, nullptr, nullptr, 1u, inst};
  return APG_OK;
}

// drec / dcount (may be null): the solid-set count's distinct records per
// bucket (k_sk_bucket_dd's dout), n_drec of them in all.  sk_up_launch
// queues the bucket pass on ctx->stream (grid_frac of a resident round: the
// side-stream form leaves the rest of each CU to the main stream's kernels);
// sk_up_finish waits for it, runs the overflowed buckets and reads the
// results back.
template <typename RB>
static int sk_up_launch(apg_ctx* ctx, const RB* cur, const uint64_t* boff, uint64_t nb, uint64_t n_rec, int K1,
                        bool wide, const SkOut& u, const SK16* drec, const uint32_t* dcount, uint64_t n_drec,
                        double grid_frac = 1.0) {
  SkP p = make_skp(K1);
  p.wide = wide;
  APG_CHECK_HIP(hipMemsetAsync(u.ghist, 0, u.hist_len * 8, ctx->stream));
  APG_CHECK_HIP(hipMemsetAsync(u.gstats, 0, 5 * 8, ctx->stream));
  APG_CHECK_HIP(hipMemsetAsync(u.inst, 0, 8, ctx->stream));
  uint64_t grid = resident_grid(ctx, k_sk_bucket<false, RB, kSkThreads, kSkTab, 20, true>, kSkThreads, nb);
  if (grid_frac < 1.0) grid = std::max<uint64_t>(1, (uint64_t)((double)grid * grid_frac));
  // algorithmic bytes: the records read (the distinct ones with their
  // multiplicity where the solid-set count folded them) and the bucket bounds
  kbegin(ctx, "sk_bucket", (dcount ? n_drec * sizeof(SK16) : n_rec * sizeof(RB)) + (nb + 1) * 8 + (dcount ? nb * 4 : 0));
  // APG_SK_UP_SORT=1: the LDS counting-sort form of the pass (A/B; read per call)
  const char* se = getenv("APG_SK_UP_SORT");
  if (nb && se && !strcmp(se, "1")) {
    uint64_t sg = resident_grid(ctx, k_sk_up_sort<RB>, 256, nb);
    if (grid_frac < 1.0) sg = std::max<uint64_t>(1, (uint64_t)((double)sg * grid_frac));
    k_sk_up_sort<RB><<<(uint32_t)sg, 256, 0, ctx->stream>>>(cur, boff, nb, p, u, drec, dcount);
  } else if (nb) {
    k_sk_bucket<false, RB, kSkThreads, kSkTab, 20, true><<<(uint32_t)grid, kSkThreads, 0, ctx->stream>>>(
        cur, boff, nb, p, u, nullptr, nullptr, drec, dcount);
  }
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return APG_OK;
}

template <typename RB>
static int sk_up_finish(apg_ctx* ctx, const RB* cur, const uint64_t* boff, uint64_t nb, uint64_t n_rec, int K1,
                        bool wide, const SkOut& u, bool folded, uint64_t* hist, size_t hist_len, SkResult* res) {
  SkP p = make_skp(K1);
  p.wide = wide;
  unsigned long long hs[5];
  uint64_t up_inst = 0;  // owned K+1-mer instances the sub-bucket pass counted
  APG_TRY(d2h_sync(ctx, hs, u.gstats, sizeof hs));
  if (hs[1]) {  // overflowed buckets: by sub-bucket, as in sk_stage_count_t
    unsigned long long* nk = u.gstats + 3;
    APG_CHECK_HIP(hipMemsetAsync(nk, 0, 8, ctx->stream));
    const uint32_t n_ovf = (uint32_t)hs[1];
    uint32_t* osz = nullptr;
    uint64_t* opre = nullptr;
    APG_TRY(workspace_t(ctx, "sk_osz", n_ovf, &osz));
    APG_TRY(workspace_t(ctx, "sk_opre", (uint64_t)n_ovf + 1, &opre));
    k_sk_ovf_sizes<<<(n_ovf + 255) / 256, 256, 0, ctx->stream>>>(boff, u.ovf_list, n_ovf, osz);
    APG_TRY(scan_u32_u64(ctx, osz, n_ovf, opre, "sko"));
    const uint32_t g2 = (uint32_t)ctx->n_cu * 8;
    k_sk_big_kmers<RB, true><<<g2, 256, 0, ctx->stream>>>(cur, boff, u.ovf_list, opre, n_ovf, nk);
    unsigned long long nbk = 0;
    APG_TRY(d2h_sync(ctx, &nbk, nk, 8));
    // APG_SK_OVF=global: the owned K+1-mers through one global table
    const char* oe = getenv("APG_SK_OVF");
    if (!(oe && !strcmp(oe, "global"))) {
      vlog(ctx, "sk count (K+1 of K records): %llu buckets overflow the LDS table -> sub-buckets", hs[1]);
      kbegin(ctx, "sk_bucket_global", nbk * 16 * 5);
      APG_TRY((ovf_lds_count<RB, true>(ctx, cur, boff, u.ovf_list, opre, n_ovf, p, nbk, false, u, g2, &up_inst)));
    } else {
      vlog(ctx, "sk count (K+1 of K records): %llu buckets overflow the LDS table -> global table", hs[1]);
      kbegin(ctx, "sk_bucket_global", nbk * 64);
      BigTab g{};
      uint64_t T = 0;
      APG_TRY((big_count<RB, true>(ctx, cur, boff, u.ovf_list, opre, n_ovf, p, nbk, g2, u.inst, &g, &T)));
      k_sk_big_emit<false><<<grid_for(ctx, T), 256, 0, ctx->stream>>>(g.s, T, p, u);
    }
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
    APG_TRY(d2h_sync(ctx, hs, u.gstats, sizeof hs));
  }
  unsigned long long ninst = 0;
  APG_CHECK_HIP(hipMemcpyAsync(&ninst, u.inst, 8, hipMemcpyDeviceToHost, ctx->stream));
  if (hist && hist_len) APG_CHECK_HIP(hipMemcpyAsync(hist, u.ghist, hist_len * 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(sync(ctx));
  if (hist && hist_len) hist[0] = 0;
  *res = SkResult{};
  res->n_distinct = hs[0];
  res->n_overflow_buckets = hs[1];
  res->nbuckets = nb;
  res->n_kmers = ninst + up_inst;
  res->n_records = n_rec;
  vlog(ctx, "sk count K=%d from K=%d records%s: kmers=%llu distinct=%llu ovf=%llu", K1, K1 - 1,
       folded ? " (distinct records x multiplicity)" : "", (unsigned long long)res->n_kmers, hs[0], hs[1]);
  return APG_OK;
}


template <typename RB>
static int sk_up_run(apg_ctx* ctx, const RB* cur, const uint64_t* boff, uint64_t nb, uint64_t n_rec, int K1, bool wide,
                     const SkOut& u, const SK16* drec, const uint32_t* dcount, uint64_t n_drec, uint64_t* hist,
                     size_t hist_len, SkResult* res) {
  APG_TRY(sk_up_launch(ctx, cur, boff, nb, n_rec, K1, wide, u, drec, dcount, n_drec));
  return sk_up_finish(ctx, cur, boff, nb, n_rec, K1, wide, u, dcount != nullptr, hist, hist_len, res);
}

template <typename RB>
static int sk_up_count(apg_ctx* ctx, const RB* cur, const uint64_t* boff, uint64_t nb, uint64_t n_rec, int K1,
                       bool wide, uint64_t* hist, size_t hist_len, SkResult* res) {
  SkOut u;
  APG_TRY(sk_up_alloc(ctx, nb, hist_len, &u));
  return sk_up_run(ctx, cur, boff, nb, n_rec, K1, wide, u, nullptr, nullptr, 0, hist, hist_len, res);
}

template <typename R>
static int sk_stage_count_t(apg_ctx* ctx, const R* src, R* spare, const std::vector<uint64_t>& rec_counts,
                            uint64_t n_kmers, int K, int P, bool solid, uint32_t min_solid, uint64_t* hist,
                            size_t hist_len, unsigned long long* weak, SkResult* res, uint32_t* wrec = nullptr,
                            const SK16* src16 = nullptr, int up_K = 0, uint64_t* up_hist = nullptr,
                            size_t up_hist_len = 0, SkResult* up_res = nullptr, const SKP* srcp = nullptr,
                            bool split16 = false, bool wide = false, const uint64_t* wpos = nullptr,
                            SkSelf self = SkSelf{}) {
  SkP p = make_skp(K);
  p.wide = wide;
  const int pbits = sk_ceil_log2((uint64_t)P), l1 = kSkDigitBits;
  const uint32_t B1 = 1u << l1;
  if (rec_counts.size() != (size_t)P * B1) {
    set_error("sk_stage_count: rec_counts has wrong size");
    return APG_E_ARG;
  }
  uint64_t n = 0;
  for (auto c : rec_counts) n += c;
  // record dedup (k_sk_bucket_dd, K >= kDdMinK) counts smaller buckets, unless
  // halving them would cost another partition level
  // Measured on the C2 step (40 M reads): the solid-set count with the weak
  // pass 33.4 -> 25.9 ms; the plain spectrum count 18.8 -> 22.9 ms, so by
  // default (apg_config.kmer_dedup = 0) the spectrum keeps k_sk_bucket;
  // APG_SK_DEDUP=all / none overrides the context's setting.
  const char* dd_env = getenv("APG_SK_DEDUP");  // per call (tests switch it)
  int mode = ctx->kmer_dedup;
  if (dd_env) mode = !strcmp(dd_env, "all") ? 1 : !strcmp(dd_env, "none") ? 2 : mode;
  const bool dd = K >= kDdMinK && mode != 2 && (solid || mode == 1);
  auto bits_for = [&](uint64_t per) {
    const uint64_t need = std::max<uint64_t>(1, (n_kmers + per - 1) / per);
    return std::min(32 - pbits, std::max(l1, sk_ceil_log2(need)));
  };
  // The plain spectrum count (no dedup, no solid list) may run the smaller
  // LDS table: APG_SK_TAB=1024 halves the table and the buckets (more blocks
  // per CU).  K >= 21 records hold <= 20 K-mers, so the
  // owner map shrinks with them.
  static const int tab_env = getenv("APG_SK_TAB") ? atoi(getenv("APG_SK_TAB")) : 2048;
  const bool small_tab = !solid && tab_env == 1024 && K >= 21;
  int bb = bits_for(small_tab ? kSkBucketKmers / 2 : kSkBucketKmers);
  if (dd) {
    const int bd = bits_for(kDdBucketKmers);
    if ((bd - l1 + kMaxLevelBits - 1) / kMaxLevelBits <= (bb - l1 + kMaxLevelBits - 1) / kMaxLevelBits) bb = bd;
  }
  const int rem = bb - l1;
  int nlev = (rem + kMaxLevelBits - 1) / kMaxLevelBits;
  if (nlev == 0 && P > 1) nlev = 1;  // regroup the P source segments
  std::vector<std::vector<Seg>> parents(B1);
  {
    uint64_t pos = 0;
    for (int s = 0; s < P; ++s)
      for (uint32_t l = 0; l < B1; ++l) {
        const uint64_t c = rec_counts[(size_t)s * B1 + l];
        parents[l].push_back(Seg{pos, c});
        pos += c;
      }
  }
  R *bufA = nullptr, *bufB = spare;
  uint64_t* boff = nullptr;
  APG_TRY(workspace_t(ctx, "sk_boff", (1ull << bb) + 1, &boff));
  const R* cur = src;
  uint64_t nb = B1;
  int consumed = pbits + l1;
  // The multi-GPU owner's records (SK16 + receive index) travel the levels
  // packed (SKP, 16 bytes instead of 24) when the sender cut them to <= 32
  // bases (split16), the receive index fits 32 bits and the bucket bits
  // below the shard bits fit the packed key (22 bits): the first level packs,
  // the middle ones move SKP, the last unpacks.  The packed key holds the
  // minimizer key's bits below the shard bits, so its digits sit pbits
  // higher than in the SK16 key (kshift).
  const bool pack16 = std::is_same<R, SK24>::value && src16 && split16 && nlev >= 2 && n < (1ull << 32) &&
                      bb <= kSkpKeyBits;
  bool packed = srcp != nullptr;
  const int kshift = pack16 ? pbits : 0;
  // Packed records stay packed through the last level: the bucket kernels
  // read them as they are (rec_head / rec_pos), 16 bytes per record written
  // by the last level and read by the count instead of 24 (APG_SK_UNPACK=1:
  // the last level unpacks to SK24, the round-3 form)
  const char* ue = getenv("APG_SK_UNPACK");
  const bool keep_packed = std::is_same<R, SK24>::value && !(ue && !strcmp(ue, "1")) && nlev >= 1 &&
                           (srcp != nullptr || pack16);
  // the ping-pong buffers hold what the levels write: 16-byte SKP records
  // when every level keeps them packed (a C5 rank's count: 2 x 29 GB less
  // than 24-byte records), else n records of R
  const uint64_t nbuf = keep_packed ? (n * sizeof(SKP) + sizeof(R) - 1) / sizeof(R) : n;
  APG_TRY(workspace_t(ctx, kBig1, std::max<uint64_t>(nbuf, 1), &bufA));
  if (!bufB) APG_TRY(workspace_t(ctx, kBig0, std::max<uint64_t>(nbuf, 1), &bufB));
  if constexpr (std::is_same<R, SK24>::value) {  // SK16 input: widened by the first level, or here
    if (src16 && nlev == 0 && n) {
      k_sk_index24<<<grid_for(ctx, n), 256, 0, ctx->stream>>>(src16, n, spare);
      APG_CHECK_HIP(hipGetLastError());
      cur = spare;
    }
    if (srcp && nlev == 0 && n) {  // packed records and no level to unpack them
      k_skp_unpack<<<grid_for(ctx, n), 256, 0, ctx->stream>>>(srcp, n, bufA, wide);
      APG_CHECK_HIP(hipGetLastError());
      cur = bufA;
    }
  }
  if (nlev == 0) {
    std::vector<uint64_t> hb(B1 + 1, 0);
    for (uint32_t l = 0; l < B1; ++l) hb[l + 1] = hb[l] + rec_counts[l];
    APG_CHECK_HIP(hipMemcpyAsync(boff, hb.data(), (B1 + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  }
  std::vector<uint64_t> bounds;  // after the first level: one segment per parent
  for (int lev = 0; lev < nlev; ++lev) {
    const int bits = rem / nlev + (lev < rem % nlev ? 1 : 0);
    consumed += bits;
    R* dst = (cur == bufA) ? bufB : bufA;
    std::vector<uint64_t> hb;
    const bool last = lev + 1 == nlev;
    const PartParents parents_v = lev ? PartParents(bounds) : PartParents(parents);
    bool done = false;
    if constexpr (std::is_same<R, SK24>::value) {
      if (src16 && lev == 0 && pack16) {  // SK16 -> SKP with the input index (the record's mask slot)
        dst = bufA != spare ? bufA : bufB;
        APG_TRY((part_level<SK16, SKP>(ctx, src16, reinterpret_cast<SKP*>(dst), parents_v, 64 - consumed, bits, n, boff,
                                       &hb, "s24", kshift)));
        packed = true;
        done = true;
      } else if (src16 && lev == 0) {  // SK16 -> SK24 with the input index (the record's mask slot)
        dst = bufA != spare ? bufA : bufB;
        APG_TRY((part_level<SK16, SK24>(ctx, src16, dst, parents_v, 64 - consumed, bits, n, boff,
                                        last ? nullptr : &hb, "s24")));
        done = true;
      } else if (packed) {  // packed records through the levels, unpacked by the last
        const SKP* in = reinterpret_cast<const SKP*>(cur);
        if (last && keep_packed)
          APG_TRY((part_level<SKP, SKP>(ctx, in, reinterpret_cast<SKP*>(dst), parents_v, 64 - consumed + kshift, bits, n,
                                        boff, nullptr, "s24")));
        else if (last)
          APG_TRY((part_level<SKP, SK24>(ctx, in, dst, parents_v, 64 - consumed + kshift, bits, n, boff, nullptr, "s24",
                                         0, wide)));
        else
          APG_TRY((part_level<SKP, SKP>(ctx, in, reinterpret_cast<SKP*>(dst), parents_v, 64 - consumed + kshift, bits, n,
                                        boff, &hb, "s24")));
        done = true;
      }
    }
    if (!done)
      APG_TRY(part_level<R>(ctx, cur, dst, parents_v, 64 - consumed, bits, n, boff, last ? nullptr : &hb,
                            sizeof(R) == sizeof(SK24) ? "s24" : "s"));
    nb = parents_v.size() << bits;
    if (!last) bounds.swap(hb);
    cur = dst;
  }
  if (ctx->verbose && nb) {  // bucket skew: the largest buckets (records)
    std::vector<uint64_t> hb(nb + 1);
    APG_TRY(d2h_sync(ctx, hb.data(), boff, (nb + 1) * 8));
    std::vector<uint64_t> sz(nb);
    for (uint64_t b = 0; b < nb; ++b) sz[b] = hb[b + 1] - hb[b];
    std::sort(sz.begin(), sz.end(), std::greater<uint64_t>());
    uint64_t over = 0;
    for (uint64_t b = 0; b < nb && sz[b] > 8 * (n / nb + 1); ++b) over += sz[b];
    vlog(ctx, "sk buckets: %llu, mean %.0f records, largest %llu %llu %llu %llu, %llu records in buckets > 8x mean",
         (unsigned long long)nb, (double)n / nb, (unsigned long long)sz[0], (unsigned long long)sz[std::min<uint64_t>(1, nb - 1)],
         (unsigned long long)sz[std::min<uint64_t>(2, nb - 1)], (unsigned long long)sz[std::min<uint64_t>(3, nb - 1)],
         (unsigned long long)over);
  }
  // the bucket pass over the partitioned records, as they are: RB = R, or
  // SKP when the packed records stayed packed (keep_packed)
  auto buckets = [&](const auto* cur) -> int {
    using RB = std::remove_const_t<std::remove_pointer_t<decltype(cur)>>;
    // outputs
    const uint64_t hl = std::max<uint64_t>(hist_len, 2);
    unsigned long long *ghist = nullptr, *gstats = nullptr;
    uint32_t* ovf = nullptr;
    APG_TRY(workspace_t(ctx, "sk_hist", hl, &ghist));
    uint32_t* redo = nullptr;
    // distinct, overflow, solid, scratch, handed back, distinct records written (dout)
    APG_TRY(workspace_t(ctx, "sk_gstats", 6, &gstats));
    APG_TRY(workspace_t(ctx, "sk_ovf", std::max<uint64_t>(nb, 1), &ovf));
    APG_TRY(workspace_t(ctx, "sk_redo", std::max<uint64_t>(nb, 1), &redo));
    APG_CHECK_HIP(hipMemsetAsync(ghist, 0, hl * 8, ctx->stream));
    APG_CHECK_HIP(hipMemsetAsync(gstats, 0, 6 * 8, ctx->stream));
    // The fused K+1 spectrum (up_K) rides on the record dedup: the solid-set
    // count folds records with their flanks and hands each bucket's distinct
    // records (with multiplicity) to the K+1 pass through the free partition
    // buffer (APG_SK_UP_DD=0: the K+1 pass reads every record instead).
    const bool up_dd_env = !getenv("APG_SK_UP_DD") || strcmp(getenv("APG_SK_UP_DD"), "0") != 0;
    R* dbuf = ((const void*)cur == (const void*)bufA) ? bufB : bufA;
    const bool up_dd = up_K && dd && solid && up_dd_env && RecPos<RB>::value && dbuf && (const void*)dbuf != (const void*)cur &&
                       (const void*)dbuf != (const void*)src16;
    uint32_t* dcount = nullptr;
    if (up_dd) APG_TRY(workspace_t(ctx, "sk_dcount", std::max<uint64_t>(nb, 1), &dcount));
    uint64_t solid_cap = 0;
    uint64_t* sl = nullptr;
    if (solid) {  // capacity: each solid K-mer has >= min_solid instances; grown and rerun if exceeded
      ctx->pc_list_valid = false;  // "pc_solid" is about to be overwritten
      ctx->pc_ext_valid = false;
      // the previous pass's correction tables are dead from here until this
      // count has written its own list into "pc_solid" (cleared there): a
      // failed allocation may release them before, never after
      ctx->ws_dead |= kRoomCorrection;
      solid_cap = std::max<uint64_t>(1024, n_kmers / std::max<uint32_t>(min_solid, 1) / 8);
    }
    // the chunked list (kSolidChunk slots per reservation, compacted into
    // "pc_solid" afterwards): room for every block's partly used chunks
    uint32_t* sused = nullptr;
    auto solid_bufs = [&]() -> int {
      solid_cap = (solid_cap + kSolidChunk - 1) / kSolidChunk * kSolidChunk;
      APG_TRY(workspace_t(ctx, "sk_solid_sparse", solid_cap, &sl));
      APG_TRY(workspace_t(ctx, "sk_sused", solid_cap / kSolidChunk, &sused));
      return APG_OK;
    };
    if (solid) {
      solid_cap += (uint64_t)ctx->n_cu * 16 * kSolidChunk;
      APG_TRY(solid_bufs());
    }
    static const bool prof = getenv("APG_SK_PROF") != nullptr;
    unsigned long long* dprof = nullptr;
    if (prof) {
      APG_TRY(workspace_t(ctx, "sk_prof", 8, &dprof));
      APG_CHECK_HIP(hipMemsetAsync(dprof, 0, 64, ctx->stream));
    }
    SkOut o{ghist, hl, gstats, ovf, sl, solid_cap, min_solid, solid ? weak : nullptr, solid ? wrec : nullptr, dprof,
             (uint32_t)(!solid || (hist && hist_len))};
    o.sused = sused;
    o.wpos = solid ? wpos : nullptr;
    if (solid && weak && wrec) {
      o.self_lo = self.lo;
      o.self_n = self.n;
      o.self_send = self.send;
    }
    o.n_sused = solid ? solid_cap / kSolidChunk : 0;
    // the weak-pass variant (SK24 records) runs 512-thread blocks: its per-wave
    // LDS (owner map, recorded slots) and the table amortised over 8 waves give
    // 16 waves per CU, where 256-thread blocks fit only 3 per CU
    constexpr int NTB = RecPos<RB>::value ? 512 : kSkThreads;
    static const bool own40 = getenv("APG_SK_OWN40") != nullptr;  // A/B: the K <= 20 owner map at K >= 21
    const bool own20 = K >= 21 && !solid && !own40;  // the plain spectrum count's variants
    auto plain = [&](auto kern) { return resident_grid(ctx, kern, NTB, nb); };
    const uint64_t grid = solid        ? resident_grid(ctx, k_sk_bucket<true, RB, NTB>, NTB, nb)
                          : small_tab  ? plain(k_sk_bucket<false, RB, NTB, 1024, 20>)
                          : own20      ? plain(k_sk_bucket<false, RB, NTB, kSkTab, 20>)
                                       : resident_grid(ctx, k_sk_bucket<false, RB, NTB>, NTB, nb);
    // record dedup first (K >= kDdMinK), k_sk_bucket for the buckets it hands back
    // (a launch over a device-side count: no host round trip in between)
    const uint64_t grid_dd = !dd ? 0
                             : solid ? resident_grid(ctx, k_sk_bucket_dd<true, RB>, kDdThreads, nb)
                                     : resident_grid(ctx, k_sk_bucket_dd<false, RB>, kDdThreads, nb);
    // An overflow list (buckets ovl[0, n_ovf)) counted on ctx->stream: the
    // sub-bucket LDS path, or the global table (APG_SK_OVF=global).
    auto run_ovf = [&](const uint32_t* ovl, uint32_t n_ovf) -> int {
      unsigned long long* nk = gstats + 3;
      APG_CHECK_HIP(hipMemsetAsync(nk, 0, 8, ctx->stream));
      uint32_t* osz = nullptr;
      uint64_t* opre = nullptr;
      APG_TRY(workspace_t(ctx, "sk_osz", n_ovf, &osz));
      APG_TRY(workspace_t(ctx, "sk_opre", (uint64_t)n_ovf + 1, &opre));
      k_sk_ovf_sizes<<<(n_ovf + 255) / 256, 256, 0, ctx->stream>>>(boff, ovl, n_ovf, osz);
      APG_TRY(scan_u32_u64(ctx, osz, n_ovf, opre, "sko"));
      const uint32_t g2 = (uint32_t)ctx->n_cu * 8;  // persistent: the flattened list's size stays on the device
      k_sk_big_kmers<RB><<<g2, 256, 0, ctx->stream>>>(cur, boff, ovl, opre, n_ovf, nk);
      unsigned long long nbk = 0;
      APG_TRY(d2h_sync(ctx, &nbk, nk, 8));
      vlog(ctx, "sk count: %u buckets overflow the LDS table (%llu K-mers)", n_ovf, nbk);
      // APG_SK_OVF=global: every overflowed K-mer through one global table
      // (the round-4 path); default: sub-bucket counting in LDS
      const char* oe = getenv("APG_SK_OVF");
      const bool ovf_global = oe && !strcmp(oe, "global");
      if (!ovf_global) {
        // entries written once, moved by one level (count read + move), read
        // by the count and the weak pass
        kbegin(ctx, "sk_bucket_global", nbk * 16 * 6);
        APG_TRY(ovf_lds_count<RB>(ctx, cur, boff, ovl, opre, n_ovf, p, nbk, solid, o, g2));
      } else {
        kbegin(ctx, "sk_bucket_global", nbk * 64);
        BigTab g{};
        uint64_t T = 0;
        APG_TRY((big_count<RB, false>(ctx, cur, boff, ovl, opre, n_ovf, p, nbk, g2, nullptr, &g, &T)));
        if (solid)
          k_sk_big_emit<true><<<grid_for(ctx, T), 256, 0, ctx->stream>>>(g.s, T, p, o);
        else
          k_sk_big_emit<false><<<grid_for(ctx, T), 256, 0, ctx->stream>>>(g.s, T, p, o);
        if constexpr (RecPos<RB>::value) {
          if (o.weak || o.wrec)
            k_sk_big_weak<RB><<<g2, 256, 0, ctx->stream>>>(cur, boff, ovl, opre, n_ovf, p, g, min_solid, o);
        }
      }
      kend(ctx);
      APG_CHECK_HIP(hipGetLastError());
      return APG_OK;
    };
    uint64_t n_drec = 0;
    for (int attempt = 0;; ++attempt) {
      // The heavy buckets (over kSkHeavyRecords records: repeat families,
      // tandem arrays) always overflow; with record dedup they are listed
      // before the bucket pass and counted on the side stream beside it
      // (APG_SK_HEAVY_SIDE=0: after it, with the rest of the overflow).
      uint32_t n_heavy = 0;
      uint32_t* heavy = nullptr;
      hipStream_t hs_side = nullptr;
      o.skip_heavy = 0;
      {
        static const bool heavy_side = !(getenv("APG_SK_HEAVY_SIDE") && !strcmp(getenv("APG_SK_HEAVY_SIDE"), "0"));
        if (heavy_side && dd && solid && attempt == 0 && nb) {
          unsigned long long* nh = nullptr;
          APG_TRY(workspace_t(ctx, "sk_heavy", std::max<uint64_t>(nb, 1), &heavy));
          APG_TRY(workspace_t(ctx, "sk_nheavy", 1, &nh));
          APG_CHECK_HIP(hipMemsetAsync(nh, 0, 8, ctx->stream));
          k_sk_heavy<<<grid_for(ctx, nb), 256, 0, ctx->stream>>>(boff, nb, heavy, nh);
          unsigned long long h = 0;
          APG_TRY(d2h_sync(ctx, &h, nh, 8));
          n_heavy = (uint32_t)h;
          hs_side = n_heavy ? side_stream(ctx) : nullptr;
          if (hs_side) {
            // every workspace the overflow path uses is allocated before the
            // bucket pass is queued (a grow would free under it)
            o.skip_heavy = 1;
            hipEvent_t ev = nullptr;
            APG_CHECK_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            APG_CHECK_HIP(hipEventRecord(ev, ctx->stream));
            APG_CHECK_HIP(hipStreamWaitEvent(hs_side, ev, 0));
            APG_CHECK_HIP(hipEventDestroy(ev));
          } else {
            n_heavy = 0;
          }
        }
      }
      // Algorithmic bytes (inputs read once + outputs written once): the records
      // and bucket offsets; the weak output (one bit per K-mer instance, or a
      // 4-byte mask per record in the multi-GPU form); the solid list is added
      // once its length is known.  The weak pass's L2-hot re-read of the
      // records is not algorithmic and is not counted.
      const uint64_t weak_out = o.weak ? n_kmers / 8 : (o.wrec ? n * 4 : 0);
      kbegin(ctx, solid ? "sk_bucket_solid" : "sk_bucket", n * sizeof(RB) + (nb + 1) * 8 + weak_out);
      if (dd) {
        if (solid) {
          k_sk_bucket_dd<true, RB><<<grid_dd, kDdThreads, 0, ctx->stream>>>(
              cur, boff, nb, p, o, redo, up_dd ? reinterpret_cast<SK16*>(dbuf) : nullptr, dcount);
          k_sk_bucket<true, RB, NTB><<<grid, NTB, 0, ctx->stream>>>(cur, boff, nb, p, o, redo, gstats + 4);
        } else {
          k_sk_bucket_dd<false, RB><<<grid_dd, kDdThreads, 0, ctx->stream>>>(cur, boff, nb, p, o, redo);
          k_sk_bucket<false, RB, NTB><<<grid, NTB, 0, ctx->stream>>>(cur, boff, nb, p, o, redo, gstats + 4);
        }
      } else if (solid) {
        k_sk_bucket<true, RB, NTB><<<grid, NTB, 0, ctx->stream>>>(cur, boff, nb, p, o);
      } else if (small_tab) {
        k_sk_bucket<false, RB, NTB, 1024, 20><<<grid, NTB, 0, ctx->stream>>>(cur, boff, nb, p, o);
      } else if (own20) {
        k_sk_bucket<false, RB, NTB, kSkTab, 20><<<grid, NTB, 0, ctx->stream>>>(cur, boff, nb, p, o);
      } else {
        k_sk_bucket<false, RB, NTB><<<grid, NTB, 0, ctx->stream>>>(cur, boff, nb, p, o);
      }
      kend(ctx);
      APG_CHECK_HIP(hipGetLastError());
      if (n_heavy) {  // beside the bucket pass, then joined into the main stream
        {
          StreamSwap sw(ctx, hs_side);
          APG_TRY(run_ovf(heavy, n_heavy));
        }
        hipEvent_t ev = nullptr;
        APG_CHECK_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        APG_CHECK_HIP(hipEventRecord(ev, hs_side));
        APG_CHECK_HIP(hipStreamWaitEvent(ctx->stream, ev, 0));
        APG_CHECK_HIP(hipEventDestroy(ev));
      }
      unsigned long long hs[6];
      APG_TRY(d2h_sync(ctx, hs, gstats, sizeof hs));
      n_drec = hs[5];
      if (hs[1]) {  // overflowed buckets (the LDS table filled)
        APG_TRY(run_ovf(ovf, (uint32_t)hs[1]));
        APG_TRY(d2h_sync(ctx, hs, gstats, sizeof hs));
      }
      if (prof) {
        unsigned long long hp[8];
        APG_TRY(d2h_sync(ctx, hp, dprof, sizeof hp));
        fprintf(stderr, "[sk_prof] K=%d solid=%d dedup %.3g flatten %.3g insert %.3g weak %.3g emit %.3g clear %.3g redo %llu\n", K,
                (int)solid, (double)hp[0], (double)hp[1], (double)hp[2], (double)hp[3], (double)hp[4], (double)hp[5], hs[4]);
      }
      if (up_dd) kbytes_add(ctx, "sk_bucket_solid", n_drec * sizeof(SK16) + nb * 4);  // distinct records out
      if (!solid || hs[2] <= solid_cap) {
        uint64_t n_solid = 0;
        uint64_t* dense = nullptr;
        if (solid) {  // the chunked list -> dense "pc_solid"
          const uint64_t n_chunks = hs[2] / kSolidChunk;
          uint64_t* offs = nullptr;
          APG_TRY(workspace_t(ctx, "sk_soffs", n_chunks + 1, &offs));
          APG_TRY(scan_u32_u64(ctx, sused, n_chunks, offs, "sks"));
          APG_TRY(d2h_sync(ctx, &n_solid, offs + n_chunks, 8));
          APG_TRY(workspace_t(ctx, "pc_solid", std::max<uint64_t>(n_solid, 1), &dense));
          kbegin(ctx, "solid_compact", n_solid * 16 + n_chunks * 12);
          if (n_chunks)
            k_solid_compact<<<(uint32_t)std::min<uint64_t>(n_chunks, (uint64_t)ctx->n_cu * 8), 256, 0, ctx->stream>>>(
                sl, sused, offs, n_chunks, dense);
          kend(ctx);
          APG_CHECK_HIP(hipGetLastError());
          kbytes_add(ctx, "sk_bucket_solid", n_solid * 8);
          ctx->ws_dead &= ~kRoomCorrection;  // "pc_solid" holds this pass's list: live
        }
        res->n_distinct = hs[0];
        res->n_overflow_buckets = hs[1] + n_heavy;
        res->n_solid = n_solid;
        res->solid = dense;
        res->nbuckets = nb;
        res->n_redo_buckets = dd ? hs[4] : 0;
        break;
      }
      if (attempt >= 2) {
        set_error("sk count: solid list overflow persists");
        return APG_E_STATE;
      }
      vlog(ctx, "sk count: %llu solid K-mers exceed the list (%llu), recounting", hs[2], (unsigned long long)solid_cap);
      solid_cap = hs[2] + hs[2] / 8;
      APG_TRY(solid_bufs());
      o.solid = sl;
      o.solid_cap = solid_cap;
      o.sused = sused;
      o.n_sused = solid_cap / kSolidChunk;
      APG_CHECK_HIP(hipMemsetAsync(ghist, 0, hl * 8, ctx->stream));
      APG_CHECK_HIP(hipMemsetAsync(gstats, 0, 6 * 8, ctx->stream));
    }
    if (hist && hist_len) {
      APG_TRY(d2h_sync(ctx, hist, ghist, hist_len * 8));
      hist[0] = 0;
    }
    res->n_kmers = n_kmers;
    res->n_records = n;
    vlog(ctx, "sk count: K=%d P=%d records=%llu kmers=%llu levels=%d buckets=%llu distinct=%llu redo=%llu ovf=%llu", K,
         P, (unsigned long long)n, (unsigned long long)n_kmers, nlev, (unsigned long long)nb,
         (unsigned long long)res->n_distinct, (unsigned long long)res->n_redo_buckets,
         (unsigned long long)res->n_overflow_buckets);
    if constexpr (RecPos<RB>::value) {
      if (up_K && up_dd) {
        SkOut u;
        APG_TRY(sk_up_alloc(ctx, nb, up_hist_len, &u));
        const SK16* drec = reinterpret_cast<const SK16*>(dbuf);
        // Side stream (APG_SK_UP_SIDE=0: in line): the K+1 pass needs nothing the
        // caller computes next (PreCorrect's candidates, decisions and edits
        // touch neither the records nor their buckets), so it runs beside them
        // on APG_SK_UP_FRAC (default 1.0) of a resident round of blocks, and the
        // caller joins it (side_join) before it returns.
        const char* se = getenv("APG_SK_UP_SIDE");
        const bool side = !(se && !strcmp(se, "0"));
        const hipStream_t sd = side ? side_stream(ctx) : nullptr;
        if (sd) {
          const char* fe = getenv("APG_SK_UP_FRAC");
          const double frac = fe ? std::min(1.0, std::max(0.05, atof(fe))) : 0.85;
          auto launch = [=]() -> int {
            hipEvent_t ev = nullptr;
            APG_CHECK_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
            APG_CHECK_HIP(hipEventRecord(ev, ctx->stream));  // the records and dout are complete
            APG_CHECK_HIP(hipStreamWaitEvent(sd, ev, 0));
            APG_CHECK_HIP(hipEventDestroy(ev));
            StreamSwap sw(ctx, sd);
            return sk_up_launch(ctx, cur, boff, nb, n, up_K, wide, u, drec, dcount, n_drec, frac);
          };
          // APG_SK_UP_AT=s: launched at PreCorrect's stage s (0: now, 1: after
          // the extension table, 2: after the candidate scan — the default: the
          // pass then runs beside the lookup-bound decisions and edits, not the
          // LDS-staged candidate scan; same box, APG_SK_UP_FRAC 0.75 / 1.0:
          // s = 0 160.1 / —, s = 1 163.2 / 162.8, s = 2 160.9 / 158.5 ms)
          const char* ae = getenv("APG_SK_UP_AT");
          // Round 4's last layout (PreCorrect's link pass ahead of the
          // decisions): stage 1 on 0.85 of a round, beside the candidate scan,
          // the inserts and the link pass — same box 141.5-142.2 vs 145.3-145.8
          // ms per step for stage 2 on a full round (0.80: 141.6, 0.92: 143.2,
          // stage 0 at 0.85: 142.2)
          ctx->side_kick_at = ae ? atoi(ae) : ctx->side_kick_default;
          if (ctx->side_kick_at <= 0)
            APG_TRY(launch());
          else
            ctx->side_kick = launch;
          ctx->side_finish = [=]() -> int {
            StreamSwap sw(ctx, sd);
            return sk_up_finish(ctx, cur, boff, nb, n, up_K, wide, u, true, up_hist, up_hist_len, up_res);
          };
        } else {
          APG_TRY(sk_up_run(ctx, cur, boff, nb, n, up_K, wide, u, drec, dcount, n_drec, up_hist, up_hist_len, up_res));
        }
      } else if (up_K) {
        APG_TRY(sk_up_count(ctx, cur, boff, nb, n, up_K, wide, up_hist, up_hist_len, up_res));
      }
    }
    return APG_OK;
  };
  if constexpr (std::is_same<R, SK24>::value) {
    if (keep_packed) return buckets(reinterpret_cast<const SKP*>(cur));
  }
  return buckets(cur);
}

int sk_stage_count(apg_ctx* ctx, const SK16* src, SK16* spare, const std::vector<uint64_t>& rec_counts,
                   uint64_t n_kmers, int K, int P, bool solid, uint32_t min_solid, uint64_t* hist, size_t hist_len,
                   SkResult* res) {
  return sk_stage_count_t<SK16>(ctx, src, spare, rec_counts, n_kmers, K, P, solid, min_solid, hist, hist_len, nullptr,
                                res);
}

// Solid set of a whole read set (P = 1) plus the weak-instance bitmap: bit
// base_off[r] + j of `weak` (zeroed here; (n_bases + 63) / 64 + 1 words) is
// set iff K-mer j of read r has count < min_solid.  Needs K >= 9 (a record's
// K-mers fit one 32-bit mask).
bool sk_can_fuse_up(int K) { return K >= 9 && K + 1 <= 32 && make_skp(K).m == make_skp(K + 1).m; }

int sk_solid_weak(apg_ctx* ctx, const apg_dreads* dr, int K, uint32_t min_solid, unsigned long long* weak,
                  SkResult* res, uint64_t* up_hist, size_t up_hist_len, SkResult* up_res) {
  APG_REQUIRE(K >= 9 && K <= 32, "sk_solid_weak: K must be in [9, 32]");
  const bool up = up_res != nullptr;
  APG_REQUIRE(!up || sk_can_fuse_up(K), "sk_solid_weak: the K+1 spectrum cannot ride on this K");
  APG_REQUIRE(up_hist_len == 0 || up_hist_len >= 2, "spectrum: hist_len must be 0 or >= 2");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const uint64_t words = dr->n_bases / 64 + 2;
  APG_CHECK_HIP(hipMemsetAsync(weak, 0, words * 8, ctx->stream));
  // Packed partition records (SKP, 16 bytes instead of 24 through the
  // scatter and the partition levels): positions below 2^32 with records
  // split into pieces of <= 32 bases, or (wide) below 2^34 with pieces of
  // <= 31 bases and two position bits in the base word — 40 M reads of
  // 100 bp are 4.0 G bases, 50 M (C4 per GPU) 5.0 G, 80 M 8.0 G
  // (APG_SK_PACK=0: SK24 throughout; APG_SK_PACK=wide: the wide form at any
  // size, for tests)
  const char* pe = getenv("APG_SK_PACK");
  const bool force_wide = pe && !strcmp(pe, "wide");
  const bool pack0 = !(pe && !strcmp(pe, "0")) && dr->n_bases < (1ull << 34);
  const bool wide = pack0 && (force_wide || dr->n_bases >= (1ull << 32));
  const bool pack = pack0 && (!wide || K <= 31);
  const uint32_t split = !pack ? 0u : wide ? (uint32_t)std::min(32 - K, 15) : sk_pack_split(K);
  std::vector<uint64_t> rc, kc;
  APG_TRY(sk_count(ctx, dr, K, 1, &rc, &kc, split));
  uint64_t n = 0, nk = 0;
  for (auto c : rc) n += c;
  for (auto c : kc) nk += c;
  SK24* buf = nullptr;
  APG_TRY(workspace_t(ctx, kBig0, std::max<uint64_t>(n, 1), &buf));
  if (pack)
    APG_TRY(sk_scatter_o<SkpOut>(ctx, dr, K, 1, SkpOut{reinterpret_cast<SKP*>(buf), wide}, sizeof(SKP), split));
  else
    APG_TRY(sk_scatter_t<SK24>(ctx, dr, K, 1, buf));
  vlog(ctx, "solid count: %s records (%llu bases)", !pack ? "24-byte" : wide ? "packed wide (34-bit position)" : "packed",
       (unsigned long long)dr->n_bases);
  ctx->sk_record_form = !pack ? 0 : wide ? 2 : 1;
  return sk_stage_count_t<SK24>(ctx, buf, buf, rc, nk, K, 1, true, min_solid, nullptr, 0, weak, res, nullptr, nullptr,
                                up ? K + 1 : 0, up_hist, up_hist_len, up_res,
                                pack ? reinterpret_cast<const SKP*>(buf) : nullptr, false, wide);
}

__global__ void k_sk_index24(const SK16* __restrict__ in, uint64_t n, SK24* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const SK16 x = in[i];
    out[i] = SK24{x.w0, x.w1, i};
  }
}

// Owner side of the multi-GPU weak-mask return: the solid set of the
// received 16-byte records (as sk_stage_count in solid mode) and, for every
// received record i, the mask of its K-mers whose count is < min_solid in
// wrec[i] — the records travel with their receive index as position, so the
// bucket kernel's weak pass writes each mask with a plain store.
int sk_shard_solid_weak(apg_ctx* ctx, const SK16* recv, const std::vector<uint64_t>& rec_counts, uint64_t n_kmers,
                        int K, int P, uint32_t min_solid, uint32_t* wrec, SkResult* res, int up_K, uint64_t* up_hist,
                        size_t up_hist_len, SkResult* up_res, bool split_recs, unsigned long long* weak,
                        const uint64_t* wpos, SkSelf self) {
  APG_REQUIRE(K >= 9 && K <= 32, "sk_shard_solid_weak: K must be in [9, 32]");
  uint64_t n = 0;
  for (auto c : rec_counts) n += c;
  SK24* buf = nullptr;
  APG_TRY(workspace_t(ctx, kBig0, std::max<uint64_t>(n, 1), &buf));
  // weak + wpos (world size 1): the weak bits straight into the reads' bitmap
  // at wpos[receive index], no per-record masks; weak + wpos + wrec (P > 1):
  // the self-owned records' bits so, the others' masks into wrec (SkSelf)
  APG_REQUIRE(!weak || wpos, "sk_shard_solid_weak: weak bits need the send positions");
  APG_REQUIRE(!(weak && wrec) || self.lo + self.n <= n, "sk_shard_solid_weak: self segment out of range");
  if (n > self.n && wrec) APG_CHECK_HIP(hipMemsetAsync(wrec, 0, (n - self.n) * 4, ctx->stream));
  ctx->sk_record_form = 3;
  // the first partition level reads the SK16 records and writes them as SK24
  // with their receive index (no separate widening pass)
  return sk_stage_count_t<SK24>(ctx, buf, buf, rec_counts, n_kmers, K, P, true, min_solid, nullptr, 0, weak, res,
                                wrec, recv, up_K, up_hist, up_hist_len, up_res, nullptr, split_recs, false,
                                weak ? wpos : nullptr, self);
}

__global__ void k_sk_sum_kmers(const SK16* __restrict__ rec, uint64_t n, unsigned long long* __restrict__ out) {
  unsigned long long c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c += (uint32_t)(rec[i].w0 >> 32) & 0xff;
  wave_add(out, c);
}

// K-mer instances carried by n records (device).
uint64_t sk_sum_kmers(apg_ctx* ctx, const SK16* recs, uint64_t n, int* rc) {
  *rc = APG_OK;
  unsigned long long* d = nullptr;
  if ((*rc = workspace_t(ctx, "sk_sum", 1, &d)) != APG_OK) return 0;
  unsigned long long h = 0;
  if (hipMemsetAsync(d, 0, 8, ctx->stream) != hipSuccess) {
    *rc = APG_E_HIP;
    return 0;
  }
  if (n) k_sk_sum_kmers<<<grid_for(ctx, n), 256, 0, ctx->stream>>>(recs, n, d);
  if (hipMemcpyAsync(&h, d, 8, hipMemcpyDeviceToHost, ctx->stream) != hipSuccess || (*rc = sync(ctx)) != APG_OK) {
    if (*rc == APG_OK) *rc = APG_E_HIP;
    return 0;
  }
  return h;
}

// Whole-read-set count (P = 1).
int sk_spectrum(apg_ctx* ctx, const apg_dreads* dr, int K, bool solid, uint32_t min_solid, uint64_t* hist,
                size_t hist_len, SkResult* res) {
  APG_REQUIRE(ctx && dr, "spectrum: NULL ctx/reads");
  APG_REQUIRE(K >= 1 && K <= 32, "spectrum: K must be in [1, 32] for the 64-bit path");
  APG_REQUIRE(hist_len == 0 || hist_len >= 2, "spectrum: hist_len must be 0 or >= 2");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  std::vector<uint64_t> rc, kc;
  APG_TRY(sk_count(ctx, dr, K, 1, &rc, &kc));
  uint64_t n = 0, nk = 0;
  for (auto c : rc) n += c;
  for (auto c : kc) nk += c;
  SK16* buf = nullptr;
  APG_TRY(workspace_t(ctx, kBig0, std::max<uint64_t>(n, 1), &buf));
  APG_TRY(sk_scatter(ctx, dr, K, 1, buf));
  return sk_stage_count(ctx, buf, buf, rc, nk, K, 1, solid, min_solid, hist, hist_len, res);
}

}  // namespace apg
