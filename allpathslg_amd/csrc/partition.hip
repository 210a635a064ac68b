// partition.hip — the device-wide scan and the LDS-staged hash-partition
// level of the k-mer counting pipelines (8-byte hash records and 16-byte
// super-k-mer records; the level is a template over the record type).  See
// partition.hpp.
#include <algorithm>
#include <string>
#include <type_traits>
#include <vector>

#include "apg_core.hpp"
#include "kmer_common.hpp"
#include "partition.hpp"

namespace apg {

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

int scan_u32_u64(apg_ctx* ctx, const uint32_t* d_in, uint64_t n, uint64_t* d_out, const char* tag) {
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

// Several scans of the same length at once (FillFragments' lengths, bytes
// and filled flags): one launch per phase for all columns instead of one per
// column; column c's tile sums at tsum[c * (nt + 1)].
struct ScanCols {
  const uint32_t* in[kScanColsMax];
  uint64_t* out[kScanColsMax];
};
__global__ void __launch_bounds__(kScanThreads) k_scanc_tiles(ScanCols c, uint64_t n, uint64_t nt,
                                                              uint64_t* __restrict__ tsum) {
  __shared__ uint64_t sm[32];
  const uint32_t col = blockIdx.y;
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i)
    if (base + i < n) s += c.in[col][base + i];
  uint64_t tot;
  block_exclusive_scan<uint64_t>(s, sm, &tot);
  if (threadIdx.x == 0) tsum[col * (nt + 1) + blockIdx.x] = tot;
}
__global__ void __launch_bounds__(kScanThreads) k_scanc_apply(ScanCols c, uint64_t n, uint64_t nt,
                                                              const uint64_t* __restrict__ tsum) {
  __shared__ uint64_t sm[32];
  const uint32_t col = blockIdx.y;
  const uint64_t* ts = tsum + col * (nt + 1);
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + threadIdx.x * kScanItems;
  uint32_t v[kScanItems];
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    v[i] = base + i < n ? c.in[col][base + i] : 0;
    s += v[i];
  }
  uint64_t tot;
  uint64_t run = block_exclusive_scan<uint64_t>(s, sm, &tot) + ts[blockIdx.x];
  uint64_t* out = c.out[col];
#pragma unroll
  for (int i = 0; i < kScanItems; ++i) {
    if (base + i < n) out[base + i] = run;
    run += v[i];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = ts[nt];
}

int scan_cols_u32_u64(apg_ctx* ctx, int ncol, const uint32_t* const* d_in, uint64_t n, uint64_t* const* d_out,
                      const char* tag) {
  APG_REQUIRE(ncol >= 1 && ncol <= kScanColsMax, "scan_cols_u32_u64: 1 .. kScanColsMax columns");
  const uint64_t nt = std::max<uint64_t>(1, (n + kScanTile - 1) / kScanTile);
  APG_REQUIRE(nt < (1ull << 31), "scan_cols_u32_u64: too many tiles");
  uint64_t* tsum = nullptr;
  APG_TRY(workspace_t(ctx, (std::string("scan_tsum_") + tag).c_str(), (nt + 1) * ncol, &tsum));
  ScanCols c{};
  for (int i = 0; i < ncol; ++i) {
    c.in[i] = d_in[i];
    c.out[i] = d_out[i];
  }
  kbegin(ctx, "scan", ncol * (n * 4 * 2 + (n + 1) * 8));
  k_scanc_tiles<<<dim3((uint32_t)nt, ncol), kScanThreads, 0, ctx->stream>>>(c, n, nt, tsum);
  for (int i = 0; i < ncol; ++i) k_scan_tsum<<<1, 1024, 0, ctx->stream>>>(tsum + i * (nt + 1), nt);
  k_scanc_apply<<<dim3((uint32_t)nt, ncol), kScanThreads, 0, ctx->stream>>>(c, n, nt, tsum);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return APG_OK;
}

// ------------------------------------------------------------------------
// Stage B: partition levels.  Records of each parent group are split by the
// next `bits` (<= 8) hash bits.  Chunks (runs of records inside one parent)
// are counted into a row-major [chunk][digit] matrix (one coalesced row per
// chunk); a per-parent column scan turns it into each chunk's starting offset
// inside every child, and the children's starts.  The scatter stages a
// kTile-record tile in LDS sorted by digit, so each wave writes contiguous
// per-child runs instead of 8-byte scattered stores.
// ------------------------------------------------------------------------
constexpr int kPartThreads = 256;
constexpr int kScanGroups = 4;                    // 1024-thread column scan

struct Chunk {
  uint64_t start;   // first record
  uint32_t len;     // records
  uint32_t parent;  // parent group
};

// Scatter tile: 60 KiB of LDS (2 workgroups per CU).  A tile puts ~tile /
// 2^bits records in each child run; runs shorter than a few 128-byte L2 lines
// leave partial lines that the next tile of the same chunk completes only if
// the line is still in L2 — with 256 children per workgroup and 4 resident
// workgroups per CU the open lines (32 MiB) overflowed the L2s and the PMC
// passes showed ~2.3x the algorithmic write + read bytes for SK24
// (profiles/r02_v5/pmc).  Twice the tile and half the residency: runs twice
// as long, a quarter of the open lines.
// APG_PART_TILE_BYTES / APG_PART_WPE: compile-time A/B of the scatter tile
// (LDS bytes per block) and its waves-per-EU bound (scripts/build_variants.sh)
#ifndef APG_PART_TILE_BYTES
#define APG_PART_TILE_BYTES 61440
#endif
#ifndef APG_PART_WPE
#define APG_PART_WPE 2
#endif
constexpr int kPartTileBytes = APG_PART_TILE_BYTES;
template <typename R>
struct PartGeom {
  static constexpr int items = (kPartTileBytes / (int)sizeof(R)) / kPartThreads;
  static constexpr int tile = items * kPartThreads;
};

template <typename R>
__global__ void __launch_bounds__(kPartThreads) k_part_count(const R* __restrict__ rec,
                                                             const Chunk* __restrict__ ch, int shift, uint32_t ndig,
                                                             uint32_t* __restrict__ cmat) {
  __shared__ uint32_t hist[256];
  const Chunk c = ch[blockIdx.x];
  hist[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t dmask = ndig - 1;
  const R* p = rec + c.start;
  for (uint32_t i = threadIdx.x; i < c.len; i += blockDim.x) atomicAdd(&hist[(rkey(p[i]) >> shift) & dmask], 1u);
  __syncthreads();
  if (threadIdx.x < ndig) cmat[(uint64_t)blockIdx.x * ndig + threadIdx.x] = hist[threadIdx.x];
}

// One workgroup per parent: pre[row][d] = sum of column d over the parent's
// earlier rows; child[p*ndig + d] = pstart[p] + sum_{d' < d} column total(d').
__global__ void __launch_bounds__(kPartThreads* kScanGroups) k_part_scan(const uint32_t* __restrict__ cmat,
                                                                         const uint32_t* __restrict__ prow,
                                                                         const uint64_t* __restrict__ pstart,
                                                                         uint32_t ndig, uint32_t* __restrict__ pre,
                                                                         uint64_t* __restrict__ child) {
  __shared__ uint32_t gsum[kScanGroups][256];
  __shared__ unsigned long long scan_sm[64];
  const uint32_t p = blockIdx.x, tid = threadIdx.x, d = tid & 255, g = tid >> 8;
  const uint32_t r0 = prow[p], r1 = prow[p + 1], nr = r1 - r0;
  const uint32_t q = (nr + kScanGroups - 1) / kScanGroups;
  const uint32_t a = min(r1, r0 + g * q), b = min(r1, a + q);
  const bool col = d < ndig;
  uint32_t s = 0;
  if (col) {
#pragma unroll 8
    for (uint32_t r = a; r < b; ++r) s += cmat[(uint64_t)r * ndig + d];
  }
  gsum[g][d] = s;
  __syncthreads();
  uint32_t run = 0, tot = 0;
  for (uint32_t k = 0; k < kScanGroups; ++k) {
    if (k < g) run += gsum[k][d];
    tot += gsum[k][d];
  }
  if (col) {
#pragma unroll 8
    for (uint32_t r = a; r < b; ++r) {
      const uint64_t i = (uint64_t)r * ndig + d;
      const uint32_t x = cmat[i];
      pre[i] = run;
      run += x;
    }
  }
  unsigned long long all;
  const unsigned long long ex =
      block_exclusive_scan<unsigned long long>((g == 0 && col) ? (unsigned long long)tot : 0ull, scan_sm, &all);
  if (g == 0 && col) child[(uint64_t)p * ndig + d] = pstart[p] + ex;
}

// The partition key of a record from its first 64-bit word (rkey).
template <typename R>
__device__ __forceinline__ uint64_t rkey_w0(uint64_t w0) {
  if constexpr (sizeof(R) == 8 || std::is_same<R, SKP>::value)
    return w0;
  else
    return w0 << 32;  // SK16 / SK24 / SK48: the minimizer key
}

// RI -> RO: the same record (RO == RI), an SK16 that leaves as an SK24
// carrying its input index (the multi-GPU solid count: the index of a
// received record is where its weak mask goes back; the first level widens
// the records instead of a separate pass over them), or a packed SKP that
// leaves unpacked (the single-GPU solid count's last level).
template <typename RI, typename RO = RI>
__global__ void __launch_bounds__(kPartThreads) __attribute__((amdgpu_waves_per_eu(1, APG_PART_WPE))) k_part_scatter(
    const RI* __restrict__ rec, const Chunk* __restrict__ ch, int shift, uint32_t ndig,
    const uint32_t* __restrict__ pre, const uint64_t* __restrict__ child, RO* __restrict__ out, int kshift, bool wide) {
  static_assert(std::is_same<RI, RO>::value || (sizeof(RI) == 16 && sizeof(RO) == 24) ||
                    (std::is_same<RI, SK16>::value && std::is_same<RO, SKP>::value),
                "RI -> RO: same, 16 -> 24, or SK16 -> SKP");
  constexpr bool kPack = std::is_same<RI, SK16>::value && std::is_same<RO, SKP>::value;
  shift += kPack ? kshift : 0;  // the packed key's digits sit kshift bits higher
  using R = RO;
  constexpr int kPartItems = PartGeom<R>::items;
  constexpr int kTile = PartGeom<R>::tile;
  constexpr uint32_t kQ = sizeof(R) / 8;    // 64-bit words per record, held as words (no 24/48-byte
                                            // aggregates in registers: those went to scratch)
  constexpr uint32_t kQi = sizeof(RI) / 8;  // words read per record
  static_assert(sizeof(R) % 8 == 0, "record size must be a multiple of 8 bytes");
  __shared__ __attribute__((aligned(16))) uint64_t stage[kTile * kQ];
  __shared__ unsigned long long cur[256];
  __shared__ uint32_t lcnt[256];
  __shared__ uint32_t lstart[256];
  __shared__ uint32_t scan_sm[64];
  // Records whose size is not 8 or 16 bytes leave the tile as a word stream
  // (lane i -> word i of a digit run) so every store instruction covers
  // whole 64-byte lines; record-per-lane stores of 24/48-byte records write
  // partial lines (profiles/r01_pmc_v10).  sdig: digit of each staged record.
  constexpr bool kWords = sizeof(R) > 16;
  using W = std::conditional_t<sizeof(R) % 16 == 0, SK16, uint64_t>;
  constexpr uint32_t kWpr = sizeof(R) / sizeof(W);
  __shared__ uint8_t sdig[kWords ? kTile : 1];
  const Chunk c = ch[blockIdx.x];
  const uint32_t tid = threadIdx.x;
  const uint64_t dmask = ndig - 1;
  if (tid < ndig) cur[tid] = child[(uint64_t)c.parent * ndig + tid] + pre[(uint64_t)blockIdx.x * ndig + tid];
  const uint64_t* base = reinterpret_cast<const uint64_t*>(rec + c.start);
  uint64_t v[kPartItems][kQ];
  auto load = [&](uint32_t t) {  // tile starting at record t
#pragma unroll
    for (int i = 0; i < kPartItems; ++i) {
      const uint32_t idx = t + i * kPartThreads + tid;
      if (idx < c.len) {
        if constexpr (std::is_same<RI, SKP>::value && !std::is_same<RO, SKP>::value) {
          skp_unpack(base[(uint64_t)idx * 2], base[(uint64_t)idx * 2 + 1], v[i], wide);
        } else if constexpr (kPack) {
          skp_pack(base[(uint64_t)idx * 2], base[(uint64_t)idx * 2 + 1], c.start + idx, kshift, v[i]);
        } else {
#pragma unroll
          for (uint32_t q = 0; q < kQi; ++q) v[i][q] = base[(uint64_t)idx * kQi + q];
          if constexpr (kQi < kQ) v[i][kQi] = c.start + idx;  // the input index
        }
      }
    }
  };
  load(0);
  for (uint32_t t0 = 0; t0 < c.len; t0 += kTile) {
    const uint32_t tn = min((uint32_t)kTile, c.len - t0);
    lcnt[tid] = 0;
    __syncthreads();
    uint32_t pos[kPartItems];
#pragma unroll
    for (int i = 0; i < kPartItems; ++i) {
      const uint32_t idx = i * kPartThreads + tid;
      if (idx < tn) pos[i] = atomicAdd(&lcnt[(rkey_w0<R>(v[i][0]) >> shift) & dmask], 1u);
    }
    __syncthreads();
    uint32_t tot;
    const uint32_t ex = block_exclusive_scan<uint32_t>(lcnt[tid], scan_sm, &tot);
    lstart[tid] = ex;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPartItems; ++i) {
      const uint32_t idx = i * kPartThreads + tid;
      if (idx < tn) {
        const uint32_t d = (uint32_t)((rkey_w0<R>(v[i][0]) >> shift) & dmask);
        const uint32_t sl = lstart[d] + pos[i];
#pragma unroll
        for (uint32_t q = 0; q < kQ; ++q) stage[sl * kQ + q] = v[i][q];
        if constexpr (kWords) sdig[sl] = (uint8_t)d;
      }
    }
    __syncthreads();
    load(t0 + kTile);  // the next tile's loads: in flight while this tile leaves LDS
    if constexpr (kWords) {
      const W* sw = reinterpret_cast<const W*>(stage);
      W* ow = reinterpret_cast<W*>(out);
      for (uint32_t i = tid; i < tn * kWpr; i += kPartThreads) {
        const uint32_t r = i / kWpr, k = i - r * kWpr;
        const uint32_t d = sdig[r];
        ow[(cur[d] + (r - lstart[d])) * kWpr + k] = sw[i];
      }
    } else {
      const R* sr = reinterpret_cast<const R*>(stage);
      for (uint32_t i = tid; i < tn; i += kPartThreads) {
        const R x = sr[i];
        const uint32_t d = (uint32_t)((rkey(x) >> shift) & dmask);
        out[cur[d] + (i - lstart[d])] = x;
      }
    }
    __syncthreads();
    if (tid < ndig) cur[tid] += lcnt[tid];
  }
}

// One partition level: every parent's segments -> ndig children per parent.
// Writes the children's start offsets to d_child (nparents*ndig + 1) and, if
// host_child, copies them to the host.
template <typename R, typename RO>
int part_level(apg_ctx* ctx, const R* src, RO* dst, const PartParents& parents, int shift, int bits,
               uint64_t n, uint64_t* d_child, std::vector<uint64_t>* host_child, const char* tag, int kshift,
               bool wide) {
  constexpr int kTile = PartGeom<RO>::tile;
  // the count / scan / scatter kernels keep one LDS counter per child (256)
  APG_REQUIRE(bits >= 0 && bits <= 8, "part_level: a level splits into 1 .. 256 children");
  const uint32_t ndig = 1u << bits;
  const uint64_t np = parents.size();
  // ~24K chunks per level: enough workgroups, short count-matrix rows
  const uint64_t chunk = std::max<uint64_t>(4 * kTile, ((n / 24576) + kTile - 1) / kTile * kTile);
  // host scratch kept across calls (capacity reused: the chunk list of a
  // 648 M-record level is ~25 K entries, rebuilt between levels on the
  // critical path)
  static thread_local std::vector<Chunk> chunks;
  static thread_local std::vector<uint32_t> prow;
  static thread_local std::vector<uint64_t> pstart;
  chunks.clear();
  chunks.reserve(n / chunk + np + 1);
  prow.resize(np + 1);
  pstart.resize(np);
  uint64_t pos = 0;
  auto add = [&](uint64_t p, const Seg& s) -> bool {
    if (s.len >= (1ull << 32)) return false;
    for (uint64_t o = 0; o < s.len; o += chunk)
      chunks.push_back(Chunk{s.start + o, (uint32_t)std::min<uint64_t>(chunk, s.len - o), (uint32_t)p});
    pos += s.len;
    return true;
  };
  for (uint64_t p = 0; p < np; ++p) {
    prow[p] = (uint32_t)chunks.size();
    pstart[p] = pos;
    bool ok = true;
    if (parents.lists) {
      for (const Seg& s : (*parents.lists)[p]) ok = ok && add(p, s);
    } else {
      const std::vector<uint64_t>& b = *parents.bounds;
      ok = add(p, Seg{b[p], b[p + 1] - b[p]});
    }
    if (!ok) {
      set_error("part_level: parent group exceeds 2^32 records");
      return APG_E_UNSUPPORTED;
    }
  }
  prow[np] = (uint32_t)chunks.size();
  if (chunks.empty()) chunks.push_back(Chunk{0, 0, 0});  // keep launches non-empty
  const uint64_t nrow = chunks.size();
  Chunk* d_chunks = nullptr;
  uint64_t* d_pstart = nullptr;
  uint32_t *d_prow = nullptr, *cmat = nullptr, *pre = nullptr;
  APG_TRY(workspace_t(ctx, (std::string(tag) + "p_chunks").c_str(), nrow, &d_chunks));
  APG_TRY(workspace_t(ctx, (std::string(tag) + "p_prow").c_str(), np + 1, &d_prow));
  APG_TRY(workspace_t(ctx, (std::string(tag) + "p_pstart").c_str(), np, &d_pstart));
  APG_TRY(workspace_t(ctx, (std::string(tag) + "p_cmat").c_str(), nrow * ndig, &cmat));
  APG_TRY(workspace_t(ctx, (std::string(tag) + "p_pre").c_str(), nrow * ndig, &pre));
  APG_CHECK_HIP(hipMemcpyAsync(d_chunks, chunks.data(), nrow * sizeof(Chunk), hipMemcpyHostToDevice, ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(d_prow, prow.data(), (np + 1) * 4, hipMemcpyHostToDevice, ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(d_pstart, pstart.data(), np * 8, hipMemcpyHostToDevice, ctx->stream));
  const uint64_t nb = np * ndig;
  APG_CHECK_HIP(hipMemcpyAsync(d_child + nb, &n, 8, hipMemcpyHostToDevice, ctx->stream));
  kbegin(ctx, (std::string(tag) + "_part_count").c_str(), n * sizeof(R) + nrow * ndig * 4);
  k_part_count<R><<<(uint32_t)nrow, kPartThreads, 0, ctx->stream>>>(src, d_chunks, shift, ndig, cmat);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  kbegin(ctx, (std::string(tag) + "_part_scan").c_str(), nrow * ndig * 12 + nb * 8);
  k_part_scan<<<(uint32_t)np, kPartThreads * kScanGroups, 0, ctx->stream>>>(cmat, d_prow, d_pstart, ndig, pre,
                                                                             d_child);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  kbegin(ctx, (std::string(tag) + "_part_scatter").c_str(), n * (sizeof(R) + sizeof(RO)) + nrow * ndig * 4);
  k_part_scatter<R, RO><<<(uint32_t)nrow, kPartThreads, 0, ctx->stream>>>(src, d_chunks, shift, ndig, pre, d_child,
                                                                          dst, kshift, wide);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  if (host_child) {
    host_child->resize(nb + 1);
    APG_TRY(d2h_sync(ctx, host_child->data(), d_child, (nb + 1) * 8));
  }
  return APG_OK;
}


template int part_level<uint64_t, uint64_t>(apg_ctx*, const uint64_t*, uint64_t*, const PartParents&,
                                            int, int, uint64_t, uint64_t*, std::vector<uint64_t>*, const char*, int, bool);
template int part_level<SK16, SK16>(apg_ctx*, const SK16*, SK16*, const PartParents&, int, int,
                                    uint64_t, uint64_t*, std::vector<uint64_t>*, const char*, int, bool);
template int part_level<SK16, SK24>(apg_ctx*, const SK16*, SK24*, const PartParents&, int, int,
                                    uint64_t, uint64_t*, std::vector<uint64_t>*, const char*, int, bool);
template int part_level<SKP, SKP>(apg_ctx*, const SKP*, SKP*, const PartParents&, int, int,
                                  uint64_t, uint64_t*, std::vector<uint64_t>*, const char*, int, bool);
template int part_level<SK16, SKP>(apg_ctx*, const SK16*, SKP*, const PartParents&, int, int,
                                   uint64_t, uint64_t*, std::vector<uint64_t>*, const char*, int, bool);
template int part_level<SKP, SK24>(apg_ctx*, const SKP*, SK24*, const PartParents&, int, int,
                                   uint64_t, uint64_t*, std::vector<uint64_t>*, const char*, int, bool);
template int part_level<SK24, SK24>(apg_ctx*, const SK24*, SK24*, const PartParents&, int, int,
                                    uint64_t, uint64_t*, std::vector<uint64_t>*, const char*, int, bool);
template int part_level<SK48, SK48>(apg_ctx*, const SK48*, SK48*, const PartParents&, int, int,
                                    uint64_t, uint64_t*, std::vector<uint64_t>*, const char*, int, bool);

}  // namespace apg

extern "C" int apg_partition_u64(apg_ctx* ctx, const uint64_t* d_in, uint64_t n, int shift, int bits,
                                 uint64_t* d_out, uint64_t* d_child) {
  APG_REQUIRE(ctx && d_child && (n == 0 || (d_in && d_out)), "apg_partition_u64: NULL argument");
  APG_REQUIRE(bits >= 0 && bits <= 8, "apg_partition_u64: bits must be in [0, 8] (one LDS counter per child)");
  APG_REQUIRE(shift >= 0 && shift + bits <= 64, "apg_partition_u64: bits [shift, shift + bits) outside the key");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  std::vector<std::vector<apg::Seg>> parents(1);
  if (n) parents[0].push_back(apg::Seg{0, n});
  // a 0-bit level is one child: the records copied as they are
  APG_TRY(apg::part_level<uint64_t>(ctx, d_in, d_out, parents, bits ? shift : 0, bits, n, d_child, nullptr, "pu"));
  return apg::sync(ctx);
}

