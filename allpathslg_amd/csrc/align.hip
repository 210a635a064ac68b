// align.hip — read-to-unibase aligners and column consensus on MI355X.
//
// Replaces the pairwise aligners feeding CRefMerger / LongReadConsensus
// ([R:M] src/pairwise_aligners/PerfectAlignment*, KmerAligner,
// SmithWatBanded.cc; [R:L] CRefMerger / LongReadConsensus; reference snapshot
// empty).  Semantics: SURVEY §A.7 as pinned in include/apg.h;
// CPU restatement in oracle/align_oracle.c.
//
//   gap-free   one thread per (read, target, offset): 32 bases per XOR +
//              popcount of the 2-bit difference mask; qualities summed only
//              over mismatch bits.  VALU/latency bound, not HBM.
//   banded SW  w <= 9 (k_banded_sw_lds): one lane per pair, directions kept on
//              the CU (last 32 rows in VGPRs, the rest in LDS), score and
//              direction in one min3; w <= 15 (k_banded_sw_lane): one lane per
//              pair, directions through HBM; above: one wavefront per pair,
//              one lane per band diagonal (chunks of
//              64 diagonals): a DP row is one step per lane (diagonal and
//              vertical predecessors are the lane's own and its neighbour's
//              previous-row values) plus a wave min-plus prefix scan for the
//              horizontal chain (D[i][k] = min_{k'<=k} X[k'] + 3 (k - k')).
//              Directions (2 bits/cell) are ballot-packed per row into a
//              per-wave scratch; lane 0 walks the traceback.  Max-plus, not a
//              sum of products: no MFMA formulation applies.
//   consensus  per placed base an atomic add of its quality into the target
//              column's 4 vote counters, then one thread per column decides.
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "apg_core.hpp"
#include "exchange.hpp"
#include "kmer_common.hpp"

namespace apg {

struct AlnPair {  // == apg_aln_pair
  uint32_t s, t;
  int32_t off;
  uint32_t flags;
};

struct SeqSet {
  const uint64_t* base_off;
  const uint64_t* byte_off;
  const uint8_t* packed;
  const uint8_t* quals;
};

__device__ __forceinline__ uint32_t abase(const uint8_t* rd, uint32_t i) { return (rd[i >> 2] >> (2 * (i & 3))) & 3; }

__device__ __forceinline__ uint64_t rev2a(uint64_t x) {  // reverse the 32 2-bit groups
  x = __builtin_bitreverse64(x);
  return ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
}

// 32 bases [j, j+32) of a packed read, LSB-first (base j in bits 0-1).  Reads
// 12 bytes from the aligned word holding base j (device buffers have slack).
__device__ __forceinline__ uint64_t load_lsb64(const uint8_t* rd, uint32_t j) {
  const uintptr_t addr = (uintptr_t)(rd + (j >> 2));
  const uint32_t* w = reinterpret_cast<const uint32_t*>(addr & ~(uintptr_t)3);
  const int sh = (int)(addr & 3) * 8 + 2 * (int)(j & 3);
  const uint64_t q0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  return sh ? (q0 >> sh) | ((uint64_t)w[2] << (64 - sh)) : q0;
}

// n <= 32 bases [i, i+n) of the aligned S (reverse complement if rc) in the
// low 2n bits, LSB-first.
__device__ __forceinline__ uint64_t s_window(const uint8_t* rd, uint32_t L, uint32_t i, uint32_t n, bool rc) {
  if (!rc) return load_lsb64(rd, i);
  // S'[i + t] = 3 - S[L-1-i-t]: the window of S at a = L-i-n, reversed, complemented
  const uint64_t W = load_lsb64(rd, L - i - n);
  return ~rev2a(W) >> (2 * (32 - n));
}

__global__ void __launch_bounds__(256) k_gapfree(SeqSet S, SeqSet T, const AlnPair* __restrict__ pairs, uint64_t n,
                                                 uint32_t* __restrict__ out) {
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    const AlnPair pr = pairs[k];
    const uint32_t Ls = (uint32_t)(S.base_off[pr.s + 1] - S.base_off[pr.s]);
    const uint32_t Lt = (uint32_t)(T.base_off[pr.t + 1] - T.base_off[pr.t]);
    const uint8_t* sr = S.packed + S.byte_off[pr.s];
    const uint8_t* tr = T.packed + T.byte_off[pr.t];
    const uint8_t* sq = S.quals ? S.quals + S.base_off[pr.s] : nullptr;
    const bool rc = pr.flags & 1;
    const int64_t lo = std::max<int64_t>(0, -(int64_t)pr.off);
    const int64_t hi = std::min<int64_t>((int64_t)Ls, (int64_t)Lt - pr.off);
    uint32_t ov = 0, mm = 0, qs = 0;
    for (int64_t i0 = lo; i0 < hi; i0 += 32) {
      const uint32_t nb = (uint32_t)std::min<int64_t>(32, hi - i0);
      const uint64_t mask = nb == 32 ? ~0ull : ((1ull << (2 * nb)) - 1);
      const uint64_t x = (s_window(sr, Ls, (uint32_t)i0, nb, rc) ^ load_lsb64(tr, (uint32_t)(i0 + pr.off))) & mask;
      uint64_t bits = (x | (x >> 1)) & 0x5555555555555555ull;
      ov += nb;
      mm += (uint32_t)__popcll(bits);
      if (sq) {
        while (bits) {
          const uint32_t t = (uint32_t)__ffsll((long long)bits) - 1;
          bits &= bits - 1;
          const uint32_t i = (uint32_t)i0 + (t >> 1);
          qs += rc ? sq[Ls - 1 - i] : sq[i];
        }
      }
    }
    uint4 o;
    o.x = ov;
    o.y = mm;
    o.z = qs;
    o.w = (uint32_t)pr.off;
    reinterpret_cast<uint4*>(out)[k] = o;
  }
}

// ---------------------------------------------------------------------------
// Banded Smith-Waterman (semi-global: all of S, free ends in T)
// ---------------------------------------------------------------------------
constexpr int kSwChunks = 4;  // band <= 256 diagonals (w <= 127)
constexpr int32_t kSwInf = 1 << 29;
constexpr uint32_t DIR_START = 0, DIR_DIAG = 1, DIR_HORZ = 2, DIR_VERT = 3;

struct SwOut {
  int32_t* res;     // 8 per pair
  int32_t* blocks;  // max_blocks x (gap, len) per pair, or null
  uint32_t max_blocks;
};

__host__ __device__ inline uint64_t sw_scratch_words(uint32_t rows_cap, int nch) {
  return (uint64_t)(rows_cap + 1) * nch * 2 + (2ull * rows_cap + 64 * kSwChunks + 64) / 8;
}

// Wave inclusive prefix min.
__device__ __forceinline__ int32_t wave_prefix_min(int32_t x) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int32_t y = __shfl_up(x, o, 64);
    if (lane >= o) x = min(x, y);
  }
  return x;
}

__global__ void __launch_bounds__(256) k_banded_sw(SeqSet S, SeqSet T, const AlnPair* __restrict__ pairs, uint64_t n,
                                                   int w, uint64_t* __restrict__ scratch, uint32_t rows_cap,
                                                   SwOut o) {
  const int lane = lane_id();
  const uint64_t wid = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave_id();
  const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const int band = 2 * w + 1;
  const int nch = (band + 63) >> 6;
  // per-wave scratch: directions [row][chunk] (bit0 mask, bit1 mask), then
  // the traceback's move bytes (<= 2 rows + band)
  uint64_t* dirs = scratch + wid * sw_scratch_words(rows_cap, nch);
  uint8_t* moves = reinterpret_cast<uint8_t*>(dirs + (uint64_t)(rows_cap + 1) * nch * 2);
  for (uint64_t k = wid; k < n; k += nw) {
    const AlnPair pr = pairs[k];
    const int Ls = (int)(S.base_off[pr.s + 1] - S.base_off[pr.s]);
    const int Lt = (int)(T.base_off[pr.t + 1] - T.base_off[pr.t]);
    const uint8_t* sr = S.packed + S.byte_off[pr.s];
    const uint8_t* tr = T.packed + T.byte_off[pr.t];
    const bool rc = pr.flags & 1;
    const int dmin = pr.off - w;
    // row 0: free T prefix
    int32_t Dp[kSwChunks];
#pragma unroll
    for (int c = 0; c < kSwChunks; ++c) {
      const int kk = c * 64 + lane;
      const int j = dmin + kk;
      Dp[c] = (c < nch && kk < band && j >= 0 && j <= Lt) ? 0 : kSwInf;
    }
    for (int i = 1; i <= Ls; ++i) {
      const uint32_t sb = rc ? 3 - abase(sr, (uint32_t)(Ls - i)) : abase(sr, (uint32_t)(i - 1));
      int32_t Dn[kSwChunks];
      int32_t carry = kSwInf;  // D[i] of the previous chunk's last diagonal (horizontal chain)
#pragma unroll
      for (int c = 0; c < kSwChunks; ++c) {
        if (c >= nch) {
          Dn[c] = kSwInf;
          continue;
        }
        const int kk = c * 64 + lane;
        const int j = i + dmin + kk;
        const bool valid = kk < band && j >= 0 && j <= Lt;
        // vertical predecessor D[i-1][j] sits on diagonal kk+1
        int32_t up = __shfl_down(Dp[c], 1, 64);
        const int32_t nxt0 = (c + 1 < kSwChunks) ? __shfl(Dp[c + 1 < kSwChunks ? c + 1 : c], 0, 64) : kSwInf;
        if (lane == 63) up = (c + 1 < nch) ? nxt0 : kSwInf;
        int32_t diagC = kSwInf, vertC = kSwInf;
        if (valid && j >= 1 && Dp[c] < kSwInf) diagC = Dp[c] + (sb == abase(tr, (uint32_t)(j - 1)) ? 0 : 2);
        if (valid && up < kSwInf) vertC = up + 3;
        const int32_t X = valid ? min(diagC, vertC) : kSwInf;
        // horizontal chain: D[kk] = min(X[kk], D[kk-1] + 3) = min_{k'<=kk} X[k'] + 3 (kk - k')
        const int32_t Y = X >= kSwInf ? kSwInf : X - 3 * lane;
        int32_t pm = wave_prefix_min(Y);
        int32_t D = pm >= kSwInf / 2 ? kSwInf : pm + 3 * lane;
        if (carry < kSwInf) D = min(D, carry + 3 * (lane + 1));
        if (!valid) D = kSwInf;
        // direction, with the oracle's tie order: diagonal > gap in S > gap in T
        int32_t left = __shfl_up(D, 1, 64);
        if (lane == 0) left = carry;
        const int32_t horzC = (valid && j >= 1 && left < kSwInf) ? left + 3 : kSwInf;
        uint32_t dir = DIR_START;
        if (D < kSwInf) dir = diagC == D ? DIR_DIAG : horzC == D ? DIR_HORZ : DIR_VERT;
        const uint64_t b0 = __ballot(dir & 1), b1 = __ballot(dir & 2);
        if (lane == 0) {
          uint64_t* row = dirs + ((uint64_t)i * nch + c) * 2;
          row[0] = b0;
          row[1] = b1;
        }
        carry = __shfl(D, 63, 64);
        Dn[c] = D;
      }
#pragma unroll
      for (int c = 0; c < kSwChunks; ++c) Dp[c] = Dn[c];
    }
    // end: min over the last row, ties to the smallest j (= smallest diagonal)
    unsigned long long best = ~0ull;
#pragma unroll
    for (int c = 0; c < kSwChunks; ++c) {
      if (c < nch && Dp[c] < kSwInf) {
        const unsigned long long key = ((unsigned long long)(uint32_t)Dp[c] << 32) | (uint32_t)(c * 64 + lane);
        best = min(best, key);
      }
    }
    for (int off = 32; off > 0; off >>= 1) best = min(best, (unsigned long long)__shfl_xor((long long)best, off, 64));
    if (lane == 0) {
      int32_t* r = o.res + 8 * k;
      for (int q = 0; q < 8; ++q) r[q] = 0;
      if (best == ~0ull) {
        r[7] = 1;
      } else {
        int kk = (int)(best & 0xffffffffu);
        int i = Ls;
        r[0] = (int32_t)(best >> 32);
        r[2] = Ls + dmin + kk;
        // traceback into the wave's move buffer (backwards), then blocks forward
        int nm = 0, mm = 0, gs = 0, gt = 0;
        while (i > 0) {
          const int c = kk >> 6, l = kk & 63;
          const uint64_t* row = dirs + ((uint64_t)i * nch + c) * 2;
          const uint32_t d = (uint32_t)((row[0] >> l) & 1) | ((uint32_t)((row[1] >> l) & 1) << 1);
          if (d == DIR_DIAG) {
            const int j = i + dmin + kk;
            const uint32_t sb = rc ? 3 - abase(sr, (uint32_t)(Ls - i)) : abase(sr, (uint32_t)(i - 1));
            mm += sb != abase(tr, (uint32_t)(j - 1));
            moves[nm++] = 0;
            --i;
          } else if (d == DIR_HORZ) {  // T base against a gap in S
            moves[nm++] = 1;
            ++gs;
            --kk;
          } else {  // S base against a gap in T
            moves[nm++] = 2;
            ++gt;
            --i;
            ++kk;
          }
        }
        r[1] = dmin + kk;  // row 0: j = dmin + kk
        r[3] = mm;
        r[4] = gs;
        r[5] = gt;
        // blocks, forward order (same rule as the oracle)
        uint32_t nb = 0;
        int gap = 0, len = 0;
        bool over = false;
        int32_t* blk = o.blocks ? o.blocks + 2 * (uint64_t)k * o.max_blocks : nullptr;
        for (int q = nm - 1; q >= 0; --q) {
          const uint8_t m = moves[q];
          if (m == 0) {
            ++len;
            continue;
          }
          if (len > 0) {
            if (blk && nb < o.max_blocks) {
              blk[2 * nb] = gap;
              blk[2 * nb + 1] = len;
            } else if (blk) {
              over = true;
            }
            ++nb;
            gap = 0;
            len = 0;
          }
          gap += m == 1 ? 1 : -1;
        }
        if (len > 0 || gap != 0 || nb == 0) {
          if (blk && nb < o.max_blocks) {
            blk[2 * nb] = gap;
            blk[2 * nb + 1] = len;
          } else if (blk) {
            over = true;
          }
          ++nb;
        }
        r[6] = (int32_t)nb;
        r[7] = over ? 2 : 0;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Banded SW, one lane per pair (bands of <= BW diagonals, w <= 15): the DP
// row lives in the lane's registers (D[kk], diagonal kk = j - i - dmin), so a
// cell is a handful of VALU ops with no cross-lane traffic; 64 pairs per wave
// instead of one.  Row i: D[kk] = min(D'[kk] + sub, D'[kk+1] + 3, D[kk-1] + 3)
// (D' = row i-1), the same recurrence, tie order and end rule as k_banded_sw.
// The 2-bit directions of a row are one u64, stored lane-interleaved
// (dirs[i * nthr + thread], coalesced); the traceback re-reads them (L2-hot).
// mismatches = (cost - 3 * gaps) / 2: every path cost is 2 per mismatch plus 3
// per gap base, so no base is re-read.  Blocks: the traceback sees the moves
// backwards, so a first pass counts them and a second writes block r - q.
// ---------------------------------------------------------------------------
// 32 bases [p, p+32) of a target, p possibly negative (bases before the target
// read as 0) or past its end (0): reads stay inside the target set's slack.
__device__ __forceinline__ uint64_t sw_tload(const uint8_t* tr, int Lt, int p) {
  if (p >= Lt || p <= -32) return 0;
  if (p < 0) return load_lsb64(tr, 0) << (2 * (-p));
  return load_lsb64(tr, (uint32_t)p);
}

template <int BW>
__global__ void __launch_bounds__(256) k_banded_sw_lane(SeqSet S, SeqSet T, const AlnPair* __restrict__ pairs,
                                                        uint64_t n, int w, uint64_t* __restrict__ dirs, SwOut o) {
  const uint64_t gt = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
  const int band = 2 * w + 1;
  for (uint64_t k = gt; k < n; k += nthr) {
    const AlnPair pr = pairs[k];
    const int Ls = (int)(S.base_off[pr.s + 1] - S.base_off[pr.s]);
    const int Lt = (int)(T.base_off[pr.t + 1] - T.base_off[pr.t]);
    const uint8_t* sr = S.packed + S.byte_off[pr.s];
    const uint8_t* tr = T.packed + T.byte_off[pr.t];
    const bool rc = pr.flags & 1;
    const int dmin = pr.off - w;
    int32_t D[BW];
#pragma unroll
    for (int kk = 0; kk < BW; ++kk) {
      const int j = dmin + kk;
      D[kk] = (kk < band && j >= 0 && j <= Lt) ? 0 : kSwInf;
    }
    // target bases from tp = i + dmin - 1 (row i's T[j-1] for kk = 0), 64 buffered
    int tp = dmin;
    unsigned __int128 tb = (unsigned __int128)sw_tload(tr, Lt, tp) |
                           ((unsigned __int128)sw_tload(tr, Lt, tp + 32) << 64);
    int have = 64;
    uint64_t sw64 = 0;
    int sq = 0;  // S window start (rc: bases [sq, sq+32) hold S[Ls - i])
    for (int i = 1; i <= Ls; ++i) {
      uint32_t sb;
      if (!rc) {
        if (((i - 1) & 31) == 0) sw64 = load_lsb64(sr, (uint32_t)(i - 1));
        sb = (uint32_t)(sw64 >> (2 * ((i - 1) & 31))) & 3;
      } else {
        const int q = Ls - i;
        if (i == 1 || q < sq) {
          sq = q >= 31 ? q - 31 : 0;
          sw64 = load_lsb64(sr, (uint32_t)sq);
        }
        sb = 3 - ((uint32_t)(sw64 >> (2 * (q - sq))) & 3);
      }
      const uint64_t trow = (uint64_t)tb;
      uint64_t dw = 0;
      int32_t left = kSwInf;
      const int j0 = i + dmin;
#pragma unroll
      for (int kk = 0; kk < BW; ++kk) {
        if (kk < band) {  // wave-uniform
          const int j = j0 + kk;
          const bool valid = j >= 0 && j <= Lt;
          const uint32_t tbase = (uint32_t)(trow >> (2 * kk)) & 3;
          const int32_t diag = (valid && j >= 1) ? D[kk] + (sb == tbase ? 0 : 2) : kSwInf;
          const int32_t vert = (valid && kk + 1 < band) ? D[kk + 1 < BW ? kk + 1 : kk] + 3 : kSwInf;
          const int32_t horz = (valid && j >= 1 && kk >= 1) ? left + 3 : kSwInf;
          int32_t d = min(min(diag, vert), horz);
          uint32_t dir = DIR_START;
          if (d >= kSwInf)
            d = kSwInf;
          else
            dir = d == diag ? DIR_DIAG : d == horz ? DIR_HORZ : DIR_VERT;
          D[kk] = d;
          left = d;
          dw |= (uint64_t)dir << (2 * kk);
        }
      }
      dirs[(uint64_t)i * nthr + gt] = dw;
      tb >>= 2;
      ++tp;
      if (--have < 32) {
        tb |= (unsigned __int128)sw_tload(tr, Lt, tp + have) << (2 * have);
        have += 32;
      }
    }
    unsigned long long best = ~0ull;
#pragma unroll
    for (int kk = 0; kk < BW; ++kk)
      if (kk < band && D[kk] < kSwInf) best = min(best, ((unsigned long long)(uint32_t)D[kk] << 32) | (uint32_t)kk);
    int32_t* r = o.res + 8 * k;
    if (best == ~0ull) {
      reinterpret_cast<int4*>(r)[0] = int4{0, 0, 0, 0};
      reinterpret_cast<int4*>(r)[1] = int4{0, 0, 0, 1};
      continue;
    }
    const int cost = (int)(best >> 32);
    const int kend = (int)(best & 0xffffffffu);
    // traceback pass 1: gaps, start, blocks (reverse segmentation, see above)
    int gs = 0, gtn = 0, nrev = 0;  // nrev: blocks completed before reaching m_0
    int lastlen = -1, lastgap = 0;  // block r (the forward-last), once complete
    int len = 0, gap = 0;
    bool inG = false;
    int kk = kend, i = Ls, ci = -1;
    uint64_t dw = 0;
    while (i > 0) {
      if (i != ci) {
        dw = dirs[(uint64_t)i * nthr + gt];
        ci = i;
      }
      const uint32_t d = (uint32_t)(dw >> (2 * kk)) & 3;
      if (d == DIR_DIAG) {
        if (inG) {
          if (nrev == 0) {
            lastlen = len;
            lastgap = gap;
          }
          ++nrev;
          len = 0;
          gap = 0;
          inG = false;
        }
        ++len;
        --i;
      } else if (d == DIR_HORZ) {
        inG = true;
        ++gap;
        ++gs;
        --kk;
      } else {
        inG = true;
        --gap;
        ++gtn;
        --i;
        ++kk;
      }
    }
    // block 0 = (gap, len) now; block r = (lastgap, lastlen) if nrev > 0
    const bool emit_r = nrev == 0 ? true : (lastlen > 0 || lastgap != 0);
    const int nb = nrev + (emit_r ? 1 : 0);  // nrev == 0: block 0 is block r, always emitted (nb == 0 rule)
    reinterpret_cast<int4*>(r)[0] = int4{cost, dmin + kk, Ls + dmin + kend, (cost - 3 * (gs + gtn)) / 2};
    const bool over = o.blocks && (uint32_t)nb > o.max_blocks;
    reinterpret_cast<int4*>(r)[1] = int4{gs, gtn, nb, over ? 2 : 0};
    if (!o.blocks) continue;
    // pass 2: blocks, forward index r - q for the q-th completed in reverse
    int32_t* blk = o.blocks + 2 * k * (uint64_t)o.max_blocks;
    auto put = [&](int idx, int g, int l) {
      if (idx >= 0 && (uint32_t)idx < o.max_blocks) {
        blk[2 * idx] = g;
        blk[2 * idx + 1] = l;
      }
    };
    const int rr = nrev;  // forward index of the reverse-first block
    int q = 0;
    len = 0;
    gap = 0;
    inG = false;
    kk = kend;
    i = Ls;
    ci = -1;
    while (i > 0) {
      if (i != ci) {
        dw = dirs[(uint64_t)i * nthr + gt];
        ci = i;
      }
      const uint32_t d = (uint32_t)(dw >> (2 * kk)) & 3;
      if (d == DIR_DIAG) {
        if (inG) {
          if (q > 0 || emit_r) put(rr - q, gap, len);
          ++q;
          len = 0;
          gap = 0;
          inG = false;
        }
        ++len;
        --i;
      } else if (d == DIR_HORZ) {
        inG = true;
        ++gap;
        --kk;
      } else {
        inG = true;
        --gap;
        --i;
        ++kk;
      }
    }
    if (q > 0 || emit_r) put(rr - q, gap, len);
  }
}

// ---------------------------------------------------------------------------
// Banded SW, one lane per pair, directions on the CU (w <= 9).
// Same recurrence, tie order, end rule and outputs as k_banded_sw_lane,
// re-shaped for the VALU:
//  * a cell holds 4 * cost + code (code 0 diagonal, 1 gap in S = horizontal,
//    2 gap in T = vertical), so one min3 over the three candidates is both the
//    recurrence and the tie rule (diagonal before horizontal before vertical =
//    the smaller code first); the row keeps 4 * cost (code bits cleared) and
//    the code goes to the row's direction word;
//  * the band is a template parameter (W = w): no per-cell band test, and a
//    wave whose pairs keep the whole band inside their targets (the common
//    case) runs its rows without validity tests;
//  * a row's directions are 2 bits x band: diagonals 0..15 in one word, the
//    rest (band 17 / 19: 2 / 6 bits) packed over rows into side words.  The
//    last kSwVRows rows of a pair stay in VGPRs and the earlier ones go to LDS
//    (one wave per workgroup, lane-interleaved words: conflict-free), so no
//    direction reaches HBM and the LDS a wave needs (18.7 KiB for 100-base
//    reads at w = 8) lets two waves share each SIMD.  Registers take only
//    static indices, so the wave's lanes step through rows in lockstep,
//    aligned at their last row (shorter reads idle first), and the traceback
//    walks the rows in the same lockstep, each lane taking its horizontal moves
//    within a row before the move that leaves it.
// Per cell: mismatch bit, diagonal add, vertical add, horizontal add, min3,
// the cost mask and the pack (v_alignbit): about 7 VALU.
// ---------------------------------------------------------------------------
constexpr int32_t kSw4Inf = 1 << 28;
constexpr int kSwLdsMaxW = 9;
constexpr int kSwVRows = 32;  // rows whose directions stay in VGPRs

__host__ __device__ constexpr int sw_lds_side_bits(int w) { return 2 * (2 * w + 1) > 32 ? 2 * (2 * w + 1) - 32 : 0; }
__host__ __device__ constexpr int sw_lds_rows_per_side(int w) {
  return sw_lds_side_bits(w) ? 32 / sw_lds_side_bits(w) : 1;
}
// 32-bit LDS words per lane for reads of up to rows_cap bases
__host__ __device__ inline uint32_t sw_lds_words(int w, uint32_t rows_cap) {
  const uint32_t rows = rows_cap > (uint32_t)kSwVRows ? rows_cap - kSwVRows : 0;
  const uint32_t rps = (uint32_t)sw_lds_rows_per_side(w);
  return rows + (sw_lds_side_bits(w) ? (rows + rps - 1) / rps : 0);
}

// the last kSwVRows rows' direction words: register vectors indexed by a
// wave-uniform row slot (indirect register moves, no unrolled copies of the
// row body — those overflowed the instruction cache)
typedef uint32_t SwV32 __attribute__((ext_vector_type(kSwVRows)));
typedef uint32_t SwV8 __attribute__((ext_vector_type(8)));
template <int W>
struct SwVDirs {
  SwV32 m;
  SwV8 s;  // side words (band 17 / 19: 2 / 7 used)
};
static_assert((kSwVRows + 4) / 5 <= 8, "side words of the register rows");

// one DP row: G (4 x cost of row i-1, in place -> row i), mm = mismatch bit
// of diagonal kk at bit 2 kk, j0 = column of diagonal 0
template <int W, bool CHECK>
__device__ __forceinline__ void sw_lds_row(int32_t (&G)[2 * W + 1], uint64_t mm, int j0, int Lt, uint32_t& mainw,
                                           uint32_t& sidew) {
  constexpr int B = 2 * W + 1;
  int32_t hz = kSw4Inf;  // horizontal predecessor: row i, diagonal kk - 1
  mainw = 0;
  sidew = 0;
#pragma unroll
  for (int kk = 0; kk < B; ++kk) {
    const uint32_t mis = __builtin_amdgcn_ubfe((uint32_t)(mm >> (kk < 16 ? 0 : 32)), (uint32_t)(2 * kk) & 31u, 1u);
    const int32_t diag = G[kk] + (int32_t)(mis << 3);  // v_bfe + v_lshl_add
    const int32_t vert = kk + 1 < B ? G[kk + 1 < B ? kk + 1 : kk] + 14 : kSw4Inf;  // 4 * 3 + code 2
    int32_t d = min(min(diag, vert), hz + 13);                                       // 4 * 3 + code 1
    if (CHECK && (uint32_t)(j0 + kk) > (uint32_t)Lt) d = kSw4Inf;                   // outside the target
    // the code enters the word from the top (one v_alignbit: no mask + or)
    if (kk < 16)
      mainw = __builtin_amdgcn_alignbit((uint32_t)d, mainw, 2u);
    else
      sidew = __builtin_amdgcn_alignbit((uint32_t)d, sidew, 2u);
    hz = G[kk] = d & ~3;
  }
  if constexpr (B < 16) mainw >>= 32 - 2 * B;  // diagonal 0 at bits 0..1
  if constexpr (B > 16 && B < 32) sidew >>= 32 - 2 * (B - 16);
}

// sw_tload without branches (a load under a per-lane branch makes the
// compiler wait for every load in flight where the branches join): the
// address is clamped into the target and the result fixed up by selects.
__device__ __forceinline__ uint64_t sw_tload_nb(const uint8_t* tr, int Lt, int p) {
  const int pc = min(max(p, 0), max(Lt - 1, 0));
  const uint64_t v = load_lsb64(tr, (uint32_t)pc);
  const uint64_t lo = p > -32 ? v << (2 * min(-p, 31)) : 0;  // p < 0: bases before the target read as 0
  return p >= Lt ? 0 : p < 0 ? lo : v;
}

// The DP rows of one pair, in blocks of 32 lockstep steps (step t is the
// lane's row t - off): a block's 32 bases of S and of T were loaded during the
// previous block and the next block's are loaded at its start, so no global
// load is waited on inside the row loop (one or two waves per SIMD cannot
// hide that).  Steps 1 .. nL write their rows to LDS; the final block (steps
// nL + 1 .. nL + 32, every lane's last 32 rows) keeps them in V.
template <int W, bool CHECK>
__device__ __forceinline__ void sw_lds_dp(int32_t (&G)[2 * W + 1], const uint8_t* sr, const uint8_t* tr, int Ls, int Lt,
                                          bool rc, int dmin, int off, int nL, uint32_t* mainrow, uint32_t* siderow,
                                          SwVDirs<W>& V) {
  constexpr int SB = sw_lds_side_bits(W), RPS = sw_lds_rows_per_side(W);
  // S window of the block whose first row is i0: bases [sq, sq + 32) hold its
  // rows (rc: S[Ls - i]); clamped at 0 (rows < 1 of idle steps are not used)
  auto s_start = [&](int i0) { return rc ? max(Ls - i0 - 31, 0) : max(i0 - 1, 0); };
  int t0 = nL + 1 - 32 * ((nL + 31) / 32);  // first block start (<= 1)
  int i0 = t0 - off;
  // T: tb holds T[tp .. tp + 64) at a block's start (tp = i0 + dmin - 1)
  unsigned __int128 tb = (unsigned __int128)sw_tload_nb(tr, Lt, i0 + dmin - 1) |
                         ((unsigned __int128)sw_tload_nb(tr, Lt, i0 + dmin - 1 + 32) << 64);
  int sq = s_start(i0);
  uint64_t sw64 = load_lsb64(sr, (uint32_t)min(sq, max(Ls - 1, 0)));
  uint64_t swn = 0, tn = 0;  // the next block's windows, in flight
  bool first = true;
  auto next_block = [&]() {
    if (!first) {  // take the windows loaded during the previous block, before issuing the next
      sq = s_start(i0);
      sw64 = swn;
      tb |= (unsigned __int128)tn << 64;  // 32 rows consumed: T[tp, tp + 32) remain in the low half
    }
    first = false;
    swn = load_lsb64(sr, (uint32_t)min(s_start(i0 + 32), max(Ls - 1, 0)));  // unused past the read's end
    tn = sw_tload_nb(tr, Lt, i0 + dmin - 1 + 64);
  };
  auto row = [&](int i, uint32_t& mw, uint32_t& sw) {
    const int q = rc ? Ls - i : i - 1;
    const uint32_t b = (uint32_t)(sw64 >> ((2 * (q - sq)) & 63)) & 3;
    const uint32_t sb = rc ? 3 - b : b;
    const uint64_t x = (uint64_t)tb ^ (sb * 0x5555555555555555ull);
    const uint64_t mm = (x | (x >> 1)) & 0x5555555555555555ull;
    sw_lds_row<W, CHECK>(G, mm, i + dmin, Lt, mw, sw);
  };
  uint32_t sacc = 0;
  int sfill = 0, sidx = 0;
  for (; t0 <= nL; t0 += 32, i0 += 32) {  // rows to LDS
    next_block();
    for (int r = 0; r < 32; ++r) {
      const int i = i0 + r;
      if (i >= 1) {
        uint32_t mw, sw;
        row(i, mw, sw);
        mainrow[(uint32_t)(i - 1) * 64] = mw;
        if (SB) {
          sacc |= sw << (SB * sfill);
          if (++sfill == RPS) {
            siderow[(uint32_t)sidx * 64] = sacc;
            ++sidx;
            sacc = 0;
            sfill = 0;
          }
        }
      }
      tb >>= 2;
    }
  }
  if (SB && sfill) siderow[(uint32_t)sidx * 64] = sacc;
  next_block();  // the last 32 rows: directions in registers
  V.s = SwV8(0u);
  for (int r = 0; r < kSwVRows; ++r) {  // r is wave-uniform
    const int i = i0 + r;
    uint32_t mw = 0, sw = 0;
    if (i >= 1 && i <= Ls) row(i, mw, sw);
    V.m[r] = mw;
    if (SB) V.s[r / RPS] |= sw << (SB * (r % RPS));
    tb >>= 2;
  }
}

// The traceback from (Ls, kend) in the DP's lockstep: row by row from the
// last, each lane's horizontal moves inside the row, then the diagonal or
// vertical move that leaves it; move(d) sees every move in reverse order.
// Returns the diagonal the path starts on (row 0).
template <int W, typename F>
__device__ __forceinline__ int sw_lds_walk(int Ls, int kend, int off, int nL, const uint32_t* mainrow,
                                           const uint32_t* siderow, const SwVDirs<W>& V, F&& move) {
  constexpr int SB = sw_lds_side_bits(W), RPS = sw_lds_rows_per_side(W);
  int kk = kend;
  auto in_row = [&](uint32_t mw, uint32_t sw) {
    for (;;) {
      const uint32_t d = kk < 16 ? (mw >> (2 * kk)) & 3 : (sw >> (2 * (kk - 16))) & 3;
      move(d);
      if (d == 1) {
        --kk;
        continue;
      }
      if (d == 2) ++kk;
      break;
    }
  };
  for (int r = kSwVRows - 1; r >= 0; --r) {  // r is wave-uniform
    const int i = nL + 1 + r - off;
    if (i >= 1 && i <= Ls) in_row(V.m[r], SB ? V.s[r / RPS] >> (SB * (r % RPS)) : 0u);
  }
  // LDS rows: the next row's words load while this row is walked
  auto words = [&](int i, uint32_t& mw, uint32_t& sw) {
    const uint32_t rr = (uint32_t)max(i - 1, 0);
    mw = mainrow[rr * 64];
    sw = SB ? siderow[(rr / RPS) * 64] >> (SB * (rr % RPS)) : 0u;
  };
  uint32_t nm, ns;
  words(nL - off, nm, ns);
  for (int i = nL - off; i >= 1; --i) {
    const uint32_t mw = nm, sw = ns;
    words(i - 1, nm, ns);
    in_row(mw, sw);
  }
  return kk;
}

template <int W>
__global__ void __launch_bounds__(64) k_banded_sw_lds(SeqSet S, SeqSet T, const AlnPair* __restrict__ pairs, uint64_t n,
                                                      uint32_t rows_cap, SwOut o) {
  constexpr int B = 2 * W + 1;
  extern __shared__ uint32_t sw_lds[];
  const int lane = (int)threadIdx.x;
  const uint32_t lds_rows = rows_cap > (uint32_t)kSwVRows ? rows_cap - kSwVRows : 0;
  uint32_t* mainrow = sw_lds + lane;                              // word of row i at (i - 1) * 64
  uint32_t* siderow = sw_lds + (uint64_t)lds_rows * 64 + lane;    // side word (i - 1) / RPS
  const uint64_t stride = (uint64_t)gridDim.x * 64;
  uint64_t k = (uint64_t)blockIdx.x * 64 + lane;
  // the next pair's record and sequence bounds load during this pair's DP
  AlnPair pr{};
  int Ls = 0, Lt = 0;
  const uint8_t* sr = nullptr;
  const uint8_t* tr = nullptr;
  auto meta = [&](const AlnPair& a, int& ls, int& lt, const uint8_t*& s_, const uint8_t*& t_) {
    ls = (int)(S.base_off[a.s + 1] - S.base_off[a.s]);
    lt = (int)(T.base_off[a.t + 1] - T.base_off[a.t]);
    s_ = S.packed + S.byte_off[a.s];
    t_ = T.packed + T.byte_off[a.t];
  };
  if (k < n) {
    pr = pairs[k];
    meta(pr, Ls, Lt, sr, tr);
  }
  AlnPair prn{};
  int Lsn = 0, Ltn = 0;
  const uint8_t* srn = nullptr;
  const uint8_t* trn = nullptr;
  for (; k < n; k += stride, pr = prn, Ls = Lsn, Lt = Ltn, sr = srn, tr = trn) {
    prn = pairs[min(k + stride, n - 1)];  // unconditional (see sw_tload_nb); unused past the end
    const bool rc = pr.flags & 1;
    const int dmin = pr.off - W;
    int maxLs = Ls;  // lockstep rows: the wave's longest read
#pragma unroll
    for (int sh = 32; sh > 0; sh >>= 1) maxLs = max(maxLs, __shfl_xor(maxLs, sh, 64));
    const int off = maxLs - Ls;
    const int nL = max(maxLs - kSwVRows, 0);
    int32_t G[B];
#pragma unroll
    for (int kk = 0; kk < B; ++kk) G[kk] = (uint32_t)(dmin + kk) <= (uint32_t)Lt ? 0 : kSw4Inf;
    SwVDirs<W> V;
    // the whole band inside the target on every row (row 0 included)
    const bool inside = dmin >= 0 && Ls + dmin + B - 1 <= Lt;
    if (__all(inside))
      sw_lds_dp<W, false>(G, sr, tr, Ls, Lt, rc, dmin, off, nL, mainrow, siderow, V);
    else
      sw_lds_dp<W, true>(G, sr, tr, Ls, Lt, rc, dmin, off, nL, mainrow, siderow, V);
    meta(prn, Lsn, Ltn, srn, trn);  // lands during the traceback
    unsigned long long best = ~0ull;
#pragma unroll
    for (int kk = 0; kk < B; ++kk)
      if (G[kk] < kSw4Inf / 2) best = min(best, ((unsigned long long)(uint32_t)(G[kk] >> 2) << 32) | (uint32_t)kk);
    int32_t* r = o.res + 8 * k;
    if (best == ~0ull) {
      reinterpret_cast<int4*>(r)[0] = int4{0, 0, 0, 0};
      reinterpret_cast<int4*>(r)[1] = int4{0, 0, 0, 1};
      continue;
    }
    const int cost = (int)(best >> 32);
    const int kend = (int)(best & 0xffffffffu);
    // traceback pass 1: gaps, start, blocks (reverse segmentation, as in k_banded_sw_lane)
    int gs = 0, gtn = 0, nrev = 0;
    int lastlen = -1, lastgap = 0;
    int len = 0, gap = 0;
    bool inG = false;
    // (state updates as selects: branches here make the compiler keep the
    // counters in scratch behind a selected pointer)
    const int kst = sw_lds_walk<W>(Ls, kend, off, nL, mainrow, siderow, V, [&](uint32_t d) {
      const bool dg = d == 0, close = dg && inG;
      const bool keep = close && nrev == 0;
      lastlen = keep ? len : lastlen;
      lastgap = keep ? gap : lastgap;
      nrev += close ? 1 : 0;
      len = close ? 1 : dg ? len + 1 : len;
      gap = close ? 0 : gap + (d == 1 ? 1 : d == 2 ? -1 : 0);
      inG = !dg;
      gs += d == 1 ? 1 : 0;
      gtn += d == 2 ? 1 : 0;
    });
    const bool emit_r = nrev == 0 ? true : (lastlen > 0 || lastgap != 0);
    const int nb = nrev + (emit_r ? 1 : 0);
    reinterpret_cast<int4*>(r)[0] = int4{cost, dmin + kst, Ls + dmin + kend, (cost - 3 * (gs + gtn)) / 2};
    const bool over = o.blocks && (uint32_t)nb > o.max_blocks;
    reinterpret_cast<int4*>(r)[1] = int4{gs, gtn, nb, over ? 2 : 0};
    if (!o.blocks) continue;
    int32_t* blk = o.blocks + 2 * k * (uint64_t)o.max_blocks;
    auto put = [&](int idx, int g, int l) {
      if (idx >= 0 && (uint32_t)idx < o.max_blocks) {
        blk[2 * idx] = g;
        blk[2 * idx + 1] = l;
      }
    };
    const int rr = nrev;
    int q = 0;
    len = 0;
    gap = 0;
    inG = false;
    sw_lds_walk<W>(Ls, kend, off, nL, mainrow, siderow, V, [&](uint32_t d) {
      const bool dg = d == 0, close = dg && inG;
      if (close && (q > 0 || emit_r)) put(rr - q, gap, len);
      q += close ? 1 : 0;
      len = close ? 1 : dg ? len + 1 : len;
      gap = close ? 0 : gap + (d == 1 ? 1 : d == 2 ? -1 : 0);
      inG = !dg;
    });
    if (q > 0 || emit_r) put(rr - q, gap, len);
  }
}

// ---------------------------------------------------------------------------
// Consensus
// ---------------------------------------------------------------------------
// Votes through an LDS column window: a block takes kVoteChunk consecutive
// placements (wave per placement, lane per base, so a wave's votes hit
// consecutive columns), accumulates them in a window of kVoteWin columns
// starting at the chunk's first placement, and flushes the window's nonzero
// counters with one coalesced global atomic each.  Correct for any placement
// order (votes outside the window go straight to global atomics); placements
// sorted by (target, offset) — apg_unipath_locs with APG_ULOCS_SORTED — land
// almost entirely in the window, so a column takes one global atomic per
// chunk instead of one per placed base (coverage x fewer).
constexpr int kVoteThreads = 256;
struct VoteMeta {
  uint64_t rbyte, rbase;  // read's packed byte offset and base (quality) offset
  uint64_t col0;          // global column facing read position 0 (tb + offset; may wrap below 0)
  uint32_t L;
  int32_t lo, hi;         // read positions [lo, hi) inside the target
  uint32_t flags;
};
constexpr uint32_t kVoteChunk = 128;
constexpr uint32_t kVoteWin = 2048;        // columns x 4 u32 counters = 32 KiB of LDS
constexpr uint32_t kVoteStride = kVoteWin + 1;  // one counter plane per base, planes offset by one bank

// Only columns [c0, c1) are counted, into votes[(column - c0) * 4 + base]:
// the whole target set in one plane (c0 = 0, c1 = columns), or one chunk of
// it at a time (apg_sharded_consensus bounds its planes that way).
__global__ void __launch_bounds__(kVoteThreads) k_votes(SeqSet R, SeqSet T, const AlnPair* __restrict__ plc,
                                                        uint64_t n, uint64_t c0, uint64_t c1,
                                                        uint32_t* __restrict__ votes) {
  // plane-major counters win[b * kVoteStride + column]: a wave's lanes vote
  // on consecutive columns, mostly for the same base, so their LDS atomics hit
  // consecutive banks (column-major [column][4] was a 4-way bank conflict)
  __shared__ uint32_t win[4 * kVoteStride];
  __shared__ unsigned long long g0s;
  __shared__ uint32_t span;
  __shared__ VoteMeta pm[kVoteChunk];
  const uint32_t tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  for (uint32_t x = tid; x < 4 * kVoteStride; x += kVoteThreads) win[x] = 0;
  const uint64_t nchunks = (n + kVoteChunk - 1) / kVoteChunk;
  for (uint64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const uint64_t k0 = c * kVoteChunk, k1 = std::min<uint64_t>(n, k0 + kVoteChunk);
    if (tid == 0) {
      const AlnPair p = plc[k0];
      const int64_t g = (int64_t)T.base_off[p.t] + p.off;
      g0s = g < 0 ? 0ull : (unsigned long long)g;
      span = 0;
    }
    // the chunk's placement metadata, one placement per thread: the dependent
    // offset loads of all placements are in flight at once instead of one
    // placement after another per wave
    if (tid < k1 - k0) {
      const AlnPair p = plc[k0 + tid];
      const uint64_t rb = R.base_off[p.s], tb = T.base_off[p.t];
      const uint32_t L = (uint32_t)(R.base_off[p.s + 1] - rb);
      const uint32_t Lt = (uint32_t)(T.base_off[p.t + 1] - tb);
      const int32_t lo = std::max<int32_t>(0, -p.off);
      const int32_t hi = (int32_t)std::min<int64_t>((int64_t)L, (int64_t)Lt - p.off);
      pm[tid] = VoteMeta{R.byte_off[p.s], rb, tb + (uint64_t)(int64_t)p.off, L, lo, hi, p.flags};
    }
    __syncthreads();  // also orders the previous chunk's window clear
    const uint64_t g0 = g0s;
    uint32_t myspan = 0;
    // two placements per wave step: both placements' bases and qualities are
    // loaded before either one's votes, so their load latencies overlap
    constexpr uint32_t NW = kVoteThreads / 64;
    auto vote = [&](const VoteMeta& m, int64_t i, uint32_t b, uint32_t qq) {
      const uint64_t col = m.col0 + (uint64_t)i;
      const uint64_t d = col - g0;  // wraps (huge) when col < g0
      if (col - c0 >= c1 - c0) return;  // outside this plane (also col < c0: wraps)
      if (d < kVoteWin) {
        atomicAdd(&win[b * kVoteStride + d], qq);
        myspan = std::max<uint32_t>(myspan, (uint32_t)d + 1);
      } else {
        atomicAdd(&votes[(col - c0) * 4 + b], qq);
      }
    };
    auto fetch = [&](const VoteMeta& m, int64_t i, uint32_t* b, uint32_t* qq) {
      const uint8_t* rd = R.packed + m.rbyte;
      const uint8_t* q = R.quals + m.rbase;
      if (m.flags & 1) {
        *b = 3 - abase(rd, (uint32_t)(m.L - 1 - i));
        *qq = q[m.L - 1 - i];
      } else {
        *b = abase(rd, (uint32_t)i);
        *qq = q[i];
      }
    };
    const uint32_t nk = (uint32_t)(k1 - k0);
    for (uint32_t kk = wave; kk < nk; kk += 2 * NW) {
      const bool hasB = kk + NW < nk;
      const VoteMeta ma = pm[kk];
      const VoteMeta mb = hasB ? pm[kk + NW] : ma;
      const int64_t na = (int64_t)ma.hi - ma.lo, nb = hasB ? (int64_t)mb.hi - mb.lo : 0;
      const int64_t n = na > nb ? na : nb;
      for (int64_t t = lane; t < n; t += 64) {
        uint32_t ba = 0, qa = 0, bb = 0, qb = 0;
        if (t < na) fetch(ma, ma.lo + t, &ba, &qa);
        if (t < nb) fetch(mb, mb.lo + t, &bb, &qb);
        if (qa) vote(ma, ma.lo + t, ba, qa);
        if (qb) vote(mb, mb.lo + t, bb, qb);
      }
    }
    if (myspan) atomicMax(&span, myspan);
    __syncthreads();
    const uint32_t sp = span;
    for (uint32_t x = tid; x < sp * 4; x += kVoteThreads) {  // x = column * 4 + base: coalesced global atomics
      const uint32_t w = (x & 3) * kVoteStride + (x >> 2);
      const uint32_t v = win[w];
      if (v) {  // only in-plane votes reach the window: g0 + x / 4 lies in [c0, c1)
        atomicAdd(&votes[(g0 - c0) * 4 + x], v);
        win[w] = 0;
      }
    }
  }
}

// columns [c0, c1) from the plane of k_votes(c0, c1)
__global__ void k_decide(SeqSet T, uint64_t n_targets, uint64_t c0, uint64_t c1, const uint32_t* __restrict__ votes,
                         uint8_t* __restrict__ cons, uint8_t* __restrict__ cq) {
  for (uint64_t col = c0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; col < c1;
       col += (uint64_t)gridDim.x * blockDim.x) {
    // target of this column: binary search over base_off
    uint64_t lo = 0, hi = n_targets;
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) / 2;
      if (T.base_off[mid] <= col)
        lo = mid;
      else
        hi = mid;
    }
    const uint32_t tbase = abase(T.packed + T.byte_off[lo], (uint32_t)(col - T.base_off[lo]));
    const uint4 v4 = reinterpret_cast<const uint4*>(votes)[col - c0];
    const uint32_t v[4] = {v4.x, v4.y, v4.z, v4.w};
    uint32_t win = tbase;
    for (uint32_t b = 0; b < 4; ++b)
      if (v[b] > v[win]) win = b;
    uint32_t other = 0;
    for (uint32_t b = 0; b < 4; ++b)
      if (b != win && v[b] > other) other = v[b];
    const uint32_t dq = v[win] - other;
    cons[col] = (uint8_t)win;
    cq[col] = (uint8_t)(dq > 60 ? 60 : dq);
  }
}

}  // namespace apg

using namespace apg;

namespace {

SeqSet seqset(const apg_dreads* d) { return SeqSet{d->d_base_off, d->d_byte_off, d->d_packed, d->d_quals}; }

// Host-side id/offset validation of a pair list (host API variants).
int check_pairs(const apg_aln_pair* p, uint64_t n, uint64_t nS, uint64_t nT, const char* who) {
  for (uint64_t k = 0; k < n; ++k)
    if (p[k].s_id >= nS || p[k].t_id >= nT) {
      set_error(std::string(who) + ": pair " + std::to_string(k) + " names a sequence out of range");
      return APG_E_ARG;
    }
  return APG_OK;
}

// Copies a host pair list to a device workspace.
int pairs_to_dev(apg_ctx* ctx, const apg_aln_pair* p, uint64_t n, AlnPair** d) {
  APG_TRY(workspace_t(ctx, "a_pairs", std::max<uint64_t>(n, 1), d));
  if (n) APG_CHECK_HIP(hipMemcpyAsync(*d, p, n * sizeof(AlnPair), hipMemcpyHostToDevice, ctx->stream));
  return APG_OK;
}

}  // namespace

extern "C" {

int apg_gapfree_dev(apg_ctx* ctx, const apg_dreads* S, const apg_dreads* T, const apg_aln_pair* d_pairs, uint64_t n,
                    apg_gapfree_hit* d_out) {
  APG_TRY(dreads_quals_ready(S));
  APG_TRY(dreads_quals_ready(T));
  APG_REQUIRE(ctx && S && T, "apg_gapfree: NULL argument");
  APG_REQUIRE(n == 0 || (d_pairs && d_out), "apg_gapfree: NULL pairs/out");
  static_assert(sizeof(apg_aln_pair) == sizeof(AlnPair), "pair layout");
  static_assert(sizeof(apg_gapfree_hit) == 16, "hit layout");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  kbegin(ctx, "gapfree", n * (16 + 16) + n * 2 * 32);
  if (n)
    k_gapfree<<<grid_for(ctx, n), 256, 0, ctx->stream>>>(seqset(S), seqset(T), reinterpret_cast<const AlnPair*>(d_pairs),
                                                          n, reinterpret_cast<uint32_t*>(d_out));
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return sync(ctx);
}

int apg_gapfree(apg_ctx* ctx, const apg_reads* S, const apg_reads* T, const apg_aln_pair* pairs, uint64_t n,
                apg_gapfree_hit* out) {
  APG_REQUIRE(ctx && S && T && (n == 0 || (pairs && out)), "apg_gapfree: NULL argument");
  APG_TRY(check_pairs(pairs, n, S->n_reads, T->n_reads, "apg_gapfree"));
  apg_dreads *dS = nullptr, *dT = nullptr;
  APG_TRY(apg_reads_upload(ctx, S, &dS));
  int rc = apg_reads_upload(ctx, T, &dT);
  AlnPair* dp = nullptr;
  apg_gapfree_hit* dout = nullptr;
  if (rc == APG_OK) rc = pairs_to_dev(ctx, pairs, n, &dp);
  if (rc == APG_OK) rc = workspace_t(ctx, "a_out", std::max<uint64_t>(n, 1), &dout);
  if (rc == APG_OK) rc = apg_gapfree_dev(ctx, dS, dT, reinterpret_cast<apg_aln_pair*>(dp), n, dout);
  if (rc == APG_OK && n) {
    if (hipMemcpy(out, dout, n * sizeof(apg_gapfree_hit), hipMemcpyDeviceToHost) != hipSuccess) {
      set_error("apg_gapfree: D2H failed");
      rc = APG_E_HIP;
    }
  }
  apg_reads_free(dS);
  apg_reads_free(dT);
  return rc;
}

int apg_banded_sw_dev(apg_ctx* ctx, const apg_dreads* S, const apg_dreads* T, const apg_aln_pair* d_pairs, uint64_t n,
                      int band_w, apg_sw_hit* d_out, int32_t* d_blocks, uint32_t max_blocks) {
  APG_TRY(dreads_quals_ready(S));
  APG_TRY(dreads_quals_ready(T));
  APG_REQUIRE(ctx && S && T, "apg_banded_sw: NULL argument");
  APG_REQUIRE(n == 0 || (d_pairs && d_out), "apg_banded_sw: NULL pairs/out");
  APG_REQUIRE(band_w >= 0 && 2 * band_w + 1 <= 64 * kSwChunks, "apg_banded_sw: band_w must be in [0, 127]");
  APG_REQUIRE(!d_blocks || max_blocks > 0, "apg_banded_sw: max_blocks must be > 0 with a block buffer");
  static_assert(sizeof(apg_sw_hit) == 32, "hit layout");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  if (n == 0) return APG_OK;
  const uint32_t rows_cap = (uint32_t)std::max<uint64_t>(S->max_len, 1);
  SwOut o{reinterpret_cast<int32_t*>(d_out), d_blocks, d_blocks ? max_blocks : 0};
  if (d_blocks)  // entries past a pair's n_blocks read as zero
    APG_CHECK_HIP(hipMemsetAsync(d_blocks, 0, n * (uint64_t)max_blocks * 8, ctx->stream));
  const uint64_t lds_bytes = band_w <= kSwLdsMaxW ? 4ull * 64 * sw_lds_words(band_w, rows_cap) : ~0ull;
  if (lds_bytes <= 160ull * 1024 && !std::getenv("APG_SW_NO_LDS")) {  // directions in LDS, one wave per block
    const uint32_t grid = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + 63) / 64, (uint64_t)ctx->n_cu * 64));
    // pairs + results + the S / T bases: the direction rows never leave the CU
    kbegin(ctx, "banded_sw", n * (16 + 32) + n * (uint64_t)rows_cap / 4 * 2);
    const SeqSet ss = seqset(S), ts = seqset(T);
    const AlnPair* pp = reinterpret_cast<const AlnPair*>(d_pairs);
    auto go = [&](auto kern) -> int {
      if (lds_bytes > 64 * 1024)
        APG_CHECK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds_bytes));
      kern<<<grid, 64, (size_t)lds_bytes, ctx->stream>>>(ss, ts, pp, n, rows_cap, o);
      return APG_OK;
    };
    int rc = APG_OK;
    switch (band_w) {
      case 0: rc = go(k_banded_sw_lds<0>); break;
      case 1: rc = go(k_banded_sw_lds<1>); break;
      case 2: rc = go(k_banded_sw_lds<2>); break;
      case 3: rc = go(k_banded_sw_lds<3>); break;
      case 4: rc = go(k_banded_sw_lds<4>); break;
      case 5: rc = go(k_banded_sw_lds<5>); break;
      case 6: rc = go(k_banded_sw_lds<6>); break;
      case 7: rc = go(k_banded_sw_lds<7>); break;
      case 8: rc = go(k_banded_sw_lds<8>); break;
      default: rc = go(k_banded_sw_lds<9>); break;
    }
    kend(ctx);
    APG_TRY(rc);
    APG_CHECK_HIP(hipGetLastError());
    return sync(ctx);
  }
  if (band_w <= 15) {  // lane per pair: 64 pairs per wave, the row in registers
    // direction rows for every thread of the grid: <= ~256 MiB
    const uint64_t per_thread = 8ull * (rows_cap + 1);
    const uint64_t max_thr = std::max<uint64_t>(256, (256ull << 20) / per_thread);
    const uint32_t grid = (uint32_t)std::max<uint64_t>(
        1, std::min<uint64_t>({(n + 255) / 256, (uint64_t)ctx->n_cu * 4, max_thr / 256}));
    const uint64_t nthr = (uint64_t)grid * 256;
    uint64_t* dirs = nullptr;
    APG_TRY(workspace_t(ctx, "a_sw_dirs", nthr * (rows_cap + 1), &dirs));
    // pairs + results + the S / T bases, and the direction rows written and re-read
    kbegin(ctx, "banded_sw", n * (16 + 32) + n * (uint64_t)rows_cap * (8 + 8 + 1));
    const SeqSet ss = seqset(S), ts = seqset(T);
    const AlnPair* pp = reinterpret_cast<const AlnPair*>(d_pairs);
    if (band_w <= 7)
      k_banded_sw_lane<16><<<grid, 256, 0, ctx->stream>>>(ss, ts, pp, n, band_w, dirs, o);
    else if (band_w <= 11)
      k_banded_sw_lane<24><<<grid, 256, 0, ctx->stream>>>(ss, ts, pp, n, band_w, dirs, o);
    else
      k_banded_sw_lane<32><<<grid, 256, 0, ctx->stream>>>(ss, ts, pp, n, band_w, dirs, o);
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
    return sync(ctx);
  }
  const int nch = (2 * band_w + 1 + 63) / 64;
  const uint32_t grid = grid_for(ctx, n, 4);  // 4 waves per block, one pair per wave
  const uint64_t waves = (uint64_t)grid * 4;
  uint64_t* scratch = nullptr;
  APG_TRY(workspace_t(ctx, "a_sw_scratch", waves * sw_scratch_words(rows_cap, nch), &scratch));
  kbegin(ctx, "banded_sw", n * (16 + 32) + n * (uint64_t)rows_cap * (2 * band_w + 1) / 4);
  k_banded_sw<<<grid, 256, 0, ctx->stream>>>(seqset(S), seqset(T), reinterpret_cast<const AlnPair*>(d_pairs), n, band_w,
                                              scratch, rows_cap, o);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return sync(ctx);
}

int apg_banded_sw(apg_ctx* ctx, const apg_reads* S, const apg_reads* T, const apg_aln_pair* pairs, uint64_t n,
                  int band_w, apg_sw_hit* out, int32_t* blocks, uint32_t max_blocks) {
  APG_REQUIRE(ctx && S && T && (n == 0 || (pairs && out)), "apg_banded_sw: NULL argument");
  APG_TRY(check_pairs(pairs, n, S->n_reads, T->n_reads, "apg_banded_sw"));
  apg_dreads *dS = nullptr, *dT = nullptr;
  APG_TRY(apg_reads_upload(ctx, S, &dS));
  int rc = apg_reads_upload(ctx, T, &dT);
  AlnPair* dp = nullptr;
  apg_sw_hit* dout = nullptr;
  int32_t* dblk = nullptr;
  if (rc == APG_OK) rc = pairs_to_dev(ctx, pairs, n, &dp);
  if (rc == APG_OK) rc = workspace_t(ctx, "a_out", std::max<uint64_t>(n, 1), &dout);
  if (rc == APG_OK && blocks) rc = workspace_t(ctx, "a_blocks", std::max<uint64_t>(2 * n * max_blocks, 1), &dblk);
  if (rc == APG_OK)
    rc = apg_banded_sw_dev(ctx, dS, dT, reinterpret_cast<apg_aln_pair*>(dp), n, band_w, dout, dblk, max_blocks);
  if (rc == APG_OK && n) {
    bool ok = hipMemcpy(out, dout, n * sizeof(apg_sw_hit), hipMemcpyDeviceToHost) == hipSuccess;
    if (blocks) ok = ok && hipMemcpy(blocks, dblk, 2 * n * max_blocks * 4, hipMemcpyDeviceToHost) == hipSuccess;
    if (!ok) {
      set_error("apg_banded_sw: D2H failed");
      rc = APG_E_HIP;
    }
  }
  apg_reads_free(dS);
  apg_reads_free(dT);
  return rc;
}

int apg_consensus_dev(apg_ctx* ctx, const apg_dreads* R, const apg_dreads* T, const apg_aln_pair* d_plc, uint64_t n,
                      uint8_t* d_bases, uint8_t* d_quals) {
  APG_TRY(dreads_quals_ready(R));
  APG_TRY(dreads_quals_ready(T));
  APG_REQUIRE(ctx && R && T, "apg_consensus: NULL argument");
  APG_REQUIRE(n == 0 || d_plc, "apg_consensus: NULL placements");
  APG_REQUIRE(n == 0 || R->d_quals, "apg_consensus: the placed reads need qualities");
  APG_REQUIRE(T->n_bases == 0 || (d_bases && d_quals), "apg_consensus: NULL outputs");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const uint64_t NT = T->n_bases;
  uint32_t* votes = nullptr;
  APG_TRY(workspace_t(ctx, "a_votes", std::max<uint64_t>(4 * NT, 4), &votes));
  APG_CHECK_HIP(hipMemsetAsync(votes, 0, std::max<uint64_t>(4 * NT, 4) * 4, ctx->stream));
  kbegin(ctx, "consensus_votes", n * 16 + R->n_bytes + R->n_bases);
  if (n)
    k_votes<<<resident_grid(ctx, k_votes, kVoteThreads, (n + kVoteChunk - 1) / kVoteChunk), kVoteThreads, 0,
              ctx->stream>>>(seqset(R), seqset(T), reinterpret_cast<const AlnPair*>(d_plc), n, 0, NT, votes);
  kend(ctx);
  kbegin(ctx, "consensus_decide", NT * 18);
  if (NT)
    k_decide<<<grid_for(ctx, NT), 256, 0, ctx->stream>>>(seqset(T), T->n_reads, 0, NT, votes, d_bases, d_quals);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return sync(ctx);
}

// Sharded consensus (SURVEY §8e "alignment": unibases replicated, reads
// sharded): each rank's placements vote into a plane of the replicated
// targets' columns, the planes are summed over the ranks (RCCL allreduce),
// and every rank decides every column.  The plane covers at most
// 2^28 columns (4 GiB) at a time: larger target sets are voted chunk by chunk,
// each chunk a pass over the placements restricted to its columns.
int apg_sharded_consensus(apg_ctx* ctx, apg_comm* comm, const apg_dreads* R, const apg_dreads* T,
                          const apg_aln_pair* d_plc, uint64_t n, uint8_t* d_bases, uint8_t* d_quals) {
  APG_TRY(dreads_quals_ready(R));
  APG_TRY(dreads_quals_ready(T));
  APG_REQUIRE(ctx && comm && R && T, "apg_sharded_consensus: NULL argument");
  Comm* c = comm_of(comm);
  APG_REQUIRE(c && c->ctx == ctx, "apg_sharded_consensus: the communicator belongs to another context");
  APG_REQUIRE(n == 0 || d_plc, "apg_sharded_consensus: NULL placements");
  APG_REQUIRE(n == 0 || R->d_quals, "apg_sharded_consensus: the placed reads need qualities");
  APG_REQUIRE(T->n_bases == 0 || (d_bases && d_quals), "apg_sharded_consensus: NULL outputs");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const uint64_t NT = T->n_bases;
  // every rank must hold the same targets: the planes are summed column by
  // column.  Maxima of the shape and of its complement (= ~minima), so every
  // rank sees a mismatch and all fail here together, before the vote loop's
  // collectives (a rank failing alone would leave the others waiting there).
  uint64_t mx[4] = {NT, T->n_reads, ~NT, ~T->n_reads};
  APG_TRY(c->allreduce_u64(mx, 4, APG_COMM_MAX));
  APG_REQUIRE(mx[0] == NT && mx[1] == T->n_reads && ~mx[2] == NT && ~mx[3] == T->n_reads,
              "apg_sharded_consensus: ranks hold different target sets");
  static const uint64_t kChunk = getenv("APG_CONS_CHUNK") ? strtoull(getenv("APG_CONS_CHUNK"), nullptr, 10) : (1ull << 28);
  const uint64_t chunk = std::max<uint64_t>(1, std::min<uint64_t>(NT, kChunk));
  APG_TRY(ws_release_graph_temps(ctx, 16 * chunk));  // the vote plane beside a sharded build's dead temporaries
  uint32_t* votes = nullptr;
  APG_TRY(workspace_t(ctx, "a_votes", std::max<uint64_t>(4 * chunk, 4), &votes));
  for (uint64_t c0 = 0; c0 < NT; c0 += chunk) {
    const uint64_t c1 = std::min(NT, c0 + chunk);
    APG_CHECK_HIP(hipMemsetAsync(votes, 0, (c1 - c0) * 16, ctx->stream));
    kbegin(ctx, "consensus_votes", n * 16 + R->n_bytes + R->n_bases);
    if (n)
      k_votes<<<resident_grid(ctx, k_votes, kVoteThreads, (n + kVoteChunk - 1) / kVoteChunk), kVoteThreads, 0,
                ctx->stream>>>(seqset(R), seqset(T), reinterpret_cast<const AlnPair*>(d_plc), n, c0, c1, votes);
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
    APG_TRY(c->allreduce_dev_u32(votes, 4 * (c1 - c0)));
    kbegin(ctx, "consensus_decide", (c1 - c0) * 18);
    k_decide<<<grid_for(ctx, c1 - c0), 256, 0, ctx->stream>>>(seqset(T), T->n_reads, c0, c1, votes, d_bases, d_quals);
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
  }
  return sync(ctx);
}

int apg_consensus(apg_ctx* ctx, const apg_reads* R, const apg_reads* T, const apg_aln_pair* plc, uint64_t n,
                  uint8_t* bases, uint8_t* quals) {
  APG_REQUIRE(ctx && R && T && (n == 0 || plc), "apg_consensus: NULL argument");
  APG_TRY(check_pairs(plc, n, R->n_reads, T->n_reads, "apg_consensus"));
  apg_dreads *dR = nullptr, *dT = nullptr;
  APG_TRY(apg_reads_upload(ctx, R, &dR));
  int rc = apg_reads_upload(ctx, T, &dT);
  AlnPair* dp = nullptr;
  uint8_t *db = nullptr, *dq = nullptr;
  const uint64_t NT = dT ? dT->n_bases : 0;
  if (rc == APG_OK) rc = pairs_to_dev(ctx, plc, n, &dp);
  if (rc == APG_OK) rc = workspace_t(ctx, "a_cons", std::max<uint64_t>(NT, 1), &db);
  if (rc == APG_OK) rc = workspace_t(ctx, "a_consq", std::max<uint64_t>(NT, 1), &dq);
  if (rc == APG_OK) rc = apg_consensus_dev(ctx, dR, dT, reinterpret_cast<apg_aln_pair*>(dp), n, db, dq);
  if (rc == APG_OK && NT) {
    if (hipMemcpy(bases, db, NT, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(quals, dq, NT, hipMemcpyDeviceToHost) != hipSuccess) {
      set_error("apg_consensus: D2H failed");
      rc = APG_E_HIP;
    }
  }
  apg_reads_free(dR);
  apg_reads_free(dT);
  return rc;
}

}  // extern "C"
