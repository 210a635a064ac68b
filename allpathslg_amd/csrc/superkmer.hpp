// superkmer.hpp — device building blocks of the minimizer (super-k-mer)
// front ends: K <= 32 counting (superkmer.hip) and the K <= 96 unipath node
// builder (unipath.hip).  Reads are walked in LDS tiles, one thread per read,
// with rolling canonical m-mers and a van Herk / Gil-Werman window minimum.
#pragma once

#include <cstdint>

#include <hip/hip_runtime.h>

namespace apg {

// Reverse the order of the 32 2-bit bases of x: bit reversal, then each bit
// pair swapped back (one v_bfi per 32-bit half).
__device__ __forceinline__ uint32_t sk_rev2_32(uint32_t x) {
  x = __builtin_bitreverse32(x);
  return ((x >> 1) & 0x55555555u) | ((x << 1) & 0xaaaaaaaau);
}
__device__ __forceinline__ uint64_t sk_rev2(uint64_t x) {
  return ((uint64_t)sk_rev2_32((uint32_t)x) << 32) | sk_rev2_32((uint32_t)(x >> 32));
}

// 32 bases [j, j+32) of a packed read, LSB-first (12 bytes read from the
// aligned word holding base j; device read buffers carry slack).
__device__ __forceinline__ uint64_t sk_lsb64(const uint8_t* rd, uint32_t j) {
  const uintptr_t addr = (uintptr_t)(rd + (j >> 2));
  const uint32_t* w = reinterpret_cast<const uint32_t*>(addr & ~(uintptr_t)3);
  const int sh = (int)(addr & 3) * 8 + 2 * (int)(j & 3);
  const uint64_t q0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  return sh ? (q0 >> sh) | ((uint64_t)w[2] << (64 - sh)) : q0;
}

__device__ __forceinline__ uint64_t sk_fmix(uint64_t z) {
  z = (z ^ (z >> 33)) * 0xff51afd7ed558ccdull;
  z = (z ^ (z >> 33)) * 0xc4ceb9fe1a85ec53ull;
  return z ^ (z >> 33);
}

// Minimizer order of canonical m-mer c (a 32-bit hash).  The partition key
// of a super-k-mer is a second, bijective mix of its minimizer's order value:
// minimizers are window minima, so their order values crowd near zero, and
// partitioning on them directly would overload the low buckets.
__device__ __forceinline__ uint32_t sk_fmix32(uint32_t v) {  // murmur3 fmix32: a bijection
  v ^= v >> 16;
  v *= 0x85ebca6bu;
  v ^= v >> 13;
  v *= 0xc2b2ae35u;
  v ^= v >> 16;
  return v;
}
__device__ __forceinline__ uint32_t mmer_order(uint64_t c) {  // c < 4^20
  return sk_fmix32(((uint32_t)c ^ 0x2545f491u) ^ ((uint32_t)(c >> 32) * 0x9e3779b1u));
}
__device__ __forceinline__ uint32_t part_key(uint32_t v) { return sk_fmix32(v ^ 0x6b43a9b5u); }

struct SkReads {
  const uint64_t* base_off;
  const uint64_t* byte_off;
  const uint8_t* packed;
  uint64_t n_reads;
};

__device__ __forceinline__ void sk_read_range(uint64_t n, uint32_t G, uint32_t b, uint64_t* r0, uint64_t* r1) {
  *r0 = (n * b) / G;
  *r1 = (n * (b + 1)) / G;
}

// A tile: up to NT consecutive reads whose packed bytes (plus the
// 12-byte window overrun) fit kSkTileBytes, copied into LDS with one
// coalesced pass so the walk below never waits on HBM.  A read too long for
// a tile is walked from global memory on its own.
constexpr uint32_t kSkTileBytes = 8192;
template <int NT>
struct SkTile {
  uint32_t words[kSkTileBytes / 4];
  uint32_t rlen[NT];
  uint32_t rbo[NT];  // byte offset of the read in `words`
};

// Loads the tile starting at read t0 (< r1); returns its read count, or 0
// when read t0 alone exceeds a tile.  Block-uniform; ends with a barrier.
template <int NT>
__device__ __forceinline__ uint32_t sk_load_tile(const SkReads& rv, uint64_t t0, uint64_t r1, SkTile<NT>& T) {
  const uint32_t tid = threadIdx.x;
  const uint64_t b0 = rv.byte_off[t0] & ~3ull;
  const uint64_t r = t0 + tid;
  bool fits = false;
  if (r < r1) {
    const uint32_t len = (uint32_t)(rv.base_off[r + 1] - rv.base_off[r]);
    const uint64_t bo = rv.byte_off[r] - b0;
    fits = bo + (len + 3) / 4 + 12 <= kSkTileBytes;
    T.rlen[tid] = len;
    T.rbo[tid] = (uint32_t)bo;
  }
  const uint32_t n = (uint32_t)__syncthreads_count(fits);
  if (n) {
    const uint32_t nw = (T.rbo[n - 1] + (T.rlen[n - 1] + 3) / 4 + 12 + 3) / 4;
    const uint32_t* g = reinterpret_cast<const uint32_t*>(rv.packed + b0);
    for (uint32_t i = tid; i < nw; i += NT) T.words[i] = g[i];
  }
  __syncthreads();
  return n;
}

// One thread per read of the tile (a GLOBAL tile: thread 0 walks the one long
// read from HBM).  The read is rolled base by base (fw / rc m-mer, order of
// the canonical one); the minimum of each window of w orders comes from the
// van Herk / Gil-Werman block scheme — orders are taken in blocks of w, the
// finished block is turned into suffix minima in this thread's LDS column
// (sb[t * NT], conflict-free), and window [i, i+w-1] = min(suffix of
// block k-1 from i, prefix of block k up to i+w-1) — so every lane does the
// same work per base with no rescans.  f(rd, L, a, n, key) per record: K-mers
// [a, a+n) sharing minimizer order `key`, n <= maxnk.
// P: any parameter struct with K, m, w, maxnk, mmask (2m-bit mask).
template <int NT, bool GLOBAL, typename P, typename F>
__device__ __forceinline__ void sk_walk(const SkReads& rv, const P& p, const SkTile<NT>& T, uint64_t t0, uint32_t n,
                                        uint32_t* sb, F f) {
  const uint32_t q = threadIdx.x;
  if (q >= (GLOBAL ? 1u : n)) return;
  const uint32_t L = T.rlen[q];
  if (L < (uint32_t)p.K) return;
  const uint8_t* rd = GLOBAL ? rv.packed + rv.byte_off[t0] : reinterpret_cast<const uint8_t*>(T.words) + T.rbo[q];
  const uint32_t w = (uint32_t)p.w, m = (uint32_t)p.m, maxnk = (uint32_t)p.maxnk;
  const int rsh = 2 * p.m - 2;
  uint64_t fw = 0, rc = 0;
  uint32_t byte = 0, pre = 0, t = 0, key = 0, ra = 0, rn = 0;
  for (uint32_t j = 0; j < L; ++j) {  // base j
    if ((j & 3) == 0) byte = rd[j >> 2];
    const uint64_t b = (byte >> (2 * (j & 3))) & 3;
    fw = ((fw << 2) | b) & p.mmask;
    rc = (rc >> 2) | ((3 - b) << rsh);
    if (j + 1 < m) continue;
    const uint32_t v = mmer_order(fw < rc ? fw : rc);  // m-mer x = j + 1 - m, offset t in its block
    pre = t == 0 ? v : min(pre, v);
    const uint32_t suf = t + 1 < w ? sb[(t + 1) * NT] : 0xffffffffu;
    sb[t * NT] = v;
    const uint32_t x = j + 1 - m;
    if (x + 1 >= w) {  // K-mer i = x + 1 - w
      const uint32_t kk = min(suf, pre);
      if (x + 1 == w) {
        key = kk;
        ra = 0;
        rn = 1;
      } else if (kk == key && rn < maxnk) {
        ++rn;
      } else {
        f(rd, L, ra, rn, key);
        key = kk;
        ra = x + 1 - w;
        rn = 1;
      }
    }
    if (++t == w) {  // block done: suffix minima in place
      for (int u = (int)w - 2; u >= 0; --u) sb[u * NT] = min(sb[u * NT], sb[(u + 1) * NT]);
      t = 0;
    }
  }
  f(rd, L, ra, rn, key);
}

}  // namespace apg
