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
// One multiply per 32-bit half: a window minimum compares the high bits,
// which a multiply by an odd constant makes depend on every bit below them
// (round 5: the walks are VALU-bound and integer multiplies issue at a
// quarter rate — murmur's fmix32 here cost `sk_count` 4.66 vs 4.28 ms and
// `usk_count` 2.97 vs 2.58 ms; any order is correct: a K-mer's minimizer is
// a function of the K-mer, so all its instances share a bucket).
__device__ __forceinline__ uint32_t mmer_order(uint64_t c) {
  return (((uint32_t)c ^ 0x2545f491u) * 0x9e3779b1u) ^ ((uint32_t)(c >> 32) * 0x85ebca6bu);
}
__device__ __forceinline__ uint32_t part_key(uint32_t v) { return sk_fmix32(v ^ 0x6b43a9b5u); }
// mmer_order of an m-mer with m <= 16 (c < 2^32: the high word's term is 0).
__device__ __forceinline__ uint32_t mmer_order32(uint32_t c) { return (c ^ 0x2545f491u) * 0x9e3779b1u; }

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
// 12-byte window overrun) fit BYTES, copied into LDS with one coalesced pass
// so the walk below never waits on HBM.  A read too long for a tile is
// walked from global memory on its own.
constexpr uint32_t kSkTileBytes = 8192;
template <int NT, uint32_t BYTES = kSkTileBytes>
struct SkTile {
  static constexpr uint32_t kBytes = BYTES;
  uint32_t words[BYTES / 4];
  uint32_t rlen[NT];
  uint32_t rbo[NT];  // byte offset of the read in `words`
  uint32_t lmax;     // longest read of the tile (block-uniform walk bound)
};

// Loads the tile starting at read t0 (< r1); returns its read count, or 0
// when read t0 alone exceeds a tile.  Block-uniform; ends with a barrier.
template <int NT, uint32_t BYTES>
__device__ __forceinline__ uint32_t sk_load_tile(const SkReads& rv, uint64_t t0, uint64_t r1, SkTile<NT, BYTES>& T) {
  const uint32_t tid = threadIdx.x;
  const uint64_t b0 = rv.byte_off[t0] & ~3ull;
  const uint64_t r = t0 + tid;
  bool fits = false;
  uint32_t len = 0;
  if (tid == 0) T.lmax = 0;
  if (r < r1) {
    len = (uint32_t)(rv.base_off[r + 1] - rv.base_off[r]);
    const uint64_t bo = rv.byte_off[r] - b0;
    fits = bo + (len + 3) / 4 + 12 <= BYTES;
    T.rlen[tid] = len;
    T.rbo[tid] = (uint32_t)bo;
  }
  const uint32_t n = (uint32_t)__syncthreads_count(fits);
  if (n) {
    if (tid < n) atomicMax(&T.lmax, len);
    const uint32_t nw = (T.rbo[n - 1] + (T.rlen[n - 1] + 3) / 4 + 12 + 3) / 4;
    const uint32_t* g = reinterpret_cast<const uint32_t*>(rv.packed + b0);
    for (uint32_t i = tid; i < nw; i += NT) T.words[i] = g[i];
  }
  __syncthreads();
  return n;
}

// Base accessors: the 16 bases [x, x+16) of a read as 32 bits, LSB-first —
// from an LDS tile (two aligned words and one v_alignbit) or from HBM.
template <uint32_t NWORDS>
struct SkLdsBases {
  const uint32_t* W;
  uint32_t bit0;  // the read's first bit in W
  __device__ __forceinline__ uint32_t at(uint32_t x) const {
    const uint32_t bo = bit0 + 2 * x;
    const uint32_t i = min(bo >> 5, NWORDS - 2);  // prefetches past the tile read stale words, never past W
    return __builtin_amdgcn_alignbit(W[i + 1], W[i], bo & 31);
  }
  // at(x) in two halves for x a multiple of 16 (bit offset bit0 mod 32): the
  // aligned words now, joined when needed, so a prefetch's LDS latency is
  // not waited on at the load
  __device__ __forceinline__ uint2 words(uint32_t x) const {
    const uint32_t i = min((bit0 + 2 * x) >> 5, NWORDS - 2);
    return make_uint2(W[i], W[i + 1]);
  }
  __device__ __forceinline__ uint32_t join(uint2 w) const { return __builtin_amdgcn_alignbit(w.y, w.x, bit0 & 31); }
};
struct SkGlobalBases {
  const uint8_t* rd;
  __device__ __forceinline__ uint32_t at(uint32_t x) const { return (uint32_t)sk_lsb64(rd, x); }
};

// The walk of one read: rolled base by base (fw / rc m-mer, m <= 16, order of
// the canonical one); the minimum of each window of w orders comes from the
// van Herk / Gil-Werman block scheme — orders are taken in blocks of w, the
// finished block is turned into suffix minima in this thread's LDS column
// (sb[t * NT], conflict-free), and window [i, i+w-1] = min(suffix of block
// k-1 from i, prefix of block k up to i+w-1) — so every lane does the same
// work per base with no rescans.  A record is a run of K-mers [a, a+n) that
// share minimizer order `key`, n <= maxnk.
//
// TWO (long windows, the K = 96 walk: w = 81): a two-level column.  The
// finished block keeps only its coarse suffix minima per segment of SB
// m-mers (CS); the segment the window's left edge is in gets its fine suffix
// minima recomputed from the read's bases when the edge enters it (FS: SB
// orders re-hashed once per SB steps); the current block keeps its running
// segment minima (SM) and prefix minimum.  Per thread 2 ceil(w/SB) + 1 + SB
// column words instead of w (31 for w = 81, SB = 8).
// Column layout at sb (stride NT): SM[0, NS) | CS[0, NS] | FS[0, SB).
// P: any parameter struct with K, m <= 16, w, maxnk, mmask (2m-bit mask).
constexpr int kSkSeg = 8;
__host__ __device__ constexpr int sk_walk2_words(int w) { return 2 * ((w + kSkSeg - 1) / kSkSeg) + 1 + kSkSeg; }

// U: the m-mer register type — uint32_t for m <= 16 (P::U), uint64_t up to 31.
template <typename U>
__device__ __forceinline__ uint32_t sk_order(U c) {
  if constexpr (sizeof(U) == 4)
    return mmer_order32(c);
  else
    return mmer_order(c);
}

template <int NT, bool TWO, typename B, typename U>
struct SkWalker {
  uint32_t w, m, maxnk, rsh, NS;
  U mmask;
  uint32_t* sb;
  B bases;
  U fw = 0, rc = 0;
  uint32_t pre = 0, t = 0, key = 0, ra = 0, rn = 0, segmin = 0, blk0 = 0;

  template <typename P>
  __device__ __forceinline__ SkWalker(const P& p, uint32_t* col, B b)
      : w((uint32_t)p.w), m((uint32_t)p.m), maxnk((uint32_t)p.maxnk), rsh(2 * (uint32_t)p.m - 2),
        NS(((uint32_t)p.w + kSkSeg - 1) / kSkSeg), mmask((U)p.mmask), sb(col), bases(b) {}

  // canonical order of the m-mer at base x, from the bases
  __device__ __forceinline__ uint32_t order_at(uint32_t x) const {
    if constexpr (sizeof(U) == 4) {
      const uint32_t Wm = bases.at(x);
      return mmer_order32(min(sk_rev2_32(Wm) >> (32 - 2 * m), ~Wm & mmask));
    } else {
      const uint64_t Wm = (uint64_t)bases.at(x) | ((uint64_t)bases.at(x + 16) << 32);
      const uint64_t f2 = sk_rev2(Wm) >> (64 - 2 * m), r2 = ~Wm & mmask;
      return mmer_order(f2 < r2 ? f2 : r2);
    }
  }

  // Base j (value b); true when a record closed: K-mers [oa, oa + on), key ok.
  __device__ __forceinline__ bool step(uint32_t j, uint32_t b, uint32_t& oa, uint32_t& on, uint32_t& ok) {
    fw = ((fw << 2) | (U)b) & mmask;
    rc = (rc >> 2) | ((U)(3 - b) << rsh);
    if (j + 1 < m) return false;
    const uint32_t v = sk_order<U>(fw < rc ? fw : rc);  // m-mer x = j + 1 - m, offset t in its block
    const uint32_t x = j + 1 - m;
    pre = t == 0 ? v : min(pre, v);
    uint32_t suf = 0xffffffffu;
    if constexpr (TWO) {
      uint32_t* SM = sb;
      uint32_t* CS = sb + NS * NT;
      uint32_t* FS = sb + (2 * NS + 1) * NT;
      segmin = (t % kSkSeg) == 0 ? v : min(segmin, v);
      if ((t % kSkSeg) == kSkSeg - 1 || t + 1 == w) SM[(t / kSkSeg) * NT] = segmin;
      const uint32_t u = t + 1;
      if (x + 1 >= w && u < w) {  // the previous block's suffix from u
        const uint32_t sg = u / kSkSeg, uo = u % kSkSeg;
        if (uo == 0 || t == 0) {  // the edge entered segment sg: its fine suffix minima, re-hashed
          const uint32_t lo = sg * kSkSeg, ne = min(lo + (uint32_t)kSkSeg, w) - lo;
          const uint32_t pb = blk0 - w + lo;  // base (= m-mer index) of the segment's first m-mer
          uint32_t r = 0xffffffffu;
          for (uint32_t e = ne; e-- > 0;) {
            r = min(r, order_at(pb + e));
            FS[e * NT] = r;
          }
        }
        suf = min(FS[uo * NT], CS[(sg + 1) * NT]);
      }
    } else {
      if (t + 1 < w) suf = sb[(t + 1) * NT];
      sb[t * NT] = v;
    }
    bool closed = false;
    if (x + 1 >= w) {  // K-mer i = x + 1 - w
      const uint32_t kk = min(suf, pre);
      if (x + 1 == w) {
        key = kk;
        ra = 0;
        rn = 1;
      } else if (kk == key && rn < maxnk) {
        ++rn;
      } else {
        oa = ra;
        on = rn;
        ok = key;
        closed = true;
        key = kk;
        ra = x + 1 - w;
        rn = 1;
      }
    }
    if (++t == w) {  // block done
      if constexpr (TWO) {  // its coarse suffix minima
        uint32_t* SM = sb;
        uint32_t* CS = sb + NS * NT;
        CS[NS * NT] = 0xffffffffu;
        for (int g = (int)NS - 1; g >= 0; --g) CS[g * NT] = min(SM[g * NT], CS[(g + 1) * NT]);
        blk0 += w;
      } else {  // suffix minima in place
        for (int u = (int)w - 2; u >= 0; --u) sb[u * NT] = min(sb[u * NT], sb[(u + 1) * NT]);
      }
      t = 0;
    }
    return closed;
  }
};

constexpr uint32_t kSkChunk = 16;  // bases per walk chunk (one prefetched word)

// A wave's record queue: a ring of CAPW descriptors in LDS.  Lanes whose
// record closed at this base append it (ballot + mbcnt); every few bases the
// wave hands the pending ones out 64 at a time — emission (the digit counts,
// the descriptor store) then runs on full waves, not once per base for the
// few lanes whose record closed there.  head / tail are wave-uniform; the
// caller drains often enough that fewer than CAPW are ever pending.
template <uint32_t CAPW>
struct SkWaveQ {
  uint64_t* q;
  uint32_t head = 0, tail = 0;
  __device__ __forceinline__ void push(bool c, uint64_t d) {
    const uint64_t m = __ballot(c);
    const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (c) q[(tail + r) & (CAPW - 1)] = d;
    tail += (uint32_t)__popcll(m);
  }
  template <typename E>
  __device__ __forceinline__ void drain(E emit) {  // every full wave's worth
    for (; tail - head >= 64; head += 64) emit(q[(head + __lane_id()) & (CAPW - 1)]);
  }
  template <typename E>
  __device__ __forceinline__ void flush(E emit) {
    drain(emit);
    if (__lane_id() < tail - head) emit(q[(head + __lane_id()) & (CAPW - 1)]);
    head = tail;
  }
};

// The walk with the van Herk column in registers, for a window length WN = w
// known at compile time: a block of w m-mers is one unrolled pass whose
// offset t is a constant, so the column col[t] is a register — no LDS column
// and, for long windows, no second-level re-hash (the two-level column
// hashes every m-mer twice; this walk hashes it once).  Records as SkWalker's
// over the read's Lw bases (Lw = 0: none; else Lw >= K), as descriptors
// key | a << 32 | n << 48 | q << 56 through the wave's queue `wq`
// (SkWaveQ<CAPW>, drained every S bases: 64 + 64 S <= CAPW) to emit(d).
// Lanes past their read run on with their records frozen; the block loop
// ends when no lane of the wave has m-mers left (the base accessor must
// tolerate reads past the read: SkLdsBases clamps to its tile).  Every lane
// of the wave calls it.  MM = p.m, also fixed at compile time (the rolls'
// shifts and mask constant).
template <int WN, int MM, int S, uint32_t CAPW, typename U, typename P, typename LB, typename E>
__device__ __forceinline__ void sk_walk_regs(const P& p, const LB& bases, uint32_t Lw, uint32_t q, uint64_t* wq,
                                             E emit) {
  static_assert(64 + 64 * S <= CAPW && (CAPW & (CAPW - 1)) == 0, "queue ring");
  static_assert(2 * MM <= 8 * (int)sizeof(U), "m-mer register");
  if (__ballot(Lw != 0) == 0) return;
  SkWaveQ<CAPW> Q{wq};
  const uint64_t qd = (uint64_t)q << 56;
  constexpr uint32_t m = MM, rsh = 2 * MM - 2;
  const uint32_t maxnk = (uint32_t)p.maxnk;
  constexpr U mmask = 2 * MM == 8 * sizeof(U) ? ~(U)0 : (((U)1 << (2 * MM)) - 1);
  const uint32_t nm = Lw ? Lw + 1 - m : 0;  // the read's m-mers
  uint32_t cur = bases.at(0), j = 0;
  uint2 nxt = bases.words(kSkChunk);
  U fw = 0, rc = 0;
  auto roll = [&]() {  // base j (wave-uniform: every lane is at the same base)
    if (j % kSkChunk == 0 && j) {
      cur = bases.join(nxt);
      nxt = bases.words(j + kSkChunk);
    }
    const uint32_t b = (cur >> (2 * (j % kSkChunk))) & 3u;
    fw = ((fw << 2) | (U)b) & mmask;
    rc = (rc >> 2) | ((U)(3u - b) << rsh);
    ++j;
  };
  auto desc = [&](uint32_t a, uint32_t n, uint32_t key) {
    return (uint64_t)key | ((uint64_t)a << 32) | ((uint64_t)n << 48) | qd;
  };
  while (j + 1 < m) roll();
  uint32_t col[WN], pre = 0;
#pragma unroll
  for (int t = 0; t < WN; ++t) {  // block 0: m-mers [0, w), the first K-mer at its end
    roll();
    const uint32_t v = sk_order<U>(fw < rc ? fw : rc);
    pre = t == 0 ? v : min(pre, v);
    col[t] = v;
  }
  uint32_t key = pre, ra = 0, rn = 1;
  for (uint32_t x0 = WN; __ballot(x0 < nm) != 0; x0 += WN) {
#pragma unroll
    for (int u = WN - 2; u >= 0; --u) col[u] = min(col[u], col[u + 1]);  // the finished block's suffix minima
#pragma unroll
    for (int t = 0; t < WN; ++t) {  // m-mer x0 + t closes K-mer x0 + t + 1 - w
      roll();
      const uint32_t v = sk_order<U>(fw < rc ? fw : rc);
      pre = t == 0 ? v : min(pre, v);
      const uint32_t kk = t + 1 < WN ? min(col[t + 1], pre) : pre;
      col[t] = v;  // the previous block's col[t] was read one step ago
      const bool live = x0 + t < nm;
      const bool closed = live && !(kk == key && rn < maxnk);
      const uint64_t d = desc(ra, rn, key);
      if (live) {
        rn = closed ? 1u : rn + 1;
        ra = closed ? x0 + t + 1 - WN : ra;
        key = kk;
      }
      Q.push(closed, d);
      if (t % S == S - 1 || t == WN - 1) Q.drain(emit);
    }
  }
  Q.push(Lw != 0, desc(ra, rn, key));
  Q.flush(emit);
}

// Record descriptors the count pass keeps so the scatter pass need not walk
// the reads again: block b's go to desc[lo(r0), lo(r1)), lo(r) = base_off[r]
// / div (the block's share of a bases / div budget), tile by tile, with each
// tile's count at tcnt[t0].  A block with more records than its region, or a
// record starting past base 65535 of a read, sets flag[b]: the scatter pass
// walks that block again.  Descriptor: key | a << 32 | n << 48 | q << 56.
struct SkDesc {
  uint64_t* desc;  // null: no descriptors (the scatter pass walks)
  uint32_t* tcnt;
  uint32_t* flag;
  uint32_t div;
  uint64_t slots;  // desc capacity: regions are clamped to it
  __device__ __forceinline__ uint64_t lo(const SkReads& rv, uint64_t r) const {
    const uint64_t x = rv.base_off[r] / div;
    return x < slots ? x : slots;
  }
};
__device__ __forceinline__ uint64_t sk_desc_pack(uint32_t key, uint32_t a, uint32_t n, uint32_t q) {
  return (uint64_t)key | ((uint64_t)a << 32) | ((uint64_t)n << 48) | ((uint64_t)q << 56);
}

// The count pass's side of the descriptors: per-block slot counter and
// overflow flag in LDS, a tile's count written by thread 0 between tiles.
struct SkDescWriter {
  const SkDesc& dd;
  uint64_t lo, cap;
  uint32_t* pos;   // LDS counter
  uint32_t* ovf;   // LDS flag
  uint32_t prev = 0;
  __device__ __forceinline__ SkDescWriter(const SkDesc& d, const SkReads& rv, uint64_t r0, uint64_t r1, uint32_t* p,
                                          uint32_t* o)
      : dd(d), lo(d.desc ? d.lo(rv, r0) : 0), cap(d.desc ? d.lo(rv, r1) - lo : 0), pos(p), ovf(o) {}
  __device__ __forceinline__ void put(uint32_t a, uint32_t n, uint32_t key, uint32_t q) {
    if (!dd.desc) return;
    const uint32_t i = atomicAdd(pos, 1u);
    if (i < cap && a <= 0xffffu)
      dd.desc[lo + i] = sk_desc_pack(key, a, n, q);
    else
      *ovf = 1;
  }
  // thread 0, after the barrier that ends tile t0 (all its records put)
  __device__ __forceinline__ void tile_done(uint64_t t0) {
    if (!dd.desc || threadIdx.x != 0) return;
    const uint32_t now = *pos;
    dd.tcnt[t0] = now - prev;
    prev = now;
  }
  __device__ __forceinline__ void block_done() {
    if (dd.desc && threadIdx.x == 0) dd.flag[blockIdx.x] = *ovf || *pos > cap;
  }
};

// The scatter pass's side: the block's tiles again (for their bases), each
// tile's descriptors handed to f lane-parallel, t0 = the tile's first read
// meanwhile (f may read it).  Returns false (nothing done) when the block
// must walk.  Block-uniform.
template <int NT, typename TT, typename F>
__device__ __forceinline__ bool sk_replay(const SkDesc& dd, const SkReads& rv, uint64_t r0, uint64_t r1, TT& T,
                                          uint64_t& t0, F f) {
  if (!dd.desc || dd.flag[blockIdx.x]) return false;
  uint64_t off = dd.lo(rv, r0);
  for (t0 = r0; t0 < r1;) {
    const uint32_t n = sk_load_tile(rv, t0, r1, T);
    const uint32_t c = dd.tcnt[t0];
    const uint8_t* g = rv.packed + rv.byte_off[t0];  // a read too long for a tile: from HBM
    for (uint32_t i = threadIdx.x; i < c; i += NT) {
      const uint64_t d = dd.desc[off + i];
      const uint32_t q = (uint32_t)(d >> 56);
      f(n ? reinterpret_cast<const uint8_t*>(T.words) + T.rbo[q] : g, T.rlen[q], (uint32_t)(d >> 32) & 0xffffu,
        (uint32_t)(d >> 48) & 0xffu, (uint32_t)d, q);
    }
    off += c;
    __syncthreads();
    t0 += n ? n : 1;
  }
  return true;
}

// A read too long for a tile: thread 0 walks it from HBM and hands each
// record straight to f(rd, L, a, n, key, q = 0).
template <int NT, bool TWO, typename P, typename TT, typename F>
__device__ __forceinline__ void sk_walk_global(const SkReads& rv, const P& p, const TT& T, uint64_t t0, uint32_t* sb,
                                               F f) {
  if (threadIdx.x != 0) return;
  const uint32_t L = T.rlen[0];
  if (L < (uint32_t)p.K) return;
  const uint8_t* rd = rv.packed + rv.byte_off[t0];
  SkWalker<NT, TWO, SkGlobalBases, typename P::U> W(p, sb, SkGlobalBases{rd});
  uint32_t word = 0, a, n, k;
  for (uint32_t j = 0; j < L; ++j) {
    if ((j & 15) == 0) word = W.bases.at(j);
    if (W.step(j, (word >> (2 * (j & 15))) & 3, a, n, k)) f(rd, L, a, n, k, 0u);
  }
  f(rd, L, W.ra, W.rn, W.key, 0u);
}

// Records of a tile, parked in LDS as they close and handed to f in
// lane-parallel passes (a record closes on a few lanes per base: called in
// place, f would run once per closing base with most of the wave idle).
// Descriptor: key | a << 32 | n << 48 | q << 56 (q = the read's lane).
template <int CAP>
struct SkList {
  uint32_t cnt;
  uint64_t d[CAP];
};
// LDS words the register walk's record queues take (sk_walk_tile, WN > 0):
// one SkWaveQ ring per wave at the start of the walk's dynamic LDS.
__host__ __device__ constexpr int sk_regq_drain(int WN) { return WN >= 32 ? 4 : 2; }
__host__ __device__ constexpr uint32_t sk_regq_capw(int WN) { return WN >= 32 ? 512u : 256u; }
__host__ __device__ constexpr uint32_t sk_regq_words(int NT, int WN) {
  return (uint32_t)(NT / 64) * sk_regq_capw(WN) * 2u;
}

// Every thread of the block walks the tile's read q = threadIdx.x (if any)
// in chunks of kSkChunk bases.  LIST: between chunks the block drains the
// list when it is half full (and after the last chunk) — for an f that is
// costly per call (building and storing a record); otherwise f runs in place
// (a pair of LDS atomics).  f(rd, L, a, n, key, q) per record, in no
// particular order.  Block-uniform.  WN > 0 (no LIST, WN == p.w, MM == p.m):
// the walk with the column in registers (sk_walk_regs).
template <int NT, bool TWO, bool LIST, int WN = 0, int MM = 0, typename P, typename TT, int CAP, typename F>
__device__ __forceinline__ void sk_walk_tile(const P& p, const TT& T, uint32_t n, uint32_t* sb, SkList<CAP>& lst,
                                             F f) {
  const uint32_t q = threadIdx.x;
  const uint32_t L = q < n ? T.rlen[q] : 0;
  const uint32_t Lw = L >= (uint32_t)p.K ? L : 0;  // bases this thread walks
  using LB = SkLdsBases<TT::kBytes / 4>;
  SkWalker<NT, TWO, LB, typename P::U> W(p, sb, LB{T.words, (q < n ? T.rbo[q] : 0u) * 8});
  auto emit = [&](uint64_t d) {
    const uint32_t r = (uint32_t)(d >> 56);
    f(reinterpret_cast<const uint8_t*>(T.words) + T.rbo[r], T.rlen[r], (uint32_t)(d >> 32) & 0xffffu,
      (uint32_t)(d >> 48) & 0xffu, (uint32_t)d, r);
  };
  auto push = [&](uint32_t a, uint32_t nk, uint32_t key) {
    const uint64_t d = (uint64_t)key | ((uint64_t)a << 32) | ((uint64_t)nk << 48) | ((uint64_t)q << 56);
    if constexpr (!LIST) {
      emit(d);
      return;
    }
    const uint32_t i = atomicAdd(&lst.cnt, 1u);
    if (i < (uint32_t)CAP)
      lst.d[i] = d;
    else
      emit(d);  // list full: this record alone, in place
  };
  if constexpr (!LIST && WN > 0) {  // the waves' queues: sk_regq_words(NT, WN) words from sb - q
    constexpr int S = sk_regq_drain(WN);
    constexpr uint32_t CAPW = sk_regq_capw(WN);
    uint64_t* wq = reinterpret_cast<uint64_t*>(sb - q) + (q / 64) * CAPW;
    sk_walk_regs<WN, MM, S, CAPW, typename P::U>(p, W.bases, Lw, q, wq, emit);
    return;
  }
  if constexpr (!LIST) {  // no barriers: each lane walks its own read to its end
    uint32_t cur = Lw ? W.bases.at(0) : 0, nxt = Lw > kSkChunk ? W.bases.at(kSkChunk) : 0;
    uint32_t a, nk, k;
#pragma unroll 4  // loop control and uniform-branch SALU per base: 7.0 -> 6.45 ms sk_count (8: same)
    for (uint32_t j = 0; j < Lw; ++j) {
      if ((j % kSkChunk) == 0 && j) {
        cur = nxt;
        if (j + kSkChunk < Lw) nxt = W.bases.at(j + kSkChunk);
      }
      if (W.step(j, (cur >> (2 * (j % kSkChunk))) & 3, a, nk, k)) push(a, nk, k);
    }
    if (Lw) push(W.ra, W.rn, W.key);
    return;
  }
  const uint32_t Lmax = T.lmax;
  uint32_t nxt = Lw ? W.bases.at(0) : 0;
  for (uint32_t c0 = 0; c0 < Lmax; c0 += kSkChunk) {
    const uint32_t cur = nxt;
    if (c0 + kSkChunk < Lw) nxt = W.bases.at(c0 + kSkChunk);  // in flight during this chunk
    const uint32_t c1 = min(c0 + kSkChunk, Lw);
    uint32_t a, nk, k;
    for (uint32_t j = c0; j < c1; ++j)
      if (W.step(j, (cur >> (2 * (j - c0))) & 3, a, nk, k)) push(a, nk, k);
    if (c0 < Lw && Lw <= c0 + kSkChunk) push(W.ra, W.rn, W.key);  // the read's last record
    __syncthreads();
    const bool last = c0 + kSkChunk >= Lmax;
    if (__syncthreads_count(q == 0 && lst.cnt >= (uint32_t)CAP / 2) || last) {
      const uint32_t m = min(lst.cnt, (uint32_t)CAP);
      for (uint32_t i = q; i < m; i += NT) emit(lst.d[i]);
      __syncthreads();
      if (q == 0) lst.cnt = 0;
      __syncthreads();
    }
  }
}

}  // namespace apg
