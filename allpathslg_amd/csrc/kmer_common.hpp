// kmer_common.hpp — device/host helpers shared by the k-mer kernels.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace apg {

// Table-order hash of SURVEY §A.3 (see apg.h): splitmix64's finaliser with
// shifts scaled to w = 2K bits and multipliers masked to w bits — a bijection
// on w bits.  Restated independently in oracle/kmer_oracle.c (ork_hash).
struct HashP {
  uint64_t mask, c1, c2;
  int s1, s2, s3, w;
};

__host__ __device__ inline int hash_shift(int w, int num) {
  int s = (w * num) / 64;
  return s < 1 ? 1 : s;
}

__host__ __device__ inline HashP make_hashp(int K) {
  HashP p;
  p.w = 2 * K;
  p.mask = p.w >= 64 ? ~0ull : ((1ull << p.w) - 1);
  p.c1 = (0xbf58476d1ce4e5b9ull & p.mask) | 1;
  p.c2 = (0x94d049bb133111ebull & p.mask) | 1;
  p.s1 = hash_shift(p.w, 30);
  p.s2 = hash_shift(p.w, 27);
  p.s3 = hash_shift(p.w, 31);
  return p;
}

__host__ __device__ inline uint64_t khash(const HashP& p, uint64_t x) {
  x &= p.mask;
  x ^= x >> p.s1;
  x = (x * p.c1) & p.mask;
  x ^= x >> p.s2;
  x = (x * p.c2) & p.mask;
  x ^= x >> p.s3;
  return x;
}

__host__ __device__ inline uint64_t inv_xorshift(uint64_t y, int s, int w, uint64_t mask) {
  uint64_t x = y;
  for (int i = 0; i * s < w; ++i) x = y ^ (x >> s);
  return x & mask;
}

__host__ __device__ inline uint64_t inv_odd(uint64_t c) {
  uint64_t v = c;
  for (int i = 0; i < 5; ++i) v *= 2 - c * v;
  return v;
}

__host__ __device__ inline uint64_t kunhash(const HashP& p, uint64_t h) {
  uint64_t x = h & p.mask;
  x = inv_xorshift(x, p.s3, p.w, p.mask);
  x = (x * inv_odd(p.c2)) & p.mask;
  x = inv_xorshift(x, p.s2, p.w, p.mask);
  x = (x * inv_odd(p.c1)) & p.mask;
  x = inv_xorshift(x, p.s1, p.w, p.mask);
  return x;
}

// Call f(hash) for every canonical K-mer (K <= 32) of one 2-bit packed read, in
// read order.  fw = sum b[i+j] 4^(K-1-j); rc = the same on the reverse
// complement; canonical = min(fw, rc)  (SURVEY §A.3).
template <typename F>
__device__ __forceinline__ void for_each_kmer_hash(const uint8_t* __restrict__ read, uint32_t len, int K,
                                                   const HashP& hp, F&& f) {
  uint64_t fw = 0, rc = 0;
  const int rsh = 2 * K - 2;
  uint32_t byte = 0;
  for (uint32_t i = 0; i < len; ++i) {
    if ((i & 3) == 0) byte = read[i >> 2];
    const uint64_t b = (byte >> (2 * (i & 3))) & 3;
    fw = ((fw << 2) | b) & hp.mask;
    rc = (rc >> 2) | ((3 - b) << rsh);
    if (i + 1 >= (uint32_t)K) f(khash(hp, fw < rc ? fw : rc));
  }
}

// Incremental form of for_each_kmer_hash: a thread's rolling state over one
// read, so k-mers can be produced a few at a time (staged scatter rounds).
struct KmerRoller {
  const uint8_t* read;
  uint32_t len, i, byte;
  uint64_t fw, rc;
  int K;

  __device__ __forceinline__ void init(const uint8_t* r, uint32_t n, int k, const HashP& hp) {
    read = r;
    len = n;
    K = k;
    i = 0;
    byte = 0;
    fw = rc = 0;
    const uint32_t prime = n < (uint32_t)(k - 1) ? n : (uint32_t)(k - 1);
    for (uint32_t j = 0; j < prime; ++j) roll(hp);
  }
  __device__ __forceinline__ void roll(const HashP& hp) {
    if ((i & 3) == 0) byte = read[i >> 2];
    const uint64_t b = (byte >> (2 * (i & 3))) & 3;
    fw = ((fw << 2) | b) & hp.mask;
    rc = (rc >> 2) | ((3 - b) << (2 * K - 2));
    ++i;
  }
  __device__ __forceinline__ bool more() const { return i < len; }
  // Next k-mer hash (call only when more()).
  __device__ __forceinline__ uint64_t next(const HashP& hp) {
    roll(hp);
    return khash(hp, fw < rc ? fw : rc);
  }
};

// ---- wave / block primitives (wave64) -------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ int wave_id() { return threadIdx.x >> 6; }
// LDS hand-off between the lanes of ONE wave (no block barrier): LDS serves a
// wave's operations in order, so this only has to stop the compiler from
// moving LDS accesses across it.
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1; }

// Lanes of this wave holding the same nb-bit digit (a 64-wide match_any built
// from nb ballots).  Invalid lanes match nobody and get 0.
__device__ __forceinline__ uint64_t wave_match(uint32_t d, bool valid, int nb) {
  uint64_t peers = __ballot(valid);
  for (int bit = 0; bit < nb; ++bit) {
    const bool set = (d >> bit) & 1;
    const uint64_t bal = __ballot(set);
    peers &= set ? bal : ~bal;
  }
  return valid ? peers : 0;
}

// Wave-aggregated append: every active lane calls it (converged); lanes with
// pred get consecutive slots from ONE atomicAdd per wave on *ctr.  Returns
// the lane's slot (meaningless where !pred).
__device__ __forceinline__ unsigned long long wave_append(unsigned long long* ctr, bool pred,
                                                          unsigned long long amount = 1) {
  const uint64_t m = __ballot(pred);
  if (m == 0) return 0;
  const int leader = __ffsll((long long)m) - 1;
  unsigned long long base = 0;
  if (lane_id() == leader) base = atomicAdd(ctr, (unsigned long long)__popcll(m) * amount);
  base = __shfl(base, leader, 64);
  return base + (unsigned long long)__popcll(m & lanemask_lt()) * amount;
}

template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* smem, T* total);

// Block-aggregated append: every thread of the block calls it with its count
// of items to append; ONE atomicAdd per block call reserves the block's
// slots (same-address atomics serialise chip-wide, so per-wave appends over
// hundreds of millions of items are contention-bound).  sm: >= 32 u32 of LDS
// scan scratch; sbase: one LDS u64.  Returns the thread's first slot.
__device__ __forceinline__ unsigned long long block_append(unsigned long long* ctr, uint32_t count, uint32_t* sm,
                                                           unsigned long long* sbase) {
  uint32_t tot;
  const uint32_t ex = block_exclusive_scan<uint32_t>(count, sm, &tot);
  if (threadIdx.x == 0) *sbase = tot ? atomicAdd(ctr, (unsigned long long)tot) : 0ull;
  __syncthreads();
  const unsigned long long b = *sbase + ex;
  __syncthreads();
  return b;
}

// Wave-aggregated add of per-lane values: one atomic per wave.
__device__ __forceinline__ void wave_add(unsigned long long* ctr, unsigned long long v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_down(v, o, 64);
  if (lane_id() == 0 && v) atomicAdd(ctr, v);
}

template <typename T>
__device__ __forceinline__ T wave_inclusive_scan(T x) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

// 32-bit inclusive wave scan on DPP lane moves (no LDS round trips): a
// Kogge-Stone scan inside each 16-lane row (row_shr 1, 2, 4, 8), then row
// 15's total broadcast into rows 1 and 3 and row 31's into rows 2 and 3
// (GFX9 row_bcast, which gfx950 keeps).  Lanes with no source add 0.
template <>
__device__ __forceinline__ uint32_t wave_inclusive_scan<uint32_t>(uint32_t x) {
  int v = (int)x;
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);  // row_shr:1
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);  // row_shr:2
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return (uint32_t)v;
}

// Exclusive scan across the block (blockDim.x <= 1024, multiple of 64).
// smem must hold >= 32 T.  Every thread must call; returns the exclusive
// prefix and writes the block total to *total.  Ends with a barrier.
template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* smem, T* total) {
  const int lane = lane_id(), wave = wave_id(), nw = blockDim.x >> 6;
  T x = wave_inclusive_scan(v);
  if (lane == 63) smem[wave] = x;
  __syncthreads();
  if (wave == 0) {
    T s = lane < nw ? smem[lane] : T(0);
    s = wave_inclusive_scan(s);
    if (lane < 16) smem[16 + lane] = s;
  }
  __syncthreads();
  const T base = wave > 0 ? smem[16 + wave - 1] : T(0);
  *total = smem[16 + nw - 1];
  __syncthreads();
  return base + x - v;
}

}  // namespace apg
