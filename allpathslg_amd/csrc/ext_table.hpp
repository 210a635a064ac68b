// ext_table.hpp — the (K-1)-mer extension table of a solid K-mer set, shared
// by PreCorrect (precorrect.hip) and FillFragments (fill.hip).
//
// One 8-byte slot per canonical (K-1)-mer: key << 8 | 4 left + 4 right
// extension bits (2 <= K <= 29).  Every solid K-mer x inserts its first K-1
// bases with x's last base as a successor and its last K-1 bases with x's
// first base as a predecessor, so
//   K-mer [i, i+K) of a read is solid  <=>  succ((K-1)-mer i) holds b[i+K-1]
//                                      <=>  pred((K-1)-mer i+1) holds b[i].
// One lookup therefore answers two adjacent K-mers of a read (pred and succ of
// the (K-1)-mer between them) or all 4 successors of a walk node, where a hash
// set of K-mers needs one lookup per K-mer.  Linear probing, load <= 0.25
// (table = 4 slots per solid K-mer): nearly every lookup is one 64-byte line.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "apg_core.hpp"
#include "kmer_common.hpp"

namespace apg {

constexpr uint64_t kExtEmpty = ~0ull;

__device__ __forceinline__ uint64_t f_rev2(uint64_t x) {
  x = __builtin_bitreverse64(x);
  return ((x >> 1) & 0x5555555555555555ull) | ((x & 0x5555555555555555ull) << 1);
}

// reverse complement of an n-base MSB-first value (1 <= n <= 32)
__host__ __device__ __forceinline__ uint64_t rc_bases(uint64_t w, int n, uint64_t mask) {
#ifdef __HIP_DEVICE_COMPILE__
  return (f_rev2(w) >> (64 - 2 * n)) ^ mask;
#else
  uint64_t r = 0;
  for (int i = 0; i < n; ++i) {
    r = (r << 2) | (3 - (w & 3));
    w >>= 2;
  }
  return r & mask;
#endif
}

__device__ __forceinline__ uint32_t rev4(uint32_t x) {
  return ((x & 1) << 3) | ((x & 2) << 1) | ((x & 4) >> 1) | ((x & 8) >> 3);
}

struct ExtTab {
  unsigned long long* slot;
  uint64_t mask;
  HashP h1;  // slot hash of canonical (K-1)-mers
  uint64_t m1;
  int n1;  // K-1
};

// Probing starts at the first slot of the key's aligned group of kExtGrp
// slots (32 bytes) and runs linearly from there, so a lookup reads the group
// at once (two 16-byte loads in flight together) and almost always finds the
// key, or the empty slot that proves it absent, in it: one memory round trip
// per lookup, where slot-by-slot probing paid a second one for every key not
// in its home slot — and a wave waits for its slowest lane.
constexpr uint64_t kExtGrp = 4;
__device__ __forceinline__ uint64_t ext_home(const ExtTab& t, uint64_t c) {
  return khash(t.h1, c) & t.mask & ~(kExtGrp - 1);
}

// The 8 extension bits of canonical (K-1)-mer c (0 if absent).
__device__ __forceinline__ uint32_t ext_bits(const ExtTab& t, uint64_t c) {
  uint64_t g = ext_home(t, c);
  for (;;) {
    const ulonglong2* q = reinterpret_cast<const ulonglong2*>(t.slot + g);
    const ulonglong2 a = q[0], b = q[1];
    const unsigned long long v[kExtGrp] = {a.x, a.y, b.x, b.y};
#pragma unroll
    for (uint32_t j = 0; j < kExtGrp; ++j) {
      if (v[j] == kExtEmpty) return 0;
      if ((v[j] >> 8) == c) return (uint32_t)(v[j] & 0xff);
    }
    g = (g + kExtGrp) & t.mask;
  }
}

// 4-bit successor mask of the (K-1)-mer w (MSB-first, fw orientation)
__device__ __forceinline__ uint32_t ext_succ(const ExtTab& t, uint64_t w, uint32_t* nlook) {
  const uint64_t r = rc_bases(w, t.n1, t.m1);
  const uint32_t e = ext_bits(t, w < r ? w : r);
  ++*nlook;
  uint32_t m = 0;
  if (w <= r) m |= e >> 4;
  if (r <= w) m |= rev4(e & 15);
  return m;
}

// Predecessor (bits 0-3) and successor (bits 4-7) masks, in read
// orientation, of the (K-1)-mer whose bases are the LSB-first value y (base
// t of the (K-1)-mer at bits 2t, 2t+1).  The LSB-first value complemented is
// the MSB-first value of the reverse complement.
__device__ __forceinline__ uint32_t ext_masks_lsb(const ExtTab& t, uint64_t y) {
  const uint64_t fw = f_rev2(y) >> (64 - 2 * t.n1);
  const uint64_t rc = y ^ t.m1;
  const uint32_t e = ext_bits(t, fw < rc ? fw : rc);
  uint32_t m = 0;
  if (fw <= rc) m |= e;
  if (rc <= fw) m |= rev4(e >> 4) | (rev4(e & 15) << 4);
  return m;
}

// Build the extension table of a solid list (khash(K) of canonical K-mers) in
// workspace `ws` (2 <= K <= 29); asynchronous on ctx->stream.
int ext_build(apg_ctx* ctx, const uint64_t* list, uint64_t n_solid, int K, const char* ws, const char* kname,
              ExtTab* out);
}  // namespace apg
