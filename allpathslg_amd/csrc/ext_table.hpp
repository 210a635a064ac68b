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
  int n1;    // K-1
  int mz;    // 0, or 16: minimizer homes (APG_EXT_MZ=1; K-1 >= 17), see ext_mz_home
};

// Minimizer homes (mz = 16).  A walk step, a read's next (K-1)-mer or an
// alternative's covering (K-1)-mers mostly share their canonical 16-mer
// minimizer with the previous lookup (77 % of the gap walk's consecutive
// lookups, tools/fill_walk_model.c), so a (K-1)-mer's home is an 8-slot line
// chosen by its minimizer: consecutive lookups then read the same line,
// which the previous one left in L2.  A minimizer class the build counted
// as large (kMzBig instances: repeats) keeps its (K-1)-mers at their own
// hash homes and leaves a marker — a slot with no extension bits holding the
// minimizer — in its line; a lookup that meets the marker before an empty
// slot looks the (K-1)-mer up at its own home.  Real entries always carry an
// extension bit.  Order of 16-mers: the canonical value XOR a constant.
constexpr uint32_t kMzXor = 0x5bd1e995u;
constexpr uint64_t kMzLine = 8;
constexpr uint32_t kMzBig = 16;  // class instances (each (K-1)-mer counted about twice)
__host__ __device__ __forceinline__ uint64_t ext_mix(uint64_t z) {
  z = (z ^ (z >> 31)) * 0x7fb5d329728ea185ull;
  z = (z ^ (z >> 27)) * 0x81dadef4bc2dd44dull;
  return z ^ (z >> 33);
}
// canonical (K-1)-mer c and its reverse complement r (MSB-first, n1 bases)
__device__ __forceinline__ uint32_t ext_minimizer(const ExtTab& t, uint64_t c, uint64_t r) {
  uint32_t best = 0xffffffffu;
  const int last = t.n1 - 16;
  for (int i = 0; i <= last; ++i) {
    const uint32_t f = (uint32_t)(c >> (2 * (last - i))), b = (uint32_t)(r >> (2 * i));
    best = min(best, min(f, b) ^ kMzXor);
  }
  return best ^ kMzXor;
}
__device__ __forceinline__ uint64_t ext_mz_home(const ExtTab& t, uint32_t mzv) {
  return ext_mix(mzv) & t.mask & ~(kMzLine - 1);
}

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

// The 8 extension bits of canonical (K-1)-mer c (0 if absent), at its own
// hash home.
__device__ __forceinline__ uint32_t ext_bits_hash(const ExtTab& t, uint64_t c) {
  uint64_t g = ext_home(t, c);
  for (;;) {
    const ulonglong2* q = reinterpret_cast<const ulonglong2*>(t.slot + g);
    const ulonglong2 a = q[0], b = q[1];
    const unsigned long long v[kExtGrp] = {a.x, a.y, b.x, b.y};
#pragma unroll
    for (uint32_t j = 0; j < kExtGrp; ++j) {
      if (v[j] == kExtEmpty) return 0;
      if ((v[j] >> 8) == c && (v[j] & 0xff)) return (uint32_t)(v[j] & 0xff);  // (not a minimizer marker)
    }
    g = (g + kExtGrp) & t.mask;
  }
}

// ... or (MZ: the table has minimizer homes, t.mz) from its minimizer's
// line; r = its reverse complement.  MZ is a template parameter so that the
// kernels built without it keep their register budget.
template <bool MZ = false>
__device__ __forceinline__ uint32_t ext_bits(const ExtTab& t, uint64_t c, uint64_t r) {
  if (!MZ) return ext_bits_hash(t, c);
  const uint32_t mzv = ext_minimizer(t, c, r);
  uint64_t g = ext_mz_home(t, mzv);
  for (;;) {  // the line group by group (two 16-byte loads each: fewer live registers than the whole line)
    const ulonglong2* q = reinterpret_cast<const ulonglong2*>(t.slot + g);
    const ulonglong2 a = q[0], b = q[1];
    const unsigned long long v[kExtGrp] = {a.x, a.y, b.x, b.y};
#pragma unroll
    for (uint32_t j = 0; j < kExtGrp; ++j) {
      if (v[j] == kExtEmpty) return 0;
      const uint32_t bits = (uint32_t)(v[j] & 0xff);
      if ((v[j] >> 8) == (bits ? c : (uint64_t)mzv)) return bits ? bits : ext_bits_hash(t, c);
    }
    g = (g + kExtGrp) & t.mask;
  }
}

// 4-bit successor mask of the (K-1)-mer w (MSB-first, fw orientation)
template <bool MZ = false>
__device__ __forceinline__ uint32_t ext_succ(const ExtTab& t, uint64_t w, uint32_t* nlook) {
  const uint64_t r = rc_bases(w, t.n1, t.m1);
  const uint32_t e = w < r ? ext_bits<MZ>(t, w, r) : ext_bits<MZ>(t, r, w);
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
template <bool MZ = false>
__device__ __forceinline__ uint32_t ext_masks_lsb(const ExtTab& t, uint64_t y) {
  const uint64_t fw = f_rev2(y) >> (64 - 2 * t.n1);
  const uint64_t rc = y ^ t.m1;
  const uint32_t e = fw < rc ? ext_bits<MZ>(t, fw, rc) : ext_bits<MZ>(t, rc, fw);
  uint32_t m = 0;
  if (fw <= rc) m |= e;
  if (rc <= fw) m |= rev4(e >> 4) | (rev4(e & 15) << 4);
  return m;
}

// Build the extension table of a solid list (khash(K) of canonical K-mers) in
// workspace `ws` (2 <= K <= 29); asynchronous on ctx->stream.
int ext_build(apg_ctx* ctx, const uint64_t* list, uint64_t n_solid, int K, const char* ws, const char* kname,
              ExtTab* out);
// The table the context's last correction pass built (pc_ext_*), for reuse.
ExtTab ext_last(apg_ctx* ctx, int K);
}  // namespace apg
