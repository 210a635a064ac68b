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
//
// Two-level slots (K <= 25, the default; APG_EXT_TWO=0 for the one-level
// layout): key << 16 | pp << 12 | ss << 8 | succ << 4 | pred, where ss is the
// successor mask of the (K-1)-mer's successor when it has exactly one, and pp
// the predecessor mask of its predecessor when it has exactly one (a link pass
// after the inserts, k_ext_link).  A walk through a non-branching (K-1)-mer
// learns its next node's successors with it, so along a path every other node
// needs no lookup of its own (tools/fill_walk_model.c: 43 % fewer FillFragments
// lookups on the repeat-rich genome).
#pragma once

#include <cstdlib>
#include <cstring>

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
  int ks;  // key shift: 16 with the two-level bits, 8 without
  int hs;  // home hash: 64 - log2(slots) for the multiplicative one, 0 for khash(h1)
};

// The slot layout for K (the builder and every reuse of a built table agree).
inline bool ext_two_level(int K) {
  static const bool on = [] {
    const char* e = getenv("APG_EXT_TWO");
    return !(e && !strcmp(e, "0"));
  }();
  return on && 2 * (K - 1) + 16 <= 64;
}
// Homes by a xorshift + one 64-bit multiply whose top bits index the table
// (a third of the instructions of khash's two multiply rounds; APG_EXT_HASH=0
// for khash).  Round 4, same box: main step 144.3 / 145.0 vs 144.1 ms with
// khash (fill -0.2 ms, inserts +0.5, decisions +0.4), repeat-rich step 187.2
// vs 189.6 ms; round 5, same box: main 142.3 vs 142.4 ms, repeat-rich 181.0
// vs 181.9 ms (fill 38.4 vs 39.6 ms) — the default since.
inline ExtTab ext_tab(unsigned long long* slot, uint64_t mask, int K) {
  static const bool mul = [] {
    const char* e = getenv("APG_EXT_HASH");
    return !(e && !strcmp(e, "0"));
  }();
  return ExtTab{slot, mask, make_hashp(K - 1), (1ull << (2 * (K - 1))) - 1, K - 1, ext_two_level(K) ? 16 : 8,
                mul ? 64 - __builtin_popcountll(mask) : 0};
}

// Probing starts at the first slot of the key's aligned group of kExtGrp
// slots (32 bytes) and runs linearly from there, so a lookup reads the group
// at once (two 16-byte loads in flight together) and almost always finds the
// key, or the empty slot that proves it absent, in it: one memory round trip
// per lookup, where slot-by-slot probing paid a second one for every key not
// in its home slot — and a wave waits for its slowest lane.
constexpr uint64_t kExtGrp = 4;
// HM: 1 when the caller knows the table uses the multiplicative home (t.hs
// != 0), so no khash constants are held for the other form
template <int HM = 0>
__device__ __forceinline__ uint64_t ext_home(const ExtTab& t, uint64_t c) {
  if (HM || t.hs) return (((c ^ (c >> 29)) * 0x9e3779b97f4a7c15ull) >> t.hs) & ~(kExtGrp - 1);
  return khash(t.h1, c) & t.mask & ~(kExtGrp - 1);
}

// The extension bits of canonical (K-1)-mer c (0 if absent): pred | succ << 4,
// and with two-level slots ss << 8 | pp << 12.  KS: the key shift when the
// caller knows it at compile time (0: t.ks).
template <int KS = 0, int HM = 0>
__device__ __forceinline__ uint32_t ext_bits(const ExtTab& t, uint64_t c) {
  const int ks = KS ? KS : t.ks;
  uint64_t g = ext_home<HM>(t, c);
  for (;;) {
    const ulonglong2* q = reinterpret_cast<const ulonglong2*>(t.slot + g);
    const ulonglong2 a = q[0], b = q[1];
    const unsigned long long v[kExtGrp] = {a.x, a.y, b.x, b.y};
#pragma unroll
    for (uint32_t j = 0; j < kExtGrp; ++j) {
      if (v[j] == kExtEmpty) return 0;
      if ((v[j] >> ks) == c) return (uint32_t)(v[j] & ((1u << ks) - 1));
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
  if (w <= r) m |= (e >> 4) & 15;
  if (r <= w) m |= rev4(e & 15);
  return m;
}

// ext_succ | ss << 4 | 256 when ss is known: w has exactly one successor
// and the table is two-level (palindromes excepted: their two orientations
// share one slot).
template <int KS = 0, int HM = 0>
__device__ __forceinline__ uint32_t ext_succ2(const ExtTab& t, uint64_t w, uint32_t* nlook) {
  const uint64_t r = rc_bases(w, t.n1, t.m1);
  const uint32_t e = ext_bits<KS, HM>(t, w < r ? w : r);
  ++*nlook;
  uint32_t m = 0, x = 0;
  if (w <= r) m |= (e >> 4) & 15, x = (e >> 8) & 15;
  if (r <= w) m |= rev4(e & 15), x = rev4((e >> 12) & 15);
  const bool ok = (KS ? KS : t.ks) == 16 && w != r && __popc(m) == 1;
  return m | (ok ? (x << 4) | 256u : 0u);
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
  if (fw <= rc) m |= e & 0xff;
  if (rc <= fw) m |= rev4((e >> 4) & 15) | (rev4(e & 15) << 4);
  return m;
}

// ext_masks_lsb | ss << 8 | pp << 12 in read orientation, bit 16 when ss is
// known (exactly one successor), bit 17 when pp is (exactly one predecessor).
__device__ __forceinline__ uint32_t ext_masks2_lsb(const ExtTab& t, uint64_t y) {
  const uint64_t fw = f_rev2(y) >> (64 - 2 * t.n1);
  const uint64_t rc = y ^ t.m1;
  const uint32_t e = ext_bits(t, fw < rc ? fw : rc);
  // A palindromic (K-1)-mer (fw == rc) shares one slot between its two
  // orientations: an insert records a K-mer around it as a succ bit or as a
  // pred bit depending on which orientation is canonical, so both readings
  // are OR'ed (ext_masks_lsb's rule); its two-level bits are never known.
  if (fw == rc) return (e & 0xff) | rev4((e >> 4) & 15) | (rev4(e & 15) << 4);
  uint32_t m = e;
  if (rc < fw) m = rev4((e >> 4) & 15) | (rev4(e & 15) << 4) | (rev4((e >> 12) & 15) << 8) | (rev4((e >> 8) & 15) << 12);
  if (t.ks != 16) return m & 0xff;
  return m | (__popc((m >> 4) & 15) == 1 ? 1u << 16 : 0u) | (__popc(m & 15) == 1 ? 1u << 17 : 0u);
}

// A lookup split in two, so that a lane can have several in flight: issue
// reads the home group of an LSB-first (K-1)-mer (ext_masks_lsb's argument),
// finish scans it (and probes on in the rare case the group holds neither
// the key nor an empty slot) and returns ext_masks_lsb's value.  Independent
// lookups issued together cost about one round trip, not one each.
struct ExtProbe {
  uint64_t c, g;
  ulonglong2 a, b;
  bool fw, rc;  // the (K-1)-mer is its own canonical form / its reverse complement is
};
__device__ __forceinline__ ExtProbe ext_issue_lsb(const ExtTab& t, uint64_t y) {
  ExtProbe p;
  const uint64_t fw = f_rev2(y) >> (64 - 2 * t.n1);
  const uint64_t rc = y ^ t.m1;
  p.fw = fw <= rc;
  p.rc = rc <= fw;
  p.c = fw < rc ? fw : rc;
  p.g = ext_home(t, p.c);
  const ulonglong2* q = reinterpret_cast<const ulonglong2*>(t.slot + p.g);
  p.a = q[0];
  p.b = q[1];
  return p;
}
__device__ __forceinline__ uint32_t ext_finish(const ExtTab& t, const ExtProbe& p) {
  uint32_t e = 0;
  const unsigned long long v[kExtGrp] = {p.a.x, p.a.y, p.b.x, p.b.y};
  bool done = false;
#pragma unroll
  for (uint32_t j = 0; j < kExtGrp; ++j) {
    if (done) continue;
    if (v[j] == kExtEmpty) {
      done = true;
    } else if ((v[j] >> t.ks) == p.c) {
      e = (uint32_t)(v[j] & 0xff);
      done = true;
    }
  }
  if (!done) {  // the group is full of other keys: on from the next group
    uint64_t g = (p.g + kExtGrp) & t.mask;
    for (;;) {
      const ulonglong2* q = reinterpret_cast<const ulonglong2*>(t.slot + g);
      const ulonglong2 a = q[0], b = q[1];
      const unsigned long long w[kExtGrp] = {a.x, a.y, b.x, b.y};
      bool hit = false;
#pragma unroll
      for (uint32_t j = 0; j < kExtGrp; ++j) {
        if (hit) continue;
        if (w[j] == kExtEmpty) {
          hit = true;
        } else if ((w[j] >> t.ks) == p.c) {
          e = (uint32_t)(w[j] & 0xff);
          hit = true;
        }
      }
      if (hit) break;
      g = (g + kExtGrp) & t.mask;
    }
  }
  uint32_t m = 0;
  if (p.fw) m |= e;
  if (p.rc) m |= rev4(e >> 4) | (rev4(e & 15) << 4);
  return m;
}

// Build the extension table of a solid list (khash(K) of canonical K-mers) in
// workspace `ws` (2 <= K <= 29); asynchronous on ctx->stream.  link = false
// leaves the two-level bits to a later ext_link (readers of the pred / succ
// bits alone may run beside that pass: it writes only bits 8-15).
int ext_build(apg_ctx* ctx, const uint64_t* list, uint64_t n_solid, int K, const char* ws, const char* kname,
              ExtTab* out, bool link = true);
// frac: of ext_link's usual grid (a trickle beside other work)
int ext_link(apg_ctx* ctx, const ExtTab& t, uint64_t n_solid, double frac = 1.0);
}  // namespace apg
