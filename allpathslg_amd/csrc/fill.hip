// fill.hip — FillFragments on MI355X: close each frag pair (A, B) into the
// fragment it was read from, through the solid K-mer graph.  Spec: the
// closure rule and search order pinned in include/apg.h (apg_fill_fragments);
// CPU restatement oracle/fill_oracle.c (recalled reference: [R:M]
// src/paths/FillFragments.cc, grep target only — snapshot empty).
//
//   1. k_fill_ext_insert: the solid K-mer set (hashes of canonical K-mers) is
//      turned into a (K-1)-mer extension table: one 8-byte slot per canonical
//      (K-1)-mer = key << 8 | 4 left + 4 right extension bits (K <= 25:
//      key << 16 with the two-level bits that k_ext_link adds, ext_table.hpp).
//      K-mer x is solid  <=>  the slot of x's first K-1 bases holds x's last
//      base as a successor.  One lookup therefore answers all 4 successors of
//      a walk node, where a hash set of K-mers would need 4 — and with the
//      two-level bits, the next node's successors too when the node has one.
//   2. k_fill: one thread per pair.  Overlap closures (I < La+Lf) by 32-base
//      word compares of A's suffix with F = rc(B)'s prefix, bridge K-mers by
//      extension lookups; then the depth-first walk from A's last K-1 bases,
//      entirely in registers: the path is a 128-bit base string, the branch
//      points a 64-bit depth mask, so backtracking jumps straight to the
//      deepest open branch (one re-lookup) instead of unwinding a stack.
//   3. three u32 -> u64 scans (bases, bytes, index of filled pairs) and
//      k_fill_write: the filled fragments as a device read set (2-bit packed,
//      byte-aligned, pair order) ready for the K=96 unipath stage.
#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "apg_core.hpp"
#include "kmer_common.hpp"
#include "kmer_internal.hpp"
#include "ext_table.hpp"
#include "partition.hpp"

namespace apg {

constexpr uint32_t kFillMaxGap = 63;
// apg_spectrum_precorrect_fill_dev: the PreCorrect stage that kicks the fused
// K+1 count onto the side stream (APG_SK_UP_AT_FILL overrides)
constexpr int kFillUpKick = 1;

// (key, bit) from slot s on, v = slot s as already read
__device__ __forceinline__ void ext_set_from(const ExtTab& t, uint64_t key, uint32_t bit, uint64_t s,
                                             unsigned long long v) {
  const unsigned long long want = (key << t.ks) | bit;
  for (;;) {
    if (v == kExtEmpty) {
      v = atomicCAS(&t.slot[s], kExtEmpty, want);
      if (v == kExtEmpty) return;
    }
    if ((v >> t.ks) == key) {
      if (!(v & bit)) atomicOr(&t.slot[s], (unsigned long long)bit);
      return;
    }
    s = (s + 1) & t.mask;
    v = t.slot[s];
  }
}
__device__ __forceinline__ void ext_set(const ExtTab& t, uint64_t key, uint32_t bit) {
  const uint64_t s = ext_home(t, key);  // linear from the aligned group (ext_bits reads it whole)
  ext_set_from(t, key, bit, s, t.slot[s]);
}

// A solid K-mer's two (K-1)-mers: both home slots read before either is
// resolved (two table lines in flight per lane instead of one).
__global__ void k_fill_ext_insert(const uint64_t* __restrict__ solid, uint64_t n, HashP hK, ExtTab t) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c = kunhash(hK, solid[i]);
    // successor c & 3 of u = c >> 2; predecessor (c's first base) of v = c & m1
    const uint64_t u = c >> 2, ur = rc_bases(u, t.n1, t.m1);
    const uint32_t b = (uint32_t)(c & 3);
    const uint64_t ku = u <= ur ? u : ur;
    const uint32_t bu = u <= ur ? 16u << b : 1u << (3 - b);
    const uint64_t v = c & t.m1, vr = rc_bases(v, t.n1, t.m1);
    const uint32_t a = (uint32_t)(c >> (2 * t.n1));
    const uint64_t kv = v <= vr ? v : vr;
    const uint32_t bv = v <= vr ? 1u << a : 16u << (3 - a);
    const uint64_t su = ext_home(t, ku), sv = ext_home(t, kv);
    const unsigned long long xu = t.slot[su], xv = t.slot[sv];
    ext_set_from(t, ku, bu, su, xu);
    ext_set_from(t, kv, bv, sv, xv);
  }
}

// Sorted inserts: each solid K-mer's two (K-1)-mer entries, key << 8 | bit,
// with the top D bits of their home slot above them (D <= 8, D <= 64 - 8 -
// 2(K-1)),
// are grouped by those bits (one partition level) before they are inserted,
// so the concurrent inserts work on a few table regions at a time instead of
// the whole table: the claims and ORs meet lines the last ones left in the
// caches, where the unsorted inserts read and wrote back a random line each.
__global__ void k_ext_entries(const uint64_t* __restrict__ solid, uint64_t n, HashP hK, ExtTab t, int lgT, int D,
                              uint64_t* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c = kunhash(hK, solid[i]);
    const uint64_t u = c >> 2, ur = rc_bases(u, t.n1, t.m1);
    const uint32_t b = (uint32_t)(c & 3);
    const uint64_t ku = u <= ur ? u : ur;
    const uint32_t bu = u <= ur ? 16u << b : 1u << (3 - b);
    const uint64_t v = c & t.m1, vr = rc_bases(v, t.n1, t.m1);
    const uint32_t a = (uint32_t)(c >> (2 * t.n1));
    const uint64_t kv = v <= vr ? v : vr;
    const uint32_t bv = v <= vr ? 1u << a : 16u << (3 - a);
    const uint64_t du = ext_home(t, ku) >> (lgT - D), dv = ext_home(t, kv) >> (lgT - D);
    out[2 * i] = (du << (64 - D)) | (ku << 8) | bu;
    out[2 * i + 1] = (dv << (64 - D)) | (kv << 8) | bv;
  }
}
__global__ void k_ext_insert_entries(const uint64_t* __restrict__ e, uint64_t m, ExtTab t, int D) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t x = e[j];
    ext_set(t, (x << D) >> (D + 8), (uint32_t)x & 0xffu);
  }
}

// Two-level bits of every occupied slot (ext_table.hpp): the successor mask
// of its unique successor and the predecessor mask of its unique
// predecessor, both lookups in flight together.  The inserts are complete,
// so the pred / succ bits every lookup here reads are final; the store
// changes only bits 8-15 of the slot's low word.
__global__ void k_ext_link(ExtTab t) {
  const int n1 = t.n1;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s <= t.mask;
       s += (uint64_t)gridDim.x * blockDim.x) {
    const unsigned long long v = t.slot[s];
    if (v == kExtEmpty) continue;
    const uint64_t c = v >> 16;
    const uint32_t P = (uint32_t)v & 15, S = (uint32_t)(v >> 4) & 15;
    const bool us = __popc(S) == 1, up = __popc(P) == 1;
    if (!(us || up) || c == rc_bases(c, n1, t.m1)) continue;
    // LSB-first forms (ext_issue_lsb's argument) of the successor and the
    // predecessor, in c's orientation
    const uint64_t y = f_rev2(c) >> (64 - 2 * n1);
    const uint64_t ys = (y >> 2) | ((uint64_t)(us ? __ffs(S) - 1 : 0) << (2 * (n1 - 1)));
    const uint64_t yp = ((y << 2) & t.m1) | (uint64_t)(up ? __ffs(P) - 1 : 0);
    ExtProbe qs, qp;
    if (us) qs = ext_issue_lsb(t, ys);
    if (up) qp = ext_issue_lsb(t, yp);
    const uint32_t ss = us ? (ext_finish(t, qs) >> 4) & 15 : 0u;
    const uint32_t pp = up ? ext_finish(t, qp) & 15 : 0u;
    if (ss | pp) t.slot[s] = v | ((unsigned long long)ss << 8) | ((unsigned long long)pp << 12);
  }
}

int ext_link(apg_ctx* ctx, const ExtTab& t, uint64_t n_solid, double frac) {
  if (t.ks != 16 || !n_solid) return APG_OK;
  // algorithmic bytes: the table read + ~2 (K-1)-mers per solid K-mer, each
  // with two 32-byte group reads and its slot written back
  kbegin(ctx, "ext_link", (t.mask + 1) * 8 + n_solid * (2 * 64 + 8));
  const uint64_t g = grid_for(ctx, t.mask + 1);
  k_ext_link<<<std::max<uint64_t>(1, (uint64_t)(g * frac)), 256, 0, ctx->stream>>>(t);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return APG_OK;
}

int ext_build(apg_ctx* ctx, const uint64_t* list, uint64_t n_solid, int K, const char* ws, const char* kname,
              ExtTab* out, bool link) {
  // 4 slots per solid K-mer: load <= 0.5 even if no two solid K-mers share a
  // (K-1)-mer, ~0.25 on a genome, so nearly every lookup ends in the home
  // group.  When that does not fit the device (human-scale replicated solid
  // sets: 2.6 G solid 24-mers -> 2^34 slots = 137 GB), the counting stages'
  // dead buffers are released first, and if it still does not fit the table
  // takes 2 slots per solid K-mer (load <= 0.5 on a genome: 69 GB at human
  // scale; DESIGN.md §7 memory model).
  // APG_EXT_SLOTS=s: s slots per solid K-mer before rounding to a power of
  // two (A/B; default 4)
  static const uint64_t spk = getenv("APG_EXT_SLOTS") ? std::max(1, atoi(getenv("APG_EXT_SLOTS"))) : 4;
  uint64_t T = 1024;
  while (T < spk * n_solid) T <<= 1;
  {
    auto it = ctx->ws.find(ws);
    const uint64_t have = it == ctx->ws.end() ? 0 : it->second.bytes;
    const uint64_t need = T * 8 + 16;
    if (need > have) {
      // room for the table and what the correction pass allocates after it
      // (candidates, decisions, the fused K+1 count's buffers: a few GB at a
      // C5 rank, which ran out of memory on 2.8 GB of candidates with only
      // the 2 GiB margin)
      APG_TRY(ws_make_room(ctx, need - have + (8ull << 30), kRoomDescriptors));
      if (device_free_bytes(ctx) < need - have + (2ull << 30) && T > 1024) {
        T >>= 1;
        vlog(ctx, "ext table: %llu slots (load <= 0.5 by memory)", (unsigned long long)T);
      }
    }
  }
  unsigned long long* slot = nullptr;
  APG_TRY(workspace_t(ctx, ws, T, &slot));
  APG_CHECK_HIP(hipMemsetAsync(slot, 0xff, T * 8, ctx->stream));
  *out = ext_tab(slot, T - 1, K);
  // sorted inserts (APG_EXT_SORTED=1; default: in list order) when the digit
  // fits beside the entry and the two entry buffers (16 B per solid K-mer
  // each) do.  Measured on the bench step (same box): inserts 9.42 -> 7.36 ms
  // but entries + partition 2.6-3.4 ms more on the auxiliary stream, step
  // 144.6 -> 147.2 ms; kept as an A/B switch.
  int lgT = 0;
  while ((1ull << lgT) < T) ++lgT;
  // D <= 8: a partition level splits into at most 256 children (partition.hip)
  const int D = std::min(8, std::min(lgT - 2, 64 - 8 - 2 * (K - 1)));
  static const bool sorted_on = getenv("APG_EXT_SORTED") && !strcmp(getenv("APG_EXT_SORTED"), "1");
  bool sorted = sorted_on && D >= 6 && n_solid >= (1u << 16) && 2 * n_solid < (1ull << 32);  // part_level: < 2^32 per group
  if (sorted) {
    const uint64_t need = 2 * 2 * n_solid * 8;
    if (device_free_bytes(ctx) < need + (4ull << 30)) sorted = false;
  }
  if (sorted) {
    uint64_t *e0 = nullptr, *e1 = nullptr, *child = nullptr;
    APG_TRY(workspace_t(ctx, "ext_e0", 2 * n_solid, &e0));
    APG_TRY(workspace_t(ctx, "ext_e1", 2 * n_solid, &e1));
    APG_TRY(workspace_t(ctx, "ext_child", (1ull << D) + 1, &child));
    kbegin(ctx, "ext_entries", n_solid * (8 + 16));
    k_ext_entries<<<grid_for(ctx, n_solid), 256, 0, ctx->stream>>>(list, n_solid, make_hashp(K), *out, lgT, D, e0);
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
    const std::vector<std::vector<Seg>> parents{{Seg{0, 2 * n_solid}}};
    APG_TRY(part_level<uint64_t>(ctx, e0, e1, parents, 64 - D, D, 2 * n_solid, child, nullptr, "ext"));
    kbegin(ctx, kname, n_solid * 2 * (8 + 64));
    k_ext_insert_entries<<<grid_for(ctx, 2 * n_solid), 256, 0, ctx->stream>>>(e1, 2 * n_solid, *out, D);
    kend(ctx);
  } else {
    kbegin(ctx, kname, n_solid * (8 + 2 * 64));
    if (n_solid)
      k_fill_ext_insert<<<grid_for(ctx, n_solid), 256, 0, ctx->stream>>>(list, n_solid, make_hashp(K), *out);
    kend(ctx);
  }
  APG_CHECK_HIP(hipGetLastError());
  return link ? ext_link(ctx, *out, n_solid) : APG_OK;
}

// 32 bases [pos, pos+32) of a packed read as an LSB-first word (base pos at
// bits 0-1).  Aligned u32 loads; may read up to 12 bytes past the read (the
// read sets carry 64 bytes of slack).
__device__ __forceinline__ uint64_t bases32(const uint8_t* p, uint32_t pos) {
  const uintptr_t a = (uintptr_t)p + (pos >> 2);
  const uint32_t* q = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = 8 * (uint32_t)(a & 3) + 2 * (pos & 3);
  const uint64_t lo = (uint64_t)q[0] | ((uint64_t)q[1] << 32);
  return sh ? (lo >> sh) | ((uint64_t)q[2] << (64 - sh)) : lo;
}

__device__ __forceinline__ uint64_t lmask(uint32_t nb) { return nb >= 32 ? ~0ull : ((1ull << (2 * nb)) - 1); }

// F = rc(B): bases [t, t+32) of F as an LSB-first word; bases past F's end
// are garbage.
__device__ __forceinline__ uint64_t fwin(const uint8_t* B, uint32_t Lf, uint32_t t) {
  const uint32_t m = Lf - t;
  if (m >= 32) return ~f_rev2(bases32(B, Lf - t - 32));
  return ~(f_rev2(bases32(B, 0) & lmask(m)) >> (2 * (32 - m)));
}

// Every K-mer of a packed read (L >= K) solid: one extension lookup per
// K-mer (its first K-1 bases hold its last base as a successor).  Bases are
// streamed 32 at a time from one LSB-first word.
template <int HM = 0>
__device__ __forceinline__ bool read_solid(const ExtTab& t, const uint8_t* R, uint32_t L, uint32_t* nlook) {
  const int n1 = t.n1;
  uint64_t buf = bases32(R, 0);
  uint64_t w = f_rev2(buf & lmask(n1)) >> (64 - 2 * n1);  // first K-1 bases, MSB-first
  uint32_t pend = 0;  // the next (K-1)-mer's successors from a two-level slot | 16
  for (uint32_t i = n1; i < L; ++i) {
    if ((i & 31) == 0) buf = bases32(R, i);
    const uint32_t b = (uint32_t)(((i & 31) == 0 ? buf : buf >> (2 * (i & 31))) & 3);
    uint32_t m = pend & 15;
    if (!(pend & 16)) {
      const uint32_t x = ext_succ2<0, HM>(t, w, nlook);
      m = x & 15;
      pend = x >> 4;
    } else {
      pend = 0;
    }
    if (!((m >> b) & 1)) return false;
    w = ((w << 2) | b) & t.m1;
  }
  return true;
}

// Both reads of a pair solid throughout.  cl (or null): the pair's clean
// flags from the correction pass that used this solid set (1 clean, 0 not,
// 2 not derived -> look the read's K-mers up).
template <int HM = 0>
__device__ __forceinline__ bool pair_solid(const ExtTab& t, const uint8_t* A, uint32_t La, const uint8_t* B,
                                           uint32_t Lf, const uint8_t* cl, uint32_t* nlook) {
  const uint32_t fa = cl ? cl[0] : 2u, fb = cl ? cl[1] : 2u;
  if (fa == 0 || fb == 0) return false;
  if (fa == 2 && !read_solid<HM>(t, A, La, nlook)) return false;
  if (fb == 2 && !read_solid<HM>(t, B, Lf, nlook)) return false;
  return true;
}

struct FillReads {
  const uint64_t* base_off;
  const uint64_t* byte_off;
  const uint8_t* packed;
  uint64_t n_pairs;
};

struct FillP {
  int K;
  uint32_t min_insert, max_insert, max_steps;
};

struct FillRec {
  uint64_t pv_lo, pv_hi;  // gap path bases, MSB-first
  uint32_t len;           // closure length I (filled) or 0
  uint32_t meta;          // status | d << 8 | overlap o << 16
};

enum { kFillOk = 0, kFillNone = 1, kFillAmbiguous = 2, kFillBudget = 3, kFillSkip = 4 };

struct FillCounters {
  unsigned long long st[5];
  unsigned long long lookups;
};

// last K-1 bases of A ++ path[0, d) (MSB-first)
__device__ __forceinline__ uint64_t walk_window(uint64_t atail, unsigned __int128 pv, uint32_t d, const ExtTab& t) {
  if (d >= (uint32_t)t.n1) return (uint64_t)pv & t.m1;
  return ((atail << (2 * d)) | (uint64_t)pv) & t.m1;
}

// Optional two passes (APG_FILL_CAP1=c): pass 1 (every pair, list == null)
// searches with a cap of c expansions and defers the pairs that reach it;
// pass 2 runs the deferred ones (list, *list_n) with the full max_steps.  The
// walk is deterministic, so a pair that ends within the cap ends exactly as
// it would with the full budget.  They kept one deep search from holding a
// whole wave before lanes refilled one by one; with the refill, one pass is
// faster (same box, fill ms iid / repeat-rich genome: cap 96 11.29 / 44.5,
// 48 11.36 / 45.8, 192 11.09 / 46.3, 384 11.10 / 51.0, one pass 11.05 /
// 42.0 — the second pass re-walked every deferred pair's first c steps).
constexpr uint32_t kFillCap1 = 1u << 30;
// A wave refills its idle lanes with new pairs once at most this many lanes
// are still walking (APG_FILL_REFILL for A/B: a higher mark keeps more lanes
// walking, a lower one batches more lanes into each refill's start phase).
#ifndef APG_FILL_REFILL_DEF  // compile-time A/B (scripts/build_fill_variants.sh)
#define APG_FILL_REFILL_DEF 32
#endif
constexpr int kFillRefill = APG_FILL_REFILL_DEF;
// Free steps after an iteration's lookup (APG_FILL_XSTEPS; APG_FILL_XCACHED=1
// lets cached branch points be free steps too), taken only when at least
// APG_FILL_XPCT % of the wave's lanes have one.  Same box, fill ms on the iid
// / repeat-rich genome: 1 step without cached 14.26 / 52.65, 8 with 14.60 /
// 57.09, none 16.16 / 51.70; then (another box) 1 step at 75 % 11.29 / 44.70,
// at 0 % 11.28 / 48.10, none 12.68 / 43.67 (scripts/diag/fill_rep.py): a
// free step runs while the wave's other lanes wait, so only the common
// chains pay.  Round 5 (lean form, fused backtracks; compile-time variants,
// one box): 75 % 10.57 / 37.77, 60 % 10.60 / 38.40, 50 % 10.58 / 37.29,
// 40 % 10.55 / 37.10 -> 40 %; 2 free steps no change; a refill mark of 24
// 10.91 / 43.31, 44 12.06 / 36.65, 40 with 50 % 11.06 / 35.10, and a mark
// raised to 40 after 32-128 refill-free iterations 10.78 / 37.6-38.5 (the
// main step's genome prefers 32).
#ifndef APG_FILL_XSTEPS_DEF  // compile-time A/B (scripts/build_fill_variants.sh)
#define APG_FILL_XSTEPS_DEF 1
#endif
constexpr int kFillXsteps = APG_FILL_XSTEPS_DEF;
#ifndef APG_FILL_XPCT_DEF  // compile-time A/B (scripts/build_fill_variants.sh)
#define APG_FILL_XPCT_DEF 40
#endif
constexpr int kFillXpct = APG_FILL_XPCT_DEF;

// One thread per pair, lanes persistent.  The gap walk is a state machine
// that makes exactly ONE extension lookup per iteration whatever the lane is
// doing (visiting a node, testing a closure's K-1 bridge K-mers, re-reading
// an open branch point), so the wave's lanes issue their lookups together: a
// loop nest (walk step, then the closure test's up to K-2 lookups, then a
// backtrack lookup) made every lane wait for the longest closure test of
// each step.  A lane whose pair is done sits idle until the wave refills
// (wave-aggregated fetch from *next), so a wave is no longer held by its
// slowest pair.  Per lane the lookups, their order and the result are the
// same as the nested search (oracle/fill_oracle.c).
// LEAN (the default): the knobs at their defaults, folded at compile time —
// one pass (cap = max_steps), the branch cache and the bridge filter on,
// kFillRefill, kFillXsteps free steps at kFillXpct %, the multiplicative
// table home — which frees scalar registers the runtime knobs held (the
// general form spills more SGPRs to VGPR lanes); any APG_FILL_* A/B knob
// set (or APG_EXT_HASH=0) selects the general form.
template <int KS, bool LEAN>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_fill(FillReads rv, FillP p, ExtTab t, FillRec* __restrict__ rec,
                                              uint32_t* __restrict__ lens, uint32_t* __restrict__ nbytes,
                                              uint32_t* __restrict__ ones, uint8_t* __restrict__ status_out,
                                              const uint8_t* __restrict__ clean, FillCounters* __restrict__ cnt,
                                              uint32_t cap, const uint32_t* __restrict__ list,
                                              const unsigned long long* __restrict__ list_n,
                                              uint32_t* __restrict__ defer, unsigned long long* __restrict__ ndefer,
                                              unsigned long long* __restrict__ next, bool bcache, bool bfilt,
                                              int refill_, int xsteps_) {
  if constexpr (LEAN) {
    cap = p.max_steps;
    list = nullptr;
    list_n = nullptr;
    defer = nullptr;
    ndefer = nullptr;
    bcache = true;
    bfilt = true;
  }
  // cached backtracks fused into the visit that ends a branch (bcache; the
  // general form: xsteps bit 9 clear)
  const bool fuse = LEAN || (bcache && !(xsteps_ & 512));
  const int refill = LEAN ? kFillRefill : refill_;
  const int xsteps = LEAN ? (kFillXsteps | (kFillXpct << 16)) : xsteps_;
  uint32_t c_ok = 0, c_none = 0, c_amb = 0, c_bud = 0, c_skip = 0;  // registers, not a scratch array
  uint32_t nlook = 0;
  const int K = p.K, n1 = t.n1;
  const uint64_t nwork = list ? *list_n : rv.n_pairs;
  // the lane's pair and its search state
  bool act = false, budget = false;
  uint64_t i = 0, atail = 0, f0 = 0, brm = 0;
  uint32_t LaLf = 0, gmax = 0, dlo = 0, fb0 = 0, d = 0, steps = 0, mode = 0, j = 0, mnode = 0, dd = 0;
  uint32_t n_clos = 0, clos_I = 0, clos_meta = 0;
  unsigned __int128 pv = 0, clos_pv = 0;
  // Two-level slots (ext_table.hpp), one register: bits 0-4 ("pend") the
  // next iteration's mask | 16 when the last lookup already returned it (the
  // walk's next node or the next bridge K-mer after a non-branching (K-1)-mer),
  // bits 8-12 the visited node's such bits, for the step down after its
  // closure test.
  uint32_t pq = 0;
  // wk: the next lookup's (K-1)-mer, set by each transition
  uint64_t wk = 0;
  const uint64_t m1s = t.m1 >> 2;
  // mode 3's keys: the reverse complement of G (j == 16) or of c1 ++ G[0, K-2)
  // (c1 the lowest pending predecessor in j); an LSB-first value complemented
  // is the MSB-first value of its reverse complement
  auto bkey = [&]() -> uint64_t {
    return j == 16 ? (f0 & t.m1) ^ t.m1 : ((((f0 & m1s) ^ m1s) << 2) | (3u - (__ffs(j) - 1)));
  };
  // successor mask of the path's open branch points at depths < 32 (4 bits
  // per depth, 16 depths per word; 100-bp pairs walk < 35 deep): a
  // backtrack to one reads its node's mask here instead of looking it up
  // again — a walk of L leaves re-reads L - 1 branch points, and the
  // repeat-rich pairs (the BUDGET ones) are wide trees.  Two words and
  // selects, not an indexed array (that went to scratch), keep the kernel
  // at 4 waves / SIMD; deeper branch points are looked up as before.
  uint64_t bm0 = 0, bm1 = 0;
  // Bridge filter (bfilt, K >= 3): a closure at a node with window w needs
  // the bridge K-mers w[j, K-1) ++ F[0, j+1) solid for j = 0 .. K-2.  The
  // last two depend only on w's last two bases: before its walk a lane
  // looks up F's first (K-1)-mer G's predecessors c1 and, for each, the
  // predecessors c2 of c1 ++ G[0, K-2) (mode 3: 1 + |P1| lookups through
  // the reverse complements' successor masks), and bk holds bit c2*4 + c1
  // for every solid pair.  A node is a closure candidate only if its
  // window's last two bases are in bk, and the bridge test then checks
  // j = 1 .. K-4 only.  The result is the same; the failing bridge tests
  // (29 % of a walk's lookups on a repeat-rich genome, 30 % on the iid
  // one: tools/fill_walk_model.c) mostly go — 21 % / 18 % fewer iterations.
  uint32_t bk = 0xffffu;
  const int jend = bfilt && n1 >= 2 ? n1 - 2 : n1;  // bridge K-mers [1, jend) by lookup
  auto mask_at = [&](uint32_t dep) -> uint32_t {
    return (uint32_t)((dep < 16 ? bm0 : bm1) >> (4 * (dep & 15))) & 15u;
  };
  auto mask_set = [&](uint32_t dep, uint32_t m) {
    const uint32_t sh = 4 * (dep & 15);
    const uint64_t keep = ~(15ull << sh), v = (uint64_t)m << sh;
    bm0 = dep < 16 ? (bm0 & keep) | v : bm0;
    bm1 = dep >= 16 ? (bm1 & keep) | v : bm1;
  };

  auto emit = [&](uint32_t st, const FillRec& out) {
    rec[i] = out;
    lens[i] = out.len;
    nbytes[i] = (out.len + 3) >> 2;
    ones[i] = st == kFillOk;
    if (status_out) status_out[i] = (uint8_t)st;
    c_ok += st == kFillOk;
    c_none += st == kFillNone;
    c_amb += st == kFillAmbiguous;
    c_bud += st == kFillBudget;
    c_skip += st == kFillSkip;
  };
  // closures counted (overlap phase and walk done): status out, or defer
  auto conclude = [&]() {
    if (!LEAN && budget && n_clos < 2 && cap < p.max_steps) {  // pass 1: search again with the full budget
      defer[atomicAdd(ndefer, 1ull)] = (uint32_t)i;
      return;
    }
    FillRec out{0, 0, 0, 0};
    uint32_t st;
    if (n_clos >= 2)
      st = kFillAmbiguous;
    else if (budget)
      st = kFillBudget;
    else if (n_clos == 0)
      st = kFillNone;
    else {
      st = kFillOk;
      out.len = clos_I;
      out.pv_lo = (uint64_t)clos_pv;
      out.pv_hi = (uint64_t)(clos_pv >> 64);
    }
    out.meta = st == kFillOk ? st | clos_meta : st;
    emit(st, out);
  };
  // pair i: checks and overlap closures; act = true if the gap walk follows
  auto start = [&]() {
    const uint32_t La = (uint32_t)(rv.base_off[2 * i + 1] - rv.base_off[2 * i]);
    const uint32_t Lf = (uint32_t)(rv.base_off[2 * i + 2] - rv.base_off[2 * i + 1]);
    LaLf = La + Lf;
    pq = 0;
    const uint8_t* A = rv.packed + rv.byte_off[2 * i];
    const uint8_t* B = rv.packed + rv.byte_off[2 * i + 1];
    const uint32_t lo = max(p.min_insert, max(La, Lf));
    if (La < (uint32_t)K || Lf < (uint32_t)K || (p.max_insert >= La + Lf && p.max_insert - (La + Lf) > kFillMaxGap)) {
      emit(kFillSkip, FillRec{0, 0, 0, kFillSkip});
      return;
    }
    if (!pair_solid<LEAN ? 1 : 0>(t, A, La, B, Lf, clean ? clean + 2 * i : nullptr, &nlook)) {
      emit(kFillNone, FillRec{0, 0, 0, kFillNone});  // S must be a path of solid K-mers
      return;
    }
    // A's last K-1 bases, MSB-first; F's first 32 bases, LSB-first
    atail = f_rev2(bases32(A, La - n1) & lmask(n1)) >> (64 - 2 * n1);
    f0 = fwin(B, Lf, 0);
    n_clos = 0;
    clos_I = 0;
    clos_meta = 0;
    clos_pv = 0;
    budget = false;
    // overlap closures, I ascending (o descending): A's suffix [s, La) with
    // s = La - o = I - Lf against F's prefix.  Candidate offsets come 32 at a
    // time from a bit-parallel filter — A's bases at s .. s+3 equal F's first
    // four (one bit per offset from four XOR / OR / AND masks over a word of
    // A) — and only candidates get the exact word compare; the ~1 in 256
    // offsets that pass by chance cost a compare each.  Offsets with o < 4
    // skip the filter.  A per-offset loop (a sliding 32-base window) cost
    // ~40 % of the kernel.
    const uint32_t hi_ov = min(p.max_insert, La + Lf - 1);
    if (lo <= hi_ov) {
      constexpr uint64_t r0 = 0x5555555555555555ull;  // low bit of every base
      const uint32_t s_lo = lo - Lf, s_hi = hi_ov - Lf;  // lo >= Lf
      const uint32_t s_f = La > 3 ? La - 3 : 0;        // offsets from here on have o < 4
      const uint64_t c0 = (f0 & 3) * r0, c1 = ((f0 >> 2) & 3) * r0, c2 = ((f0 >> 4) & 3) * r0,
                     c3 = ((f0 >> 6) & 3) * r0;
      auto eqm = [](uint64_t x, uint64_t c) {  // bases of x equal to c's: their low bits
        const uint64_t y = x ^ c;
        return ~(y | (y >> 1)) & r0;
      };
      auto from = [](uint32_t t) { return t >= 32 ? 0ull : ~((1ull << (2 * t)) - 1) & r0; };  // offsets >= t
      uint32_t wb = s_lo & ~31u;
      uint64_t cur = bases32(A, wb);
      for (; wb <= s_hi && n_clos < 2; wb += 32) {
        const uint64_t nx = bases32(A, wb + 32);
        uint64_t m = eqm(cur, c0) & eqm((cur >> 2) | (nx << 62), c1) & eqm((cur >> 4) | (nx << 60), c2) &
                     eqm((cur >> 6) | (nx << 58), c3);
        m |= from(s_f > wb ? s_f - wb : 0);                                 // o < 4: unfiltered
        m &= from(s_lo > wb ? s_lo - wb : 0) & ~from(s_hi - wb + 1);        // [s_lo, s_hi]
        cur = nx;
        for (; m && n_clos < 2; m &= m - 1) {
          const uint32_t sft = wb + (uint32_t)(__builtin_ctzll(m) >> 1);
          const uint32_t o = La - sft, I = Lf + sft;
          bool match = true;
          for (uint32_t c = 0; c < o && match; c += 32)
            match = ((bases32(A, sft + c) ^ (c == 0 ? f0 : fwin(B, Lf, c))) & lmask(min(32u, o - c))) == 0;
          if (!match) continue;
          if (o + 2 <= (uint32_t)K) {  // bridge K-mers: A's tail rolled through F[o, K-1)
            uint64_t w = atail;
            uint32_t pm = 0;  // two-level: the next bridge (K-1)-mer's successors | 16
            for (uint32_t jj = 0; jj + o + 2 <= (uint32_t)K && match; ++jj) {
              const uint32_t b = (uint32_t)(f0 >> (2 * (o + jj))) & 3;
              uint32_t mm = pm & 15;
              if (!(pm & 16)) {
                const uint32_t x = ext_succ2<0, LEAN ? 1 : 0>(t, w, &nlook);
                mm = x & 15;
                pm = x >> 4;
              } else {
                pm = 0;
              }
              match = (mm >> b) & 1;
              w = ((w << 2) | b) & t.m1;
            }
          }
          if (match && ++n_clos == 1) {
            clos_I = I;
            clos_meta = o << 16;
          }
        }
      }
    }
    if (n_clos < 2 && p.max_insert >= La + Lf) {  // gap closures: depth-first walk, bases A<C<G<T
      gmax = p.max_insert - (La + Lf);
      dlo = lo > La + Lf ? lo - (La + Lf) : 0;
      fb0 = (uint32_t)f0 & 3;
      pv = 0;
      brm = 0;  // depths whose node still has unexplored children
      d = steps = mode = 0;
      wk = atail;  // the walk's root: A's last K-1 bases
      if (bfilt && n1 >= 2) {  // the bridge filter's lookups first
        mode = 3;
        j = 16;
        bk = 0;
        wk = bkey();
      }
      act = true;
      return;
    }
    conclude();
  };
  // a closure at depth d (its bridge K-mers all solid); true if the pair is ambiguous
  auto closure = [&]() {
    if (++n_clos == 1) {
      clos_I = LaLf + d;
      clos_pv = pv;
      clos_meta = d << 8;
    }
    return n_clos >= 2;
  };

  bool more = true;
  bool fin = false;  // LEAN: a finished pair not concluded yet
  for (;;) {
    while (more && __popcll(__ballot(act)) <= refill) {  // refill the idle lanes (wave-uniform)
      if (LEAN && fin) {  // a finished pair's status, before its lane takes new work
        conclude();
        fin = false;
      }
      const uint64_t idle = __ballot(!act);
      const unsigned long long k = wave_append(next, !act);  // the wave's next popc(idle) work items
      more = __shfl(k, 63 - __clzll((long long)idle), 64) + 1 < nwork;
      if (!act && k < nwork) {
        i = list ? list[k] : k;
        start();
      }
    }
    if (!__ballot(act)) break;
    if (!act) continue;
    // A step whose mask is already known (a two-level slot's next node or
    // bridge K-mer, or a cached branch point) follows in the same iteration:
    // at most one lookup per iteration, up to xsteps & 255 free steps after
    // it (cached branch points among them if xsteps & 256).
    // one walk step (LEAN: the lookup step, then at most one free step,
    // written out twice instead of an inner loop — fewer values carried
    // around a back edge: repeat-rich `fill` 38.1 -> 35.3 ms, iid 10.55 ->
    // 10.21 ms on one box); true when the pair's search ended
    auto step = [&]() -> bool {
      // LEAN fuses every backtrack to a cached branch point into its visit:
      // mode 2 is left only for depths >= 32, which are never cached
      const bool cached = !LEAN && bcache && mode == 2 && dd < 32;
      const uint64_t key = wk;
      uint32_t m, m2 = 0;
      if (cached) {
        m = mask_at(dd);
      } else if (pq & 16) {
        m = pq & 15;
      } else {
        const uint32_t x = ext_succ2<KS, LEAN ? 1 : 0>(t, key, &nlook);
        m = x & 15;
        m2 = x >> 4;
      }
      pq &= ~0xffu;
      bool visit = false, done = false;
      if (mode == 0) {  // node (pv, d)
        mnode = m;
        pq = m2 << 8;
        visit = true;
        if (d >= dlo && ((m >> fb0) & 1) && ((bk >> (key & 15)) & 1)) {  // closure test: the K-1 bridge K-mers
          if (jend > 1) {
            mode = 1;
            j = 1;
            wk = ((key << 2) | fb0) & t.m1;
            pq |= m2;  // m2 is set only if fb0 is the one successor
            visit = false;
          } else if (closure()) {
            done = true;
            visit = false;
          }
        }
      } else if (mode == 1) {  // bridge K-mer j of the closure test at depth d
        const uint32_t b = (uint32_t)(f0 >> (2 * j)) & 3;
        const bool ok = (m >> b) & 1;
        if (ok && (int)j + 1 < jend) {
          wk = ((wk << 2) | b) & t.m1;
          ++j;
          pq |= m2;
        } else if (ok && closure()) {
          done = true;
        } else {
          mode = 0;
          visit = true;
        }
      } else if (mode == 3) {  // bridge filter: predecessors of G, then of c1 ++ G[0, K-2)
        const uint32_t pm = rev4(m);  // pred(x) bit c = succ(rc(x)) bit 3 - c
        if (j == 16) {
          j = pm;
        } else {
          const uint32_t c1 = __ffs(j) - 1;
          bk |= ((pm & 1) | ((pm & 2) << 3) | ((pm & 4) << 6) | ((pm & 8) << 9)) << c1;
          j &= j - 1;
        }
        if (j == 0) {
          mode = 0;  // the walk from depth 0
          wk = atail;
        } else {
          wk = bkey();
        }
      } else {  // open branch point at depth dd: the sibling after the base taken there
        const uint32_t bb = (uint32_t)(pv >> (2 * (d - dd - 1))) & 3;
        const uint32_t rest = m & ~((2u << bb) - 1);
        const uint32_t b2 = __ffs(rest) - 1;  // rest != 0: dd was marked open
        if (!(rest >> (b2 + 1))) brm &= ~(1ull << dd);
        pv = ((pv >> (2 * (d - dd))) << 2) | b2;
        d = dd + 1;
        mode = 0;
        wk = ((key << 2) | b2) & t.m1;  // key: the window at dd
      }
      if (visit) {  // the walk's step from node (pv, d) with successor mask mnode
        bool down = false;
        if (d < gmax) {
          if (++steps > cap) {
            budget = true;
            done = true;
          } else if (mnode) {
            const uint32_t b = __ffs(mnode) - 1;
            if (mnode >> (b + 1)) {
              brm |= 1ull << d;
              if (d < 32) mask_set(d, mnode);  // an open branch point: its mask for the backtracks
            }
            pv = (pv << 2) | b;
            ++d;
            down = true;
            wk = walk_window(atail, pv, d, t);  // the child's window
            pq |= (pq >> 8) & 0xffu;  // set only if b is the node's one successor
          }
        }
        if (!done && !down) {
          if (!brm) {
            done = true;  // search exhausted
          } else {
            dd = 63 - __clzll((long long)brm);
            const uint64_t wdd = walk_window(atail, pv >> (2 * (d - dd)), dd, t);
            if (fuse && dd < 32) {
              // the backtrack to a branch point whose mask its visit kept:
              // taken now (mode 2's transition), so the sibling's lookup is
              // the next iteration's, not the one after an iteration with
              // no lookup for this lane
              const uint32_t bb = (uint32_t)(pv >> (2 * (d - dd - 1))) & 3;
              const uint32_t rest = mask_at(dd) & ~((2u << bb) - 1);
              const uint32_t b2 = __ffs(rest) - 1;
              if (!(rest >> (b2 + 1))) brm &= ~(1ull << dd);
              pv = ((pv >> (2 * (d - dd))) << 2) | b2;
              d = dd + 1;
              mode = 0;
              wk = ((wdd << 2) | b2) & t.m1;
            } else {
              mode = 2;
              wk = wdd;
            }
          }
        }
      }
      return done;
    };
    if constexpr (LEAN) {
      bool done = step();
      if (!done) {
        const bool can = (pq & 16) != 0;
        if ((uint32_t)__popcll(__ballot(can)) * 100u >= (uint32_t)__popcll(__ballot(true)) * (uint32_t)kFillXpct && can)
          done = step();
      }
      if (done) {  // its status goes out at the wave's next refill (or at the end)
        act = false;
        fin = true;
      }
      continue;
    }
    for (int xs = 0;; ++xs) {
      // ---- one lookup (a node or a closure's bridge K-mer; an open branch
      // point at depth dd < d reads the mask its visit kept)
      const bool cached = bcache && mode == 2 && dd < 32;
      if (xs > 0) {
        // a free step runs while the wave's other lanes wait: taken only when
        // at least (xsteps >> 16) % of the lanes still here have one
        const bool can = (cached && (xsteps & 256)) || (pq & 16);
        if (xs > (xsteps & 255)) break;
        if ((uint32_t)__popcll(__ballot(can)) * 100u < (uint32_t)__popcll(__ballot(true)) * ((uint32_t)xsteps >> 16))
          break;
        if (!can) break;
      }
      const uint64_t key = wk;
      uint32_t m, m2 = 0;
      if (cached) {
        m = mask_at(dd);
      } else if (pq & 16) {
        m = pq & 15;
      } else {
        const uint32_t x = ext_succ2<KS, LEAN ? 1 : 0>(t, key, &nlook);
        m = x & 15;
        m2 = x >> 4;
      }
      pq &= ~0xffu;
      bool visit = false, done = false;
      if (mode == 0) {  // node (pv, d)
        mnode = m;
        pq = m2 << 8;
        visit = true;
        if (d >= dlo && ((m >> fb0) & 1) && ((bk >> (key & 15)) & 1)) {  // closure test: the K-1 bridge K-mers
          if (jend > 1) {
            mode = 1;
            j = 1;
            wk = ((key << 2) | fb0) & t.m1;
            pq |= m2;  // m2 is set only if fb0 is the one successor
            visit = false;
          } else if (closure()) {
            done = true;
            visit = false;
          }
        }
      } else if (mode == 1) {  // bridge K-mer j of the closure test at depth d
        const uint32_t b = (uint32_t)(f0 >> (2 * j)) & 3;
        const bool ok = (m >> b) & 1;
        if (ok && (int)j + 1 < jend) {
          wk = ((wk << 2) | b) & t.m1;
          ++j;
          pq |= m2;
        } else if (ok && closure()) {
          done = true;
        } else {
          mode = 0;
          visit = true;
        }
      } else if (mode == 3) {  // bridge filter: predecessors of G, then of c1 ++ G[0, K-2)
        const uint32_t pm = rev4(m);  // pred(x) bit c = succ(rc(x)) bit 3 - c
        if (j == 16) {
          j = pm;
        } else {
          const uint32_t c1 = __ffs(j) - 1;
          bk |= ((pm & 1) | ((pm & 2) << 3) | ((pm & 4) << 6) | ((pm & 8) << 9)) << c1;
          j &= j - 1;
        }
        if (j == 0) {
          mode = 0;  // the walk from depth 0
          wk = atail;
        } else {
          wk = bkey();
        }
      } else {  // open branch point at depth dd: the sibling after the base taken there
        const uint32_t bb = (uint32_t)(pv >> (2 * (d - dd - 1))) & 3;
        const uint32_t rest = m & ~((2u << bb) - 1);
        const uint32_t b2 = __ffs(rest) - 1;  // rest != 0: dd was marked open
        if (!(rest >> (b2 + 1))) brm &= ~(1ull << dd);
        pv = ((pv >> (2 * (d - dd))) << 2) | b2;
        d = dd + 1;
        mode = 0;
        wk = ((key << 2) | b2) & t.m1;  // key: the window at dd
      }
      if (visit) {  // the walk's step from node (pv, d) with successor mask mnode
        bool down = false;
        if (d < gmax) {
          if (++steps > cap) {
            budget = true;
            done = true;
          } else if (mnode) {
            const uint32_t b = __ffs(mnode) - 1;
            if (mnode >> (b + 1)) {
              brm |= 1ull << d;
              if (d < 32) mask_set(d, mnode);  // an open branch point: its mask for the backtracks
            }
            pv = (pv << 2) | b;
            ++d;
            down = true;
            wk = walk_window(atail, pv, d, t);  // the child's window
            pq |= (pq >> 8) & 0xffu;  // set only if b is the node's one successor
          }
        }
        if (!done && !down) {
          if (!brm) {
            done = true;  // search exhausted
          } else {
            dd = 63 - __clzll((long long)brm);
            const uint64_t wdd = walk_window(atail, pv >> (2 * (d - dd)), dd, t);
            if (fuse && dd < 32) {
              // the backtrack to a branch point whose mask its visit kept:
              // taken now (mode 2's transition), so the sibling's lookup is
              // the next iteration's, not the one after an iteration with
              // no lookup for this lane
              const uint32_t bb = (uint32_t)(pv >> (2 * (d - dd - 1))) & 3;
              const uint32_t rest = mask_at(dd) & ~((2u << bb) - 1);
              const uint32_t b2 = __ffs(rest) - 1;
              if (!(rest >> (b2 + 1))) brm &= ~(1ull << dd);
              pv = ((pv >> (2 * (d - dd))) << 2) | b2;
              d = dd + 1;
              mode = 0;
              wk = ((wdd << 2) | b2) & t.m1;
            } else {
              mode = 2;
              wk = wdd;
            }
          }
        }
      }
      if (done) {
        act = false;
        conclude();
        break;
      }
    }
  }
  if (LEAN && fin) conclude();
  wave_add(&cnt->st[kFillOk], c_ok);
  wave_add(&cnt->st[kFillNone], c_none);
  wave_add(&cnt->st[kFillAmbiguous], c_amb);
  wave_add(&cnt->st[kFillBudget], c_bud);
  wave_add(&cnt->st[kFillSkip], c_skip);
  wave_add(&cnt->lookups, nlook);
}

__device__ __forceinline__ uint32_t packed_base(const uint8_t* r, uint32_t i) { return (r[i >> 2] >> (2 * (i & 3))) & 3; }

// Filled fragments out: kFillWLanes lanes per pair, lane l writes output
// bytes l, l + kFillWLanes, ... (4 bases each), so a wave's stores cover
// contiguous 4-byte runs of 16 fragments.  A wave serves 16 pairs at once:
// the per-pair chain of dependent loads (record, scans, offsets) is what
// bounds the kernel, and 16 lanes per pair (4 pairs per wave) took 3.9 ms
// for the C2 step against 2.7 ms here.  S = A ++ F[ov, Lf) (overlap closure)
// or A ++ path[0, d) ++ F (gap closure, ov = 0), F = rc(B).
constexpr uint32_t kFillWLanes = 4;

__global__ void __launch_bounds__(256) k_fill_write(FillReads rv, const FillRec* __restrict__ rec,
                                                    const uint64_t* __restrict__ bscan,
                                                    const uint64_t* __restrict__ yscan,
                                                    const uint64_t* __restrict__ iscan, uint64_t* __restrict__ out_boff,
                                                    uint64_t* __restrict__ out_yoff, uint8_t* __restrict__ out,
                                                    unsigned long long* __restrict__ n_bad) {
  const uint32_t lane = threadIdx.x % kFillWLanes;
  const uint64_t groups = (uint64_t)gridDim.x * (blockDim.x / kFillWLanes);
  for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x / kFillWLanes) + threadIdx.x / kFillWLanes; i < rv.n_pairs;
       i += groups) {
    const FillRec r = rec[i];
    if (!r.len) continue;
    const uint64_t y0 = yscan[i];
    if (lane == 0) {
      const uint64_t j = iscan[i];
      out_boff[j] = bscan[i];
      out_yoff[j] = y0;
    }
    const uint32_t La = (uint32_t)(rv.base_off[2 * i + 1] - rv.base_off[2 * i]);
    const uint32_t Lf = (uint32_t)(rv.base_off[2 * i + 2] - rv.base_off[2 * i + 1]);
    const uint8_t* A = rv.packed + rv.byte_off[2 * i];
    const uint8_t* B = rv.packed + rv.byte_off[2 * i + 1];
    uint8_t* o = out + y0;
    const uint32_t I = r.len;
    const unsigned __int128 pv = ((unsigned __int128)r.pv_hi << 64) | r.pv_lo;
    const uint32_t ov = r.meta >> 16, d = (r.meta >> 8) & 0xff;
    // a record is S = A ++ path[0, d) ++ F[ov, Lf): anything else is an
    // internal error, reported, and its bases are not read
    if ((uint64_t)La + Lf + d != (uint64_t)I + ov || ov > Lf || ov > La) {
      if (lane == 0) atomicAdd(n_bad, 1ull);
      continue;
    }
    const uint32_t nby = (I + 3) / 4;
    for (uint32_t y = lane; y < nby; y += kFillWLanes) {
      const uint32_t t0 = 4 * y;
      if (t0 + 4 <= La) {  // A is byte-aligned like S
        o[y] = A[y];
        continue;
      }
      if (t0 >= La + d && t0 + 4 <= I) {  // four bases of F = rc(B): B[S0-3 .. S0] reversed, complemented
        const uint32_t S0 = Lf - 1 - (t0 - La - d + ov);
        const uint32_t e = S0 - 3, sh = 2 * (e & 3);
        const uint32_t w16 = (uint32_t)B[e >> 2] | ((uint32_t)B[(e >> 2) + 1] << 8);
        const uint32_t x = (w16 >> sh) & 0xff;  // b(S0-3) b(S0-2) b(S0-1) b(S0), LSB-first
        const uint32_t r = ((x & 3) << 6) | (((x >> 2) & 3) << 4) | (((x >> 4) & 3) << 2) | (x >> 6);
        o[y] = (uint8_t)(~r & 0xff);
        continue;
      }
      uint32_t acc = 0;
      for (uint32_t t = t0; t < t0 + 4 && t < I; ++t) {
        uint32_t b;
        if (t < La)
          b = packed_base(A, t);
        else if (t < La + d)
          b = (uint32_t)(pv >> (2 * (d - 1 - (t - La)))) & 3;
        else
          b = 3 - packed_base(B, Lf - 1 - (t - La - d + ov));
        acc |= b << (2 * (t & 3));
      }
      o[y] = (uint8_t)acc;
    }
  }
}

static int fill_check(const apg_fill_params& p) {
  APG_REQUIRE(p.K >= 2 && p.K <= 29, "apg_fill_fragments: K must be in [2, 29]");
  APG_REQUIRE(p.min_insert <= p.max_insert, "apg_fill_fragments: min_insert > max_insert");
  APG_REQUIRE(p.min_solid >= 1, "apg_fill_fragments: min_solid must be >= 1");
  return APG_OK;
}

// Allocate (or reuse) the device read set of the filled fragments.
static int filled_alloc(apg_ctx* ctx, apg_dreads** io, uint64_t n, uint64_t nbases, uint64_t nbytes) {
  apg_dreads* d = *io;
  if (d && (d->ctx != ctx || !d->fill_owned)) {
    set_error("apg_fill_fragments_dev: *filled must be NULL or a previous apg_fill_fragments_dev output");
    return APG_E_ARG;
  }
  if (!d) {
    d = new (std::nothrow) apg_dreads();
    if (!d) return APG_E_NOMEM;
    d->ctx = ctx;
    d->device = ctx->device;
    d->fill_owned = true;
    *io = d;
  }
  if (d->cap_reads < n + 1) {
    if (d->d_base_off) APG_CHECK_HIP(hipFree(d->d_base_off));
    if (d->d_byte_off) APG_CHECK_HIP(hipFree(d->d_byte_off));
    d->d_base_off = d->d_byte_off = nullptr;
    d->cap_reads = 0;
    const uint64_t c = n + 1 + (n + 1) / 8;
    APG_CHECK_HIP(hipMalloc(&d->d_base_off, c * 8));
    APG_CHECK_HIP(hipMalloc(&d->d_byte_off, c * 8));
    d->cap_reads = c;
  }
  if (d->cap_bytes < nbytes + 64) {
    if (d->d_packed) APG_CHECK_HIP(hipFree(d->d_packed));
    d->d_packed = nullptr;
    d->cap_bytes = 0;
    const uint64_t c = nbytes + nbytes / 8 + 64;
    APG_CHECK_HIP(hipMalloc(&d->d_packed, c));
    APG_CHECK_HIP(hipMemsetAsync(d->d_packed, 0, c, ctx->stream));
    d->cap_bytes = c;
  }
  static std::atomic<uint64_t> g_fill{3ull << 61};
  d->gen = g_fill.fetch_add(1);  // new contents: per-read-set plans are stale
  d->n_reads = n;
  d->n_bases = nbases;
  d->n_bytes = nbytes;
  d->shape_hash = 0;  // shape produced on the device: not known to the host
  return APG_OK;
}

static int fill_impl(apg_ctx* ctx, const apg_dreads* dr, const apg_fill_params& p, const uint64_t* d_solid,
                     uint64_t n_solid, apg_dreads** filled, uint8_t* d_status, apg_fill_stats* st) {
  APG_REQUIRE(dr->n_reads % 2 == 0, "apg_fill_fragments: pairs must be an even number of reads (2i, 2i+1)");
  ctx->ws_dead &= ~kRoomCorrection;  // the correction tables are read again
  const uint64_t np = dr->n_reads / 2;
  std::memset(st, 0, sizeof *st);
  st->n_pairs = np;
  const uint64_t* list = d_solid;
  const uint8_t* clean = nullptr;
  bool have_ext = false;
  ExtTab et{};
  if (!list && n_solid == 0) {
    if (p.flags & APG_FILL_LAST_SOLID) {
      APG_REQUIRE(ctx->pc_list_valid, "apg_fill_fragments: APG_FILL_LAST_SOLID but no correction pass ran on ctx");
      APG_REQUIRE(ctx->pc_K == p.K, "apg_fill_fragments: last correction pass used another K");
      list = ctx->pc_list;
      n_solid = ctx->pc_n;
      // the pass's clean flags answer "every K-mer of the read solid" for the
      // reads it corrected (these very bases: same generation)
      if (ctx->clean_valid && ctx->clean_gen == dr->gen) clean = ctx->pc_clean;
      // ... and the pass's extension table is this very solid set's
      if (ctx->pc_ext_valid) {
        et = ext_tab(ctx->pc_ext_slot, ctx->pc_ext_mask, p.K);
        have_ext = true;
      }
    } else {  // the pairs' own solid K-mers
      SkResult sr;
      APG_TRY(sk_spectrum(ctx, dr, p.K, true, p.min_solid, nullptr, 0, &sr));
      list = sr.solid;
      n_solid = sr.n_solid;
      ctx->pc_list_valid = false;  // "pc_solid" now holds this list
      ctx->pc_ext_valid = false;
    }
  }
  APG_REQUIRE(n_solid == 0 || list, "apg_fill_fragments: solid set pointer is NULL");
  st->n_solid = n_solid;
  if (!have_ext) APG_TRY(ext_build(ctx, list, n_solid, p.K, "fill_ext", "fill_ext", &et));

  FillRec* rec = nullptr;
  uint32_t *lens = nullptr, *nby = nullptr, *ones = nullptr;
  uint64_t *bscan = nullptr, *yscan = nullptr, *iscan = nullptr;
  unsigned long long* cnt = nullptr;
  const uint64_t npc = std::max<uint64_t>(np, 1);
  APG_TRY(workspace_t(ctx, "fill_rec", npc, &rec));
  APG_TRY(workspace_t(ctx, "fill_lens", npc, &lens));
  APG_TRY(workspace_t(ctx, "fill_nby", npc, &nby));
  APG_TRY(workspace_t(ctx, "fill_ones", npc, &ones));
  APG_TRY(workspace_t(ctx, "fill_bscan", npc + 1, &bscan));
  APG_TRY(workspace_t(ctx, "fill_yscan", npc + 1, &yscan));
  APG_TRY(workspace_t(ctx, "fill_iscan", npc + 1, &iscan));
  APG_TRY(workspace_t(ctx, "fill_cnt", 6, &cnt));
  APG_CHECK_HIP(hipMemsetAsync(cnt, 0, 6 * 8, ctx->stream));
  const FillReads rv{dr->d_base_off, dr->d_byte_off, dr->d_packed, np};
  const FillP fp{p.K, p.min_insert, p.max_insert, p.max_steps};
  uint32_t* defer = nullptr;
  unsigned long long* ndefer = nullptr;
  APG_TRY(workspace_t(ctx, "fill_defer", npc, &defer));
  // deferred count, next pair of pass 1 / pass 2, inconsistent records (k_fill_write)
  APG_TRY(workspace_t(ctx, "fill_ndefer", 4, &ndefer));
  APG_CHECK_HIP(hipMemsetAsync(ndefer, 0, 4 * 8, ctx->stream));
  kbegin(ctx, "fill", dr->n_bytes + 16 * dr->n_reads + np * (sizeof(FillRec) + 12));
  if (np) {
    FillCounters* fc = reinterpret_cast<FillCounters*>(cnt);
    // lanes are persistent (work fetched per wave): one resident round of blocks
    const bool two = et.ks == 16;
    const uint32_t grid = two ? resident_grid(ctx, k_fill<16, true>, 256, (np + 255) / 256)
                              : resident_grid(ctx, k_fill<8, true>, 256, (np + 255) / 256);
    // APG_FILL_BRANCH_CACHE=0: backtracks look their branch point up again (A/B)
    const char* be = getenv("APG_FILL_BRANCH_CACHE");
    const bool bcache = !(be && !strcmp(be, "0"));
    // APG_FILL_BRIDGE_FILTER=0: every closure candidate tested K-mer by K-mer (A/B)
    const char* bfe = getenv("APG_FILL_BRIDGE_FILTER");
    const bool bfilt = !(bfe && !strcmp(bfe, "0"));
    const char* rfe = getenv("APG_FILL_REFILL");
    const int refill = rfe ? std::max(0, std::min(63, atoi(rfe))) : kFillRefill;
    // APG_FILL_XSTEPS: free steps after an iteration's lookup (0: one step per iteration)
    const char* xse = getenv("APG_FILL_XSTEPS");
    const char* xce = getenv("APG_FILL_XCACHED");  // 1: cached branch points may be free steps
    const char* xpe = getenv("APG_FILL_XPCT");  // free steps only when this % of the lanes have one
    const int xpct = std::min(100, std::max(0, xpe ? atoi(xpe) : kFillXpct));
    const char* fbe = getenv("APG_FILL_FUSE_BT");  // 0: a cached backtrack takes an iteration of its own (A/B)
    const int xsteps = std::min(255, xse ? std::max(0, atoi(xse)) : kFillXsteps) | (xce && !strcmp(xce, "1") ? 256 : 0) |
                       (fbe && !strcmp(fbe, "0") ? 512 : 0) | (xpct << 16);
    const char* c1e = getenv("APG_FILL_CAP1");  // pass 1's expansion cap (A/B)
    const uint32_t cap1 = c1e ? (uint32_t)std::max(1, atoi(c1e)) : kFillCap1;
    auto fill = [&](auto kern) {
      kern<<<grid, 256, 0, ctx->stream>>>(rv, fp, et, rec, lens, nby, ones, d_status, clean, fc,
                                          std::min(cap1, p.max_steps), nullptr, nullptr, defer, ndefer,
                                          ndefer + 1, bcache, bfilt, refill, xsteps);
      if (p.max_steps > cap1)  // the deferred pairs: a device-side count, no host round trip
        kern<<<grid, 256, 0, ctx->stream>>>(rv, fp, et, rec, lens, nby, ones, d_status, clean, fc, p.max_steps,
                                            defer, ndefer, nullptr, nullptr, ndefer + 2, bcache, bfilt, refill, xsteps);
    };
    // the general form when any A/B knob is set (APG_FILL_LEAN=0 forces it)
    const char* le = getenv("APG_FILL_LEAN");
    const bool lean = !(le && !strcmp(le, "0")) && et.hs != 0 && bcache && bfilt && refill == kFillRefill &&
                      xsteps == (kFillXsteps | (kFillXpct << 16)) && cap1 >= p.max_steps;
    if (two && lean)
      fill(k_fill<16, true>);
    else if (two)
      fill(k_fill<16, false>);
    else if (lean)
      fill(k_fill<8, true>);
    else
      fill(k_fill<8, false>);
  }
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  {
    const uint32_t* const ins[3] = {lens, nby, ones};
    uint64_t* const outs[3] = {bscan, yscan, iscan};
    APG_TRY(scan_cols_u32_u64(ctx, 3, ins, np, outs, "fby"));
  }
  unsigned long long hc[6];
  uint64_t tot[3];
  APG_CHECK_HIP(hipMemcpyAsync(hc, cnt, sizeof hc, hipMemcpyDeviceToHost, ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(&tot[0], bscan + np, 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(&tot[1], yscan + np, 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(d2h_sync(ctx, &tot[2], iscan + np, 8));
  kbytes_add(ctx, "fill", hc[5] * 64);  // one random 64-byte table line per extension lookup
  st->n_filled = hc[kFillOk];
  st->n_none = hc[kFillNone];
  st->n_ambiguous = hc[kFillAmbiguous];
  st->n_budget = hc[kFillBudget];
  st->n_skip = hc[kFillSkip];
  st->lookups = hc[5];
  st->filled_bases = tot[0];
  if (!filled) return APG_OK;
  const uint64_t nf = tot[2];
  APG_TRY(filled_alloc(ctx, filled, nf, tot[0], tot[1]));
  apg_dreads* fd = *filled;
  fd->max_len = nf ? p.max_insert : 0;
  kbegin(ctx, "fill_write", np * (sizeof(FillRec) + 24) + tot[1] + nf * 16);
  if (np)
    k_fill_write<<<grid_for(ctx, np, 256 / kFillWLanes), 256, 0, ctx->stream>>>(rv, rec, bscan, yscan, iscan,
                                                                                 fd->d_base_off, fd->d_byte_off,
                                                                                 fd->d_packed, ndefer + 3);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  APG_CHECK_HIP(hipMemcpyAsync(fd->d_base_off + nf, bscan + np, 8, hipMemcpyDeviceToDevice, ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(fd->d_byte_off + nf, yscan + np, 8, hipMemcpyDeviceToDevice, ctx->stream));
  APG_CHECK_HIP(hipMemsetAsync(fd->d_packed + tot[1], 0, 64, ctx->stream));
  unsigned long long nbad = 0;
  APG_TRY(d2h_sync(ctx, &nbad, ndefer + 3, 8));
  if (nbad) {
    set_error("apg_fill_fragments: inconsistent fill records (internal error)");
    return APG_E_STATE;
  }
  return APG_OK;
}

}  // namespace apg

using namespace apg;

extern "C" {

void apg_fill_defaults(apg_fill_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->K = 24;
  p->min_insert = 126;
  p->max_insert = 234;
  p->max_steps = 1024;
  p->min_solid = 3;
}

int apg_fill_fragments_dev(apg_ctx* ctx, const apg_dreads* pairs, const apg_fill_params* pp, const void* d_solid,
                           uint64_t n_solid, apg_dreads** filled, uint8_t* d_status, apg_fill_stats* stats) {
  APG_REQUIRE(ctx && pairs, "apg_fill_fragments_dev: NULL argument");
  apg_fill_params p;
  if (pp)
    p = *pp;
  else
    apg_fill_defaults(&p);
  APG_TRY(fill_check(p));
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  apg_fill_stats st;
  APG_TRY(fill_impl(ctx, pairs, p, static_cast<const uint64_t*>(d_solid), d_solid ? n_solid : 0, filled, d_status,
                    &st));
  if (stats) *stats = st;
  return APG_OK;
}

int apg_spectrum_precorrect_fill_dev(apg_ctx* ctx, apg_dreads* reads, int K_spec, uint64_t* hist, size_t hist_len,
                                     apg_kstats* kstats, const apg_pc_params* pp, apg_pc_stats* pstats,
                                     const apg_fill_params* fp, apg_dreads** filled, uint8_t* d_status,
                                     apg_fill_stats* fstats) {
  APG_REQUIRE(ctx && reads, "apg_spectrum_precorrect_fill_dev: NULL argument");
  apg_fill_params f;
  if (fp)
    f = *fp;
  else
    apg_fill_defaults(&f);
  f.flags |= APG_FILL_LAST_SOLID;
  APG_TRY(fill_check(f));
  apg_pc_params p;
  if (pp)
    p = *pp;
  else
    apg_pc_defaults(&p);
  APG_REQUIRE(f.K == p.K, "apg_spectrum_precorrect_fill_dev: FillFragments and PreCorrect need the same K");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  // the fused K+1 count stays on the side stream past PreCorrect, beside
  // FillFragments' kernels (FillFragments reads the corrected reads and the
  // pass's extension table, never the K-records or their buckets), and is
  // kicked at stage APG_SK_UP_AT_FILL (default kFillUpKick) of the pass
  // unless APG_SK_UP_AT says otherwise; stage 4 = after PreCorrect
  static const int kick = getenv("APG_SK_UP_AT_FILL") ? atoi(getenv("APG_SK_UP_AT_FILL")) : kFillUpKick;
  ctx->side_kick_default = kick;
  int rc = spectrum_precorrect_impl(ctx, reads, K_spec, hist, hist_len, kstats, &p, pstats, false);
  ctx->side_kick_default = 1;
  if (rc == APG_OK) rc = side_kick(ctx, 4);
  apg_fill_stats st;
  std::memset(&st, 0, sizeof st);
  if (rc == APG_OK) rc = fill_impl(ctx, reads, f, nullptr, 0, filled, d_status, &st);
  const int rj = side_join(ctx);  // the K+1 spectrum lands here
  if (rc == APG_OK) rc = rj;
  if (rc == APG_OK) rc = up_kstats_fill(ctx);
  ctx->up_kstats = nullptr;
  if (rc == APG_OK && fstats) *fstats = st;
  return rc;
}

int apg_fill_fragments(apg_ctx* ctx, const apg_reads* pairs, const apg_fill_params* pp, const uint64_t* solid,
                       uint64_t n_solid, apg_reads* out, uint8_t* status, apg_fill_stats* stats) {
  APG_REQUIRE(ctx && pairs && out, "apg_fill_fragments: NULL argument");
  APG_REQUIRE(n_solid == 0 || solid, "apg_fill_fragments: solid is NULL");
  std::memset(out, 0, sizeof(*out));
  apg_fill_params p;
  if (pp)
    p = *pp;
  else
    apg_fill_defaults(&p);
  APG_TRY(fill_check(p));
  APG_REQUIRE(!(p.flags & APG_FILL_LAST_SOLID) || solid == nullptr,
              "apg_fill_fragments: give either a solid set or APG_FILL_LAST_SOLID");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  apg_dreads* dr = nullptr;
  APG_TRY(apg_reads_upload(ctx, pairs, &dr));
  uint64_t* d_solid = nullptr;
  uint8_t* d_status = nullptr;
  apg_dreads* fd = nullptr;
  apg_fill_stats st;
  std::memset(&st, 0, sizeof st);
  const uint64_t np = pairs->n_reads / 2;
  int rc = APG_OK;
  auto hip = [&](hipError_t e) {
    if (e != hipSuccess && rc == APG_OK) {
      set_error(std::string("apg_fill_fragments: ") + hipGetErrorString(e));
      rc = APG_E_HIP;
    }
  };
  if (n_solid) {
    hip(hipMalloc(&d_solid, n_solid * 8));
    if (rc == APG_OK) hip(hipMemcpyAsync(d_solid, solid, n_solid * 8, hipMemcpyHostToDevice, ctx->stream));
  }
  if (rc == APG_OK && status && np) hip(hipMalloc(&d_status, np));
  if (rc == APG_OK) rc = apg_fill_fragments_dev(ctx, dr, &p, d_solid, n_solid, &fd, d_status, &st);
  if (rc == APG_OK) {
    const uint64_t n = fd->n_reads;
    out->n_reads = n;
    uint64_t* bo = (uint64_t*)std::malloc((n + 1) * 8);
    uint64_t* yo = (uint64_t*)std::malloc((n + 1) * 8);
    uint8_t* pk = (uint8_t*)std::calloc(fd->n_bytes + 64, 1);
    out->base_off = bo;
    out->byte_off = yo;
    out->packed = pk;
    if (!bo || !yo || !pk) {
      set_error("apg_fill_fragments: host allocation failed");
      rc = APG_E_NOMEM;
    } else {
      hip(hipMemcpyAsync(bo, fd->d_base_off, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
      hip(hipMemcpyAsync(yo, fd->d_byte_off, (n + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
      if (fd->n_bytes) hip(hipMemcpyAsync(pk, fd->d_packed, fd->n_bytes, hipMemcpyDeviceToHost, ctx->stream));
      if (d_status) hip(hipMemcpyAsync(status, d_status, np, hipMemcpyDeviceToHost, ctx->stream));
      hip(hipStreamSynchronize(ctx->stream));
    }
    if (rc != APG_OK) apg_reads_release(out);
  }
  if (d_solid) (void)hipFree(d_solid);
  if (d_status) (void)hipFree(d_status);
  apg_reads_free(fd);
  apg_reads_free(dr);
  if (rc == APG_OK && stats) *stats = st;
  return rc;
}

}  // extern "C"
