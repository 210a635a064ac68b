// unipath.hip — MI355X-native unipath graph builder for K <= 96.
//
// Replaces CommonPather/ReadsToPaths, Unipather and the unipath adjacency ->
// HyperKmerPath step of RunAllPathsLG ([R:M] src/paths/ReadsToPathsCoreX.cc,
// src/paths/Unipath.cc, src/paths/HyperKmerPath.h; reference snapshot empty,
// SURVEY §0.1).  Semantics: SURVEY §A.5-A.6 as made operational in DESIGN.md
// and restated on the CPU in oracle/unipath_oracle.cpp.
//
// Pipeline (U = unipath stage):
//   U1 uhll                        sizing pass: one thread per read rolls the
//      192-bit fw/rc K-mer; instance count + HyperLogLog distinct estimate
//   U2 uinsert_reads               every instance {canonical key, hash56 |
//      extension bits} goes into a global open-addressing node table (claim
//      by CAS on a tag, full-key compare, OR of new extension bits)
//   U3 tab_count / tab_scatter     table -> dense node array grouped by the
//      top 5 hash bits (the shard order of the multi-GPU exchange)
//   U4 node_insert                 open-addressing index of the node array
//   U5 links                       unique successor/predecessor per directed
//      node (v = 2*node + orientation)
//   U6 ranking                     sparse ruling set: heads + every 32nd node
//      walk their segment; pointer jumping over rulers; cycles are cut before
//      their min K-mer (min found by pointer jumping) and ranking reruns
//   U7 pairs                       (u, rc u) keys, LSD radix sort on 192 bits
//   U8 outputs                     ids, unibases, HyperKmerPath vertices
//      (lock-free union-find over unipath ends), per-read KmerPaths
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "apg_core.hpp"
#include "exchange.hpp"
#include "kmer_common.hpp"
#include "partition.hpp"
#include "superkmer.hpp"

namespace apg {

constexpr uint32_t kNone = 0xffffffffu;

// ---------------------------------------------------------------------------
// 192-bit K-mer keys: limbs (a, b, c), a most significant, value right-aligned
// ---------------------------------------------------------------------------
struct K3 {
  uint64_t a, b, c;
};

struct KeyP {
  int K;
  uint64_t ma, mb, mc;  // masks of the 2K-bit value per limb
};

static KeyP make_keyp(int K) {
  KeyP p;
  p.K = K;
  const int bits = 2 * K;
  p.mc = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
  p.mb = bits >= 128 ? ~0ull : bits <= 64 ? 0 : ((1ull << (bits - 64)) - 1);
  p.ma = bits >= 192 ? ~0ull : bits <= 128 ? 0 : ((1ull << (bits - 128)) - 1);
  return p;
}

__device__ __forceinline__ bool k3_lt(const K3& x, const K3& y) {
  if (x.a != y.a) return x.a < y.a;
  if (x.b != y.b) return x.b < y.b;
  return x.c < y.c;
}
__device__ __forceinline__ bool k3_eq(const K3& x, const K3& y) { return x.a == y.a && x.b == y.b && x.c == y.c; }

__device__ __forceinline__ K3 push_right(const K3& k, uint64_t base, const KeyP& p) {
  K3 r;
  r.a = ((k.a << 2) | (k.b >> 62)) & p.ma;
  r.b = ((k.b << 2) | (k.c >> 62)) & p.mb;
  r.c = ((k.c << 2) | base) & p.mc;
  return r;
}

// rc of the K-mer after appending `base` to the fw K-mer: shift right 2, put
// the complement at the top (bit 2K-2).
__device__ __forceinline__ K3 rc_roll(const K3& r, uint64_t base, const KeyP& p) {
  K3 o;
  o.c = (r.c >> 2) | (r.b << 62);
  o.b = (r.b >> 2) | (r.a << 62);
  o.a = r.a >> 2;
  const int pos = 2 * p.K - 2;
  const uint64_t x = 3 - base;
  if (pos >= 128)
    o.a |= x << (pos - 128);
  else if (pos >= 64)
    o.b |= x << (pos - 64);
  else
    o.c |= x << pos;
  o.a &= p.ma;
  o.b &= p.mb;
  o.c &= p.mc;
  return o;
}

// reverse the 32 2-bit groups: per 32-bit half a bit reverse, then the bits
// of each pair swapped back (v_bfrev + two shifts + one v_bfi: 8 VALU for the
// 64 bits, against 17 for the mask-and-shift ladder with a byte swap)
__device__ __forceinline__ uint64_t rev2(uint64_t x) { return sk_rev2(x); }

// x >> s for a 192-bit (a:b:c) value, 0 <= s <= 192
__device__ __forceinline__ K3 shr192(const K3& x, int s) {
  if (s == 0) return x;
  if (s >= 192) return K3{0, 0, 0};
  if (s < 64) return K3{x.a >> s, (x.b >> s) | (x.a << (64 - s)), (x.c >> s) | (x.b << (64 - s))};
  if (s == 64) return K3{0, x.a, x.b};
  if (s < 128) return K3{0, x.a >> (s - 64), (x.b >> (s - 64)) | (x.a << (128 - s))};
  if (s == 128) return K3{0, 0, x.a};
  return K3{0, 0, x.a >> (s - 128)};
}

__device__ __forceinline__ K3 revcomp(const K3& k, const KeyP& p) {
  // complement + reverse all 96 2-bit groups, then right-align the 2K bits
  K3 r = shr192(K3{rev2(~k.c), rev2(~k.b), rev2(~k.a)}, 192 - 2 * p.K);
  r.a &= p.ma;
  r.b &= p.mb;
  r.c &= p.mc;
  return r;
}

// The 96 bases [j, j+96) of a 2-bit LSB-first packed read as a 192-bit
// LSB-first value (base j in the low bits of .c).  Reads up to 28 bytes from
// the 4-byte-aligned word holding base j (device read buffers carry slack).
__device__ __forceinline__ K3 load_lsb192(const uint8_t* rd, uint32_t j) {
  const uintptr_t addr = (uintptr_t)(rd + (j >> 2));
  const uint32_t* w = reinterpret_cast<const uint32_t*>(addr & ~(uintptr_t)3);
  const int sh = (int)(addr & 3) * 8 + 2 * (int)(j & 3);  // < 32
  const uint64_t q0 = (uint64_t)w[0] | ((uint64_t)w[1] << 32);
  const uint64_t q1 = (uint64_t)w[2] | ((uint64_t)w[3] << 32);
  const uint64_t q2 = (uint64_t)w[4] | ((uint64_t)w[5] << 32);
  const uint64_t q3 = (uint64_t)w[6];
  if (sh == 0) return K3{q2, q1, q0};
  return K3{(q2 >> sh) | (q3 << (64 - sh)), (q1 >> sh) | (q2 << (64 - sh)), (q0 >> sh) | (q1 << (64 - sh))};
}

__device__ __forceinline__ uint64_t fmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// Partition / index hash of a canonical key: top 56 bits used (low byte holds
// the extension bits in KRec.meta).
__device__ __forceinline__ uint64_t key_hash(const K3& k) {
  return fmix64(k.a ^ fmix64(k.b ^ fmix64(k.c ^ 0x5851f42d4c957f2dull))) & ~0xffull;
}

__device__ __forceinline__ K3 rec_key(const KRec& r) { return K3{r.k0, r.k1, r.k2}; }
__device__ __forceinline__ uint32_t comp4(uint32_t s) {  // bit b -> bit 3-b
  return ((s & 1) << 3) | ((s & 2) << 1) | ((s & 4) >> 1) | ((s & 8) >> 3);
}
__device__ __forceinline__ uint32_t read_base(const uint8_t* rd, uint32_t i) {
  return (rd[i >> 2] >> (2 * (i & 3))) & 3;
}

// canonical key, orientation (0: fw is canonical, incl. palindromes) and the
// instance's extension bits in canonical orientation (left | right << 4)
__device__ __forceinline__ void canon_ext(const K3& fw, const K3& rc, int a, int b, K3* key, uint32_t* ext) {
  const bool pal = k3_eq(fw, rc);
  const bool fwc = pal || k3_lt(fw, rc);
  const uint32_t la = a >= 0 ? 1u << a : 0, rb = b >= 0 ? 1u << b : 0;
  const uint32_t ca = a >= 0 ? 1u << (3 - a) : 0, cb = b >= 0 ? 1u << (3 - b) : 0;
  uint32_t L, R;
  if (pal) {
    L = la | cb;
    R = rb | ca;
  } else if (fwc) {
    L = la;
    R = rb;
  } else {
    L = cb;
    R = ca;
  }
  *key = fwc ? fw : rc;
  *ext = L | (R << 4);
}

struct ReadsV {
  const uint64_t* base_off;
  const uint64_t* byte_off;
  const uint8_t* packed;
  uint64_t n_reads;
};

// Rolling state over one read for 192-bit K-mers.
struct Roller3 {
  const uint8_t* rd;
  uint32_t len, i;
  K3 fw, rc;
  __device__ __forceinline__ void init(const uint8_t* r, uint32_t n, const KeyP& p) {
    rd = r;
    len = n;
    if (n >= (uint32_t)p.K) {
      prime(0, p);
      return;
    }
    i = 0;
    fw = K3{0, 0, 0};
    rc = K3{0, 0, 0};
    const uint32_t m = n < (uint32_t)(p.K - 1) ? n : (uint32_t)(p.K - 1);
    for (uint32_t j = 0; j < m; ++j) step(p);
  }
  // State after stepping through the K-1 bases [j, j+K-1) (needs j+K-1 <=
  // len), built from packed words instead of K-1 single-base steps:
  //   fw = those bases MSB-first;  rc = complement of them LSB-first, << 2.
  __device__ __forceinline__ void prime(uint32_t j, const KeyP& p) {
    const int bits = 2 * (p.K - 1);
    const K3 W = load_lsb192(rd, j);
    const uint64_t mc = bits >= 64 ? ~0ull : ((1ull << bits) - 1);
    const uint64_t mb = bits >= 128 ? ~0ull : bits <= 64 ? 0 : ((1ull << (bits - 64)) - 1);
    const uint64_t ma = bits <= 128 ? 0 : ((1ull << (bits - 128)) - 1);  // bits <= 190
    fw = shr192(K3{rev2(W.c), rev2(W.b), rev2(W.a)}, 192 - bits);
    const K3 R{(W.a ^ ~0ull) & ma, (W.b ^ ~0ull) & mb, (W.c ^ ~0ull) & mc};
    rc = K3{((R.a << 2) | (R.b >> 62)) & p.ma, ((R.b << 2) | (R.c >> 62)) & p.mb, (R.c << 2) & p.mc};
    i = j + (uint32_t)(p.K - 1);
  }
  __device__ __forceinline__ void step(const KeyP& p) {
    const uint64_t b = read_base(rd, i);
    fw = push_right(fw, b, p);
    rc = rc_roll(rc, b, p);
    ++i;
  }
  __device__ __forceinline__ bool more() const { return i < len; }
  // reposition so that the next step() completes the K-mer starting at base j
  __device__ __forceinline__ void seek(uint32_t j, const KeyP& p) { prime(j, p); }
  // next K-mer instance as a KRec
  __device__ __forceinline__ KRec next(const KeyP& p) {
    step(p);
    const uint32_t j = i - p.K;  // start of this K-mer
    const int a = j > 0 ? (int)read_base(rd, j - 1) : -1;
    const int b = i < len ? (int)read_base(rd, i) : -1;
    K3 key;
    uint32_t ext;
    canon_ext(fw, rc, a, b, &key, &ext);
    return KRec{key.a, key.b, key.c, key_hash(key) | ext};
  }
};

// ---------------------------------------------------------------------------
// U1-U3: distinct nodes through one global open-addressing table.
//
// Every K-mer instance (rolled from the reads, or a received record) is
// inserted into a table of 64-byte slots {tag, key, hash56 | OR of extension
// bits}; tag 0 = empty, hash56 | 1 = being written, hash56 | 2 = published.
// An instance probes from mulhi(hash, T), loading tag and key of a slot in
// one round trip: an empty slot is claimed by CAS on the tag, the key
// written with coherent stores and the tag published; a published slot with
// the same hash and key gets the instance's extension bits OR-ed in (only
// when new).  All table traffic uses agent-scope (cross-XCD coherent)
// accesses, no cache-maintenance fences.  With coverage c the table sees c
// reads per write, so the 1.7 G x 32-byte instances of the bench never touch
// HBM as records: only the reads (0.9 GB) and one slot line per probe move.
// The probe loop is wave-uniform (one probe per pending lane per trip) so a
// lane waiting on a slot another lane of its own wave is writing never
// blocks that writer.  A distinct-count estimate (HyperLogLog over the same
// hash, taken in the sizing pass) sets T ~ 2x distinct; a probe run longer
// than kMaxProbe marks overflow and the host rebuilds with 2T.
// ---------------------------------------------------------------------------
constexpr int kUThreads = 256;
constexpr int kUDigitBits = 5;  // node groups (top hash bits): shard-major order for the exchange
constexpr int kHllBits = 12;    // 4096 HyperLogLog registers
constexpr uint32_t kMaxProbe = 1u << 14;

// One table slot per 64-byte line: a probe's tag and key share one HBM access.
struct __attribute__((aligned(64))) USlot {
  uint64_t k0, k1, k2, meta;
  unsigned long long tag;  // 0 empty, hash56 | 1 being written, hash56 | 2 published
  uint64_t pad[3];
};

struct UTab {
  USlot* slot;
  uint64_t T;
  unsigned long long* ovf;  // [0] overflow flag, [1] probes (one 64-byte slot line each)
};

__device__ __forceinline__ uint64_t tab_home(uint64_t h, uint64_t T) { return __umul64hi(h, T); }

// Table words are read and written with agent-scope (cross-XCD coherent)
// loads/stores instead of cache-invalidating acquire/release fences: a slot's
// key is written once, before its tag is published, and never changes.
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld_agent64(const uint64_t* p) {
  return (uint64_t)ld_agent(reinterpret_cast<const unsigned long long*>(p));
}
__device__ __forceinline__ void st_agent64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// One probe step of a pending instance (key k, hash h with low byte 0,
// extension bits e) at slot *s, given the slot's view.  Returns true when the
// instance is settled.
//
// Fast path: one plain (L2-cacheable, wide) read of the slot line.  A
// published slot never changes key, so a line cached after the publish is
// exact; a line cached before it shows the tag as empty or busy, which sends
// the probe down the coherent path (CAS / agent-scope re-read).  `coh` makes
// the next probe of a busy slot coherent, so a stale "busy" cannot loop.
// The slot line as the probe sees it (plain or coherent read).
struct SlotView {
  uint64_t a, b, c, m;
  unsigned long long tag;
};

__device__ __forceinline__ SlotView slot_read(const USlot* sl, bool coh) {
  if (coh)
    return SlotView{ld_agent64(&sl->k0), ld_agent64(&sl->k1), ld_agent64(&sl->k2), ld_agent64(&sl->meta),
                    ld_agent(&sl->tag)};
  // the 40 used bytes only (two 16-byte and one 8-byte load), not the pad
  const uint4* q = reinterpret_cast<const uint4*>(sl);
  const uint4 a = q[0], b = q[1];
  const unsigned long long t = sl->tag;
  return SlotView{(uint64_t)a.x | ((uint64_t)a.y << 32), (uint64_t)a.z | ((uint64_t)a.w << 32),
                  (uint64_t)b.x | ((uint64_t)b.y << 32), (uint64_t)b.z | ((uint64_t)b.w << 32), t};
}

// Settle (or advance) one probe given the slot view v read at *s.
__device__ __forceinline__ bool tab_probe(const UTab& t, const K3& k, uint64_t h, uint32_t e, uint64_t* s,
                                          uint32_t* probes, bool* coh, const SlotView& v) {
  USlot* sl = t.slot + *s;
  unsigned long long cur = v.tag;
  uint64_t a = v.a, b = v.b, c = v.c, m = v.m;
  if (cur == 0) {
    const unsigned long long prev = atomicCAS(&sl->tag, 0ull, (unsigned long long)(h | 1));
    if (prev == 0) {
      st_agent64(&sl->k0, k.a);
      st_agent64(&sl->k1, k.b);
      st_agent64(&sl->k2, k.c);
      st_agent64(&sl->meta, h | e);
      // the four coherent stores complete before the tag is published
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __hip_atomic_store(&sl->tag, (unsigned long long)(h | 2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
    cur = prev;  // coherent: the key is re-read below if it must be compared
    a = b = c = ~0ull;
  }
  if ((cur & ~0xffull) == h) {
    if ((cur & 0xff) == 1) {  // being written: look again next trip, coherently
      *coh = true;
      return false;
    }
    if (!((a == k.a) & (b == k.b) & (c == k.c))) {  // stale line or a true hash collision: re-read
      a = ld_agent64(&sl->k0);
      b = ld_agent64(&sl->k1);
      c = ld_agent64(&sl->k2);
      m = ld_agent64(&sl->meta);
    }
    if ((a == k.a) & (b == k.b) & (c == k.c)) {
      if (e & ~(uint32_t)m & 0xff) atomicOr(reinterpret_cast<unsigned long long*>(&sl->meta), (unsigned long long)e);
      return true;
    }
  }
  *coh = false;
  *s = *s + 1 == t.T ? 0 : *s + 1;
  if (++*probes > kMaxProbe) {
    atomicOr(t.ovf, 1ull);
    return true;  // dropped: the host rebuilds with a larger table
  }
  return false;
}

// Sizing pass: instance count and HyperLogLog registers of the key hashes.
__global__ void __launch_bounds__(kUThreads) k_uhll(ReadsV rv, KeyP kp, uint32_t* __restrict__ hll,
                                                   unsigned long long* __restrict__ n_inst) {
  __shared__ uint32_t reg[1 << kHllBits];
  for (uint32_t i = threadIdx.x; i < (1u << kHllBits); i += blockDim.x) reg[i] = 0;
  __syncthreads();
  unsigned long long cnt = 0;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rv.n_reads;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t len = (uint32_t)(rv.base_off[r + 1] - rv.base_off[r]);
    if (len < (uint32_t)kp.K) continue;
    Roller3 ro;
    ro.init(rv.packed + rv.byte_off[r], len, kp);
    while (ro.more()) {
      const uint64_t h = ro.next(kp).meta & ~0xffull;
      const uint32_t j = (uint32_t)(h >> (64 - kHllBits));
      const uint32_t rho = (uint32_t)__clzll((long long)((h << kHllBits) | (1ull << (kHllBits + 7)))) + 1;
      atomicMax(&reg[j], rho);
      ++cnt;
    }
  }
  wave_add(n_inst, cnt);
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < (1u << kHllBits); i += blockDim.x)
    if (reg[i]) atomicMax(&hll[i], reg[i]);
}

// Insert every K-mer instance of the reads.  Each lane keeps kPend
// instances in flight: per trip it refills its empty entries from its read
// (rolling; next read when exhausted), issues all their slot reads, then
// settles them — kPend slot lines in flight per lane instead of one.
constexpr int kPend = 1;  // measured: 4 in flight (142 VGPRs, 3 waves/SIMD) is slower than 1 at 8 waves

__global__ void __launch_bounds__(kUThreads) k_uinsert_reads(ReadsV rv, KeyP kp, UTab t) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  Roller3 ro;
  ro.i = ro.len = 0;
  bool started = false, live = true;
  unsigned long long n_probe = 0;
  bool pend[kPend], coh[kPend];
  K3 k[kPend];
  uint64_t h[kPend], s[kPend];
  uint32_t e[kPend], probes[kPend];
#pragma unroll
  for (int q = 0; q < kPend; ++q) {
    pend[q] = coh[q] = false;
    h[q] = s[q] = 0;
    e[q] = probes[q] = 0;
    k[q] = K3{0, 0, 0};
  }
  for (;;) {
#pragma unroll
    for (int q = 0; q < kPend; ++q) {
      while (!pend[q] && live) {  // per lane: next instance, or next read
        if (started && ro.more()) {
          const KRec x = ro.next(kp);
          k[q] = rec_key(x);
          h[q] = x.meta & ~0xffull;
          e[q] = (uint32_t)(x.meta & 0xff);
          s[q] = tab_home(h[q], t.T);
          probes[q] = 0;
          coh[q] = false;
          pend[q] = true;
        } else {
          if (started) r += stride;
          started = true;
          if (r >= rv.n_reads) {
            live = false;
          } else {
            const uint32_t len = (uint32_t)(rv.base_off[r + 1] - rv.base_off[r]);
            ro.i = ro.len = 0;
            if (len >= (uint32_t)kp.K) ro.init(rv.packed + rv.byte_off[r], len, kp);
          }
        }
      }
    }
    bool any = false;
#pragma unroll
    for (int q = 0; q < kPend; ++q) any |= pend[q];
    if (!__ballot(any)) break;
    SlotView v[kPend];
#pragma unroll
    for (int q = 0; q < kPend; ++q)
      if (pend[q]) v[q] = slot_read(t.slot + s[q], coh[q]);
#pragma unroll
    for (int q = 0; q < kPend; ++q) {
      n_probe += pend[q];
      if (pend[q] && tab_probe(t, k[q], h[q], e[q], &s[q], &probes[q], &coh[q], v[q])) pend[q] = false;
    }
  }
  wave_add(t.ovf + 1, n_probe);
}

// Insert records (32-byte KRec with extension bits), e.g. received nodes.
__global__ void __launch_bounds__(kUThreads) k_uinsert_recs(const KRec* __restrict__ rec, uint64_t n, UTab t) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  bool pend = false;
  K3 k{0, 0, 0};
  uint64_t h = 0, s = 0;
  uint32_t e = 0, probes = 0;
  bool coh = false;
  unsigned long long n_probe = 0;
  for (;;) {
    if (!pend && i < n) {
      const KRec x = rec[i];
      i += stride;
      k = rec_key(x);
      h = x.meta & ~0xffull;
      e = (uint32_t)(x.meta & 0xff);
      s = tab_home(h, t.T);
      probes = 0;
      coh = false;
      pend = true;
    }
    if (!__ballot(pend)) break;
    n_probe += pend;
    if (pend && tab_probe(t, k, h, e, &s, &probes, &coh, slot_read(t.slot + s, coh))) pend = false;
  }
  wave_add(t.ovf + 1, n_probe);
}

// Compaction: published slots grouped by the top kUDigitBits hash bits.
// Pass 1 counts per (digit, block) into cmat[digit * G + block].
__global__ void __launch_bounds__(kUThreads) k_tab_count(const USlot* __restrict__ slot, uint64_t T,
                                                        uint32_t* __restrict__ cmat) {
  __shared__ uint32_t hist[1 << kUDigitBits];
  const uint32_t G = gridDim.x, b = blockIdx.x;
  if (threadIdx.x < (1u << kUDigitBits)) hist[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t s0 = T * b / G, s1 = T * (b + 1) / G;
  for (uint64_t s = s0 + threadIdx.x; s < s1; s += blockDim.x) {
    const unsigned long long x = slot[s].tag;
    if (x) atomicAdd(&hist[x >> (64 - kUDigitBits)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < (1u << kUDigitBits)) cmat[(uint64_t)threadIdx.x * G + b] = hist[threadIdx.x];
}

__global__ void __launch_bounds__(kUThreads) k_tab_scatter(const USlot* __restrict__ slot, uint64_t T,
                                                          const uint64_t* __restrict__ omat, KRec* __restrict__ out) {
  __shared__ unsigned long long cur[1 << kUDigitBits];
  const uint32_t G = gridDim.x, b = blockIdx.x;
  if (threadIdx.x < (1u << kUDigitBits)) cur[threadIdx.x] = omat[(uint64_t)threadIdx.x * G + b];
  __syncthreads();
  const uint64_t s0 = T * b / G, s1 = T * (b + 1) / G;
  for (uint64_t s = s0 + threadIdx.x; s < s1; s += blockDim.x) {
    const USlot& x = slot[s];
    if (x.tag) out[atomicAdd(&cur[x.tag >> (64 - kUDigitBits)], 1ull)] = KRec{x.k0, x.k1, x.k2, x.meta};
  }
}

__global__ void k_digit_starts_u(const uint64_t* __restrict__ omat, uint32_t ndig, uint32_t G,
                                 uint64_t* __restrict__ ds) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d <= ndig) ds[d] = omat[(uint64_t)d * G];
}

// Node index: open addressing over 64-bit slots {32 tag bits of the key hash,
// node id}, linear probing from the hash's low bits.  A probe reads the node
// record only when the tag matches, so a lookup is one slot read and
// (almost always) one record read, where id-only slots made every probe of a
// collision chain a dependent slot + record pair.
constexpr uint64_t kIdxEmpty = ~0ull;
__device__ __forceinline__ uint32_t idx_tag(uint64_t h56) { return (uint32_t)(h56 >> 24); }

// nodes [i0, N) into the index
__global__ void k_node_insert(const KRec* __restrict__ nodes, uint64_t i0, uint64_t N,
                              unsigned long long* __restrict__ idx, uint64_t tmask) {
  for (uint64_t i = i0 + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t h = nodes[i].meta >> 8;
    const unsigned long long want = ((unsigned long long)idx_tag(h) << 32) | i;  // i < 2^31: never empty
    uint64_t s = h & tmask;
    while (atomicCAS(&idx[s], kIdxEmpty, want) != kIdxEmpty) s = (s + 1) & tmask;
  }
}

struct NodeIdx {
  const KRec* nodes;
  const unsigned long long* idx;
  uint64_t tmask;
  __device__ __forceinline__ uint32_t find(const K3& k) const {
    const uint64_t h = key_hash(k) >> 8;
    const uint32_t tag = idx_tag(h);
    uint64_t s = h & tmask;
    for (;;) {
      const unsigned long long e = idx[s];
      if (e == kIdxEmpty) return kNone;
      if ((uint32_t)(e >> 32) == tag) {
        const uint32_t i = (uint32_t)e;
        const KRec& r = nodes[i];
        if (r.k0 == k.a && r.k1 == k.b && r.k2 == k.c) return i;
      }
      s = (s + 1) & tmask;
    }
  }
};

__device__ __forceinline__ K3 dseq(const KRec* nodes, uint32_t v, const KeyP& p) {
  const K3 k = rec_key(nodes[v >> 1]);
  return (v & 1) ? revcomp(k, p) : k;
}
__device__ __forceinline__ uint32_t out_set(uint32_t ext, uint32_t o) { return o ? comp4(ext & 15) : (ext >> 4); }
__device__ __forceinline__ uint32_t in_set(uint32_t ext, uint32_t o) { return o ? comp4(ext >> 4) : (ext & 15); }

// directed node whose sequence is s (kNone if absent)
__device__ __forceinline__ uint32_t directed_of(const NodeIdx& ni, const K3& s, const KeyP& p) {
  const K3 r = revcomp(s, p);
  const bool fw = !k3_lt(r, s);
  const uint32_t n = ni.find(fw ? s : r);
  return n == kNone ? kNone : 2 * n + (fw ? 0 : 1);
}

// ---------------------------------------------------------------------------
// U5: unique links
// ---------------------------------------------------------------------------
// Per directed node ranking state, one 16-byte record: a walk step touches
// one cache line instead of four arrays.
struct DN {
  uint32_t nxt, prv, ruler, lrank;
};

// Unique links resolved inside a bucket (k_usk_bucket, lsucc): a K-mer's
// successor in a read almost always has the same minimizer, so it is in the
// same bucket's LDS table.  Per node and orientation: the successor directed
// node (2 * id + orientation), kNone (no unique link: the rules of k_links),
// or kLsGlobal (the successor is in another bucket: k_links looks it up in
// the node index).
constexpr uint32_t kLsGlobal = 0xfefefefeu;  // > any directed node id (N < kLsMaxNodes)
constexpr uint64_t kLsMaxNodes = 0x7f000000ull;

// lsucc (may be null): links the node buckets resolved (k_usk_bucket); only
// kLsGlobal orientations are looked up here.
__global__ void k_links(NodeIdx ni, uint64_t N, KeyP kp, DN* __restrict__ dn, unsigned long long* __restrict__ stat,
                        const uint2* __restrict__ lsucc) {
  unsigned long long nl = 0, bad = 0, ng = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint2 ls = lsucc ? lsucc[i] : make_uint2(kLsGlobal, kLsGlobal);
#pragma unroll
    for (uint32_t o = 0; o < 2; ++o) {
      const uint32_t w = o ? ls.y : ls.x;
      if (w >= kLsGlobal) continue;  // kNone, kLsGlobal
      dn[2 * i + o].nxt = w;
      dn[w].prv = (uint32_t)(2 * i + o);
      ++nl;
    }
    if (ls.x != kLsGlobal && ls.y != kLsGlobal) continue;
    const KRec x = ni.nodes[i];
    const K3 key = rec_key(x);
    if (k3_eq(key, revcomp(key, kp))) continue;  // palindromic K-mers never link
    const uint32_t ext = (uint32_t)(x.meta & 0xff);
    for (uint32_t o = 0; o < 2; ++o) {
      if ((o ? ls.y : ls.x) != kLsGlobal) continue;
      const uint32_t out = out_set(ext, o);
      if (__popc(out) != 1) continue;
      ++ng;
      const uint32_t b = __ffs(out) - 1;
      const K3 s = o ? revcomp(key, kp) : key;
      const K3 t = push_right(s, b, kp);
      const uint32_t w = directed_of(ni, t, kp);
      if (w == kNone) {
        ++bad;
        continue;
      }
      const K3 wk = rec_key(ni.nodes[w >> 1]);
      if (k3_eq(wk, revcomp(wk, kp))) continue;
      const uint32_t wext = (uint32_t)(ni.nodes[w >> 1].meta & 0xff);
      if (__popc(in_set(wext, w & 1)) != 1) continue;
      dn[2 * i + o].nxt = w;
      dn[w].prv = (uint32_t)(2 * i + o);
      ++nl;
    }
  }
  for (int s = 32; s > 0; s >>= 1) {
    nl += __shfl_down(nl, s, 64);
    bad += __shfl_down(bad, s, 64);
    ng += __shfl_down(ng, s, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    if (nl) atomicAdd(&stat[0], nl);
    if (bad) atomicAdd(&stat[1], bad);
    if (ng) atomicAdd(&stat[2], ng);
  }
}

// ---------------------------------------------------------------------------
// U6: ranking (ruling set + pointer jumping), cycle cutting
// ---------------------------------------------------------------------------
constexpr uint32_t kRulerMask = 31;  // sampled rulers: 1 in 32

__device__ __forceinline__ bool is_ruler(uint32_t v, const DN* dn) {
  return dn[v].prv == kNone || ((uint32_t)fmix64(v) & kRulerMask) == 0;
}

struct RankBufs {
  DN* dn;
  uint32_t *rnext, *seglen;
  unsigned long long* state;  // per ruler: x (ptr or head) | done << 32 | off << 33
  uint32_t *rlist, *alist0, *alist1;
};

__device__ __forceinline__ unsigned long long st_pack(uint32_t x, bool done, uint64_t off) {
  return (unsigned long long)x | ((unsigned long long)done << 32) | ((unsigned long long)off << 33);
}
__device__ __forceinline__ uint32_t st_x(unsigned long long s) { return (uint32_t)s; }
__device__ __forceinline__ bool st_done(unsigned long long s) { return (s >> 32) & 1; }
__device__ __forceinline__ uint64_t st_off(unsigned long long s) { return s >> 33; }

constexpr int kTI = 16;                 // items per thread per tile
constexpr uint64_t kTileN = 256 * kTI;  // items per block tile (one append atomic each)

__global__ void __launch_bounds__(256) k_find_rulers(uint64_t D, RankBufs rb, unsigned long long* __restrict__ nrul) {
  __shared__ uint32_t sm[64];
  __shared__ unsigned long long sb;
  const uint64_t ntiles = (D + kTileN - 1) / kTileN;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    uint32_t flags = 0, cnt = 0;
#pragma unroll
    for (int i = 0; i < kTI; ++i) {
      const uint64_t v = t * kTileN + (uint64_t)i * 256 + threadIdx.x;
      if (v < D) {
        rb.dn[v].ruler = kNone;
        if (is_ruler((uint32_t)v, rb.dn)) {
          flags |= 1u << i;
          ++cnt;
        }
      }
    }
    unsigned long long j = block_append(nrul, cnt, sm, &sb);
#pragma unroll
    for (int i = 0; i < kTI; ++i)
      if (flags & (1u << i)) rb.rlist[j++] = (uint32_t)(t * kTileN + (uint64_t)i * 256 + threadIdx.x);
  }
}

// Each ruler walks its segment (up to the next ruler / end): one thread per
// ruler, so every lane of a wave walks.
__global__ void k_walk(uint64_t R, uint64_t D, RankBufs rb) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < R; i += (uint64_t)gridDim.x * blockDim.x) {
    // one dependent load per step: the successor's whole record is read once,
    // for its ruler test (prv) and as the next step's state; the sampled
    // ruler test (hash bits) needs no load
    const uint32_t v = rb.rlist[i];
    uint32_t x = v, r = 0;
    uint32_t y = rb.dn[v].nxt;
    for (uint64_t guard = 0; guard <= D; ++guard) {
      rb.dn[x].ruler = v;
      rb.dn[x].lrank = r++;
      if (y == kNone || ((uint32_t)fmix64(y) & kRulerMask) == 0) {
        rb.rnext[v] = y;
        break;
      }
      const DN ny = rb.dn[y];
      if (ny.prv == kNone) {  // a head (is_ruler's other case)
        rb.rnext[v] = y;
        break;
      }
      x = y;
      y = ny.nxt;
    }
    rb.seglen[v] = r;
  }
}

// every ruler starts as a finished head; ruler successors are then linked
__global__ void k_ruler_state0(uint64_t R, RankBufs rb) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < R; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = rb.rlist[i];
    rb.state[r] = st_pack(r, true, 0);
  }
}
__global__ void __launch_bounds__(256) k_ruler_state1(uint64_t R, RankBufs rb, unsigned long long* __restrict__ nact) {
  __shared__ uint32_t sm[64];
  __shared__ unsigned long long sb;
  const uint64_t ntiles = (R + kTileN - 1) / kTileN;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    uint32_t flags = 0, cnt = 0;
    uint32_t ss[kTI];
#pragma unroll
    for (int i = 0; i < kTI; ++i) {
      const uint64_t k = t * kTileN + (uint64_t)i * 256 + threadIdx.x;
      ss[i] = kNone;
      if (k < R) {
        const uint32_t r = rb.rlist[k];
        const uint32_t s = rb.rnext[r];  // a ruler whose unique ruler predecessor is r
        if (s != kNone) {
          rb.state[s] = st_pack(r, false, rb.seglen[r]);
          ss[i] = s;
          flags |= 1u << i;
          ++cnt;
        }
      }
    }
    unsigned long long j = block_append(nact, cnt, sm, &sb);
#pragma unroll
    for (int i = 0; i < kTI; ++i)
      if (flags & (1u << i)) rb.alist0[j++] = ss[i];
  }
}

// Asynchronous pointer jumping over the still-active rulers.  A state word is
// a consistent (pointer, distance) pair read and written as one 8-byte
// access, so a stale read is still a valid jump.
// nin: the active-list length on the device (the previous round's nout), so
// rounds queue back to back without a host read of each count
__global__ void __launch_bounds__(256) k_ruler_jump(const unsigned long long* __restrict__ nin,
                                                    const uint32_t* __restrict__ ain,
                                                    unsigned long long* __restrict__ state, uint32_t* __restrict__ aout,
                                                    unsigned long long* __restrict__ nout) {
  __shared__ uint32_t sm[64];
  __shared__ unsigned long long sb;
  const uint64_t n = *nin;
  const uint64_t ntiles = (n + kTileN - 1) / kTileN;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    uint32_t flags = 0, cnt = 0;
    uint32_t rr[kTI];
#pragma unroll
    for (int i = 0; i < kTI; ++i) {
      const uint64_t k = t * kTileN + (uint64_t)i * 256 + threadIdx.x;
      rr[i] = 0;
      if (k < n) {
        const uint32_t r = ain[k];
        const unsigned long long s = __hip_atomic_load(&state[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long q = __hip_atomic_load(&state[st_x(s)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&state[r], st_pack(st_x(q), st_done(q), st_off(s) + st_off(q)), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        rr[i] = r;
        if (!st_done(q)) {
          flags |= 1u << i;
          ++cnt;
        }
      }
    }
    unsigned long long j = block_append(nout, cnt, sm, &sb);
#pragma unroll
    for (int i = 0; i < kTI; ++i)
      if (flags & (1u << i)) aout[j++] = rr[i];
  }
}

// cyclic directed nodes: unvisited, or on a ruler that never reached a head
// cyclic directed nodes (unvisited, or on a ruler that never reached a head)
// to clist; every other node's head, rank and (at a chain's tail) the chain
// length and tail in the same pass — when no node is cyclic (the rule) the
// ranking is final, and after a cycle cut the pass runs again
__global__ void __launch_bounds__(256) k_rank_mark(uint64_t D, RankBufs rb, uint32_t* __restrict__ clist,
                                                   unsigned long long* __restrict__ ncyc, uint32_t* __restrict__ head,
                                                   uint32_t* __restrict__ rank, uint32_t* __restrict__ chainlen,
                                                   uint32_t* __restrict__ tail_of) {
  __shared__ uint32_t sm[64];
  __shared__ unsigned long long sb;
  const uint64_t ntiles = (D + kTileN - 1) / kTileN;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    uint32_t flags = 0, cnt = 0;
#pragma unroll
    for (int i = 0; i < kTI; ++i) {
      const uint64_t v = t * kTileN + (uint64_t)i * 256 + threadIdx.x;
      if (v < D) {
        const DN d = rb.dn[v];
        const unsigned long long s = d.ruler == kNone ? 0ull : rb.state[d.ruler];
        if (d.ruler == kNone || !st_done(s)) {
          flags |= 1u << i;
          ++cnt;
        } else {
          const uint32_t h = st_x(s);
          const uint32_t k = (uint32_t)(st_off(s) + d.lrank);
          head[v] = h;
          rank[v] = k;
          if (d.nxt == kNone) {
            chainlen[h] = k + 1;
            tail_of[h] = (uint32_t)v;
          }
        }
      }
    }
    unsigned long long j = block_append(ncyc, cnt, sm, &sb);
#pragma unroll
    for (int i = 0; i < kTI; ++i)
      if (flags & (1u << i)) clist[j++] = (uint32_t)(t * kTileN + (uint64_t)i * 256 + threadIdx.x);
  }
}

__device__ __forceinline__ uint32_t seq_min(const KRec* nodes, uint32_t x, uint32_t y, const KeyP& p) {
  return k3_lt(dseq(nodes, y, p), dseq(nodes, x, p)) ? y : x;
}
__global__ void k_cyc_init(uint64_t C, const uint32_t* __restrict__ clist, const DN* __restrict__ dn,
                           uint32_t* __restrict__ cm, uint32_t* __restrict__ cn) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < C; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = clist[i];
    cm[v] = v;
    cn[v] = dn[v].nxt;
  }
}
__global__ void k_cyc_jump(uint64_t C, const uint32_t* __restrict__ clist, const KRec* __restrict__ nodes, KeyP kp,
                           const uint32_t* __restrict__ cm0, const uint32_t* __restrict__ cn0, uint32_t* __restrict__ cm1,
                           uint32_t* __restrict__ cn1) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < C; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = clist[i];
    const uint32_t n = cn0[v];
    cm1[v] = seq_min(nodes, cm0[v], cm0[n], kp);
    cn1[v] = cn0[n];
  }
}
// Cut each (C, rc C) pair once, before the smaller of the two cycles' minima.
__global__ void k_cyc_cut(uint64_t C, const uint32_t* __restrict__ clist, const KRec* __restrict__ nodes, KeyP kp,
                          const uint32_t* __restrict__ cm, DN* __restrict__ dn,
                          unsigned long long* __restrict__ ncut) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < C; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = clist[i];
    if (cm[v] != v) continue;
    const uint32_t mr = cm[v ^ 1];
    if (mr != v && !k3_lt(dseq(nodes, v, kp), dseq(nodes, mr, kp))) continue;
    const uint32_t p = dn[v].prv;
    const bool mirror = dn[v ^ 1].nxt == (p ^ 1) && (v ^ 1) != p;
    dn[p].nxt = kNone;
    dn[v].prv = kNone;
    if (mirror) {
      dn[v ^ 1].nxt = kNone;
      dn[p ^ 1].prv = kNone;
    }
    atomicAdd(ncut, 1ull);
  }
}

// final per-node head and rank; tails record their chain's length
// ---------------------------------------------------------------------------
// U7: unipath pairs and their order
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool pair_emit(uint32_t h, const DN* dn, const uint32_t* tail_of, const KRec* nodes,
                                          const KeyP& kp) {
  if (dn[h].prv != kNone) return false;
  const uint32_t rh = tail_of[h] ^ 1;  // head of the rc path
  if (rh == h) return true;            // palindromic path: its own partner
  // once per (u, rc u): smaller head K-mer; equal only for a palindromic K-mer's two nodes
  const K3 hs = dseq(nodes, h, kp), rs = dseq(nodes, rh, kp);
  return k3_lt(hs, rs) || (k3_eq(hs, rs) && h < rh);
}

__global__ void __launch_bounds__(256) k_pairs(uint64_t D, const DN* __restrict__ dn,
                                               const uint32_t* __restrict__ tail_of, const KRec* __restrict__ nodes,
                                               KeyP kp, uint64_t* __restrict__ pk0, uint64_t* __restrict__ pk1,
                                               uint64_t* __restrict__ pk2, uint32_t* __restrict__ ph,
                                               unsigned long long* __restrict__ np, unsigned long long* __restrict__ nu) {
  __shared__ uint32_t sm[64];
  __shared__ unsigned long long sb;
  unsigned long long units = 0;
  const uint64_t ntiles = (D + kTileN - 1) / kTileN;
  for (uint64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    uint32_t flags = 0, cnt = 0;
#pragma unroll
    for (int i = 0; i < kTI; ++i) {
      const uint64_t v = t * kTileN + (uint64_t)i * 256 + threadIdx.x;
      if (v < D && pair_emit((uint32_t)v, dn, tail_of, nodes, kp)) {
        flags |= 1u << i;
        ++cnt;
      }
    }
    unsigned long long j = block_append(np, cnt, sm, &sb);
#pragma unroll
    for (int i = 0; i < kTI; ++i) {
      if (!(flags & (1u << i))) continue;
      const uint32_t h = (uint32_t)(t * kTileN + (uint64_t)i * 256 + threadIdx.x);
      const K3 hs = dseq(nodes, h, kp);
      pk0[j] = hs.a;
      pk1[j] = hs.b;
      pk2[j] = hs.c;
      ph[j] = h;
      ++j;
      units += (tail_of[h] ^ 1) == h ? 1 : 2;
    }
  }
  wave_add(nu, units);
}

// Stable LSD radix pass over (key, payload) columns: digit = (key[sel] >> shift) & 255.
constexpr int kSortThreads = 256;
constexpr int kSortTile = 4096;

__global__ void __launch_bounds__(kSortThreads) k_lsd_count(const uint64_t* __restrict__ key, uint64_t n, int shift,
                                                            uint32_t* __restrict__ cmat) {
  __shared__ uint32_t hist[256];
  const uint32_t G = gridDim.x, b = blockIdx.x;
  hist[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t s = (uint64_t)b * kSortTile, e = min(n, s + kSortTile);
  for (uint64_t i = s + threadIdx.x; i < e; i += kSortThreads) atomicAdd(&hist[(key[i] >> shift) & 255], 1u);
  __syncthreads();
  cmat[(uint64_t)threadIdx.x * G + b] = hist[threadIdx.x];
}

struct SortCols {
  const uint64_t *k0, *k1, *k2;
  const uint32_t* pay;
  uint64_t *o0, *o1, *o2;
  uint32_t* opay;
};

// omat: the scanned count matrix, or null: the block's digit bases from the
// raw counts cmat (few tiles: every block reads the whole matrix, no scan
// launches — the pass is launch-bound at the unipath counts of a genome)
constexpr uint32_t kSortFuseTiles = 128;
__global__ void __launch_bounds__(kSortThreads) k_lsd_scatter(SortCols c, int sel, uint64_t n, int shift,
                                                              const uint64_t* __restrict__ omat,
                                                              const uint32_t* __restrict__ cmat) {
  constexpr int nw = kSortThreads / 64;
  __shared__ uint32_t wh[nw][256];
  __shared__ unsigned long long base[256];
  const uint32_t G = gridDim.x, b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t s = (uint64_t)b * kSortTile, e = min(n, s + kSortTile);
  const uint32_t tn = (uint32_t)(e - s);
  const uint64_t* key = sel == 0 ? c.k0 : sel == 1 ? c.k1 : c.k2;
  if (omat) {
    base[threadIdx.x] = omat[(uint64_t)threadIdx.x * G + b];
  } else {
    // digit d = thread: its total over all tiles and over the tiles before b
    const uint32_t* row = cmat + (uint64_t)threadIdx.x * G;
    uint32_t tot = 0, before = 0;
    for (uint32_t q = 0; q < G; ++q) {
      const uint32_t x = row[q];
      tot += x;
      before += q < b ? x : 0u;
    }
    wh[0][threadIdx.x] = tot;
    __syncthreads();
    if (threadIdx.x == 0) {  // 256 digit totals, exclusive scan
      unsigned long long run = 0;
      for (int d = 0; d < 256; ++d) {
        const uint32_t x = wh[0][d];
        base[d] = run;
        run += x;
      }
    }
    __syncthreads();
    base[threadIdx.x] += before;
    __syncthreads();  // wh is cleared below
  }
  for (int d = lane; d < 256; d += 64) wh[w][d] = 0;
  const uint32_t rows = (tn + 63) / 64, rpw = (rows + nw - 1) / nw;
  const uint32_t r0 = min(rows, w * rpw), r1 = min(rows, r0 + rpw);
  const uint64_t lt = (1ull << lane) - 1;
  for (uint32_t r = r0; r < r1; ++r) {
    const uint32_t idx = r * 64 + lane;
    const bool valid = idx < tn;
    const uint32_t d = valid ? (uint32_t)((key[s + idx] >> shift) & 255) : 0;
    const uint64_t peers = wave_match(d, valid, 8);
    if (valid && (peers & lt) == 0) wh[w][d] += __popcll(peers);
  }
  __syncthreads();
  {  // wave offsets within the block, in wave order (stability)
    const uint32_t d = threadIdx.x;
    uint32_t run = 0;
    for (int k = 0; k < nw; ++k) {
      const uint32_t x = wh[k][d];
      wh[k][d] = run;
      run += x;
    }
  }
  __syncthreads();
  for (uint32_t r = r0; r < r1; ++r) {
    const uint32_t idx = r * 64 + lane;
    const bool valid = idx < tn;
    const uint32_t d = valid ? (uint32_t)((key[s + idx] >> shift) & 255) : 0;
    const uint64_t peers = wave_match(d, valid, 8);
    if (valid) {
      const uint64_t pos = base[d] + wh[w][d] + __popcll(peers & lt);
      c.o0[pos] = c.k0[s + idx];
      c.o1[pos] = c.k1[s + idx];
      c.o2[pos] = c.k2[s + idx];
      c.opay[pos] = c.pay[s + idx];
    }
    __builtin_amdgcn_wave_barrier();
    if (valid && (peers & lt) == 0) wh[w][d] += __popcll(peers);
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ void k_digit_or(const uint64_t* __restrict__ k0, const uint64_t* __restrict__ k1,
                           const uint64_t* __restrict__ k2, uint64_t n, unsigned long long* __restrict__ orv,
                           unsigned long long* __restrict__ andv) {
  unsigned long long o[3] = {0, 0, 0}, a[3] = {~0ull, ~0ull, ~0ull};
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    o[0] |= k0[i];
    o[1] |= k1[i];
    o[2] |= k2[i];
    a[0] &= k0[i];
    a[1] &= k1[i];
    a[2] &= k2[i];
  }
  for (int j = 0; j < 3; ++j) {
    atomicOr(&orv[j], o[j]);
    atomicAnd(&andv[j], a[j]);
  }
}

// The pair-key sort's one-pass form (u_sort_keys): keys binned by their most
// significant varying bits, each bin ranked in LDS by full 192-bit
// comparison with ties by input position — the same order as the stable LSD
// passes, in a handful of launches instead of ~22 launch-bound passes.
// The bin digit: bits [lo, lo + bits) of the most significant varying key
// word, which the host hands over as its own pointer `kw` (a per-thread
// select among the three words, uniform as it is, was compiled on gfx950
// into a path that loaded through an unset address register for word 2).
struct MsdDigit {
  int lo;  // lowest bit of the bin digit
  uint32_t mask;
};
__device__ __forceinline__ uint32_t msd_bin(const uint64_t* kw, uint64_t i, MsdDigit d) {
  return (uint32_t)(kw[i] >> d.lo) & d.mask;
}
__global__ void k_msd_count(const uint64_t* __restrict__ kw, uint64_t n, MsdDigit d, uint32_t* __restrict__ cnt) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[msd_bin(kw, i, d)], 1u);
}
// bin cursors start at 0 (cur zeroed); the largest bin goes to *mx
__global__ void k_msd_scatter(SortCols c, const uint64_t* __restrict__ kw, uint64_t n, MsdDigit d,
                              const uint64_t* __restrict__ off, uint32_t* __restrict__ cur, uint32_t* __restrict__ sidx,
                              const uint32_t* __restrict__ cnt, uint64_t nbins, unsigned int* __restrict__ mx) {
  const uint64_t t0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, st = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = t0; i < n; i += st) {
    const uint32_t b = msd_bin(kw, i, d);
    const uint64_t pos = off[b] + atomicAdd(&cur[b], 1u);
    if (pos >= n) {  // cannot happen with consistent counts; refuses the one-pass form
      atomicMax(mx, 0xffffffffu);
      continue;
    }
    c.o0[pos] = c.k0[i];
    c.o1[pos] = c.k1[i];
    c.o2[pos] = c.k2[i];
    c.opay[pos] = c.pay[i];
    sidx[pos] = (uint32_t)i;
  }
  unsigned int m = 0;
  for (uint64_t b = t0; b < nbins; b += st) m = max(m, cnt[b]);
  if (m) atomicMax(mx, m);
}
constexpr uint32_t kBinSortMax = 1024;
// one workgroup per bin: out[bin start + rank] = payload, rank = keys below
// it (input position breaking ties)
__global__ void __launch_bounds__(256) k_bin_sort(const uint64_t* __restrict__ b0, const uint64_t* __restrict__ b1,
                                                  const uint64_t* __restrict__ b2, const uint32_t* __restrict__ bp,
                                                  const uint32_t* __restrict__ sidx, const uint64_t* __restrict__ off,
                                                  uint32_t* __restrict__ out) {
  __shared__ uint64_t s0[kBinSortMax], s1[kBinSortMax], s2[kBinSortMax];
  __shared__ uint32_t si[kBinSortMax];
  const uint64_t beg = off[blockIdx.x];
  const uint32_t m = (uint32_t)(off[blockIdx.x + 1] - beg);
  if (m > kBinSortMax) return;  // the host checked the largest bin
  if (m <= 1) {
    if (m == 1 && threadIdx.x == 0) out[beg] = bp[beg];
    return;
  }
  for (uint32_t t = threadIdx.x; t < m; t += blockDim.x) {
    s0[t] = b0[beg + t];
    s1[t] = b1[beg + t];
    s2[t] = b2[beg + t];
    si[t] = sidx[beg + t];
  }
  __syncthreads();
  for (uint32_t t = threadIdx.x; t < m; t += blockDim.x) {
    const uint64_t x0 = s0[t], x1 = s1[t], x2 = s2[t];
    const uint32_t xi = si[t];
    uint32_t r = 0;
    for (uint32_t j = 0; j < m; ++j) {
      const uint64_t y0 = s0[j], y1 = s1[j], y2 = s2[j];
      r += y0 < x0 || (y0 == x0 && (y1 < x1 || (y1 == x1 && (y2 < x2 || (y2 == x2 && si[j] < xi)))));
    }
    out[beg + r] = bp[beg + t];
  }
}

// emitted unipath indices of every pair and of both paths' heads
__global__ void k_assign(uint64_t P, const uint32_t* __restrict__ ph, const uint32_t* __restrict__ tail_of,
                         const uint64_t* __restrict__ ustart, const uint32_t* __restrict__ chainlen,
                         uint32_t* __restrict__ uni_of_head, uint32_t* __restrict__ uhead, uint64_t* __restrict__ ulen,
                         uint64_t* __restrict__ urc) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < P; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t h = ph[j];
    const uint32_t rh = tail_of[h] ^ 1;
    const uint64_t u = ustart[j];
    uni_of_head[h] = (uint32_t)u;
    uhead[u] = h;
    ulen[u] = chainlen[h];
    if (rh == h) {
      urc[u] = u;
    } else {
      uni_of_head[rh] = (uint32_t)(u + 1);
      uhead[u + 1] = rh;
      ulen[u + 1] = chainlen[rh];
      urc[u] = u + 1;
      urc[u + 1] = u;
    }
  }
}

__global__ void k_pair_sizes(uint64_t P, const uint32_t* __restrict__ ph, const uint32_t* __restrict__ tail_of,
                             uint32_t* __restrict__ sz) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < P; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t h = ph[j];
    sz[j] = (tail_of[h] ^ 1) == h ? 1u : 2u;
  }
}

__global__ void k_u64_max(const uint64_t* __restrict__ x, uint64_t n, unsigned long long* __restrict__ mx) {
  unsigned long long m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    m = max(m, (unsigned long long)x[i]);
  for (int o = 32; o > 0; o >>= 1) m = max(m, (unsigned long long)__shfl_down(m, o, 64));
  if (lane_id() == 0 && m) atomicMax(mx, m);
}

__global__ void k_u32_of(const uint64_t* __restrict__ x, uint64_t n, uint32_t add, uint32_t* __restrict__ y) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    y[i] = (uint32_t)x[i] + add;
}

// ---------------------------------------------------------------------------
// U8: outputs
// ---------------------------------------------------------------------------
__global__ void k_unibases(uint64_t D, const KRec* __restrict__ nodes, KeyP kp, const uint32_t* __restrict__ head,
                           const uint32_t* __restrict__ rank, const uint32_t* __restrict__ uni_of_head,
                           const uint64_t* __restrict__ ub_off, uint8_t* __restrict__ ub) {
  for (uint64_t v0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v0 < D; v0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t v = (uint32_t)v0;
    const uint32_t u = uni_of_head[head[v]];
    const uint64_t o = ub_off[u] + rank[v];
    const KRec& x = nodes[v >> 1];
    // last base of seq(v): of the key (fw), or the complement of its first base (rc)
    const int tb = 2 * (kp.K - 1);
    const uint64_t first = ((tb >= 128 ? x.k0 : tb >= 64 ? x.k1 : x.k2) >> (tb & 63)) & 3;
    ub[o + kp.K - 1] = (uint8_t)((v & 1) ? 3 - first : (x.k2 & 3));
    if (rank[v] == 0) {
      const K3 s = dseq(nodes, v, kp);
      for (int t = 0; t < kp.K - 1; ++t) {  // base t of the K-mer
        const int bit = 2 * (kp.K - 1 - t);
        const uint64_t limb = bit >= 128 ? s.a : bit >= 64 ? s.b : s.c;
        ub[o + t] = (uint8_t)((limb >> (bit & 63)) & 3);
      }
    }
  }
}

__device__ __forceinline__ uint32_t uf_find(uint32_t* par, uint32_t x) {
  for (;;) {
    const uint32_t p = par[x];
    if (p == x) return x;
    const uint32_t g = par[p];
    if (g != p) atomicCAS(&par[x], p, g);  // path halving
    x = p;
  }
}
__device__ __forceinline__ void uf_union(uint32_t* par, uint32_t x, uint32_t y) {
  for (;;) {
    x = uf_find(par, x);
    y = uf_find(par, y);
    if (x == y) return;
    if (x > y) {
      const uint32_t t = x;
      x = y;
      y = t;
    }
    // hook the larger root under the smaller: roots stay class minima
    if (atomicCAS(&par[y], y, x) == y) return;
  }
}

__global__ void k_uf_init(uint64_t n, uint32_t* __restrict__ par) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    par[i] = (uint32_t)i;
}

__global__ void k_adjacency(uint64_t U, NodeIdx ni, KeyP kp, const uint32_t* __restrict__ uhead,
                            const uint32_t* __restrict__ tail_of, const uint32_t* __restrict__ head,
                            const uint32_t* __restrict__ uni_of_head, uint32_t* __restrict__ par,
                            unsigned long long* __restrict__ bad) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < U; u += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t t = tail_of[uhead[u]];
    const uint32_t ext = (uint32_t)(ni.nodes[t >> 1].meta & 0xff);
    const uint32_t out = out_set(ext, t & 1);
    if (!out) continue;
    const K3 s = dseq(ni.nodes, t, kp);
    for (uint32_t b = 0; b < 4; ++b) {
      if (!(out & (1u << b))) continue;
      const uint32_t w = directed_of(ni, push_right(s, b, kp), kp);
      if (w == kNone) {
        atomicAdd(bad, 1ull);
        continue;
      }
      uf_union(par, (uint32_t)(2 * u + 1), 2 * uni_of_head[head[w]]);
    }
  }
}

__global__ void k_uf_roots(uint64_t n, uint32_t* __restrict__ par, uint32_t* __restrict__ is_root) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t r = uf_find(par, (uint32_t)i);
    is_root[i] = r == i;
  }
}

__global__ void k_hkp_edges(uint64_t U, uint32_t* __restrict__ par, const uint64_t* __restrict__ vid,
                            uint64_t* __restrict__ from, uint64_t* __restrict__ to) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < U; u += (uint64_t)gridDim.x * blockDim.x) {
    from[u] = vid[uf_find(par, (uint32_t)(2 * u))];
    to[u] = vid[uf_find(par, (uint32_t)(2 * u + 1))];
  }
}

// Per-read KmerPath: ids of the read's K-mers, run-length compressed into
// intervals of consecutive ids.  WRITE = false counts intervals only.
// Read KmerPaths.  One index lookup per interval, not per K-mer: if the read's
// K-mer at j is node v at rank r of unipath u, its next K-mers are the next
// nodes of u for as long as both last — every interior node of a unipath has
// a single out-extension and the read's next base is one of v's recorded
// out-extensions — so the run is min(K-mers left in the read, len(u) - r)
// consecutive ids.  Runs whose ids continue each other merge (as per-K-mer
// appending would).
template <bool WRITE>
__global__ void k_read_paths(ReadsV rv, NodeIdx ni, KeyP kp, const uint32_t* __restrict__ head,
                             const uint32_t* __restrict__ rank, const uint32_t* __restrict__ uni_of_head,
                             const uint64_t* __restrict__ id_base, const uint64_t* __restrict__ ulen,
                             uint32_t* __restrict__ nint, const uint64_t* __restrict__ ioff,
                             uint64_t* __restrict__ istart, uint64_t* __restrict__ ilen,
                             unsigned long long* __restrict__ bad) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rv.n_reads;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t len = (uint32_t)(rv.base_off[r + 1] - rv.base_off[r]);
    uint32_t k = 0;
    uint64_t cs = 0, cl = 0;
    const uint64_t o = WRITE ? ioff[r] : 0;
    if (len >= (uint32_t)kp.K) {
      const uint32_t nk = len - kp.K + 1;
      Roller3 ro;
      ro.init(rv.packed + rv.byte_off[r], len, kp);
      uint32_t j = 0;  // K-mer index the next step() completes
      while (j < nk) {
        ro.step(kp);
        const uint32_t v = directed_of(ni, ro.fw, kp);
        if (v == kNone) {
          atomicAdd(bad, 1ull);
          ++j;
          continue;
        }
        const uint32_t u = uni_of_head[head[v]];
        const uint64_t id = id_base[u] + rank[v];
        const uint32_t run = (uint32_t)min((uint64_t)(nk - j), ulen[u] - rank[v]);
        if (cl && cs + cl == id) {
          cl += run;
        } else {
          if (cl && WRITE) {
            istart[o + k - 1] = cs;
            ilen[o + k - 1] = cl;
          }
          cs = id;
          cl = run;
          ++k;
        }
        j += run;
        if (run > 1 && j < nk) ro.seek(j, kp);
      }
      if (cl && WRITE) {
        istart[o + k - 1] = cs;
        ilen[o + k - 1] = cl;
      }
    }
    if (!WRITE) nint[r] = k;
  }
}

// ---------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------
// ---------------------------------------------------------------------------
// U1'-U3' (monolithic builds): distinct nodes through minimizer partitions.
//
// Each read is cut into super-k-mers (runs of K-mers sharing the minimizer
// of their canonical m-mers, m = min(31, max(10, K-8)), superkmer.hpp), and
// each run travels as one 48-byte record carrying its bases plus the base on
// either side (the extension bases).  Records are partitioned on the
// minimizer key (every instance of a canonical K-mer has the same minimizer,
// so a K-mer never spans two buckets) until a bucket holds ~kUskBucketKmers
// instances; one workgroup per bucket expands its K-mers into an LDS table
// keyed by the full 192-bit canonical key (OR of extension bits), and
// appends the bucket's distinct nodes to the node array — one global atomic
// per bucket.  At coverage c this replaces c random slot-line accesses per
// node of the global table (U2) by ~48 / (average run) bytes of sequential
// record traffic per instance.  A bucket whose distinct K-mers overflow the
// LDS table (low coverage, repeats) is expanded into instances that go
// through the U2 table instead.
// ---------------------------------------------------------------------------
constexpr int kUskThreads = 128;   // walk workgroups: van Herk columns w x 128 x 4 B of LDS
constexpr int kUskMaxBlocks = 8192;
constexpr int kUskBases = 160;     // bases per record
constexpr int kUskMaxW = 112;      // w = K - m + 1
constexpr int kUskMaxNk = 63;
constexpr int kUskDigitBits = 5;
constexpr uint64_t kUskBucketKmers = 2048;
constexpr uint32_t kUskTab = 1024;  // LDS table slots: tag u32, key 3 x u64, ext u32
// APG_USK_TAB=512: a first pass with a 512-slot table (24 KiB of LDS per
// block, five blocks per CU instead of four: the bench buckets hold ~140
// distinct K-mers) and the buckets it overflows again with kUskTab slots.
constexpr uint32_t kUskTabSmall = 512;
// probes before a bucket is declared full (linear probing at load <= 0.9 stays
// far below; a full table must not cost every later instance 1024 probes)
constexpr uint32_t kUskProbeMax = 128;
// 64 records per round keeps the block at 39.5 KiB of LDS: four blocks per CU
// instead of three at 128 (usk_bucket 15.9 -> 14.5 ms on the C2 step)
constexpr int kUskChunk = 64;       // records flattened per round
constexpr int kUskBThreads = 256;
constexpr int kUskWalk2MinW = 24;  // windows longer than this walk with sk_walk2 (a third of the LDS column)

constexpr int kUskListCap = 256;   // parked records per tile (2 KiB of LDS)
using UskTile = SkTile<kUskThreads, 6144>;  // 128 fragments of <= ~180 bases

// dynamic LDS of the walk kernels: the van Herk column of each thread, then
// the per-digit counters
struct UskP {
  using U = uint64_t;  // m <= 31
  int K, m, w, maxnk;
  uint64_t mmask;
  int two;  // the two-level column (w > kUskWalk2MinW; APG_USK_FLAT=1: single-level for every w)
  int reg;  // the count walk keeps its column in registers (w == kUskRegW; APG_USK_REG=0: off)
};
constexpr int kUskRegW = 66;  // the window of the K = 96 walk (m = kUskRegM)
constexpr int kUskRegM = 31;

__host__ __device__ inline uint32_t usk_column_words(const UskP& p) {
  return (uint32_t)(p.two ? sk_walk2_words(p.w) : p.w) * kUskThreads;
}
// the count pass's walk LDS: with the register column only the waves' record
// queues and one column of the two-level walk for a read too long for a tile
// (thread 0, stride 1): 8 KiB instead of the 13.5 KiB column, so eight
// blocks per CU fit instead of seven
__host__ __device__ inline uint32_t usk_count_words(const UskP& p) {
  if (!p.reg) return usk_column_words(p);
  const uint32_t q = sk_regq_words(kUskThreads, kUskRegW), c = (uint32_t)sk_walk2_words(p.w);
  return q > c ? q : c;
}
static size_t usk_walk_lds(const UskP& p, int D, size_t per_digit) {
  return (size_t)usk_column_words(p) * 4 + ((size_t)1 << D) * per_digit;
}

static UskP make_uskp(int K) {
  UskP p;
  p.K = K;
  p.m = K <= 10 ? K : std::min(31, std::max(10, K - 8));
  p.w = K - p.m + 1;
  p.maxnk = std::min(kUskBases - K - 1, kUskMaxNk);
  p.mmask = (1ull << (2 * p.m)) - 1;
  static const bool flat = [] {
    const char* e = getenv("APG_USK_FLAT");
    return e && !strcmp(e, "1");
  }();
  p.two = !flat && p.w > kUskWalk2MinW;
  static const bool reg = [] {
    const char* e = getenv("APG_USK_REG");
    return !(e && !strcmp(e, "0"));
  }();
  p.reg = reg && p.w == kUskRegW && p.m == kUskRegM;
  return p;
}

// Record of K-mers [a, a+n) of a read of length L with minimizer order key.
__device__ __forceinline__ SK48 make_urec(const uint8_t* rd, uint32_t L, uint32_t a, uint32_t n, uint32_t key, int K) {
  const uint32_t hl = a > 0, end = a + n + (uint32_t)K - 1, hr = end < L;
  const uint32_t s0 = a - hl, nb = hl + n + (uint32_t)K - 1 + hr;
  SK48 r;
  r.w0 = (uint64_t)part_key(key) | ((uint64_t)n << 32) | ((uint64_t)(hl | (hr << 1)) << 40);
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    const uint32_t lo = 32 * k;
    uint64_t x = lo < nb ? sk_lsb64(rd, s0 + lo) : 0;
    if (nb - lo < 32 && lo < nb) x &= (1ull << (2 * (nb - lo))) - 1;
    r.b[k] = x;
  }
  return r;
}

// The block's reads [r0, r1), tile by tile: the single-level column for short
// windows, the two-level one (sk_walk2_words) for long.
template <bool LIST, int CAP, typename F, typename TD>
__device__ __forceinline__ void usk_walk_tiles(const SkReads& rv, const UskP& p, uint64_t r0, uint64_t r1, UskTile& T,
                                               uint32_t* sb, SkList<CAP>& lst, F f, TD tile_done) {
  const bool two = p.two;
  for (uint64_t t0 = r0; t0 < r1;) {
    const uint32_t n = sk_load_tile(rv, t0, r1, T);
    if (n) {
      if (!LIST && p.reg)
        sk_walk_tile<kUskThreads, true, LIST, kUskRegW, kUskRegM>(p, T, n, sb, lst, f);
      else if (two)
        sk_walk_tile<kUskThreads, true, LIST>(p, T, n, sb, lst, f);
      else
        sk_walk_tile<kUskThreads, false, LIST>(p, T, n, sb, lst, f);
    } else if (!LIST && p.reg) {  // the count pass's column: stride 1 (usk_count_words)
      sk_walk_global<1, true>(rv, p, T, t0, sb - threadIdx.x, f);
    } else if (two) {
      sk_walk_global<kUskThreads, true>(rv, p, T, t0, sb, f);
    } else {
      sk_walk_global<kUskThreads, false>(rv, p, T, t0, sb, f);
    }
    __syncthreads();
    tile_done(t0);
    t0 += n ? n : 1;
  }
}

// Per-(digit, block) record counts and per-digit K-mer counts.
__global__ void __launch_bounds__(kUskThreads) k_usk_count(SkReads rv, UskP p, int D, uint32_t* __restrict__ cmat,
                                                           unsigned long long* __restrict__ kdig, SkDesc dd) {
  __shared__ UskTile T;
  __shared__ SkList<1> lst;  // f runs in place
  __shared__ uint32_t dpos, dovf;
  extern __shared__ uint32_t usk_sb[];  // the walk columns, then hist[ndig], khist[ndig]
  const uint32_t ndig = 1u << D;
  uint32_t* hist = usk_sb + usk_count_words(p);
  uint32_t* khist = hist + ndig;
  const uint32_t G = gridDim.x, b = blockIdx.x;
  for (uint32_t i = threadIdx.x; i < ndig; i += blockDim.x) hist[i] = khist[i] = 0;
  if (threadIdx.x == 0) lst.cnt = dpos = dovf = 0;
  uint64_t r0, r1;
  sk_read_range(rv.n_reads, G, b, &r0, &r1);
  SkDescWriter W(dd, rv, r0, r1, &dpos, &dovf);
  auto f = [&](const uint8_t*, uint32_t, uint32_t a, uint32_t n, uint32_t key, uint32_t q) {
    const uint32_t d = D ? part_key(key) >> (32 - D) : 0;
    atomicAdd(&hist[d], 1u);
    atomicAdd(&khist[d], n);
    W.put(a, n, key, q);
  };
  usk_walk_tiles<false>(rv, p, r0, r1, T, usk_sb + threadIdx.x, lst, f, [&](uint64_t t0) { W.tile_done(t0); });
  W.block_done();
  for (uint32_t i = threadIdx.x; i < ndig; i += blockDim.x) {
    cmat[(uint64_t)i * G + b] = hist[i];
    if (khist[i]) atomicAdd(&kdig[i], (unsigned long long)khist[i]);
  }
}

__global__ void __launch_bounds__(kUskThreads) k_usk_scatter(SkReads rv, UskP p, int D,
                                                             const uint64_t* __restrict__ omat, SK48* __restrict__ out,
                                                             SkDesc dd) {
  __shared__ UskTile T;
  __shared__ SkList<kUskListCap> lst;
  extern __shared__ uint32_t usk_sb[];  // the walk columns, then cur[ndig]
  const uint32_t ndig = 1u << D;
  unsigned long long* cur = reinterpret_cast<unsigned long long*>(usk_sb + usk_column_words(p));
  const uint32_t G = gridDim.x, b = blockIdx.x;
  for (uint32_t d = threadIdx.x; d < ndig; d += blockDim.x) cur[d] = omat[(uint64_t)d * G + b];
  if (threadIdx.x == 0) lst.cnt = 0;
  uint64_t r0, r1;
  sk_read_range(rv.n_reads, G, b, &r0, &r1);
  auto f = [&](const uint8_t* rd, uint32_t L, uint32_t a, uint32_t n, uint32_t key, uint32_t) {
    const SK48 x = make_urec(rd, L, a, n, key, p.K);
    const uint32_t d = D ? (uint32_t)x.w0 >> (32 - D) : 0;
    out[atomicAdd(&cur[d], 1ull)] = x;
  };
  uint64_t t0 = r0;
  if (sk_replay<kUskThreads>(dd, rv, r0, r1, T, t0, f)) return;  // the count pass's descriptors
  usk_walk_tiles<true>(rv, p, r0, r1, T, usk_sb + threadIdx.x, lst, f, [](uint64_t) {});
}

__global__ void k_usk_digit_starts(const uint64_t* __restrict__ omat, uint32_t ndig, uint32_t G,
                                   uint64_t* __restrict__ ds) {
  const uint32_t d = blockIdx.x * blockDim.x + threadIdx.x;
  if (d <= ndig) ds[d] = omat[(uint64_t)d * G];
}

// 64 bits of a record's base string from bit `bit` (< 320; zeros past it).
__device__ __forceinline__ uint64_t urec_bits(const SK48& r, uint32_t bit) {
  const uint32_t q = bit >> 6, s = bit & 63;
  const uint64_t lo = r.b[q], hi = q < 4 ? r.b[q + 1] : 0;
  return s ? (lo >> s) | (hi << (64 - s)) : lo;
}

// K-mer t of a record (K bases from record base hl + t): canonical key and
// extension bits in canonical orientation.
__device__ __forceinline__ void urec_kmer(const SK48& r, uint32_t t, const KeyP& kp, K3* key, uint32_t* ext) {
  const uint32_t n = (uint32_t)(r.w0 >> 32) & 0xff, fl = (uint32_t)(r.w0 >> 40) & 3;
  const uint32_t hl = fl & 1, hr = fl >> 1;
  const uint32_t K = (uint32_t)kp.K, nb = hl + n + K - 1 + hr, st = hl + t;
  const K3 W{urec_bits(r, 2 * st + 128), urec_bits(r, 2 * st + 64), urec_bits(r, 2 * st)};
  const K3 fw = shr192(K3{rev2(W.c), rev2(W.b), rev2(W.a)}, 192 - 2 * kp.K);
  const K3 rc{~W.a & kp.ma, ~W.b & kp.mb, ~W.c & kp.mc};
  const int a = st > 0 ? (int)((r.b[(st - 1) >> 5] >> (2 * ((st - 1) & 31))) & 3) : -1;
  const int b = st + K < nb ? (int)((r.b[(st + K) >> 5] >> (2 * ((st + K) & 31))) & 3) : -1;
  canon_ext(fw, rc, a, b, key, ext);
}

__device__ __forceinline__ uint32_t usk_slot_hash(const K3& k) {
  const uint64_t x = k.c ^ (k.b * 0x9e3779b97f4a7c15ull) ^ (k.a * 0xc2b2ae3d27d4eb4full);
  return sk_fmix32((uint32_t)x ^ (uint32_t)(x >> 32));
}

struct UskOut {
  KRec* nodes;
  uint64_t cap;
  unsigned long long* gs;  // [0] nodes appended
  uint32_t* ovf_list;      // overflowed buckets, counted by *novf
  unsigned long long* novf;
  uint2* lsucc;  // may be null: per node, its two orientations' local links (usk_links_local)
  uint32_t dedup;  // fold identical records of a chunk before flattening
  unsigned long long* dstat;  // may be null: records, instances, records folded, instances folded
  // may be null: the node index (k_node_insert's table) built as nodes are
  // appended, for the nodes with id < idx_lim (gs[4] counts the rest)
  unsigned long long* idx;
  uint64_t tmask, idx_lim;
  // diagnostics (APG_USK_PROF): thread 0's clock64 sums per phase — chunk
  // load + dedup, scan + owner map, inserts, node ranks, nodes + index + local links
  unsigned long long* prof = nullptr;
};

// The node index of the single-GPU build, made by the node buckets
// (usk_stage) instead of k_node_insert: valid when idx != null.
struct PreIdx {
  unsigned long long* idx = nullptr;
  uint64_t T = 0;
};

// 32-bit fingerprint of a K=96 record (its full content: n, flank flags, bases)
__device__ __forceinline__ uint32_t urec_fp(const SK48& r) {
  uint64_t x = (r.w0 >> 32) * 0x9e3779b97f4a7c15ull;
#pragma unroll
  for (int k = 0; k < 5; ++k) x = fmix64(x ^ r.b[k]);
  return (uint32_t)(x >> 32);
}


// One workgroup per bucket (grid-stride); blist (or null): the buckets to
// run, nbuckets of them (the ones a smaller table overflowed).
template <uint32_t TAB, int WPE = 1>
__global__ void __launch_bounds__(kUskBThreads) __attribute__((amdgpu_waves_per_eu(WPE)))
k_usk_bucket(const SK48* __restrict__ rec,
                                                             const uint64_t* __restrict__ boff, uint64_t nbuckets,
                                                             const uint32_t* __restrict__ blist, KeyP kp, UskOut o) {
  constexpr uint32_t kUskTab = TAB;
  __shared__ uint32_t tag[kUskTab];
  __shared__ uint64_t ka[kUskTab], kb[kUskTab], kc[kUskTab];
  __shared__ uint32_t text[kUskTab];
  __shared__ __attribute__((aligned(16))) SK48 crec[kUskChunk];  // emit: the occupied slots in rank order (u16)
  __shared__ uint32_t koff[kUskChunk];
  __shared__ uint32_t dht[2 * kUskChunk];  // dedup: fingerprint bits | leader lane, 0 = empty
  __shared__ __attribute__((aligned(16))) uint8_t owner[kUskChunk * kUskMaxNk];
  __shared__ uint32_t scan_sm[64];
  __shared__ int ovf;
  __shared__ unsigned long long sbase;
  constexpr int TB = __builtin_ctz(kUskTab);
  static_assert(kUskChunk * kUskMaxNk >= 2 * TAB, "owner doubles as the slot ranks");
  uint16_t* rnk = reinterpret_cast<uint16_t*>(owner);  // emit: slot -> rank in the bucket's node list
  static_assert(sizeof(SK48) * kUskChunk >= 2 * TAB, "crec doubles as the rank -> slot list");
  uint16_t* slot_of = reinterpret_cast<uint16_t*>(crec);
  const uint32_t tid = threadIdx.x;
  unsigned long long pt[5] = {0, 0, 0, 0, 0}, t0 = 0;
  const bool prof = o.prof != nullptr && tid == 0;
  auto mark = [&](int ph) {
    if (prof) {
      const unsigned long long t1 = clock64();
      if (ph > 0) pt[ph - 1] += t1 - t0;
      t0 = t1;
    }
  };
  // The block's buckets bkt, bkt + grid, ... are one record stream: the next
  // chunk's records (this bucket's or the next bucket's first) are loaded
  // while the current chunk is counted.
  auto bucket = [&](uint64_t q) -> uint64_t { return blist ? blist[q] : q; };
  uint64_t bkt = blockIdx.x, off = 0;  // bkt: index into the bucket list
  uint32_t nr = 0;
  if (bkt < nbuckets) {
    const uint64_t b0 = bucket(bkt);
    off = boff[b0];
    nr = (uint32_t)(boff[b0 + 1] - off);
  }
  SK48 pre{};
  if (tid < kUskChunk && tid < nr) pre = rec[off + tid];
  if (tid < 2 * kUskChunk) dht[tid] = 0;
  __syncthreads();  // the dedup table is empty before the first chunk's claims
  for (; bkt < nbuckets;) {
    const uint64_t nbk = bkt + gridDim.x;
    uint64_t noff = 0;
    uint32_t nnr = 0;
    if (nbk < nbuckets) {
      const uint64_t b1 = bucket(nbk);
      noff = boff[b1];
      nnr = (uint32_t)(boff[b1 + 1] - noff);
    }
    auto advance = [&]() {
      bkt = nbk;
      off = noff;
      nr = nnr;
    };
    if (nr == 0) {  // block-uniform
      if (tid < kUskChunk && tid < nnr) pre = rec[noff + tid];
      advance();
      continue;
    }
    for (uint32_t s = tid; s < kUskTab; s += kUskBThreads) tag[s] = 0;
    if (tid == 0) ovf = 0;
    mark(0);
    for (uint32_t c0 = 0; c0 < nr; c0 += kUskChunk) {
      // the table filled in an earlier chunk (block-uniform after the chunk's
      // barrier): the rest of the bucket goes to the global table as well, so
      // stop here and load the next bucket's first records
      if (c0 && ovf) {
        if (tid < kUskChunk && tid < nnr) pre = rec[noff + tid];
        break;
      }
      uint32_t nk = 0, lead = tid;
      if (tid < kUskChunk && c0 + tid < nr) {
        nk = (uint32_t)(pre.w0 >> 32) & 0xff;
        crec[tid] = pre;
        if (o.dedup) {  // claim the record's fingerprint, or find its leader
          const uint32_t fp = urec_fp(pre);
          const uint32_t want = ((fp | 64u) & ~63u) | tid;
          for (uint32_t sl = fp & (2 * kUskChunk - 1);; sl = (sl + 1) & (2 * kUskChunk - 1)) {
            const uint32_t old = atomicCAS(&dht[sl], 0u, want);
            if (old == 0) break;
            if ((old & ~63u) == (want & ~63u)) {
              lead = old & 63u;
              break;
            }
          }
        }
      }
      if (tid < kUskChunk) {
        if (c0 + kUskChunk < nr) {
          if (c0 + kUskChunk + tid < nr) pre = rec[off + c0 + kUskChunk + tid];
        } else if (tid < nnr) {
          pre = rec[noff + tid];
        }
      }
      // Record dedup: at fragment coverage c, every fragment that spans a
      // whole super-k-mer emits the same record (its bases and flanks are the
      // genome's), so a chunk holds repeated ones (30 % of the bench step's
      // records, 24 % of its K-mer instances); a record equal to another of the
      // chunk adds no node and no extension bit, and is not flattened.  Lanes
      // < 64 own the records: a 128-slot LDS table of fingerprints names each
      // fingerprint's first claimant, and a record is dropped only if it
      // equals that leader's record exactly (a fingerprint collision keeps
      // both).
      if (o.dedup) {  // block-uniform
        __syncthreads();  // the chunk's records and claims
        if (tid < 2 * kUskChunk) dht[tid] = 0;  // for the next chunk (no lane reads the table past the barrier)
        if (nk && lead != tid) {
          const SK48& a = crec[lead];
          const SK48& m = crec[tid];
          if (a.w0 == m.w0 && a.b[0] == m.b[0] && a.b[1] == m.b[1] && a.b[2] == m.b[2] && a.b[3] == m.b[3] &&
              a.b[4] == m.b[4]) {
            if (o.dstat) {
              atomicAdd(&o.dstat[2], 1ull);
              atomicAdd(&o.dstat[3], (unsigned long long)nk);
            }
            nk = 0;
          }
        }
      }
      if (o.dstat && tid < kUskChunk && c0 + tid < nr) {
        atomicAdd(&o.dstat[0], 1ull);
        atomicAdd(&o.dstat[1], (unsigned long long)((crec[tid].w0 >> 32) & 0xff));
      }
      mark(1);
      uint32_t tot;
      const uint32_t ex = block_exclusive_scan<uint32_t>(nk, scan_sm, &tot);  // barrier: table clear visible
      if (tid < kUskChunk) koff[tid] = ex;
      for (uint32_t u = 0; u < nk; ++u) owner[ex + u] = (uint8_t)tid;
      __syncthreads();
      mark(2);
      for (uint32_t f = tid; f < tot; f += kUskBThreads) {
        const uint32_t i = owner[f];
        K3 key;
        uint32_t e;
        urec_kmer(crec[i], f - koff[i], kp, &key, &e);
        const uint32_t h = usk_slot_hash(key);
        const uint32_t tv = (h & ~3u) | 2u;
        uint32_t s = h >> (32 - TB);
        for (uint32_t probe = 0;;) {
          // the slot's tag, key words and extension bits read together: one
          // LDS round trip on the common hit path (tag, then each key word
          // after the previous compare cost four)
          const uint32_t tg = tag[s];
          uint64_t xa = ka[s], xb = kb[s], xc = kc[s];
          const uint32_t xt = text[s];
          if (tg == 0) {
            const uint32_t prev = atomicCAS(&tag[s], 0u, 1u);
            if (prev == 0) {
              ka[s] = key.a;
              kb[s] = key.b;
              kc[s] = key.c;
              text[s] = e;
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
              __hip_atomic_store(&tag[s], tv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
              break;
            }
            continue;  // claimed meanwhile: read the slot again
          }
          if (tg == 1) continue;  // being written by a lane that publishes in the same pass
          if (tg == tv) {
            if (xa != key.a || xb != key.b || xc != key.c) {
              // the key words may have been read before the tag that
              // published them: read them again, ordered after it
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
              xa = ka[s];
              xb = kb[s];
              xc = kc[s];
            }
            if (xa == key.a && xb == key.b && xc == key.c) {
              if (e & ~xt) atomicOr(&text[s], e);  // a stale xt only costs an extra OR
              break;
            }
          }
          s = (s + 1) & (kUskTab - 1);
          if (++probe == kUskProbeMax) {
            ovf = 1;  // table full: the bucket goes through the global table
            break;
          }
        }
      }
      __syncthreads();
      mark(3);
    }
    if (ovf) {
      if (tid == 0) o.ovf_list[atomicAdd(o.novf, 1ull)] = (uint32_t)bucket(bkt);
      __syncthreads();
      advance();
      continue;
    }
    uint32_t nn = 0;
    for (uint32_t s = tid; s < kUskTab; s += kUskBThreads) nn += tag[s] != 0;
    uint32_t tot;
    uint32_t j = block_exclusive_scan<uint32_t>(nn, scan_sm, &tot);
    // the bucket's node ids: the add is in flight while the ranks are written
    unsigned long long b0 = 0;
    if (tid == 0 && tot) b0 = atomicAdd(&o.gs[0], (unsigned long long)tot);
    for (uint32_t s = tid; s < kUskTab; s += kUskBThreads)
      if (tag[s] != 0) {
        rnk[s] = (uint16_t)j;  // owner and crec are free: every instance is inserted
        slot_of[j++] = (uint16_t)s;
      }
    if (tid == 0) sbase = b0;
    __syncthreads();  // every slot's rank, the base
    const unsigned long long b = sbase;
    mark(4);
    // The nodes by rank (full lanes): the node, its index entry, its local
    // links.  The index insert's first probe is in flight during the links;
    // a taken slot probes on after them (load <= 1/2 by idx_lim).
    for (uint32_t r = tid; r < tot; r += kUskBThreads) {
      const uint32_t s = slot_of[r];
      const unsigned long long id = b + r;
      if (id >= o.cap) continue;
      const K3 key{ka[s], kb[s], kc[s]};
      const uint32_t ext = text[s];
      const uint64_t kh = key_hash(key);
      o.nodes[id] = KRec{key.a, key.b, key.c, kh | ext};
      bool ix = false;  // index entry as k_node_insert makes it
      uint64_t q = 0;
      unsigned long long want = 0, prev = kIdxEmpty;
      if (o.idx) {
        if (id < o.idx_lim) {
          const uint64_t h = kh >> 8;
          want = ((unsigned long long)idx_tag(h) << 32) | id;
          q = h & o.tmask;
          prev = atomicCAS(&o.idx[q], kIdxEmpty, want);
          ix = true;
        } else {
          atomicAdd(&o.gs[4], 1ull);
        }
      }
      if (o.lsucc) {  // block-uniform
        // the rules of k_links, with the successor looked up in this table
        const K3 rk = revcomp(key, kp);
        uint32_t res[2] = {kNone, kNone};
        if (!k3_eq(key, rk)) {  // palindromic K-mers never link
#pragma unroll
          for (uint32_t d = 0; d < 2; ++d) {
            const uint32_t out = out_set(ext, d);
            if (__popc(out) != 1) continue;
            const uint32_t bo = __ffs(out) - 1;
            const K3 t = push_right(d ? rk : key, bo, kp);
            const K3 tr = rc_roll(d ? key : rk, bo, kp);  // revcomp(t) by a shift
            const bool fw = !k3_lt(tr, t);
            const K3 c = fw ? t : tr;
            const uint32_t h = usk_slot_hash(c);
            const uint32_t tv = (h & ~3u) | 2u;
            uint32_t sl = h >> (32 - TB), hit = kUskTab;
            for (uint32_t probe = 0; probe < kUskProbeMax; ++probe) {
              const uint32_t tg = tag[sl];  // the table is complete: read the slot at once
              const uint64_t xa = ka[sl], xb = kb[sl], xc = kc[sl];
              if (tg == 0) break;
              if (tg == tv && xa == c.a && xb == c.b && xc == c.c) {
                hit = sl;
                break;
              }
              sl = (sl + 1) & (kUskTab - 1);
            }
            if (hit == kUskTab) {
              res[d] = kLsGlobal;
              continue;
            }
            if (k3_eq(t, tr)) continue;  // palindromic successor
            if (__popc(in_set(text[hit], fw ? 0u : 1u)) != 1) continue;
            res[d] = (uint32_t)(2 * (b + rnk[hit])) + (fw ? 0u : 1u);
          }
        }
        o.lsucc[id] = make_uint2(res[0], res[1]);
      }
      if (ix && prev != kIdxEmpty) {
        do {
          q = (q + 1) & o.tmask;
        } while (atomicCAS(&o.idx[q], kIdxEmpty, want) != kIdxEmpty);
      }
    }
    __syncthreads();
    mark(5);
    advance();
  }
  if (prof)
    for (int i = 0; i < 5; ++i) atomicAdd(&o.prof[i], pt[i]);
}

// Instances of the overflowed buckets as 32-byte KRecs (for the U2 table).
__global__ void k_usk_ovf_count(const SK48* __restrict__ rec, const uint64_t* __restrict__ boff,
                                const uint32_t* __restrict__ ovf_list, uint32_t n_ovf,
                                unsigned long long* __restrict__ n_inst) {
  unsigned long long c = 0;
  for (uint32_t q = blockIdx.x; q < n_ovf; q += gridDim.x) {
    const uint32_t b = ovf_list[q];
    for (uint64_t i = boff[b] + threadIdx.x; i < boff[b + 1]; i += blockDim.x) c += (uint32_t)(rec[i].w0 >> 32) & 0xff;
  }
  wave_add(n_inst, c);
}

__global__ void k_usk_ovf_expand(const SK48* __restrict__ rec, const uint64_t* __restrict__ boff,
                                 const uint32_t* __restrict__ ovf_list, uint32_t n_ovf, KeyP kp,
                                 unsigned long long* __restrict__ cursor, KRec* __restrict__ out) {
  for (uint32_t q = blockIdx.x; q < n_ovf; q += gridDim.x) {
    const uint32_t b = ovf_list[q];
    for (uint64_t i = boff[b] + threadIdx.x; i < boff[b + 1]; i += blockDim.x) {
      const SK48 r = rec[i];
      const uint32_t n = (uint32_t)(r.w0 >> 32) & 0xff;
      unsigned long long at = atomicAdd(cursor, (unsigned long long)n);
      for (uint32_t t = 0; t < n; ++t) {
        K3 key;
        uint32_t e;
        urec_kmer(r, t, kp, &key, &e);
        out[at + t] = KRec{key.a, key.b, key.c, key_hash(key) | e};
      }
    }
  }
}

static int ceil_log2_u(uint64_t x) {
  int b = 0;
  while ((1ull << b) < x) ++b;
  return b;
}


// Host arrays the caller owns (std::free).  Large ones are 2 MiB-aligned and
// advised as transparent huge pages: the D2H workers' copies first-touch the
// pages, and 4 KiB faults held the copy to ~13-16 GB/s (scripts/diag/d2h_rate.py).
static void* host_alloc(uint64_t bytes) {
  constexpr uint64_t kHuge = 2ull << 20;
  if (bytes < 2 * kHuge) return std::malloc(std::max<uint64_t>(bytes, 1));
  const uint64_t b = (bytes + kHuge - 1) & ~(kHuge - 1);
  void* p = std::aligned_alloc(kHuge, b);
  if (p && !std::getenv("APG_NO_THP")) (void)madvise(p, b, MADV_HUGEPAGE);
  return p;
}

template <typename T>
static T* host_dup(const T* d, uint64_t n, std::vector<D2HJob>* jobs, int* rc) {
  T* h = (T*)host_alloc(std::max<uint64_t>(n, 1) * sizeof(T));
  if (!h) {
    *rc = APG_E_NOMEM;
    return nullptr;
  }
  if (n) jobs->push_back(D2HJob{h, d, n * sizeof(T)});
  return h;
}

static int d2h_u64(apg_ctx* ctx, const unsigned long long* d, unsigned long long* h, int n) {
  return d2h_sync(ctx, h, d, (size_t)n * 8);
}

// HyperLogLog estimate of the distinct count from 2^kHllBits registers.
static double hll_estimate(const std::vector<uint32_t>& reg) {
  const double m = (double)reg.size();
  double sum = 0;
  uint64_t zeros = 0;
  for (uint32_t r : reg) {
    sum += std::ldexp(1.0, -(int)r);
    zeros += r == 0;
  }
  const double alpha = 0.7213 / (1.0 + 1.079 / m);
  double e = alpha * m * m / sum;
  if (e <= 2.5 * m && zeros) e = m * std::log(m / (double)zeros);
  return e;
}

// Sizing pass over reads: instance count and distinct estimate.
static int u_size(apg_ctx* ctx, const apg_dreads* dr, const KeyP& kp, uint64_t* n_inst, double* est) {
  ReadsV rv{dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->n_reads};
  uint32_t* hll = nullptr;
  unsigned long long* cnt = nullptr;
  APG_TRY(workspace_t(ctx, "u_hll", 1u << kHllBits, &hll));
  APG_TRY(workspace_t(ctx, "u_ninst", 1, &cnt));
  APG_CHECK_HIP(hipMemsetAsync(hll, 0, (1u << kHllBits) * 4, ctx->stream));
  APG_CHECK_HIP(hipMemsetAsync(cnt, 0, 8, ctx->stream));
  kbegin(ctx, "u_size", dr->n_bytes + 16 * dr->n_reads);
  if (dr->n_reads) k_uhll<<<grid_for(ctx, dr->n_reads), kUThreads, 0, ctx->stream>>>(rv, kp, hll, cnt);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  std::vector<uint32_t> reg(1u << kHllBits);
  unsigned long long n = 0;
  APG_CHECK_HIP(hipMemcpyAsync(reg.data(), hll, reg.size() * 4, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(d2h_sync(ctx, &n, cnt, 8));
  *n_inst = n;
  *est = n ? std::min<double>((double)n, hll_estimate(reg)) : 0.0;
  return APG_OK;
}

// Distinct nodes of reads (dr) or of records (rec, n_rec) into workspace
// "u_nodes", grouped by the top kUDigitBits hash bits; digit_counts (may be
// null) receives the per-group node counts.
static int u_build_nodes(apg_ctx* ctx, const apg_dreads* dr, const KRec* rec, uint64_t n_rec, const KeyP& kp,
                         double est, KRec** nodes_out, uint64_t* N_out, std::vector<uint64_t>* digit_counts) {
  const uint32_t ndig = 1u << kUDigitBits;
  // ~3 slots per distinct K-mer (load ~0.32): fewer probes per instance
  // (~1.25 vs ~1.45 at load 0.48) for 1.5x the table (64 B per slot)
  uint64_t T = std::max<uint64_t>(4096, (uint64_t)(3.0 * est * 1.05) + 1);
  UTab t{};
  unsigned long long* ovf = nullptr;
  APG_TRY(workspace_t(ctx, "u_tabovf", 2, &ovf));
  for (int attempt = 0;; ++attempt) {
    APG_TRY(workspace_t(ctx, "u_tabslot", T, &t.slot));
    t.T = T;
    t.ovf = ovf;
    APG_CHECK_HIP(hipMemsetAsync(t.slot, 0, T * sizeof(USlot), ctx->stream));
    APG_CHECK_HIP(hipMemsetAsync(ovf, 0, 16, ctx->stream));
    if (dr) {
      ReadsV rv{dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->n_reads};
      kbegin(ctx, "u_insert", dr->n_bytes + 16 * dr->n_reads);
      if (dr->n_reads) k_uinsert_reads<<<grid_for(ctx, dr->n_reads), kUThreads, 0, ctx->stream>>>(rv, kp, t);
      kend(ctx);
    } else {
      kbegin(ctx, "u_insert_recs", n_rec * sizeof(KRec));
      if (n_rec) k_uinsert_recs<<<grid_for(ctx, n_rec), kUThreads, 0, ctx->stream>>>(rec, n_rec, t);
      kend(ctx);
    }
    APG_CHECK_HIP(hipGetLastError());
    unsigned long long of[2] = {0, 0};
    APG_TRY(d2h_sync(ctx, of, ovf, 16));
    kbytes_add(ctx, dr ? "u_insert" : "u_insert_recs", of[1] * 64);  // one 64-byte slot line per probe
    if (!of[0]) break;
    if (attempt >= 6) {
      set_error("unipaths: node table overflow persists");
      return APG_E_STATE;
    }
    vlog(ctx, "unipaths: node table of %llu slots overflowed, rebuilding at 2x", (unsigned long long)T);
    T *= 2;
  }
  // compaction, grouped by digit
  const uint32_t G = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(2048, T / 4096));
  uint32_t* cmat = nullptr;
  uint64_t *omat = nullptr, *dstart = nullptr;
  APG_TRY(workspace_t(ctx, "u_cmat", (uint64_t)ndig * G, &cmat));
  APG_TRY(workspace_t(ctx, "u_omat", (uint64_t)ndig * G + 1, &omat));
  APG_TRY(workspace_t(ctx, "u_dstart", ndig + 1, &dstart));
  kbegin(ctx, "u_tab_compact", T * 8 + (uint64_t)(est * 72));
  k_tab_count<<<G, kUThreads, 0, ctx->stream>>>(t.slot, T, cmat);
  APG_TRY(scan_u32_u64(ctx, cmat, (uint64_t)ndig * G, omat, "ut"));
  k_digit_starts_u<<<1, 64, 0, ctx->stream>>>(omat, ndig, G, dstart);
  std::vector<uint64_t> ds(ndig + 1);
  APG_TRY(d2h_sync(ctx, ds.data(), dstart, (ndig + 1) * 8));
  const uint64_t N = ds[ndig];
  KRec* nodes = nullptr;
  APG_TRY(workspace_t(ctx, "u_nodes", std::max<uint64_t>(N, 1), &nodes));
  k_tab_scatter<<<G, kUThreads, 0, ctx->stream>>>(t.slot, T, omat, nodes);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  if (digit_counts) {
    digit_counts->resize(ndig);
    for (uint32_t d = 0; d < ndig; ++d) (*digit_counts)[d] = ds[d + 1] - ds[d];
  }
  vlog(ctx, "unipaths: %llu distinct nodes (estimate %.0f), table %llu slots", (unsigned long long)N, est,
       (unsigned long long)T);
  *nodes_out = nodes;
  *N_out = N;
  return APG_OK;
}

// U4 index + U5..U8 on a complete node set; read KmerPaths for `dr` (may be
// null when no read paths are requested).
// U6: rank the directed nodes' unique links (rb.dn) by a sparse ruling set;
// cycles are cut before their minimum K-mer and ranking reruns.  Outputs per
// directed node its chain head and rank, per head its chain length and tail.
static int u_rank_all(apg_ctx* ctx, const KRec* nodes, uint64_t N, const KeyP& kp, RankBufs& rb,
                      unsigned long long* gs, apg_unipath_stats* st, uint32_t** head, uint32_t** rank,
                      uint32_t** chainlen, uint32_t** tail_of) {
  const uint64_t D = 2 * N;
  APG_TRY(workspace_t(ctx, "u_rnext", std::max<uint64_t>(D, 1), &rb.rnext));
  APG_TRY(workspace_t(ctx, "u_seglen", std::max<uint64_t>(D, 1), &rb.seglen));
  APG_TRY(workspace_t(ctx, "u_state", std::max<uint64_t>(D, 1), &rb.state));
  APG_TRY(workspace_t(ctx, "u_rlist", std::max<uint64_t>(D, 1), &rb.rlist));
  APG_TRY(workspace_t(ctx, "u_alist0", std::max<uint64_t>(D, 1), &rb.alist0));
  APG_TRY(workspace_t(ctx, "u_alist1", std::max<uint64_t>(D, 1), &rb.alist1));
  for (int attempt = 0; attempt < 3; ++attempt) {
    APG_CHECK_HIP(hipMemsetAsync(gs + 8, 0, 8 * 8, ctx->stream));
    kbegin(ctx, "u_find_rulers", D * 12);
    k_find_rulers<<<grid_for(ctx, D), 256, 0, ctx->stream>>>(D, rb, gs + 8);
    kend(ctx);
    unsigned long long hr;
    APG_TRY(d2h_u64(ctx, gs + 8, &hr, 1));
    const uint64_t R = hr;
    kbegin(ctx, "u_walk", D * 16);
    k_walk<<<grid_for(ctx, R), 256, 0, ctx->stream>>>(R, D, rb);
    kend(ctx);
    k_ruler_state0<<<grid_for(ctx, R), 256, 0, ctx->stream>>>(R, rb);
    k_ruler_state1<<<grid_for(ctx, R), 256, 0, ctx->stream>>>(R, rb, gs + 9);
    APG_CHECK_HIP(hipGetLastError());
    unsigned long long na;
    APG_TRY(d2h_u64(ctx, gs + 9, &na, 1));
    uint32_t *ain = rb.alist0, *aout = rb.alist1;
    const int max_rounds = ceil_log2_u(R + 1) + 2;
    // rounds in batches of kJumpBatch between host reads of the active count
    // (a round after the list empties is an empty launch); round it reads
    // its length from jc[it - 1] (round 0: k_ruler_state1's count, gs + 9)
    constexpr int kJumpBatch = 3;
    unsigned long long* jc = nullptr;
    APG_TRY(workspace_t(ctx, "u_jcnt", (uint64_t)max_rounds + 1, &jc));
    APG_CHECK_HIP(hipMemsetAsync(jc, 0, ((uint64_t)max_rounds + 1) * 8, ctx->stream));
    const uint32_t jgrid = grid_for(ctx, na);
    for (int it = 0; it < max_rounds && na; ++it) {
      kbegin(ctx, "u_ruler_jump", na * 48);
      k_ruler_jump<<<jgrid, 256, 0, ctx->stream>>>(it ? jc + it - 1 : gs + 9, ain, rb.state, aout, jc + it);
      kend(ctx);
      std::swap(ain, aout);
      if ((it + 1) % kJumpBatch == 0 || it + 1 == max_rounds) APG_TRY(d2h_u64(ctx, jc + it, &na, 1));
    }
    APG_CHECK_HIP(hipGetLastError());
    // cycles? (and the final ranks of every other node)
    uint32_t* clist = nullptr;
    APG_TRY(workspace_t(ctx, "u_clist", std::max<uint64_t>(D, 1), &clist));
    APG_TRY(workspace_t(ctx, "u_head", std::max<uint64_t>(D, 1), head));
    APG_TRY(workspace_t(ctx, "u_rank", std::max<uint64_t>(D, 1), rank));
    APG_TRY(workspace_t(ctx, "u_chainlen", std::max<uint64_t>(D, 1), chainlen));
    APG_TRY(workspace_t(ctx, "u_tailof", std::max<uint64_t>(D, 1), tail_of));
    kbegin(ctx, "u_rank_final", D * 24);
    k_rank_mark<<<grid_for(ctx, D), 256, 0, ctx->stream>>>(D, rb, clist, gs + 12, *head, *rank, *chainlen, *tail_of);
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
    unsigned long long hc;
    APG_TRY(d2h_u64(ctx, gs + 12, &hc, 1));
    if (hc == 0) break;
    if (attempt == 2) {
      set_error("unipaths: cycles remain after cutting (internal error)");
      return APG_E_STATE;
    }
    // min K-mer of every cycle by pointer jumping, then cut; ranking reruns
    const uint64_t C = hc;
    uint32_t *cm0 = rb.alist0, *cn0 = rb.alist1, *cm1 = rb.rnext, *cn1 = rb.seglen;  // free D-sized scratch
    k_cyc_init<<<grid_for(ctx, C), 256, 0, ctx->stream>>>(C, clist, rb.dn, cm0, cn0);
    const int cr = ceil_log2_u(C + 1) + 1;
    for (int it = 0; it < cr; ++it) {
      k_cyc_jump<<<grid_for(ctx, C), 256, 0, ctx->stream>>>(C, clist, nodes, kp, cm0, cn0, cm1, cn1);
      std::swap(cm0, cm1);
      std::swap(cn0, cn1);
    }
    k_cyc_cut<<<grid_for(ctx, C), 256, 0, ctx->stream>>>(C, clist, nodes, kp, cm0, rb.dn, gs + 13);
    APG_CHECK_HIP(hipGetLastError());
    unsigned long long hcut;
    APG_TRY(d2h_u64(ctx, gs + 13, &hcut, 1));
    st->n_cycles_cut += hcut;
    vlog(ctx, "unipaths: %llu cyclic directed nodes, %llu cuts", hc, hcut);
  }

  return APG_OK;
}

// Stable LSD radix sort of P 192-bit keys (pk[0..2], scratch pk[3..5]) with
// a u32 payload (ph, scratch ph2), skipping digits constant over all keys;
// *sorted = the payload array holding the result.
static int u_sort_keys(apg_ctx* ctx, uint64_t P, uint64_t* pk[6], uint32_t* ph, uint32_t* ph2,
                       unsigned long long* gs, uint32_t** sorted) {
  *sorted = ph;
  {
    APG_CHECK_HIP(hipMemsetAsync(gs + 16, 0, 3 * 8, ctx->stream));
    APG_CHECK_HIP(hipMemsetAsync(gs + 20, 0xff, 3 * 8, ctx->stream));
    k_digit_or<<<grid_for(ctx, P), 256, 0, ctx->stream>>>(pk[0], pk[1], pk[2], P, gs + 16, gs + 20);
    unsigned long long ho[7];
    APG_TRY(d2h_u64(ctx, gs + 16, ho, 7));
    const uint64_t Gs = std::max<uint64_t>(1, (P + kSortTile - 1) / kSortTile);
    uint32_t* scm = nullptr;
    uint64_t* som = nullptr;
    APG_TRY(workspace_t(ctx, "u_scm", 256 * Gs, &scm));
    APG_TRY(workspace_t(ctx, "u_som", 256 * Gs + 1, &som));
    uint64_t *a0 = pk[0], *a1 = pk[1], *a2 = pk[2], *b0 = pk[3], *b1 = pk[4], *b2 = pk[5];
    uint32_t *ap = ph, *bp = ph2;
    // One-pass form (APG_U_SORT=lsd: the LSD passes only): bins on the most
    // significant varying bits (~32 keys each), ranked in LDS; a bin over
    // kBinSortMax keys sends the whole sort to the LSD passes below.
    static const bool lsd_only = getenv("APG_U_SORT") && !strcmp(getenv("APG_U_SORT"), "lsd");
    int top = -1;
    for (int sel = 0; sel < 3 && top < 0; ++sel)
      if (ho[sel] ^ ho[4 + sel]) top = sel;
    if (!lsd_only && P > 1 && P < (1ull << 32) && top >= 0) {
      const uint64_t vary = ho[top] ^ ho[4 + top];
      const int hi = 63 - __builtin_clzll(vary);
      const int want = std::max(1, std::min(16, ceil_log2_u((P + 31) / 32)));
      const int lo = std::max(0, hi - want + 1);
      const MsdDigit dg{lo, (uint32_t)((1ull << (hi - lo + 1)) - 1)};
      const uint64_t* kw = top == 0 ? a0 : top == 1 ? a1 : a2;
      const uint64_t nbins = (uint64_t)dg.mask + 1;
      uint32_t *bcnt = nullptr, *bcur = nullptr, *sidx = nullptr;
      uint64_t* boff = nullptr;
      unsigned int* bmax = nullptr;
      APG_TRY(workspace_t(ctx, "u_sbcnt", 2 * nbins + 2, &bcnt));
      APG_TRY(workspace_t(ctx, "u_sboff", nbins + 1, &boff));
      APG_TRY(workspace_t(ctx, "u_sidx", P, &sidx));
      bcur = bcnt + nbins;
      bmax = bcnt + 2 * nbins;
      APG_CHECK_HIP(hipMemsetAsync(bcnt, 0, (2 * nbins + 2) * 4, ctx->stream));
      kbegin(ctx, "u_sort_bins", P * 24 * 3 + P * 8);
      k_msd_count<<<grid_for(ctx, P), 256, 0, ctx->stream>>>(kw, P, dg, bcnt);
      APG_TRY(scan_u32_u64(ctx, bcnt, nbins, boff, "usb"));
      k_msd_scatter<<<grid_for(ctx, P), 256, 0, ctx->stream>>>(SortCols{a0, a1, a2, ap, b0, b1, b2, bp}, kw, P, dg, boff,
                                                               bcur, sidx, bcnt, nbins, bmax);
      kend(ctx);
      APG_CHECK_HIP(hipGetLastError());
      unsigned int hmax = 0;
      APG_TRY(d2h_sync(ctx, &hmax, bmax, 4));
      vlog(ctx, "unipaths: pair keys %llu, bins %llu (word %d bits %d-%d), largest %u", (unsigned long long)P,
           (unsigned long long)nbins, top, lo, hi, hmax);
      // APG_U_SORT_BINMAX (tests): a lower bin limit, so the LSD fallback runs
      static const uint32_t binmax = [] {
        const char* e = getenv("APG_U_SORT_BINMAX");
        return e ? std::min<uint32_t>(kBinSortMax, (uint32_t)std::max(0, atoi(e))) : kBinSortMax;
      }();
      if (hmax <= binmax) {
        kbegin(ctx, "u_sort_rank", P * 28 * 2);
        k_bin_sort<<<(uint32_t)nbins, 256, 0, ctx->stream>>>(b0, b1, b2, bp, sidx, boff, ap);
        kend(ctx);
        APG_CHECK_HIP(hipGetLastError());
        *sorted = ap;
        return APG_OK;
      }
      vlog(ctx, "unipaths: pair-key bin of %u keys: LSD passes", hmax);
    }
      for (int sel = 2; sel >= 0 && P > 1; --sel) {
      const uint64_t varying = ho[sel] ^ ho[4 + sel];  // bits not constant over all keys
      for (int shift = 0; shift < 64; shift += 8) {
        if (((varying >> shift) & 255) == 0) continue;
        const uint64_t* key = sel == 0 ? a0 : sel == 1 ? a1 : a2;
        kbegin(ctx, "u_sort_count", P * 8);
        k_lsd_count<<<Gs, kSortThreads, 0, ctx->stream>>>(key, P, shift, scm);
        kend(ctx);
        const bool fuse = Gs <= kSortFuseTiles;
        if (!fuse) APG_TRY(scan_u32_u64(ctx, scm, 256 * Gs, som, "us"));
        SortCols c{a0, a1, a2, ap, b0, b1, b2, bp};
        kbegin(ctx, "u_sort_scatter", P * 28 * 2);
        k_lsd_scatter<<<Gs, kSortThreads, 0, ctx->stream>>>(c, sel, P, shift, fuse ? nullptr : som, scm);
        kend(ctx);
        std::swap(a0, b0);
        std::swap(a1, b1);
        std::swap(a2, b2);
        std::swap(ap, bp);
      }
    }
    APG_CHECK_HIP(hipGetLastError());
    *sorted = ap;
    }
  return APG_OK;
}

static int u_graph(apg_ctx* ctx, const KRec* nodes, uint64_t N, const apg_dreads* dr, const apg_unipath_params& prm,
                   apg_unipath_graph* out, apg_unipath_stats* st, const uint2* lsucc = nullptr,
                   const PreIdx* pidx = nullptr) {
  const int K = prm.K;
  const KeyP kp = make_keyp(K);
  st->n_nodes = N;
  ctx->gstate.valid = false;
  if (N >= (1ull << 31)) {
    set_error("unipaths: more than 2^31 distinct K-mers on one device");
    return APG_E_UNSUPPORTED;
  }
  const uint64_t D = 2 * N;
  const uint64_t n = st->n_instances;
  unsigned long long* gs = nullptr;  // general device counters
  APG_TRY(workspace_t(ctx, "u_gs", 32, &gs));
  APG_CHECK_HIP(hipMemsetAsync(gs, 0, 32 * 8, ctx->stream));
  ReadsV rv{nullptr, nullptr, nullptr, 0};
  if (dr) rv = ReadsV{dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->n_reads};

  // ---- U4 index --------------------------------------------------------------
  uint64_t T = 1024;
  unsigned long long* idx = nullptr;
  if (pidx && pidx->idx) {  // built by the node buckets (usk_stage)
    idx = pidx->idx;
    T = pidx->T;
  } else {
    while (T < 2 * N) T <<= 1;
    APG_TRY(workspace_t(ctx, "u_idx", T, &idx));
    APG_CHECK_HIP(hipMemsetAsync(idx, 0xff, T * 8, ctx->stream));
    kbegin(ctx, "u_node_insert", N * 40);
    k_node_insert<<<grid_for(ctx, N), 256, 0, ctx->stream>>>(nodes, 0, N, idx, T - 1);
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
  }
  const NodeIdx ni{nodes, idx, T - 1};

  // ---- U5 --------------------------------------------------------------------
  RankBufs rb{};
  APG_TRY(workspace_t(ctx, "u_dn", std::max<uint64_t>(D, 1), &rb.dn));
  APG_CHECK_HIP(hipMemsetAsync(rb.dn, 0xff, D * sizeof(DN), ctx->stream));
  // algorithmic bytes: ~2 index lookups per node, or with the buckets' local
  // links the 8-byte link record per node (+ 64 B per remaining lookup, added
  // below)
  kbegin(ctx, "u_links", lsucc ? N * 8 : N * 64);
  k_links<<<grid_for(ctx, N), 256, 0, ctx->stream>>>(ni, N, kp, rb.dn, gs + 4, lsucc);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  unsigned long long hl[3];
  APG_TRY(d2h_u64(ctx, gs + 4, hl, 3));
  if (lsucc) kbytes_add(ctx, "u_links", hl[2] * 64);  // the index lookups left to this pass
  st->n_links = hl[0];
  if (hl[1]) {
    set_error("unipaths: read-supported edge to a missing K-mer (internal error)");
    return APG_E_STATE;
  }

  // ---- U6 --------------------------------------------------------------------
  uint32_t *head = nullptr, *rank = nullptr, *chainlen = nullptr, *tail_of = nullptr;
  APG_TRY(u_rank_all(ctx, nodes, N, kp, rb, gs, st, &head, &rank, &chainlen, &tail_of));

  // ---- U7 --------------------------------------------------------------------
  // pair keys (one per (u, rc u)): at most N pairs
  uint64_t *pk[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  uint32_t *ph = nullptr, *ph2 = nullptr;
  const uint64_t PM = std::max<uint64_t>(N, 1);
  const char* pkn[6] = {"u_pk0", "u_pk1", "u_pk2", "u_pk3", "u_pk4", "u_pk5"};
  for (int i = 0; i < 6; ++i) APG_TRY(workspace_t(ctx, pkn[i], PM, &pk[i]));
  APG_TRY(workspace_t(ctx, "u_ph", PM, &ph));
  APG_TRY(workspace_t(ctx, "u_ph2", PM, &ph2));
  kbegin(ctx, "u_pairs", D * 12);
  k_pairs<<<grid_for(ctx, D), 256, 0, ctx->stream>>>(D, rb.dn, tail_of, nodes, kp, pk[0], pk[1], pk[2], ph, gs + 14,
                                                     gs + 15);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  unsigned long long hp[2];
  APG_TRY(d2h_u64(ctx, gs + 14, hp, 2));
  const uint64_t P = hp[0], U = hp[1];
  st->n_unipaths = U;
  // LSD radix sort of (k0, k1, k2) with payload h, skipping constant digits
  APG_TRY(u_sort_keys(ctx, P, pk, ph, ph2, gs, &ph));
  uint32_t *sz = nullptr, *uni_of_head = nullptr, *uhead = nullptr;
  uint64_t *ustart = nullptr, *ulen = nullptr, *urc = nullptr, *id_base = nullptr, *ub_off = nullptr;
  APG_TRY(workspace_t(ctx, "u_sz", PM, &sz));
  APG_TRY(workspace_t(ctx, "u_ustart", PM + 1, &ustart));
  APG_TRY(workspace_t(ctx, "u_uoh", std::max<uint64_t>(D, 1), &uni_of_head));
  APG_TRY(workspace_t(ctx, "u_uhead", std::max<uint64_t>(U, 1), &uhead));
  APG_TRY(workspace_t(ctx, "u_ulen", std::max<uint64_t>(U, 1), &ulen));
  APG_TRY(workspace_t(ctx, "u_urc", std::max<uint64_t>(U, 1), &urc));
  APG_TRY(workspace_t(ctx, "u_idbase", U + 1, &id_base));
  APG_TRY(workspace_t(ctx, "u_uboff", U + 1, &ub_off));
  k_pair_sizes<<<grid_for(ctx, P), 256, 0, ctx->stream>>>(P, ph, tail_of, sz);
  APG_TRY(scan_u32_u64(ctx, sz, P, ustart, "ua"));
  k_assign<<<grid_for(ctx, P), 256, 0, ctx->stream>>>(P, ph, tail_of, ustart, chainlen, uni_of_head, uhead, ulen, urc);
  APG_CHECK_HIP(hipGetLastError());
  // ids and unibase offsets: scans over lengths (u32 copies of ulen)
  uint32_t* lens32 = nullptr;
  APG_TRY(workspace_t(ctx, "u_lens32", std::max<uint64_t>(U, 1), &lens32));
  k_u32_of<<<grid_for(ctx, U), 256, 0, ctx->stream>>>(ulen, U, 0, lens32);
  APG_TRY(scan_u32_u64(ctx, lens32, U, id_base, "ui"));
  k_u32_of<<<grid_for(ctx, U), 256, 0, ctx->stream>>>(ulen, U, (uint32_t)(K - 1), lens32);
  APG_TRY(scan_u32_u64(ctx, lens32, U, ub_off, "uu"));
  if (U) k_u64_max<<<grid_for(ctx, U), 256, 0, ctx->stream>>>(ulen, U, gs + 26);
  APG_CHECK_HIP(hipGetLastError());

  // Read paths, count pass: on the auxiliary stream beside U8 (unibases and
  // HyperKmerPath need nothing it writes; APG_U_PATHS_AUX=0: in line after U8)
  const bool want_paths = dr && (prm.flags & APG_UNIPATH_READ_PATHS) != 0;
  uint32_t* nint = nullptr;
  uint64_t *ioff = nullptr, *istart = nullptr, *ilen = nullptr;
  uint64_t NI = 0;
  const char* pe = getenv("APG_U_PATHS_AUX");
  const hipStream_t pax = want_paths && !(pe && !strcmp(pe, "0")) ? aux_stream(ctx) : nullptr;
  const uint32_t rg = want_paths ? grid_for(ctx, dr->n_reads) : 1;
  auto paths_count = [&]() -> int {
    kbegin(ctx, "u_read_paths_count", dr->n_bytes + n * 8);
    k_read_paths<false><<<rg, 256, 0, ctx->stream>>>(rv, ni, kp, head, rank, uni_of_head, id_base, ulen, nint,
                                                     nullptr, nullptr, nullptr, gs + 25);
    kend(ctx);
    return scan_u32_u64(ctx, nint, dr->n_reads, ioff, "up");
  };
  if (want_paths) {
    APG_TRY(workspace_t(ctx, "u_nint", std::max<uint64_t>(dr->n_reads, 1), &nint));
    APG_TRY(workspace_t(ctx, "u_ioff", dr->n_reads + 1, &ioff));
    if (pax) {
      hipEvent_t ready = nullptr;
      APG_CHECK_HIP(hipEventCreateWithFlags(&ready, hipEventDisableTiming));
      APG_CHECK_HIP(hipEventRecord(ready, ctx->stream));  // id_base, ulen, uni_of_head complete
      APG_CHECK_HIP(hipStreamWaitEvent(pax, ready, 0));
      APG_CHECK_HIP(hipEventDestroy(ready));
      StreamSwap sw(ctx, pax);
      APG_TRY(paths_count());
    }
  }

  // ---- U8 --------------------------------------------------------------------
  uint64_t tot_ub = 0;
  APG_TRY(d2h_sync(ctx, &tot_ub, ub_off + U, 8));
  uint8_t* ub = nullptr;
  APG_TRY(workspace_t(ctx, "u_ub", std::max<uint64_t>(tot_ub, 1), &ub));
  kbegin(ctx, "u_unibases", D * 16 + tot_ub);
  k_unibases<<<grid_for(ctx, D), 256, 0, ctx->stream>>>(D, nodes, kp, head, rank, uni_of_head, ub_off, ub);
  kend(ctx);
  uint32_t *par = nullptr, *isroot = nullptr;
  uint64_t *vid = nullptr, *from = nullptr, *to = nullptr;
  APG_TRY(workspace_t(ctx, "u_par", std::max<uint64_t>(2 * U, 1), &par));
  APG_TRY(workspace_t(ctx, "u_isroot", std::max<uint64_t>(2 * U, 1), &isroot));
  APG_TRY(workspace_t(ctx, "u_vid", 2 * U + 1, &vid));
  APG_TRY(workspace_t(ctx, "u_from", std::max<uint64_t>(U, 1), &from));
  APG_TRY(workspace_t(ctx, "u_to", std::max<uint64_t>(U, 1), &to));
  k_uf_init<<<grid_for(ctx, 2 * U), 256, 0, ctx->stream>>>(2 * U, par);
  kbegin(ctx, "u_adjacency", U * 64);
  k_adjacency<<<grid_for(ctx, U), 256, 0, ctx->stream>>>(U, ni, kp, uhead, tail_of, head, uni_of_head, par, gs + 24);
  kend(ctx);
  k_uf_roots<<<grid_for(ctx, 2 * U), 256, 0, ctx->stream>>>(2 * U, par, isroot);
  APG_TRY(scan_u32_u64(ctx, isroot, 2 * U, vid, "uv"));
  k_hkp_edges<<<grid_for(ctx, U), 256, 0, ctx->stream>>>(U, par, vid, from, to);
  APG_CHECK_HIP(hipGetLastError());
  unsigned long long hv[2];
  APG_CHECK_HIP(hipMemcpyAsync(hv, vid + 2 * U, 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(d2h_sync(ctx, hv + 1, gs + 24, 8));
  st->n_vertices = hv[0];
  if (hv[1]) {
    set_error("unipaths: adjacency edge to a missing K-mer (internal error)");
    return APG_E_STATE;
  }
  // read paths
  if (want_paths) {
    if (pax) {  // the count pass ran beside U8: its total, then the write pass here
      StreamSwap sw(ctx, pax);
      APG_TRY(d2h_sync(ctx, &NI, ioff + dr->n_reads, 8));
    } else {
      APG_TRY(paths_count());
      APG_TRY(d2h_sync(ctx, &NI, ioff + dr->n_reads, 8));
    }
    APG_TRY(workspace_t(ctx, "u_istart", std::max<uint64_t>(NI, 1), &istart));
    APG_TRY(workspace_t(ctx, "u_ilen", std::max<uint64_t>(NI, 1), &ilen));
    kbegin(ctx, "u_read_paths_write", dr->n_bytes + n * 8 + NI * 16);
    k_read_paths<true><<<rg, 256, 0, ctx->stream>>>(rv, ni, kp, head, rank, uni_of_head, id_base, ulen, nullptr,
                                                    ioff, istart, ilen, gs + 25);
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
    st->n_intervals = NI;
  }
  {
    unsigned long long ml = 0;
    APG_TRY(d2h_u64(ctx, gs + 26, &ml, 1));
    st->max_len = ml;
  }
  {
    apg_ctx::GState& g = ctx->gstate;
    g.K = K;
    g.n_nodes = N;
    g.n_unipaths = U;
    g.tmask = T - 1;
    g.nodes = nodes;
    g.idx = idx;
    g.head = head;
    g.rank = rank;
    g.uoh = uni_of_head;
    g.ulen = ulen;
    g.urc = urc;
    g.ub_off = ub_off;
    g.ub = ub;
    g.uloc = nullptr;  // rebuilt on the next apg_unipath_locs
    g.sharded = false;
    g.vu = g.vr = nullptr;
    g.comm = nullptr;
    g.n_shards = 1;
    g.valid = true;
  }
  if (!out) return APG_OK;

  // ---- host copies ------------------------------------------------------------
  int rc = APG_OK;
  std::vector<D2HJob> jobs;  // every array through the pinned staging, after one sync
  std::memset(out, 0, sizeof(*out));
  out->K = K;
  out->n_nodes = N;
  out->n_unipaths = U;
  out->len = host_dup(ulen, U, &jobs, &rc);
  out->id_base = host_dup(id_base, U, &jobs, &rc);
  out->rc = host_dup(urc, U, &jobs, &rc);
  out->ub_off = host_dup(ub_off, U + 1, &jobs, &rc);
  out->unibases = host_dup(ub, tot_ub, &jobs, &rc);
  out->n_vertices = hv[0];
  out->from = host_dup(from, U, &jobs, &rc);
  out->to = host_dup(to, U, &jobs, &rc);
  out->n_reads = want_paths ? dr->n_reads : 0;
  out->n_intervals = NI;
  if (want_paths) {
    out->path_off = host_dup(ioff, dr->n_reads + 1, &jobs, &rc);
    out->path_start = host_dup(istart, NI, &jobs, &rc);
    out->path_len = host_dup(ilen, NI, &jobs, &rc);
  }
  if (rc == APG_OK) rc = sync(ctx);
  const auto t_d2h = std::chrono::steady_clock::now();
  if (rc == APG_OK) rc = d2h_bulk(ctx, jobs);
  if (ctx->verbose) {
    uint64_t bytes = 0;
    for (const auto& j : jobs) bytes += j.bytes;
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_d2h).count();
    vlog(ctx, "unipaths: graph to host %.1f MB in %.1f ms (%.1f GB/s)", bytes / 1e6, ms, bytes / 1e6 / std::max(ms, 1e-3));
  }
  return rc;
}

// U1'-U3': distinct nodes through minimizer partitions, in three steps that
// the single-GPU build chains directly and the multi-GPU build splits around
// an all_to_all of the 48-byte records (P shards = the top log2 P key bits):
//   usk_plan     count records per (shard, digit) and per-block offsets
//   usk_scatter  the records, grouped by (shard, digit)
//   usk_stage    partition levels of one shard's records (P source segments
//                per digit) + LDS buckets -> distinct nodes in "usk_nodes"
// The count pass's dynamic LDS: its walk words, then hist[ndig], khist[ndig].
static size_t usk_count_lds(const UskP& p, int D) { return (size_t)usk_count_words(p) * 4 + ((size_t)1 << D) * 8; }

// Walk grid cap: two full rounds of the resident blocks of the count pass or
// of the scatter pass, whichever holds more per CU (see sk_blocks; the two
// passes share the grid: the scatter replays the count's per-block
// descriptor regions)
static uint64_t usk_grid_cap(const apg_ctx* ctx, const UskP& p, int D) {
  int occ = 0, occ_c = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k_usk_scatter, kUskThreads, usk_walk_lds(p, D, 8)) !=
          hipSuccess ||
      occ < 1)
    occ = 4;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ_c, k_usk_count, kUskThreads, usk_count_lds(p, D)) ==
      hipSuccess)
    occ = std::max(occ, occ_c);
  else
    (void)hipGetLastError();
  return std::min<uint64_t>(kUskMaxBlocks, (uint64_t)std::max(ctx->n_cu, 1) * occ * 2);
}

// Record descriptors of the count pass (SkDesc, superkmer.hpp): fragments
// carry ~1 record per 48 bases at K = 96; one 8-byte slot per kUskDescDiv.
constexpr uint32_t kUskDescDiv = 16;
static int usk_desc_bufs(apg_ctx* ctx, const apg_dreads* dr, uint32_t G, SkDesc* out) {
  const char* env = getenv("APG_SK_DESC");  // "0": off; a number: bases per slot (tests force overflow)
  const uint32_t div = env && atoi(env) > 0 ? (uint32_t)atoi(env) : kUskDescDiv;
  *out = SkDesc{nullptr, nullptr, nullptr, div, 0};
  if ((env && !strcmp(env, "0")) || !dr->n_reads || !dr->n_bases) return APG_OK;
  out->slots = dr->n_bases / div + 1;
  APG_TRY(workspace_t(ctx, "usk_desc", out->slots, &out->desc));
  APG_TRY(workspace_t(ctx, "usk_dtcnt", dr->n_reads, &out->tcnt));
  APG_TRY(workspace_t(ctx, "usk_dflag", G, &out->flag));
  return APG_OK;
}

static int usk_plan(apg_ctx* ctx, const apg_dreads* dr, const UskP& p, int P, std::vector<uint64_t>* h,
                    std::vector<uint64_t>* kd, uint32_t* G_out) {
  if (p.w > kUskMaxW) {
    set_error("unipaths: minimizer window exceeds kUskMaxW");
    return APG_E_UNSUPPORTED;
  }
  const int D = ceil_log2_u((uint64_t)P) + kUskDigitBits;
  const uint32_t ndig = 1u << D;
  const uint32_t G =
      (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(usk_grid_cap(ctx, p, D), (dr->n_reads + kUskThreads - 1) / kUskThreads));
  SkReads rv{dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->n_reads};
  const size_t sb_bytes = usk_count_lds(p, D);
  uint32_t* cmat = nullptr;
  uint64_t *omat = nullptr, *ds = nullptr;
  unsigned long long* kdig = nullptr;
  APG_TRY(workspace_t(ctx, "usk_cmat", (uint64_t)ndig * G, &cmat));
  APG_TRY(workspace_t(ctx, "usk_omat", (uint64_t)ndig * G + 1, &omat));
  APG_TRY(workspace_t(ctx, "usk_ds", ndig + 1, &ds));
  APG_TRY(workspace_t(ctx, "usk_kdig", ndig, &kdig));
  APG_CHECK_HIP(hipMemsetAsync(kdig, 0, ndig * 8, ctx->stream));
  if (!dr->n_reads) APG_CHECK_HIP(hipMemsetAsync(cmat, 0, (uint64_t)ndig * G * 4, ctx->stream));
  SkDesc dd;
  APG_TRY(usk_desc_bufs(ctx, dr, G, &dd));
  kbegin(ctx, "usk_count", dr->n_bytes + 16 * dr->n_reads);
  if (dr->n_reads) k_usk_count<<<G, kUskThreads, sb_bytes, ctx->stream>>>(rv, p, D, cmat, kdig, dd);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  APG_TRY(scan_u32_u64(ctx, cmat, (uint64_t)ndig * G, omat, "usk"));
  k_usk_digit_starts<<<(ndig + 256) / 256, 256, 0, ctx->stream>>>(omat, ndig, G, ds);
  h->assign(ndig + 1, 0);
  kd->assign(ndig, 0);
  APG_CHECK_HIP(hipMemcpyAsync(h->data(), ds, (ndig + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(d2h_sync(ctx, kd->data(), kdig, ndig * 8));
  *G_out = G;
  auto& us = ctx->urstate;
  us.valid = true;
  us.gen = dr->gen;
  us.K = p.K;
  us.P = P;
  us.G = G;
  us.n = (*h)[ndig];
  us.desc = dd.desc != nullptr;
  if (us.desc) kbytes_add(ctx, "usk_count", us.n * 8);  // the records' descriptors, written
  return APG_OK;
}

static int usk_scatter(apg_ctx* ctx, const apg_dreads* dr, const UskP& p, int P, uint32_t G, SK48* out) {
  const int D = ceil_log2_u((uint64_t)P) + kUskDigitBits;
  SkReads rv{dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->n_reads};
  const size_t sb_bytes = usk_walk_lds(p, D, 8);  // + hist, khist (count) or cursors (scatter)
  uint64_t* omat = nullptr;
  APG_TRY(workspace_t(ctx, "usk_omat", (uint64_t)(1u << D) * G + 1, &omat));
  const auto& us = ctx->urstate;
  SkDesc dd{nullptr, nullptr, nullptr, kUskDescDiv, 0};
  if (us.valid && us.desc && us.gen == dr->gen && us.G == G && us.K == p.K && us.P == P)
    APG_TRY(usk_desc_bufs(ctx, dr, G, &dd));
  kbegin(ctx, "usk_scatter", dr->n_bytes + 16 * dr->n_reads + ctx->urstate.n * (sizeof(SK48) + (dd.desc ? 8 : 0)));
  if (dr->n_reads) k_usk_scatter<<<G, kUskThreads, sb_bytes, ctx->stream>>>(rv, p, D, omat, out, dd);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  return APG_OK;
}

// One shard's records src (rc = counts [src * 32 + digit], src-major layout)
// -> distinct nodes.  The records' top log2(P) + kUskDigitBits key bits are
// consumed; `spare` (may be src itself when it may be overwritten) is a
// second record buffer.
// lsucc_out (may be null): the buckets' local links for k_links (null on
// return when they could not be kept: overflowed nodes beyond the list, or
// too many nodes)
static int usk_stage(apg_ctx* ctx, const SK48* src, const std::vector<uint64_t>& rc, uint64_t nk, const KeyP& kp,
                     int P, KRec** nodes_out, uint64_t* N_out, uint2** lsucc_out = nullptr, PreIdx* pidx = nullptr) {
  const int pbits = ceil_log2_u((uint64_t)P);
  const int D = kUskDigitBits;
  const uint32_t ndig = 1u << D;
  if (rc.size() != (size_t)P * ndig) {
    set_error("unipaths: record counts have the wrong size");
    return APG_E_ARG;
  }
  uint64_t n = 0;
  for (auto c : rc) n += c;
  SK48 *bufA = nullptr, *bufB = nullptr;
  APG_TRY(workspace_t(ctx, kBig0, std::max<uint64_t>(n, 1) + 1, &bufA));
  APG_TRY(workspace_t(ctx, kBig1, std::max<uint64_t>(n, 1) + 1, &bufB));
  // partition levels on the key bits below the shard + digit bits
  // APG_USK_BUCKET_KMERS=n: instances per node bucket the levels aim for (A/B)
  static const uint64_t bk_kmers = getenv("APG_USK_BUCKET_KMERS") ? std::max(64, atoi(getenv("APG_USK_BUCKET_KMERS")))
                                                                  : kUskBucketKmers;
  const uint64_t need = std::max<uint64_t>(1, (nk + bk_kmers - 1) / bk_kmers);
  const int bb = std::min(32 - pbits, std::max(D, ceil_log2_u(need)));
  const int rem = bb - D;
  int nlev = (rem + kMaxLevelBits - 1) / kMaxLevelBits;
  if (nlev == 0 && P > 1) nlev = 1;  // regroup the P source segments
  std::vector<std::vector<Seg>> parents(ndig);
  {
    uint64_t pos = 0;
    for (int s = 0; s < P; ++s)
      for (uint32_t d = 0; d < ndig; ++d) {
        const uint64_t c = rc[(size_t)s * ndig + d];
        parents[d].push_back(Seg{pos, c});
        pos += c;
      }
  }
  uint64_t* boff = nullptr;
  APG_TRY(workspace_t(ctx, "usk_boff", (1ull << bb) + 1, &boff));
  if (nlev == 0) {
    std::vector<uint64_t> hb(ndig + 1, 0);
    for (uint32_t d = 0; d < ndig; ++d) hb[d + 1] = hb[d] + rc[d];
    APG_CHECK_HIP(hipMemcpyAsync(boff, hb.data(), (ndig + 1) * 8, hipMemcpyHostToDevice, ctx->stream));
  }
  const SK48* cur = src;
  uint64_t nb = ndig;
  int consumed = pbits + D;
  std::vector<uint64_t> bounds;  // after the first level: one segment per parent
  for (int lev = 0; lev < nlev; ++lev) {
    const int bits = rem / nlev + (lev < rem % nlev ? 1 : 0);
    consumed += bits;
    SK48* dst = cur == bufA ? bufB : bufA;
    std::vector<uint64_t> hb;
    const bool last = lev + 1 == nlev;
    const PartParents pp = lev ? PartParents(bounds) : PartParents(parents);
    APG_TRY(part_level<SK48>(ctx, cur, dst, pp, 64 - consumed, bits, n, boff, last ? nullptr : &hb, "usk"));
    nb = pp.size() << bits;
    if (!last) bounds.swap(hb);
    cur = dst;
  }
  // buckets -> nodes
  unsigned long long* gs = nullptr;
  uint32_t* ovf = nullptr;
  APG_TRY(workspace_t(ctx, "usk_gs", 6, &gs));
  APG_TRY(workspace_t(ctx, "usk_ovf", std::max<uint64_t>(nb, 1), &ovf));
  // APG_USK_TAB=512: small-table first pass, its overflowed buckets again
  // with the full table (gs[5] counts them, listed in ovf1)
  const char* te = getenv("APG_USK_TAB");
  const bool small_tab = te && !strncmp(te, "512", 3);
  const bool small_w6 = te && !strcmp(te, "512w6");  // VGPRs capped for 6 waves / SIMD (spills)
  uint32_t* ovf1 = nullptr;
  if (small_tab) APG_TRY(workspace_t(ctx, "usk_ovf1", std::max<uint64_t>(nb, 1), &ovf1));
  uint64_t cap = std::max<uint64_t>(1 << 20, nk / 4);
  KRec* nodes = nullptr;
  unsigned long long hs[5];
  const uint64_t grid = resident_grid(ctx, k_usk_bucket<kUskTab>, kUskBThreads, nb);
  const uint64_t grid_s = small_w6 ? resident_grid(ctx, k_usk_bucket<kUskTabSmall, 6>, kUskBThreads, nb)
                                   : resident_grid(ctx, k_usk_bucket<kUskTabSmall>, kUskBThreads, nb);
  // APG_USK_DEDUP=0: every record flattened (A/B)
  const char* de = getenv("APG_USK_DEDUP");
  const bool dedup = !(de && !strcmp(de, "0"));
  // APG_USK_DEDUP_STATS=1: count records / instances and what the dedup folds (stderr)
  unsigned long long* dstat = nullptr;
  if (getenv("APG_USK_DEDUP_STATS")) {
    APG_TRY(workspace_t(ctx, "usk_dstat", 4, &dstat));
    APG_CHECK_HIP(hipMemsetAsync(dstat, 0, 32, ctx->stream));
  }
  // The node index built by the buckets (APG_U_IDX_BUCKETS=0: by
  // k_node_insert in u_graph): sized before the node count is known, at
  // 2 slots per 8 instances (the bench step: 2^28 slots for 65 M nodes); a
  // build with more nodes than half of it falls back to k_node_insert.
  const char* ie = getenv("APG_U_IDX_BUCKETS");
  unsigned long long* pre_idx = nullptr;
  uint64_t pre_T = 1024;
  if (pidx && !(ie && !strcmp(ie, "0"))) {
    while (pre_T < 2 * std::max<uint64_t>(nk / 8, 1)) pre_T <<= 1;
    APG_TRY(workspace_t(ctx, "u_idx", pre_T, &pre_idx));
  }
  // APG_U_LOCAL_LINKS=0: every link through the node index (A/B)
  const char* le = getenv("APG_U_LOCAL_LINKS");
  const bool want_ls = lsucc_out && !(le && !strcmp(le, "0"));
  uint2* ls = nullptr;
  for (;;) {
    APG_TRY(workspace_t(ctx, "usk_nodes", cap, &nodes));
    if (want_ls) APG_TRY(workspace_t(ctx, "usk_lsucc", cap, &ls));
    APG_CHECK_HIP(hipMemsetAsync(gs, 0, 6 * 8, ctx->stream));
    if (pre_idx) APG_CHECK_HIP(hipMemsetAsync(pre_idx, 0xff, pre_T * 8, ctx->stream));
    UskOut uo{nodes, cap, gs, ovf, gs + 1, ls, dedup ? 1u : 0u, dstat, pre_idx, pre_T - 1, pre_T / 2};
    static const bool uprof = getenv("APG_USK_PROF") != nullptr;
    if (uprof) {
      APG_TRY(workspace_t(ctx, "usk_prof", 8, &uo.prof));
      APG_CHECK_HIP(hipMemsetAsync(uo.prof, 0, 64, ctx->stream));
    }
    kbegin(ctx, "usk_bucket", n * sizeof(SK48) + (nb + 1) * 8);
    if (small_tab) {
      UskOut u1 = uo;
      u1.ovf_list = ovf1;
      u1.novf = gs + 5;
      if (small_w6)
        k_usk_bucket<kUskTabSmall, 6><<<grid_s, kUskBThreads, 0, ctx->stream>>>(cur, boff, nb, nullptr, kp, u1);
      else
        k_usk_bucket<kUskTabSmall><<<grid_s, kUskBThreads, 0, ctx->stream>>>(cur, boff, nb, nullptr, kp, u1);
      APG_CHECK_HIP(hipGetLastError());
      unsigned long long n1 = 0;
      APG_TRY(d2h_u64(ctx, gs + 5, &n1, 1));
      if (n1)
        k_usk_bucket<kUskTab><<<std::min<uint64_t>(grid, n1), kUskBThreads, 0, ctx->stream>>>(cur, boff, n1, ovf1,
                                                                                               kp, uo);
    } else {
      k_usk_bucket<kUskTab><<<grid, kUskBThreads, 0, ctx->stream>>>(cur, boff, nb, nullptr, kp, uo);
    }
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
    APG_TRY(d2h_u64(ctx, gs, hs, 5));
    if (hs[0] <= cap) break;
    vlog(ctx, "unipaths: %llu nodes exceed the node list (%llu), rerunning", hs[0], (unsigned long long)cap);
    cap = hs[0] + hs[0] / 8;
  }
  {
    static const bool uprof = getenv("APG_USK_PROF") != nullptr;
    if (uprof) {
      unsigned long long* dp = nullptr;
      APG_TRY(workspace_t(ctx, "usk_prof", 8, &dp));
      unsigned long long hp[5];
      APG_TRY(d2h_u64(ctx, dp, hp, 5));
      const double tot = (double)(hp[0] + hp[1] + hp[2] + hp[3] + hp[4]) + 1e-9;
      fprintf(stderr, "[usk_prof] load+dedup %.3f scan+owner %.3f insert %.3f ranks %.3f nodes+index+links %.3f (shares of thread 0's clocks)\n",
              hp[0] / tot, hp[1] / tot, hp[2] / tot, hp[3] / tot, hp[4] / tot);
    }
  }
  if (dstat) {
    unsigned long long d4[4];
    APG_TRY(d2h_u64(ctx, dstat, d4, 4));
    fprintf(stderr, "[usk_dedup] records %llu instances %llu folded records %llu folded instances %llu\n", d4[0], d4[1],
            d4[2], d4[3]);
  }
  uint64_t N = hs[0];
  if (pre_idx && hs[4]) pre_idx = nullptr;  // nodes past half of the index: k_node_insert rebuilds it
  kbytes_add(ctx, "usk_bucket", N * (sizeof(KRec) + (ls ? sizeof(uint2) : 0) + (pre_idx ? 64 : 0)));
  if (hs[1]) {  // overflowed buckets: their instances through the U2 table
    const uint32_t n_ovf = (uint32_t)hs[1];
    const uint32_t g2 = (uint32_t)std::min<uint64_t>(n_ovf, (uint64_t)ctx->n_cu * 8);
    APG_CHECK_HIP(hipMemsetAsync(gs + 2, 0, 16, ctx->stream));
    k_usk_ovf_count<<<g2, 256, 0, ctx->stream>>>(cur, boff, ovf, n_ovf, gs + 2);
    unsigned long long ni[2];
    APG_TRY(d2h_u64(ctx, gs + 2, ni, 2));
    KRec* inst = nullptr;
    APG_TRY(workspace_t(ctx, "usk_inst", std::max<unsigned long long>(ni[0], 1), &inst));
    kbegin(ctx, "usk_ovf_expand", ni[0] * sizeof(KRec));
    k_usk_ovf_expand<<<g2, 256, 0, ctx->stream>>>(cur, boff, ovf, n_ovf, kp, gs + 3, inst);
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
    KRec* fnodes = nullptr;
    uint64_t fN = 0;
    APG_TRY(u_build_nodes(ctx, nullptr, inst, ni[0], kp, (double)ni[0], &fnodes, &fN, nullptr));
    if (N + fN > cap) {  // grow, keeping the bucket nodes
      KRec* tmp = nullptr;
      APG_TRY(workspace_t(ctx, "usk_inst", std::max<uint64_t>(N, 1), &tmp));  // inst no longer needed
      APG_CHECK_HIP(hipMemcpyAsync(tmp, nodes, N * sizeof(KRec), hipMemcpyDeviceToDevice, ctx->stream));
      APG_TRY(workspace_t(ctx, "usk_nodes", N + fN, &nodes));
      APG_CHECK_HIP(hipMemcpyAsync(nodes, tmp, N * sizeof(KRec), hipMemcpyDeviceToDevice, ctx->stream));
    }
    APG_CHECK_HIP(hipMemcpyAsync(nodes + N, fnodes, fN * sizeof(KRec), hipMemcpyDeviceToDevice, ctx->stream));
    vlog(ctx, "unipaths: %u buckets overflow the LDS table (%llu instances, %llu nodes) -> global table", n_ovf,
         ni[0], (unsigned long long)fN);
    // the overflowed buckets' nodes link through the index (kLsGlobal bytes)
    if (ls && N + fN <= cap)
      APG_CHECK_HIP(hipMemsetAsync(ls + N, 0xfe, fN * sizeof(uint2), ctx->stream));
    else
      ls = nullptr;
    if (pre_idx && N + fN <= pre_T / 2) {  // their index entries
      if (fN) k_node_insert<<<grid_for(ctx, fN), 256, 0, ctx->stream>>>(nodes, N, N + fN, pre_idx, pre_T - 1);
      APG_CHECK_HIP(hipGetLastError());
    } else {
      pre_idx = nullptr;
    }
    N += fN;
  }
  if (N >= kLsMaxNodes) ls = nullptr;
  if (lsucc_out) *lsucc_out = ls;
  if (pidx) *pidx = PreIdx{pre_idx, pre_idx ? pre_T : 0};
  vlog(ctx, "unipaths: K=%d P=%d records=%llu instances=%llu levels=%d buckets=%llu nodes=%llu", kp.K, P,
       (unsigned long long)n, (unsigned long long)nk, nlev, (unsigned long long)nb, (unsigned long long)N);
  *nodes_out = nodes;
  *N_out = N;
  return APG_OK;
}

__global__ void k_usk_sum(const SK48* __restrict__ rec, uint64_t n, unsigned long long* __restrict__ out) {
  unsigned long long c = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    c += (uint32_t)(rec[i].w0 >> 32) & 0xff;
  wave_add(out, c);
}

// Single-GPU: plan + scatter into kBig0 (usk_stage's first buffer) + stage.
static int u_sk_nodes(apg_ctx* ctx, const apg_dreads* dr, const KeyP& kp, KRec** nodes_out, uint64_t* N_out,
                      uint64_t* n_inst, uint2** lsucc_out, PreIdx* pidx) {
  const UskP p = make_uskp(kp.K);
  std::vector<uint64_t> h, kd;
  uint32_t G = 0;
  APG_TRY(usk_plan(ctx, dr, p, 1, &h, &kd, &G));
  const uint32_t ndig = 1u << kUskDigitBits;
  const uint64_t n = h[ndig];
  uint64_t nk = 0;
  for (auto x : kd) nk += x;
  *n_inst = nk;
  // the correction stage's tables are dead here: released only under memory
  // pressure (record ping-pong + node table ~ 3 record arrays)
  APG_TRY(ws_make_room(ctx, 3 * n * sizeof(SK48), kRoomCorrection));  // descriptors stay: the scatter replays them
  ctx->ws_dead |= kRoomCorrection;  // and a failed allocation of the graph stages may release them
  SK48* recs = nullptr;
  APG_TRY(workspace_t(ctx, kBig0, std::max<uint64_t>(n, 1) + 1, &recs));
  APG_TRY(usk_scatter(ctx, dr, p, 1, G, recs));
  std::vector<uint64_t> rc(ndig);
  for (uint32_t d = 0; d < ndig; ++d) rc[d] = h[d + 1] - h[d];
  return usk_stage(ctx, recs, rc, nk, kp, 1, nodes_out, N_out, lsucc_out, pidx);
}

static int unipaths_impl(apg_ctx* ctx, const apg_dreads* dr, const apg_unipath_params& prm, apg_unipath_graph* out,
                         apg_unipath_stats* st) {
  const KeyP kp = make_keyp(prm.K);
  std::memset(st, 0, sizeof(*st));
  uint64_t n = 0;
  KRec* nodes = nullptr;
  uint64_t N = 0;
  uint2* lsucc = nullptr;
  PreIdx pidx;
  APG_TRY(u_sk_nodes(ctx, dr, kp, &nodes, &N, &n, &lsucc, &pidx));
  st->n_instances = n;
  return u_graph(ctx, nodes, N, dr, prm, out, st, lsucc, &pidx);
}

}  // namespace apg

using namespace apg;

extern "C" {

void apg_unipath_defaults(apg_unipath_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->K = 96;
  p->flags = APG_UNIPATH_READ_PATHS;
}

// apg_unipath_graph_free: apg_graphio.cpp (host memory only)

int apg_unipaths_dev(apg_ctx* ctx, const apg_dreads* reads, const apg_unipath_params* pp, apg_unipath_graph* out,
                     apg_unipath_stats* stats) {
  APG_REQUIRE(ctx && reads, "apg_unipaths: NULL argument");
  apg_unipath_params p;
  if (pp)
    p = *pp;
  else
    apg_unipath_defaults(&p);
  APG_REQUIRE(p.K >= 1 && p.K <= 96, "apg_unipaths: K must be in [1, 96]");
  if (out) std::memset(out, 0, sizeof(*out));  // a failure frees only what this call allocated
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  apg_unipath_stats st;
  const int rc = unipaths_impl(ctx, reads, p, out, &st);
  if (rc != APG_OK && out) apg_unipath_graph_free(out);
  if (stats) *stats = st;
  return rc;
}

int apg_unipaths(apg_ctx* ctx, const apg_reads* reads, const apg_unipath_params* p, apg_unipath_graph* out,
                 apg_unipath_stats* stats) {
  APG_REQUIRE(ctx && reads && out, "apg_unipaths: NULL argument");
  apg_dreads* dr = nullptr;
  APG_TRY(apg_reads_upload(ctx, reads, &dr));
  const int rc = apg_unipaths_dev(ctx, dr, p, out, stats);
  apg_reads_free(dr);
  return rc;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// Sharded (multi-GPU) unipath build: instance counting sharded by hash,
// distinct nodes gathered by the caller, graph compacted on every rank.
// ---------------------------------------------------------------------------
namespace apg {
static int ushard_check(int K, int P) {
  APG_REQUIRE(K >= 1 && K <= 96, "unipath shard: K must be in [1, 96]");
  APG_REQUIRE(P >= 1 && P <= (1 << kUDigitBits) && (P & (P - 1)) == 0,
              "unipath shard: n_shards must be a power of two in [1, 32]");
  return APG_OK;
}
}  // namespace apg

extern "C" {

int apg_ushard_bins(int n_shards) {
  if (ushard_check(96, n_shards) != APG_OK) return APG_E_ARG;
  return (1 << kUDigitBits) / n_shards;
}

int apg_ushard_count(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards, uint64_t* counts,
                     uint64_t* n_instances) {
  if (ctx) ctx->gstate.valid = false;  // may overwrite the node array of the last graph
  APG_REQUIRE(ctx && reads && counts, "apg_ushard_count: NULL argument");
  APG_TRY(ushard_check(K, n_shards));
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const KeyP kp = make_keyp(K);
  auto& us = ctx->ustate;
  us.valid = false;
  uint64_t n = 0;
  double est = 0;
  APG_TRY(u_size(ctx, reads, kp, &n, &est));
  KRec* nodes = nullptr;
  uint64_t N = 0;
  std::vector<uint64_t> c;
  APG_TRY(u_build_nodes(ctx, reads, nullptr, 0, kp, est, &nodes, &N, &c));
  for (size_t i = 0; i < c.size(); ++i) counts[i] = c[i];  // digit = shard * bins + group: shard-major
  if (n_instances) *n_instances = n;
  us.valid = true;
  us.gen = reads->gen;
  us.K = K;
  us.n = n;
  us.n_local = N;
  us.local_ready = true;
  return APG_OK;
}

int apg_ushard_scatter(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards, void* d_send) {
  APG_REQUIRE(ctx && reads, "apg_ushard_scatter: NULL argument");
  APG_TRY(ushard_check(K, n_shards));
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  auto& us = ctx->ustate;
  if (!us.valid || !us.local_ready || us.gen != reads->gen || us.K != K) {
    std::vector<uint64_t> c(1 << kUDigitBits);
    APG_TRY(apg_ushard_count(ctx, reads, K, n_shards, c.data(), nullptr));
  }
  APG_REQUIRE(us.n_local == 0 || d_send, "apg_ushard_scatter: d_send is NULL");
  KRec* nodes = nullptr;
  APG_TRY(workspace_t(ctx, "u_nodes", std::max<uint64_t>(us.n_local, 1), &nodes));
  if (us.n_local)
    APG_CHECK_HIP(hipMemcpyAsync(d_send, nodes, us.n_local * sizeof(KRec), hipMemcpyDeviceToDevice, ctx->stream));
  return sync(ctx);
}

int apg_ushard_nodes(apg_ctx* ctx, const void* d_recv, const uint64_t* recv_counts, int K, int n_shards,
                     uint64_t* n_nodes) {
  if (ctx) ctx->gstate.valid = false;  // may overwrite the node array of the last graph
  APG_REQUIRE(ctx && recv_counts && n_nodes, "apg_ushard_nodes: NULL argument");
  APG_TRY(ushard_check(K, n_shards));
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const int P = n_shards, B = (1 << kUDigitBits) / P;
  uint64_t n = 0;
  for (int i = 0; i < P * B; ++i) n += recv_counts[i];
  APG_REQUIRE(n == 0 || d_recv, "apg_ushard_nodes: d_recv is NULL");
  KRec* nodes = nullptr;
  uint64_t N = 0;
  ctx->ustate.local_ready = false;  // "u_nodes" is about to hold this shard's merged nodes
  APG_TRY(u_build_nodes(ctx, nullptr, static_cast<const KRec*>(d_recv), n, make_keyp(K), (double)n, &nodes, &N,
                        nullptr));
  APG_TRY(sync(ctx));
  ctx->ustate.n_nodes = N;
  ctx->ustate.n_recv = n;
  *n_nodes = N;
  return APG_OK;
}

int apg_ushard_export(apg_ctx* ctx, void* d_out) {
  APG_REQUIRE(ctx, "apg_ushard_export: NULL ctx");
  const uint64_t N = ctx->ustate.n_nodes;
  if (N == 0) return APG_OK;
  APG_REQUIRE(d_out, "apg_ushard_export: d_out is NULL");
  KRec* nodes = nullptr;
  APG_TRY(workspace_t(ctx, "u_nodes", N, &nodes));
  APG_CHECK_HIP(hipMemcpyAsync(d_out, nodes, N * sizeof(KRec), hipMemcpyDeviceToDevice, ctx->stream));
  return sync(ctx);
}

int apg_unipaths_from_nodes(apg_ctx* ctx, const void* d_nodes, uint64_t n_nodes, const apg_dreads* reads,
                            const apg_unipath_params* pp, apg_unipath_graph* out, apg_unipath_stats* stats) {
  APG_REQUIRE(ctx, "apg_unipaths_from_nodes: NULL ctx");
  APG_REQUIRE(n_nodes == 0 || d_nodes, "apg_unipaths_from_nodes: d_nodes is NULL");
  apg_unipath_params p;
  if (pp)
    p = *pp;
  else
    apg_unipath_defaults(&p);
  APG_REQUIRE(p.K >= 1 && p.K <= 96, "apg_unipaths_from_nodes: K must be in [1, 96]");
  if (out) std::memset(out, 0, sizeof(*out));  // a failure frees only what this call allocated
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  apg_unipath_stats st;
  std::memset(&st, 0, sizeof st);
  st.n_instances = ctx->ustate.n_recv;
  const int rc = u_graph(ctx, static_cast<const KRec*>(d_nodes), n_nodes, reads, p, out, &st);
  if (rc != APG_OK && out) apg_unipath_graph_free(out);
  if (stats) *stats = st;
  return rc;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// UnipathLocs (apg_unipath_locs, spec in include/apg.h; CPU restatement
// oracle/locs_oracle.c).  Recalled reference [R:M]: BuildUnipathLocs /
// ReadLocationLG (src/paths/UnipathLocs*), grep target only.
//
//   k_ulocs<false>  thread per read: roll the read's K-mers (read
//                   orientation), one node-index lookup each (a 100-bp read
//                   has 5 96-mers, so a lookup per K-mer is cheaper than
//                   verifying unipath runs), count the (u, s) changes
//   scan            per-read location offsets
//   k_ulocs<true>   the same walk, writing 16-byte locations (+ rc mirrors)
//   sort (flag)     key (u << 32 | s + 2^31), payload = location index,
//                   stable LSD radix (pathsdb.hip) -> gather
// ---------------------------------------------------------------------------
namespace apg {

struct ULoc {  // == apg_aln_pair
  uint32_t read, unipath;
  int32_t start;
  uint32_t flags;
};

struct GView {
  NodeIdx ni;
  const uint64_t* uloc;  // directed node -> unipath << 32 | rank (one line instead of three dependent ones)
  const uint64_t *ulen, *urc;
};

__global__ void k_uloc_table(uint64_t D, const uint32_t* __restrict__ head, const uint32_t* __restrict__ rank,
                             const uint32_t* __restrict__ uoh, uint64_t* __restrict__ uloc) {
  for (uint64_t v = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; v < D; v += (uint64_t)gridDim.x * blockDim.x)
    uloc[v] = (uint64_t)uoh[head[v]] << 32 | rank[v];
}

template <bool WRITE>
__global__ void __launch_bounds__(256) k_ulocs(ReadsV rv, GView g, KeyP kp, uint32_t flags,
                                               uint32_t* __restrict__ nloc, const uint64_t* __restrict__ loff,
                                               ULoc* __restrict__ out, unsigned long long* __restrict__ cnt) {
  const uint32_t per = (flags & APG_ULOCS_RC) ? 2u : 1u;
  uint64_t missing = 0, placed = 0, lookups = 0;
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < rv.n_reads;
       r += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t len = (uint32_t)(rv.base_off[r + 1] - rv.base_off[r]);
    uint32_t k = 0;
    const uint64_t o = WRITE ? loff[r] : 0;
    if (len >= (uint32_t)kp.K) {
      const uint32_t nk = len - kp.K + 1;
      Roller3 ro;
      ro.init(rv.packed + rv.byte_off[r], len, kp);
      uint32_t pu = 0xffffffffu;
      int64_t ps = 0;
      lookups += nk;
      for (uint32_t j = 0; j < nk; ++j) {
        ro.step(kp);
        const uint32_t v = directed_of(g.ni, ro.fw, kp);
        if (v == kNone) {
          ++missing;
          continue;
        }
        const uint64_t ul = g.uloc[v];
        const uint32_t u = (uint32_t)(ul >> 32);
        const int64_t st = (int64_t)(uint32_t)ul - (int64_t)j;
        if (u == pu && st == ps) continue;
        pu = u;
        ps = st;
        if (WRITE) {
          out[o + k] = ULoc{(uint32_t)r, u, (int32_t)st, 0u};
          if (per == 2) {
            const int64_t ulb = (int64_t)g.ulen[u] + kp.K - 1;
            out[o + k + 1] = ULoc{(uint32_t)r, (uint32_t)g.urc[u], (int32_t)(ulb - (st + (int64_t)len)), APG_ALN_RC};
          }
        }
        k += per;
      }
    }
    placed += k != 0;
    if (!WRITE) nloc[r] = k;
  }
  if (!WRITE) {
    wave_add(&cnt[0], missing);
    wave_add(&cnt[1], placed);
    wave_add(&cnt[2], lookups);
  }
}

__global__ void k_ulocs_keys(const ULoc* __restrict__ loc, uint64_t n, uint64_t* __restrict__ key,
                             uint32_t* __restrict__ val) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const ULoc x = loc[i];
    key[i] = ((uint64_t)x.unipath << 32) | (uint32_t)((int64_t)x.start + (1ll << 31));
    val[i] = (uint32_t)i;
  }
}

__global__ void k_ulocs_gather(const ULoc* __restrict__ loc, const uint32_t* __restrict__ perm, uint64_t n,
                               ULoc* __restrict__ out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    out[i] = loc[perm[i]];
}

// unibases (one base per byte) -> 2-bit packed reads, one byte-aligned read
// per unipath: thread per output byte.
__global__ void k_pack_unibases(const uint8_t* __restrict__ ub, const uint64_t* __restrict__ ub_off, uint64_t U,
                                const uint64_t* __restrict__ byte_off, uint8_t* __restrict__ packed) {
  const uint64_t nby = byte_off[U];
  for (uint64_t y = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; y < nby; y += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t lo = 0, hi = U;  // unipath of byte y: largest u with byte_off[u] <= y
    while (hi - lo > 1) {
      const uint64_t mid = (lo + hi) >> 1;
      if (byte_off[mid] <= y)
        lo = mid;
      else
        hi = mid;
    }
    const uint64_t b0 = ub_off[lo] + (y - byte_off[lo]) * 4, e = ub_off[lo + 1];
    uint8_t x = 0;
    for (int t = 0; t < 4; ++t)
      if (b0 + t < e) x |= (uint8_t)((ub[b0 + t] & 3) << (2 * t));
    packed[y] = x;
  }
}

__global__ void k_ub_byte_lens(const uint64_t* __restrict__ ub_off, uint64_t U, uint32_t* __restrict__ nby) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < U; u += (uint64_t)gridDim.x * blockDim.x)
    nby[u] = (uint32_t)((ub_off[u + 1] - ub_off[u] + 3) / 4);
}

static int ulocs_run(apg_ctx* ctx, const apg_dreads* dr, uint32_t flags, const ULoc** d_out, uint64_t* n_out,
                     apg_uloc_stats* st) {
  const apg_ctx::GState& gs = ctx->gstate;
  APG_REQUIRE(gs.valid, "apg_unipath_locs: no unipath graph in this context (run apg_unipaths first)");
  APG_REQUIRE(!gs.sharded, "apg_unipath_locs: the last graph was built sharded (use apg_sharded_unipath_locs)");
  APG_REQUIRE((flags & ~(APG_ULOCS_RC | APG_ULOCS_SORTED)) == 0, "apg_unipath_locs: unknown flags");
  APG_REQUIRE(dr->n_reads < (1ull << 32), "apg_unipath_locs: more than 2^32 reads");
  APG_REQUIRE(dr->max_len < (1ull << 30), "apg_unipath_locs: read longer than 2^30 bases");
  const KeyP kp = make_keyp(gs.K);
  // directed node -> (unipath, rank) table, once per graph
  uint64_t* uloc = nullptr;
  const uint64_t D = 2 * gs.n_nodes;
  APG_TRY(workspace_t(ctx, "ul_uloc", std::max<uint64_t>(D, 1), &uloc));
  if (ctx->gstate.uloc != uloc) {
    kbegin(ctx, "ulocs_table", D * 20);
    if (D) k_uloc_table<<<grid_for(ctx, D), 256, 0, ctx->stream>>>(D, gs.head, gs.rank, gs.uoh, uloc);
    kend(ctx);
    APG_CHECK_HIP(hipGetLastError());
    ctx->gstate.uloc = uloc;
  }
  const GView g{NodeIdx{static_cast<const KRec*>(gs.nodes), gs.idx, gs.tmask}, uloc, gs.ulen, gs.urc};
  const ReadsV rv{dr->d_base_off, dr->d_byte_off, dr->d_packed, dr->n_reads};
  const uint64_t R = dr->n_reads;
  uint32_t* nloc = nullptr;
  uint64_t* loff = nullptr;
  unsigned long long* cnt = nullptr;
  APG_TRY(workspace_t(ctx, "ul_n", std::max<uint64_t>(R, 1), &nloc));
  APG_TRY(workspace_t(ctx, "ul_off", R + 1, &loff));
  APG_TRY(workspace_t(ctx, "ul_cnt", 3, &cnt));
  APG_CHECK_HIP(hipMemsetAsync(cnt, 0, 24, ctx->stream));
  const uint32_t grid = grid_for(ctx, R);
  // algorithmic bytes: packed reads + offsets + per-read count, and one
  // random 64-byte index line per K-mer lookup (added once counted)
  kbegin(ctx, "ulocs_count", dr->n_bytes + 20 * R);
  if (R) k_ulocs<false><<<grid, 256, 0, ctx->stream>>>(rv, g, kp, flags, nloc, nullptr, nullptr, cnt);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  APG_TRY(scan_u32_u64(ctx, nloc, R, loff, "ul"));
  uint64_t NL = 0;
  unsigned long long hc[3] = {0, 0, 0};
  APG_CHECK_HIP(hipMemcpyAsync(&NL, loff + R, 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(d2h_sync(ctx, hc, cnt, 24));
  const uint64_t nk = hc[2];
  kbytes_add(ctx, "ulocs_count", nk * 64);
  APG_REQUIRE(NL < (1ull << 32), "apg_unipath_locs: more than 2^32 locations");
  ULoc* loc = nullptr;
  APG_TRY(workspace_t(ctx, "ul_loc", std::max<uint64_t>(NL, 1), &loc));
  kbegin(ctx, "ulocs_write", dr->n_bytes + 16 * R + nk * 64 + NL * sizeof(ULoc));
  if (R) k_ulocs<true><<<grid, 256, 0, ctx->stream>>>(rv, g, kp, flags, nullptr, loff, loc, cnt);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  const ULoc* res = loc;
  if ((flags & APG_ULOCS_SORTED) && NL > 1) {
    uint64_t *k1 = nullptr, *k2 = nullptr;
    uint32_t *v1 = nullptr, *v2 = nullptr;
    ULoc* sorted = nullptr;
    APG_TRY(workspace_t(ctx, "ul_k1", NL, &k1));
    APG_TRY(workspace_t(ctx, "ul_k2", NL, &k2));
    APG_TRY(workspace_t(ctx, "ul_v1", NL, &v1));
    APG_TRY(workspace_t(ctx, "ul_v2", NL, &v2));
    APG_TRY(workspace_t(ctx, "ul_sorted", NL, &sorted));
    k_ulocs_keys<<<grid_for(ctx, NL), 256, 0, ctx->stream>>>(loc, NL, k1, v1);
    bool in2 = false;
    kbegin(ctx, "ulocs_sort", NL * 24);
    APG_TRY(sort_u64_u32(ctx, k1, v1, k2, v2, NL, &in2));
    kend(ctx);
    k_ulocs_gather<<<grid_for(ctx, NL), 256, 0, ctx->stream>>>(loc, in2 ? v2 : v1, NL, sorted);
    APG_CHECK_HIP(hipGetLastError());
    res = sorted;
  }
  APG_TRY(sync(ctx));
  *d_out = res;
  *n_out = NL;
  if (st) {
    st->n_reads = R;
    st->n_placed = hc[1];
    st->n_locs = NL;
    st->n_missing = hc[0];
  }
  return APG_OK;
}

}  // namespace apg

extern "C" {

int apg_unipath_locs_dev(apg_ctx* ctx, const apg_dreads* reads, uint32_t flags, const apg_aln_pair** d_locs,
                         uint64_t* n_locs, apg_uloc_stats* stats) {
  APG_REQUIRE(ctx && reads && d_locs && n_locs, "apg_unipath_locs_dev: NULL argument");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  APG_TRY(ws_release_graph_temps(ctx, (reads->n_bases + 16 * reads->n_reads) * 64));
  const ULoc* p = nullptr;
  APG_TRY(ulocs_run(ctx, reads, flags, &p, n_locs, stats));
  *d_locs = reinterpret_cast<const apg_aln_pair*>(p);
  return APG_OK;
}

int apg_unipath_locs(apg_ctx* ctx, const apg_reads* reads, uint32_t flags, apg_aln_pair** locs, uint64_t* n_locs,
                     apg_uloc_stats* stats) {
  APG_REQUIRE(ctx && reads && locs && n_locs, "apg_unipath_locs: NULL argument");
  *locs = nullptr;
  *n_locs = 0;
  apg_dreads* d = nullptr;
  APG_TRY(apg_reads_upload(ctx, reads, &d));
  const ULoc* p = nullptr;
  uint64_t n = 0;
  int rc = ulocs_run(ctx, d, flags, &p, &n, stats);
  if (rc == APG_OK) {
    auto* h = static_cast<apg_aln_pair*>(std::malloc(std::max<uint64_t>(n, 1) * sizeof(apg_aln_pair)));
    if (!h) {
      rc = APG_E_NOMEM;
    } else if (n && hipMemcpy(h, p, n * sizeof(apg_aln_pair), hipMemcpyDeviceToHost) != hipSuccess) {
      std::free(h);
      set_error("apg_unipath_locs: device-to-host copy failed");
      rc = APG_E_HIP;
    } else {
      *locs = h;
      *n_locs = n;
    }
  }
  apg_reads_free(d);
  return rc;
}

int apg_unibases_dev(apg_ctx* ctx, apg_dreads** out) {
  APG_REQUIRE(ctx && out, "apg_unibases_dev: NULL argument");
  *out = nullptr;
  const apg_ctx::GState& gs = ctx->gstate;
  APG_REQUIRE(gs.valid, "apg_unibases_dev: no unipath graph in this context (run apg_unipaths first)");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const uint64_t U = gs.n_unipaths;
  std::vector<uint64_t> hoff(U + 1, 0);
  if (U) APG_CHECK_HIP(hipMemcpyAsync(hoff.data(), gs.ub_off, (U + 1) * 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(sync(ctx));
  std::vector<uint64_t> hby(U + 1, 0);
  APG_TRY(apg_byte_offsets(hoff.data(), U, hby.data()));
  apg_reads hr;
  std::memset(&hr, 0, sizeof hr);
  hr.n_reads = 0;  // shape only: the data is produced on the device below
  apg_dreads* d = nullptr;
  APG_TRY(apg_reads_upload(ctx, &hr, &d));
  hipError_t e = hipSuccess;
  auto fail = [&](const char* what) {
    set_error(std::string("apg_unibases_dev: ") + what + ": " + hipGetErrorString(e));
    apg_reads_free(d);
    return APG_E_HIP;
  };
  (void)hipFree(d->d_base_off);
  (void)hipFree(d->d_byte_off);
  (void)hipFree(d->d_packed);
  d->d_base_off = d->d_byte_off = nullptr;
  d->d_packed = nullptr;
  d->n_reads = U;
  d->shape_hash = 0;
  d->n_bases = hoff[U];
  d->n_bytes = hby[U];
  for (uint64_t u = 0; u < U; ++u) d->max_len = std::max<uint64_t>(d->max_len, hoff[u + 1] - hoff[u]);
  if ((e = hipMalloc(&d->d_base_off, (U + 1) * 8)) != hipSuccess) return fail("alloc");
  if ((e = hipMalloc(&d->d_byte_off, (U + 1) * 8)) != hipSuccess) return fail("alloc");
  if ((e = hipMalloc(&d->d_packed, d->n_bytes + 64)) != hipSuccess) return fail("alloc");
  if ((e = hipMemsetAsync(d->d_packed, 0, d->n_bytes + 64, ctx->stream)) != hipSuccess) return fail("memset");
  if ((e = hipMemcpyAsync(d->d_base_off, gs.ub_off, (U + 1) * 8, hipMemcpyDeviceToDevice, ctx->stream)) != hipSuccess)
    return fail("copy");
  if ((e = hipMemcpyAsync(d->d_byte_off, hby.data(), (U + 1) * 8, hipMemcpyHostToDevice, ctx->stream)) != hipSuccess)
    return fail("copy");
  kbegin(ctx, "unibases_pack", d->n_bases + d->n_bytes);
  if (d->n_bytes)
    k_pack_unibases<<<grid_for(ctx, d->n_bytes), 256, 0, ctx->stream>>>(gs.ub, d->d_base_off, U, d->d_byte_off,
                                                                        d->d_packed);
  kend(ctx);
  if ((e = hipGetLastError()) != hipSuccess) return fail("pack");
  if ((e = hipStreamSynchronize(ctx->stream)) != hipSuccess) return fail("sync");
  *out = d;
  return APG_OK;
}

}  // extern "C"

extern "C" {

int apg_urec_count(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards, uint64_t* counts,
                   uint64_t* n_instances) {
  APG_REQUIRE(ctx && reads && counts, "apg_urec_count: NULL argument");
  APG_REQUIRE(K >= 1 && K <= 96, "apg_urec_count: K must be in [1, 96]");
  APG_REQUIRE(n_shards >= 1 && n_shards <= 8 && (n_shards & (n_shards - 1)) == 0,
              "apg_urec_count: n_shards must be a power of two <= 8");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const UskP p = make_uskp(K);
  std::vector<uint64_t> h, kd;
  uint32_t G = 0;
  APG_TRY(usk_plan(ctx, reads, p, n_shards, &h, &kd, &G));
  const uint32_t ndig = (uint32_t)n_shards << kUskDigitBits;
  uint64_t nk = 0;
  for (uint32_t d = 0; d < ndig; ++d) {
    counts[d] = h[d + 1] - h[d];
    nk += kd[d];
  }
  if (n_instances) *n_instances = nk;
  // send + receive + partition ping-pong of the 48-byte records; the
  // correction stage's tables are dead by now (released only under pressure)
  APG_TRY(ws_make_room(ctx, 4 * h[ndig] * sizeof(SK48), kRoomCorrection));  // descriptors stay for the scatter
  ctx->ws_dead |= kRoomCorrection;  // and a failed allocation of the graph stages may release them
  return APG_OK;
}

int apg_urec_scatter(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards, void* d_send) {
  APG_REQUIRE(ctx && reads, "apg_urec_scatter: NULL argument");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const auto& us = ctx->urstate;
  if (!us.valid || us.gen != reads->gen || us.K != K || us.P != n_shards) {
    std::vector<uint64_t> c((size_t)n_shards << kUskDigitBits);
    APG_TRY(apg_urec_count(ctx, reads, K, n_shards, c.data(), nullptr));
  }
  APG_REQUIRE(ctx->urstate.n == 0 || d_send, "apg_urec_scatter: d_send is NULL");
  APG_TRY(usk_scatter(ctx, reads, make_uskp(K), n_shards, ctx->urstate.G, static_cast<SK48*>(d_send)));
  return sync(ctx);
}

int apg_urec_nodes(apg_ctx* ctx, const void* d_recv, const uint64_t* recv_counts, int K, int n_shards,
                   uint64_t* n_nodes) {
  APG_REQUIRE(ctx && recv_counts && n_nodes, "apg_urec_nodes: NULL argument");
  APG_REQUIRE(K >= 1 && K <= 96, "apg_urec_nodes: K must be in [1, 96]");
  APG_REQUIRE(n_shards >= 1 && n_shards <= 8 && (n_shards & (n_shards - 1)) == 0,
              "apg_urec_nodes: n_shards must be a power of two <= 8");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  ctx->gstate.valid = false;  // "usk_nodes" is about to be rewritten
  ctx->urstate.n_nodes = 0;
  ctx->urstate.lsucc = nullptr;
  ctx->urstate.idx = nullptr;
  ctx->urstate.idx_T = 0;
  const size_t nc = (size_t)n_shards << kUskDigitBits;
  std::vector<uint64_t> rc(recv_counts, recv_counts + nc);
  uint64_t n = 0;
  for (auto c : rc) n += c;
  APG_REQUIRE(n == 0 || d_recv, "apg_urec_nodes: d_recv is NULL");
  const SK48* recs = static_cast<const SK48*>(d_recv);
  unsigned long long* sum = nullptr;
  APG_TRY(workspace_t(ctx, "usk_sum", 1, &sum));
  APG_CHECK_HIP(hipMemsetAsync(sum, 0, 8, ctx->stream));
  if (n) k_usk_sum<<<grid_for(ctx, n), 256, 0, ctx->stream>>>(recs, n, sum);
  unsigned long long nk = 0;
  APG_TRY(d2h_u64(ctx, sum, &nk, 1));
  KRec* nodes = nullptr;
  uint64_t N = 0;
  // the buckets also resolve the links inside themselves and build the node
  // index as they append nodes (the single-GPU build's two savings): the
  // sharded graph (ushard_graph.inc) then looks up only the successors in
  // other buckets, locally or by a query to their owner
  uint2* ls = nullptr;
  PreIdx pidx;
  APG_TRY(usk_stage(ctx, recs, rc, nk, make_keyp(K), n_shards, &nodes, &N, &ls, &pidx));
  ctx->urstate.n_nodes = N;
  ctx->urstate.lsucc = ls;
  ctx->urstate.idx = pidx.idx;
  ctx->urstate.idx_T = pidx.idx ? pidx.T : 0;
  *n_nodes = N;
  return APG_OK;
}

int apg_urec_export(apg_ctx* ctx, void* d_out) {
  APG_REQUIRE(ctx, "apg_urec_export: NULL ctx");
  const uint64_t N = ctx->urstate.n_nodes;
  if (N == 0) return APG_OK;
  APG_REQUIRE(d_out, "apg_urec_export: d_out is NULL");
  KRec* nodes = nullptr;
  APG_TRY(workspace_t(ctx, "usk_nodes", N, &nodes));
  APG_CHECK_HIP(hipMemcpyAsync(d_out, nodes, N * sizeof(KRec), hipMemcpyDeviceToDevice, ctx->stream));
  return sync(ctx);
}

}  // extern "C"

// ---------------------------------------------------------------------------
// UnipathCoverage (apg_unipath_coverage, spec in include/apg.h; CPU
// restatement oracle/ucov_oracle.c)
// ---------------------------------------------------------------------------
namespace apg {

// placements per unipath: each wave finds runs of equal unipath ids among its
// 64 consecutive placements (sorted input: long runs) and adds each run with
// one atomic
__global__ void __launch_bounds__(256) k_ucov_count(const ULoc* __restrict__ loc, uint64_t n, uint64_t U,
                                                    unsigned long long* __restrict__ cnt,
                                                    unsigned long long* __restrict__ bad) {
  const int lane = lane_id();
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x; i0 < n; i0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = i0 + threadIdx.x;
    const bool v = i < n;
    const uint32_t u = v ? loc[i].unipath : 0xffffffffu;
    const uint32_t pu = (uint32_t)__shfl_up((int)u, 1, 64);
    const bool head = v && (lane == 0 || pu != u);
    const uint64_t heads = __ballot(head);
    const uint32_t nvalid = (uint32_t)__popcll(__ballot(v));  // valid lanes are a prefix
    if (head) {
      const uint64_t above = lane == 63 ? 0 : heads & ~((2ull << lane) - 1);
      const uint32_t end = min(above ? (uint32_t)(__ffsll((long long)above) - 1) : 64u, nvalid);
      const unsigned long long len = end - (uint32_t)lane;
      if (u < U)
        atomicAdd(&cnt[u], len);
      else
        atomicAdd(bad, len);
    }
  }
}

__global__ void k_ucov_cov(uint64_t U, const unsigned long long* __restrict__ cnt, const uint64_t* __restrict__ ulen,
                           double* __restrict__ cov) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < U; u += (uint64_t)gridDim.x * blockDim.x)
    cov[u] = ulen[u] ? (double)cnt[u] / (double)ulen[u] : 0.0;
}

__global__ void k_ucov_cn(uint64_t U, const double* __restrict__ cov, double c0, uint32_t* __restrict__ cn) {
  for (uint64_t u = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; u < U; u += (uint64_t)gridDim.x * blockDim.x)
    cn[u] = c0 > 0.0 ? (uint32_t)floor(cov[u] / c0 + 0.5) : 0u;
}

}  // namespace apg

extern "C" {

void apg_ucov_defaults(apg_ucov_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->min_len = 500;
}

int apg_unipath_coverage_dev(apg_ctx* ctx, const apg_aln_pair* d_locs, uint64_t n_locs, const apg_ucov_params* pp,
                             uint64_t* counts, double* cov, uint32_t* copy_number, apg_ucov_stats* stats) {
  using namespace apg;
  APG_REQUIRE(ctx, "apg_unipath_coverage: NULL ctx");
  APG_REQUIRE(n_locs == 0 || d_locs, "apg_unipath_coverage: d_locs is NULL");
  const auto& g = ctx->gstate;
  APG_REQUIRE(g.valid, "apg_unipath_coverage: no unipath graph on this context (run apg_unipaths first; the "
                       "sharded compaction keeps no whole graph)");
  apg_ucov_params p;
  if (pp)
    p = *pp;
  else
    apg_ucov_defaults(&p);
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const uint64_t U = g.n_unipaths;
  unsigned long long* cnt = nullptr;
  double* dcov = nullptr;
  uint32_t* dcn = nullptr;
  APG_TRY(workspace_t(ctx, "uc_cnt", U + 1, &cnt));  // [U] = rejected placements
  APG_TRY(workspace_t(ctx, "uc_cov", std::max<uint64_t>(U, 1), &dcov));
  APG_TRY(workspace_t(ctx, "uc_cn", std::max<uint64_t>(U, 1), &dcn));
  APG_CHECK_HIP(hipMemsetAsync(cnt, 0, (U + 1) * 8, ctx->stream));
  kbegin(ctx, "ucov_count", n_locs * 16 + U * 8);
  if (n_locs)
    k_ucov_count<<<grid_for(ctx, n_locs), 256, 0, ctx->stream>>>(reinterpret_cast<const ULoc*>(d_locs), n_locs, U, cnt,
                                                                  cnt + U);
  kend(ctx);
  if (U) k_ucov_cov<<<grid_for(ctx, U), 256, 0, ctx->stream>>>(U, cnt, g.ulen, dcov);
  APG_CHECK_HIP(hipGetLastError());
  std::vector<double> hc(U);
  std::vector<uint64_t> hl(U);
  unsigned long long nbad = 0;
  if (U) {
    APG_CHECK_HIP(hipMemcpyAsync(hc.data(), dcov, U * 8, hipMemcpyDeviceToHost, ctx->stream));
    APG_CHECK_HIP(hipMemcpyAsync(hl.data(), g.ulen, U * 8, hipMemcpyDeviceToHost, ctx->stream));
  }
  APG_TRY(d2h_sync(ctx, &nbad, cnt + U, 8));
  APG_REQUIRE(nbad == 0, "apg_unipath_coverage: placements on unipaths the graph does not have");
  // length-weighted median of cov over the long unipaths
  std::vector<std::pair<double, uint64_t>> lv;
  uint64_t W = 0;
  for (uint64_t u = 0; u < U; ++u)
    if (hl[u] >= p.min_len) {
      lv.emplace_back(hc[u], hl[u]);
      W += hl[u];
    }
  std::sort(lv.begin(), lv.end());
  double c0 = 0.0;
  uint64_t acc = 0;
  for (const auto& x : lv) {
    acc += x.second;
    if (2 * acc >= W) {
      c0 = x.first;
      break;
    }
  }
  if (U) k_ucov_cn<<<grid_for(ctx, U), 256, 0, ctx->stream>>>(U, dcov, c0, dcn);
  APG_CHECK_HIP(hipGetLastError());
  if (counts && U) APG_CHECK_HIP(hipMemcpyAsync(counts, cnt, U * 8, hipMemcpyDeviceToHost, ctx->stream));
  if (cov && U) std::memcpy(cov, hc.data(), U * 8);
  if (copy_number && U) APG_CHECK_HIP(hipMemcpyAsync(copy_number, dcn, U * 4, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(sync(ctx));
  if (stats) {
    stats->c0 = c0;
    stats->n_long = lv.size();
    stats->n_locs = n_locs;
    stats->n_bad = nbad;
  }
  return APG_OK;
}

int apg_unipath_coverage(apg_ctx* ctx, const apg_aln_pair* locs, uint64_t n_locs, const apg_ucov_params* p,
                         uint64_t* counts, double* cov, uint32_t* copy_number, apg_ucov_stats* stats) {
  using namespace apg;
  APG_REQUIRE(ctx && (n_locs == 0 || locs), "apg_unipath_coverage: NULL argument");
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  apg_aln_pair* d = nullptr;
  APG_TRY(workspace_t(ctx, "uc_locs", std::max<uint64_t>(n_locs, 1), &d));
  if (n_locs) APG_CHECK_HIP(hipMemcpyAsync(d, locs, n_locs * sizeof(apg_aln_pair), hipMemcpyHostToDevice, ctx->stream));
  return apg_unipath_coverage_dev(ctx, d, n_locs, p, counts, cov, copy_number, stats);
}

}  // extern "C"

#include "ushard_graph.inc"
