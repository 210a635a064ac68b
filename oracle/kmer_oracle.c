/*
 * oracle/kmer_oracle.c — CPU restatement of the k-mer spectrum path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline) — never as the product path.
 *
 * PARITY UNPINNED: /root/reference is empty, so this file
 * restates the recalled ALLPATHS-LG algorithm as pinned down by SURVEY.md §A
 * (decisions [D]); it is validated by first-principles known-answer tests
 *  in tests/test_oracle.py and by committed golden fixtures in
 * tests/golden/ produced from it.  Recalled reference locations are grep
 * targets, not line citations:
 *   - k-mer extraction/canonicalisation: [R:M] src/kmers/naif_kmer/Kmers.h,
 *     NaifKmerizer.h (rolling 2-bit k-mer, canonical = min(fw, rc)).
 *   - counting: [R:M] NaifKmerizer block sort + KernelKmerStorer summarize
 *     (sort, merge equal k-mers into (k-mer, frequency)).
 *   - spectrum: [R:M] src/kmers/KmerSpectra.h KmerSpectrum (h[m]).
 * Deliberately simple: one thread, generate -> LSD radix sort -> run-length.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

/* ---- SURVEY §A.3 table-order hash: bijection on w = 2K bits ------------- */
/* splitmix64's finaliser with shifts scaled to w bits and multipliers masked */
/* to w bits (odd => invertible mod 2^w).  At K = 32 it IS splitmix64.       */
static uint64_t wmask(int w) { return w >= 64 ? ~0ull : ((1ull << w) - 1); }
static int sh(int w, int num) { int s = (w * num) / 64; return s < 1 ? 1 : s; }

uint64_t ork_hash(int K, uint64_t x) {
  const int w = 2 * K;
  const uint64_t m = wmask(w);
  const uint64_t c1 = (0xbf58476d1ce4e5b9ull & m) | 1, c2 = (0x94d049bb133111ebull & m) | 1;
  x &= m;
  x ^= x >> sh(w, 30);
  x = (x * c1) & m;
  x ^= x >> sh(w, 27);
  x = (x * c2) & m;
  x ^= x >> sh(w, 31);
  return x;
}

static uint64_t inv_xorshift(uint64_t y, int s, int w) {
  uint64_t x = y;
  for (int i = 0; i * s < w; ++i) x = y ^ (x >> s);
  return x & wmask(w);
}
static uint64_t inv_odd(uint64_t c) {
  uint64_t v = c; /* Newton: 3 -> 6 -> 12 -> 24 -> 48 -> 96 correct bits */
  for (int i = 0; i < 5; ++i) v *= 2 - c * v;
  return v;
}
uint64_t ork_unhash(int K, uint64_t h) {
  const int w = 2 * K;
  const uint64_t m = wmask(w);
  const uint64_t c1 = (0xbf58476d1ce4e5b9ull & m) | 1, c2 = (0x94d049bb133111ebull & m) | 1;
  uint64_t x = h & m;
  x = inv_xorshift(x, sh(w, 31), w);
  x = (x * inv_odd(c2)) & m;
  x = inv_xorshift(x, sh(w, 27), w);
  x = (x * inv_odd(c1)) & m;
  x = inv_xorshift(x, sh(w, 30), w);
  return x;
}

/* ---- reads ---------------------------------------------------------------- */
static inline int base_at(const uint8_t* packed, uint64_t byte0, uint64_t i) {
  return (packed[byte0 + (i >> 2)] >> (2 * (i & 3))) & 3;
}

uint64_t ork_count_instances(uint64_t n_reads, const uint64_t* base_off, int K) {
  uint64_t n = 0;
  for (uint64_t r = 0; r < n_reads; ++r) {
    uint64_t len = base_off[r + 1] - base_off[r];
    if (len >= (uint64_t)K) n += len - K + 1;
  }
  return n;
}

/* Canonical k-mers of every read, in read order, written as hashes.
 * fw = sum b[i+j] 4^(K-1-j); rc likewise on the reverse complement (§A.3). */
uint64_t ork_extract_hashes(uint64_t n_reads, const uint64_t* base_off,
                            const uint64_t* byte_off, const uint8_t* packed, int K,
                            uint64_t* out) {
  const uint64_t m = wmask(2 * K);
  uint64_t n = 0;
  for (uint64_t r = 0; r < n_reads; ++r) {
    const uint64_t len = base_off[r + 1] - base_off[r];
    uint64_t fw = 0, rc = 0;
    for (uint64_t i = 0; i < len; ++i) {
      const uint64_t b = (uint64_t)base_at(packed, byte_off[r], i);
      fw = ((fw << 2) | b) & m;
      rc = (rc >> 2) | ((3 - b) << (2 * K - 2));
      if (i + 1 >= (uint64_t)K) {
        const uint64_t c = fw < rc ? fw : rc;
        out[n++] = ork_hash(K, c);
      }
    }
  }
  return n;
}

/* LSD radix sort of 64-bit values on their low `bits` bits, 8 bits a pass. */
static void radix_sort_u64(uint64_t* a, uint64_t n, int bits) {
  uint64_t* tmp = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
  uint64_t* src = a;
  uint64_t* dst = tmp;
  for (int shift = 0; shift < bits; shift += 8) {
    uint64_t cnt[257];
    memset(cnt, 0, sizeof cnt);
    for (uint64_t i = 0; i < n; ++i) cnt[((src[i] >> shift) & 255) + 1]++;
    for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
    for (uint64_t i = 0; i < n; ++i) dst[cnt[(src[i] >> shift) & 255]++] = src[i];
    uint64_t* t = src; src = dst; dst = t;
  }
  if (src != a) memcpy(a, src, n * sizeof(uint64_t));
  free(tmp);
}

/* (hash, count) table in ascending hash order.  Returns #distinct, or
 * UINT64_MAX on allocation failure.  Caller frees *hashes / *counts. */
uint64_t ork_kmer_count(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off,
                        const uint8_t* packed, int K, uint64_t** hashes, uint32_t** counts) {
  const uint64_t n = ork_count_instances(n_reads, base_off, K);
  uint64_t* h = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
  if (!h) return UINT64_MAX;
  ork_extract_hashes(n_reads, base_off, byte_off, packed, K, h);
  radix_sort_u64(h, n, 2 * K);
  uint32_t* c = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
  if (!c) { free(h); return UINT64_MAX; }
  uint64_t d = 0;
  for (uint64_t i = 0; i < n;) {
    uint64_t j = i + 1;
    while (j < n && h[j] == h[i]) ++j;
    h[d] = h[i];
    c[d] = (uint32_t)(j - i);
    ++d;
    i = j;
  }
  *hashes = h;
  *counts = c;
  return d;
}

/* KmerSpectrum: hist[m] += 1 per distinct k-mer of count m; last bin is >=. */
void ork_spectrum(const uint32_t* counts, uint64_t nd, uint64_t* hist, uint64_t hist_len) {
  memset(hist, 0, hist_len * sizeof(uint64_t));
  for (uint64_t i = 0; i < nd; ++i) {
    uint64_t m = counts[i];
    if (m >= hist_len - 1) m = hist_len - 1;
    hist[m]++;
  }
}

void ork_free(void* p) { free(p); }
