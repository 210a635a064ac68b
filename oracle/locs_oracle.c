/* locs_oracle.c — CPU restatement of UnipathLocs, the placement of reads on
 * unipaths (TEST INFRASTRUCTURE ONLY: the checker of allpathslg_amd's
 * apg_unipath_locs; never linked into the product).
 *
 * Parity unpinned: /root/reference is empty.  Recalled
 * reference [R:M]: BuildUnipathLocs / ReadLocationLG, src/paths/UnipathLocs*
 * (grep target only, no lines to cite).  The operational spec is the one
 * pinned in include/apg.h (apg_unipath_locs):
 *   - the graph's directed K-mers are indexed from the unibases: the K-mer at
 *     rank k of unipath u is unibases[u][k .. k+K) (u and rc(u) are both
 *     stored, so every directed K-mer of the graph has exactly one (u, k));
 *   - K-mer j of read r found at (u, k) places the read at s = k - j; a
 *     location (r, u, s, 0) is emitted whenever (u, s) differs from the
 *     read's last emitted pair; absent K-mers are skipped and counted;
 *   - ORL_RC: each location is followed by (r, rc(u), len(u)+K-1-(s+L), 1);
 *   - ORL_SORTED: stable sort by (u, s).
 * Written independently of the HIP kernels (plain hash table over the
 * unibase K-mers, K-mers recomputed base by base), so agreement means both
 * follow the spec. */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

#define ORL_RC 1u
#define ORL_SORTED 2u

typedef struct {
  uint64_t w[3]; /* K-mer, 2 bits per base, base 0 in the highest used bits */
} kmer3;

static void kmer_of(const uint8_t* b, int K, kmer3* x) {
  memset(x, 0, sizeof *x);
  for (int i = 0; i < K; ++i) {
    /* shift left by 2 over three limbs (w[0] most significant) */
    x->w[0] = (x->w[0] << 2) | (x->w[1] >> 62);
    x->w[1] = (x->w[1] << 2) | (x->w[2] >> 62);
    x->w[2] = (x->w[2] << 2) | (uint64_t)(b[i] & 3);
  }
}

static uint64_t kmer_hash(const kmer3* x) {
  uint64_t h = 0x9e3779b97f4a7c15ull;
  for (int i = 0; i < 3; ++i) {
    h ^= x->w[i] + 0x9e3779b97f4a7c15ull + (h << 6) + (h >> 2);
    h *= 0xbf58476d1ce4e5b9ull;
    h ^= h >> 31;
  }
  return h;
}

typedef struct {
  kmer3 key;
  uint32_t u, k;
  int used;
} slot;

typedef struct {
  uint32_t r, u;
  int32_t s;
  uint32_t f;
  uint64_t ord; /* emission index: the stable tie-break */
} loc;

static int loc_cmp(const void* a, const void* b) {
  const loc* x = (const loc*)a;
  const loc* y = (const loc*)b;
  if (x->u != y->u) return x->u < y->u ? -1 : 1;
  if (x->s != y->s) return x->s < y->s ? -1 : 1;
  return x->ord < y->ord ? -1 : x->ord > y->ord;
}

/* unibases: one base per byte, unipath u = [ub_off[u], ub_off[u+1]).
 * Reads: 2-bit packed, LSB-first, byte-aligned per read.  out: 4 u32 per
 * location (read, unipath, start as int32, flags), malloc'd; release with
 * ork_free.  stats: [0] reads placed, [1] K-mers missing. */
int orl_locs(uint64_t U, const uint64_t* ulen, const uint64_t* urc, const uint64_t* ub_off, const uint8_t* ub, int K,
             uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed,
             uint32_t flags, uint32_t** out, uint64_t* n_out, uint64_t* stats) {
  *out = NULL;
  *n_out = 0;
  stats[0] = stats[1] = 0;
  if (K < 1 || K > 96) return -1;
  uint64_t nk = 0;
  for (uint64_t u = 0; u < U; ++u) nk += ulen[u];
  uint64_t T = 1024;
  while (T < 2 * nk + 2) T <<= 1;
  slot* tab = (slot*)calloc(T, sizeof(slot));
  if (!tab) return -2;
  for (uint64_t u = 0; u < U; ++u)
    for (uint64_t k = 0; k < ulen[u]; ++k) {
      kmer3 x;
      kmer_of(ub + ub_off[u] + k, K, &x);
      uint64_t s = kmer_hash(&x) & (T - 1);
      while (tab[s].used && memcmp(&tab[s].key, &x, sizeof x)) s = (s + 1) & (T - 1);
      if (tab[s].used) { /* a directed K-mer in two places: not a unipath graph */
        free(tab);
        return -3;
      }
      tab[s].key = x;
      tab[s].u = (uint32_t)u;
      tab[s].k = (uint32_t)k;
      tab[s].used = 1;
    }
  uint64_t cap = 1024, n = 0;
  loc* L = (loc*)malloc(cap * sizeof(loc));
  uint8_t* rb = NULL;
  uint64_t rcap = 0;
  if (!L) {
    free(tab);
    return -2;
  }
  for (uint64_t r = 0; r < n_reads; ++r) {
    const uint64_t len = base_off[r + 1] - base_off[r];
    if (len > rcap) {
      rcap = len;
      free(rb);
      rb = (uint8_t*)malloc(rcap);
      if (!rb) {
        free(tab);
        free(L);
        return -2;
      }
    }
    const uint8_t* p = packed + byte_off[r];
    for (uint64_t i = 0; i < len; ++i) rb[i] = (p[i >> 2] >> (2 * (i & 3))) & 3;
    int have = 0, placed = 0;
    uint32_t pu = 0;
    int64_t ps = 0;
    for (uint64_t j = 0; j + (uint64_t)K <= len; ++j) {
      kmer3 x;
      kmer_of(rb + j, K, &x);
      uint64_t s = kmer_hash(&x) & (T - 1);
      while (tab[s].used && memcmp(&tab[s].key, &x, sizeof x)) s = (s + 1) & (T - 1);
      if (!tab[s].used) {
        ++stats[1];
        continue;
      }
      const uint32_t u = tab[s].u;
      const int64_t st = (int64_t)tab[s].k - (int64_t)j;
      if (have && u == pu && st == ps) continue;
      have = 1;
      pu = u;
      ps = st;
      placed = 1;
      if (n + 2 > cap) {
        cap *= 2;
        loc* L2 = (loc*)realloc(L, cap * sizeof(loc));
        if (!L2) {
          free(tab);
          free(L);
          free(rb);
          return -2;
        }
        L = L2;
      }
      L[n] = (loc){(uint32_t)r, u, (int32_t)st, 0u, n};
      ++n;
      if (flags & ORL_RC) {
        const int64_t ulb = (int64_t)ulen[u] + K - 1;
        L[n] = (loc){(uint32_t)r, (uint32_t)urc[u], (int32_t)(ulb - (st + (int64_t)len)), 1u, n};
        ++n;
      }
    }
    stats[0] += placed;
  }
  if (flags & ORL_SORTED) qsort(L, n, sizeof(loc), loc_cmp);
  uint32_t* o = (uint32_t*)malloc((n ? n : 1) * 4 * sizeof(uint32_t));
  if (!o) {
    free(tab);
    free(L);
    free(rb);
    return -2;
  }
  for (uint64_t i = 0; i < n; ++i) {
    o[4 * i] = L[i].r;
    o[4 * i + 1] = L[i].u;
    o[4 * i + 2] = (uint32_t)L[i].s;
    o[4 * i + 3] = L[i].f;
  }
  free(tab);
  free(L);
  free(rb);
  *out = o;
  *n_out = n;
  return 0;
}
