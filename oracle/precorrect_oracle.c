/*
 * oracle/precorrect_oracle.c — CPU restatement of PreCorrect / FindErrors
 * (SURVEY.md §A.4 as pinned in include/apg.h).  TEST INFRASTRUCTURE ONLY.
 *
 * PARITY UNPINNED: the reference snapshot is empty; the recalled
 * modules are [R:M-L] src/PreCorrect.cc and [R:M] src/FindErrors.cc /
 * naif_kmer/KernelErrorFinder (grep targets, no line citations possible).
 * The rule restated here: solid = canonical K-mer count >= min_solid; per
 * read, left to right on the current read, a base with Q < max_q whose every
 * covering K-mer is weak is suspect; the unique alternative (A<C<G<T) making
 * every covering K-mer solid replaces it, Q := min(Q of neighbours).
 * Solid lookup: the sorted (hash, count) table from ork_kmer_count, binary
 * searched — deliberately a different structure from the GPU hash table.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "solidset.h"

static int get_base(const uint8_t* rd, uint32_t i) { return (rd[i >> 2] >> (2 * (i & 3))) & 3; }

static uint64_t kmer_hash_at(const uint8_t* rd, uint32_t j, int K, uint32_t p, int alt) {
  const uint64_t m = K >= 32 ? ~0ull : ((1ull << (2 * K)) - 1);
  uint64_t fw = 0, rc = 0;
  for (int t = 0; t < K; ++t) {
    const uint32_t i = j + (uint32_t)t;
    const uint64_t b = (i == p) ? (uint64_t)alt : (uint64_t)get_base(rd, i);
    fw = ((fw << 2) | b) & m;
    rc = (rc >> 2) | ((3 - b) << (2 * K - 2));
  }
  return ork_hash(K, fw < rc ? fw : rc);
}

/* binary search of h in the ascending solid-hash array */
static int is_solid(const uint64_t* solid, uint64_t ns, uint64_t h) {
  uint64_t lo = 0, hi = ns;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (solid[mid] < h)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < ns && solid[lo] == h;
}

static void correct_read(const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed, uint8_t* quals, int K,
                         uint32_t maxq, const uint64_t* h, uint64_t ns, uint64_t r, uint64_t* stats);

/* One correction pass against the ascending solid-hash array h[0..ns). */
static void correct(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed,
                    uint8_t* quals, int K, uint32_t maxq, const uint64_t* h, uint64_t ns, uint64_t* stats) {
  /* reads are independent (counts are not updated within a pass): one
   * thread per read, counters reduced */
  uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
#pragma omp parallel for schedule(dynamic, 1024) reduction(+ : s0, s1, s2, s3)
  for (uint64_t r = 0; r < n_reads; ++r) {
    uint64_t st[4] = {0, 0, 0, 0};
    correct_read(base_off, byte_off, packed, quals, K, maxq, h, ns, r, st);
    s0 += st[0], s1 += st[1], s2 += st[2], s3 += st[3];
  }
  stats[0] += s0, stats[1] += s1, stats[2] += s2, stats[3] += s3;
}

static void correct_read(const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed, uint8_t* quals, int K,
                         uint32_t maxq, const uint64_t* h, uint64_t ns, uint64_t r, uint64_t* stats) {
  {
    const uint32_t L = (uint32_t)(base_off[r + 1] - base_off[r]);
    if (L < (uint32_t)K) return;
    uint8_t* rd = packed + byte_off[r];
    uint8_t* q = quals + base_off[r];
    for (uint32_t p = 0; p < L; ++p) {
      if (q[p] >= maxq) continue;
      const uint32_t jlo = p + 1 >= (uint32_t)K ? p + 1 - (uint32_t)K : 0;
      const uint32_t jhi = p < L - (uint32_t)K ? p : L - (uint32_t)K;
      int weak = 1;
      for (uint32_t j = jlo; j <= jhi && weak; ++j)
        if (is_solid(h, ns, kmer_hash_at(rd, j, K, 0xffffffffu, 0))) weak = 0;
      if (!weak) continue;
      stats[0]++;
      const int orig = get_base(rd, p);
      int ncand = 0, cand = 0;
      for (int alt = 0; alt < 4; ++alt) {
        if (alt == orig) continue;
        int ok = 1;
        for (uint32_t j = jlo; j <= jhi && ok; ++j)
          if (!is_solid(h, ns, kmer_hash_at(rd, j, K, p, alt))) ok = 0;
        if (ok) {
          ++ncand;
          cand = alt;
        }
      }
      if (ncand == 1) {
        const int sh = 2 * (int)(p & 3);
        rd[p >> 2] = (uint8_t)((rd[p >> 2] & ~(3u << sh)) | ((unsigned)cand << sh));
        uint32_t nq = 255;
        if (p > 0 && q[p - 1] < nq) nq = q[p - 1];
        if (p + 1 < L && q[p + 1] < nq) nq = q[p + 1];
        q[p] = (uint8_t)nq;
        stats[1]++;
      } else if (ncand > 1) {
        stats[2]++;
      } else {
        stats[3]++;
      }
    }
  }
}

static int pass(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed,
                uint8_t* quals, int K, uint32_t min_solid, uint32_t maxq, uint64_t* stats) {
  uint64_t *h = NULL;
  uint32_t* c = NULL;
  const uint64_t nd = ork_kmer_count(n_reads, base_off, byte_off, packed, K, &h, &c);
  if (nd == UINT64_MAX) return -1;
  uint64_t ns = 0;
  for (uint64_t i = 0; i < nd; ++i)
    if (c[i] >= min_solid) h[ns++] = h[i]; /* stays ascending */
  free(c);
  stats[4] = ns;
  correct(n_reads, base_off, byte_off, packed, quals, K, maxq, h, ns, stats);
  free(h);
  return 0;
}

static int cmp_u64(const void* a, const void* b) {
  const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}

/* One pass against a caller-given solid hash set (any order; sorted here). */
int ork_precorrect_solid(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed,
                         uint8_t* quals, int K, uint32_t maxq, const uint64_t* solid, uint64_t ns, uint64_t* stats) {
  memset(stats, 0, 5 * sizeof(uint64_t));
  uint64_t* h = (uint64_t*)malloc((ns ? ns : 1) * sizeof(uint64_t));
  if (!h) return -1;
  if (ns) memcpy(h, solid, ns * sizeof(uint64_t));
  qsort(h, ns, sizeof(uint64_t), cmp_u64);
  stats[4] = ns;
  correct(n_reads, base_off, byte_off, packed, quals, K, maxq, h, ns, stats);
  free(h);
  return 0;
}

/* In place.  stats[0..4] = suspect, corrected, ambiguous, uncorrectable,
 * solid-in-last-cycle (summed over cycles except [4]). */
int ork_precorrect(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed,
                   uint8_t* quals, int K, uint32_t min_solid, uint32_t maxq, uint32_t n_cycles, uint64_t* stats) {
  memset(stats, 0, 5 * sizeof(uint64_t));
  for (uint32_t c = 0; c < n_cycles; ++c)
    if (pass(n_reads, base_off, byte_off, packed, quals, K, min_solid, maxq, stats)) return -1;
  return 0;
}

/* ------------------------------------------------------------------------- */
/* bench.py's CPU baseline (a fair baseline): the same rule as
 * correct_read, with every K-mer of the read kept as rolling (fw, rc) keys —
 * a substitution at p changes K-mer j's keys by one 2-bit XOR each, at
 * shift 2(K-1-(p-j)) in fw and 2(p-j) in rc — and solid lookups through a
 * hash table of the solid set (solidset.h).  Outputs equal ork_precorrect's
 * (tests/test_cpu_baseline.py). */
static void correct_read_fast(const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed, uint8_t* quals,
                              int K, uint32_t maxq, const OSolid* set, uint64_t r, uint64_t* fw, uint64_t* rc,
                              uint8_t* sol, uint64_t* stats) {
  const uint32_t L = (uint32_t)(base_off[r + 1] - base_off[r]);
  if (L < (uint32_t)K) return;
  uint8_t* rd = packed + byte_off[r];
  uint8_t* q = quals + base_off[r];
  const uint32_t nk = L - (uint32_t)K + 1;
  const uint64_t m = K >= 32 ? ~0ull : ((1ull << (2 * K)) - 1);
  uint64_t f = 0, c = 0;
  for (uint32_t i = 0; i < L; ++i) {
    const uint64_t b = (uint64_t)get_base(rd, i);
    f = ((f << 2) | b) & m;
    c = (c >> 2) | ((3 - b) << (2 * K - 2));
    if (i + 1 >= (uint32_t)K) {
      const uint32_t j = i + 1 - (uint32_t)K;
      fw[j] = f;
      rc[j] = c;
      sol[j] = (uint8_t)osolid_has(set, ork_hash(K, f < c ? f : c));
    }
  }
  for (uint32_t p = 0; p < L; ++p) {
    if (q[p] >= maxq) continue;
    const uint32_t jlo = p + 1 >= (uint32_t)K ? p + 1 - (uint32_t)K : 0;
    const uint32_t jhi = p < nk - 1 ? p : nk - 1;
    int weak = 1;
    for (uint32_t j = jlo; j <= jhi && weak; ++j)
      if (sol[j]) weak = 0;
    if (!weak) continue;
    stats[0]++;
    const int orig = get_base(rd, p);
    int ncand = 0, cand = 0;
    for (int alt = 0; alt < 4; ++alt) {
      if (alt == orig) continue;
      const uint64_t x = (uint64_t)(orig ^ alt);
      int ok = 1;
      for (uint32_t j = jlo; j <= jhi && ok; ++j) {
        const uint64_t f2 = fw[j] ^ (x << (2 * (K - 1 - (int)(p - j)))), c2 = rc[j] ^ (x << (2 * (p - j)));
        if (!osolid_has(set, ork_hash(K, f2 < c2 ? f2 : c2))) ok = 0;
      }
      if (ok) {
        ++ncand;
        cand = alt;
      }
    }
    if (ncand == 1) {
      const int sh = 2 * (int)(p & 3);
      rd[p >> 2] = (uint8_t)((rd[p >> 2] & ~(3u << sh)) | ((unsigned)cand << sh));
      uint32_t nq = 255;
      if (p > 0 && q[p - 1] < nq) nq = q[p - 1];
      if (p + 1 < L && q[p + 1] < nq) nq = q[p + 1];
      q[p] = (uint8_t)nq;
      const uint64_t x = (uint64_t)(orig ^ cand);
      for (uint32_t j = jlo; j <= jhi; ++j) {  /* the covering K-mers now carry the new base */
        fw[j] ^= x << (2 * (K - 1 - (int)(p - j)));
        rc[j] ^= x << (2 * (p - j));
        sol[j] = (uint8_t)osolid_has(set, ork_hash(K, fw[j] < rc[j] ? fw[j] : rc[j]));
      }
      stats[1]++;
    } else if (ncand > 1) {
      stats[2]++;
    } else {
      stats[3]++;
    }
  }
}

static int correct_fast(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed,
                        uint8_t* quals, int K, uint32_t maxq, const OSolid* set, uint64_t* stats) {
  uint32_t maxL = 0;
  for (uint64_t r = 0; r < n_reads; ++r)
    if (base_off[r + 1] - base_off[r] > maxL) maxL = (uint32_t)(base_off[r + 1] - base_off[r]);
  uint64_t s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  int fail = 0;
#pragma omp parallel reduction(+ : s0, s1, s2, s3)
  {
    uint64_t* fw = (uint64_t*)malloc((maxL + 1) * sizeof(uint64_t));
    uint64_t* rc = (uint64_t*)malloc((maxL + 1) * sizeof(uint64_t));
    uint8_t* sol = (uint8_t*)malloc(maxL + 1);
    if (!fw || !rc || !sol) {
#pragma omp atomic write
      fail = 1;
    }
#pragma omp for schedule(dynamic, 1024)
    for (uint64_t r = 0; r < n_reads; ++r) {
      if (!fw || !rc || !sol) continue;
      uint64_t st[4] = {0, 0, 0, 0};
      correct_read_fast(base_off, byte_off, packed, quals, K, maxq, set, r, fw, rc, sol, st);
      s0 += st[0], s1 += st[1], s2 += st[2], s3 += st[3];
    }
    free(fw), free(rc), free(sol);
  }
  if (fail) return -1;
  stats[0] += s0, stats[1] += s1, stats[2] += s2, stats[3] += s3;
  return 0;
}

/* one pass against a caller-given solid set (ork_precorrect_solid's fast form) */
int ork_precorrect_solid_fast(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed,
                              uint8_t* quals, int K, uint32_t maxq, const uint64_t* solid, uint64_t ns,
                              uint64_t* stats) {
  memset(stats, 0, 5 * sizeof(uint64_t));
  if (K < 2 || K > 29) return -1;
  OSolid set;
  if (osolid_build_table(&set, solid, ns)) return -1;
  stats[4] = ns;
  const int rc = correct_fast(n_reads, base_off, byte_off, packed, quals, K, maxq, &set, stats);
  free(set.tab);
  return rc;
}

int ork_precorrect_fast(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed,
                        uint8_t* quals, int K, uint32_t min_solid, uint32_t maxq, uint32_t n_cycles, uint64_t* stats) {
  memset(stats, 0, 5 * sizeof(uint64_t));
  if (K < 2 || K > 29) return -1;
  for (uint32_t cyc = 0; cyc < n_cycles; ++cyc) {
    uint64_t* h = NULL;
    uint32_t* c = NULL;
    const uint64_t nd = ork_kmer_count(n_reads, base_off, byte_off, packed, K, &h, &c);
    if (nd == UINT64_MAX) return -1;
    uint64_t ns = 0;
    for (uint64_t i = 0; i < nd; ++i)
      if (c[i] >= min_solid) h[ns++] = h[i];
    free(c);
    OSolid set;
    if (osolid_build_table(&set, h, ns)) {
      free(h);
      return -1;
    }
    free(h);
    stats[4] = ns;
    const int rc = correct_fast(n_reads, base_off, byte_off, packed, quals, K, maxq, &set, stats);
    free(set.tab);
    if (rc) return -1;
  }
  return 0;
}
