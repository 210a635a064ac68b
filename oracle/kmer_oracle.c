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
 * Deliberately simple: generate -> LSD radix sort -> run-length; the
 * independent per-read extraction and the per-partition sorts run on the
 * OpenMP threads given (the CPU baseline's host-cores figure).
 */
#include <omp.h>
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

/* Parallel sort: one MSD pass on the top 8 of `bits` bits (per-thread
 * histograms, stable scatter), then every partition LSD-sorted on its own
 * thread.  Same result as radix_sort_u64. */
static int psort_u64(uint64_t* a, uint64_t n, int bits) {
  const int T = omp_get_max_threads();
  if (T <= 1 || n < (1u << 20) || bits <= 8) {
    radix_sort_u64(a, n, bits);
    return 0;
  }
  const int top = bits - 8;
  uint64_t* tmp = (uint64_t*)malloc(n * sizeof(uint64_t));
  uint64_t* cnt = (uint64_t*)calloc((size_t)T * 256, sizeof(uint64_t));
  if (!tmp || !cnt) {
    free(tmp), free(cnt);
    return -1;
  }
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    const uint64_t lo = n * (uint64_t)t / T, hi = n * (uint64_t)(t + 1) / T;
    uint64_t* c = cnt + (size_t)t * 256;
    for (uint64_t i = lo; i < hi; ++i) c[(a[i] >> top) & 255]++;
#pragma omp barrier
#pragma omp single
    {
      uint64_t run = 0;
      for (int d = 0; d < 256; ++d)
        for (int u = 0; u < T; ++u) {
          const uint64_t x = cnt[(size_t)u * 256 + d];
          cnt[(size_t)u * 256 + d] = run;
          run += x;
        }
    }
    for (uint64_t i = lo; i < hi; ++i) tmp[c[(a[i] >> top) & 255]++] = a[i];
  }
  uint64_t start[257];
  start[0] = 0;
  for (int d = 0; d < 256; ++d) start[d + 1] = cnt[(size_t)(T - 1) * 256 + d];
  free(cnt);
#pragma omp parallel for schedule(dynamic, 1)
  for (int d = 0; d < 256; ++d) {
    radix_sort_u64(tmp + start[d], start[d + 1] - start[d], top);
    memcpy(a + start[d], tmp + start[d], (start[d + 1] - start[d]) * sizeof(uint64_t));
  }
  free(tmp);
  return 0;
}

/* Run-length count of the ascending h[0..n) in place; counts into *counts. */
static uint64_t run_length(uint64_t* h, uint64_t n, uint32_t** counts) {
  uint32_t* c = (uint32_t*)malloc((n ? n : 1) * sizeof(uint32_t));
  if (!c) return UINT64_MAX;
  uint64_t d = 0;
  for (uint64_t i = 0; i < n;) {
    uint64_t j = i + 1;
    while (j < n && h[j] == h[i]) ++j;
    h[d] = h[i];
    c[d] = (uint32_t)(j - i);
    ++d;
    i = j;
  }
  *counts = c;
  return d;
}

/* (hash, count) table in ascending hash order.  Returns #distinct, or
 * UINT64_MAX on allocation failure.  Caller frees *hashes / *counts. */
uint64_t ork_kmer_count(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off,
                        const uint8_t* packed, int K, uint64_t** hashes, uint32_t** counts) {
  /* instance offset of every read, then the reads' hashes in parallel */
  uint64_t* ioff = (uint64_t*)malloc((n_reads + 1) * sizeof(uint64_t));
  if (!ioff) return UINT64_MAX;
  ioff[0] = 0;
  for (uint64_t r = 0; r < n_reads; ++r) {
    const uint64_t len = base_off[r + 1] - base_off[r];
    ioff[r + 1] = ioff[r] + (len >= (uint64_t)K ? len - K + 1 : 0);
  }
  const uint64_t n = ioff[n_reads];
  uint64_t* h = (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
  if (!h) {
    free(ioff);
    return UINT64_MAX;
  }
#pragma omp parallel for schedule(dynamic, 4096)
  for (uint64_t r = 0; r < n_reads; ++r)
    ork_extract_hashes(1, base_off + r, byte_off + r, packed, K, h + ioff[r]);
  free(ioff);
  if (psort_u64(h, n, 2 * K)) {
    free(h);
    return UINT64_MAX;
  }
  *hashes = h;
  return run_length(h, n, counts);
}

/* Parcel of the counted table (KmerParcels' K-mer-space partition, [R:M]
 * src/kmers/KmerParcels.h): the (hash, count) entries with lo <= hash < hi,
 * ascending.  Extraction keeps only the parcel's instances (per-thread
 * buffers), so a 1/256 parcel of a 40 M-read set needs ~1/256 of the memory. */
uint64_t ork_kmer_count_range(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off,
                              const uint8_t* packed, int K, uint64_t lo, uint64_t hi, uint64_t** hashes,
                              uint32_t** counts) {
  const uint64_t m = wmask(2 * K);
  const int T = omp_get_max_threads();
  uint64_t** buf = (uint64_t**)calloc((size_t)T, sizeof(uint64_t*));
  uint64_t* len = (uint64_t*)calloc((size_t)T, sizeof(uint64_t));
  int fail = 0;
#pragma omp parallel num_threads(T)
  {
    const int t = omp_get_thread_num();
    uint64_t cap = 1 << 16, used = 0;
    uint64_t* b = (uint64_t*)malloc(cap * sizeof(uint64_t));
#pragma omp for schedule(dynamic, 4096)
    for (uint64_t r = 0; r < n_reads; ++r) {
      const uint64_t L = base_off[r + 1] - base_off[r];
      uint64_t fw = 0, rc = 0;
      for (uint64_t i = 0; i < L; ++i) {
        const uint64_t x = (uint64_t)base_at(packed, byte_off[r], i);
        fw = ((fw << 2) | x) & m;
        rc = (rc >> 2) | ((3 - x) << (2 * K - 2));
        if (i + 1 < (uint64_t)K) continue;
        const uint64_t hv = ork_hash(K, fw < rc ? fw : rc);
        if (hv < lo || hv >= hi || !b) continue;
        if (used == cap) {
          cap *= 2;
          uint64_t* nb = (uint64_t*)realloc(b, cap * sizeof(uint64_t));
          if (!nb) {
            free(b);
            b = NULL;
            continue;
          }
          b = nb;
        }
        b[used++] = hv;
      }
    }
    if (!b) {
#pragma omp atomic write
      fail = 1;
    }
    buf[t] = b;
    len[t] = used;
  }
  uint64_t n = 0;
  for (int t = 0; t < T; ++t) n += len[t];
  uint64_t* h = fail ? NULL : (uint64_t*)malloc((n ? n : 1) * sizeof(uint64_t));
  uint64_t at = 0;
  for (int t = 0; t < T; ++t) {
    if (h && len[t]) memcpy(h + at, buf[t], len[t] * sizeof(uint64_t));
    at += len[t];
    free(buf[t]);
  }
  free(buf), free(len);
  if (!h) return UINT64_MAX;
  if (psort_u64(h, n, 2 * K)) {
    free(h);
    return UINT64_MAX;
  }
  *hashes = h;
  return run_length(h, n, counts);
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

/* KmerSpectrum's genome-size estimate (include/apg.h apg_kspec_estimate, the
 * spec restated; [R:M] src/kmers/KmerSpectra.h, grep target only): the
 * valley where the error K-mers' decline ends, the single-copy peak after it,
 * genome positions = genomic instances / the peak's mean coverage (rounded).  u[] = {valley,
 * peak, genome_size, genomic_kmers, genomic_instances, error_kmers,
 * error_instances}; d[] = {coverage, repeat_fraction, het_ratio}. */
void ork_kspec_estimate(const uint64_t* h, uint64_t len, uint64_t* u, double* d) {
  memset(u, 0, 7 * sizeof(uint64_t));
  d[0] = d[1] = d[2] = 0.0;
  if (len < 3) return;
  uint64_t v = 0;
  for (uint64_t m = 1; m + 2 < len; ++m)
    if (h[m] < h[m + 1]) {
      v = m;
      break;
    }
  if (v == 0) return;
  uint64_t p = 0, best = 0;
  for (uint64_t m = v + 1; m + 1 < len; ++m)
    if (h[m] > best) {
      best = h[m];
      p = m;
    }
  for (uint64_t m = 1; m < len; ++m) {
    if (m < v) {
      u[5] += h[m];
      u[6] += m * h[m];
    } else {
      u[3] += h[m];
      u[4] += m * h[m];
    }
  }
  u[0] = v;
  u[1] = p;
  if (p == 0) return;
  /* mean coverage of the single-copy peak: m in [v, min(2p - v, len - 2)] */
  unsigned __int128 s0 = 0, s1 = 0;
  uint64_t hi = 2 * p - v;
  if (hi > len - 2) hi = len - 2;
  for (uint64_t m = v; m <= hi; ++m) {
    s0 += h[m];
    s1 += (unsigned __int128)m * h[m];
  }
  d[0] = (double)s1 / (double)s0;
  u[2] = (uint64_t)(((unsigned __int128)u[4] * s0 + s1 / 2) / s1);
  if (u[2] > u[3]) d[1] = (double)(u[2] - u[3]) / (double)u[2];
  if (p >= 2) d[2] = (double)h[p / 2] / (double)h[p];
}

void ork_free(void* p) { free(p); }

/* Host threads of the OpenMP loops (0: OMP_NUM_THREADS / all cores). */
void ork_set_threads(int n) {
  if (n > 0) omp_set_num_threads(n);
}
int ork_threads(void) { return omp_get_max_threads(); }
