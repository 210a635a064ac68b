/* san_oracle.c — the CPU restatement (oracle/, TEST INFRASTRUCTURE) under
 * -fsanitize=address,undefined: its known-answer
 * tests run here on OpenMP threads, in C, with no Python in the
 * process, so every allocation and index of the restatement is checked:
 *   - spectrum of an error-free tiling: every interior K-mer seen L-K+1
 *     times, sum m*h[m] = instances, parcel counts add up to the table;
 *   - PreCorrect: a low-quality substitution in one read of a 40x tiling is
 *     corrected and nothing else changes;
 *   - FillFragments of error-free pairs: every pair closes to its insert;
 *   - gap-free / banded SW / consensus of exact placements: 0 mismatches,
 *     cost 0, consensus = target;
 *   - ErrorCorrectJump trim of solid reads keeps whole reads. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../oracle/oracle.h"

static int fails = 0;
#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c);     \
      ++fails;                                                         \
    }                                                                  \
  } while (0)

static uint64_t st = 0x2545F4914F6CDD1Dull;
static uint64_t rnd(void) {
  st ^= st << 13;
  st ^= st >> 7;
  st ^= st << 17;
  return st;
}

typedef struct {
  uint64_t n;
  uint64_t *bo, *yo;
  uint8_t *packed, *quals;
} Reads;

static void reads_alloc(Reads* r, uint64_t n, const uint32_t* lens) {
  r->n = n;
  r->bo = calloc(n + 1, 8);
  r->yo = calloc(n + 1, 8);
  for (uint64_t i = 0; i < n; ++i) {
    r->bo[i + 1] = r->bo[i] + lens[i];
    r->yo[i + 1] = r->yo[i] + (lens[i] + 3) / 4;
  }
  r->packed = calloc(r->yo[n] + 64, 1);
  r->quals = malloc(r->bo[n] + 1);
  memset(r->quals, 40, r->bo[n] + 1);
}
static void reads_free(Reads* r) {
  free(r->bo);
  free(r->yo);
  free(r->packed);
  free(r->quals);
}
static void put_base(Reads* r, uint64_t i, uint32_t j, uint8_t b) {
  uint8_t* p = r->packed + r->yo[i] + j / 4;
  *p = (uint8_t)((*p & ~(3u << (2 * (j % 4)))) | (b << (2 * (j % 4))));
}
static uint8_t get_base(const Reads* r, uint64_t i, uint32_t j) {
  return (r->packed[r->yo[i] + j / 4] >> (2 * (j % 4))) & 3;
}

/* reads of length L starting at every `step`-th position of g (forward strand) */
static void tiling(Reads* r, const uint8_t* g, uint64_t G, uint32_t L, uint32_t step) {
  const uint64_t n = (G - L) / step + 1;
  uint32_t* lens = malloc(n * 4);
  for (uint64_t i = 0; i < n; ++i) lens[i] = L;
  reads_alloc(r, n, lens);
  free(lens);
  for (uint64_t i = 0; i < n; ++i)
    for (uint32_t j = 0; j < L; ++j) put_base(r, i, j, g[i * step + j]);
}

static void kat_spectrum(const uint8_t* g, uint64_t G) {
  Reads r;
  const int K = 25;
  const uint32_t L = 100;
  tiling(&r, g, G, L, 1);
  uint64_t* h = NULL;
  uint32_t* c = NULL;
  const uint64_t nd = ork_kmer_count(r.n, r.bo, r.yo, r.packed, K, &h, &c);
  uint64_t hist[1024] = {0};
  ork_spectrum(c, nd, hist, 1024);
  uint64_t inst = 0;
  for (int m = 1; m < 1024; ++m) inst += (uint64_t)m * hist[m];
  CHECK(inst == r.n * (L - K + 1));
  CHECK(inst == ork_count_instances(r.n, r.bo, K));
  CHECK(hist[L - K + 1] >= G - 2 * L);  /* interior K-mers: every read over them */
  CHECK(nd == G - K + 1);                /* a random genome has no repeated 25-mer */
  /* parcels of the hash space add up to the table */
  uint64_t tot = 0;
  for (int p = 0; p < 4; ++p) {
    uint64_t *ph = NULL;
    uint32_t* pc = NULL;
    const uint64_t lo = (uint64_t)p << 62, hi = p == 3 ? 0 : (uint64_t)(p + 1) << 62;
    tot += ork_kmer_count_range(r.n, r.bo, r.yo, r.packed, K, lo, hi, &ph, &pc);
    ork_free(ph);
    ork_free(pc);
  }
  CHECK(tot == nd);
  ork_free(h);
  ork_free(c);
  reads_free(&r);
}

static void kat_precorrect(const uint8_t* g, uint64_t G) {
  Reads r;
  tiling(&r, g, 4000 < G ? 4000 : G, 100, 2);  /* ~50x */
  const uint64_t victim = r.n / 2;
  const uint32_t pos = 50;
  const uint8_t orig = get_base(&r, victim, pos);
  put_base(&r, victim, pos, (uint8_t)((orig + 1) & 3));
  r.quals[r.bo[victim] + pos] = 5;
  uint64_t stats[8] = {0};
  CHECK(ork_precorrect(r.n, r.bo, r.yo, r.packed, r.quals, 24, 3, 20, 1, stats) == 0);
  CHECK(get_base(&r, victim, pos) == orig);
  CHECK(stats[1] == 1); /* n_corrected */
  reads_free(&r);
}

static void kat_fill_align(const uint8_t* g, uint64_t G) {
  /* pairs (A, B) of an insert of 180: A = g[s, s+100), B = rc(g[s+80, s+180)) */
  const uint64_t np = 400;
  uint32_t* lens = malloc(2 * np * 4);
  for (uint64_t i = 0; i < 2 * np; ++i) lens[i] = 100;
  Reads r;
  reads_alloc(&r, 2 * np, lens);
  free(lens);
  for (uint64_t p = 0; p < np; ++p) {
    const uint64_t s = (p * 37) % (G - 200);
    for (uint32_t j = 0; j < 100; ++j) {
      put_base(&r, 2 * p, j, g[s + j]);
      put_base(&r, 2 * p + 1, j, (uint8_t)(3 - g[s + 179 - j]));
    }
  }
  /* solid set: every 24-mer of the genome (counted from an error-free tiling) */
  Reads t;
  tiling(&t, g, G, 100, 1);
  uint64_t* hs = NULL;
  uint32_t* cs = NULL;
  const uint64_t ns = ork_kmer_count(t.n, t.bo, t.yo, t.packed, 24, &hs, &cs);
  uint8_t* status = calloc(np, 1);
  uint32_t* flen = calloc(np, 4);
  uint8_t* fb = NULL;
  uint64_t fst[12] = {0};
  CHECK(orf_fill(r.n, r.bo, r.yo, r.packed, 24, hs, ns, 126, 234, 1024, status, flen, &fb, fst) == 0);
  uint64_t ok = 0;
  for (uint64_t p = 0; p < np; ++p) ok += status[p] == 0 && flen[p] == 180;
  CHECK(ok == np);
  ork_free(fb);
  /* ErrorCorrectJump trim: every K-mer solid -> whole reads kept */
  uint32_t* keep = calloc(r.n, 4);
  oje_trim(r.n, r.bo, r.yo, r.packed, 24, hs, ns, 40, keep);
  uint64_t whole = 0;
  for (uint64_t i = 0; i < r.n; ++i) whole += keep[i] == 100;
  CHECK(whole == r.n);
  free(keep);
  /* aligners: read 2p placed on the genome at its start */
  Reads T;
  uint32_t tl = (uint32_t)G;
  reads_alloc(&T, 1, &tl);
  for (uint64_t j = 0; j < G; ++j) put_base(&T, 0, (uint32_t)j, g[j]);
  uint32_t* pairs = malloc(np * 16);
  for (uint64_t p = 0; p < np; ++p) {
    pairs[4 * p] = (uint32_t)(2 * p);
    pairs[4 * p + 1] = 0;
    pairs[4 * p + 2] = (uint32_t)((p * 37) % (G - 200));
    pairs[4 * p + 3] = 0;
  }
  uint32_t* gf = calloc(np, 16);
  ora_gapfree(r.bo, r.yo, r.packed, r.quals, T.bo, T.yo, T.packed, pairs, np, gf);
  uint64_t exact = 0;
  for (uint64_t p = 0; p < np; ++p) exact += gf[4 * p] == 100 && gf[4 * p + 1] == 0;
  CHECK(exact == np);
  int32_t* sw = calloc(np, 32);
  ora_banded_sw(r.bo, r.yo, r.packed, T.bo, T.yo, T.packed, pairs, np, 8, sw, NULL, 0);
  uint64_t zero = 0;
  for (uint64_t p = 0; p < np; ++p) zero += sw[8 * p] == 0 && sw[8 * p + 7] == 0;
  CHECK(zero == np);
  uint8_t* cons = calloc(G, 1);
  uint8_t* cq = calloc(G, 1);
  ora_consensus(r.bo, r.yo, r.packed, r.quals, T.bo, T.yo, T.packed, 1, pairs, np, cons, cq);
  uint64_t same = 0;
  for (uint64_t j = 0; j < G; ++j) same += cons[j] == g[j];
  CHECK(same == G);
  free(cons);
  free(cq);
  free(sw);
  free(gf);
  free(pairs);
  free(status);
  free(flen);
  ork_free(hs);
  ork_free(cs);
  reads_free(&T);
  reads_free(&t);
  reads_free(&r);
}

int main(void) {
  const uint64_t G = 60000;
  uint8_t* g = malloc(G);
  for (uint64_t i = 0; i < G; ++i) g[i] = (uint8_t)(rnd() >> 62);
  ork_set_threads(4);
  kat_spectrum(g, G);
  kat_precorrect(g, G);
  kat_fill_align(g, G);
  free(g);
  printf("san_oracle: %s (%d failures)\n", fails ? "FAILED" : "ok", fails);
  return fails ? 1 : 0;
}
