/*
 * oracle/fill_oracle.c — CPU restatement of FillFragments (SURVEY.md §8f next
 * #1; recalled [R:M] src/paths/FillFragments.cc — a grep target only, the
 * reference snapshot is empty).  TEST INFRASTRUCTURE ONLY:
 * loaded by tests/ and bench.py's cpu_baseline leg, never by libapg.
 *
 * PARITY UNPINNED against the real ALLPATHS-LG.  The rule restated here is
 * the one include/apg.h (apg_fill_fragments) pins:
 *
 *   Pair i = reads (2i, 2i+1) = (A, B), FR: F = rc(B) is the fragment's end
 *   in A's orientation.  A closure of length I is a sequence S of length I
 *   with S[0, La) = A and S[I-Lf, I) = F (agreeing where they overlap),
 *   I in [max(min_insert, La, Lf), max_insert], and EVERY K-mer of S solid
 *   (S is a path of the solid K-mer graph): A's and F's own K-mers, and the
 *   bridge K-mers contained in neither (starting at p in [La-K+1, I-Lf-1]).
 *   Exactly one closure over all I: the pair is filled with S.
 *
 *   Search order (it decides BUDGET vs AMBIGUOUS): overlap lengths I < La+Lf
 *   ascending, then a depth-first walk from A's last K-1 bases over solid
 *   K-mers, bases A<C<G<T, depth d = I - La - Lf in [0, max_insert-La-Lf]; at
 *   each node the closure test comes first, then (d < max depth) the node is
 *   expanded; every expansion counts one step, more than max_steps steps ends
 *   the pair as BUDGET; a second closure ends it as AMBIGUOUS.
 *
 * Solid lookup: binary search of the ascending solid-hash array (ork_hash of
 * the canonical K-mer) — a different structure from the GPU's (K-1)-mer
 * extension table.  orf_fill_fast (bench.py's CPU baseline only) runs the
 * same search through a hash table of the same set (solidset.h).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"
#include "solidset.h"

enum { FILL_OK = 0, FILL_NONE = 1, FILL_AMBIGUOUS = 2, FILL_BUDGET = 3, FILL_SKIP = 4 };
#define FILL_MAX_GAP 63

typedef struct {
  int K;
  const OSolid* solid;
  const uint8_t* A;
  uint32_t La;
  const uint8_t* F;
  uint32_t Lf;
  uint32_t dlo, gmax;
  uint32_t max_steps, steps;
  uint32_t n_clos, clos_I;
  int budget_hit;
  uint64_t lookups;
  uint8_t path[FILL_MAX_GAP + 1], clos_path[FILL_MAX_GAP + 1];
} FillState;

static int cmp_hash(const void* a, const void* b) {
  const uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? -1 : x > y;
}

/* solid(K-mer given by K base codes) */
static int solid_codes(FillState* s, const uint8_t* b) {
  const int K = s->K;
  const uint64_t m = K >= 32 ? ~0ull : ((1ull << (2 * K)) - 1);
  uint64_t fw = 0, rc = 0;
  for (int t = 0; t < K; ++t) {
    fw = ((fw << 2) | b[t]) & m;
    rc = (rc >> 2) | ((uint64_t)(3 - b[t]) << (2 * K - 2));
  }
  s->lookups++;
  return osolid_has(s->solid, ork_hash(K, fw < rc ? fw : rc));
}

/* base pos of A ++ path[0, d) ++ F */
static uint8_t gap_base(const FillState* s, uint32_t d, uint32_t pos) {
  if (pos < s->La) return s->A[pos];
  if (pos < s->La + d) return s->path[pos - s->La];
  return s->F[pos - s->La - d];
}

/* closure of length La+Lf+d through path[0, d): its K-1 bridge K-mers */
static int closure_gap(FillState* s, uint32_t d) {
  uint8_t km[32];
  const uint32_t K = (uint32_t)s->K;
  for (uint32_t p = s->La + d - K + 1; p <= s->La + d - 1; ++p) {
    for (uint32_t t = 0; t < K; ++t) km[t] = gap_base(s, d, p + t);
    if (!solid_codes(s, km)) return 0;
  }
  return 1;
}

/* closure of length I = La+Lf-o, o >= 1 */
static int closure_overlap(FillState* s, uint32_t o) {
  for (uint32_t t = 0; t < o; ++t)
    if (s->A[s->La - o + t] != s->F[t]) return 0;
  const uint32_t K = (uint32_t)s->K;
  if (o + 2 > K) return 1; /* o >= K-1: no bridge K-mer */
  uint8_t km[32];
  for (uint32_t p = s->La - K + 1; p <= s->La - o - 1; ++p) {
    for (uint32_t t = 0; t < K; ++t) {
      const uint32_t q = p + t;
      km[t] = q < s->La ? s->A[q] : s->F[q - s->La + o];
    }
    if (!solid_codes(s, km)) return 0;
  }
  return 1;
}

/* returns 1 when the search must stop (second closure or budget) */
static int dfs(FillState* s, uint32_t d) {
  if (d >= s->dlo && closure_gap(s, d)) {
    if (++s->n_clos == 1) {
      s->clos_I = s->La + s->Lf + d;
      memcpy(s->clos_path, s->path, d);
    }
    if (s->n_clos >= 2) return 1;
  }
  if (d == s->gmax) return 0;
  if (++s->steps > s->max_steps) {
    s->budget_hit = 1;
    return 1;
  }
  const uint32_t K = (uint32_t)s->K;
  uint8_t km[32];
  for (uint32_t t = 0; t + 1 < K; ++t) km[t] = gap_base(s, d, s->La + d - (K - 1) + t);
  for (uint8_t b = 0; b < 4; ++b) {
    km[K - 1] = b;
    if (!solid_codes(s, km)) continue;
    s->path[d] = b;
    if (dfs(s, d + 1)) return 1;
  }
  return 0;
}

static void unpack(const uint8_t* pk, uint32_t L, uint8_t* out) {
  for (uint32_t i = 0; i < L; ++i) out[i] = (pk[i >> 2] >> (2 * (i & 3))) & 3;
}

/*
 * Pairs (2i, 2i+1) of the read set.  solid: hashes of solid canonical K-mers,
 * any order.  Outputs per pair: status[i], flen[i] (I when filled, else 0).
 * *out_bases (malloc'd, release with ork_free): the filled fragments' base
 * codes, one byte per base, concatenated in pair order.  stats[0..6] =
 * filled, none, ambiguous, budget, skip, filled bases, solid lookups.
 * Returns 0, or -1 on allocation failure / bad arguments.
 */
/* One pair (2i, 2i+1): status, closure length (0 unless filled), and for a
 * gap closure its bridge bases in path[]; returns the solid lookups made.
 * Pairs are independent: orf_fill runs them on the OpenMP threads. */
static uint64_t fill_pair(const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed, int K,
                          const OSolid* h, uint32_t min_insert, uint32_t max_insert,
                          uint32_t max_steps, uint64_t i, uint8_t* A, uint8_t* B, uint8_t* F, uint8_t* status,
                          uint32_t* flen, uint8_t* path) {
  const uint32_t La = (uint32_t)(base_off[2 * i + 1] - base_off[2 * i]);
  const uint32_t Lf = (uint32_t)(base_off[2 * i + 2] - base_off[2 * i + 1]);
  flen[i] = 0;
  uint32_t lo = min_insert;
  if (La > lo) lo = La;
  if (Lf > lo) lo = Lf;
  if (La < (uint32_t)K || Lf < (uint32_t)K || (max_insert >= La + Lf && max_insert - (La + Lf) > FILL_MAX_GAP)) {
    status[i] = FILL_SKIP;
    return 0;
  }
  unpack(packed + byte_off[2 * i], La, A);
  unpack(packed + byte_off[2 * i + 1], Lf, B);
  for (uint32_t t = 0; t < Lf; ++t) F[t] = (uint8_t)(3 - B[Lf - 1 - t]);
  FillState s;
  memset(&s, 0, sizeof s);
  s.K = K, s.solid = h, s.A = A, s.La = La, s.F = F, s.Lf = Lf, s.max_steps = max_steps;
  /* S must be a path of solid K-mers: A's own and F's own K-mers first */
  int clean = 1;
  for (uint32_t j = 0; j + (uint32_t)K <= La && clean; ++j) clean = solid_codes(&s, A + j);
  for (uint32_t j = 0; j + (uint32_t)K <= Lf && clean; ++j) clean = solid_codes(&s, F + j);
  if (!clean) {
    status[i] = FILL_NONE;
    return s.lookups;
  }
  int stop = 0;
  for (uint32_t I = lo; I <= max_insert && I < La + Lf && !stop; ++I) {
    if (closure_overlap(&s, La + Lf - I)) {
      if (++s.n_clos == 1) s.clos_I = I;
      if (s.n_clos >= 2) stop = 1;
    }
  }
  if (!stop && max_insert >= La + Lf) {
    s.gmax = max_insert - (La + Lf);
    s.dlo = lo > La + Lf ? lo - (La + Lf) : 0;
    dfs(&s, 0);
  }
  uint8_t st;
  if (s.n_clos >= 2)
    st = FILL_AMBIGUOUS;
  else if (s.budget_hit)
    st = FILL_BUDGET;
  else if (s.n_clos == 0)
    st = FILL_NONE;
  else
    st = FILL_OK;
  status[i] = st;
  if (st == FILL_OK) {
    flen[i] = s.clos_I;
    memcpy(path, s.clos_path, FILL_MAX_GAP + 1);
  }
  return s.lookups;
}

/*
 * Pairs (2i, 2i+1) of the read set.  solid: hashes of solid canonical K-mers,
 * any order.  Outputs per pair: status[i], flen[i] (I when filled, else 0).
 * *out_bases (malloc'd, release with ork_free): the filled fragments' base
 * codes, one byte per base, concatenated in pair order.  stats[0..6] =
 * filled, none, ambiguous, budget, skip, filled bases, solid lookups.
 * Returns 0, or -1 on allocation failure / bad arguments.
 */
static int fill_impl(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed,
                     int K, const uint64_t* solid, uint64_t ns, uint32_t min_insert, uint32_t max_insert,
                     uint32_t max_steps, uint8_t* status, uint32_t* flen, uint8_t** out_bases, uint64_t* stats,
                     int table) {
  memset(stats, 0, 7 * sizeof(uint64_t));
  *out_bases = NULL;
  if ((n_reads & 1) || K < 2 || K > 32) return -1;
  OSolid set;
  memset(&set, 0, sizeof set);
  uint64_t* h = NULL;
  if (table) {
    if (osolid_build_table(&set, solid, ns)) return -1;
    h = set.tab;
  } else {
    h = (uint64_t*)malloc((ns ? ns : 1) * sizeof(uint64_t));
    if (!h) return -1;
    if (ns) memcpy(h, solid, ns * sizeof(uint64_t));
    qsort(h, ns, sizeof(uint64_t), cmp_hash);
    set.sorted = h;
    set.n = ns;
  }
  uint32_t maxL = 0;
  for (uint64_t r = 0; r < n_reads; ++r) {
    const uint32_t L = (uint32_t)(base_off[r + 1] - base_off[r]);
    if (L > maxL) maxL = L;
  }
  const uint64_t n_pairs = n_reads / 2;
  uint8_t* paths = (uint8_t*)malloc((n_pairs ? n_pairs : 1) * (FILL_MAX_GAP + 1));
  if (!paths) {
    free(h);
    return -1;
  }
  uint64_t lookups = 0;
  int fail = 0;
#pragma omp parallel reduction(+ : lookups)
  {
    uint8_t* A = (uint8_t*)malloc(maxL + 1);
    uint8_t* B = (uint8_t*)malloc(maxL + 1);
    uint8_t* F = (uint8_t*)malloc(maxL + 1);
    if (!A || !B || !F) {
#pragma omp atomic write
      fail = 1;
    }
#pragma omp for schedule(dynamic, 64)
    for (uint64_t i = 0; i < n_pairs; ++i)
      if (A && B && F)
        lookups += fill_pair(base_off, byte_off, packed, K, &set, min_insert, max_insert, max_steps, i, A, B, F,
                             status, flen, paths + i * (FILL_MAX_GAP + 1));
    free(A), free(B), free(F);
  }
  free(h);
  if (fail) {
    free(paths);
    return -1;
  }
  stats[6] = lookups;
  uint64_t total = 0;
  for (uint64_t i = 0; i < n_pairs; ++i) {
    stats[status[i]]++;
    total += flen[i];
  }
  stats[5] = total;
  uint8_t* out = (uint8_t*)malloc(total ? total : 1);
  if (!out) {
    free(paths);
    return -1;
  }
  /* S = A ++ path ++ F (gap), or A ++ F[o, Lf) (overlap o = La+Lf-I) */
  uint64_t used = 0;
  uint8_t* A = (uint8_t*)malloc(maxL + 1);
  uint8_t* B = (uint8_t*)malloc(maxL + 1);
  for (uint64_t i = 0; i < n_pairs && A && B; ++i) {
    const uint32_t I = flen[i];
    if (!I) continue;
    const uint32_t La = (uint32_t)(base_off[2 * i + 1] - base_off[2 * i]);
    const uint32_t Lf = (uint32_t)(base_off[2 * i + 2] - base_off[2 * i + 1]);
    unpack(packed + byte_off[2 * i], La, A);
    unpack(packed + byte_off[2 * i + 1], Lf, B);
    uint8_t* S = out + used;
    memcpy(S, A, La);
    uint8_t* Fp = S + I - Lf; /* F's bases land at the end of S */
    if (I < La + Lf) {
      const uint32_t o = La + Lf - I;
      for (uint32_t t = o; t < Lf; ++t) S[La + t - o] = (uint8_t)(3 - B[Lf - 1 - t]);
    } else {
      const uint32_t d = I - La - Lf;
      memcpy(S + La, paths + i * (FILL_MAX_GAP + 1), d);
      for (uint32_t t = 0; t < Lf; ++t) Fp[t] = (uint8_t)(3 - B[Lf - 1 - t]);
    }
    used += I;
  }
  free(A), free(B), free(paths);
  *out_bases = out;
  return 0;
}

int orf_fill(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed, int K,
             const uint64_t* solid, uint64_t ns, uint32_t min_insert, uint32_t max_insert, uint32_t max_steps,
             uint8_t* status, uint32_t* flen, uint8_t** out_bases, uint64_t* stats) {
  return fill_impl(n_reads, base_off, byte_off, packed, K, solid, ns, min_insert, max_insert, max_steps, status, flen,
                   out_bases, stats, 0);
}

/* bench.py's CPU baseline: the same fill, solid lookups through a hash table */
int orf_fill_fast(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed, int K,
                  const uint64_t* solid, uint64_t ns, uint32_t min_insert, uint32_t max_insert, uint32_t max_steps,
                  uint8_t* status, uint32_t* flen, uint8_t** out_bases, uint64_t* stats) {
  return fill_impl(n_reads, base_off, byte_off, packed, K, solid, ns, min_insert, max_insert, max_steps, status, flen,
                   out_bases, stats, 1);
}
