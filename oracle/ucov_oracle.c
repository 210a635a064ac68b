/* ucov_oracle.c — CPU restatement of UnipathCoverage: placements per unipath,
 * placements per K-mer, the genome-wide coverage and copy-number estimates
 * (TEST INFRASTRUCTURE ONLY: the checker of allpathslg_amd's
 * apg_unipath_coverage; never linked into the product).
 *
 * Parity unpinned: /root/reference is empty.  Recalled
 * reference [R:M]: UnipathCoverage, src/paths/UnipathCoverage* (grep target
 * only).  The operational spec is the one pinned in include/apg.h
 * (apg_unipath_coverage):
 *   n[u]   = placements with t_id == u;
 *   cov[u] = (double)n[u] / (double)len[u];
 *   c0     = length-weighted median of cov over unipaths with len >= min_len
 *            (ascending cov, first whose cumulative length L has 2L >= total);
 *   cn[u]  = c0 > 0 ? floor(cov[u] / c0 + 0.5) : 0.
 * Written independently of the HIP kernels (a plain counting loop and an
 * insertion-free qsort selection). */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include "oracle.h"

typedef struct {
  double cov;
  uint64_t len;
} ouc_item;

static int ouc_cmp(const void* a, const void* b) {
  const double x = ((const ouc_item*)a)->cov, y = ((const ouc_item*)b)->cov;
  return x < y ? -1 : x > y ? 1 : 0;
}

/* pairs: n rows of 4 u32 (read, unipath, start, flags).  Returns 0, or -1 on
 * a placement whose unipath is out of range, -2 on allocation failure. */
int ouc_coverage(uint64_t U, const uint64_t* ulen, const uint32_t* pairs, uint64_t n, uint64_t min_len,
                 uint64_t* counts, double* cov, uint32_t* cn, double* c0_out, uint64_t* n_long) {
  for (uint64_t u = 0; u < U; ++u) counts[u] = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t u = pairs[4 * i + 1];
    if (u >= U) return -1;
    ++counts[u];
  }
  uint64_t m = 0, W = 0;
  ouc_item* it = (ouc_item*)malloc((U ? U : 1) * sizeof(ouc_item));
  if (!it) return -2;
  for (uint64_t u = 0; u < U; ++u) {
    cov[u] = ulen[u] ? (double)counts[u] / (double)ulen[u] : 0.0;
    if (ulen[u] >= min_len) {
      it[m].cov = cov[u];
      it[m].len = ulen[u];
      W += ulen[u];
      ++m;
    }
  }
  qsort(it, m, sizeof(ouc_item), ouc_cmp);
  double c0 = 0.0;
  uint64_t acc = 0;
  for (uint64_t j = 0; j < m; ++j) {
    acc += it[j].len;
    if (2 * acc >= W) {
      c0 = it[j].cov;
      break;
    }
  }
  free(it);
  for (uint64_t u = 0; u < U; ++u) cn[u] = c0 > 0.0 ? (uint32_t)floor(cov[u] / c0 + 0.5) : 0u;
  *c0_out = c0;
  *n_long = m;
  return 0;
}
