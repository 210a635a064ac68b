/* ecj_oracle.c — CPU restatement of ErrorCorrectJump's trimming step (TEST
 * INFRASTRUCTURE ONLY: the checker of allpathslg_amd's
 * apg_error_correct_jump; never linked into the product).
 *
 * Parity unpinned: /root/reference is empty; recalled
 * reference [R:M] src/paths/ErrorCorrectJump.cc (grep target only).  Spec
 * (include/apg.h apg_error_correct_jump): after one PreCorrect pass of the
 * jump reads against the fragment reads' solid set (precorrect_oracle.c,
 * ork_precorrect_solid), each read keeps its longest prefix whose K-mers are
 * all solid: keep = L if every K-mer is solid, else j0 + K - 1 for the first
 * non-solid K-mer j0; keep = 0 if L < K or keep < min_keep.  Solidity is a
 * binary search of ork_hash(K, canonical K-mer) in the sorted solid hashes —
 * independent of the GPU's extension table. */
#include <stdint.h>
#include <stdlib.h>

#include "oracle.h"

static int has(const uint64_t* s, uint64_t n, uint64_t x) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) / 2;
    if (s[mid] < x)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < n && s[lo] == x;
}

/* solid: ascending khash values.  keep: one u32 per read. */
void oje_trim(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed, int K,
              const uint64_t* solid, uint64_t ns, uint32_t min_keep, uint32_t* keep) {
  const uint64_t mask = K == 32 ? ~0ull : (1ull << (2 * K)) - 1;
  /* reads are independent: OpenMP over them (full-size C3 parity) */
#pragma omp parallel for schedule(dynamic, 4096)
  for (uint64_t r = 0; r < n_reads; ++r) {
    const uint64_t L = base_off[r + 1] - base_off[r];
    const uint8_t* p = packed + byte_off[r];
    uint32_t k = 0;
    if (L >= (uint64_t)K) {
      uint64_t j0 = L - K + 1; /* first non-solid K-mer (none: nk) */
      for (uint64_t j = 0; j + K <= L; ++j) {
        uint64_t fw = 0, rc = 0;
        for (int t = 0; t < K; ++t) {
          const uint64_t b = (p[(j + t) >> 2] >> (2 * ((j + t) & 3))) & 3;
          fw = (fw << 2) | b;
          rc |= (3 - b) << (2 * t);
        }
        fw &= mask;
        const uint64_t c = fw < rc ? fw : rc;
        if (!has(solid, ns, ork_hash(K, c))) {
          j0 = j;
          break;
        }
      }
      k = j0 == L - K + 1 ? (uint32_t)L : (uint32_t)(j0 + K - 1);
      if (k < min_keep) k = 0;
    }
    keep[r] = k;
  }
}
