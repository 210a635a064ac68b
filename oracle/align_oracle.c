/*
 * oracle/align_oracle.c — CPU restatement of the read-to-unibase aligners and
 * the column consensus (SURVEY.md §A.7 as pinned in include/apg.h).
 * TEST INFRASTRUCTURE ONLY.
 *
 * PARITY UNPINNED: the reference snapshot is empty.  Recalled
 * reference modules (grep targets, no line citations possible):
 *   gap-free   [R:M] src/pairwise_aligners/PerfectAlignment*, KmerAligner
 *   banded SW  [R:M] src/pairwise_aligners/SmithWatBanded.cc (integer costs:
 *              mismatch 2, gap 3 per base [R:L-M])
 *   consensus  [R:L] CRefMerger / LongReadConsensus (names from BASELINE.json;
 *              closest recall src/paths/long/), restated in SURVEY §A.7.
 * Deliberately plain full-matrix code (no band-diagonal tricks, no bit
 * parallelism) so it shares no structure with the HIP kernels.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "oracle.h"

static int base_at(const uint8_t* rd, uint64_t i) { return (rd[i >> 2] >> (2 * (i & 3))) & 3; }

/* Base i of read r as aligned (flags bit0: reverse complement). */
static int sbase(const uint8_t* rd, uint32_t L, uint32_t i, int rc) {
  return rc ? 3 - base_at(rd, L - 1 - i) : base_at(rd, i);
}
static int squal(const uint8_t* q, uint32_t L, uint32_t i, int rc) { return q ? (rc ? q[L - 1 - i] : q[i]) : 0; }

/* out[4*k..]: overlap, mismatches, qsum, offset echo (as uint32). */
void ora_gapfree(const uint64_t* s_base_off, const uint64_t* s_byte_off, const uint8_t* s_packed,
                 const uint8_t* s_quals, const uint64_t* t_base_off, const uint64_t* t_byte_off,
                 const uint8_t* t_packed, const uint32_t* pairs /* 4 per pair */, uint64_t n, uint32_t* out) {
  for (uint64_t k = 0; k < n; ++k) {
    const uint32_t s = pairs[4 * k], t = pairs[4 * k + 1], flags = pairs[4 * k + 3];
    const int32_t off = (int32_t)pairs[4 * k + 2];
    const uint32_t Ls = (uint32_t)(s_base_off[s + 1] - s_base_off[s]);
    const uint32_t Lt = (uint32_t)(t_base_off[t + 1] - t_base_off[t]);
    const uint8_t* sr = s_packed + s_byte_off[s];
    const uint8_t* tr = t_packed + t_byte_off[t];
    const uint8_t* sq = s_quals ? s_quals + s_base_off[s] : NULL;
    const int rc = flags & 1;
    uint32_t ov = 0, mm = 0, qs = 0;
    for (uint32_t i = 0; i < Ls; ++i) {
      const int64_t j = (int64_t)off + i;
      if (j < 0 || j >= (int64_t)Lt) continue;
      ++ov;
      if (sbase(sr, Ls, i, rc) != base_at(tr, (uint64_t)j)) {
        ++mm;
        qs += (uint32_t)squal(sq, Ls, i, rc);
      }
    }
    out[4 * k] = ov;
    out[4 * k + 1] = mm;
    out[4 * k + 2] = qs;
    out[4 * k + 3] = (uint32_t)off;
  }
}

#define SW_INF 0x3fffffff
enum { DIR_START = 0, DIR_DIAG = 1, DIR_HORZ = 2, DIR_VERT = 3 };

/* Banded semi-global alignment of S (all of it) into T (free ends), band of
 * diagonals d = j - i in [off - w, off + w] (and 0 <= j <= |T|).
 *   D[0][j] = 0 in band (free T prefix)
 *   D[i][j] = min(D[i-1][j-1] + (S[i-1] == T[j-1] ? 0 : 2),   diagonal
 *                 D[i][j-1] + 3,                                gap in S
 *                 D[i-1][j] + 3)                                gap in T
 * ties: diagonal > gap in S > gap in T.  End: min over band cells of row |S|,
 * ties to the smallest j.  Traceback records blocks (gap, len): gap > 0 skips
 * T bases (gap in S), gap < 0 skips S bases (gap in T), then len columns of
 * S/T pairs.
 * res[8*k..]: cost, t_begin, t_end, mismatches, gap_s, gap_t, n_blocks, status
 * (status 0 ok, 1 no band cell reaches row |S|, 2 block buffer too small).
 * blocks: max_blocks (gap, len) int32 pairs per pair (may be NULL). */
void ora_banded_sw(const uint64_t* s_base_off, const uint64_t* s_byte_off, const uint8_t* s_packed,
                   const uint64_t* t_base_off, const uint64_t* t_byte_off, const uint8_t* t_packed,
                   const uint32_t* pairs, uint64_t n, int w, int32_t* res, int32_t* blocks, uint32_t max_blocks) {
  for (uint64_t k = 0; k < n; ++k) {
    const uint32_t s = pairs[4 * k], t = pairs[4 * k + 1], flags = pairs[4 * k + 3];
    const int32_t off = (int32_t)pairs[4 * k + 2];
    const int Ls = (int)(s_base_off[s + 1] - s_base_off[s]);
    const int Lt = (int)(t_base_off[t + 1] - t_base_off[t]);
    const uint8_t* sr = s_packed + s_byte_off[s];
    const uint8_t* tr = t_packed + t_byte_off[t];
    const int rc = flags & 1;
    int32_t* r = res + 8 * k;
    memset(r, 0, 8 * sizeof(int32_t));
    const size_t cols = (size_t)Lt + 1;
    int32_t* D = (int32_t*)malloc((size_t)(Ls + 1) * cols * sizeof(int32_t));
    uint8_t* dir = (uint8_t*)malloc((size_t)(Ls + 1) * cols);
    for (int i = 0; i <= Ls; ++i)
      for (int j = 0; j <= Lt; ++j) {
        const size_t c = (size_t)i * cols + (size_t)j;
        D[c] = SW_INF;
        dir[c] = DIR_START;
        const int d = j - i;
        if (d < off - w || d > off + w) continue;
        if (i == 0) {
          D[c] = 0;
          continue;
        }
        int32_t best = SW_INF;
        uint8_t bd = DIR_START;
        if (j >= 1 && D[c - cols - 1] < SW_INF) {
          const int32_t v = D[c - cols - 1] + (sbase(sr, (uint32_t)Ls, (uint32_t)(i - 1), rc) == base_at(tr, (uint64_t)(j - 1)) ? 0 : 2);
          best = v;
          bd = DIR_DIAG;
        }
        if (j >= 1 && D[c - 1] < SW_INF && D[c - 1] + 3 < best) {
          best = D[c - 1] + 3;
          bd = DIR_HORZ;
        }
        if (D[c - cols] < SW_INF && D[c - cols] + 3 < best) {
          best = D[c - cols] + 3;
          bd = DIR_VERT;
        }
        D[c] = best;
        dir[c] = bd;
      }
    int bj = -1;
    for (int j = 0; j <= Lt; ++j) {
      const size_t c = (size_t)Ls * cols + (size_t)j;
      if (D[c] < SW_INF && (bj < 0 || D[c] < D[(size_t)Ls * cols + (size_t)bj])) bj = j;
    }
    if (bj < 0) {
      r[7] = 1;
      free(D);
      free(dir);
      continue;
    }
    r[0] = D[(size_t)Ls * cols + (size_t)bj];
    r[2] = bj;
    /* traceback, collecting moves in reverse */
    int i = Ls, j = bj, nm = 0;
    char* mv = (char*)malloc((size_t)(Ls + Lt + 2));
    int mm = 0, gs = 0, gt = 0;
    while (i > 0) {
      const uint8_t d = dir[(size_t)i * cols + (size_t)j];
      if (d == DIR_DIAG) {
        if (sbase(sr, (uint32_t)Ls, (uint32_t)(i - 1), rc) != base_at(tr, (uint64_t)(j - 1))) ++mm;
        mv[nm++] = 'M';
        --i;
        --j;
      } else if (d == DIR_HORZ) {
        mv[nm++] = 'S';  /* T base against a gap in S */
        ++gs;
        --j;
      } else {
        mv[nm++] = 'T';  /* S base against a gap in T */
        ++gt;
        --i;
      }
    }
    r[1] = j;
    r[3] = mm;
    r[4] = gs;
    r[5] = gt;
    /* blocks, forward order: each run of aligned columns closes a block
     * (gap before it, run length); optimal paths never put opposite gaps
     * side by side (one mismatch, 2, beats two gaps, 6), so a gap is a
     * signed count; trailing gaps form a final (gap, 0) block. */
    uint32_t nb = 0;
    int gap = 0, len = 0, over = 0;
    for (int q = nm - 1; q >= 0; --q) {
      const char c = mv[q];
      if (c == 'M') {
        ++len;
        continue;
      }
      if (len > 0) {
        if (blocks && nb < max_blocks) {
          blocks[2 * ((size_t)k * max_blocks + nb)] = gap;
          blocks[2 * ((size_t)k * max_blocks + nb) + 1] = len;
        } else if (blocks) {
          over = 1;
        }
        ++nb;
        gap = 0;
        len = 0;
      }
      gap += c == 'S' ? 1 : -1;
    }
    if (len > 0 || gap != 0 || nb == 0) {
      if (blocks && nb < max_blocks) {
        blocks[2 * ((size_t)k * max_blocks + nb)] = gap;
        blocks[2 * ((size_t)k * max_blocks + nb) + 1] = len;
      } else if (blocks) {
        over = 1;
      }
      ++nb;
    }
    r[6] = (int32_t)nb;
    r[7] = over ? 2 : 0;
    free(mv);
    free(D);
    free(dir);
  }
}

/* Column consensus of reads placed gap-free on targets.  Each placed base
 * votes its quality for its base at target column (offset + i); per column
 * the base with the largest vote sum wins, ties go to the target's own base,
 * then to the smaller base code; Q = min(60, winner sum - best other sum).
 * Columns without votes keep the target base with Q = 0. */
void ora_consensus(const uint64_t* r_base_off, const uint64_t* r_byte_off, const uint8_t* r_packed,
                   const uint8_t* r_quals, const uint64_t* t_base_off, const uint64_t* t_byte_off,
                   const uint8_t* t_packed, uint64_t n_targets, const uint32_t* plc, uint64_t n, uint8_t* cons,
                   uint8_t* cq) {
  const uint64_t NT = t_base_off[n_targets];
  uint64_t* votes = (uint64_t*)calloc((size_t)NT * 4 + 4, sizeof(uint64_t));
  for (uint64_t k = 0; k < n; ++k) {
    const uint32_t r = plc[4 * k], t = plc[4 * k + 1], flags = plc[4 * k + 3];
    const int32_t off = (int32_t)plc[4 * k + 2];
    const uint32_t L = (uint32_t)(r_base_off[r + 1] - r_base_off[r]);
    const uint32_t Lt = (uint32_t)(t_base_off[t + 1] - t_base_off[t]);
    const uint8_t* rd = r_packed + r_byte_off[r];
    const uint8_t* q = r_quals + r_base_off[r];
    for (uint32_t i = 0; i < L; ++i) {
      const int64_t j = (int64_t)off + i;
      if (j < 0 || j >= (int64_t)Lt) continue;
      votes[(t_base_off[t] + (uint64_t)j) * 4 + (uint64_t)sbase(rd, L, i, flags & 1)] +=
          (uint64_t)squal(q, L, i, flags & 1);
    }
  }
  for (uint64_t t = 0; t < n_targets; ++t) {
    const uint64_t L = t_base_off[t + 1] - t_base_off[t];
    for (uint64_t j = 0; j < L; ++j) {
      const uint64_t col = t_base_off[t] + j;
      const int tb = base_at(t_packed + t_byte_off[t], j);
      const uint64_t* v = votes + col * 4;
      int win = tb;
      for (int b = 0; b < 4; ++b)
        if (v[b] > v[win] || (v[b] == v[win] && b != tb && win != tb && b < win)) win = b;
      uint64_t other = 0;
      for (int b = 0; b < 4; ++b)
        if (b != win && v[b] > other) other = v[b];
      const uint64_t dq = v[win] - other;
      cons[col] = (uint8_t)win;
      cq[col] = (uint8_t)(dq > 60 ? 60 : dq);
    }
  }
  free(votes);
}
