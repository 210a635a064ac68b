/*
 * fill_walk_model.c — a CPU model of k_fill's gap walk (fill.hip) that counts
 * its extension-table lookups by kind, for sizing FillFragments changes
 * before they reach the GPU.  Not a checker: tests/ compare the kernel with
 * oracle/fill_oracle.c.
 *
 * Input (tools/fill_walk_model.py writes both):
 *   solid.bin: u64 n, then n canonical K-mers (2-bit, MSB-first)
 *   reads.bin: u64 n_reads, u32 L, then n_reads x L base codes (pairs 2i, 2i+1)
 * Per pair, as the kernel: both reads solid, the overlap closures, then the
 * depth-first walk (bases A<C<G<T, max_steps expansions, gmax deep) with one
 * lookup per node, per closure-bridge K-mer and per re-read branch point at
 * depth >= 32 (shallower ones come from the kernel's register cache).
 * Reports: statuses, node / bridge / backtrack lookups per status, and the
 * bridge lookups left by the two-base backward filter (fill.hip `bk`) plus
 * its own 1 + |P1| lookups per walking pair.
 *
 * gcc -O2 -o fill_walk_model fill_walk_model.c
 * ./fill_walk_model K solid.bin reads.bin [min_insert max_insert max_steps]
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t* tk;
static uint8_t* tv;
static uint64_t tmask, m1;
static int n1;

static uint64_t mix(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdull;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ull;
  return x ^ (x >> 33);
}
static uint64_t rcb(uint64_t w, int n) {
  uint64_t r = 0;
  for (int i = 0; i < n; i++, w >>= 2) r = (r << 2) | (3 - (w & 3));
  return r;
}
static uint32_t rev4(uint32_t x) { return ((x & 1) << 3) | ((x & 2) << 1) | ((x & 4) >> 1) | ((x & 8) >> 3); }
/* slot of canonical (K-1)-mer c: bits 0-3 predecessors, 4-7 successors (c's orientation) */
static uint8_t* slot(uint64_t c, int ins) {
  for (uint64_t g = mix(c) & tmask;; g = (g + 1) & tmask) {
    if (tk[g] == ~0ull) {
      if (!ins) return NULL;
      tk[g] = c;
      tv[g] = 0;
      return &tv[g];
    }
    if (tk[g] == c) return &tv[g];
  }
}
static uint32_t succ(uint64_t w) {
  const uint64_t r = rcb(w, n1);
  const uint8_t* s = slot(w < r ? w : r, 0);
  const uint32_t e = s ? *s : 0;
  uint32_t m = 0;
  if (w <= r) m |= e >> 4;
  if (r <= w) m |= rev4(e & 15);
  return m;
}
static uint32_t pred(uint64_t w) { return rev4(succ(rcb(w, n1))); }

static int rd(void* p, size_t sz, size_t n, FILE* f) { return fread(p, sz, n, f) == n; }

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s K solid.bin reads.bin [min_insert max_insert max_steps]\n", argv[0]);
    return 2;
  }
  const int K = atoi(argv[1]);
  const uint32_t min_ins = argc > 4 ? atoi(argv[4]) : 126, max_ins = argc > 5 ? atoi(argv[5]) : 234,
                 max_steps = argc > 6 ? atoi(argv[6]) : 1024;
  n1 = K - 1;
  m1 = (1ull << (2 * n1)) - 1;
  FILE* f = fopen(argv[2], "rb");
  uint64_t ns = 0;
  if (!f || !rd(&ns, 8, 1, f)) return 1;
  uint64_t* sol = malloc(ns * 8 + 8);
  if (!rd(sol, 8, ns, f)) return 1;
  fclose(f);
  uint64_t cap = 1;
  while (cap < ns * 4) cap <<= 1;
  tmask = cap - 1;
  tk = malloc(cap * 8);
  tv = malloc(cap);
  memset(tk, 0xff, cap * 8);
  for (uint64_t i = 0; i < ns; i++)
    for (int o = 0; o < 2; o++) {  /* both orientations: first K-1 bases get a successor, last K-1 a predecessor */
      const uint64_t y = o ? rcb(sol[i], K) : sol[i];
      const uint64_t a = y >> 2, b = y & m1, ra = rcb(a, n1), rb = rcb(b, n1);
      const uint32_t last = y & 3, first = (y >> (2 * n1)) & 3;
      uint8_t* s = slot(a < ra ? a : ra, 1);
      *s |= a <= ra ? 1u << (4 + last) : 1u << (3 - last);
      s = slot(b < rb ? b : rb, 1);
      *s |= b <= rb ? 1u << first : 1u << (4 + 3 - first);
    }
  f = fopen(argv[3], "rb");
  uint64_t nr = 0;
  uint32_t L = 0;
  if (!f || !rd(&nr, 8, 1, f) || !rd(&L, 4, 1, f) || L > 255) return 1;
  uint8_t* reads = malloc(nr * L);
  if (!rd(reads, 1, nr * L, f)) return 1;
  fclose(f);

  uint64_t st[4] = {0}, look[4][3] = {{0}}, filt_pre = 0, filt_bridge = 0, vis_tot[4] = {0}, vis_dist[4] = {0};
  /* per-pair caches keyed by position: node windows by depth (1-way, 2-way
     most-recent-first), bridge K-mer j's window by j */
  uint64_t hit_n1 = 0, hit_n2 = 0, hit_b = 0, hit_bf = 0;
  /* two-level slots: a lookup also returns the successor mask of a node's
     unique successor, so the node after a looked-up non-branching one (walk
     child or next bridge K-mer) costs no lookup */
  uint64_t two_node = 0, two_bridge = 0, two_bridge_f = 0;
  for (uint64_t p = 0; p < nr / 2; p++) {
    const uint8_t *A = reads + 2 * p * L, *B = reads + (2 * p + 1) * L;
    uint8_t F[256];
    for (uint32_t t = 0; t < L; t++) F[t] = 3 - B[L - 1 - t];
    int clean = 1;
    for (uint32_t j = 0; j + K <= L && clean; j++) {
      uint64_t w = 0, v = 0;
      for (int t = 0; t < n1; t++) w = (w << 2) | A[j + t], v = (v << 2) | F[j + t];
      clean = ((succ(w) >> A[j + n1]) & 1) && ((succ(v) >> F[j + n1]) & 1);
    }
    if (!clean) {
      st[1]++;
      continue;
    }
    const uint32_t lo = min_ins > L ? min_ins : L;
    uint32_t nclos = 0;
    for (uint32_t I = lo; I <= max_ins && I < 2 * L && nclos < 2; I++) {
      const uint32_t o = 2 * L - I;
      int ok = 1;
      for (uint32_t t = 0; t < o && ok; t++) ok = A[L - o + t] == F[t];
      if (ok && o + 2 <= (uint32_t)K) {
        uint64_t w = 0;
        for (int t = 0; t < n1; t++) w = (w << 2) | A[L - n1 + t];
        for (uint32_t jj = 0; jj + o + 2 <= (uint32_t)K && ok; jj++) {
          ok = (succ(w) >> F[o + jj]) & 1;
          w = ((w << 2) | F[o + jj]) & m1;
        }
      }
      nclos += ok;
    }
    if (nclos >= 2 || max_ins < 2 * L) {
      st[nclos >= 2 ? 2 : nclos ? 0 : 1]++;
      continue;
    }
    const uint32_t gmax = max_ins - 2 * L, dlo = lo > 2 * L ? lo - 2 * L : 0;
    /* the backward filter: bk bit c2*4 + c1 when c2 c1 ++ G's bridge K-mers are solid */
    uint64_t G = 0;
    for (int t = 0; t < n1; t++) G = (G << 2) | F[t];
    uint32_t bk = 0;
    const uint32_t P1 = pred(G);
    filt_pre++;
    for (uint32_t c1 = 0; c1 < 4; c1++)
      if ((P1 >> c1) & 1) {
        const uint32_t P2 = pred(((uint64_t)c1 << (2 * (n1 - 1))) | (G >> 2));
        filt_pre++;
        for (uint32_t c2 = 0; c2 < 4; c2++)
          if ((P2 >> c2) & 1) bk |= 1u << (c2 * 4 + c1);
      }
    uint64_t atail = 0;
    for (int t = 0; t < n1; t++) atail = (atail << 2) | A[L - n1 + t];
    uint8_t path[64];
    uint32_t mask[64], nextb[64], steps = 0, d = 0;
    int phys[64], known = 0;
    uint64_t ln = 0, lb = 0, lk = 0;
    uint64_t ck[64][2], cb[32];
    for (int t = 0; t < 64; t++) ck[t][0] = ck[t][1] = ~0ull;
    for (int t = 0; t < 32; t++) cb[t] = ~0ull;
    int budget = 0, stop = 0;
    /* distinct walk states (depth, window) of this pair: what a memoised
       walk would look up (duplicates share their subtree) */
    static uint64_t vs_k[4096];
    memset(vs_k, 0xff, sizeof vs_k);
    uint64_t nvis = 0, ndist = 0;
    for (;;) {  /* visit node (path[0, d)) */
      uint64_t w = atail;
      for (uint32_t t = 0; t < d; t++) w = ((w << 2) | path[t]) & m1;
      const uint32_t m = succ(w);
      ln++;
      {
        const uint64_t key = (w << 6) | d;
        nvis++;
        for (uint64_t g = mix(key) & 4095;; g = (g + 1) & 4095) {
          if (vs_k[g] == key) break;
          if (vs_k[g] == ~0ull) {
            vs_k[g] = key;
            ndist++;
            break;
          }
        }
      }
      phys[d] = !known;
      two_node += !known;
      known = 0;
      if (ck[d][0] == w) hit_n1++, hit_n2++;
      else {
        if (ck[d][1] == w) hit_n2++;
        ck[d][1] = ck[d][0];
        ck[d][0] = w;
      }
      mask[d] = m;
      if (d >= dlo && ((m >> F[0]) & 1)) {
        int ok = 1;
        uint64_t ww = ((w << 2) | F[0]) & m1;
        int bknown = phys[d] && __builtin_popcount(m) == 1, bphys = 0;
        for (int j = 1; j < n1 && ok; j++) {
          const uint32_t sj = succ(ww);
          bphys = !bknown;
          two_bridge += bphys;
          if (((bk >> (w & 15)) & 1) && j < n1 - 2) two_bridge_f += bphys;
          bknown = bphys && __builtin_popcount(sj) == 1;
          ok = (succ(ww) >> F[j]) & 1;
          lb++;
          if (cb[j] == ww) {
            hit_b++;
            if (((bk >> (w & 15)) & 1) && j < n1 - 2) hit_bf++;
          }
          cb[j] = ww;
          if (((bk >> (w & 15)) & 1) && j < n1 - 2) filt_bridge++;
          ww = ((ww << 2) | F[j]) & m1;
        }
        if (ok && ++nclos >= 2) break;
      }
      int down = 0;
      if (d < gmax) {
        if (++steps > max_steps) {
          budget = 1;
          break;
        }
        if (m) {
          known = phys[d] && __builtin_popcount(m) == 1;
          path[d] = __builtin_ctz(m);
          nextb[d] = path[d] + 1;
          d++;
          down = 1;
        }
      }
      if (down) continue;
      for (;;) {  /* backtrack to the deepest open branch point */
        if (d == 0) {
          stop = 1;
          break;
        }
        d--;
        const uint32_t rest = mask[d] >> nextb[d];
        if (rest) {
          lk += d >= 32;
          known = 0;
          path[d] = nextb[d] + __builtin_ctz(rest);
          nextb[d] = path[d] + 1;
          d++;
          break;
        }
      }
      if (stop) break;
    }
    const int s = nclos >= 2 ? 2 : budget ? 3 : nclos ? 0 : 1;
    st[s]++;
    vis_tot[s] += nvis, vis_dist[s] += ndist;
    look[s][0] += ln, look[s][1] += lb, look[s][2] += lk;
  }
  static const char* nm[4] = {"filled", "none", "ambiguous", "budget"};
  for (int s = 0; s < 4; s++)
    printf("%-9s node visits %11llu, distinct (depth, window) states %11llu\n", nm[s],
           (unsigned long long)vis_tot[s], (unsigned long long)vis_dist[s]);
  uint64_t tot = 0, br = 0;
  for (int s = 0; s < 4; s++) {
    printf("%-9s pairs %10llu  walk lookups: node %11llu bridge %11llu backtrack %9llu\n", nm[s],
           (unsigned long long)st[s], (unsigned long long)look[s][0], (unsigned long long)look[s][1],
           (unsigned long long)look[s][2]);
    tot += look[s][0] + look[s][1] + look[s][2];
    br += look[s][1];
  }
  printf("walk lookups %llu, bridge %llu (%.1f %%); with the backward filter: bridge %llu + filter %llu "
         "-> %.1f %% fewer walk lookups\n",
         (unsigned long long)tot, (unsigned long long)br, 100.0 * br / (tot ? tot : 1),
         (unsigned long long)filt_bridge, (unsigned long long)filt_pre,
         100.0 * ((double)br - filt_bridge - filt_pre) / (tot ? tot : 1));
  printf("two-level slots: node lookups %llu of %llu, bridge %llu of %llu (filtered: %llu of %llu)\n",
         (unsigned long long)two_node, (unsigned long long)(tot - br), (unsigned long long)two_bridge,
         (unsigned long long)br, (unsigned long long)two_bridge_f, (unsigned long long)filt_bridge);
  printf("position caches: node by depth 1-way %llu (%.1f %% of node lookups), 2-way %llu (%.1f %%); "
         "bridge by j %llu (%.1f %% of bridge lookups; %llu of the filtered ones)\n",
         (unsigned long long)hit_n1, 100.0 * hit_n1 / (tot - br), (unsigned long long)hit_n2,
         100.0 * hit_n2 / (tot - br), (unsigned long long)hit_b, 100.0 * hit_b / (br ? br : 1),
         (unsigned long long)hit_bf);
  return 0;
}
