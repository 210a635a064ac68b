// apg_synth.cpp — deterministic synthetic genome + paired-read simulator
// (SURVEY.md §B).  Stands in for PrepareAllPathsInputs' real data, which is not
// in the container.  Host-only; every pair is generated from its own
// xoshiro256** stream seeded by (seed, pair index), so any rank regenerates any
// slice without coordination and results do not depend on the thread count.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

#include "../../include/apg.h"

namespace {

inline uint64_t splitmix64(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

struct Xoshiro256ss {
  uint64_t s[4];
  explicit Xoshiro256ss(uint64_t seed) {
    uint64_t t = seed;
    for (auto& v : s) v = splitmix64(t);
  }
  static inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  inline uint64_t next() {
    const uint64_t r = rotl(s[1] * 5, 7) * 9;
    const uint64_t t = s[1] << 17;
    s[2] ^= s[0];
    s[3] ^= s[1];
    s[1] ^= s[2];
    s[0] ^= s[3];
    s[2] ^= t;
    s[3] = rotl(s[3], 45);
    return r;
  }
  // Uniform double in [0, 1) from the top 53 bits.
  inline double uniform() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
  // Uniform integer in [0, n) (n > 0), multiply-shift (bias < 2^-64 * n).
  inline uint64_t below(uint64_t n) { return (uint64_t)(((__uint128_t)next() * n) >> 64); }
  inline double gaussian() {
    double u1 = uniform();
    double u2 = uniform();
    if (u1 < 1e-300) u1 = 1e-300;
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
};

constexpr uint64_t kGenomeBlock = 1ull << 20;

inline uint64_t stream_seed(uint64_t seed, uint64_t salt, uint64_t idx) {
  uint64_t t = seed ^ (salt * 0xd1b54a32d192ed03ull);
  t += idx * 0x9e3779b97f4a7c15ull;
  return splitmix64(t);
}

unsigned n_threads(uint32_t want) {
  unsigned hw = std::thread::hardware_concurrency();
  if (hw == 0) hw = 4;
  unsigned t = want ? want : hw;
  return std::max(1u, std::min(t, 64u));
}

template <typename F>
void parallel_for(uint64_t n, unsigned threads, F f) {
  if (n == 0) return;
  threads = (unsigned)std::min<uint64_t>(threads, n);
  if (threads <= 1) {
    f(0, n);
    return;
  }
  std::vector<std::thread> ts;
  const uint64_t chunk = (n + threads - 1) / threads;
  for (unsigned t = 0; t < threads; ++t) {
    uint64_t a = t * chunk, b = std::min(n, a + chunk);
    if (a >= b) break;
    ts.emplace_back([=] { f(a, b); });
  }
  for (auto& th : ts) th.join();
}

struct Fragment {
  uint64_t start, len;
  bool flip;  // read A comes from the reverse strand
};

// The first draws of pair k's stream: fragment length ~ N(mean, sd) clamped to
// [L, min(G, 10*mean + L)], start, strand.  Shared by the read and the
// fragment generators so a fragment is exactly its pair's insert.
inline Fragment draw_fragment(Xoshiro256ss& rng, const apg_synth_params* p) {
  const uint64_t L = p->read_len, G = p->genome_len;
  double f = p->insert_mean + p->insert_sd * rng.gaussian();
  uint64_t flen = (uint64_t)std::llround(std::max<double>(f, (double)L));
  flen = std::min<uint64_t>(flen, std::min<uint64_t>(G, 10ull * p->insert_mean + L));
  const uint64_t start = rng.below(G - flen + 1);
  const bool flip = rng.next() & 1;
  return {start, flen, flip};
}

}  // namespace

extern "C" {

int apg_synth_genome(uint64_t genome_len, uint64_t seed, uint8_t* out) {
  if (!out && genome_len) return APG_E_ARG;
  const uint64_t nblocks = (genome_len + kGenomeBlock - 1) / kGenomeBlock;
  parallel_for(nblocks, n_threads(0), [&](uint64_t a, uint64_t b) {
    for (uint64_t blk = a; blk < b; ++blk) {
      Xoshiro256ss rng(stream_seed(seed, 1, blk));
      const uint64_t s = blk * kGenomeBlock, e = std::min(genome_len, s + kGenomeBlock);
      for (uint64_t i = s; i < e; i += 32) {
        uint64_t w = rng.next();
        for (uint64_t j = i; j < std::min(e, i + 32); ++j, w >>= 2) out[j] = (uint8_t)(w & 3);
      }
    }
  });
  return APG_OK;
}

void apg_repeat_defaults(apg_repeat_params* p) {
  if (!p) return;
  std::memset(p, 0, sizeof(*p));
  p->n_families = 3;
  const uint32_t len[3] = {300, 6000, 1000};
  const double frac[3] = {0.10, 0.05, 0.005}, div[3] = {0.12, 0.04, 0.002};
  for (int f = 0; f < 3; ++f) {
    p->family_len[f] = len[f];
    p->family_frac[f] = frac[f];
    p->family_div[f] = div[f];
  }
  p->tandem_frac = 0.01;
  p->tandem_unit_max = 60;
  p->tandem_array_max = 4000;
}

// One sequential stream (salt 2): the injection order fixes the result.
int apg_synth_repeats(uint64_t genome_len, uint64_t seed, const apg_repeat_params* p, uint8_t* g) {
  if (!p || (!g && genome_len) || p->n_families > APG_MAX_REPEAT_FAMILIES) return APG_E_ARG;
  Xoshiro256ss rng(stream_seed(seed, 2, 0));
  auto mutate = [&](uint8_t b, double rate) -> uint8_t {
    if (rate > 0 && rng.uniform() < rate) return (uint8_t)((b + 1 + rng.below(3)) & 3);
    return b;
  };
  for (uint32_t f = 0; f < p->n_families; ++f) {
    const uint64_t L = p->family_len[f];
    if (L == 0 || L > genome_len) continue;
    std::vector<uint8_t> cons(L);
    for (auto& b : cons) b = (uint8_t)(rng.next() & 3);
    const uint64_t target = (uint64_t)(p->family_frac[f] * (double)genome_len);
    for (uint64_t covered = 0; covered < target; covered += L) {
      const uint64_t at = rng.below(genome_len - L + 1);
      const bool rc = rng.next() & 1;
      for (uint64_t i = 0; i < L; ++i) {
        const uint8_t b = rc ? (uint8_t)(3 - cons[L - 1 - i]) : cons[i];
        g[at + i] = mutate(b, p->family_div[f]);
      }
    }
  }
  const uint64_t ttarget = (uint64_t)(p->tandem_frac * (double)genome_len);
  const uint32_t umax = std::max<uint32_t>(1, p->tandem_unit_max);
  const uint64_t amax = std::max<uint64_t>(2, p->tandem_array_max);
  std::vector<uint8_t> unit(umax);
  for (uint64_t covered = 0; covered < ttarget;) {
    const uint32_t u = 1 + (uint32_t)rng.below(umax);
    for (uint32_t i = 0; i < u; ++i) unit[i] = (uint8_t)(rng.next() & 3);
    const uint64_t lo = 2ull * u, hi = std::max<uint64_t>(lo, std::min<uint64_t>(amax, genome_len));
    const uint64_t len = std::min<uint64_t>(genome_len, lo + rng.below(hi - lo + 1));
    const uint64_t at = rng.below(genome_len - len + 1);
    for (uint64_t i = 0; i < len; ++i) g[at + i] = mutate(unit[i % u], 0.01);
    covered += len;
  }
  return APG_OK;
}

int apg_synth_sizes(const apg_synth_params* p, uint64_t* n_reads, uint64_t* n_bases,
                    uint64_t* n_packed_bytes) {
  if (!p) return APG_E_ARG;
  const uint64_t nr = 2 * p->n_pairs;
  if (n_reads) *n_reads = nr;
  if (n_bases) *n_bases = nr * p->read_len;
  if (n_packed_bytes) *n_packed_bytes = nr * ((p->read_len + 3) / 4);
  return APG_OK;
}

int apg_synth_reads(const apg_synth_params* p, const uint8_t* genome, uint64_t* base_off,
                    uint64_t* byte_off, uint8_t* packed, uint8_t* quals) {
  if (!p || !genome || !base_off || !byte_off || !packed) return APG_E_ARG;
  const uint64_t L = p->read_len, G = p->genome_len;
  if (L == 0 || G < L) return APG_E_ARG;
  const uint64_t rb = (L + 3) / 4;
  const uint64_t nr = 2 * p->n_pairs;
  for (uint64_t i = 0; i <= nr; ++i) {
    base_off[i] = i * L;
    byte_off[i] = i * rb;
  }
  const double lo = p->err_lo, hi = p->err_hi;
  parallel_for(p->n_pairs, n_threads(p->threads), [&](uint64_t a, uint64_t b) {
    std::vector<uint8_t> r1(L), r2(L), q1(L), q2(L);
    for (uint64_t k = a; k < b; ++k) {
      Xoshiro256ss rng(stream_seed(p->seed, 2, p->first_pair + k));
      const Fragment fr = draw_fragment(rng, p);
      const uint64_t start = fr.start, flen = fr.len;
      const bool flip = fr.flip;
      // FR pair: read A = forward of [start, start+L), read B = rc of [start+flen-L, start+flen).
      for (uint64_t i = 0; i < L; ++i) {
        r1[i] = genome[start + i];
        r2[i] = (uint8_t)(3 - genome[start + flen - 1 - i]);
      }
      if (flip) std::swap(r1, r2);
      for (int rd = 0; rd < 2; ++rd) {
        auto& r = rd ? r2 : r1;
        auto& q = rd ? q2 : q1;
        for (uint64_t i = 0; i < L; ++i) {
          const double e = L > 1 ? lo + (hi - lo) * (double)i / (double)(L - 1) : lo;
          if (rng.uniform() < e) {
            r[i] = (uint8_t)((r[i] + 1 + rng.below(3)) & 3);
            q[i] = (uint8_t)(2 + rng.below(19));
          } else {
            q[i] = 40;
          }
        }
        const uint64_t ridx = 2 * k + rd;
        uint8_t* dst = packed + ridx * rb;
        std::memset(dst, 0, rb);
        for (uint64_t i = 0; i < L; ++i) dst[i >> 2] |= (uint8_t)(r[i] << (2 * (i & 3)));
        if (quals) std::memcpy(quals + ridx * L, q.data(), L);
      }
    }
  });
  return APG_OK;
}

int apg_synth_layout(const apg_synth_params* p, uint64_t* start, uint32_t* flen, uint8_t* flip) {
  if (!p || !start || !flen || !flip) return APG_E_ARG;
  if (p->read_len == 0 || p->genome_len < p->read_len) return APG_E_ARG;
  parallel_for(p->n_pairs, n_threads(p->threads), [&](uint64_t a, uint64_t b) {
    for (uint64_t k = a; k < b; ++k) {
      Xoshiro256ss rng(stream_seed(p->seed, 2, p->first_pair + k));
      const Fragment fr = draw_fragment(rng, p);
      start[k] = fr.start;
      flen[k] = (uint32_t)fr.len;
      flip[k] = fr.flip ? 1 : 0;
    }
  });
  return APG_OK;
}

int apg_synth_fragments(const apg_synth_params* p, uint64_t* base_off, uint64_t* byte_off, const uint8_t* genome,
                        uint8_t* packed) {
  if (!p || !base_off || !byte_off) return APG_E_ARG;
  const uint64_t L = p->read_len, G = p->genome_len, n = p->n_pairs;
  if (L == 0 || G < L) return APG_E_ARG;
  if (!packed) {  // sizing pass: offsets only
    std::vector<uint64_t> len(n);
    parallel_for(n, n_threads(p->threads), [&](uint64_t a, uint64_t b) {
      for (uint64_t k = a; k < b; ++k) {
        Xoshiro256ss rng(stream_seed(p->seed, 2, p->first_pair + k));
        len[k] = draw_fragment(rng, p).len;
      }
    });
    base_off[0] = byte_off[0] = 0;
    for (uint64_t k = 0; k < n; ++k) {
      base_off[k + 1] = base_off[k] + len[k];
      byte_off[k + 1] = byte_off[k] + (len[k] + 3) / 4;
    }
    return APG_OK;
  }
  if (!genome) return APG_E_ARG;
  parallel_for(n, n_threads(p->threads), [&](uint64_t a, uint64_t b) {
    for (uint64_t k = a; k < b; ++k) {
      Xoshiro256ss rng(stream_seed(p->seed, 2, p->first_pair + k));
      const Fragment fr = draw_fragment(rng, p);
      if (fr.len != base_off[k + 1] - base_off[k]) continue;  // offsets not from the sizing pass
      uint8_t* dst = packed + byte_off[k];
      std::memset(dst, 0, (fr.len + 3) / 4);
      for (uint64_t i = 0; i < fr.len; ++i) {
        const uint8_t b = fr.flip ? (uint8_t)(3 - genome[fr.start + fr.len - 1 - i]) : genome[fr.start + i];
        dst[i >> 2] |= (uint8_t)(b << (2 * (i & 3)));
      }
    }
  });
  return APG_OK;
}

}  // extern "C"
