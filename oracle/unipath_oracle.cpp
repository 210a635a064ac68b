// oracle/unipath_oracle.cpp — CPU restatement of the K <= 96 unipath builder
// (ReadsToPaths + MakeRcDb + Unipather + unipath adjacency / HyperKmerPath),
// following SURVEY.md §A.5-A.6 as made operational in DESIGN.md §Unipaths.
// TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench cpu_baseline).
//
// PARITY UNPINNED: reference snapshot empty.  Recalled grep
// targets: [R:M] src/paths/ReadsToPathsCoreX.cc, src/paths/Unipath.cc,
// src/paths/KmerPath.h, src/paths/HyperKmerPath.h, src/paths/KmerBaseBroker.h.
//
// Deliberately simple: sort + binary search, sequential walks; the
// independent per-read and per-node loops (instances, links, read paths) and
// the instance sort run on the OpenMP threads given.
//   nodes      canonical K-mers of the reads; ext bits = read-supported
//              neighbour bases (left/right of the canonical orientation)
//   directed   v = 2*node + o (o = 1: reverse complement); seq(v)
//   links      v -> w iff out(v) = {b} and w = seq(v)[1..]+b has in(w) = 1,
//              neither node palindromic
//   cycles     cut once per (C, rc C) pair before the min-seq node m:
//              edges prev(m)->m and rc(m)->rc(prev(m)) are removed
//   unipaths   paths; pair key = min(seq(head), seq(rc(tail))); pairs sorted
//              by key, emitted as u (smaller head) then rc(u) (palindromic
//              paths once); k-mer ids contiguous in emitted order
//   HKP        vertices = union of (end of u) and (start of v) over every
//              graph edge tail(u) -> head(v); numbered by smallest
//              (2*unipath + end) member; edge i = unipath i
#include <omp.h>
#include <parallel/algorithm>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <vector>
#include <cstdio>

static double oru_t0 = 0;
static void oru_phase(const char* what) {
  if (!std::getenv("ORU_VERBOSE")) return;
  const double t = omp_get_wtime();
  std::fprintf(stderr, "[oru] %-12s %8.2f s\n", what, oru_t0 ? t - oru_t0 : 0.0);
  oru_t0 = t;
}

namespace {

struct Key {
  uint64_t a, b, c;  // big-endian limbs of the 2K-bit value
  bool operator<(const Key& o) const {
    if (a != o.a) return a < o.a;
    if (b != o.b) return b < o.b;
    return c < o.c;
  }
  bool operator==(const Key& o) const { return a == o.a && b == o.b && c == o.c; }
};

int g_K;
uint64_t g_ma, g_mb, g_mc;  // per-limb masks of the 2K-bit value (set_k)

void set_k(int K) {
  g_K = K;
  const int bits = 2 * K;
  auto lm = [](int n) { return n >= 64 ? ~0ull : n <= 0 ? 0ull : ((1ull << n) - 1); };
  g_mc = lm(bits);
  g_mb = lm(bits - 64);
  g_ma = lm(bits - 128);
}

Key mask_key(Key k) {
  k.a &= g_ma;
  k.b &= g_mb;
  k.c &= g_mc;
  return k;
}

Key push_right(Key k, uint64_t base) {  // (k << 2 | base) & mask
  Key r;
  r.a = ((k.a << 2) | (k.b >> 62)) & g_ma;
  r.b = ((k.b << 2) | (k.c >> 62)) & g_mb;
  r.c = ((k.c << 2) | base) & g_mc;
  return r;
}

uint64_t get_base(const Key& k, int i) {  // base i (0 = first) of the K-mer
  const int bit = 2 * (g_K - 1 - i);
  const uint64_t limb = bit >= 128 ? k.a : bit >= 64 ? k.b : k.c;
  return (limb >> (bit & 63)) & 3;
}

// Reverse complement of the K-mer: the 192-bit value's 2-bit groups reversed
// (limbs swapped, each limb's groups reversed), complemented, then shifted
// down by the 192 - 2K unused bits.
uint64_t rev2_limb(uint64_t x) {
  x = ((x >> 2) & 0x3333333333333333ull) | ((x & 0x3333333333333333ull) << 2);
  x = ((x >> 4) & 0x0f0f0f0f0f0f0f0full) | ((x & 0x0f0f0f0f0f0f0f0full) << 4);
  return __builtin_bswap64(x);
}
Key revcomp(const Key& k) {
  uint64_t a = ~rev2_limb(k.c), b = ~rev2_limb(k.b), c = ~rev2_limb(k.a);  // full 192-bit reversal
  const int sh = 192 - 2 * g_K;  // drop the low `sh` bits (the unused high bases, now at the bottom)
  const int q = sh / 64, r = sh % 64;
  uint64_t l[3] = {a, b, c};  // l[0] most significant
  uint64_t o[3] = {0, 0, 0};
  for (int i = 2; i >= 0; --i) {  // o = l >> sh (192-bit)
    const int src = i - q;
    if (src < 0) continue;
    uint64_t v = r ? (l[src] >> r) : l[src];
    if (r && src - 1 >= 0) v |= l[src - 1] << (64 - r);
    o[i] = v;
  }
  return mask_key(Key{o[0], o[1], o[2]});
}

int read_base(const uint8_t* rd, uint64_t i) { return (rd[i >> 2] >> (2 * (i & 3))) & 3; }

struct Node {
  Key key;
  uint8_t left, right;  // ext bit sets (bit b = base b)
  uint64_t count;
  uint64_t id[2];  // K-mer id of each orientation (set once the unipaths are numbered)
};

std::vector<Node> g_nodes;

// Node lookup: an open-addressing index over g_nodes (load <= 0.5, linear
// probing) keyed by a mix of the key's limbs — O(1) where a binary search over
// a C2-size node array (64 M) made the read paths dominate the oracle's time.
std::vector<int64_t> g_index;
uint64_t g_index_mask = 0;

uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
uint64_t key_mix(const Key& k) {
  return mix64(k.a * 0x9e3779b97f4a7c15ull ^ k.b * 0xc2b2ae3d27d4eb4full ^ (k.c + 0x165667b19e3779f9ull));
}

void build_index() {
  uint64_t T = 2;
  while (T < 2 * (uint64_t)g_nodes.size()) T <<= 1;
  g_index.assign(T, -1);
  g_index_mask = T - 1;
  const int64_t N = (int64_t)g_nodes.size();
  int64_t* tab = g_index.data();
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < N; ++i) {
    for (uint64_t h = key_mix(g_nodes[i].key) & g_index_mask;; h = (h + 1) & g_index_mask) {
      int64_t expect = -1;
      if (__atomic_compare_exchange_n(&tab[h], &expect, i, false, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) break;
    }
  }
}

int64_t find_node(const Key& k) {
  for (uint64_t h = key_mix(k) & g_index_mask;; h = (h + 1) & g_index_mask) {
    const int64_t i = g_index[h];
    if (i < 0) return -1;
    if (g_nodes[i].key == k) return i;
  }
}

// Rolling reverse complement: rc of (window << 2 | b) = rc >> 2 with the
// complement of b as the first (most significant) base.
Key push_left_rc(Key r, uint64_t b) {
  Key o;
  o.c = (r.c >> 2) | (r.b << 62);
  o.b = (r.b >> 2) | (r.a << 62);
  o.a = r.a >> 2;
  const int bit = 2 * (g_K - 1);
  const uint64_t v = (3 - b) << (bit & 63);
  if (bit >= 128)
    o.a |= v;
  else if (bit >= 64)
    o.b |= v;
  else
    o.c |= v;
  return o;
}

Key seq(int64_t v) {
  const Key& k = g_nodes[v >> 1].key;
  return (v & 1) ? revcomp(k) : k;
}
bool palin(int64_t node) { return revcomp(g_nodes[node].key) == g_nodes[node].key; }
uint8_t comp_set(uint8_t s) {
  uint8_t r = 0;
  for (int b = 0; b < 4; ++b)
    if (s & (1 << b)) r |= 1 << (3 - b);
  return r;
}
uint8_t out_set(int64_t v) { return (v & 1) ? comp_set(g_nodes[v >> 1].left) : g_nodes[v >> 1].right; }
uint8_t in_set(int64_t v) { return (v & 1) ? comp_set(g_nodes[v >> 1].right) : g_nodes[v >> 1].left; }
int64_t directed_of(const Key& s) {  // directed node whose sequence is s
  const Key r = revcomp(s);
  const bool fw = !(r < s);  // canonical = min(s, rc s); palindrome -> o = 0
  const int64_t n = find_node(fw ? s : r);
  if (n < 0) return -1;
  return 2 * n + (fw ? 0 : 1);
}
int64_t succ_by(int64_t v, int b) {  // directed successor of v through base b
  const Key s = seq(v);
  Key t = push_right(s, (uint64_t)b);
  return directed_of(t);
}
int popc(uint8_t x) { return __builtin_popcount(x); }

}  // namespace

extern "C" {

typedef struct oru_result {
  uint64_t n_nodes;
  uint64_t n_unipaths;
  uint64_t* len;       // [n_unipaths]
  uint64_t* id_base;   // [n_unipaths]
  uint64_t* rc;        // [n_unipaths]
  uint64_t* ub_off;    // [n_unipaths + 1]
  uint8_t* unibases;   // [ub_off[n_unipaths]] base codes
  uint64_t n_vertices;
  uint64_t* from;      // [n_unipaths]
  uint64_t* to;        // [n_unipaths]
  uint64_t n_reads;
  uint64_t* path_off;  // [n_reads + 1]
  uint64_t n_intervals;
  uint64_t* path_start;  // [n_intervals]
  uint64_t* path_len;    // [n_intervals]
} oru_result;

}  // extern "C"

template <typename T>
static T* dup(const std::vector<T>& v) {
  T* p = (T*)std::malloc(std::max<size_t>(1, v.size()) * sizeof(T));
  if (!v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
  return p;
}

static int build_graph(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed,
                       int K, oru_result* out);

extern "C" {

int oru_build(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed, int K,
              oru_result* out) {
  if (K < 1 || K > 96 || !out) return -1;
  set_k(K);
  std::memset(out, 0, sizeof(*out));
  // ---- 1. instances -> nodes with extension bits -------------------------
  // In hash parcels of the canonical key (the reference's KmerParcels idea,
  // here only to bound the checker's memory: a C2-size input has 1.6 G
  // instances): each pass re-rolls every read, keeps the instances of its
  // parcel, sorts them and folds equal keys into nodes.
  struct Inst {
    Key key;
    uint32_t h;  // low bits of key_mix(key): the bucket table's slot
    uint8_t left, right;
  };
  uint64_t n_inst = 0;
  for (uint64_t r = 0; r < n_reads; ++r) {
    const uint64_t L = base_off[r + 1] - base_off[r];
    n_inst += L >= (uint64_t)K ? L - K + 1 : 0;
  }
  // ORU_PARCEL_INSTANCES (tests): a smaller parcel, so that small inputs take several passes
  uint64_t per_parcel = 1ull << 28;
  if (const char* e = std::getenv("ORU_PARCEL_INSTANCES")) per_parcel = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));
  const uint64_t parcels = std::max<uint64_t>(1, (n_inst + per_parcel - 1) / per_parcel);
  oru_phase("start");
  g_nodes.clear();
  const int nt = omp_get_max_threads();
  constexpr int kBuckets = 256;  // by the top 8 bits of key_mix: each folded by one thread in its own table
  for (uint64_t pc = 0; pc < parcels; ++pc) {
    std::vector<std::vector<Inst>> part((size_t)nt * kBuckets);
#pragma omp parallel
    {
      std::vector<Inst>* mine = &part[(size_t)omp_get_thread_num() * kBuckets];
#pragma omp for schedule(dynamic, 1024)
      for (uint64_t r = 0; r < n_reads; ++r) {
        const uint64_t L = base_off[r + 1] - base_off[r];
        const uint8_t* rd = packed + byte_off[r];
        if (L < (uint64_t)K) continue;
        Key f{0, 0, 0}, rc{0, 0, 0};
        for (uint64_t i = 0; i < (uint64_t)K - 1; ++i) {
          f = push_right(f, read_base(rd, i));
          rc = push_left_rc(rc, read_base(rd, i));
        }
        for (uint64_t i = 0; i + K <= L; ++i) {
          f = push_right(f, read_base(rd, i + K - 1));
          rc = push_left_rc(rc, read_base(rd, i + K - 1));
          const Key& canon = rc < f ? rc : f;
          const uint64_t h = key_mix(canon);
          if (parcels > 1 && (h >> 20) % parcels != pc) continue;
          const int a = i > 0 ? read_base(rd, i - 1) : -1;
          const int b = i + K < L ? read_base(rd, i + K) : -1;
          const uint8_t la = a >= 0 ? 1 << a : 0, rb = b >= 0 ? 1 << b : 0;
          const uint8_t ca = a >= 0 ? 1 << (3 - a) : 0, cb = b >= 0 ? 1 << (3 - b) : 0;
          Inst x;
          if (f == rc) {
            x = {f, (uint32_t)h, (uint8_t)(la | cb), (uint8_t)(rb | ca)};
          } else if (f < rc) {
            x = {f, (uint32_t)h, la, rb};
          } else {
            x = {rc, (uint32_t)h, cb, ca};
          }
          mine[h >> 56].push_back(x);
        }
      }
    }
    oru_phase("  extract");
    // fold equal keys: per bucket an open-addressing table over its nodes
    std::vector<std::vector<Node>> bn(kBuckets);
#pragma omp parallel for schedule(dynamic, 1)
    for (int bk = 0; bk < kBuckets; ++bk) {
      size_t cnt = 0;
      for (int t = 0; t < nt; ++t) cnt += part[(size_t)t * kBuckets + bk].size();
      uint64_t T = 16;
      while (T < 2 * cnt) T <<= 1;
      std::vector<int64_t> tab(T, -1);
      std::vector<Node>& nodes = bn[bk];
      for (int t = 0; t < nt; ++t) {
        std::vector<Inst>& v = part[(size_t)t * kBuckets + bk];
        for (const Inst& x : v) {
          for (uint64_t sl = x.h & (T - 1);; sl = (sl + 1) & (T - 1)) {
            const int64_t i = tab[sl];
            if (i < 0) {
              tab[sl] = (int64_t)nodes.size();
              nodes.push_back(Node{x.key, x.left, x.right, 1, {0, 0}});
              break;
            }
            Node& n = nodes[i];
            if (n.key == x.key) {
              n.left |= x.left;
              n.right |= x.right;
              n.count++;
              break;
            }
          }
        }
        std::vector<Inst>().swap(v);
      }
    }
    oru_phase("  fold");
    for (auto& v : bn) g_nodes.insert(g_nodes.end(), v.begin(), v.end());
  }
  __gnu_parallel::sort(g_nodes.begin(), g_nodes.end(), [](const Node& x, const Node& y) { return x.key < y.key; });
  oru_phase("nodes");
  return build_graph(n_reads, base_off, byte_off, packed, K, out);
}

// Graph of an explicit node set (keys: 3 limbs each, ext: left | right << 4)
// plus KmerPaths of the given reads — the multi-GPU path's "gathered nodes".
int oru_graph_from_nodes(uint64_t n_nodes, const uint64_t* keys, const uint8_t* ext, uint64_t n_reads,
                         const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed, int K,
                         oru_result* out) {
  if (K < 1 || K > 96 || !out) return -1;
  set_k(K);
  std::memset(out, 0, sizeof(*out));
  g_nodes.clear();
  for (uint64_t i = 0; i < n_nodes; ++i)
    g_nodes.push_back(Node{Key{keys[3 * i], keys[3 * i + 1], keys[3 * i + 2]}, (uint8_t)(ext[i] & 15),
                           (uint8_t)(ext[i] >> 4), 0, {0, 0}});
  std::sort(g_nodes.begin(), g_nodes.end(), [](const Node& x, const Node& y) { return x.key < y.key; });
  out->n_nodes = n_nodes;
  return build_graph(n_reads, base_off, byte_off, packed, K, out);
}

static uint64_t fmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

// Every K-mer instance of the reads: canonical key limbs, instance extension
// bits (left | right << 4) and the 56-bit partition hash of the key (same
// function as the GPU's key_hash: shard = top bits).  Returns the count;
// outputs may be NULL to size.
uint64_t oru_instances(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed,
                       int K, uint64_t* keys, uint8_t* ext, uint64_t* hash) {
  set_k(K);
  uint64_t n = 0;
  for (uint64_t r = 0; r < n_reads; ++r) {
    const uint64_t L = base_off[r + 1] - base_off[r];
    const uint8_t* rd = packed + byte_off[r];
    if (L < (uint64_t)K) continue;
    Key f{0, 0, 0};
    for (uint64_t i = 0; i < (uint64_t)K - 1; ++i) f = push_right(f, read_base(rd, i));
    for (uint64_t i = 0; i + K <= L; ++i, ++n) {
      f = push_right(f, read_base(rd, i + K - 1));
      if (!keys) continue;
      const Key rc = revcomp(f);
      const int a = i > 0 ? read_base(rd, i - 1) : -1;
      const int b = i + K < L ? read_base(rd, i + K) : -1;
      const uint8_t la = a >= 0 ? 1 << a : 0, rb = b >= 0 ? 1 << b : 0;
      const uint8_t ca = a >= 0 ? 1 << (3 - a) : 0, cb = b >= 0 ? 1 << (3 - b) : 0;
      Key k;
      uint8_t L4, R4;
      if (f == rc) {
        k = f, L4 = la | cb, R4 = rb | ca;
      } else if (f < rc) {
        k = f, L4 = la, R4 = rb;
      } else {
        k = rc, L4 = cb, R4 = ca;
      }
      keys[3 * n] = k.a;
      keys[3 * n + 1] = k.b;
      keys[3 * n + 2] = k.c;
      ext[n] = (uint8_t)(L4 | (R4 << 4));
      hash[n] = fmix64(k.a ^ fmix64(k.b ^ fmix64(k.c ^ 0x5851f42d4c957f2dull))) & ~0xffull;
    }
  }
  return n;
}

}  // extern "C"

static int build_graph(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed,
                       int K, oru_result* out) {
  const int64_t N = (int64_t)g_nodes.size(), D = 2 * N;
  out->n_nodes = (uint64_t)N;
  build_index();
  oru_phase("index");
  // ---- 2. unique links --------------------------------------------------
  std::vector<int64_t> nxt(D, -1), prv(D, -1);
  int bad = 0;
#pragma omp parallel for schedule(dynamic, 4096)
  for (int64_t v = 0; v < D; ++v) {  // w's unique predecessor alone writes prv[w]
    if (palin(v >> 1)) continue;
    const uint8_t o = out_set(v);
    if (popc(o) != 1) continue;
    const int b = __builtin_ctz(o);
    const int64_t w = succ_by(v, b);
    if (w < 0) {  // read-supported edge must land on a node
#pragma omp atomic write
      bad = 1;
      continue;
    }
    if (palin(w >> 1) || popc(in_set(w)) != 1) continue;
    nxt[v] = w;
    prv[w] = v;
  }
  if (bad) return -2;
  oru_phase("links");
  // ---- 3. cut cycles ------------------------------------------------------
  {
    std::vector<char> onpath(D, 0);  // chains from distinct heads are disjoint: no write races
#pragma omp parallel for schedule(dynamic, 4096)
    for (int64_t v = 0; v < D; ++v)
      if (prv[v] < 0)
        for (int64_t x = v; x >= 0 && !onpath[x]; x = nxt[x]) onpath[x] = 1;
    std::vector<char> done(D, 0);
    for (int64_t v = 0; v < D; ++v) {
      if (onpath[v] || done[v]) continue;
      std::vector<int64_t> cyc;
      int64_t x = v;
      do {
        cyc.push_back(x);
        x = nxt[x];
      } while (x != v);
      // the rc cycle contains rc(v) = v ^ 1
      std::vector<int64_t> rcyc;
      x = v ^ 1;
      do {
        rcyc.push_back(x);
        x = nxt[x];
      } while (x != (v ^ 1));
      int64_t m = cyc[0];
      for (int64_t y : cyc)
        if (seq(y) < seq(m)) m = y;
      for (int64_t y : rcyc)
        if (seq(y) < seq(m)) m = y;
      for (int64_t y : cyc) done[y] = 1;
      for (int64_t y : rcyc) done[y] = 1;
      const int64_t p = prv[m];
      nxt[p] = -1;
      prv[m] = -1;
      if (nxt[m ^ 1] == (p ^ 1)) {  // mirror edge rc(m) -> rc(p) (absent if it was the same edge)
        nxt[m ^ 1] = -1;
        prv[p ^ 1] = -1;
      }
    }
  }
  oru_phase("cycles");
  // ---- 4. paths -> unipath pairs ------------------------------------------
  struct PathRec {
    int64_t head, tail;
    uint64_t len;
  };
  std::vector<PathRec> paths;  // one per head, in directed-node order
  for (int64_t v = 0; v < D; ++v)
    if (prv[v] < 0) paths.push_back(PathRec{v, v, 0});
  std::vector<int64_t> path_of(D, -1), rank_of(D, -1);
#pragma omp parallel for schedule(dynamic, 1024)
  for (size_t pi = 0; pi < paths.size(); ++pi) {
    PathRec& p = paths[pi];
    for (int64_t x = p.head; x >= 0; x = nxt[x]) {
      path_of[x] = (int64_t)pi;
      rank_of[x] = (int64_t)p.len++;
      p.tail = x;
    }
  }
  struct Pair {
    Key key;
    int64_t u, r;  // path indices (r == u: palindromic)
  };
  std::vector<Pair> pairs;
  for (size_t i = 0; i < paths.size(); ++i) {
    const int64_t rp = path_of[paths[i].tail ^ 1];
    const Key hs = seq(paths[i].head), rs = seq(paths[rp].head);
    if ((int64_t)i == rp) {
      pairs.push_back({hs, (int64_t)i, (int64_t)i});
    } else if (hs < rs || (hs == rs && paths[i].head < paths[rp].head)) {  // == only for a palindromic K-mer
      pairs.push_back({hs, (int64_t)i, rp});
    }
  }
  std::sort(pairs.begin(), pairs.end(), [](const Pair& x, const Pair& y) { return x.key < y.key; });
  std::vector<int64_t> order;  // emitted unipath index -> path index
  std::vector<uint64_t> rcv;
  for (const Pair& p : pairs) {
    const uint64_t i = order.size();
    order.push_back(p.u);
    if (p.r == p.u) {
      rcv.push_back(i);
    } else {
      order.push_back(p.r);
      rcv.push_back(i + 1);
      rcv.push_back(i);
    }
  }
  const uint64_t U = order.size();
  std::vector<int64_t> uni_of_path(paths.size());
  for (uint64_t i = 0; i < U; ++i) uni_of_path[order[i]] = (int64_t)i;
  std::vector<uint64_t> len(U), base(U), ub_off(U + 1, 0);
  uint64_t idb = 0;
  for (uint64_t i = 0; i < U; ++i) {
    len[i] = paths[order[i]].len;
    base[i] = idb;
    idb += len[i];
    ub_off[i + 1] = ub_off[i] + (uint64_t)K - 1 + len[i];
  }
  oru_phase("paths");
  std::vector<uint8_t> ub(ub_off[U]);
#pragma omp parallel for schedule(dynamic, 64)
  for (uint64_t i = 0; i < U; ++i) {
    uint64_t o = ub_off[i];
    const int64_t h = paths[order[i]].head;
    const Key hs = seq(h);
    for (int t = 0; t < K - 1; ++t) ub[o++] = (uint8_t)get_base(hs, t);
    for (int64_t x = h; x >= 0; x = nxt[x])  // last base of seq(x): rc's is the complement of the key's first
      ub[o++] = (uint8_t)((x & 1) ? 3 - get_base(g_nodes[x >> 1].key, 0) : get_base(g_nodes[x >> 1].key, K - 1));
  }
  oru_phase("unibases");
  // ---- 5. HyperKmerPath vertices -------------------------------------------
  std::vector<uint64_t> par(2 * U);
  for (uint64_t i = 0; i < 2 * U; ++i) par[i] = i;
  auto findp = [&](uint64_t x) {
    while (par[x] != x) {
      par[x] = par[par[x]];
      x = par[x];
    }
    return x;
  };
  for (uint64_t i = 0; i < U; ++i) {
    const int64_t t = paths[order[i]].tail;
    const uint8_t o = out_set(t);
    for (int b = 0; b < 4; ++b) {
      if (!(o & (1 << b))) continue;
      const int64_t w = succ_by(t, b);
      if (w < 0) return -3;
      const uint64_t j = (uint64_t)uni_of_path[path_of[w]];
      uint64_t x = findp(2 * i + 1), y = findp(2 * j);
      if (x != y) {
        if (x < y)
          par[y] = x;
        else
          par[x] = y;
      }
    }
  }
  std::vector<uint64_t> vid(2 * U, UINT64_MAX);
  uint64_t nv = 0;
  for (uint64_t e = 0; e < 2 * U; ++e) {  // members in increasing order: first visit = smallest
    const uint64_t r = findp(e);
    if (vid[r] == UINT64_MAX) vid[r] = nv++;
  }
  std::vector<uint64_t> from(U), to(U);
  for (uint64_t i = 0; i < U; ++i) {
    from[i] = vid[findp(2 * i)];
    to[i] = vid[findp(2 * i + 1)];
  }
  oru_phase("hkp");
  // ---- 6. read paths ---------------------------------------------------------
  // per read: its id intervals (runs of consecutive ids); two passes over the
  // reads (count, then write at the prefix-summed offsets), each K-mer looked
  // up on its own — in chunks of 64 K-mers whose index slots and then node
  // records are prefetched before they are read
#pragma omp parallel for schedule(static)
  for (int64_t v = 0; v < D; ++v) g_nodes[v >> 1].id[v & 1] = base[uni_of_path[path_of[v]]] + (uint64_t)rank_of[v];
  // one pass: each thread logs its reads' runs as (read, start id, length);
  // the runs of a read are contiguous in one thread's log
  struct Run {
    uint64_t read, start, len;
  };
  const int nthr = omp_get_max_threads();
  std::vector<std::vector<Run>> runs(nthr);
  int miss = 0;
  constexpr int kChunk = 64;
#pragma omp parallel
  {
    std::vector<Run>& log = runs[omp_get_thread_num()];
    Key ck[kChunk];
    bool fw[kChunk];
    uint64_t slot[kChunk];
    int64_t idx[kChunk];
#pragma omp for schedule(dynamic, 1024)
    for (uint64_t r = 0; r < n_reads; ++r) {
      const uint64_t L = base_off[r + 1] - base_off[r];
      const uint8_t* rd = packed + byte_off[r];
      if (L < (uint64_t)K) continue;
      Key f{0, 0, 0}, rc{0, 0, 0};
      for (uint64_t i = 0; i < (uint64_t)K - 1; ++i) {
        f = push_right(f, read_base(rd, i));
        rc = push_left_rc(rc, read_base(rd, i));
      }
      bool open = false;
      for (uint64_t i0 = 0; i0 + K <= L && !miss; i0 += kChunk) {
        const int m = (int)std::min<uint64_t>(kChunk, L - K + 1 - i0);
        for (int j = 0; j < m; ++j) {
          f = push_right(f, read_base(rd, i0 + j + K - 1));
          rc = push_left_rc(rc, read_base(rd, i0 + j + K - 1));
          fw[j] = !(rc < f);  // canonical = min(s, rc s); palindrome -> o = 0
          ck[j] = fw[j] ? f : rc;
          slot[j] = key_mix(ck[j]) & g_index_mask;
          __builtin_prefetch(&g_index[slot[j]]);
        }
        for (int j = 0; j < m; ++j) {
          idx[j] = g_index[slot[j]];
          if (idx[j] >= 0) __builtin_prefetch(&g_nodes[idx[j]]);
        }
        for (int j = 0; j < m; ++j) {
          int64_t nd = idx[j];
          if (nd >= 0 && !(g_nodes[nd].key == ck[j])) nd = find_node(ck[j]);
          if (nd < 0) {
#pragma omp atomic write
            miss = 1;
            break;
          }
          const uint64_t id = g_nodes[nd].id[fw[j] ? 0 : 1];
          if (open && log.back().start + log.back().len == id)
            log.back().len++;
          else
            log.push_back(Run{r, id, 1});
          open = true;
        }
      }
    }
  }
  if (miss) return -4;
  std::vector<uint64_t> poff(n_reads + 1, 0);
#pragma omp parallel for schedule(static, 1)
  for (int t = 0; t < nthr; ++t)
    for (const Run& x : runs[t]) poff[x.read + 1]++;
  for (uint64_t r = 0; r < n_reads; ++r) poff[r + 1] += poff[r];
  std::vector<uint64_t> pst(poff[n_reads]), pln(poff[n_reads]);
#pragma omp parallel for schedule(static, 1)
  for (int t = 0; t < nthr; ++t) {
    uint64_t prev = UINT64_MAX, o = 0;
    for (const Run& x : runs[t]) {
      if (x.read != prev) o = poff[x.read], prev = x.read;
      pst[o] = x.start;
      pln[o++] = x.len;
    }
    std::vector<Run>().swap(runs[t]);
  }
  oru_phase("read paths");
  oru_phase("concat");
  out->n_unipaths = U;
  out->len = dup(len);
  out->id_base = dup(base);
  out->rc = dup(rcv);
  out->ub_off = dup(ub_off);
  out->unibases = dup(ub);
  out->n_vertices = nv;
  out->from = dup(from);
  out->to = dup(to);
  out->n_reads = n_reads;
  out->path_off = dup(poff);
  out->n_intervals = pst.size();
  out->path_start = dup(pst);
  out->path_len = dup(pln);
  g_nodes.clear();
  g_nodes.shrink_to_fit();
  return 0;
}

extern "C" {

void oru_free(oru_result* r) {
  if (!r) return;
  std::free(r->len);
  std::free(r->id_base);
  std::free(r->rc);
  std::free(r->ub_off);
  std::free(r->unibases);
  std::free(r->from);
  std::free(r->to);
  std::free(r->path_off);
  std::free(r->path_start);
  std::free(r->path_len);
  std::memset(r, 0, sizeof(*r));
}

}  // extern "C"
