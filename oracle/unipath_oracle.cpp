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

Key mask_key(Key k) {
  const int bits = 2 * g_K;
  if (bits < 192) {
    if (bits <= 64) {
      k.a = 0;
      k.b = 0;
      k.c &= bits == 64 ? ~0ull : ((1ull << bits) - 1);
    } else if (bits <= 128) {
      k.a = 0;
      k.b &= bits == 128 ? ~0ull : ((1ull << (bits - 64)) - 1);
    } else {
      k.a &= (1ull << (bits - 128)) - 1;
    }
  }
  return k;
}

Key push_right(Key k, uint64_t base) {  // (k << 2 | base) & mask
  Key r;
  r.a = (k.a << 2) | (k.b >> 62);
  r.b = (k.b << 2) | (k.c >> 62);
  r.c = (k.c << 2) | base;
  return mask_key(r);
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
};

std::vector<Node> g_nodes;

int64_t find_node(const Key& k) {
  size_t lo = 0, hi = g_nodes.size();
  while (lo < hi) {
    size_t mid = (lo + hi) / 2;
    if (g_nodes[mid].key < k)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo < g_nodes.size() && g_nodes[lo].key == k ? (int64_t)lo : -1;
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
  g_K = K;
  std::memset(out, 0, sizeof(*out));
  // ---- 1. instances -> nodes with extension bits -------------------------
  struct Inst {
    Key key;
    uint8_t left, right;
  };
  std::vector<uint64_t> ioff(n_reads + 1, 0);
  for (uint64_t r = 0; r < n_reads; ++r) {
    const uint64_t L = base_off[r + 1] - base_off[r];
    ioff[r + 1] = ioff[r] + (L >= (uint64_t)K ? L - K + 1 : 0);
  }
  std::vector<Inst> inst(ioff[n_reads]);
#pragma omp parallel for schedule(dynamic, 1024)
  for (uint64_t r = 0; r < n_reads; ++r) {
    const uint64_t L = base_off[r + 1] - base_off[r];
    const uint8_t* rd = packed + byte_off[r];
    if (L < (uint64_t)K) continue;
    Key f{0, 0, 0};
    for (uint64_t i = 0; i < (uint64_t)K - 1; ++i) f = push_right(f, read_base(rd, i));
    for (uint64_t i = 0; i + K <= L; ++i) {
      f = push_right(f, read_base(rd, i + K - 1));
      const Key rc = revcomp(f);
      const int a = i > 0 ? read_base(rd, i - 1) : -1;
      const int b = i + K < L ? read_base(rd, i + K) : -1;
      const uint8_t la = a >= 0 ? 1 << a : 0, rb = b >= 0 ? 1 << b : 0;
      const uint8_t ca = a >= 0 ? 1 << (3 - a) : 0, cb = b >= 0 ? 1 << (3 - b) : 0;
      Inst x;
      if (f == rc) {
        x = {f, (uint8_t)(la | cb), (uint8_t)(rb | ca)};
      } else if (f < rc) {
        x = {f, la, rb};
      } else {
        x = {rc, cb, ca};
      }
      inst[ioff[r] + i] = x;
    }
  }
  __gnu_parallel::sort(inst.begin(), inst.end(), [](const Inst& x, const Inst& y) { return x.key < y.key; });
  g_nodes.clear();
  for (size_t i = 0; i < inst.size();) {
    Node n{inst[i].key, 0, 0, 0};
    size_t j = i;
    for (; j < inst.size() && inst[j].key == inst[i].key; ++j) {
      n.left |= inst[j].left;
      n.right |= inst[j].right;
      n.count++;
    }
    g_nodes.push_back(n);
    i = j;
  }
  std::vector<Inst>().swap(inst);
  return build_graph(n_reads, base_off, byte_off, packed, K, out);
}

// Graph of an explicit node set (keys: 3 limbs each, ext: left | right << 4)
// plus KmerPaths of the given reads — the multi-GPU path's "gathered nodes".
int oru_graph_from_nodes(uint64_t n_nodes, const uint64_t* keys, const uint8_t* ext, uint64_t n_reads,
                         const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed, int K,
                         oru_result* out) {
  if (K < 1 || K > 96 || !out) return -1;
  g_K = K;
  std::memset(out, 0, sizeof(*out));
  g_nodes.clear();
  for (uint64_t i = 0; i < n_nodes; ++i)
    g_nodes.push_back(Node{Key{keys[3 * i], keys[3 * i + 1], keys[3 * i + 2]}, (uint8_t)(ext[i] & 15),
                           (uint8_t)(ext[i] >> 4), 0});
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
  g_K = K;
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
  // ---- 3. cut cycles ------------------------------------------------------
  {
    std::vector<char> onpath(D, 0);
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
  // ---- 4. paths -> unipath pairs ------------------------------------------
  struct PathRec {
    int64_t head, tail;
    uint64_t len;
  };
  std::vector<PathRec> paths;
  std::vector<int64_t> path_of(D, -1), rank_of(D, -1);
  for (int64_t v = 0; v < D; ++v) {
    if (prv[v] >= 0) continue;
    PathRec p{v, v, 0};
    for (int64_t x = v; x >= 0; x = nxt[x]) {
      path_of[x] = (int64_t)paths.size();
      rank_of[x] = (int64_t)p.len++;
      p.tail = x;
    }
    paths.push_back(p);
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
  std::vector<uint8_t> ub(ub_off[U]);
  for (uint64_t i = 0; i < U; ++i) {
    uint64_t o = ub_off[i];
    const int64_t h = paths[order[i]].head;
    const Key hs = seq(h);
    for (int t = 0; t < K - 1; ++t) ub[o++] = (uint8_t)get_base(hs, t);
    for (int64_t x = h; x >= 0; x = nxt[x]) ub[o++] = (uint8_t)get_base(seq(x), K - 1);
  }
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
  // ---- 6. read paths ---------------------------------------------------------
  // per read: its id intervals (runs of consecutive ids), then concatenated
  std::vector<uint64_t> poff(n_reads + 1, 0), pst, pln;
  std::vector<std::vector<uint64_t>> rst(n_reads), rln(n_reads);
  int miss = 0;
#pragma omp parallel for schedule(dynamic, 1024)
  for (uint64_t r = 0; r < n_reads; ++r) {
    const uint64_t L = base_off[r + 1] - base_off[r];
    const uint8_t* rd = packed + byte_off[r];
    if (L < (uint64_t)K) continue;
    Key f{0, 0, 0};
    for (uint64_t i = 0; i < (uint64_t)K - 1; ++i) f = push_right(f, read_base(rd, i));
    for (uint64_t i = 0; i + K <= L; ++i) {
      f = push_right(f, read_base(rd, i + K - 1));
      const int64_t v = directed_of(f);
      if (v < 0) {
#pragma omp atomic write
        miss = 1;
        break;
      }
      const uint64_t id = base[uni_of_path[path_of[v]]] + (uint64_t)rank_of[v];
      if (!rst[r].empty() && rst[r].back() + rln[r].back() == id)
        rln[r].back()++;
      else {
        rst[r].push_back(id);
        rln[r].push_back(1);
      }
    }
  }
  if (miss) return -4;
  for (uint64_t r = 0; r < n_reads; ++r) {
    pst.insert(pst.end(), rst[r].begin(), rst[r].end());
    pln.insert(pln.end(), rln[r].begin(), rln[r].end());
    poff[r + 1] = pst.size();
    std::vector<uint64_t>().swap(rst[r]);
    std::vector<uint64_t>().swap(rln[r]);
  }
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
