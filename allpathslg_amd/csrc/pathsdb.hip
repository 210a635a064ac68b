// pathsdb.hip — MakeRcDb on MI355X: reverse-complement read paths and the
// sorted interval index over forward + reverse-complement paths.
//
// Replaces MakeRcDb ([R:M] tagged_rpint; writes <reads>.paths_rc.kN and
// <reads>.pathsdb.kN; reference snapshot empty).  Spec (pinned in
// include/apg.h): a read's rc path is its forward path walked backwards with
// every id mapped into the rc partner unipath (offset o of unipath u <->
// offset len(u)-1-o of rc(u)), consecutive ids merged into intervals; the
// index lists every interval of every forward path (read order, interval
// order) then every interval of every rc path, stably sorted by start id.
// CPU restatement: oracle.make_rc_db (numpy).
//
//   rc_count / rc_write   one thread per read; pieces of an interval are
//                         found by binary search of the unipath id bases
//   db entries            (start, payload = entry index) -> stable LSD radix
//                         sort on the significant bits of start (8-bit digits,
//                         wave-match multisplit, tile order kept) -> gather
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "apg_core.hpp"
#include "kmer_common.hpp"
#include "partition.hpp"

namespace apg {

constexpr int kRsThreads = 256;
constexpr int kRsTile = 4096;

__global__ void __launch_bounds__(kRsThreads) k_rs_count(const uint64_t* __restrict__ key, uint64_t n, int shift,
                                                         uint32_t* __restrict__ cmat) {
  __shared__ uint32_t hist[256];
  const uint32_t G = gridDim.x, b = blockIdx.x;
  hist[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t s = (uint64_t)b * kRsTile, e = min(n, s + kRsTile);
  for (uint64_t i = s + threadIdx.x; i < e; i += kRsThreads) atomicAdd(&hist[(key[i] >> shift) & 255], 1u);
  __syncthreads();
  cmat[(uint64_t)threadIdx.x * G + b] = hist[threadIdx.x];
}

// Stable scatter of one 8-bit digit: waves own consecutive 64-record rows of
// the tile, so (tile, wave, lane) order = input order.
__global__ void __launch_bounds__(kRsThreads) k_rs_scatter(const uint64_t* __restrict__ key,
                                                           const uint32_t* __restrict__ val, uint64_t n, int shift,
                                                           const uint64_t* __restrict__ omat,
                                                           uint64_t* __restrict__ okey, uint32_t* __restrict__ oval) {
  constexpr int nw = kRsThreads / 64;
  __shared__ uint32_t wh[nw][256];
  __shared__ unsigned long long base[256];
  const uint32_t G = gridDim.x, b = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t s = (uint64_t)b * kRsTile, e = min(n, s + kRsTile);
  const uint32_t tn = (uint32_t)(e - s);
  base[threadIdx.x] = omat[(uint64_t)threadIdx.x * G + b];
  for (int d = lane; d < 256; d += 64) wh[w][d] = 0;
  const uint32_t rows = (tn + 63) / 64, rpw = (rows + nw - 1) / nw;
  const uint32_t r0 = min(rows, w * rpw), r1 = min(rows, r0 + rpw);
  const uint64_t lt = (1ull << lane) - 1;
  for (uint32_t r = r0; r < r1; ++r) {
    const uint32_t idx = r * 64 + lane;
    const bool valid = idx < tn;
    const uint32_t d = valid ? (uint32_t)((key[s + idx] >> shift) & 255) : 0;
    const uint64_t peers = wave_match(d, valid, 8);
    if (valid && (peers & lt) == 0) wh[w][d] += __popcll(peers);
  }
  __syncthreads();
  {
    const uint32_t d = threadIdx.x;
    uint32_t run = 0;
    for (int k = 0; k < nw; ++k) {
      const uint32_t x = wh[k][d];
      wh[k][d] = run;
      run += x;
    }
  }
  __syncthreads();
  for (uint32_t r = r0; r < r1; ++r) {
    const uint32_t idx = r * 64 + lane;
    const bool valid = idx < tn;
    const uint32_t d = valid ? (uint32_t)((key[s + idx] >> shift) & 255) : 0;
    const uint64_t peers = wave_match(d, valid, 8);
    if (valid) {
      const uint64_t pos = base[d] + wh[w][d] + __popcll(peers & lt);
      okey[pos] = key[s + idx];
      oval[pos] = val[s + idx];
    }
    __builtin_amdgcn_wave_barrier();
    if (valid && (peers & lt) == 0) wh[w][d] += __popcll(peers);  // this row's records of digit d
    __builtin_amdgcn_wave_barrier();
  }
}

__global__ void k_rs_or(const uint64_t* __restrict__ key, uint64_t n, unsigned long long* __restrict__ orv) {
  unsigned long long o = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    o |= key[i];
  for (int off = 32; off > 0; off >>= 1) o |= (unsigned long long)__shfl_down((long long)o, off, 64);
  if ((threadIdx.x & 63) == 0 && o) atomicOr(orv, o);
}

// Stable sort of (key, val) by key: ping-pongs between (k, v) and (k2, v2);
// returns which pair holds the result (false: k/v, true: k2/v2).
int sort_u64_u32(apg_ctx* ctx, uint64_t* k, uint32_t* v, uint64_t* k2, uint32_t* v2, uint64_t n, bool* in2) {
  *in2 = false;
  if (n <= 1) return APG_OK;
  unsigned long long* orv = nullptr;
  APG_TRY(workspace_t(ctx, "rs_or", 1, &orv));
  APG_CHECK_HIP(hipMemsetAsync(orv, 0, 8, ctx->stream));
  k_rs_or<<<grid_for(ctx, n), 256, 0, ctx->stream>>>(k, n, orv);
  unsigned long long bits = 0;
  APG_TRY(d2h_sync(ctx, &bits, orv, 8));
  int nbits = 0;
  while (nbits < 64 && (bits >> nbits)) ++nbits;
  const uint32_t G = (uint32_t)((n + kRsTile - 1) / kRsTile);
  uint32_t* cmat = nullptr;
  uint64_t* omat = nullptr;
  APG_TRY(workspace_t(ctx, "rs_cmat", 256ull * G, &cmat));
  APG_TRY(workspace_t(ctx, "rs_omat", 256ull * G + 1, &omat));
  uint64_t *ak = k, *bk = k2;
  uint32_t *av = v, *bv = v2;
  for (int shift = 0; shift < nbits; shift += 8) {
    k_rs_count<<<G, kRsThreads, 0, ctx->stream>>>(ak, n, shift, cmat);
    APG_TRY(scan_u32_u64(ctx, cmat, 256ull * G, omat, "rs"));
    k_rs_scatter<<<G, kRsThreads, 0, ctx->stream>>>(ak, av, n, shift, omat, bk, bv);
    std::swap(ak, bk);
    std::swap(av, bv);
    *in2 = !*in2;
  }
  APG_CHECK_HIP(hipGetLastError());
  return APG_OK;
}

// ---------------------------------------------------------------------------
// MakeRcDb
// ---------------------------------------------------------------------------
struct UniV {
  const uint64_t* id_base;  // U (ascending)
  const uint64_t* len;
  const uint64_t* rc;
  uint64_t U;
};

__device__ __forceinline__ uint64_t unipath_of(const UniV& u, uint64_t id) {  // largest u with id_base[u] <= id
  uint64_t lo = 0, hi = u.U;
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if (u.id_base[mid] <= id)
      lo = mid;
    else
      hi = mid;
  }
  return lo;
}

template <bool WRITE>
__global__ void k_rc_paths(uint64_t n_reads, const uint64_t* __restrict__ poff, const uint64_t* __restrict__ pstart,
                           const uint64_t* __restrict__ plen, UniV uv, uint32_t* __restrict__ nrc,
                           const uint64_t* __restrict__ rcoff, uint64_t* __restrict__ rstart,
                           uint64_t* __restrict__ rlen) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_reads;
       r += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t cs = 0, cl = 0;
    uint32_t k = 0;
    const uint64_t o = WRITE ? rcoff[r] : 0;
    for (uint64_t q = poff[r + 1]; q-- > poff[r];) {
      const uint64_t s = pstart[q], e = s + plen[q];
      uint64_t x = e;  // walk the interval's pieces from its end
      while (x > s) {
        const uint64_t u = unipath_of(uv, x - 1);
        const uint64_t b = uv.id_base[u];
        const uint64_t ps = s > b ? s : b;  // piece [ps, x) inside u
        const uint64_t L = uv.len[u];
        const uint64_t ru = uv.rc[u];
        const uint64_t ns = uv.id_base[ru] + (L - (x - b));  // rc piece start
        const uint64_t nl = x - ps;
        if (cl && cs + cl == ns) {
          cl += nl;
        } else {
          if (cl && WRITE) {
            rstart[o + k - 1] = cs;
            rlen[o + k - 1] = cl;
          }
          cs = ns;
          cl = nl;
          ++k;
        }
        x = ps;
      }
    }
    if (cl && WRITE) {
      rstart[o + k - 1] = cs;
      rlen[o + k - 1] = cl;
    }
    if (!WRITE) nrc[r] = k;
  }
}

// db entry keys (start) and payloads (entry index): forward intervals first.
__global__ void k_db_keys(uint64_t NF, uint64_t NR, const uint64_t* __restrict__ fstart,
                          const uint64_t* __restrict__ rstart, uint64_t* __restrict__ key, uint32_t* __restrict__ val) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < NF + NR;
       i += (uint64_t)gridDim.x * blockDim.x) {
    key[i] = i < NF ? fstart[i] : rstart[i - NF];
    val[i] = (uint32_t)i;
  }
}

// read id and position of every interval (forward or rc)
__global__ void k_db_owner(uint64_t n_reads, const uint64_t* __restrict__ off, uint32_t* __restrict__ rd,
                           uint32_t* __restrict__ pos) {
  for (uint64_t r = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; r < n_reads;
       r += (uint64_t)gridDim.x * blockDim.x)
    for (uint64_t q = off[r]; q < off[r + 1]; ++q) {
      rd[q] = (uint32_t)r;
      pos[q] = (uint32_t)(q - off[r]);
    }
}

__global__ void k_db_gather(uint64_t N, uint64_t NF, const uint32_t* __restrict__ perm, const uint64_t* __restrict__ fs,
                            const uint64_t* __restrict__ fl, const uint64_t* __restrict__ rs,
                            const uint64_t* __restrict__ rl, const uint32_t* __restrict__ frd,
                            const uint32_t* __restrict__ fpos, const uint32_t* __restrict__ rrd,
                            const uint32_t* __restrict__ rpos, apg_rpint* __restrict__ db) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < N; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t e = perm[i];
    apg_rpint x;
    if (e < NF) {
      x.start = fs[e];
      x.len = (uint32_t)fl[e];
      x.read = frd[e];
      x.pos = fpos[e];
      x.flags = 0;
    } else {
      const uint64_t j = e - NF;
      x.start = rs[j];
      x.len = (uint32_t)rl[j];
      x.read = rrd[j];
      x.pos = rpos[j];
      x.flags = APG_RPINT_RC;
    }
    db[i] = x;
  }
}

template <typename T>
static int h2d(apg_ctx* ctx, const char* name, const T* h, uint64_t n, T** d) {
  APG_TRY(workspace_t(ctx, name, std::max<uint64_t>(n, 1), d));
  if (n) APG_CHECK_HIP(hipMemcpyAsync(*d, h, n * sizeof(T), hipMemcpyHostToDevice, ctx->stream));
  return APG_OK;
}

template <typename T>
static int d2h_alloc(apg_ctx* ctx, const T* d, uint64_t n, T** h) {
  *h = static_cast<T*>(std::malloc(std::max<uint64_t>(n, 1) * sizeof(T)));
  if (!*h) return APG_E_NOMEM;
  if (n) APG_CHECK_HIP(hipMemcpyAsync(*h, d, n * sizeof(T), hipMemcpyDeviceToHost, ctx->stream));
  return APG_OK;
}

}  // namespace apg

using namespace apg;

extern "C" {

void apg_rc_db_free(apg_rc_db* db) {
  if (!db) return;
  std::free(db->rc_path_off);
  std::free(db->rc_start);
  std::free(db->rc_len);
  std::free(db->entries);
  std::memset(db, 0, sizeof(*db));
}

int apg_make_rc_db(apg_ctx* ctx, const apg_unipath_graph* g, apg_rc_db* out) {
  APG_REQUIRE(ctx && g && out, "apg_make_rc_db: NULL argument");
  APG_REQUIRE(g->n_reads == 0 || (g->path_off && (g->n_intervals == 0 || (g->path_start && g->path_len))),
              "apg_make_rc_db: graph carries no read paths");
  APG_REQUIRE(g->n_unipaths == 0 || (g->len && g->id_base && g->rc), "apg_make_rc_db: graph has no unipaths");
  static_assert(sizeof(apg_rpint) == 24, "apg_rpint layout");
  std::memset(out, 0, sizeof(*out));
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const uint64_t R = g->n_reads, U = g->n_unipaths, NF = g->n_intervals;
  APG_REQUIRE(R == 0 || g->path_off[R] == NF, "apg_make_rc_db: path_off[n_reads] != n_intervals");
  APG_REQUIRE(NF < (1ull << 31), "apg_make_rc_db: more than 2^31 intervals");
  for (uint64_t i = 0; i < NF; ++i) {
    const uint64_t s = g->path_start[i], e = s + g->path_len[i];
    if (U == 0 || e > g->id_base[U - 1] + g->len[U - 1] || g->path_len[i] == 0) {
      set_error("apg_make_rc_db: interval outside the unipath id space");
      return APG_E_ARG;
    }
  }
  uint64_t *poff, *pstart, *plen, *ub, *ul, *urc;
  APG_TRY(h2d(ctx, "db_poff", g->path_off, R + 1, &poff));
  APG_TRY(h2d(ctx, "db_pstart", g->path_start, NF, &pstart));
  APG_TRY(h2d(ctx, "db_plen", g->path_len, NF, &plen));
  APG_TRY(h2d(ctx, "db_ub", g->id_base, U, &ub));
  APG_TRY(h2d(ctx, "db_ul", g->len, U, &ul));
  APG_TRY(h2d(ctx, "db_urc", g->rc, U, &urc));
  const UniV uv{ub, ul, urc, U};
  uint32_t* nrc = nullptr;
  uint64_t* rcoff = nullptr;
  APG_TRY(workspace_t(ctx, "db_nrc", std::max<uint64_t>(R, 1), &nrc));
  APG_TRY(workspace_t(ctx, "db_rcoff", R + 1, &rcoff));
  kbegin(ctx, "db_rc_paths", R * 16 + NF * 16 * 2);
  if (R) k_rc_paths<false><<<grid_for(ctx, R), 256, 0, ctx->stream>>>(R, poff, pstart, plen, uv, nrc, nullptr, nullptr,
                                                                       nullptr);
  APG_TRY(scan_u32_u64(ctx, nrc, R, rcoff, "db"));
  uint64_t NR = 0;
  APG_TRY(d2h_sync(ctx, &NR, rcoff + R, 8));
  uint64_t *rs = nullptr, *rl = nullptr;
  APG_TRY(workspace_t(ctx, "db_rs", std::max<uint64_t>(NR, 1), &rs));
  APG_TRY(workspace_t(ctx, "db_rl", std::max<uint64_t>(NR, 1), &rl));
  if (R) k_rc_paths<true><<<grid_for(ctx, R), 256, 0, ctx->stream>>>(R, poff, pstart, plen, uv, nullptr, rcoff, rs, rl);
  kend(ctx);
  const uint64_t N = NF + NR;
  APG_REQUIRE(N < (1ull << 32), "apg_make_rc_db: more than 2^32 index entries");
  uint64_t *k1 = nullptr, *k2 = nullptr;
  uint32_t *v1 = nullptr, *v2 = nullptr, *frd = nullptr, *fpos = nullptr, *rrd = nullptr, *rpos = nullptr;
  APG_TRY(workspace_t(ctx, "db_k1", std::max<uint64_t>(N, 1), &k1));
  APG_TRY(workspace_t(ctx, "db_k2", std::max<uint64_t>(N, 1), &k2));
  APG_TRY(workspace_t(ctx, "db_v1", std::max<uint64_t>(N, 1), &v1));
  APG_TRY(workspace_t(ctx, "db_v2", std::max<uint64_t>(N, 1), &v2));
  APG_TRY(workspace_t(ctx, "db_frd", std::max<uint64_t>(NF, 1), &frd));
  APG_TRY(workspace_t(ctx, "db_fpos", std::max<uint64_t>(NF, 1), &fpos));
  APG_TRY(workspace_t(ctx, "db_rrd", std::max<uint64_t>(NR, 1), &rrd));
  APG_TRY(workspace_t(ctx, "db_rpos", std::max<uint64_t>(NR, 1), &rpos));
  apg_rpint* db = nullptr;
  APG_TRY(workspace_t(ctx, "db_out", std::max<uint64_t>(N, 1), &db));
  kbegin(ctx, "db_sort", N * 12 * 2 * 5 + N * 24);
  if (N) {
    k_db_keys<<<grid_for(ctx, N), 256, 0, ctx->stream>>>(NF, NR, pstart, rs, k1, v1);
    if (R) {
      k_db_owner<<<grid_for(ctx, R), 256, 0, ctx->stream>>>(R, poff, frd, fpos);
      k_db_owner<<<grid_for(ctx, R), 256, 0, ctx->stream>>>(R, rcoff, rrd, rpos);
    }
    bool in2 = false;
    APG_TRY(sort_u64_u32(ctx, k1, v1, k2, v2, N, &in2));
    k_db_gather<<<grid_for(ctx, N), 256, 0, ctx->stream>>>(N, NF, in2 ? v2 : v1, pstart, plen, rs, rl, frd, fpos, rrd,
                                                           rpos, db);
  }
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  out->n_reads = R;
  out->n_rc_intervals = NR;
  out->n_entries = N;
  int rc = d2h_alloc(ctx, rcoff, R + 1, &out->rc_path_off);
  if (rc == APG_OK) rc = d2h_alloc(ctx, rs, NR, &out->rc_start);
  if (rc == APG_OK) rc = d2h_alloc(ctx, rl, NR, &out->rc_len);
  if (rc == APG_OK) rc = d2h_alloc(ctx, db, N, &out->entries);
  if (rc == APG_OK) rc = sync(ctx);
  if (rc != APG_OK) apg_rc_db_free(out);
  return rc;
}

}  // extern "C"
