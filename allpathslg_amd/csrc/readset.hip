// readset.hip — device read-set assembly: ALLPATHS-LG's "all_reads", the
// K=96 CommonPather input built from several libraries, without a host round
// trip.
//
// [R:M] RunAllPathsLG builds the unipath graph from all_reads = the filled
// fragments (FillFragments) + the corrected, trimmed jump reads
// (ErrorCorrectJump), SURVEY.md §3(1) and §8f #3.  Reference snapshot empty
// (SURVEY §0.1): no file:line exists to cite.
//
// apg_reads_concat_dev: read i of input set s becomes output read
// off_s + i (off_s = reads of the earlier sets), its bases truncated to
// keep_s[i] when a keep vector is given (ErrorCorrectJump's all-solid prefix
// lengths).  Reads are never dropped, so read ids stay aligned with the
// inputs (a trimmed-away jump read is an empty read).  Bases past the kept
// length inside the last byte are cleared, so the output is byte-identical to
// a host-built set of the truncated reads.
//
//   k_cat_len   thread per read: kept length and packed byte count
//   scan        -> base_off / byte_off of the output (u64, scan_u32_u64)
//   k_cat_copy  16 lanes per read: whole bytes, the last byte masked;
//               qualities (when every input has them) 16 lanes per read
#include <atomic>
#include <cstring>
#include <new>

#include "apg_core.hpp"
#include "kmer_common.hpp"
#include "partition.hpp"

namespace apg {

// ---------------------------------------------------------------------------
// Read-set shape on the device (uploads and .fastb/.qualb loads): the offset
// tables are validated and summarised by one kernel instead of a host loop
// over every read (40 M reads: 0.35 s of host time per load in round 2).
//   k_shape  thread per read: monotone base_off, length < 2^32, byte stride
//            >= ceil(len / 4) (given byte_off) or ceil(len / 4) into nby (to
//            be scanned into byte_off), the qualb offsets equal base_off,
//            longest read, and the shape hash = n + sum_i fmix(len_i, stride_i,
//            i) (wrapping; order-sensitive through i) that apg_reads_copy_dev
//            compares instead of the tables.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t rs_fmix(uint64_t z) {
  z ^= z >> 33;
  z *= 0xff51afd7ed558ccdull;
  z ^= z >> 33;
  z *= 0xc4ceb9fe1a85ec53ull;
  z ^= z >> 33;
  return z;
}

__global__ void k_shape(const uint64_t* __restrict__ bo, const uint64_t* __restrict__ yo,
                        const uint64_t* __restrict__ qo, uint64_t n, uint32_t* __restrict__ nby,
                        unsigned long long* __restrict__ out) {
  unsigned long long bad = 0, badq = 0, h = 0, mx = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t a = bo[i], b = bo[i + 1];
    if (b < a || b - a >= (1ull << 32)) {
      ++bad;
      continue;
    }
    const uint64_t len = b - a, need = (len + 3) / 4;
    uint64_t stride = need;
    if (yo) {
      const uint64_t ya = yo[i], yb = yo[i + 1];
      if (yb < ya || yb - ya < need) ++bad;
      stride = yb - ya;
    } else {
      nby[i] = (uint32_t)need;
    }
    if (qo && qo[i + 1] != b) ++badq;
    mx = len > mx ? len : mx;
    h += rs_fmix(len ^ (stride << 40) ^ (i * 0x9e3779b97f4a7c15ull));
  }
  wave_add(&out[0], bad);
  wave_add(&out[1], badq);
  wave_add(&out[2], h);
  for (int o = 32; o > 0; o >>= 1) {
    const unsigned long long y = (unsigned long long)__shfl_xor((long long)mx, o, 64);
    mx = y > mx ? y : mx;
  }
  if ((threadIdx.x & 63) == 0 && mx) atomicMax(&out[3], mx);
}

int dreads_device_shape(apg_ctx* ctx, apg_dreads* d, const uint64_t* d_qoff, bool compute_bytes, const char* who) {
  const uint64_t n = d->n_reads;
  unsigned long long* out = nullptr;
  uint32_t* nby = nullptr;
  APG_TRY(workspace_t(ctx, "rs_shape", 4, &out));
  if (compute_bytes) APG_TRY(workspace_t(ctx, "rs_nby", std::max<uint64_t>(n, 1), &nby));
  APG_CHECK_HIP(hipMemsetAsync(out, 0, 32, ctx->stream));
  kbegin(ctx, "read_shape", (n + 1) * (compute_bytes ? 8 : 16) + (d_qoff ? (n + 1) * 8 : 0) + (compute_bytes ? n * 4 : 0));
  if (n)
    k_shape<<<grid_for(ctx, n), 256, 0, ctx->stream>>>(d->d_base_off, compute_bytes ? nullptr : d->d_byte_off, d_qoff,
                                                        n, nby, out);
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  if (compute_bytes) APG_TRY(scan_u32_u64(ctx, nby, n, d->d_byte_off, "rs"));
  unsigned long long h[4];
  uint64_t ends[4];
  APG_CHECK_HIP(hipMemcpyAsync(h, out, 32, hipMemcpyDeviceToHost, ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(&ends[0], d->d_base_off, 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(&ends[1], d->d_base_off + n, 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(&ends[2], d->d_byte_off, 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(d2h_sync(ctx, &ends[3], d->d_byte_off + n, 8));
  if (ends[0] != 0 || ends[2] != 0) {
    set_error(std::string(who) + ": offset tables must start at 0");
    return APG_E_ARG;
  }
  if (h[0]) {
    set_error(std::string(who) + ": " + std::to_string(h[0]) +
              " reads with non-monotone offsets, a length >= 2^32 or a byte stride below ceil(len/4)");
    return APG_E_ARG;
  }
  if (h[1]) {
    set_error(std::string(who) + ": qualb/fastb length mismatch (" + std::to_string(h[1]) + " reads)");
    return APG_E_IO;
  }
  d->n_bases = ends[1];
  d->n_bytes = ends[3];
  d->max_len = h[3];
  d->shape_hash = (h[2] ^ (n * 0x100000001b3ull)) | 1;
  return APG_OK;
}

__global__ void k_cat_len(const uint64_t* __restrict__ base_off, const uint32_t* __restrict__ keep, uint64_t n,
                          uint32_t* __restrict__ lens, uint32_t* __restrict__ nby) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t L = (uint32_t)(base_off[i + 1] - base_off[i]);
    if (keep && keep[i] < L) L = keep[i];
    lens[i] = L;
    nby[i] = (L + 3) / 4;
  }
}

constexpr uint32_t kCatLanes = 16;

// Input read i -> output read j0 + i: packed bytes (and qualities) copied by
// a 16-lane group; out_boff / out_yoff hold the output offsets (scanned).
__global__ void __launch_bounds__(256) k_cat_copy(const uint64_t* __restrict__ base_off,
                                                  const uint64_t* __restrict__ byte_off,
                                                  const uint8_t* __restrict__ packed, const uint8_t* __restrict__ quals,
                                                  const uint32_t* __restrict__ lens, uint64_t n, uint64_t j0,
                                                  const uint64_t* __restrict__ out_boff,
                                                  const uint64_t* __restrict__ out_yoff, uint8_t* __restrict__ out,
                                                  uint8_t* __restrict__ out_q) {
  const uint32_t lane = threadIdx.x % kCatLanes;
  const uint64_t groups = (uint64_t)gridDim.x * (blockDim.x / kCatLanes);
  for (uint64_t i = (uint64_t)blockIdx.x * (blockDim.x / kCatLanes) + threadIdx.x / kCatLanes; i < n; i += groups) {
    const uint32_t L = lens[i];
    if (!L) continue;
    const uint8_t* src = packed + byte_off[i];
    uint8_t* dst = out + out_yoff[j0 + i];
    const uint32_t nb = (L + 3) / 4;
    for (uint32_t y = lane; y < nb; y += kCatLanes) {
      uint8_t v = src[y];
      if (y == nb - 1 && (L & 3)) v &= (uint8_t)((1u << (2 * (L & 3))) - 1);
      dst[y] = v;
    }
    if (out_q) {
      const uint8_t* qs = quals + base_off[i];
      uint8_t* qd = out_q + out_boff[j0 + i];
      for (uint32_t t = lane; t < L; t += kCatLanes) qd[t] = qs[t];
    }
  }
}

}  // namespace apg

using namespace apg;

extern "C" {

int apg_reads_concat_dev(apg_ctx* ctx, const apg_dreads* const* sets, const uint32_t* const* d_keep,
                         uint32_t n_sets, apg_dreads** out) {
  APG_REQUIRE(ctx && out && (sets || n_sets == 0), "apg_reads_concat_dev: NULL argument");
  apg_dreads* d = *out;
  APG_REQUIRE(!d || (d->ctx == ctx && d->concat_owned),
              "apg_reads_concat_dev: *out must be NULL or a previous apg_reads_concat_dev output of ctx");
  uint64_t n = 0, max_len = 0;
  bool quals = n_sets > 0;
  for (uint32_t s = 0; s < n_sets; ++s) {
    APG_REQUIRE(sets[s], "apg_reads_concat_dev: NULL read set");
    APG_REQUIRE(sets[s] != d, "apg_reads_concat_dev: the output cannot also be an input");
    n += sets[s]->n_reads;
    max_len = std::max(max_len, sets[s]->max_len);
    quals = quals && sets[s]->d_quals;
    APG_TRY(dreads_quals_ready(sets[s]));
  }
  uint64_t len_bytes = 0;  // cat_len: offsets read, keep read, two u32 per read written
  for (uint32_t s = 0; s < n_sets; ++s)
    len_bytes += (sets[s]->n_reads + 1) * 8 + (d_keep && d_keep[s] ? sets[s]->n_reads * 4 : 0) + sets[s]->n_reads * 8;
  APG_CHECK_HIP(hipSetDevice(ctx->device));
  const uint64_t nc = std::max<uint64_t>(n, 1);
  uint32_t *lens = nullptr, *nby = nullptr;
  uint64_t *bscan = nullptr, *yscan = nullptr;
  APG_TRY(workspace_t(ctx, "cat_lens", nc, &lens));
  APG_TRY(workspace_t(ctx, "cat_nby", nc, &nby));
  APG_TRY(workspace_t(ctx, "cat_bscan", nc + 1, &bscan));
  APG_TRY(workspace_t(ctx, "cat_yscan", nc + 1, &yscan));
  kbegin(ctx, "cat_len", len_bytes);
  for (uint64_t s = 0, j0 = 0; s < n_sets; j0 += sets[s]->n_reads, ++s) {
    const apg_dreads* r = sets[s];
    const uint32_t* keep = d_keep ? d_keep[s] : nullptr;
    if (r->n_reads)
      k_cat_len<<<grid_for(ctx, r->n_reads), 256, 0, ctx->stream>>>(r->d_base_off, keep, r->n_reads, lens + j0,
                                                                     nby + j0);
  }
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  APG_TRY(scan_u32_u64(ctx, lens, n, bscan, "cat_b"));
  APG_TRY(scan_u32_u64(ctx, nby, n, yscan, "cat_y"));
  uint64_t tot[2];
  APG_CHECK_HIP(hipMemcpyAsync(&tot[0], bscan + n, 8, hipMemcpyDeviceToHost, ctx->stream));
  APG_TRY(d2h_sync(ctx, &tot[1], yscan + n, 8));
  const uint64_t nbases = tot[0], nbytes = tot[1];

  // output buffers (grow-only when an earlier output is passed back)
  if (!d) {
    d = new (std::nothrow) apg_dreads();
    if (!d) return APG_E_NOMEM;
    d->ctx = ctx;
    d->device = ctx->device;
    d->concat_owned = true;
    *out = d;
  }
  if (d->cap_reads < n + 1) {
    if (d->d_base_off) APG_CHECK_HIP(hipFree(d->d_base_off));
    if (d->d_byte_off) APG_CHECK_HIP(hipFree(d->d_byte_off));
    d->d_base_off = d->d_byte_off = nullptr;
    d->cap_reads = 0;
    const uint64_t c = n + 1 + (n + 1) / 8;
    APG_CHECK_HIP(hipMalloc(&d->d_base_off, c * 8));
    APG_CHECK_HIP(hipMalloc(&d->d_byte_off, c * 8));
    d->cap_reads = c;
  }
  if (d->cap_bytes < nbytes + 64) {
    if (d->d_packed) APG_CHECK_HIP(hipFree(d->d_packed));
    d->d_packed = nullptr;
    d->cap_bytes = 0;
    const uint64_t c = nbytes + nbytes / 8 + 64;
    APG_CHECK_HIP(hipMalloc(&d->d_packed, c));
    d->cap_bytes = c;
  }
  if (quals && d->cap_quals < nbases + 64) {
    if (d->d_quals) APG_CHECK_HIP(hipFree(d->d_quals));
    d->d_quals = nullptr;
    d->cap_quals = 0;
    const uint64_t c = nbases + nbases / 8 + 64;
    APG_CHECK_HIP(hipMalloc(&d->d_quals, c));
    d->cap_quals = c;
  }
  if (!quals && d->d_quals) {  // this output has no qualities
    APG_CHECK_HIP(hipFree(d->d_quals));
    d->d_quals = nullptr;
    d->cap_quals = 0;
  }
  static std::atomic<uint64_t> g_cat{5ull << 60};
  d->gen = g_cat.fetch_add(1);  // new contents: per-read-set plans are stale
  d->n_reads = n;
  d->n_bases = nbases;
  d->n_bytes = nbytes;
  d->max_len = max_len;
  d->shape_hash = 0;

  APG_CHECK_HIP(hipMemcpyAsync(d->d_base_off, bscan, (n + 1) * 8, hipMemcpyDeviceToDevice, ctx->stream));
  APG_CHECK_HIP(hipMemcpyAsync(d->d_byte_off, yscan, (n + 1) * 8, hipMemcpyDeviceToDevice, ctx->stream));
  // bytes: kept bases (and qualities) read once and written once, lengths and
  // offsets read
  kbegin(ctx, "cat_copy", 2 * nbytes + (quals ? 2 * nbases : 0) + n * 4 + (n + 1) * 32);
  uint64_t j0 = 0;
  for (uint32_t s = 0; s < n_sets; ++s) {
    const apg_dreads* r = sets[s];
    if (r->n_reads)
      k_cat_copy<<<grid_for(ctx, r->n_reads, 256 / kCatLanes), 256, 0, ctx->stream>>>(
          r->d_base_off, r->d_byte_off, r->d_packed, quals ? r->d_quals : nullptr, lens + j0, r->n_reads, j0, bscan,
          yscan, d->d_packed, quals ? d->d_quals : nullptr);
    j0 += r->n_reads;
  }
  kend(ctx);
  APG_CHECK_HIP(hipGetLastError());
  APG_CHECK_HIP(hipMemsetAsync(d->d_packed + nbytes, 0, 64, ctx->stream));
  return sync(ctx);
}

}  // extern "C"
