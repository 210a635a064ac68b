// apg_formats.cpp — read/write the on-disk read formats.
//
// "APG-fastb v0" / "APG-qualb v0" carry the same content as ALLPATHS-LG's
// feudal vecbasevector (.fastb) / vecqualvector (.qualb) ([R:M] src/feudal/,
// src/Basevector.h, src/Qualvector.h).  The feudal byte layout itself is
// unpinned (reference absent), so the header is versioned: a feudal-compatible
// v1 reader can be added without touching callers.
//
//   offset  size            field
//   0       8               magic "APGFB\0\0\0" | "APGQB\0\0\0"
//   8       4               version (0)
//   12      4               reserved (0)
//   16      8               n_reads
//   24      8               total_bases
//   32      8*(n_reads+1)   base_off (read i = bases [base_off[i], base_off[i+1]))
//   ...     payload         fastb: packed 2-bit bases, each read byte-aligned
//                           (byte_off[i] = sum_{j<i} ceil(len_j/4));
//                           qualb: one Phred byte per base
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "../../include/apg.h"

namespace apg {
void set_error(const std::string& msg);
}

namespace {

const char kFastbMagic[8] = {'A', 'P', 'G', 'F', 'B', 0, 0, 0};
const char kQualbMagic[8] = {'A', 'P', 'G', 'Q', 'B', 0, 0, 0};

struct File {
  FILE* f = nullptr;
  ~File() {
    if (f) std::fclose(f);
  }
};

int io_fail(const std::string& what) {
  apg::set_error(what);
  return APG_E_IO;
}

int write_common(const char* path, const char* magic, const apg_reads* r, const void* payload,
                 uint64_t payload_bytes) {
  if (!path || !r) return APG_E_ARG;
  const uint64_t n = r->n_reads;
  if (n && !r->base_off) return APG_E_ARG;
  const std::string tmp = std::string(path) + ".tmp";
  File fh;
  fh.f = std::fopen(tmp.c_str(), "wb");
  if (!fh.f) return io_fail("cannot open " + tmp + " for writing");
  const uint32_t ver = 0, res = 0;
  const uint64_t zero = 0;
  const uint64_t total = n ? r->base_off[n] - r->base_off[0] : 0;
  bool ok = std::fwrite(magic, 1, 8, fh.f) == 8 && std::fwrite(&ver, 4, 1, fh.f) == 1 &&
            std::fwrite(&res, 4, 1, fh.f) == 1 && std::fwrite(&n, 8, 1, fh.f) == 1 &&
            std::fwrite(&total, 8, 1, fh.f) == 1;
  if (ok) {
    if (n) {
      // Normalise so base_off[0] == 0 on disk.
      std::vector<uint64_t> bo(r->base_off, r->base_off + n + 1);
      const uint64_t b0 = bo[0];
      for (auto& v : bo) v -= b0;
      ok = std::fwrite(bo.data(), 8, n + 1, fh.f) == n + 1;
    } else {
      ok = std::fwrite(&zero, 8, 1, fh.f) == 1;
    }
  }
  if (ok && payload_bytes) ok = std::fwrite(payload, 1, payload_bytes, fh.f) == payload_bytes;
  if (!ok) return io_fail("short write to " + tmp);
  if (std::fclose(fh.f) != 0) {
    fh.f = nullptr;
    return io_fail("close failed for " + tmp);
  }
  fh.f = nullptr;
  // write-then-rename: a module killed mid-write never leaves a torn output.
  if (std::rename(tmp.c_str(), path) != 0) return io_fail("rename " + tmp + " -> " + path + " failed");
  return APG_OK;
}

int read_header(FILE* f, const char* magic, const char* path, uint64_t* n, uint64_t* total,
                std::vector<uint64_t>* base_off) {
  char m[8];
  uint32_t ver = 0, res = 0;
  if (std::fread(m, 1, 8, f) != 8 || std::memcmp(m, magic, 8) != 0)
    return io_fail(std::string("bad magic in ") + path);
  if (std::fread(&ver, 4, 1, f) != 1 || std::fread(&res, 4, 1, f) != 1 || ver != 0)
    return io_fail(std::string("unsupported version in ") + path);
  if (std::fread(n, 8, 1, f) != 1 || std::fread(total, 8, 1, f) != 1)
    return io_fail(std::string("truncated header in ") + path);
  if (*n > (1ull << 40)) return io_fail(std::string("implausible read count in ") + path);
  // the offset table must fit in the file before it is allocated: a corrupt
  // count fails here instead of in a multi-terabyte resize
  struct stat sb;
  if (fstat(fileno(f), &sb) != 0) return io_fail(std::string("cannot stat ") + path);
  if (32 + 8 * (*n + 1) > (uint64_t)sb.st_size) return io_fail(std::string("truncated offsets in ") + path);
  try {
    base_off->resize(*n + 1);
  } catch (const std::bad_alloc&) {
    return io_fail(std::string("offset table of ") + path + " does not fit in host memory");
  }
  if (std::fread(base_off->data(), 8, *n + 1, f) != *n + 1)
    return io_fail(std::string("truncated offsets in ") + path);
  // kernels index qualities by the absolute base offset: the table starts at 0
  if ((*base_off)[0] != 0) return io_fail(std::string("offset table does not start at 0 in ") + path);
  if ((*base_off)[*n] != *total) return io_fail(std::string("offset table/total mismatch in ") + path);
  for (uint64_t i = 0; i < *n; ++i)
    if ((*base_off)[i + 1] < (*base_off)[i]) return io_fail(std::string("non-monotone offsets in ") + path);
  return APG_OK;
}

}  // namespace

namespace apg {
// Header + validated offsets of an APG-fastb (qual = false) / APG-qualb file;
// *payload = the byte offset of its payload in the file (apg_load.cpp).
int fmt_read_head(const char* path, bool qual, uint64_t* n, std::vector<uint64_t>* base_off, uint64_t* payload) {
  File fh;
  fh.f = std::fopen(path, "rb");
  if (!fh.f) return io_fail(std::string("cannot open ") + path);
  uint64_t total = 0;
  const int rc = read_header(fh.f, qual ? kQualbMagic : kFastbMagic, path, n, &total, base_off);
  if (rc) return rc;
  *payload = 32 + 8 * (*n + 1);
  return APG_OK;
}
}  // namespace apg

extern "C" {

int apg_fastb_write(const char* path, const apg_reads* r) {
  if (!r) return APG_E_ARG;
  const uint64_t bytes = r->n_reads ? r->byte_off[r->n_reads] - r->byte_off[0] : 0;
  return write_common(path, kFastbMagic, r, r->n_reads ? r->packed + r->byte_off[0] : nullptr, bytes);
}

int apg_qualb_write(const char* path, const apg_reads* r) {
  if (!r) return APG_E_ARG;
  if (r->n_reads && !r->quals) return APG_E_ARG;
  const uint64_t bytes = r->n_reads ? r->base_off[r->n_reads] - r->base_off[0] : 0;
  return write_common(path, kQualbMagic, r, r->quals, bytes);
}

int apg_fastb_read(const char* path, apg_reads* out) {
  if (!path || !out) return APG_E_ARG;
  std::memset(out, 0, sizeof(*out));
  File fh;
  fh.f = std::fopen(path, "rb");
  if (!fh.f) return io_fail(std::string("cannot open ") + path);
  uint64_t n = 0, total = 0;
  std::vector<uint64_t> bo;
  int rc = read_header(fh.f, kFastbMagic, path, &n, &total, &bo);
  if (rc) return rc;
  auto* base_off = (uint64_t*)std::malloc((n + 1) * 8);
  auto* byte_off = (uint64_t*)std::malloc((n + 1) * 8);
  if (!base_off || !byte_off) {
    std::free(base_off);
    std::free(byte_off);
    return APG_E_NOMEM;
  }
  std::memcpy(base_off, bo.data(), (n + 1) * 8);
  apg_byte_offsets(base_off, n, byte_off);
  const uint64_t bytes = byte_off[n];
  auto* packed = (uint8_t*)std::malloc(bytes + 64);
  if (!packed) {
    std::free(base_off);
    std::free(byte_off);
    return APG_E_NOMEM;
  }
  if (bytes && std::fread(packed, 1, bytes, fh.f) != bytes) {
    std::free(base_off);
    std::free(byte_off);
    std::free(packed);
    return io_fail(std::string("truncated payload in ") + path);
  }
  std::memset(packed + bytes, 0, 64);
  out->n_reads = n;
  out->base_off = base_off;
  out->byte_off = byte_off;
  out->packed = packed;
  out->quals = nullptr;
  return APG_OK;
}

int apg_qualb_read(const char* path, apg_reads* io) {
  if (!path || !io) return APG_E_ARG;
  File fh;
  fh.f = std::fopen(path, "rb");
  if (!fh.f) return io_fail(std::string("cannot open ") + path);
  uint64_t n = 0, total = 0;
  std::vector<uint64_t> bo;
  int rc = read_header(fh.f, kQualbMagic, path, &n, &total, &bo);
  if (rc) return rc;
  if (io->base_off) {
    if (io->n_reads != n) return io_fail(std::string("qualb/fastb read count mismatch: ") + path);
    for (uint64_t i = 0; i <= n; ++i)
      if (io->base_off[i] - io->base_off[0] != bo[i])
        return io_fail(std::string("qualb/fastb length mismatch: ") + path);
  }
  auto* q = (uint8_t*)std::malloc(total + 64);
  if (!q) return APG_E_NOMEM;
  if (total && std::fread(q, 1, total, fh.f) != total) {
    std::free(q);
    return io_fail(std::string("truncated payload in ") + path);
  }
  if (io->quals) std::free((void*)io->quals);
  io->quals = q;
  if (!io->base_off) {
    auto* base_off = (uint64_t*)std::malloc((n + 1) * 8);
    if (!base_off) return APG_E_NOMEM;
    std::memcpy(base_off, bo.data(), (n + 1) * 8);
    io->base_off = base_off;
    io->n_reads = n;
  }
  return APG_OK;
}

void apg_reads_release(apg_reads* r) {
  if (!r) return;
  std::free((void*)r->base_off);
  std::free((void*)r->byte_off);
  std::free((void*)r->packed);
  std::free((void*)r->quals);
  std::memset(r, 0, sizeof(*r));
}

// apg_kspec_estimate: the spec is in include/apg.h (restated; checker
// oracle/kmer_oracle.c ork_kspec_estimate).
int apg_kspec_estimate(const uint64_t* hist, size_t hist_len, apg_kspec_summary* out) {
  if (!out || (!hist && hist_len)) return APG_E_ARG;
  std::memset(out, 0, sizeof(*out));
  if (hist_len < 3) return APG_OK;
  size_t v = 0;
  for (size_t m = 1; m < hist_len - 2; ++m)
    if (hist[m] < hist[m + 1]) {
      v = m;
      break;
    }
  if (!v) return APG_OK;
  size_t p = 0;
  for (size_t m = v + 1; m < hist_len - 1; ++m)
    if (hist[m] > (p ? hist[p] : 0)) p = m;
  for (size_t m = 1; m < hist_len; ++m) {
    const unsigned __int128 inst = (unsigned __int128)m * hist[m];
    if (m < v) {
      out->error_kmers += hist[m];
      out->error_instances += (uint64_t)inst;
    } else {
      out->genomic_kmers += hist[m];
      out->genomic_instances += (uint64_t)inst;
    }
  }
  out->valley = v;
  out->peak = p;
  if (!p) return APG_OK;
  unsigned __int128 s0 = 0, s1 = 0;
  const size_t hi = std::min<size_t>(2 * p - v, hist_len - 2);
  for (size_t m = v; m <= hi; ++m) {
    s0 += hist[m];
    s1 += (unsigned __int128)m * hist[m];
  }
  out->coverage = (double)s1 / (double)s0;
  out->genome_size = (uint64_t)(((unsigned __int128)out->genomic_instances * s0 + s1 / 2) / s1);
  if (out->genome_size > out->genomic_kmers)
    out->repeat_fraction = (double)(out->genome_size - out->genomic_kmers) / (double)out->genome_size;
  if (p >= 2) out->het_ratio = (double)hist[p / 2] / (double)hist[p];
  return APG_OK;
}

int apg_kspec_write(const char* path, int K, const uint64_t* hist, size_t hist_len) {
  if (!path || (!hist && hist_len)) return APG_E_ARG;
  const std::string tmp = std::string(path) + ".tmp";
  File fh;
  fh.f = std::fopen(tmp.c_str(), "w");
  if (!fh.f) return io_fail("cannot open " + tmp);
  std::fprintf(fh.f, "# KmerSpectrum K=%d bins=%zu (last bin = count >= %zu)\n", K, hist_len,
               hist_len ? hist_len - 1 : 0);
  apg_kspec_summary e;
  apg_kspec_estimate(hist, hist_len, &e);
  std::fprintf(fh.f,
               "# genome_size_estimate=%llu kmer_coverage=%.4f kmer_coverage_peak=%llu valley=%llu genomic_kmers=%llu "
               "genomic_instances=%llu error_kmers=%llu error_instances=%llu repeat_fraction=%.6f het_ratio=%.6f\n",
               (unsigned long long)e.genome_size, e.coverage, (unsigned long long)e.peak, (unsigned long long)e.valley,
               (unsigned long long)e.genomic_kmers, (unsigned long long)e.genomic_instances,
               (unsigned long long)e.error_kmers, (unsigned long long)e.error_instances, e.repeat_fraction,
               e.het_ratio);
  for (size_t m = 0; m < hist_len; ++m)
    if (hist[m]) std::fprintf(fh.f, "%zu\t%llu\n", m, (unsigned long long)hist[m]);
  if (std::fclose(fh.f) != 0) {
    fh.f = nullptr;
    return io_fail("close failed: " + tmp);
  }
  fh.f = nullptr;
  if (std::rename(tmp.c_str(), path) != 0) return io_fail("rename failed: " + tmp);
  return APG_OK;
}

}  // extern "C"
