// apg_graphio.cpp — on-disk unipath-stage objects ("APG v0"):
// KmerPaths (.paths.kK / .paths_rc.kK), unipaths (.unipaths.kK), unibases
// (.unibases.kK, APG-fastb), HyperKmerPath (.hkp.kK) and the MakeRcDb index
// (.pathsdb.kK), plus the correction / placement stages' boundary files:
// the solid set (.solid.kK), UnipathLocs (.unilocs.kK) and UnipathCoverage
// (.unipath_cov.kK).  The feudal layouts of ALLPATHS-LG's vecKmerPath /
// HyperKmerPath / tagged_rpint files are unpinned (reference absent), so these
// are versioned array containers; a feudal-compatible v1 can be added behind
// the same calls.
//
// Container: magic[8] | version u32 (0) | K u32 | n_arrays u32 | reserved u32 |
//            scalar u64 | n_arrays x {count u64, elem_bytes u32, reserved u32} |
//            the arrays' bytes in order.  Written to <file>.tmp, then renamed.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/apg.h"

namespace apg {
void set_error(const std::string& msg);
}

namespace {

struct Arr {
  const void* p;
  uint64_t count;
  uint32_t elem;
};

int io_fail(const std::string& what) {
  apg::set_error(what);
  return APG_E_IO;
}

std::string kname(const char* head, const char* ext, int K) {
  return std::string(head) + "." + ext + ".k" + std::to_string(K);
}

int write_container(const std::string& path, const char magic[8], int K, uint64_t scalar, const std::vector<Arr>& a) {
  const std::string tmp = path + ".tmp";
  FILE* f = std::fopen(tmp.c_str(), "wb");
  if (!f) return io_fail("cannot open " + tmp + " for writing");
  const uint32_t ver = 0, k = (uint32_t)K, na = (uint32_t)a.size(), res = 0;
  bool ok = std::fwrite(magic, 1, 8, f) == 8 && std::fwrite(&ver, 4, 1, f) == 1 && std::fwrite(&k, 4, 1, f) == 1 &&
            std::fwrite(&na, 4, 1, f) == 1 && std::fwrite(&res, 4, 1, f) == 1 && std::fwrite(&scalar, 8, 1, f) == 1;
  for (const Arr& x : a)
    ok = ok && std::fwrite(&x.count, 8, 1, f) == 1 && std::fwrite(&x.elem, 4, 1, f) == 1 &&
         std::fwrite(&res, 4, 1, f) == 1;
  for (const Arr& x : a)
    if (ok && x.count) ok = std::fwrite(x.p, x.elem, x.count, f) == x.count;
  if (std::fclose(f) != 0) ok = false;
  if (!ok) {
    std::remove(tmp.c_str());
    return io_fail("short write to " + tmp);
  }
  if (std::rename(tmp.c_str(), path.c_str()) != 0) return io_fail("cannot rename " + tmp);
  return APG_OK;
}

// Reads a container; arrays are malloc'd (free with apg_free).
int read_container(const std::string& path, const char magic[8], int* K, uint64_t* scalar, uint32_t want,
                   std::vector<void*>* out, std::vector<uint64_t>* counts, const std::vector<uint32_t>& elems) {
  FILE* f = std::fopen(path.c_str(), "rb");
  if (!f) return io_fail("cannot open " + path);
  char mg[8];
  uint32_t ver = 0, k = 0, na = 0, res = 0;
  uint64_t sc = 0;
  bool ok = std::fread(mg, 1, 8, f) == 8 && std::fread(&ver, 4, 1, f) == 1 && std::fread(&k, 4, 1, f) == 1 &&
            std::fread(&na, 4, 1, f) == 1 && std::fread(&res, 4, 1, f) == 1 && std::fread(&sc, 8, 1, f) == 1;
  if (!ok || std::memcmp(mg, magic, 8) != 0 || ver != 0 || na != want) {
    std::fclose(f);
    return io_fail(path + ": not an APG v0 " + std::string(magic, 5) + " file");
  }
  std::vector<uint64_t> cnt(na);
  std::vector<uint32_t> el(na);
  for (uint32_t i = 0; i < na && ok; ++i)
    ok = std::fread(&cnt[i], 8, 1, f) == 1 && std::fread(&el[i], 4, 1, f) == 1 && std::fread(&res, 4, 1, f) == 1;
  for (uint32_t i = 0; i < na && ok; ++i) ok = el[i] == elems[i];
  out->assign(na, nullptr);
  for (uint32_t i = 0; i < na && ok; ++i) {
    (*out)[i] = std::malloc(cnt[i] ? cnt[i] * el[i] : 1);
    ok = (*out)[i] && (cnt[i] == 0 || std::fread((*out)[i], el[i], cnt[i], f) == cnt[i]);
  }
  std::fclose(f);
  if (!ok) {
    for (void* p : *out) std::free(p);
    out->clear();
    return io_fail(path + ": truncated or malformed");
  }
  *K = (int)k;
  *scalar = sc;
  *counts = cnt;
  return APG_OK;
}

const char kPaths[8] = {'A', 'P', 'G', 'K', 'P', 0, 0, 0};
const char kUnip[8] = {'A', 'P', 'G', 'U', 'N', 0, 0, 0};
const char kHkp[8] = {'A', 'P', 'G', 'H', 'K', 0, 0, 0};
const char kDb[8] = {'A', 'P', 'G', 'D', 'B', 0, 0, 0};
const char kSolid[8] = {'A', 'P', 'G', 'S', 'L', 0, 0, 0};
const char kUlocs[8] = {'A', 'P', 'G', 'U', 'L', 0, 0, 0};
const char kUcov[8] = {'A', 'P', 'G', 'U', 'C', 0, 0, 0};

}  // namespace

extern "C" {

// The library-allocated arrays of a graph (host memory; apg_unipaths,
// apg_sharded_unipaths, apg_graph_read).
void apg_unipath_graph_free(apg_unipath_graph* g) {
  if (!g) return;
  std::free(g->len);
  std::free(g->id_base);
  std::free(g->rc);
  std::free(g->ub_off);
  std::free(g->unibases);
  std::free(g->from);
  std::free(g->to);
  std::free(g->path_off);
  std::free(g->path_start);
  std::free(g->path_len);
  std::memset(g, 0, sizeof(*g));
}


int apg_kmerpaths_write(const char* path, int K, uint64_t n_paths, const uint64_t* path_off, const uint64_t* start,
                        const uint64_t* len) {
  if (!path || !path_off) return APG_E_ARG;
  const uint64_t ni = path_off[n_paths];
  if (ni && (!start || !len)) return APG_E_ARG;
  return write_container(path, kPaths, K, n_paths,
                         {{path_off, n_paths + 1, 8}, {start, ni, 8}, {len, ni, 8}});
}

int apg_kmerpaths_read(const char* path, int* K, uint64_t* n_paths, uint64_t** path_off, uint64_t* n_intervals,
                       uint64_t** start, uint64_t** len) {
  if (!path || !K || !n_paths || !path_off || !n_intervals || !start || !len) return APG_E_ARG;
  std::vector<void*> a;
  std::vector<uint64_t> c;
  uint64_t sc = 0;
  int rc = read_container(path, kPaths, K, &sc, 3, &a, &c, {8, 8, 8});
  if (rc != APG_OK) return rc;
  if (c[0] != sc + 1 || c[1] != c[2] || static_cast<uint64_t*>(a[0])[sc] != c[1]) {
    for (void* p : a) std::free(p);
    return io_fail(std::string(path) + ": inconsistent KmerPaths arrays");
  }
  *n_paths = sc;
  *path_off = static_cast<uint64_t*>(a[0]);
  *n_intervals = c[1];
  *start = static_cast<uint64_t*>(a[1]);
  *len = static_cast<uint64_t*>(a[2]);
  return APG_OK;
}

int apg_graph_write(const char* head, const apg_unipath_graph* g) {
  if (!head || !g) return APG_E_ARG;
  const uint64_t U = g->n_unipaths;
  int rc = write_container(kname(head, "unipaths", g->K), kUnip, g->K, g->n_nodes,
                           {{g->len, U, 8}, {g->id_base, U, 8}, {g->rc, U, 8}});
  if (rc != APG_OK) return rc;
  rc = write_container(kname(head, "hkp", g->K), kHkp, g->K, g->n_vertices, {{g->from, U, 8}, {g->to, U, 8}});
  if (rc != APG_OK) return rc;
  // unibases as APG-fastb (pack the 1-byte bases)
  std::vector<uint64_t> bo(U + 1, 0), yo(U + 1, 0);
  for (uint64_t u = 0; u < U; ++u) {
    bo[u + 1] = g->ub_off[u + 1] - g->ub_off[0];
    yo[u + 1] = yo[u] + (bo[u + 1] - bo[u] + 3) / 4;
  }
  std::vector<uint8_t> pk(yo[U] + 1, 0);
  for (uint64_t u = 0; u < U; ++u)
    for (uint64_t i = 0; i < bo[u + 1] - bo[u]; ++i)
      pk[yo[u] + i / 4] |= (uint8_t)(g->unibases[bo[u] + i] << (2 * (i & 3)));
  apg_reads r{U, bo.data(), yo.data(), pk.data(), nullptr};
  rc = apg_fastb_write(kname(head, "unibases", g->K).c_str(), &r);
  if (rc != APG_OK) return rc;
  if (g->n_reads && g->path_off)
    rc = apg_kmerpaths_write(kname(head, "paths", g->K).c_str(), g->K, g->n_reads, g->path_off, g->path_start,
                             g->path_len);
  return rc;
}

int apg_graph_read(const char* head, int K, apg_unipath_graph* g) {
  if (!head || !g) return APG_E_ARG;
  std::memset(g, 0, sizeof(*g));
  std::vector<void*> a;
  std::vector<uint64_t> c;
  uint64_t sc = 0;
  int k = 0;
  int rc = read_container(kname(head, "unipaths", K), kUnip, &k, &sc, 3, &a, &c, {8, 8, 8});
  if (rc != APG_OK) return rc;
  g->K = k;
  g->n_nodes = sc;
  g->n_unipaths = c[0];
  g->len = static_cast<uint64_t*>(a[0]);
  g->id_base = static_cast<uint64_t*>(a[1]);
  g->rc = static_cast<uint64_t*>(a[2]);
  rc = read_container(kname(head, "hkp", K), kHkp, &k, &sc, 2, &a, &c, {8, 8});
  if (rc != APG_OK) {
    apg_unipath_graph_free(g);
    return rc;
  }
  g->n_vertices = sc;
  g->from = static_cast<uint64_t*>(a[0]);
  g->to = static_cast<uint64_t*>(a[1]);
  apg_reads ub{};
  rc = apg_fastb_read(kname(head, "unibases", K).c_str(), &ub);
  if (rc != APG_OK) {
    apg_unipath_graph_free(g);
    return rc;
  }
  const uint64_t U = g->n_unipaths;
  g->ub_off = static_cast<uint64_t*>(std::malloc((U + 1) * 8));
  const uint64_t nb = ub.n_reads ? ub.base_off[ub.n_reads] : 0;
  g->unibases = static_cast<uint8_t*>(std::malloc(nb ? nb : 1));
  if (!g->ub_off || !g->unibases || ub.n_reads != U) {
    apg_reads_release(&ub);
    apg_unipath_graph_free(g);
    return io_fail(std::string(head) + ": unibases do not match unipaths");
  }
  for (uint64_t u = 0; u <= U; ++u) g->ub_off[u] = U ? ub.base_off[u] : 0;
  for (uint64_t u = 0; u < U; ++u)
    for (uint64_t i = 0; i < ub.base_off[u + 1] - ub.base_off[u]; ++i)
      g->unibases[ub.base_off[u] + i] = (ub.packed[ub.byte_off[u] + i / 4] >> (2 * (i & 3))) & 3;
  apg_reads_release(&ub);
  // read paths are optional
  const std::string pp = kname(head, "paths", K);
  if (FILE* f = std::fopen(pp.c_str(), "rb")) {
    std::fclose(f);
    rc = apg_kmerpaths_read(pp.c_str(), &k, &g->n_reads, &g->path_off, &g->n_intervals, &g->path_start,
                            &g->path_len);
    if (rc != APG_OK) {
      apg_unipath_graph_free(g);
      return rc;
    }
  }
  return APG_OK;
}

int apg_rc_db_write(const char* head, int K, const apg_rc_db* db) {
  if (!head || !db) return APG_E_ARG;
  int rc = apg_kmerpaths_write(kname(head, "paths_rc", K).c_str(), K, db->n_reads, db->rc_path_off, db->rc_start,
                               db->rc_len);
  if (rc != APG_OK) return rc;
  return write_container(kname(head, "pathsdb", K), kDb, K, db->n_entries,
                         {{db->entries, db->n_entries, (uint32_t)sizeof(apg_rpint)}});
}

int apg_solid_write(const char* path, int K, const uint64_t* hashes, uint64_t n) {
  if (!path || (n && !hashes)) return APG_E_ARG;
  return write_container(path, kSolid, K, n, {{hashes, n, 8}});
}

int apg_solid_read(const char* path, int* K, uint64_t** hashes, uint64_t* n) {
  if (!path || !K || !hashes || !n) return APG_E_ARG;
  std::vector<void*> a;
  std::vector<uint64_t> c;
  uint64_t sc = 0;
  int rc = read_container(path, kSolid, K, &sc, 1, &a, &c, {8});
  if (rc != APG_OK) return rc;
  if (c[0] != sc) {
    std::free(a[0]);
    return io_fail(std::string(path) + ": inconsistent solid-set count");
  }
  *hashes = static_cast<uint64_t*>(a[0]);
  *n = sc;
  return APG_OK;
}

int apg_ulocs_write(const char* path, int K, uint64_t n_reads, const apg_aln_pair* locs, uint64_t n_locs) {
  if (!path || (n_locs && !locs)) return APG_E_ARG;
  return write_container(path, kUlocs, K, n_reads, {{locs, n_locs, (uint32_t)sizeof(apg_aln_pair)}});
}

int apg_ulocs_read(const char* path, int* K, uint64_t* n_reads, apg_aln_pair** locs, uint64_t* n_locs) {
  if (!path || !K || !n_reads || !locs || !n_locs) return APG_E_ARG;
  std::vector<void*> a;
  std::vector<uint64_t> c;
  int rc = read_container(path, kUlocs, K, n_reads, 1, &a, &c, {(uint32_t)sizeof(apg_aln_pair)});
  if (rc != APG_OK) return rc;
  *locs = static_cast<apg_aln_pair*>(a[0]);
  *n_locs = c[0];
  return APG_OK;
}

int apg_ucov_write(const char* path, int K, double c0, uint64_t n_unipaths, const uint64_t* counts, const double* cov,
                   const uint32_t* copy_number) {
  if (!path || (n_unipaths && (!counts || !cov || !copy_number))) return APG_E_ARG;
  uint64_t bits = 0;
  std::memcpy(&bits, &c0, 8);
  return write_container(path, kUcov, K, bits,
                         {{counts, n_unipaths, 8}, {cov, n_unipaths, 8}, {copy_number, n_unipaths, 4}});
}

int apg_ucov_read(const char* path, int* K, double* c0, uint64_t* n_unipaths, uint64_t** counts, double** cov,
                  uint32_t** copy_number) {
  if (!path || !K || !c0 || !n_unipaths || !counts || !cov || !copy_number) return APG_E_ARG;
  std::vector<void*> a;
  std::vector<uint64_t> c;
  uint64_t bits = 0;
  int rc = read_container(path, kUcov, K, &bits, 3, &a, &c, {8, 8, 4});
  if (rc != APG_OK) return rc;
  if (c[0] != c[1] || c[0] != c[2]) {
    for (void* p : a) std::free(p);
    return io_fail(std::string(path) + ": inconsistent coverage arrays");
  }
  std::memcpy(c0, &bits, 8);
  *n_unipaths = c[0];
  *counts = static_cast<uint64_t*>(a[0]);
  *cov = static_cast<double*>(a[1]);
  *copy_number = static_cast<uint32_t*>(a[2]);
  return APG_OK;
}

}  // extern "C"
