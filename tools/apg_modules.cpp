// apg_modules.cpp — drop-in command-line modules for RunAllPathsLG's hot
// path (SURVEY §8b, §3 call stack): KmerSpectrum, PreCorrect, FindErrors,
// FillFragments, ErrorCorrectJump, MergeReadSets (all_reads), CommonPather,
// Unipather, MakeRcDb, UnipathLocs, UnipathCoverage.  Same module names and KEY=VALUE argument style as the
// reference modules ([R:H] ParsedArgs; PRE/DATA/RUN directories); inputs and
// outputs are files in the RUN directory (APG v0 formats).
// One binary, dispatched on the name it is invoked under (bin/<Module> are
// symlinks).  Exit status 0 on success, 1 with a message on any error.
#include <sys/stat.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../include/apg.h"

namespace {

apg_comm* g_comm = nullptr;  // the sharded run's communicator, for Args::fail

struct Args {
  std::string module;
  std::map<std::string, std::string> kv;
  std::map<std::string, bool> used;

  std::string get(const std::string& k, const std::string& def) {
    used[k] = true;
    auto it = kv.find(k);
    return it == kv.end() ? def : it->second;
  }
  long num(const std::string& k, long def) {
    const std::string v = get(k, std::to_string(def));
    char* end = nullptr;
    const long x = std::strtol(v.c_str(), &end, 10);
    if (!end || *end) fail("argument " + k + "=" + v + " is not an integer");
    return x;
  }
  [[noreturn]] void fail(const std::string& msg) {
    std::fprintf(stderr, "%s: FATAL: %s\n", module.c_str(), msg.c_str());
    // a sharded rank: peers blocked in a collective with it error out
    // instead of waiting (RCCL would wait without end)
    if (g_comm) apg_comm_abort(g_comm);
    std::exit(1);
  }
  void check(int rc, const char* what) {
    if (rc != APG_OK) fail(std::string(what) + " failed: " + apg_last_error());
  }
  void finish() {
    for (const auto& e : kv)
      if (!used.count(e.first)) fail("unknown argument " + e.first);
  }
  std::string run_dir() {
    // PRE/DATA/RUN as in RunAllPathsLG, or RUN alone as a path
    const std::string pre = get("PRE", ""), data = get("DATA", ""), run = get("RUN", ".");
    std::string d = pre;
    if (!data.empty()) d += (d.empty() ? "" : "/") + data;
    if (!run.empty()) d += (d.empty() ? "" : "/") + run;
    return d.empty() ? "." : d;
  }
};

bool exists(const std::string& p) {
  struct stat st;
  return ::stat(p.c_str(), &st) == 0;
}

struct Ctx {
  apg_ctx* c = nullptr;
  explicit Ctx(Args& a) {
    apg_config cfg;
    std::memset(&cfg, 0, sizeof cfg);
    cfg.device = (int)a.num("DEVICE", 0);
    cfg.verbose = (int)a.num("VERBOSE", 0);
    a.check(apg_create(&cfg, &c), "apg_create");
  }
  ~Ctx() { apg_destroy(c); }
};

struct Reads {
  apg_reads r{};
  bool quals = false;
  ~Reads() { apg_reads_release(&r); }
};

std::string env_or(const char* k, const std::string& def) {
  const char* v = std::getenv(k);
  return v && *v ? std::string(v) : def;
}

// One rank of a sharded run: WORLD=N RANK=r COMM=rccl|tcp
// MASTER_ADDR MASTER_PORT (defaults from the torchrun-style environment).
// Rank r takes read pairs [np*r/N, np*(r+1)/N) of the input; every exchange
// runs inside libapg (apg_sharded_*); rank 0 writes the module's outputs.
// COMM=rccl: rank 0's RCCL id reaches the others over a short-lived TCP
// communicator; COMM=tcp: the TCP communicator carries the whole exchange
// (ranks may then share one GPU).
struct Shard {
  int rank = 0, world = 1;
  std::string mode, addr;
  int port = 29600;
  apg_comm* comm = nullptr;
  explicit Shard(Args& a) {
    // sharded only on request: WORLD= on the command line, or COMM= with the
    // launcher's WORLD_SIZE — a single-process call inside a launcher that
    // exports WORLD_SIZE stays single-process
    const bool asked = a.kv.count("WORLD") || a.kv.count("COMM");
    world = (int)a.num("WORLD", asked ? std::atol(env_or("WORLD_SIZE", "1").c_str()) : 1);
    rank = (int)a.num("RANK", std::atol(env_or("RANK", "0").c_str()));
    mode = a.get("COMM", "rccl");
    addr = a.get("MASTER_ADDR", env_or("MASTER_ADDR", "127.0.0.1"));
    port = (int)a.num("MASTER_PORT", std::atol(env_or("MASTER_PORT", "29600").c_str()));
    if (world < 1 || rank < 0 || rank >= world) a.fail("bad RANK / WORLD");
    if (mode != "rccl" && mode != "tcp") a.fail("COMM must be rccl or tcp");
  }
  ~Shard() {
    g_comm = nullptr;
    apg_comm_destroy(comm);
  }
  bool sharded() const { return world > 1; }
  void connect(Args& a, apg_ctx* ctx) {
    if (world == 1) return;
    if (mode == "tcp") {
      a.check(apg_comm_init_tcp(ctx, addr.c_str(), port, rank, world, 0, &comm), "apg_comm_init_tcp");
      g_comm = comm;
      return;
    }
    apg_comm* boot = nullptr;
    a.check(apg_comm_init_tcp(nullptr, addr.c_str(), port, rank, world, 0, &boot), "apg_comm_init_tcp (bootstrap)");
    std::vector<uint8_t> id(128, 0), all(128 * (size_t)world);
    if (rank == 0) a.check(apg_comm_unique_id(id.data()), "apg_comm_unique_id");
    std::vector<uint64_t> rb(world, 128);
    const int rc = apg_comm_allgatherv(boot, id.data(), 128, all.data(), rb.data());
    apg_comm_destroy(boot);
    a.check(rc, "bootstrap exchange");
    a.check(apg_comm_init_rccl(ctx, all.data(), rank, world, 0, &comm), "apg_comm_init_rccl");
    g_comm = comm;
  }
  void barrier(Args& a) {
    if (comm) a.check(apg_comm_barrier(comm), "apg_comm_barrier");
  }
  // this rank's whole pairs of n reads
  void range(uint64_t n, uint64_t* r0, uint64_t* r1) const {
    const uint64_t np = n / 2;
    *r0 = 2 * (np * (uint64_t)rank / (uint64_t)world);
    *r1 = rank + 1 == world ? n : 2 * (np * (uint64_t)(rank + 1) / (uint64_t)world);
  }
};

// Reads [r0, r1) of a loaded set as a standalone apg_reads view (offsets
// rebased, bases and qualities pointing into the loaded buffers).
struct Slice {
  std::vector<uint64_t> bo, yo;
  apg_reads r{};
  Slice(const apg_reads& all, uint64_t r0, uint64_t r1) : bo(r1 - r0 + 1), yo(r1 - r0 + 1) {
    for (uint64_t i = 0; i <= r1 - r0; ++i) {
      bo[i] = all.base_off[r0 + i] - all.base_off[r0];
      yo[i] = all.byte_off[r0 + i] - all.byte_off[r0];
    }
    r.n_reads = r1 - r0;
    r.base_off = bo.data();
    r.byte_off = yo.data();
    r.packed = all.packed + all.byte_off[r0];
    r.quals = all.quals ? all.quals + all.base_off[r0] : nullptr;
  }
};

struct DReads {
  apg_dreads* d = nullptr;
  ~DReads() { apg_reads_free(d); }
};

std::string part_name(const std::string& head, int rank, int world) {
  return head + ".part" + std::to_string(rank) + "of" + std::to_string(world);
}

void load_reads(Args& a, const std::string& head, bool need_quals, Reads* out) {
  const std::string fb = head + ".fastb", qb = head + ".qualb";
  if (!exists(fb)) a.fail("missing input " + fb);
  a.check(apg_fastb_read(fb.c_str(), &out->r), "reading .fastb");
  if (need_quals) {
    if (!exists(qb)) a.fail("missing input " + qb);
    apg_reads q{};
    a.check(apg_qualb_read(qb.c_str(), &q), "reading .qualb");
    if (q.n_reads != out->r.n_reads) {
      apg_reads_release(&q);
      a.fail(".qualb read count differs from .fastb");
    }
    out->r.quals = q.quals;  // adopt the quality buffer
    q.quals = nullptr;
    apg_reads_release(&q);
    out->quals = true;
  }
}

int kmer_spectrum(Args& a) {
  const std::string dir = a.run_dir();
  const std::string head = dir + "/" + a.get("READS", "frag_reads_filt");
  const int K = (int)a.num("K", 25);
  const long hist_len = a.num("HIST_LEN", 1 << 16);
  Shard sh(a);
  a.finish();
  Reads rd;
  load_reads(a, head, false, &rd);
  Ctx ctx(a);
  std::vector<uint64_t> hist((size_t)hist_len);
  apg_kstats st;
  if (sh.sharded()) {
    sh.connect(a, ctx.c);
    uint64_t r0, r1;
    sh.range(rd.r.n_reads, &r0, &r1);
    Slice sl(rd.r, r0, r1);
    DReads d;
    a.check(apg_reads_upload(ctx.c, &sl.r, &d.d), "apg_reads_upload");
    a.check(apg_sharded_spectrum(ctx.c, sh.comm, d.d, K, hist.data(), hist.size(), &st), "apg_sharded_spectrum");
    if (sh.rank != 0) return 0;  // every rank holds the global spectrum; rank 0 writes it
  } else {
    a.check(apg_kmer_spectrum(ctx.c, &rd.r, K, hist.data(), hist.size(), &st), "apg_kmer_spectrum");
  }
  const std::string out = head + ".kspec.k" + std::to_string(K);
  a.check(apg_kspec_write(out.c_str(), K, hist.data(), hist.size()), "writing .kspec");
  apg_kspec_summary e;
  a.check(apg_kspec_estimate(hist.data(), hist.size(), &e), "apg_kspec_estimate");
  std::printf("%s: %llu reads, %llu %d-mers, %llu distinct, genome size estimate %llu (K-mer coverage %llu) -> %s\n",
              a.module.c_str(), (unsigned long long)rd.r.n_reads, (unsigned long long)st.n_kmers, K,
              (unsigned long long)st.n_distinct, (unsigned long long)e.genome_size, (unsigned long long)e.peak,
              out.c_str());
  return 0;
}

// <head>.solid.k<K>: the last correction pass's solid set, ascending — what
// FillFragments (APG_FILL_LAST_SOLID in one process) uses in the next one.
void write_solid(Args& a, apg_ctx* c, const std::string& head, int K) {
  uint64_t n = 0;
  a.check(apg_solid_download(c, nullptr, &n), "apg_solid_download");
  std::vector<uint64_t> s(n + 1);
  a.check(apg_solid_download(c, s.data(), &n), "apg_solid_download");
  s.resize(n);
  std::sort(s.begin(), s.end());
  a.check(apg_solid_write((head + ".solid.k" + std::to_string(K)).c_str(), K, s.data(), n), "writing .solid");
}

struct Solid {
  uint64_t* h = nullptr;
  uint64_t n = 0;
  ~Solid() { apg_free(h); }
};

// Reads [r0, r1) of a loaded set copied out as a standalone read set (rank
// parts written by sharded runs).
void write_reads(Args& a, const std::string& head, const apg_reads& r, bool quals) {
  a.check(apg_fastb_write((head + ".fastb").c_str(), &r), "writing .fastb");
  if (quals) a.check(apg_qualb_write((head + ".qualb").c_str(), &r), "writing .qualb");
}

// Read sets concatenated in order (a part may be empty); quals kept only if
// every part has them.
struct Joined {
  std::vector<uint64_t> bo{0}, yo{0};
  std::vector<uint8_t> pk, q;
  bool quals = true;
  void add(const apg_reads& r) {
    if (!r.quals) quals = false;
    const uint64_t n = r.n_reads;
    if (n == 0) return;
    const uint64_t b0 = bo.back(), y0 = yo.back();
    for (uint64_t i = 1; i <= n; ++i) {
      bo.push_back(b0 + r.base_off[i] - r.base_off[0]);
      yo.push_back(y0 + r.byte_off[i] - r.byte_off[0]);
    }
    pk.insert(pk.end(), r.packed + r.byte_off[0], r.packed + r.byte_off[n]);
    if (quals) q.insert(q.end(), r.quals + r.base_off[0], r.quals + r.base_off[n]);
  }
  apg_reads view() {
    pk.resize(yo.back() + 64, 0);
    q.resize(bo.back() + 1, 0);
    return apg_reads{bo.size() - 1, bo.data(), yo.data(), pk.data(), quals ? q.data() : nullptr};
  }
};

int precorrect(Args& a, uint32_t default_cycles, const char* default_out) {
  const std::string dir = a.run_dir();
  const std::string in = dir + "/" + a.get("HEAD_IN", "frag_reads_filt");
  const std::string out = dir + "/" + a.get("HEAD_OUT", default_out);
  apg_pc_params p;
  apg_pc_defaults(&p);
  p.K = (int)a.num("K", p.K);
  p.min_solid = (uint32_t)a.num("MIN_SOLID", p.min_solid);
  p.max_q_suspect = (uint32_t)a.num("MAX_Q_SUSPECT", p.max_q_suspect);
  p.n_cycles = (uint32_t)a.num("NUM_CYCLES", default_cycles);
  Shard sh(a);
  a.finish();
  Reads rd;
  load_reads(a, in, true, &rd);
  Ctx ctx(a);
  const uint64_t n = rd.r.n_reads;
  const uint64_t nbytes = n ? rd.r.byte_off[n] : 0, nbases = n ? rd.r.base_off[n] : 0;
  std::vector<uint8_t> pk(nbytes + 64), q(nbases + 1);
  apg_pc_stats st;
  if (sh.sharded()) {
    // this rank's pairs corrected against the global solid set; each rank
    // writes its corrected slice as a part file, rank 0 assembles the output
    sh.connect(a, ctx.c);
    uint64_t r0, r1;
    sh.range(n, &r0, &r1);
    Slice sl(rd.r, r0, r1);
    DReads d;
    a.check(apg_reads_upload(ctx.c, &sl.r, &d.d), "apg_reads_upload");
    a.check(apg_sharded_precorrect(ctx.c, sh.comm, d.d, &p, &st), "apg_sharded_precorrect");
    const uint64_t y0 = rd.r.byte_off[r0], b0 = rd.r.base_off[r0];
    a.check(apg_reads_download(ctx.c, d.d, pk.data() + y0, q.data() + b0), "apg_reads_download");
    apg_reads part = sl.r;
    part.packed = pk.data() + y0;
    part.quals = q.data() + b0;
    const std::string ph = part_name(out, sh.rank, sh.world);
    if (sh.rank != 0) {
      a.check(apg_fastb_write((ph + ".fastb").c_str(), &part), "writing part .fastb");
      a.check(apg_qualb_write((ph + ".qualb").c_str(), &part), "writing part .qualb");
    }
    sh.barrier(a);
    if (sh.rank != 0) {
      sh.barrier(a);  // rank 0 has read every part
      return 0;
    }
    for (int r = 1; r < sh.world; ++r) {  // place every other rank's slice
      Shard other = sh;
      other.comm = nullptr;
      other.rank = r;
      uint64_t s0, s1;
      other.range(n, &s0, &s1);
      const std::string h = part_name(out, r, sh.world);
      Reads pr;
      load_reads(a, h, true, &pr);
      if (pr.r.n_reads != s1 - s0) a.fail("part " + h + " has the wrong read count");
      const uint64_t py = s1 > s0 ? pr.r.byte_off[s1 - s0] : 0, pb = s1 > s0 ? pr.r.base_off[s1 - s0] : 0;
      std::memcpy(pk.data() + rd.r.byte_off[s0], pr.r.packed, py);
      std::memcpy(q.data() + rd.r.base_off[s0], pr.r.quals, pb);
      std::remove((h + ".fastb").c_str());
      std::remove((h + ".qualb").c_str());
    }
    sh.barrier(a);
  } else {
    a.check(apg_precorrect(ctx.c, &rd.r, &p, pk.data(), q.data(), &st), "apg_precorrect");
  }
  apg_reads o = rd.r;
  o.packed = pk.data();
  o.quals = q.data();
  a.check(apg_fastb_write((out + ".fastb").c_str(), &o), "writing .fastb");
  a.check(apg_qualb_write((out + ".qualb").c_str(), &o), "writing .qualb");
  write_solid(a, ctx.c, out, p.K);
  std::printf("%s: %llu reads, %llu suspect, %llu corrected, %llu ambiguous, %llu uncorrectable -> %s.{fastb,qualb}\n",
              a.module.c_str(), (unsigned long long)n, (unsigned long long)st.n_suspect,
              (unsigned long long)st.n_corrected, (unsigned long long)st.n_ambiguous,
              (unsigned long long)st.n_uncorrectable, out.c_str());
  return 0;
}

// ErrorCorrectJump: jump reads corrected against the fragment reads' solid
// set and trimmed to their all-solid prefix; the output keeps one read per
// input read (a dropped read has length 0) so pairs keep their indices.
int error_correct_jump(Args& a) {
  const std::string dir = a.run_dir();
  const std::string fin = dir + "/" + a.get("FRAG_IN", "frag_reads_edit");
  const std::string jin = dir + "/" + a.get("HEAD_IN", "jump_reads_filt");
  const std::string out = dir + "/" + a.get("HEAD_OUT", "jump_reads_ec");
  apg_ecj_params p;
  apg_ecj_defaults(&p);
  p.K = (int)a.num("K", p.K);
  p.min_solid = (uint32_t)a.num("MIN_SOLID", p.min_solid);
  p.max_q_suspect = (uint32_t)a.num("MAX_Q_SUSPECT", p.max_q_suspect);
  p.min_keep = (uint32_t)a.num("MIN_KEEP", p.min_keep);
  Shard sh(a);
  a.finish();
  Reads fr, jr_all;
  load_reads(a, fin, false, &fr);
  load_reads(a, jin, true, &jr_all);
  Ctx ctx(a);
  apg_ecj_stats st;
  // a sharded rank corrects its slice of the jump pairs against the global
  // solid set of every rank's frag pairs (apg_sharded_error_correct_jump:
  // counted across the ranks); rank 0 joins the parts
  uint64_t j0 = 0, j1 = jr_all.r.n_reads;
  if (sh.sharded()) {
    if (jr_all.r.n_reads % 2 || fr.r.n_reads % 2) a.fail("sharded ErrorCorrectJump needs whole pairs (2i, 2i+1)");
    sh.connect(a, ctx.c);
    sh.range(jr_all.r.n_reads, &j0, &j1);
  }
  Slice js(jr_all.r, j0, j1);
  const apg_reads& jr = js.r;  // this rank's jump reads (all of them single-process)
  const uint64_t n = jr.n_reads;
  const uint64_t nbytes = n ? jr.byte_off[n] : 0, nbases = n ? jr.base_off[n] : 0;
  std::vector<uint8_t> pk(nbytes + 64), q(nbases + 1);
  std::vector<uint32_t> keep(n + 1);
  if (sh.sharded()) {
    uint64_t f0 = 0, f1 = 0;
    sh.range(fr.r.n_reads, &f0, &f1);
    Slice fs(fr.r, f0, f1);
    DReads dF, dJ, dK;
    a.check(apg_reads_upload(ctx.c, &fs.r, &dF.d), "apg_reads_upload");
    a.check(apg_reads_upload(ctx.c, &jr, &dJ.d), "apg_reads_upload");
    void* d_keep = nullptr;
    a.check(apg_device_alloc(ctx.c, (n + 1) * 4, &d_keep), "apg_device_alloc");
    int rc = apg_sharded_error_correct_jump(ctx.c, sh.comm, dF.d, dJ.d, &p, static_cast<uint32_t*>(d_keep), &st);
    if (rc == APG_OK) rc = apg_reads_download(ctx.c, dJ.d, pk.data(), q.data());
    if (rc == APG_OK) rc = apg_device_to_host(ctx.c, keep.data(), d_keep, n * 4);
    apg_device_free(ctx.c, d_keep);
    a.check(rc, "apg_sharded_error_correct_jump");
  } else {
    a.check(apg_error_correct_jump(ctx.c, &fr.r, &jr, &p, pk.data(), q.data(), keep.data(), &st),
            "apg_error_correct_jump");
  }
  // trimmed layout: read r = its first keep[r] bases
  std::vector<uint64_t> bo(n + 1, 0), yo(n + 1, 0);
  for (uint64_t r = 0; r < n; ++r) bo[r + 1] = bo[r] + keep[r];
  a.check(apg_byte_offsets(bo.data(), n, yo.data()), "apg_byte_offsets");
  std::vector<uint8_t> tp(yo[n] + 64, 0), tq(bo[n] + 1);
  for (uint64_t r = 0; r < n; ++r) {
    const uint8_t* src = pk.data() + jr.byte_off[r];
    std::memcpy(tp.data() + yo[r], src, (keep[r] + 3) / 4);
    if (keep[r] % 4) tp[yo[r] + keep[r] / 4] &= (uint8_t)((1u << (2 * (keep[r] % 4))) - 1);
    std::memcpy(tq.data() + bo[r], q.data() + jr.base_off[r], keep[r]);
  }
  apg_reads o{};
  o.n_reads = n;
  o.base_off = bo.data();
  o.byte_off = yo.data();
  o.packed = tp.data();
  o.quals = tq.data();
  Joined jn;
  if (sh.sharded()) {  // ranks hold consecutive pairs: rank order = read order
    if (sh.rank != 0) {
      write_reads(a, part_name(out, sh.rank, sh.world), o, true);
      sh.barrier(a);
      sh.barrier(a);  // rank 0 has read every part
      return 0;
    }
    sh.barrier(a);
    jn.add(o);
    for (int r = 1; r < sh.world; ++r) {
      const std::string h = part_name(out, r, sh.world);
      Reads pr;
      load_reads(a, h, true, &pr);
      jn.add(pr.r);
      std::remove((h + ".fastb").c_str());
      std::remove((h + ".qualb").c_str());
    }
    sh.barrier(a);
    o = jn.view();
  }
  a.check(apg_fastb_write((out + ".fastb").c_str(), &o), "writing .fastb");
  a.check(apg_qualb_write((out + ".qualb").c_str(), &o), "writing .qualb");
  std::printf("%s: %llu jump reads, %llu corrected, %llu whole, %llu trimmed, %llu dropped -> %s.{fastb,qualb}\n",
              a.module.c_str(), (unsigned long long)st.n_reads, (unsigned long long)st.pc.n_corrected,
              (unsigned long long)st.n_full, (unsigned long long)st.n_trimmed, (unsigned long long)st.n_dropped,
              out.c_str());
  return 0;
}

// FillFragments: frag pairs (reads 2i, 2i+1) closed into the fragments they
// were read from (apg_fill_fragments), against the solid set the correction
// module wrote (<SOLID>.solid.k<K>, SOLID defaulting to HEAD_IN) — the
// APG_FILL_LAST_SOLID set of the in-process chain — or, when no such file
// exists and SOLID= is not given, the pairs' own K-mers with count >=
// MIN_SOLID.  Output: <HEAD_OUT>.fastb, the filled fragments in pair order
// (no qualities).
int fill_fragments(Args& a) {
  const std::string dir = a.run_dir();
  const std::string in = dir + "/" + a.get("HEAD_IN", "frag_reads_corr");
  const std::string out = dir + "/" + a.get("HEAD_OUT", "filled_reads");
  const bool solid_given = a.kv.count("SOLID") > 0;
  const std::string sh_in = dir + "/" + a.get("SOLID", a.get("HEAD_IN", "frag_reads_corr"));
  apg_fill_params p;
  apg_fill_defaults(&p);
  p.K = (int)a.num("K", p.K);
  p.min_insert = (uint32_t)a.num("MIN_INSERT", p.min_insert);
  p.max_insert = (uint32_t)a.num("MAX_INSERT", p.max_insert);
  p.max_steps = (uint32_t)a.num("MAX_STEPS", p.max_steps);
  p.min_solid = (uint32_t)a.num("MIN_SOLID", p.min_solid);
  Shard sh(a);
  a.finish();
  const std::string sf = sh_in + ".solid.k" + std::to_string(p.K);
  Solid sol;
  const bool have_solid = exists(sf);
  if (solid_given && !have_solid) a.fail("missing solid set " + sf);
  if (have_solid) {
    int k = 0;
    a.check(apg_solid_read(sf.c_str(), &k, &sol.h, &sol.n), "reading .solid");
    if (k != p.K) a.fail(sf + " holds K=" + std::to_string(k) + " K-mers");
  }
  Reads rd;
  load_reads(a, in, false, &rd);
  if (rd.r.n_reads % 2) a.fail(in + ".fastb: odd read count (pairs are reads 2i, 2i+1)");
  Ctx ctx(a);
  apg_fill_stats st;
  apg_reads filled{};
  struct Rel {
    apg_reads* r;
    ~Rel() { apg_reads_release(r); }
  } rel{&filled};
  if (sh.sharded()) {
    // a rank fills its own pairs (no exchange): the solid set must be the
    // global one, so the sharded form needs the correction module's file
    if (!have_solid) a.fail("sharded FillFragments needs the correction pass's solid set (" + sf + ")");
    sh.connect(a, ctx.c);
    uint64_t r0, r1;
    sh.range(rd.r.n_reads, &r0, &r1);
    Slice sl(rd.r, r0, r1);
    DReads d, f;
    a.check(apg_reads_upload(ctx.c, &sl.r, &d.d), "apg_reads_upload");
    a.check(apg_solid_upload(ctx.c, p.K, sol.h, sol.n), "apg_solid_upload");
    p.flags |= APG_FILL_LAST_SOLID;
    a.check(apg_sharded_fill(ctx.c, sh.comm, d.d, &p, nullptr, 0, &f.d, nullptr, &st), "apg_sharded_fill");
    uint64_t nf = 0, nb = 0, ny = 0;
    a.check(apg_dreads_shape(ctx.c, f.d, &nf, &nb, &ny, nullptr, nullptr), "apg_dreads_shape");
    std::vector<uint64_t> bo(nf + 1), yo(nf + 1);
    a.check(apg_dreads_shape(ctx.c, f.d, nullptr, nullptr, nullptr, bo.data(), yo.data()), "apg_dreads_shape");
    std::vector<uint8_t> pk(ny + 64, 0);
    a.check(apg_reads_download(ctx.c, f.d, pk.data(), nullptr), "apg_reads_download");
    apg_reads mine{nf, bo.data(), yo.data(), pk.data(), nullptr};
    if (sh.rank != 0) {
      write_reads(a, part_name(out, sh.rank, sh.world), mine, false);
      sh.barrier(a);
      sh.barrier(a);  // rank 0 has read every part
      return 0;
    }
    sh.barrier(a);
    Joined j;
    j.add(mine);
    for (int r = 1; r < sh.world; ++r) {  // ranks hold consecutive pairs: rank order = pair order
      const std::string h = part_name(out, r, sh.world);
      Reads pr;
      load_reads(a, h, false, &pr);
      j.add(pr.r);
      std::remove((h + ".fastb").c_str());
    }
    sh.barrier(a);
    apg_reads o = j.view();
    write_reads(a, out, o, false);
  } else {
    if (!have_solid) p.flags &= ~APG_FILL_LAST_SOLID;
    a.check(apg_fill_fragments(ctx.c, &rd.r, &p, sol.h, sol.n, &filled, nullptr, &st), "apg_fill_fragments");
    write_reads(a, out, filled, false);
  }
  std::printf("%s: %llu pairs, %llu filled, %llu none, %llu ambiguous, %llu over budget, %llu skipped "
              "(solid set: %s, %llu K-mers) -> %s.fastb\n",
              a.module.c_str(), (unsigned long long)st.n_pairs, (unsigned long long)st.n_filled,
              (unsigned long long)st.n_none, (unsigned long long)st.n_ambiguous, (unsigned long long)st.n_budget,
              (unsigned long long)st.n_skip, have_solid ? sf.c_str() : "own count", (unsigned long long)st.n_solid,
              out.c_str());
  return 0;
}

// MergeReadSets: all_reads = the read sets of HEADS (comma-separated, in
// order) concatenated — filled fragments ++ ErrorCorrectJump's trimmed jumps
// in the RunAllPathsLG chain (a dropped jump read stays as a 0-length read, so
// pair indices hold), as apg_reads_concat_dev does on the device.  Qualities
// are written only when every input has a .qualb.
int merge_read_sets(Args& a) {
  const std::string dir = a.run_dir();
  const std::string heads = a.get("HEADS", "filled_reads,jump_reads_ec");
  const std::string out = dir + "/" + a.get("HEAD_OUT", "all_reads");
  a.finish();
  std::vector<std::string> hs;
  for (size_t b = 0; b <= heads.size();) {
    const size_t e = std::min(heads.find(',', b), heads.size());
    if (e > b) hs.push_back(dir + "/" + heads.substr(b, e - b));
    b = e + 1;
  }
  if (hs.empty()) a.fail("HEADS names no read set");
  bool quals = true;
  for (const auto& h : hs) quals = quals && exists(h + ".qualb");
  Joined j;
  for (const auto& h : hs) {
    Reads r;
    load_reads(a, h, quals, &r);
    j.add(r.r);
  }
  apg_reads o = j.view();
  write_reads(a, out, o, quals);
  std::printf("%s: %zu read sets, %llu reads, %llu bases -> %s.fastb%s\n", a.module.c_str(), hs.size(),
              (unsigned long long)o.n_reads, (unsigned long long)j.bo.back(), out.c_str(), quals ? "/.qualb" : "");
  return 0;
}

// The unipath graph of files <head>.*.k<K> rebuilt on the context, so that
// placements resolve against it (UnipathLocs / UnipathCoverage work on "the
// context's last unipath build"): the unibases, one read per unipath, give
// exactly the file's unipaths — every K-mer lies in one unipath and every
// interior link lies inside a unibase, so no unipath splits or merges, and
// the order follows the head K-mers — which is checked against the
// .unipaths / .unibases files before any placement.
void rebuild_graph(Args& a, apg_ctx* c, const std::string& head, int K, Shard* sh, apg_unipath_graph* file_g) {
  a.check(apg_graph_read(head.c_str(), K, file_g), "reading unipath files (run Unipather first)");
  Reads ub;  // <head>.unibases.k<K>: an APG-fastb file under the graph's own name (no .fastb suffix)
  const std::string ubf = head + ".unibases.k" + std::to_string(K);
  if (!exists(ubf)) a.fail("missing input " + ubf + " (run Unipather first)");
  a.check(apg_fastb_read(ubf.c_str(), &ub.r), "reading the unibases");
  apg_unipath_params p;
  apg_unipath_defaults(&p);
  p.K = K;
  apg_unipath_graph g{};
  apg_unipath_stats st;
  if (sh && sh->sharded()) {
    uint64_t r0, r1;
    // unibases are not pairs: split them evenly by read
    r0 = ub.r.n_reads * (uint64_t)sh->rank / (uint64_t)sh->world;
    r1 = ub.r.n_reads * (uint64_t)(sh->rank + 1) / (uint64_t)sh->world;
    Slice sl(ub.r, r0, r1);
    DReads d;
    a.check(apg_reads_upload(c, &sl.r, &d.d), "apg_reads_upload");
    a.check(apg_sharded_unipaths(c, sh->comm, d.d, &p, &g, &st), "apg_sharded_unipaths");
  } else {
    a.check(apg_unipaths(c, &ub.r, &p, &g, &st), "apg_unipaths");
  }
  bool same = g.n_unipaths == file_g->n_unipaths;
  for (uint64_t u = 0; same && u < g.n_unipaths; ++u) same = g.len[u] == file_g->len[u];
  const uint64_t nb = g.n_unipaths ? g.ub_off[g.n_unipaths] : 0;
  same = same && nb == (file_g->n_unipaths ? file_g->ub_off[file_g->n_unipaths] : 0) &&
         (nb == 0 || std::memcmp(g.unibases, file_g->unibases, nb) == 0);
  apg_unipath_graph_free(&g);
  if (!same) a.fail(head + ": the unipaths rebuilt from the unibases differ from the .unipaths file");
}

// UnipathLocs: placements of the reads HEAD_IN on the unipaths READS.*.k<K>
// (apg_unipath_locs: a location per change of (unipath, start) along the
// read, RC=1 with rc mirrors, SORTED=1 stably by (unipath, start)) ->
// <HEAD_IN>.unilocs.k<K>.
int unipath_locs(Args& a) {
  const std::string dir = a.run_dir();
  const std::string head = dir + "/" + a.get("READS", "all_reads");
  const std::string in = dir + "/" + a.get("HEAD_IN", "frag_reads_corr");
  const int K = (int)a.num("K", 96);
  const bool rc = a.num("RC", 1) != 0, sorted = a.num("SORTED", 1) != 0;
  Shard sh(a);
  a.finish();
  const uint32_t flags = (rc ? APG_ULOCS_RC : 0u) | (sorted ? APG_ULOCS_SORTED : 0u);
  Ctx ctx(a);
  if (sh.sharded()) sh.connect(a, ctx.c);
  apg_unipath_graph fg{};
  rebuild_graph(a, ctx.c, head, K, &sh, &fg);
  apg_unipath_graph_free(&fg);
  Reads rd;
  load_reads(a, in, false, &rd);
  const std::string out = in + ".unilocs.k" + std::to_string(K);
  apg_uloc_stats st;
  std::vector<apg_aln_pair> all;
  if (sh.sharded()) {
    uint64_t r0, r1;
    sh.range(rd.r.n_reads, &r0, &r1);
    Slice sl(rd.r, r0, r1);
    DReads d;
    a.check(apg_reads_upload(ctx.c, &sl.r, &d.d), "apg_reads_upload");
    const apg_aln_pair* dl = nullptr;
    uint64_t n = 0;
    a.check(apg_sharded_unipath_locs(ctx.c, sh.comm, d.d, flags, &dl, &n, &st), "apg_sharded_unipath_locs");
    std::vector<apg_aln_pair> mine(n);
    if (n) a.check(apg_device_to_host(ctx.c, mine.data(), dl, n * sizeof(apg_aln_pair)), "copying placements");
    for (auto& l : mine) l.s_id += (uint32_t)r0;  // this rank's reads start at read r0
    const std::string pp = part_name(in, sh.rank, sh.world) + ".unilocs.k" + std::to_string(K);
    if (sh.rank != 0) {
      a.check(apg_ulocs_write(pp.c_str(), K, r1 - r0, mine.data(), n), "writing placement part");
      sh.barrier(a);
      sh.barrier(a);
      return 0;
    }
    sh.barrier(a);
    all = std::move(mine);
    for (int r = 1; r < sh.world; ++r) {
      const std::string h = part_name(in, r, sh.world) + ".unilocs.k" + std::to_string(K);
      int k = 0;
      uint64_t nr = 0, np = 0;
      apg_aln_pair* pl = nullptr;
      a.check(apg_ulocs_read(h.c_str(), &k, &nr, &pl, &np), "reading placement part");
      all.insert(all.end(), pl, pl + np);
      apg_free(pl);
      std::remove(h.c_str());
    }
    sh.barrier(a);
    // ranks hold consecutive reads: the stable (unipath, start) order of the
    // union is the stable sort of the rank-ordered concatenation
    if (sorted)
      std::stable_sort(all.begin(), all.end(), [](const apg_aln_pair& x, const apg_aln_pair& y) {
        return x.t_id != y.t_id ? x.t_id < y.t_id : x.offset < y.offset;
      });
  } else {
    apg_aln_pair* l = nullptr;
    uint64_t n = 0;
    a.check(apg_unipath_locs(ctx.c, &rd.r, flags, &l, &n, &st), "apg_unipath_locs");
    all.assign(l, l + n);
    apg_free(l);
  }
  a.check(apg_ulocs_write(out.c_str(), K, rd.r.n_reads, all.data(), all.size()), "writing .unilocs");
  std::printf("%s: %llu reads, %llu placed, %llu locations, %llu K-mers off the graph -> %s\n", a.module.c_str(),
              (unsigned long long)st.n_reads, (unsigned long long)st.n_placed, (unsigned long long)all.size(),
              (unsigned long long)st.n_missing, out.c_str());
  return 0;
}

// UnipathCoverage: placements per unipath, placements per K-mer and the
// copy-number estimate (apg_unipath_coverage) of the placements
// <HEAD_IN>.unilocs.k<K> on the unipaths READS.*.k<K> ->
// <READS>.unipath_cov.k<K>.
int unipath_coverage(Args& a) {
  const std::string dir = a.run_dir();
  const std::string head = dir + "/" + a.get("READS", "all_reads");
  const std::string in = dir + "/" + a.get("HEAD_IN", "frag_reads_corr");
  const int K = (int)a.num("K", 96);
  apg_ucov_params p;
  apg_ucov_defaults(&p);
  p.min_len = (uint64_t)a.num("MIN_LEN", (long)p.min_len);
  a.finish();
  const std::string lf = in + ".unilocs.k" + std::to_string(K);
  if (!exists(lf)) a.fail("missing input " + lf + " (run UnipathLocs first)");
  int k = 0;
  uint64_t nr = 0, n = 0;
  apg_aln_pair* locs = nullptr;
  a.check(apg_ulocs_read(lf.c_str(), &k, &nr, &locs, &n), "reading .unilocs");
  struct Fr {
    void* p;
    ~Fr() { apg_free(p); }
  } fr{locs};
  if (k != K) a.fail(lf + " was placed at K=" + std::to_string(k));
  Ctx ctx(a);
  apg_unipath_graph fg{};
  rebuild_graph(a, ctx.c, head, K, nullptr, &fg);
  const uint64_t U = fg.n_unipaths;
  apg_unipath_graph_free(&fg);
  std::vector<uint64_t> cnt(U + 1);
  std::vector<double> cov(U + 1);
  std::vector<uint32_t> cn(U + 1);
  apg_ucov_stats st;
  a.check(apg_unipath_coverage(ctx.c, locs, n, &p, cnt.data(), cov.data(), cn.data(), &st), "apg_unipath_coverage");
  const std::string out = head + ".unipath_cov.k" + std::to_string(K);
  a.check(apg_ucov_write(out.c_str(), K, st.c0, U, cnt.data(), cov.data(), cn.data()), "writing .unipath_cov");
  std::printf("%s: %llu placements on %llu unipaths, genome-wide %.4f placements per K-mer over %llu long unipaths "
              "-> %s\n",
              a.module.c_str(), (unsigned long long)n, (unsigned long long)U, st.c0, (unsigned long long)st.n_long,
              out.c_str());
  return 0;
}

int unipaths(Args& a, bool read_paths) {
  const std::string dir = a.run_dir();
  const std::string head = dir + "/" + a.get("READS", "all_reads");
  apg_unipath_params p;
  apg_unipath_defaults(&p);
  p.K = (int)a.num("K", p.K);
  p.flags = read_paths ? APG_UNIPATH_READ_PATHS : 0;
  Shard sh(a);
  a.finish();
  Reads rd;
  load_reads(a, head, false, &rd);
  Ctx ctx(a);
  apg_unipath_graph g{};
  apg_unipath_stats st;
  if (sh.sharded()) {
    // the global graph on every rank + KmerPaths of each rank's reads: ranks
    // > 0 write their KmerPaths as parts, rank 0 joins them in read order
    sh.connect(a, ctx.c);
    uint64_t r0, r1;
    sh.range(rd.r.n_reads, &r0, &r1);
    Slice sl(rd.r, r0, r1);
    DReads d;
    a.check(apg_reads_upload(ctx.c, &sl.r, &d.d), "apg_reads_upload");
    a.check(apg_sharded_unipaths(ctx.c, sh.comm, d.d, &p, &g, &st), "apg_sharded_unipaths");
    const std::string pp = part_name(head, sh.rank, sh.world) + ".paths.k" + std::to_string(p.K);
    if (sh.rank != 0 && read_paths)
      a.check(apg_kmerpaths_write(pp.c_str(), p.K, g.n_reads, g.path_off, g.path_start, g.path_len),
              "writing KmerPath part");
    sh.barrier(a);
    if (sh.rank != 0) {
      apg_unipath_graph_free(&g);
      sh.barrier(a);
      return 0;
    }
    if (read_paths) {
      std::vector<uint64_t> off(g.path_off, g.path_off + g.n_reads + 1), start(g.path_start, g.path_start + g.n_intervals),
          len(g.path_len, g.path_len + g.n_intervals);
      for (int r = 1; r < sh.world; ++r) {
        const std::string h = part_name(head, r, sh.world) + ".paths.k" + std::to_string(p.K);
        int pk = 0;
        uint64_t pn = 0, ni = 0, *po = nullptr, *ps = nullptr, *pl = nullptr;
        a.check(apg_kmerpaths_read(h.c_str(), &pk, &pn, &po, &ni, &ps, &pl), "reading KmerPath part");
        const uint64_t base = off.back();
        for (uint64_t i = 1; i <= pn; ++i) off.push_back(base + po[i] - po[0]);
        start.insert(start.end(), ps + po[0], ps + po[pn]);
        len.insert(len.end(), pl + po[0], pl + po[pn]);
        apg_free(po);
        apg_free(ps);
        apg_free(pl);
        std::remove(h.c_str());
      }
      // hand the joined arrays to the graph (malloc'd, freed with it)
      auto dup = [](const std::vector<uint64_t>& v) {
        auto* x = static_cast<uint64_t*>(std::malloc(std::max<size_t>(1, v.size()) * 8));
        if (!v.empty()) std::memcpy(x, v.data(), v.size() * 8);
        return x;
      };
      std::free(g.path_off);
      std::free(g.path_start);
      std::free(g.path_len);
      g.n_reads = off.size() - 1;
      g.n_intervals = start.size();
      g.path_off = dup(off);
      g.path_start = dup(start);
      g.path_len = dup(len);
    }
    sh.barrier(a);
  } else {
    a.check(apg_unipaths(ctx.c, &rd.r, &p, &g, &st), "apg_unipaths");
  }
  const int rc = apg_graph_write(head.c_str(), &g);
  apg_unipath_graph_free(&g);
  a.check(rc, "writing unipath files");
  std::printf("%s: K=%d %llu nodes, %llu unipaths, %llu HKP vertices%s -> %s.*.k%d\n", a.module.c_str(), p.K,
              (unsigned long long)st.n_nodes, (unsigned long long)st.n_unipaths, (unsigned long long)st.n_vertices,
              read_paths ? ", read paths" : "", head.c_str(), p.K);
  return 0;
}

int make_rc_db(Args& a) {
  const std::string dir = a.run_dir();
  const std::string head = dir + "/" + a.get("READS", "all_reads");
  const int K = (int)a.num("K", 96);
  a.finish();
  apg_unipath_graph g{};
  a.check(apg_graph_read(head.c_str(), K, &g), "reading unipath files (run CommonPather first)");
  if (!g.path_off) {
    apg_unipath_graph_free(&g);
    a.fail("no " + head + ".paths.k" + std::to_string(K) + " (run CommonPather first)");
  }
  Ctx ctx(a);
  apg_rc_db db;
  int rc = apg_make_rc_db(ctx.c, &g, &db);
  apg_unipath_graph_free(&g);
  a.check(rc, "apg_make_rc_db");
  rc = apg_rc_db_write(head.c_str(), K, &db);
  const unsigned long long ne = db.n_entries;
  apg_rc_db_free(&db);
  a.check(rc, "writing .paths_rc / .pathsdb");
  std::printf("%s: %llu index entries -> %s.{paths_rc,pathsdb}.k%d\n", a.module.c_str(), ne, head.c_str(), K);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  Args a;
  const char* slash = std::strrchr(argv[0], '/');
  a.module = slash ? slash + 1 : argv[0];
  int first = 1;
  if (a.module == "apg_modules") {  // apg_modules <Module> KEY=VALUE ...
    if (argc < 2) {
      std::fprintf(stderr,
                   "usage: apg_modules <KmerSpectrum|PreCorrect|FindErrors|FillFragments|ErrorCorrectJump|"
                   "MergeReadSets|CommonPather|Unipather|MakeRcDb|UnipathLocs|UnipathCoverage> KEY=VALUE ...\n");
      return 1;
    }
    a.module = argv[1];
    first = 2;
  }
  for (int i = first; i < argc; ++i) {
    const char* eq = std::strchr(argv[i], '=');
    if (!eq || eq == argv[i]) a.fail(std::string("argument '") + argv[i] + "' is not KEY=VALUE");
    a.kv[std::string(argv[i], eq - argv[i])] = eq + 1;
  }
  if (a.module == "KmerSpectrum") return kmer_spectrum(a);
  if (a.module == "PreCorrect") return precorrect(a, 1, "frag_reads_edit");
  if (a.module == "FindErrors") return precorrect(a, 2, "frag_reads_corr");
  if (a.module == "CommonPather") return unipaths(a, true);
  if (a.module == "Unipather") return unipaths(a, false);
  if (a.module == "MakeRcDb") return make_rc_db(a);
  if (a.module == "ErrorCorrectJump") return error_correct_jump(a);
  if (a.module == "FillFragments") return fill_fragments(a);
  if (a.module == "MergeReadSets") return merge_read_sets(a);
  if (a.module == "UnipathLocs") return unipath_locs(a);
  if (a.module == "UnipathCoverage") return unipath_coverage(a);
  a.fail("unknown module");
}
