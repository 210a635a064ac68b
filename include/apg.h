/*
 * apg.h — C ABI of libapg, the MI355X-native k-mer spectrum / correction /
 * unipath engine that stands in for ALLPATHS-LG's first-third pipeline modules.
 *
 * Boundary.  ALLPATHS-LG has no in-process plugin API: every
 * module is an executable driven by RunAllPathsLG with KEY=VALUE arguments,
 * exchanging .fastb/.qualb/... files in the RUN directory.  The reference
 * snapshot mounted for this project is EMPTY, so no file:line
 * exists to cite; each entry point below names the *recalled* module/function
 * it replaces ([R:M] = recalled, medium confidence — grep targets for when the
 * source appears).  The drop-in CLIs under tools/ call exactly these entries.
 *
 * Conventions
 *   - extern "C", plain pointers and sizes, no C++/torch types, no exceptions.
 *   - every function returns int: 0 = APG_OK, < 0 = APG_E_*; the message of the
 *     last failure on the calling thread is apg_last_error().
 *   - one context per host thread; a context owns one HIP device and stream.
 *   - calls are synchronous: when they return, outputs are complete.
 *   - "_dev" entry points take device-resident inputs (HBM) and are what the
 *     benchmark times; the plain forms take host buffers and include H2D/D2H.
 */
#ifndef APG_H
#define APG_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define APG_ABI_VERSION 1

enum {
  APG_OK = 0,
  APG_E_ARG = -1,      /* bad argument (null pointer, K out of range, ...) */
  APG_E_HIP = -2,      /* HIP runtime failure (no device, OOM, launch error) */
  APG_E_IO = -3,       /* file open/read/write failure or bad magic */
  APG_E_STATE = -4,    /* call out of order (e.g. table not built) */
  APG_E_NOMEM = -5,    /* host allocation failure */
  APG_E_UNSUPPORTED = -6
};

/* ------------------------------------------------------------------------- */
/* Context                                                                    */
/* ------------------------------------------------------------------------- */
typedef struct apg_ctx apg_ctx;

typedef struct apg_config {
  int32_t device;   /* HIP device ordinal */
  int32_t timing;   /* 1 = record per-kernel HIP-event durations */
  int32_t verbose;  /* 1 = stage log lines on stderr */
  int32_t kmer_dedup; /* K >= 21 bucket counts through record dedup:
                         0 = solid-set counts only (default), 1 = every count, 2 = never */
  uint64_t reserved[6];
} apg_config;

int apg_abi_version(void);
const char* apg_last_error(void);
int apg_create(const apg_config* cfg, apg_ctx** out);
void apg_destroy(apg_ctx* ctx);
/* Release every cached device workspace of the context. */
int apg_trim(apg_ctx* ctx);

/* Per-kernel timing (cfg.timing = 1).  idx enumerates kernels seen so far;
 * returns APG_E_ARG past the end.  bytes = algorithmic HBM bytes (inputs read
 * once + outputs written once) summed over the launches. */
int apg_timing_get(apg_ctx* ctx, int idx, char* name, size_t name_len,
                   double* total_ms, uint64_t* launches, uint64_t* bytes);
/* Device memory of the context (DESIGN.md §7 memory model): the workspaces it
 * holds now, the most it held at once since it was made or since the last
 * call with reset_peak = 1, how often a stage released dead buffers under
 * memory pressure, and the device's used / total bytes (all processes). */
typedef struct apg_mem_stats {
  uint64_t workspace_bytes;
  uint64_t workspace_peak;
  uint64_t releases;
  uint64_t device_used;
  uint64_t device_total;
  uint64_t reserved[3];
} apg_mem_stats;
int apg_mem_stats_get(apg_ctx* ctx, int reset_peak, apg_mem_stats* out);

/* Launches of kernel idx that ran on the context's side or auxiliary stream,
 * i.e. beside the main stream's kernels: their HIP-event time is a stretched,
 * shared-CU time, not a standalone kernel time. */
int apg_timing_overlapped(apg_ctx* ctx, int idx, uint64_t* overlapped);
int apg_timing_reset(apg_ctx* ctx);

/* ------------------------------------------------------------------------- */
/* Read sets (replaces vecbasevector / vecqualvector in memory;              */
/* [R:M] src/Basevector.h, src/Qualvector.h, src/feudal/)                    */
/*                                                                            */
/* Bases are 2-bit coded A=0 C=1 G=2 T=3, 4 per byte, base i of a read at     */
/* bits 2*(i%4) of byte i/4 (LSB first).  Every read starts on a byte         */
/* boundary: byte_off[i] = sum_{j<i} ceil(len_j/4).                           */
/* ------------------------------------------------------------------------- */
typedef struct apg_reads {
  uint64_t n_reads;
  const uint64_t* base_off; /* n_reads+1: read i = bases [base_off[i], base_off[i+1]) */
  const uint64_t* byte_off; /* n_reads+1: packed bytes of read i start at byte_off[i] */
  const uint8_t* packed;    /* byte_off[n_reads] bytes */
  const uint8_t* quals;     /* optional: base_off[n_reads] Phred bytes, or NULL */
} apg_reads;

/* Device-resident copy of a read set. */
typedef struct apg_dreads apg_dreads;
int apg_reads_upload(apg_ctx* ctx, const apg_reads* reads, apg_dreads** out);
void apg_reads_free(apg_dreads* dr);
uint64_t apg_dreads_count(const apg_dreads* dr);
/* Shape of a device read set (also one produced on the device, e.g. by     */
/* apg_fill_fragments_dev or apg_unibases_dev): sizes, and the offsets       */
/* copied to base_off / byte_off (n_reads + 1 each) when those are non-NULL. */
int apg_dreads_shape(apg_ctx* ctx, const apg_dreads* dr, uint64_t* n_reads, uint64_t* n_bases,
                     uint64_t* n_bytes, uint64_t* base_off, uint64_t* byte_off);
/* Copy bases (and qualities) between two device read sets of the same shape
 * (same read lengths), on the context's stream.  Used to restore a corrected
 * read set to its uploaded state without a host round trip. */
int apg_reads_copy_dev(apg_ctx* ctx, apg_dreads* dst, const apg_dreads* src);

/* Concatenate device read sets into one: ALLPATHS-LG's all_reads, the K=96
 * CommonPather input = filled fragments + corrected, trimmed jump reads
 * ([R:M] RunAllPathsLG's all_reads assembly ahead of CommonPather; SURVEY
 * §3(1), §8f #3; reference snapshot empty, no file:line).  Read i of
 * sets[s] becomes read (reads of sets[0..s)) + i; when d_keep and d_keep[s]
 * are non-NULL it is truncated to d_keep[s][i] bases (device u32, e.g. the
 * keep lengths of apg_error_correct_jump_dev).  No read is dropped (a read
 * trimmed to 0 stays as an empty read, so ids stay aligned with the inputs);
 * bases past a kept length are cleared.  Qualities are carried when every
 * input has them.  *out: NULL (allocated here; free with apg_reads_free) or
 * an earlier output of this call on ctx, whose buffers are reused. */
int apg_reads_concat_dev(apg_ctx* ctx, const apg_dreads* const* sets, const uint32_t* const* d_keep,
                         uint32_t n_sets, apg_dreads** out);

/* Device-to-device copy on the context's stream (synchronous): moves a
 * library-owned device output (e.g. apg_unipath_locs_dev) into a caller
 * buffer. */
int apg_device_copy(apg_ctx* ctx, void* d_dst, const void* d_src, uint64_t bytes);
/* Device-to-host copy (synchronous): a library-owned device output into
 * caller host memory (the drop-in modules' file writers). */
int apg_device_to_host(apg_ctx* ctx, void* h_dst, const void* d_src, uint64_t bytes);
/* Device buffers for the *_dev entry points' caller-owned arguments (keep
 * lengths, statuses, placements) without a HIP dependency in the caller:
 * bytes on ctx's device, zero-filled; release with apg_device_free. */
int apg_device_alloc(apg_ctx* ctx, uint64_t bytes, void** d_out);
void apg_device_free(apg_ctx* ctx, void* d);

/* Fill byte_off[0..n] from base_off[0..n]. */
int apg_byte_offsets(const uint64_t* base_off, uint64_t n_reads, uint64_t* byte_off);

/* ------------------------------------------------------------------------- */
/* K-mer counting and spectrum, K <= 32                                       */
/* Replaces: naif_kmerize + KernelKmerStorer ([R:M] src/kmers/naif_kmer/)     */
/* and KmerSpectrum ([R:M] src/kmers/KmerSpectra.h), module KmerSpectrum.     */
/*                                                                            */
/* Canonical k-mer = min(fw, rc) with fw = sum b[i+j]*4^(K-1-j). */
/* Table order: ascending apg_kmer_hash(K, canonical), a bijection on 2K bits */
/* (so the order is total and independent of bucketing / shard count).        */
/* Spectrum: hist[m] = #distinct canonical k-mers seen m times; the last bin  */
/* hist[hist_len-1] accumulates every m >= hist_len-1; hist[0] = 0.           */
/* ------------------------------------------------------------------------- */
typedef struct apg_kstats {
  uint64_t n_kmers;    /* k-mer instances (sum over reads of max(0, len-K+1)) */
  uint64_t n_distinct; /* distinct canonical k-mers */
  uint64_t n_buckets;  /* hash buckets used */
  uint64_t n_overflow; /* buckets sorted by the out-of-LDS fallback */
  uint64_t max_bucket; /* largest bucket (records); reported by the hash-table counter
                          (apg_kmer_count*), 0 from the super-k-mer spectrum paths */
  uint64_t n_redo;     /* buckets the record-deduplicating counter (K >= 21) handed
                          back to the per-instance counter */
  uint64_t reserved[2];
} apg_kstats;

uint64_t apg_kmer_hash(int K, uint64_t canonical);
uint64_t apg_kmer_unhash(int K, uint64_t hash);

int apg_kmer_spectrum(apg_ctx* ctx, const apg_reads* reads, int K,
                      uint64_t* hist, size_t hist_len, apg_kstats* stats);
int apg_kmer_spectrum_dev(apg_ctx* ctx, const apg_dreads* reads, int K,
                          uint64_t* hist, size_t hist_len, apg_kstats* stats);

/* Counted table (host outputs, library-allocated; release with apg_free).
 * keys[i] (canonical k-mers) in ascending apg_kmer_hash order, counts[i] >= 1. */
int apg_kmer_count(apg_ctx* ctx, const apg_reads* reads, int K,
                   uint64_t** keys, uint32_t** counts, uint64_t* n_distinct,
                   apg_kstats* stats);
void apg_free(void* p);

/* One parcel of the counted table of a device read set: the (canonical,
 * count) entries whose apg_kmer_hash lies in [hash_lo, hash_hi), in
 * ascending hash order (host outputs, release with apg_free).  The K-mer
 * space split into hash parcels is ALLPATHS-LG's way to bound the table's
 * memory ([R:M] src/kmers/KmerParcels.h).  hash_hi = 0 means no upper
 * bound, so (0, 0) is the whole table.
 * stats: the whole read set's counts. */
int apg_kmer_count_dev(apg_ctx* ctx, const apg_dreads* reads, int K, uint64_t hash_lo, uint64_t hash_hi,
                       uint64_t** keys, uint32_t** counts, uint64_t* n_out, apg_kstats* stats);

/* One hash-partition level of the counting pipelines (partition.hip: the
 * LDS-staged count / scan / scatter of NaifKmerizer's block split, [R:M]
 * src/kmers/naif_kmer/): the n device u64 records of d_in grouped by bits
 * [shift, shift + bits) into 2^bits child runs of d_out (order inside a child
 * unspecified); d_child (2^bits + 1 device u64) receives the runs' starts,
 * d_child[2^bits] = n.  0 <= bits <= 8 and shift + bits <= 64: APG_E_ARG
 * otherwise, with nothing launched (the kernels keep one LDS counter per
 * child).  Synchronous. */
int apg_partition_u64(apg_ctx* ctx, const uint64_t* d_in, uint64_t n, int shift, int bits, uint64_t* d_out,
                      uint64_t* d_child);

/* ------------------------------------------------------------------------- */
/* Sharded counting (multi-GPU, one process per GPU).  SURVEY §8e.            */
/* Records are 16-byte super-k-mers (runs of consecutive K-mers of a read    */
/* sharing one minimizer, with their bases).  Shard s owns the  */
/* K-mers whose minimizer key has top log2(P) bits == s — every instance of  */
/* a canonical K-mer has the same minimizer — and the next 5 bits are the     */
/* group (B = apg_shard_bins(K, P) = 32).  The caller moves bytes between     */
/* ranks (torch.distributed all_to_all over RCCL/xGMI).                       */
/*   1. apg_shard_count  : counts[s*B + g] of local reads' records           */
/*   2. apg_shard_scatter: records grouped by (s, g) into d_send (16 B each)  */
/*   3. (caller) all_to_all of counts, then of d_send -> d_recv (src-major)  */
/*   4. apg_shard_spectrum: count this shard's K-mers; recv_counts[src*B+g]  */
/* P must be a power of two, 1 <= P <= 8.  Spectra of the shards add up      */
/* (all_reduce sum) to the global spectrum.                                  */
/* ------------------------------------------------------------------------- */
int apg_shard_bins(int K, int n_shards);
int apg_shard_count(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards,
                    uint64_t* counts /* host, n_shards * apg_shard_bins */);
int apg_shard_scatter(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards,
                      void* d_send /* device, sum(counts) x 16 bytes */);
int apg_shard_spectrum(apg_ctx* ctx, const void* d_recv,
                       const uint64_t* recv_counts /* host, n_shards * bins */,
                       int K, int n_shards, uint64_t* hist, size_t hist_len,
                       apg_kstats* stats);

/* ------------------------------------------------------------------------- */
/* Communicators: the exchange of a sharded run, one process per GPU          */
/* (SURVEY §8e).  ALLPATHS-LG has no collective layer (single process,        */
/* OpenMP), so these replace nothing in it: they are what the      */
/* apg_sharded_* module entry points below exchange through.                  */
/*   rccl: device buffers over RCCL (xGMI): ranks share the 128-byte id of    */
/*         apg_comm_unique_id (made on one rank, passed to all by the         */
/*         launcher); grouped point-to-point transfers of <= 1 GiB pieces on  */
/*         the context's stream.  APG_COMM_SELF_P2P also routes the segment   */
/*         to self through RCCL (world-size-1 tests of the transport).        */
/*   tcp:  host sockets, full mesh through rank 0 at master_addr:master_port. */
/*         With a ctx, device buffers are staged through pinned host memory; */
/*         with ctx = NULL the buffers are host memory.  Several ranks may    */
/*         share one GPU (tests), and the drop-in CLIs use it to bootstrap.   */
/* Collectives are blocking; every rank must call them in the same order.     */
/* Byte counts are per peer and u64; segments are contiguous in rank order.   */
/* ------------------------------------------------------------------------- */
typedef struct apg_comm apg_comm;
#define APG_COMM_SELF_P2P 1u
enum { APG_COMM_SUM = 0, APG_COMM_MAX = 1 };
int apg_comm_unique_id(void* id128);
int apg_comm_init_rccl(apg_ctx* ctx, const void* id128, int rank, int world, uint32_t flags, apg_comm** out);
int apg_comm_init_tcp(apg_ctx* ctx /* or NULL: host buffers */, const char* master_addr, int master_port,
                      int rank, int world, int timeout_ms /* <= 0: 600 s */, apg_comm** out);
void apg_comm_destroy(apg_comm* comm);
/* Tear the communicator down after a local failure so that peers blocked in
 * a collective with this rank get an error instead of waiting: rccl aborts
 * the RCCL communicator (ncclCommAbort), tcp shuts its sockets down.  Every
 * later call on comm returns APG_E_STATE; apg_comm_destroy still frees it.
 * RCCL collectives wait on the stream while polling ncclCommGetAsyncError,
 * and give up (aborting) after APG_COMM_TIMEOUT_MS (default 600 000 ms). */
int apg_comm_abort(apg_comm* comm);
int apg_comm_rank(const apg_comm* comm);
int apg_comm_world(const apg_comm* comm);
/* send: world segments of send_bytes[q] bytes (segment q goes to rank q);
 * recv: world segments of recv_bytes[q] bytes (from rank q).  Sizes must
 * agree pairwise (checked on tcp). */
int apg_comm_alltoallv(apg_comm* comm, const void* send, const uint64_t* send_bytes, void* recv,
                       const uint64_t* recv_bytes);
/* recv: every rank's send_bytes in rank order (recv_bytes[q] from rank q). */
int apg_comm_allgatherv(apg_comm* comm, const void* send, uint64_t send_bytes, void* recv,
                        const uint64_t* recv_bytes);
/* In place on host memory: element-wise sum or max over ranks. */
int apg_comm_allreduce_u64(apg_comm* comm, uint64_t* data, uint64_t n, int op);
int apg_comm_barrier(apg_comm* comm);

/* ------------------------------------------------------------------------- */
/* Read error correction (restated; semantics unpinned).         */
/* Replaces module PreCorrect ([R:M-L] src/PreCorrect.cc; n_cycles = 1) and  */
/* the spectrum part of FindErrors ([R:M] src/FindErrors.cc,                  */
/* naif_kmer/KernelErrorFinder; n_cycles = 2, recounting between passes).    */
/*                                                                            */
/* Solid = canonical K-mer with count >= min_solid over the whole read set.  */
/* Per read, positions left to right on the current (partly corrected) read: */
/* a base with Q < max_q_suspect whose every covering K-mer is weak is       */
/* suspect; of the 3 alternatives (A<C<G<T) the unique one making every      */
/* covering K-mer solid replaces it and its Q becomes min(Q of neighbours);  */
/* ambiguous / no candidate: left unchanged.  Counts are fixed within a pass.*/
/* ------------------------------------------------------------------------- */
typedef struct apg_pc_params {
  int32_t K;               /* default 24 */
  uint32_t min_solid;      /* default 3 */
  uint32_t max_q_suspect;  /* default 20 */
  uint32_t n_cycles;       /* 1 = PreCorrect, 2 = FindErrors */
  uint64_t reserved[4];
} apg_pc_params;

typedef struct apg_pc_stats {
  uint64_t n_suspect;       /* suspect positions examined (summed over cycles) */
  uint64_t n_corrected;
  uint64_t n_ambiguous;     /* > 1 alternative made every covering K-mer solid */
  uint64_t n_uncorrectable; /* no alternative did */
  uint64_t n_solid;         /* solid K-mers of the last cycle */
  uint64_t record_form;     /* records of the context's last solid-set count:
                               0 = 24-byte SK24, 1 = packed 16-byte SKP (32-bit read-set
                               positions), 2 = packed wide SKP (34-bit positions: read sets of
                               2^32 .. 2^34 bases), 3 = received records by receive index
                               (the multi-GPU owner count) */
  uint64_t reserved[2];
} apg_pc_stats;

void apg_pc_defaults(apg_pc_params* p);
/* Host buffers: out_packed has reads->byte_off[n] bytes, out_quals
 * reads->base_off[n] bytes; reads->quals is required. */
int apg_precorrect(apg_ctx* ctx, const apg_reads* reads, const apg_pc_params* p,
                   uint8_t* out_packed, uint8_t* out_quals, apg_pc_stats* stats);
/* In place on a device read set (which must carry qualities). */
int apg_precorrect_dev(apg_ctx* ctx, apg_dreads* reads, const apg_pc_params* p,
                       apg_pc_stats* stats);
/* KmerSpectrum at K_spec + PreCorrect at p->K on the same device read set,
 * one counting pass: the spectrum is taken from the correction's K-mer
 * records before any base changes (each K_spec-mer counted once, by the
 * record holding the first K-mer of its canonical form).  Results equal
 * apg_kmer_spectrum_dev(reads, K_spec) followed by apg_precorrect_dev(reads,
 * p).  The fused path needs K_spec == p->K + 1 with both K-mer sizes walking
 * the same m-mers (true for 24 / 25, the module defaults); otherwise, and for
 * the later cycles of p->n_cycles > 1, the two run one after the other.
 * hist / stats as apg_kmer_spectrum_dev. */
int apg_spectrum_precorrect_dev(apg_ctx* ctx, apg_dreads* reads, int K_spec, uint64_t* hist, size_t hist_len,
                                apg_kstats* kstats, const apg_pc_params* p, apg_pc_stats* pstats);
/* Copy a device read set's (possibly corrected) bases/quals back to host
 * buffers of the upload's sizes (quals may be NULL). */
int apg_reads_download(apg_ctx* ctx, const apg_dreads* reads, uint8_t* packed, uint8_t* quals);

/* Multi-GPU correction (replicate the solid set, reads stay
 * sharded).  Per pass: apg_shard_count / apg_shard_scatter at K -> all_to_all
 * -> apg_shard_solid (this shard's solid K-mer hashes, unordered) ->
 * apg_solid_export into a device buffer -> all_gather -> apg_precorrect_solid
 * on every rank's own reads with the union.  The solid set is a set: the
 * gathered order does not change any result. */
int apg_shard_solid(apg_ctx* ctx, const void* d_recv, const uint64_t* recv_counts /* host */,
                    int K, int n_shards, uint32_t min_solid, uint64_t* n_solid);
/* d_out: device buffer of n_solid u64 (the hash of each solid K-mer). */
int apg_solid_export(apg_ctx* ctx, void* d_out);
/* Weak-mask return (the multi-GPU form of the weak-instance bitmap that the
 * single-GPU pass builds while counting):
 *   1. apg_shard_scatter_pos: as apg_shard_scatter, plus d_pos[i] (u64) =
 *      base position of sent record i's first K-mer (stays on this rank);
 *   2. (caller) all_to_all of the records, as for apg_shard_solid;
 *   3. apg_shard_solid_weak: this shard's solid set (apg_solid_export) and
 *      d_mask[i] (u32) = mask of received record i's K-mers with count <
 *      min_solid, in receive order;
 *   4. (caller) all_to_all of the masks back (splits reversed): each rank
 *      gets the masks of its sent records in send order;
 *   5. (caller) all_gather of the solid sets;
 *   6. apg_precorrect_weak: the per-base weak bitmap from (d_pos, d_mask),
 *      then one correction pass through it — no weak-test lookups, and the
 *      pass leaves the clean flags + extension table FillFragments reuses
 *      (APG_FILL_LAST_SOLID).  Results equal apg_precorrect_solid's.
 * K in [9, 29]. */
int apg_shard_scatter_pos(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards, void* d_send, void* d_pos);
int apg_shard_solid_weak(apg_ctx* ctx, const void* d_recv, const uint64_t* recv_counts /* host */, int K,
                         int n_shards, uint32_t min_solid, void* d_mask, uint64_t* n_solid);
int apg_precorrect_weak(apg_ctx* ctx, apg_dreads* reads, const apg_pc_params* p, const void* d_solid,
                        uint64_t n_solid, const void* d_pos, const void* d_mask, uint64_t n_records,
                        apg_pc_stats* stats);
/* The solid set (apg_kmer_hash values, any order) the last correction pass on
 * this context corrected against — what APG_FILL_LAST_SOLID uses.  d_out:
 * device buffer of *n_solid u64, or NULL to query the size. */
int apg_solid_copy(apg_ctx* ctx, void* d_out, uint64_t* n_solid);
/* The same set into host memory (out: *n_solid u64 in the set's device order,
 * or NULL to query the size) — what the PreCorrect / FindErrors modules write
 * as <HEAD_OUT>.solid.k<K> for the FillFragments module of another process. */
int apg_solid_download(apg_ctx* ctx, uint64_t* out, uint64_t* n_solid);
/* Install n solid hashes (host memory, apg_kmer_hash of canonical K-mers) as
 * the context's last correction pass's set for this K: APG_FILL_LAST_SOLID
 * (apg_fill_fragments*, apg_sharded_fill) then uses it.  Replaces any earlier
 * set and its extension table. */
int apg_solid_upload(apg_ctx* ctx, int K, const uint64_t* hashes, uint64_t n);
/* One correction pass (p->n_cycles is ignored) against the given solid
 * hashes (apg_kmer_hash of canonical K-mers, device memory). */
int apg_precorrect_solid(apg_ctx* ctx, apg_dreads* reads, const apg_pc_params* p,
                         const void* d_solid, uint64_t n_solid, apg_pc_stats* stats);

/* ------------------------------------------------------------------------- */
/* FillFragments (replaces module FillFragments, [R:M]   */
/* src/paths/FillFragments.cc — recalled, no line exists to cite): close     */
/* each overlapping / short-gap frag pair into the fragment it was read      */
/* from, the K=96 unipath stage's input.  Spec (semantics unpinned):         */
/*   pair i = reads (2i, 2i+1) = (A, B), FR; F = rc(B).  A closure of length */
/*   I is a sequence S with S[0,La) = A, S[I-Lf,I) = F (equal where they     */
/*   overlap), I in [max(min_insert, La, Lf), max_insert], and every K-mer   */
/*   of S solid — S is a path of the solid K-mer graph: A's and F's own      */
/*   K-mers and the "bridge" K-mers in neither (start in [La-K+1, I-Lf-1]).  */
/*   Exactly one closure: filled with S (A's orientation).                   */
/*   Search order: overlap lengths I < La+Lf ascending, then a depth-first   */
/*   walk from A's last K-1 bases over solid K-mers (bases A<C<G<T, depth    */
/*   d = I-La-Lf); per node the closure test, then the expansion; more than  */
/*   max_steps expansions -> BUDGET, a second closure -> AMBIGUOUS.          */
/*   Pairs with La or Lf < K, or max_insert-(La+Lf) > 63, are SKIP.          */
/* Solid set: hashes (apg_kmer_hash) of canonical K-mers, given by the       */
/* caller, or APG_FILL_LAST_SOLID = the set of this context's last           */
/* PreCorrect / FindErrors pass, or (neither) counted from the pairs         */
/* themselves with min_solid.                                                */
/* ------------------------------------------------------------------------- */
#define APG_FILL_OK 0
#define APG_FILL_NONE 1
#define APG_FILL_AMBIGUOUS 2
#define APG_FILL_BUDGET 3
#define APG_FILL_SKIP 4
#define APG_FILL_LAST_SOLID 1u

typedef struct apg_fill_params {
  int32_t K;            /* default 24, 2 <= K <= 29 */
  uint32_t min_insert;  /* default 126 (180 - 3 x 18) */
  uint32_t max_insert;  /* default 234 (180 + 3 x 18) */
  uint32_t max_steps;   /* walk expansions per pair, default 1024 */
  uint32_t min_solid;   /* default 3 (own-count mode only) */
  uint32_t flags;       /* APG_FILL_LAST_SOLID */
  uint64_t reserved[3];
} apg_fill_params;

typedef struct apg_fill_stats {
  uint64_t n_pairs;
  uint64_t n_filled;
  uint64_t n_none;
  uint64_t n_ambiguous;
  uint64_t n_budget;
  uint64_t n_skip;
  uint64_t filled_bases;
  uint64_t n_solid;   /* size of the solid set used */
  uint64_t lookups;   /* (K-1)-mer extension-table lookups (implementation statistic) */
  uint64_t reserved[3];
} apg_fill_stats;

void apg_fill_defaults(apg_fill_params* p);
/* Host buffers.  solid: n_solid hashes or NULL.  out: the filled fragments in
 * pair order (library-allocated, release with apg_reads_release; no quals).
 * status: n_reads/2 bytes (APG_FILL_*) or NULL. */
int apg_fill_fragments(apg_ctx* ctx, const apg_reads* pairs, const apg_fill_params* p,
                       const uint64_t* solid, uint64_t n_solid, apg_reads* out,
                       uint8_t* status, apg_fill_stats* stats);
/* Device variant.  d_solid: device hashes or NULL.  *filled: NULL (a new
 * device read set is created) or a previous output of this call on the same
 * context (its buffers are reused); release with apg_reads_free.  filled may
 * be NULL (stats only).  d_status: device n_pairs bytes or NULL. */
int apg_fill_fragments_dev(apg_ctx* ctx, const apg_dreads* pairs, const apg_fill_params* p,
                           const void* d_solid, uint64_t n_solid, apg_dreads** filled,
                           uint8_t* d_status, apg_fill_stats* stats);
/* KmerSpectrum + PreCorrect + FillFragments of the corrected pairs in one
 * call (the module chain of SURVEY.md:126-127 on device-resident reads):
 * results equal apg_spectrum_precorrect_dev(reads, K_spec, hist, ..., pp)
 * followed by apg_fill_fragments_dev(reads, fp | APG_FILL_LAST_SOLID, NULL,
 * 0, filled, d_status).  The fused K+1 spectrum count then runs beside
 * FillFragments' kernels as well as PreCorrect's, joined before the call
 * returns (hist / kstats complete on return).  fp->K must equal pp->K. */
int apg_spectrum_precorrect_fill_dev(apg_ctx* ctx, apg_dreads* reads, int K_spec, uint64_t* hist,
                                     size_t hist_len, apg_kstats* kstats, const apg_pc_params* pp,
                                     apg_pc_stats* pstats, const apg_fill_params* fp,
                                     apg_dreads** filled, uint8_t* d_status, apg_fill_stats* fstats);

/* ------------------------------------------------------------------------- */
/* Unipath graph, 1 <= K <= 96 (default 96).  Replaces CommonPather /        */
/* ReadsToPathsCoreX ([R:M] src/paths/ReadsToPathsCoreX.cc; .paths.kN),     */
/* MakeRcDb (.pathsdb.kN, see apg_pathsdb), Unipather ([R:M]                 */
/* src/paths/Unipath.cc; .unipaths.kN, .unibases.kN via KmerBaseBroker) and  */
/* the unipath adjacency -> HyperKmerPath ([R:M] src/paths/HyperKmerPath.h). */
/* Spec: SURVEY §A.5-A.6 made operational in DESIGN.md §Unipaths (node =     */
/* canonical K-mer of the reads, read-supported edges via extension bits,    */
/* palindromic K-mers never link, cycles cut before their min K-mer, pairs  */
/* (u, rc u) sorted by min(first K-mer of u, of rc u), contiguous k-mer ids).*/
/* ------------------------------------------------------------------------- */
typedef struct apg_unipath_params {
  int32_t K;       /* default 96 */
  uint32_t flags;  /* APG_UNIPATH_* */
  uint64_t reserved[4];
} apg_unipath_params;

#define APG_UNIPATH_READ_PATHS 1u /* also compute every read's KmerPath */
#define APG_UNIPATH_GATHER_NODES 2u /* apg_sharded_unipaths: gather every node to every
                                       rank and build the whole graph there (the replicated
                                       build) instead of the sharded compaction */

typedef struct apg_unipath_stats {
  uint64_t n_instances;  /* K-mer occurrences in the reads */
  uint64_t n_nodes;      /* distinct canonical K-mers */
  uint64_t n_links;      /* unique-successor links (directed) */
  uint64_t n_cycles_cut; /* cycle pairs broken */
  uint64_t n_unipaths;
  uint64_t n_vertices;   /* HyperKmerPath vertices */
  uint64_t n_intervals;  /* read-path intervals (if requested) */
  uint64_t max_len;      /* longest unipath (K-mers) */
} apg_unipath_stats;

/* Library-allocated outputs (release with apg_unipath_graph_free).  Unipath i
 * has len[i] K-mers with ids [id_base[i], id_base[i]+len[i]), reverse
 * complement partner rc[i] (== i when palindromic), bases
 * unibases[ub_off[i] .. ub_off[i+1]) (codes 0..3, K-1+len[i] of them), and is
 * HyperKmerPath edge from[i] -> to[i].  Read r's KmerPath is intervals
 * [path_off[r], path_off[r+1]) of (path_start, path_len). */
typedef struct apg_unipath_graph {
  int32_t K;
  int32_t reserved0;
  uint64_t n_nodes;
  uint64_t n_unipaths;
  uint64_t* len;
  uint64_t* id_base;
  uint64_t* rc;
  uint64_t* ub_off;
  uint8_t* unibases;
  uint64_t n_vertices;
  uint64_t* from;
  uint64_t* to;
  uint64_t n_reads;
  uint64_t* path_off;
  uint64_t n_intervals;
  uint64_t* path_start;
  uint64_t* path_len;
} apg_unipath_graph;

void apg_unipath_defaults(apg_unipath_params* p);
int apg_unipaths(apg_ctx* ctx, const apg_reads* reads, const apg_unipath_params* p,
                 apg_unipath_graph* out, apg_unipath_stats* stats);
/* out may be NULL: build on the device, report stats only (benchmark). */
int apg_unipaths_dev(apg_ctx* ctx, const apg_dreads* reads, const apg_unipath_params* p,
                     apg_unipath_graph* out, apg_unipath_stats* stats);
void apg_unipath_graph_free(apg_unipath_graph* g);

/* Sharded unipath build (multi-GPU, one process per GPU).  Each
 * rank first reduces its own reads' K-mer instances to distinct local nodes
 * (32-byte records: 3 x u64 canonical key + hash56/extension-bits word), so
 * the exchange carries distinct K-mers, not instances.  Nodes are
 * hash-sharded like the spectrum: shard = top log2(P) bits of the 5-bit node
 * digit, B = apg_ushard_bins(P) groups per shard.
 *   1. apg_ushard_count / apg_ushard_scatter: local reads -> local nodes,
 *      grouped by digit, -> d_send
 *   2. (caller) all_to_all of counts, then of records -> d_recv (src-major)
 *   3. apg_ushard_nodes: this shard's distinct nodes (key + OR of ext bits
 *      over every rank's local nodes)
 *   4. apg_ushard_export -> (caller) all_gather of every shard's nodes
 *   5. apg_unipaths_from_nodes: the graph of the full node set (identical on
 *      every rank) + KmerPaths of this rank's reads.
 * Node sets of different shards are disjoint, so their concatenation in any
 * order gives the same graph as apg_unipaths on all reads. */
int apg_ushard_bins(int n_shards);
int apg_ushard_count(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards,
                     uint64_t* counts /* host, 32 entries: local nodes per digit, shard-major */,
                     uint64_t* n_instances /* may be NULL: K-mer instances of the reads */);
int apg_ushard_scatter(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards,
                       void* d_send /* device, sum(counts) x 32 bytes */);
int apg_ushard_nodes(apg_ctx* ctx, const void* d_recv, const uint64_t* recv_counts /* 32 */,
                     int K, int n_shards, uint64_t* n_nodes);
int apg_ushard_export(apg_ctx* ctx, void* d_out /* device, n_nodes x 32 bytes */);
int apg_unipaths_from_nodes(apg_ctx* ctx, const void* d_nodes, uint64_t n_nodes,
                            const apg_dreads* reads /* KmerPaths for these, or NULL */,
                            const apg_unipath_params* p, apg_unipath_graph* out,
                            apg_unipath_stats* stats);

/* Sharded unipath nodes through minimizer partitions (the multi-GPU form of
 * the single-GPU node build).  Records are 48-byte super-k-mers
 * (runs of K-mers sharing a minimizer, with their extension bases); shard =
 * top log2(P) bits of the minimizer key, 32 digit groups per shard:
 *   1. apg_urec_count: records per (shard, digit) into counts[P * 32]
 *      (dest-major) and the reads' K-mer instances;
 *   2. apg_urec_scatter: the records, grouped by (shard, digit) -> d_send;
 *   3. (caller) all_to_all of counts, then of records -> d_recv (src-major);
 *   4. apg_urec_nodes: this shard's distinct nodes (32-byte records as in
 *      apg_ushard_export) from the received records; apg_urec_export;
 *   5. (caller) all_gather of the node sets -> apg_unipaths_from_nodes.
 * A K-mer's instances share its minimizer, so shards never share a node; the
 * union over shards equals apg_unipaths' node set. */
int apg_urec_count(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards,
                   uint64_t* counts /* host, n_shards * 32 */, uint64_t* n_instances /* may be NULL */);
int apg_urec_scatter(apg_ctx* ctx, const apg_dreads* reads, int K, int n_shards,
                     void* d_send /* device, sum(counts) x 48 bytes */);
int apg_urec_nodes(apg_ctx* ctx, const void* d_recv, const uint64_t* recv_counts /* host, n_shards * 32 */,
                   int K, int n_shards, uint64_t* n_nodes);
int apg_urec_export(apg_ctx* ctx, void* d_out /* device, n_nodes x 32 bytes */);

/* ------------------------------------------------------------------------- */
/* MakeRcDb ([R:M] tagged_rpint; <reads>.paths_rc.kN, <reads>.pathsdb.kN).    */
/* From a graph with read paths (apg_unipaths with APG_UNIPATH_READ_PATHS):   */
/*  - rc paths: each read path walked backwards, every id mapped into the rc  */
/*    partner unipath (offset o of u <-> offset len(u)-1-o of rc(u)),         */
/*    consecutive ids merged into intervals;                                  */
/*  - index: every interval of every forward path (read order, interval       */
/*    order), then every interval of every rc path, stably sorted by start.  */
/* ------------------------------------------------------------------------- */
#define APG_RPINT_RC 1u
typedef struct apg_rpint {
  uint64_t start; /* first K-mer id of the interval */
  uint32_t len;
  uint32_t read;  /* read index */
  uint32_t pos;   /* interval index within the read's (fw or rc) path */
  uint32_t flags; /* APG_RPINT_RC: interval of the read's rc path */
} apg_rpint;

typedef struct apg_rc_db {
  uint64_t n_reads;
  uint64_t* rc_path_off;    /* n_reads + 1 */
  uint64_t n_rc_intervals;
  uint64_t* rc_start;
  uint64_t* rc_len;
  uint64_t n_entries;       /* fw + rc intervals */
  apg_rpint* entries;       /* sorted by start (stable) */
} apg_rc_db;

int apg_make_rc_db(apg_ctx* ctx, const apg_unipath_graph* g, apg_rc_db* out);
void apg_rc_db_free(apg_rc_db* db);

/* ------------------------------------------------------------------------- */
/* Read-to-unibase alignment and column consensus (restated;    */
/* semantics unpinned).  Replaces the aligners feeding CRefMerger /          */
/* LongReadConsensus ([R:M] src/pairwise_aligners/PerfectAlignment*,         */
/* KmerAligner, SmithWatBanded.cc; [R:L] CRefMerger / LongReadConsensus).    */
/*                                                                            */
/* S / R = query reads (an apg_reads / device read set), T = targets (e.g.   */
/* unibases, same packed layout).  A pair places S (its reverse complement   */
/* with APG_ALN_RC) against T so that S[0] faces T[offset].                  */
/* ------------------------------------------------------------------------- */
#define APG_ALN_RC 1u
typedef struct apg_aln_pair {
  uint32_t s_id;
  uint32_t t_id;
  int32_t offset;
  uint32_t flags; /* APG_ALN_RC */
} apg_aln_pair;

/* Gap-free: over the overlap of S and T at the offset, mismatches = popcount
 * of the 2-bit difference mask, qsum = sum of S's qualities at mismatches
 * (0 when S has no qualities).  offset is echoed. */
typedef struct apg_gapfree_hit {
  uint32_t overlap;
  uint32_t mismatches;
  uint32_t qsum;
  int32_t offset;
} apg_gapfree_hit;
int apg_gapfree(apg_ctx* ctx, const apg_reads* S, const apg_reads* T, const apg_aln_pair* pairs,
                uint64_t n, apg_gapfree_hit* out);
/* Device variant: pairs / out are device buffers; ids must be in range. */
int apg_gapfree_dev(apg_ctx* ctx, const apg_dreads* S, const apg_dreads* T,
                    const apg_aln_pair* d_pairs, uint64_t n, apg_gapfree_hit* d_out);

/* Banded Smith-Waterman, SmithWatBanded semantics as restated: all of S is
 * aligned, T has free ends; only cells on diagonals d = j - i in
 * [offset - w, offset + w] exist.  Integer costs: mismatch 2, gap 3 per base;
 * minimise.  Ties: diagonal > gap in S (T base unmatched) > gap in T (S base
 * unmatched); among equal end cells the smallest T end wins.
 * blocks (optional, max_blocks (gap, len) int32 pairs per pair): the
 * alignment as runs of aligned columns, each preceded by its gap (> 0: T
 * bases skipped, < 0: S bases skipped); trailing gaps make a final (gap, 0).
 * status: 0 ok, 1 no cell of the band reaches the end of S, 2 more blocks
 * than max_blocks (n_blocks still exact).  band_w <= 127. */
typedef struct apg_sw_hit {
  int32_t cost;
  int32_t t_begin; /* T position of the first aligned S base / gap */
  int32_t t_end;   /* one past the last T base used */
  int32_t mismatches;
  int32_t gaps_s;  /* T bases against gaps */
  int32_t gaps_t;  /* S bases against gaps */
  int32_t n_blocks;
  int32_t status;
} apg_sw_hit;
int apg_banded_sw(apg_ctx* ctx, const apg_reads* S, const apg_reads* T, const apg_aln_pair* pairs,
                  uint64_t n, int band_w, apg_sw_hit* out, int32_t* blocks /* may be NULL */,
                  uint32_t max_blocks);
int apg_banded_sw_dev(apg_ctx* ctx, const apg_dreads* S, const apg_dreads* T,
                      const apg_aln_pair* d_pairs, uint64_t n, int band_w, apg_sw_hit* d_out,
                      int32_t* d_blocks, uint32_t max_blocks);

/* Column consensus of reads placed gap-free on targets (pairs = placements):
 * every placed base votes its quality for its base at target column
 * offset + i; per column the largest vote sum wins, ties go to the target's
 * own base, then to the smaller base code; quality = min(60, winner sum -
 * best other sum).  Columns without votes keep the target base, Q = 0.
 * bases / quals: one byte per target base (target set's base order). */
int apg_consensus(apg_ctx* ctx, const apg_reads* R, const apg_reads* T, const apg_aln_pair* placements,
                  uint64_t n, uint8_t* bases, uint8_t* quals);
int apg_consensus_dev(apg_ctx* ctx, const apg_dreads* R, const apg_dreads* T,
                      const apg_aln_pair* d_placements, uint64_t n, uint8_t* d_bases, uint8_t* d_quals);

/* ------------------------------------------------------------------------- */
/* ErrorCorrectJump ([R:M] src/paths/ErrorCorrectJump.cc, grep target only: */
/* reference snapshot empty; semantics unpinned).  Spec [D]:                */
/*  - the solid set is counted on the FRAGMENT reads (canonical K-mers with  */
/*    count >= min_solid): a jump library's coverage is too low to count;    */
/*  - one PreCorrect pass (SURVEY §A.4 rule) of the jump reads against it;   */
/*  - trimming: each corrected jump read keeps its longest prefix whose      */
/*    K-mers are all solid — keep = L if every K-mer is solid, else          */
/*    j0 + K - 1 for the first non-solid K-mer j0; keep = 0 when L < K or    */
/*    keep < min_keep (the read is dropped; pairs keep their indices).       */
/* Bases and qualities are corrected in place; keep_len[r] gives the trim.   */
/* ------------------------------------------------------------------------- */
typedef struct apg_ecj_params {
  int32_t K;               /* default 24 */
  uint32_t min_solid;      /* default 3 */
  uint32_t max_q_suspect;  /* default 20 */
  uint32_t min_keep;       /* default 40 */
  uint64_t reserved[4];
} apg_ecj_params;

typedef struct apg_ecj_stats {
  apg_pc_stats pc;      /* the correction pass of the jump reads */
  uint64_t n_reads;
  uint64_t n_full;      /* every K-mer solid: not trimmed */
  uint64_t n_trimmed;   /* cut to a prefix >= min_keep */
  uint64_t n_dropped;   /* keep = 0 */
  uint64_t bases_kept;
  uint64_t reserved[3];
} apg_ecj_stats;

void apg_ecj_defaults(apg_ecj_params* p);
/* Host variant: frags / jumps in host memory; out_packed / out_quals sized  */
/* like jumps (corrected, untrimmed layout), keep_len: one u32 per jump read. */
int apg_error_correct_jump(apg_ctx* ctx, const apg_reads* frags, const apg_reads* jumps,
                           const apg_ecj_params* p, uint8_t* out_packed, uint8_t* out_quals,
                           uint32_t* keep_len, apg_ecj_stats* stats);
/* Device variant: jumps corrected in place; d_keep_len device, n_reads u32. */
int apg_error_correct_jump_dev(apg_ctx* ctx, const apg_dreads* frags, apg_dreads* jumps,
                               const apg_ecj_params* p, uint32_t* d_keep_len, apg_ecj_stats* stats);

/* ------------------------------------------------------------------------- */
/* UnipathLocs: placement of reads on the unipaths of the context's last     */
/* unipath build (apg_unipaths / apg_unipaths_dev / apg_unipaths_from_nodes; */
/* after the latter, the caller's node buffer must still be alive).          */
/* Replaces BuildUnipathLocs / ReadLocationLG ([R:M] src/paths/UnipathLocs*, */
/* grep target only: reference snapshot empty).  Spec [D]:                   */
/*  - every K-mer j of read r (read orientation) found in the graph lies at   */
/*    rank k of exactly one unipath u: the read is placed at start s = k - j */
/*    (read base 0 faces unibase base s; s may be negative or run past the  */
/*    end, as for reads hanging off a unipath end);                          */
/*  - a location {s_id = r, t_id = u, offset = s, flags = 0} is emitted for  */
/*    each K-mer whose (u, s) differs from the read's last emitted (u, s);   */
/*    K-mers absent from the graph are skipped (counted in n_missing);       */
/*  - APG_ULOCS_RC: each location is followed by its mirror on rc(u):       */
/*    {r, rc(u), (len(u) + K - 1) - (s + L_r), APG_ALN_RC};                  */
/*  - order: read order, emission order; APG_ULOCS_SORTED: stably sorted by  */
/*    (t_id, offset) — the by-unipath index.                                 */
/* Locations are apg_aln_pair placements: they feed apg_gapfree /            */
/* apg_banded_sw / apg_consensus against the unibases (apg_unibases_dev).    */
/* ------------------------------------------------------------------------- */
#define APG_ULOCS_RC 1u
#define APG_ULOCS_SORTED 2u
typedef struct apg_uloc_stats {
  uint64_t n_reads;
  uint64_t n_placed;  /* reads with >= 1 location */
  uint64_t n_locs;
  uint64_t n_missing; /* read K-mers absent from the graph */
} apg_uloc_stats;
/* Host variant: *locs is malloc'd (release with apg_free). */
int apg_unipath_locs(apg_ctx* ctx, const apg_reads* reads, uint32_t flags, apg_aln_pair** locs,
                     uint64_t* n_locs, apg_uloc_stats* stats);
/* Device variant: *d_locs points into a context workspace, valid until the  */
/* next apg_unipath_locs* call or apg_trim. */
int apg_unipath_locs_dev(apg_ctx* ctx, const apg_dreads* reads, uint32_t flags, const apg_aln_pair** d_locs,
                         uint64_t* n_locs, apg_uloc_stats* stats);
/* The last build's unibases as a new device read set (one read per unipath, */
/* no qualities; release with apg_reads_free) — the aligners' targets. */
int apg_unibases_dev(apg_ctx* ctx, apg_dreads** out);

/* ------------------------------------------------------------------------- */
/* UnipathCoverage: read coverage and copy number per unipath of the          */
/* context's last unipath build, from UnipathLocs placements.  Replaces the  */
/* coverage / copy-number half of UnipathCoverage ([R:M]                     */
/* src/paths/UnipathCoverage*, grep target only: reference snapshot empty).  */
/* Spec [D] (restated; CPU restatement oracle/ucov_oracle.c):                */
/*  - n[u]   = placements with t_id == u (every location counts once; with   */
/*             APG_ULOCS_RC mirrors n[u] == n[rc(u)]);                        */
/*  - cov[u] = (double)n[u] / (double)len[u]  (placements per K-mer, IEEE);  */
/*  - c0     = length-weighted median of cov over the unipaths with len >=   */
/*             min_len: cov values ascending, the first whose cumulative     */
/*             length L satisfies 2 L >= the total length (0 if none);       */
/*  - cn[u]  = c0 > 0 ? floor(cov[u] / c0 + 0.5) : 0  (copy-number estimate; */
/*             0 = under half the genome-wide coverage, e.g. error paths).   */
/* Counting runs on the device (wave-aggregated runs of equal unipath ids);  */
/* the median over the <= n_unipaths long unipaths is selected on the host.  */
/* ------------------------------------------------------------------------- */
typedef struct apg_ucov_params {
  uint64_t min_len; /* default 500 K-mers */
  uint64_t reserved[3];
} apg_ucov_params;
typedef struct apg_ucov_stats {
  double c0;         /* genome-wide placements per K-mer */
  uint64_t n_long;   /* unipaths with len >= min_len */
  uint64_t n_locs;
  uint64_t n_bad;    /* placements whose t_id is not a unipath (rejected: error) */
} apg_ucov_stats;
void apg_ucov_defaults(apg_ucov_params* p);
/* d_locs: n_locs placements in device memory (apg_unipath_locs_dev).  Host */
/* outputs, caller-allocated with n_unipaths entries each (any may be NULL). */
int apg_unipath_coverage_dev(apg_ctx* ctx, const apg_aln_pair* d_locs, uint64_t n_locs, const apg_ucov_params* p,
                             uint64_t* counts, double* cov, uint32_t* copy_number, apg_ucov_stats* stats);
/* Host placements (uploaded). */
int apg_unipath_coverage(apg_ctx* ctx, const apg_aln_pair* locs, uint64_t n_locs, const apg_ucov_params* p,
                         uint64_t* counts, double* cov, uint32_t* copy_number, apg_ucov_stats* stats);
/* Files (see apg_solid_write): <head>.unilocs.k<K>, <head>.unipath_cov.k<K>. */
int apg_ulocs_write(const char* path, int K, uint64_t n_reads, const apg_aln_pair* locs, uint64_t n_locs);
int apg_ulocs_read(const char* path, int* K, uint64_t* n_reads, apg_aln_pair** locs, uint64_t* n_locs);
int apg_ucov_write(const char* path, int K, double c0, uint64_t n_unipaths, const uint64_t* counts,
                   const double* cov, const uint32_t* copy_number);
int apg_ucov_read(const char* path, int* K, double* c0, uint64_t* n_unipaths, uint64_t** counts, double** cov,
                  uint32_t** copy_number);

/* ------------------------------------------------------------------------- */
/* Sharded module entry points (multi-GPU, one process per GPU):  */
/* the same modules over the union of every rank's reads, every exchange     */
/* through `comm` (which must have been made for ctx).  Each rank passes its */
/* own reads (whole pairs); results equal the single-GPU entry points on the */
/* union (tests/test_distributed.py):                                        */
/*   spectrum   the global spectrum on every rank; stats summed              */
/*   precorrect every rank's reads corrected in place against the global     */
/*              solid set (which stays on the context for                    */
/*              APG_FILL_LAST_SOLID); stats summed, n_solid global           */
/*   spectrum_precorrect  both of the above from ONE exchange of K-records    */
/*              (K_spec = p.K + 1, as apg_spectrum_precorrect_dev); falls     */
/*              back to the two entry points when not fusable                 */
/*   fill       this rank's pairs (no exchange); stats summed                */
/*   unipaths   the global graph (identical on every rank, out may be NULL)  */
/*              + KmerPaths of this rank's reads; n_instances summed         */
/* World size: a power of two <= 8 (spectrum, PreCorrect) / <= 32 (unipaths).*/
/* ------------------------------------------------------------------------- */
int apg_sharded_spectrum(apg_ctx* ctx, apg_comm* comm, const apg_dreads* reads, int K, uint64_t* hist,
                         size_t hist_len, apg_kstats* stats);
int apg_sharded_precorrect(apg_ctx* ctx, apg_comm* comm, apg_dreads* reads, const apg_pc_params* p,
                           apg_pc_stats* stats);
int apg_sharded_spectrum_precorrect(apg_ctx* ctx, apg_comm* comm, apg_dreads* reads, int K_spec, uint64_t* hist,
                                    size_t hist_len, apg_kstats* kstats, const apg_pc_params* p,
                                    apg_pc_stats* pstats);
int apg_sharded_fill(apg_ctx* ctx, apg_comm* comm, const apg_dreads* pairs, const apg_fill_params* p,
                     const void* d_solid, uint64_t n_solid, apg_dreads** filled, uint8_t* d_status,
                     apg_fill_stats* stats);
int apg_sharded_unipaths(apg_ctx* ctx, apg_comm* comm, const apg_dreads* reads, const apg_unipath_params* p,
                         apg_unipath_graph* out, apg_unipath_stats* stats);
/* ErrorCorrectJump of this rank's jump reads against the GLOBAL solid set  */
/* of every rank's fragment reads (replaces ErrorCorrectJump [R:M]          */
/* src/paths/ErrorCorrectJump.cc in the sharded flow; grep target only:      */
/* reference snapshot empty).  When `frags` are the output of this context's */
/* last apg_sharded_(spectrum_)precorrect over `comm` (same K, min_solid),   */
/* that pass's replicated solid set is reused (a pass leaves the solid set  */
/* unchanged), else it is counted across the ranks first.  Jump reads are    */
/* corrected in place and trimmed exactly as apg_error_correct_jump_dev      */
/* does on the union; stats summed over ranks (pc.n_solid: the global set).  */
int apg_sharded_error_correct_jump(apg_ctx* ctx, apg_comm* comm, const apg_dreads* frags, apg_dreads* jumps,
                                   const apg_ecj_params* p, uint32_t* d_keep_len, apg_ecj_stats* stats);
/* Read placement and consensus after a sharded build (SURVEY §8e
 * "alignment": unibases replicated, reads sharded) — the multi-GPU forms of
 * apg_unipath_locs_dev and apg_consensus_dev (BuildUnipathLocs /
 * ReadLocationLG and the aligners feeding CRefMerger / LongReadConsensus,
 * [R:M]/[R:L]; reference snapshot empty, no file:line).
 *   unipath_locs  this rank's reads on the global graph of the last
 *                 apg_sharded_unipaths on ctx (same comm): every K-mer the
 *                 rank does not own is resolved by one query to its owner
 *                 shard; the locations are exactly apg_unipath_locs' for
 *                 these reads on the single-GPU graph (s_id = index in
 *                 reads).  *d_locs: context workspace, valid until the next
 *                 locs call.  stats summed over ranks.
 *   consensus     every rank's placements of its own reads vote on the
 *                 replicated targets (e.g. apg_unibases_dev, which works after
 *                 a sharded build); the vote planes are summed over the ranks
 *                 (in <= 2^28-column chunks) and every rank gets the consensus
 *                 of every target column = apg_consensus_dev of the union.
 * Gap-free / banded alignment of the placements needs no exchange
 * (apg_gapfree_dev / apg_banded_sw_dev on each rank). */
int apg_sharded_unipath_locs(apg_ctx* ctx, apg_comm* comm, const apg_dreads* reads, uint32_t flags,
                             const apg_aln_pair** d_locs, uint64_t* n_locs, apg_uloc_stats* stats);
int apg_sharded_consensus(apg_ctx* ctx, apg_comm* comm, const apg_dreads* R, const apg_dreads* T,
                          const apg_aln_pair* d_placements, uint64_t n, uint8_t* d_bases, uint8_t* d_quals);

/* ------------------------------------------------------------------------- */
/* Synthetic reads: uniform iid genome, frag pairs 100 bp,       */
/* insert N(mean, sd), FR orientation, substitution error rate rising        */
/* linearly err_lo -> err_hi along the read; Q40 on correct bases, Q2..20 on */
/* errors.  Deterministic per (seed, read index): any shard regenerates its  */
/* slice.  Host-only (no GPU).                                               */
/* ------------------------------------------------------------------------- */
typedef struct apg_synth_params {
  uint64_t genome_len;
  uint64_t seed;
  uint64_t n_pairs;
  uint32_t read_len;
  uint32_t insert_mean;
  uint32_t insert_sd;
  uint32_t threads;     /* 0 = hardware concurrency */
  double err_lo;
  double err_hi;
  uint64_t first_pair;  /* generate pairs [first_pair, first_pair+n_pairs) */
} apg_synth_params;

/* Genome (2 bits/base, one byte per base in out) */
int apg_synth_genome(uint64_t genome_len, uint64_t seed, uint8_t* out_bases);
/* Repeats injected into a synthetic genome (in place, deterministic per     */
/* seed): interspersed families — a random consensus of family_len[f] bases, */
/* copies at random positions until family_frac[f] of the genome is covered, */
/* each copy substituted at rate family_div[f] — and tandem arrays (a random */
/* unit of 1..tandem_unit_max bases repeated to 2 units .. tandem_array_max  */
/* bases, 1 % substitutions) covering tandem_frac.  Real genomes are not in  */
/* the container; this gives the counting stages skewed buckets, */
/* high-count K-mers and collapsed / cyclic unipaths at scale.               */
#define APG_MAX_REPEAT_FAMILIES 8
typedef struct apg_repeat_params {
  uint32_t n_families;
  uint32_t tandem_unit_max;
  uint32_t family_len[APG_MAX_REPEAT_FAMILIES];
  double family_frac[APG_MAX_REPEAT_FAMILIES];
  double family_div[APG_MAX_REPEAT_FAMILIES];
  double tandem_frac;
  uint32_t tandem_array_max;
  uint32_t reserved0;
} apg_repeat_params;
/* A human-like mix: 300-bp family over 10 % at 12 % divergence (Alu-like),  */
/* 6-kb family over 5 % at 4 % (L1-like), 1-kb family over 0.5 % at 0.2 %   */
/* (young, near-identical copies), tandem arrays over 1 % (units <= 60 bp,  */
/* arrays <= 4 kb).                                                          */
void apg_repeat_defaults(apg_repeat_params* p);
int apg_synth_repeats(uint64_t genome_len, uint64_t seed, const apg_repeat_params* p, uint8_t* genome);
/* Sizes for a synth call: n_reads = 2*n_pairs, packed bytes. */
int apg_synth_sizes(const apg_synth_params* p, uint64_t* n_reads, uint64_t* n_bases,
                    uint64_t* n_packed_bytes);
/* Writes base_off[n+1], byte_off[n+1], packed[], quals[] (quals may be NULL). */
int apg_synth_reads(const apg_synth_params* p, const uint8_t* genome,
                    uint64_t* base_off, uint64_t* byte_off, uint8_t* packed,
                    uint8_t* quals);
/* Simulator truth of each pair (test / bench infrastructure): its fragment's
 * genome start, length and strand (flip = 1: read A is the reverse strand),
 * the same draws apg_synth_reads makes for that pair. */
int apg_synth_layout(const apg_synth_params* p, uint64_t* start, uint32_t* flen, uint8_t* flip);
/* The error-free fragment (insert) of each pair, in read A's orientation: the
 * "oracle fill" standing in for FillFragments (SURVEY §8d K=96 caveat) until
 * that module exists.  Call once with packed = NULL to get base_off/byte_off
 * (n_pairs + 1 each), then again with the same offsets and packed sized
 * byte_off[n_pairs] (+ slack) to fill the bases. */
int apg_synth_fragments(const apg_synth_params* p, uint64_t* base_off, uint64_t* byte_off,
                        const uint8_t* genome, uint8_t* packed);

/* ------------------------------------------------------------------------- */
/* On-disk formats ("APG-fastb v0"; feudal byte layout unpinned) */
/* ------------------------------------------------------------------------- */
int apg_fastb_write(const char* path, const apg_reads* reads);
int apg_qualb_write(const char* path, const apg_reads* reads);
/* Library-allocated; free with apg_reads_release. */
int apg_fastb_read(const char* path, apg_reads* out);
int apg_qualb_read(const char* path, apg_reads* inout /* fills quals */);
void apg_reads_release(apg_reads* r);
/* .fastb (+ optional .qualb, NULL for none) straight into a device read set:
 * the module-boundary input of a drop-in stage ([R:M] the RUN-dir
 * frag_reads_*.fastb / .qualb every module opens; src/feudal/).  Offsets are
 * read and validated as by apg_fastb_read / apg_qualb_read; the payloads go
 * file -> pinned staging -> HBM in 16 MiB chunks, `threads` workers (<= 0:
 * min(16, hardware threads)) each double-buffering pread against its own H2D
 * stream.  Same device read set as apg_fastb_read + apg_qualb_read +
 * apg_reads_upload; free with apg_reads_free.  The call returns once the
 * offsets and bases are in HBM: the qualities (4/5 of the bytes) keep
 * streaming in on a host thread of the context while the next module counts
 * the bases, and every entry point that reads them (PreCorrect / FindErrors /
 * ErrorCorrectJump, apg_reads_copy_dev, apg_reads_download,
 * apg_reads_concat_dev, the aligners, apg_reads_free, apg_trim,
 * apg_destroy) waits for that load first; a read error found there is that
 * call's error (APG_E_IO).  Environment APG_LOAD_SYNC=1: loaded before the
 * call returns. */
int apg_reads_load_dev(apg_ctx* ctx, const char* fastb, const char* qualb, int threads, apg_dreads** out);
/* Spectrum text file (.kspec): "m\tcount" lines for nonzero bins, after
 * '#' header lines that carry apg_kspec_estimate's summary. */
int apg_kspec_write(const char* path, int K, const uint64_t* hist, size_t hist_len);

/* Genome-size estimate from a K-mer spectrum — the figure KmerSpectrum
 * reports beside h[m] ([R:M] src/kmers/KmerSpectra.h: the spectrum "also
 * feeds genome-size/ploidy estimates", SURVEY.md:82; reference snapshot
 * empty, grep target only).  Host-only.  Spec [D] (restated; the oracle's
 * ork_kspec_estimate is the checker):
 *   valley v     = the smallest m in [1, hist_len-2) with hist[m] < hist[m+1]
 *                  (where the error K-mers' decline ends); 0 if none;
 *   peak p       = the smallest m in (v, hist_len-1) with the largest hist[m]
 *                  (the K-mer coverage of single-copy sequence); 0 if v = 0 or
 *                  that maximum is 0;
 *   genomic_kmers     = sum over v <= m < hist_len of hist[m];
 *   genomic_instances = sum over v <= m < hist_len of m * hist[m] (the last
 *                       bin counts as m = hist_len-1);
 *   error_kmers / error_instances: the same sums over 1 <= m < v;
 *   coverage     = S1 / S0 with S1 = sum m * hist[m], S0 = sum hist[m] over
 *                  v <= m <= min(2p - v, hist_len - 2): the mean K-mer
 *                  coverage of the single-copy peak (its mode p sits below
 *                  the mean, by up to 1/p of it);
 *   genome_size  = round(genomic_instances / coverage) = (genomic_instances *
 *                  S0 + S1/2) / S1 in 128-bit integers (0 if p = 0): genome
 *                  positions, every copy of a repeat counted;
 *   repeat_fraction = genome_size > genomic_kmers ?
 *                  (genome_size - genomic_kmers) / genome_size : 0;
 *   het_ratio    = p >= 2 ? hist[p/2] / hist[p] : 0 (a heterozygous peak at
 *                  half the coverage raises it toward 1: the ploidy hint). */
typedef struct apg_kspec_summary {
  uint64_t valley;
  uint64_t peak;
  uint64_t genome_size;
  uint64_t genomic_kmers;
  uint64_t genomic_instances;
  uint64_t error_kmers;
  uint64_t error_instances;
  double coverage;
  double repeat_fraction;
  double het_ratio;
  uint64_t reserved[2];
} apg_kspec_summary;
int apg_kspec_estimate(const uint64_t* hist, size_t hist_len, apg_kspec_summary* out);

/* Module-boundary files of the correction and placement stages (APG v0 array
 * containers):
 *   <head>.solid.k<K>        the correction pass's solid set, ascending hashes
 *   <head>.unilocs.k<K>      UnipathLocs placements (apg_aln_pair; scalar =
 *                            number of placed-from reads)
 *   <head>.unipath_cov.k<K>  UnipathCoverage: counts u64, cov f64, copy
 *                            number u32 per unipath; scalar = c0's IEEE bits
 * Readers allocate (release each array with apg_free). */
int apg_solid_write(const char* path, int K, const uint64_t* hashes, uint64_t n);
int apg_solid_read(const char* path, int* K, uint64_t** hashes, uint64_t* n);

/* Unipath-stage files, "APG v0" array containers:
 *   <head>.unipaths.k<K>  len / id_base / rc per unipath (+ n_nodes)
 *   <head>.unibases.k<K>  APG-fastb, one sequence per unipath
 *   <head>.hkp.k<K>       HyperKmerPath: from / to per edge (= unipath), n_vertices
 *   <head>.paths.k<K>     read KmerPaths (path_off, start, len), if present
 * apg_graph_read allocates; release with apg_unipath_graph_free. */
int apg_graph_write(const char* head, const apg_unipath_graph* g);
int apg_graph_read(const char* head, int K, apg_unipath_graph* g);
int apg_kmerpaths_write(const char* path, int K, uint64_t n_paths, const uint64_t* path_off,
                        const uint64_t* start, const uint64_t* len);
/* outputs malloc'd: release each with apg_free */
int apg_kmerpaths_read(const char* path, int* K, uint64_t* n_paths, uint64_t** path_off,
                       uint64_t* n_intervals, uint64_t** start, uint64_t** len);
/* <head>.paths_rc.k<K> (KmerPaths) and <head>.pathsdb.k<K> (apg_rpint array) */
int apg_rc_db_write(const char* head, int K, const apg_rc_db* db);

#ifdef __cplusplus
}
#endif
#endif /* APG_H */
