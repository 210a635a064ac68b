/* oracle/oracle.h — CPU restatement (TEST INFRASTRUCTURE ONLY; parity unpinned,
 * see kmer_oracle.c header).  Loaded by tests/ and bench.py's cpu_baseline. */
#ifndef APG_ORACLE_H
#define APG_ORACLE_H
#include <stdint.h>

uint64_t ork_hash(int K, uint64_t canonical);
uint64_t ork_unhash(int K, uint64_t hash);
uint64_t ork_count_instances(uint64_t n_reads, const uint64_t* base_off, int K);
uint64_t ork_extract_hashes(uint64_t n_reads, const uint64_t* base_off,
                            const uint64_t* byte_off, const uint8_t* packed, int K,
                            uint64_t* out);
uint64_t ork_kmer_count(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off,
                        const uint8_t* packed, int K, uint64_t** hashes, uint32_t** counts);
uint64_t ork_kmer_count_range(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off,
                              const uint8_t* packed, int K, uint64_t lo, uint64_t hi, uint64_t** hashes,
                              uint32_t** counts);
void ork_set_threads(int n);
int ork_threads(void);
void ork_spectrum(const uint32_t* counts, uint64_t nd, uint64_t* hist, uint64_t hist_len);
void ork_kspec_estimate(const uint64_t* hist, uint64_t hist_len, uint64_t* u7, double* d3);
void ork_free(void* p);
int ork_precorrect(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed,
                   uint8_t* quals, int K, uint32_t min_solid, uint32_t maxq, uint32_t n_cycles, uint64_t* stats);
int ork_precorrect_solid(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed,
                         uint8_t* quals, int K, uint32_t maxq, const uint64_t* solid, uint64_t ns, uint64_t* stats);

/* bench.py CPU-baseline forms (same outputs, faster structures; solidset.h) */
int ork_precorrect_fast(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed,
                        uint8_t* quals, int K, uint32_t min_solid, uint32_t maxq, uint32_t n_cycles, uint64_t* stats);
int ork_precorrect_solid_fast(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, uint8_t* packed,
                              uint8_t* quals, int K, uint32_t maxq, const uint64_t* solid, uint64_t ns,
                              uint64_t* stats);
int orf_fill_fast(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed, int K,
                  const uint64_t* solid, uint64_t ns, uint32_t min_insert, uint32_t max_insert, uint32_t max_steps,
                  uint8_t* status, uint32_t* flen, uint8_t** out_bases, uint64_t* stats);

int orf_fill(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed, int K,
             const uint64_t* solid, uint64_t ns, uint32_t min_insert, uint32_t max_insert, uint32_t max_steps,
             uint8_t* status, uint32_t* flen, uint8_t** out_bases, uint64_t* stats);

void ora_gapfree(const uint64_t* s_base_off, const uint64_t* s_byte_off, const uint8_t* s_packed,
                 const uint8_t* s_quals, const uint64_t* t_base_off, const uint64_t* t_byte_off,
                 const uint8_t* t_packed, const uint32_t* pairs, uint64_t n, uint32_t* out);
void ora_banded_sw(const uint64_t* s_base_off, const uint64_t* s_byte_off, const uint8_t* s_packed,
                   const uint64_t* t_base_off, const uint64_t* t_byte_off, const uint8_t* t_packed,
                   const uint32_t* pairs, uint64_t n, int w, int32_t* res, int32_t* blocks, uint32_t max_blocks);
void ora_consensus(const uint64_t* r_base_off, const uint64_t* r_byte_off, const uint8_t* r_packed,
                   const uint8_t* r_quals, const uint64_t* t_base_off, const uint64_t* t_byte_off,
                   const uint8_t* t_packed, uint64_t n_targets, const uint32_t* plc, uint64_t n, uint8_t* cons,
                   uint8_t* cq);

int orl_locs(uint64_t U, const uint64_t* ulen, const uint64_t* urc, const uint64_t* ub_off, const uint8_t* ub, int K,
             uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed,
             uint32_t flags, uint32_t** out, uint64_t* n_out, uint64_t* stats);

int ouc_coverage(uint64_t U, const uint64_t* ulen, const uint32_t* pairs, uint64_t n, uint64_t min_len,
                 uint64_t* counts, double* cov, uint32_t* cn, double* c0_out, uint64_t* n_long);

void oje_trim(uint64_t n_reads, const uint64_t* base_off, const uint64_t* byte_off, const uint8_t* packed, int K,
              const uint64_t* solid, uint64_t ns, uint32_t min_keep, uint32_t* keep);

#endif
