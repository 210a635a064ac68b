// partition.hpp — device-wide building blocks shared by the k-mer modules:
// the u32 -> u64 exclusive scan and the LDS-staged hash-partition level,
// for 8-byte hash records (K <= 32 spectrum) and 32-byte K <= 96 records.
#pragma once

#include <cstdint>
#include <vector>

#include "apg_core.hpp"

namespace apg {

// 32-byte record of one K-mer instance for K <= 96: canonical key as three
// big-endian 64-bit limbs (k0 most significant; value = sum b[i] 4^(K-1-i))
// and meta = (56-bit key hash << 8) | extension bits (left nibble = bases
// preceding the canonical K-mer, right nibble = bases following it).
struct __attribute__((aligned(16))) KRec {
  uint64_t k0, k1, k2, meta;
};

// 16-byte super-k-mer record (K <= 32 counting, superkmer.hip): w0 = 32-bit
// minimizer key | n_kmers << 32 | (reserved 8 bits) | bases 0..7 << 48;
// w1 = bases 8..39 — up to 40 bases, 2-bit LSB-first, starting at the
// super-k-mer's first base.
struct __attribute__((aligned(16))) SK16 {
  uint64_t w0, w1;
};

// SK16 + the global base position of the record's first K-mer (read r's
// K-mer j starts at base base_off[r] + j): the solid-set pass of PreCorrect
// uses it to mark every weak K-mer instance in a per-base bitmap while
// counting, so the correction needs no lookups to find weak K-mers.
struct __attribute__((aligned(8))) SK24 {
  uint64_t w0, w1, pos;
};

// 16-byte packed form of an SK24 for the partition levels of the
// single-GPU solid-set count (a record of <= 32 bases: the scatter splits
// longer ones): w0 = the partition key's top 22 bits << 42 | position (32
// bits) << 10 | n_kmers << 6 | flank bits (as SK16 bits 40..45); w1 = bases
// 0..31, 2-bit LSB-first.  The last partition level unpacks it to the SK24
// the bucket kernels read (skp_unpack), so the levels move 16 bytes per
// record instead of 24.
struct __attribute__((aligned(16))) SKP {
  uint64_t w0, w1;
};
constexpr int kSkpKeyBits = 22;

// An SK16 of <= 32 bases (n <= 15 K-mers) + a 32-bit position -> SKP; the
// packed key = bits [kshift, kshift + 22) from the top of the 32-bit key.
__host__ __device__ inline void skp_pack(uint64_t w0, uint64_t w1, uint64_t pos, int kshift, uint64_t* o) {
  const uint64_t key = (((w0 & 0xffffffffull) << kshift) & 0xffffffffull) >> (32 - kSkpKeyBits);
  const uint64_t n = (w0 >> 32) & 15, fl = (w0 >> 40) & 63;
  o[0] = (key << (64 - kSkpKeyBits)) | ((pos & 0xffffffffull) << 10) | (n << 6) | fl;
  o[1] = (w0 >> 48) | (w1 << 16);
}

// wide: the record holds <= 31 bases and w1's top two bits carry position
// bits 32..33 (read sets of 2^32 .. 2^34 bases: the scatter cuts records to
// <= 32 - K + 1 K-mers for them).
__host__ __device__ inline void skp_unpack(uint64_t w0, uint64_t w1, uint64_t* o, bool wide = false) {
  const uint64_t key32 = (w0 >> (64 - kSkpKeyBits)) << (32 - kSkpKeyBits);
  const uint64_t b = wide ? w1 & ((1ull << 62) - 1) : w1;
  o[0] = key32 | (((w0 >> 6) & 15) << 32) | ((w0 & 63) << 40) | ((b & 0xffffull) << 48);
  o[1] = b >> 16;
  o[2] = ((w0 >> 10) & 0xffffffffull) | (wide ? (w1 >> 62) << 32 : 0);
}

// 48-byte super-k-mer record of the K <= 96 unipath node builder
// (unipath.hip): w0 = 32-bit minimizer key | n_kmers << 32 | flags << 40
// (bit 0: b[] starts one base before the first K-mer, bit 1: it ends one base
// after the last — the extension bases); b = up to 160 bases, 2-bit
// LSB-first.
struct __attribute__((aligned(16))) SK48 {
  uint64_t w0;
  uint64_t b[5];
};

// The partition digit source of a record.
__host__ __device__ inline uint64_t rkey(uint64_t r) { return r; }
__host__ __device__ inline uint64_t rkey(const KRec& r) { return r.meta; }
__host__ __device__ inline uint64_t rkey(const SK16& r) { return r.w0 << 32; }  // the minimizer key
__host__ __device__ inline uint64_t rkey(const SK24& r) { return r.w0 << 32; }
__host__ __device__ inline uint64_t rkey(const SK48& r) { return r.w0 << 32; }
__host__ __device__ inline uint64_t rkey(const SKP& r) { return r.w0; }  // the key's top bits lead

constexpr int kMaxLevelBits = 8;  // max digit bits of one partition level (LDS-staged scatter)

struct Seg {
  uint64_t start, len;
};

// d_out[0..n] = exclusive prefix sums of d_in[0..n) (d_out[n] = total).
int scan_u32_u64(apg_ctx* ctx, const uint32_t* d_in, uint64_t n, uint64_t* d_out, const char* tag);
// ncol (<= kScanColsMax) such scans of the same length, launched together.
constexpr int kScanColsMax = 4;
int scan_cols_u32_u64(apg_ctx* ctx, int ncol, const uint32_t* const* d_in, uint64_t n, uint64_t* const* d_out,
                      const char* tag);

// One partition level: the records of every parent (a list of segments of
// `src`) are split by bits [shift, shift+bits) of rkey() into ndig = 2^bits
// children, written contiguously to `dst` in (parent, digit) order.  Writes
// the children's starts to d_child[0 .. nparents*ndig] (last = n) and, if
// host_child, copies them to the host.  Order inside a child is unspecified.
// RO: the output record type — R, SK24 from SK16 (the input index as pos),
// SK24 from SKP (unpacked), or SKP from SK16 (<= 32 bases; the input index as
// pos, the key's bits below its top `kshift` bits as the packed key, so the
// packed record's digits sit kshift bits higher).
// wide: SKP records in the 34-bit-position form (skp_unpack).
// The parents of a level: lists of segments, or (every level after a
// level's own children) one segment per parent, [bounds[q], bounds[q+1]) —
// the child offsets the level before copied back, with no per-parent vector
// built on the host between levels.
struct PartParents {
  const std::vector<std::vector<Seg>>* lists = nullptr;
  const std::vector<uint64_t>* bounds = nullptr;
  PartParents(const std::vector<std::vector<Seg>>& l) : lists(&l) {}
  PartParents(const std::vector<uint64_t>& b) : bounds(&b) {}
  uint64_t size() const { return lists ? lists->size() : (bounds->empty() ? 0 : bounds->size() - 1); }
};

template <typename R, typename RO = R>
int part_level(apg_ctx* ctx, const R* src, RO* dst, const PartParents& parents, int shift, int bits,
               uint64_t n, uint64_t* d_child, std::vector<uint64_t>* host_child, const char* tag, int kshift = 0,
               bool wide = false);

// Stable LSD radix sort of (key, val) pairs by key over the key's significant
// bits (pathsdb.hip): ping-pongs between (k, v) and (k2, v2); *in2 tells
// which pair holds the result.
int sort_u64_u32(apg_ctx* ctx, uint64_t* k, uint32_t* v, uint64_t* k2, uint32_t* v2, uint64_t n, bool* in2);

}  // namespace apg
