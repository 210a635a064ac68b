"""GPU parity tests for the k-mer spectrum path: libapg's HIP kernels vs the
CPU oracle (bit-exact: integer work), through the C ABI.

Parity vs real ALLPATHS-LG is unpinned (reference snapshot empty); parity vs
the repo's restatement (oracle/) and its golden fixtures is exact.
"""
import os

import numpy as np
import pytest

import oracle
from allpathslg_amd import ReadSet, kmer_hash, shard_bins, synth_genome, synth_reads

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def assert_table_equal(ctx, reads, K):
    keys, counts, st = ctx.kmer_count(reads, K)
    h, c = oracle.kmer_count(reads, K)
    ok = np.array([oracle.kmer_unhash(K, int(x)) for x in h[:50]], dtype=np.uint64)
    assert np.array_equal(keys[:50], ok)
    hk = np.array([kmer_hash(K, int(k)) for k in keys[:2000]], dtype=np.uint64)
    assert np.array_equal(hk, h[:2000])
    assert len(keys) == len(h)
    assert np.array_equal(counts, c)
    assert st["n_distinct"] == len(h)
    return keys, counts, st


def assert_spectrum_equal(ctx, reads, K, hist_len=1 << 16):
    hist, st = ctx.kmer_spectrum(reads, K, hist_len)
    expect = oracle.kmer_spectrum(reads, K, hist_len)
    assert np.array_equal(hist, expect), (np.nonzero(hist != expect)[0][:10])
    n = int(oracle.lib().ork_count_instances(reads.n_reads, reads.base_off.ctypes.data_as(oracle._u64p), K))
    assert st["n_kmers"] == n
    return hist, st


def test_golden_fixture(gpu_ctx):
    reads = ReadSet.load(os.path.join(GOLDEN, "frag_small.fastb"), os.path.join(GOLDEN, "frag_small.qualb"))
    z = np.load(os.path.join(GOLDEN, "kmer_small.npz"))
    for K in (16, 25):
        hist, _ = gpu_ctx.kmer_spectrum(reads, K)
        assert np.array_equal(hist[:4096], z[f"spec_k{K}"])
        keys, counts, _ = gpu_ctx.kmer_count(reads, K)
        hk = np.array([kmer_hash(K, int(k)) for k in keys], dtype=np.uint64)
        assert np.array_equal(hk, z[f"hash_k{K}"])
        assert np.array_equal(counts, z[f"count_k{K}"])


@pytest.mark.parametrize("K", [1, 2, 4, 12, 21, 24, 25, 31, 32])
def test_ragged_random_reads(gpu_ctx, K):
    rng = np.random.default_rng(1000 + K)
    lens = rng.integers(0, 160, size=3000)
    lens[:5] = [0, 1, K - 1 if K > 1 else 0, K, K + 1]
    seqs = [rng.integers(0, 4, size=int(n)) for n in lens]
    reads = ReadSet.from_sequences(seqs)
    assert_spectrum_equal(gpu_ctx, reads, K)
    assert_table_equal(gpu_ctx, reads, K)


def test_empty_and_tiny_sets(gpu_ctx):
    empty = ReadSet.from_sequences([])
    hist, st = gpu_ctx.kmer_spectrum(empty, 25)
    assert hist.sum() == 0 and st["n_kmers"] == 0
    short = ReadSet.from_sequences([[0, 1, 2], [], [3] * 10])
    hist, st = gpu_ctx.kmer_spectrum(short, 25)
    assert hist.sum() == 0 and st["n_kmers"] == 0
    one = ReadSet.from_sequences([[0, 1, 2, 3] * 10])
    assert_spectrum_equal(gpu_ctx, one, 25)
    assert_table_equal(gpu_ctx, one, 25)


def test_synthetic_library(gpu_ctx):
    g = synth_genome(500_000, 3)
    reads = synth_reads(g, 100_000, seed=4)
    for K in (16, 25):
        assert_spectrum_equal(gpu_ctx, reads, K)
    assert_table_equal(gpu_ctx, reads, 25)


def test_oversized_buckets_take_global_path(gpu_ctx):
    """Highly repeated k-mers (poly-A, one read copied 6000x) overflow the LDS
    bucket and must go through sort_count_global with identical results."""
    rng = np.random.default_rng(5)
    base = rng.integers(0, 4, size=100)
    seqs = [base] * 6000 + [np.zeros(100, dtype=np.uint8)] * 100
    seqs += [rng.integers(0, 4, size=100) for _ in range(20000)]
    reads = ReadSet.from_sequences(seqs)
    hist, st = assert_spectrum_equal(gpu_ctx, reads, 25)
    assert hist[6000] >= 70
    assert_table_equal(gpu_ctx, reads, 25)


def _min_mmer(m):
    """The canonical m-mer with the smallest minimizer order (superkmer.hip's
    mmer_order: murmur3 fmix32 of (lo ^ salt) ^ (hi * golden))."""
    v = np.arange(4**m, dtype=np.uint64)
    rc = np.zeros_like(v)
    x = v.copy()
    for _ in range(m):
        rc = (rc << np.uint64(2)) | (np.uint64(3) - (x & np.uint64(3)))
        x >>= np.uint64(2)
    c = np.minimum(v, rc)
    with np.errstate(over="ignore"):
        h = ((c & np.uint64(0xFFFFFFFF)).astype(np.uint32) ^ np.uint32(0x2545F491)) ^ (
            (c >> np.uint64(32)).astype(np.uint32) * np.uint32(0x9E3779B1))
        h ^= h >> np.uint32(16)
        h *= np.uint32(0x85EBCA6B)
        h ^= h >> np.uint32(13)
        h *= np.uint32(0xC2B2AE35)
        h ^= h >> np.uint32(16)
    best = int(v[np.argmin(h)])
    return np.array([(best >> (2 * (m - 1 - i))) & 3 for i in range(m)], dtype=np.uint8)


def test_superkmer_bucket_overflow_takes_global_table(gpu_ctx):
    """Every K-mer containing the globally smallest m-mer shares one
    minimizer, hence one partition: thousands of distinct K-mers overflow the
    LDS table of that bucket and are counted in the global fallback table."""
    K, m = 16, 10
    mm = _min_mmer(m)
    rng = np.random.default_rng(15)
    seqs = []
    for _ in range(20000):
        r = rng.integers(0, 4, size=100).astype(np.uint8)
        p = int(rng.integers(0, 100 - m))
        r[p : p + m] = mm
        seqs.append(r)
    reads = ReadSet.from_sequences(seqs)
    hist, st = assert_spectrum_equal(gpu_ctx, reads, K)
    assert st["n_overflow"] > 0


@pytest.fixture(scope="module")
def dd_ctx():
    """A context that counts every K >= 21 bucket through the record-dedup
    kernel (by default only the solid-set counts of PreCorrect do)."""
    from allpathslg_amd import Context

    with Context(device=0, kmer_dedup=1) as c:
        yield c


def test_record_dedup_active_and_exact(dd_ctx):
    """K >= 21 counts through the record-deduplicating bucket kernel: at
    ordinary coverage (60x) it finishes nearly every bucket itself and the
    spectrum equals the oracle's."""
    g = synth_genome(300_000, 41)
    reads = synth_reads(g, 90_000, seed=42)
    for K in (21, 24, 25, 32):
        _, st = assert_spectrum_equal(dd_ctx, reads, K)
        assert st["n_redo"] <= st["n_buckets"] // 100, K
    _, st = assert_spectrum_equal(dd_ctx, reads, 20)  # below the dedup kernel's K range
    assert st["n_redo"] == 0
    rng = np.random.default_rng(43)  # ragged reads, lengths 0..300
    seqs = []
    for _ in range(20000):
        L = int(rng.integers(0, 300))
        s = int(rng.integers(0, len(g) - 300))
        seqs.append(g[s : s + L])
    for K in (21, 25, 32):
        assert_spectrum_equal(dd_ctx, ReadSet.from_sequences(seqs), K)


def test_record_dedup_hands_back_buckets(dd_ctx):
    """Buckets the dedup kernel cannot finish in LDS.  (1) The globally
    smallest 13-mer in every read (K = 21, m = 13): one bucket of ~20000
    distinct records fills the record table -> handed back to k_sk_bucket ->
    its K-mers overflow the LDS K-mer table -> global table.  (2) 6000 copies
    of one read: records of multiplicity 6000, counted in LDS."""
    K, m = 21, 13
    mm = _min_mmer(m)
    rng = np.random.default_rng(16)
    seqs = []
    for _ in range(20000):
        r = rng.integers(0, 4, size=100).astype(np.uint8)
        p = int(rng.integers(0, 100 - m))
        r[p : p + m] = mm
        seqs.append(r)
    _, st = assert_spectrum_equal(dd_ctx, ReadSet.from_sequences(seqs), K)
    assert st["n_redo"] > 0 and st["n_overflow"] > 0
    one = rng.integers(0, 4, size=100).astype(np.uint8)
    seqs = [one] * 6000 + [rng.integers(0, 4, size=100).astype(np.uint8) for _ in range(3000)]
    hist, st = assert_spectrum_equal(dd_ctx, ReadSet.from_sequences(seqs), 25)
    assert hist[6000] >= 70


def test_small_hist_len_clamps(gpu_ctx):
    g = synth_genome(50_000, 8)
    reads = synth_reads(g, 20_000, seed=9)
    assert_spectrum_equal(gpu_ctx, reads, 25, hist_len=8)
    assert_spectrum_equal(gpu_ctx, reads, 25, hist_len=2)


def test_device_resident_and_deterministic(gpu_ctx):
    g = synth_genome(200_000, 10)
    reads = synth_reads(g, 50_000, seed=11)
    d = gpu_ctx.upload(reads)
    h1, s1 = gpu_ctx.kmer_spectrum(d, 25)
    h2, s2 = gpu_ctx.kmer_spectrum(d, 25)
    assert np.array_equal(h1, h2) and s1 == s2
    assert np.array_equal(h1, oracle.kmer_spectrum(reads, 25))
    k1 = gpu_ctx.kmer_count(reads, 25)
    k2 = gpu_ctx.kmer_count(reads, 25)
    assert np.array_equal(k1[0], k2[0]) and np.array_equal(k1[1], k2[1])
    d.free()


@pytest.mark.parametrize("P", [1, 2, 4])
def test_shard_path_loopback(gpu_ctx, P):
    """The multi-GPU data path on one GPU: P read slices -> shard_count /
    shard_scatter -> loopback all_to_all -> shard_spectrum per shard; the
    shard spectra sum to the monolithic spectrum (shard-count invariance)."""
    import torch

    K = 25
    g = synth_genome(300_000, 12)
    reads = synth_reads(g, 60_000, seed=13)
    B = shard_bins(K, P)
    parts = np.array_split(np.arange(reads.n_reads), P)
    sends, counts = [], []
    for idx in parts:
        sub = reads.subset(int(idx[0]), int(idx[-1]) + 1)
        d = gpu_ctx.upload(sub)
        c = gpu_ctx.shard_count(d, K, P)
        buf = torch.empty(max(2 * int(c.sum()), 1), dtype=torch.int64, device="cuda")  # 16-byte records
        torch.cuda.synchronize()
        gpu_ctx.shard_scatter(d, K, P, buf.data_ptr())
        sends.append(buf)
        counts.append(c.reshape(P, B))
        d.free()
    total = np.zeros(1 << 16, dtype=np.uint64)
    nd = 0
    for s in range(P):
        pieces, rc = [], []
        for p in range(P):
            starts = np.concatenate([[0], np.cumsum(counts[p].reshape(-1))]).astype(np.int64)
            a, b = starts[s * B], starts[(s + 1) * B]
            pieces.append(sends[p][2 * a : 2 * b])
            rc.append(counts[p][s])
        recv = torch.cat(pieces) if sum(x.numel() for x in pieces) else torch.empty(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        hist, st = gpu_ctx.shard_spectrum(recv.data_ptr(), np.concatenate(rc), K, P)
        total += hist
        nd += st["n_distinct"]
    expect = oracle.kmer_spectrum(reads, K)
    assert np.array_equal(total, expect)
    assert nd == int(expect.sum())


def test_bad_arguments(gpu_ctx):
    from allpathslg_amd import ApgError

    reads = ReadSet.from_sequences([[0, 1, 2, 3] * 10])
    with pytest.raises(ApgError):
        gpu_ctx.kmer_spectrum(reads, 33)
    with pytest.raises(ApgError):
        gpu_ctx.kmer_spectrum(reads, 0)
    with pytest.raises(ApgError):
        gpu_ctx.kmer_spectrum(reads, 25, hist_len=1)
    d = gpu_ctx.upload(reads)
    with pytest.raises(ApgError):
        gpu_ctx.shard_count(d, 25, 3)
    with pytest.raises(ApgError):
        gpu_ctx.shard_count(d, 25, 16)  # one node: <= 8 shards
