"""Oracle checks (CPU only): the C restatement against first-principles
known-answer tests, against an independent pure-Python
restatement, and against the committed golden fixtures.

Parity vs the real ALLPATHS-LG is UNPINNED: /root/reference is empty
(SURVEY §0.1), so no reference tests or golden vectors exist to pin to.
"""
import os

import numpy as np
import pytest

import oracle
from allpathslg_amd import ReadSet, synth_genome, synth_reads
from tests import pyoracle

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


@pytest.mark.parametrize("K", [1, 2, 5, 13, 16, 24, 25, 31, 32])
def test_hash_is_bijection(K):
    rng = np.random.default_rng(K)
    w = 2 * K
    xs = rng.integers(0, 2**63, size=2000, dtype=np.uint64) & np.uint64((1 << w) - 1 if w < 64 else 2**64 - 1)
    for x in xs[:300]:
        h = oracle.kmer_hash(K, int(x))
        assert h < 2**w
        assert oracle.kmer_unhash(K, h) == int(x)
    if w <= 12:  # exhaustive: a permutation of [0, 4^K)
        hs = {oracle.kmer_hash(K, x) for x in range(1 << w)}
        assert hs == set(range(1 << w))


def test_hash_k32_is_splitmix64_finaliser():
    def sm(x):
        m = 2**64 - 1
        x ^= x >> 30
        x = (x * 0xBF58476D1CE4E5B9) & m
        x ^= x >> 27
        x = (x * 0x94D049BB133111EB) & m
        return x ^ (x >> 31)

    for x in [0, 1, 12345, 2**63 + 7, 2**64 - 1]:
        assert oracle.kmer_hash(32, x) == sm(x)


@pytest.mark.parametrize("K", [3, 11, 25])
def test_oracle_matches_python_restatement(K):
    rng = np.random.default_rng(100 + K)
    seqs = [rng.integers(0, 4, size=int(rng.integers(0, 60))) for _ in range(80)]
    seqs += [rng.integers(0, 4, size=40)] * 5  # duplicates
    reads = ReadSet.from_sequences(seqs)
    h, c = oracle.kmer_count(reads, K)
    assert np.all(np.diff(h.astype(np.float64)) > 0) or len(h) <= 1  # strictly ascending hash
    pc = pyoracle.count(reads, K)
    got = {oracle.kmer_unhash(K, int(x)): int(y) for x, y in zip(h, c)}
    assert got == dict(pc)
    hist = oracle.spectrum_from_counts(c, 64)
    assert np.array_equal(hist, pyoracle.spectrum(pc, 64))


def test_kat_error_free_tiling():
    """reads at every start of a random genome with no repeated
    K-mer: every genomic K-mer away from the ends is seen L-K+1 times."""
    G, L, K = 3000, 50, 21
    g = synth_genome(G, 7)
    seqs = [g[s : s + L] for s in range(G - L + 1)]
    reads = ReadSet.from_sequences(seqs)
    _, c = oracle.kmer_count(reads, K)
    hist = oracle.spectrum_from_counts(c, 256)
    n_kmers = G - K + 1
    # k-mer at genome position p is covered by reads starting in [p-(L-K), p] ∩ [0, G-L]
    expect = np.zeros(256, dtype=np.uint64)
    for p in range(n_kmers):
        lo, hi = max(0, p - (L - K)), min(p, G - L)
        expect[hi - lo + 1] += 1
    assert np.array_equal(hist, expect)
    assert int(hist[L - K + 1]) == n_kmers - 2 * (L - K)


def test_kat_reverse_complement_symmetry():
    """A read and its reverse complement have identical canonical spectra."""
    rng = np.random.default_rng(3)
    s = rng.integers(0, 4, size=200)
    rc = (3 - s[::-1]).copy()
    a = oracle.kmer_count(ReadSet.from_sequences([s]), 17)
    b = oracle.kmer_count(ReadSet.from_sequences([rc]), 17)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


def test_conservation_on_synthetic():
    g = synth_genome(50_000, 11)
    reads = synth_reads(g, 2000, seed=5)
    for K in (16, 25):
        h, c = oracle.kmer_count(reads, K)
        assert int(c.sum()) == reads.n_reads * (100 - K + 1)
        hist = oracle.spectrum_from_counts(c, 1 << 16)
        assert int((hist * np.arange(len(hist), dtype=np.uint64)).sum()) == int(c.sum())


def _golden(name):
    p = os.path.join(GOLDEN, name)
    if not os.path.exists(p):
        pytest.skip(f"golden fixture {name} missing (run tests/golden/make_golden.py)")
    return p


def test_oracle_against_golden():
    reads = ReadSet.load(_golden("frag_small.fastb"), _golden("frag_small.qualb"))
    z = np.load(_golden("kmer_small.npz"))
    for K in (16, 25):
        h, c = oracle.kmer_count(reads, K)
        assert np.array_equal(h, z[f"hash_k{K}"])
        assert np.array_equal(c, z[f"count_k{K}"])
        assert np.array_equal(oracle.spectrum_from_counts(c, 1 << 16)[:4096], z[f"spec_k{K}"])


def test_precorrect_kat_single_substitutions():
    """substitutions at known positions (low Q) under ~50x
    coverage are corrected back to the genome."""
    from allpathslg_amd import synth_genome

    rng = np.random.default_rng(77)
    G, L = 4000, 100
    g = synth_genome(G, 99)
    starts = rng.integers(0, G - L + 1, size=2000)
    seqs, quals, truth, errpos = [], [], [], []
    for i, s in enumerate(starts):
        r = g[s : s + L].copy()
        q = np.full(L, 40, dtype=np.uint8)
        truth.append(r.copy())
        if i % 10 == 0:
            p = int(rng.integers(0, L))
            r[p] = (r[p] + 1 + rng.integers(0, 3)) % 4
            q[p] = 10
            errpos.append((i, p))
        seqs.append(r)
        quals.append(q)
    reads = ReadSet.from_sequences(seqs, quals)
    fixed, st = oracle.precorrect(reads, K=24)
    assert st["n_corrected"] == len(errpos)
    for i in range(reads.n_reads):
        assert np.array_equal(fixed.read(i), truth[i])
    for i, p in errpos:
        assert fixed.quals[int(fixed.base_off[i]) + p] == 40


def test_precorrect_leaves_high_quality_and_is_idempotent():
    from allpathslg_amd import synth_genome, synth_reads

    g = synth_genome(30_000, 5)
    reads = synth_reads(g, 6000, seed=6)
    fixed, st = oracle.precorrect(reads, K=24)
    assert st["n_corrected"] > 0
    hq = reads.quals >= 20
    assert np.array_equal(fixed.quals[hq], reads.quals[hq])
    # bases at high-quality positions never change
    for i in range(0, reads.n_reads, 97):
        a, b = reads.read(i), fixed.read(i)
        qq = reads.quals[int(reads.base_off[i]) : int(reads.base_off[i + 1])]
        assert np.array_equal(a[qq >= 20], b[qq >= 20])
    again, st2 = oracle.precorrect(fixed, K=24)
    assert st2["n_corrected"] <= st["n_corrected"] // 10


def _stage_golden():
    z = np.load(_golden("stages_small.npz"))
    reads = ReadSet.load(_golden("frag_small.fastb"), _golden("frag_small.qualb"))
    frags = ReadSet.load(_golden("frag_small_fill.fastb"))
    S = ReadSet.load(_golden("aln_queries.fastb"), _golden("aln_queries.qualb"))
    T = ReadSet.load(_golden("aln_targets.fastb"))
    return z, reads, frags, S, T


def test_oracle_stages_against_golden():
    """PreCorrect (1, 2 cycles), unipaths (K=31 on reads, K=96 on the pair
    fragments) and the aligners reproduce the committed fixtures."""
    z, reads, frags, S, T = _stage_golden()
    for cyc in (1, 2):
        fixed, st = oracle.precorrect(reads, K=24, n_cycles=cyc)
        assert np.array_equal(fixed.packed[: int(fixed.byte_off[-1])], z[f"pc{cyc}_packed"])
        assert np.array_equal(fixed.quals, z[f"pc{cyc}_quals"])
    for K, src in ((31, reads), (96, frags)):
        g = oracle.unipaths(src, K)
        for key in ("len", "id_base", "rc", "ub_off", "unibases", "from", "to", "path_off", "path_start", "path_len"):
            assert np.array_equal(np.asarray(g[key]), z[f"u{K}_{key}"]), (K, key)
    pairs = z["aln_pairs"]
    assert np.array_equal(oracle.gapfree(S, T, pairs), z["aln_gapfree"])
    res, blk = oracle.banded_sw(S, T, pairs, band_w=8, max_blocks=16)
    assert np.array_equal(res, z["aln_sw"]) and np.array_equal(blk, z["aln_sw_blocks"])
    b, q = oracle.consensus(S, T, pairs)
    assert np.array_equal(b, z["aln_cons_bases"]) and np.array_equal(q, z["aln_cons_quals"])


@pytest.mark.parametrize("case", ["plain", "repeats", "low_q"])
def test_precorrect_preserves_the_solid_set(case):
    """The invariant ErrorCorrectJump's reuse of the fragments' solid set
    rests on (apg_core.hpp pc_self): a PreCorrect pass leaves the reads'
    solid set unchanged — a suspect's covering K-mers are all weak, an
    accepted alternative's all solid and accepted corrections lie >= K apart,
    so only weak K-mer instances are removed and only solid ones added."""
    from allpathslg_amd import synth_genome, synth_reads

    if case == "repeats":
        g = synth_genome(300_000, 91, repeats={"tandem_frac": 0.03})
        reads = synth_reads(g, 60_000, seed=92)
    elif case == "low_q":
        g = synth_genome(200_000, 93)
        reads = synth_reads(g, 40_000, seed=94, err_lo=0.01, err_hi=0.05)
    else:
        g = synth_genome(200_000, 95)
        reads = synth_reads(g, 40_000, seed=96)
    s0 = np.sort(oracle.solid_hashes(reads, 24, 3))
    for n_cycles in (1, 2):
        fixed, st = oracle.precorrect(reads, K=24, n_cycles=n_cycles)
        assert st["n_corrected"] > 1000
        assert np.array_equal(np.sort(oracle.solid_hashes(fixed, 24, 3)), s0)
