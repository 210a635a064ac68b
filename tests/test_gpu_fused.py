"""apg_spectrum_precorrect_dev: the K=25 spectrum counted from PreCorrect's
K=24 records in the same pass (superkmer.hip rec_kmer_up) equals the two
modules run one after the other — spectrum histogram, its statistics, the
corrected bases and qualities and the correction statistics — and the CPU
restatement's spectrum.  Covers reads shorter than K, exactly K and K+1
long, long reads (tile and global walks), the repeat-rich genome (LDS-table
overflow of the K+1 pass) and the non-fusable fallback."""
import numpy as np
import pytest

import oracle
from allpathslg_amd import Context, ReadSet, synth_genome, synth_reads

pytestmark = pytest.mark.gpu


def mixed_lengths(seed=3, n=4000):
    """Genome-derived reads with substitutions, lengths 1..300 (many at the
    K boundaries 23-26), random qualities with low ones on some errors."""
    rng = np.random.default_rng(seed)
    g = synth_genome(200_000, seed)
    lens = np.concatenate([rng.integers(1, 301, n // 2), rng.choice([23, 24, 25, 26, 27, 41, 42, 100], n - n // 2)])
    seqs, quals = [], []
    for L in lens:
        s = int(rng.integers(0, len(g) - L))
        r = g[s : s + L].copy()
        q = np.full(L, 40, np.uint8)
        err = rng.random(L) < 0.01
        r[err] = (r[err] + rng.integers(1, 4, err.sum())) % 4
        q[err] = rng.integers(2, 20, err.sum())
        if rng.random() < 0.5:
            r, q = (3 - r)[::-1].copy(), q[::-1].copy()
        seqs.append(r.astype(np.uint8))
        quals.append(q)
    return ReadSet.from_sequences(seqs, quals)


def both_ways(ctx, reads, K_spec=25, K=24, n_cycles=1):
    a = ctx.upload(reads)
    b = ctx.upload(reads)
    try:
        hs, ks = ctx.kmer_spectrum(a, K_spec)
        _, ps = ctx.precorrect(a, K=K, n_cycles=n_cycles)
        hf, kf, pf = ctx.spectrum_precorrect(b, K_spec=K_spec, K=K, n_cycles=n_cycles)
        sep, fus = ctx.download(a), ctx.download(b)
    finally:
        a.free()
        b.free()
    return (hs, ks, ps, sep), (hf, kf, pf, fus)


def assert_same(sep, fus):
    hs, ks, ps, rs = sep
    hf, kf, pf, rf = fus
    assert np.array_equal(hs, hf)
    assert ks["n_kmers"] == kf["n_kmers"] and ks["n_distinct"] == kf["n_distinct"]
    assert np.array_equal(rs.packed, rf.packed) and np.array_equal(rs.quals, rf.quals)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert ps[k] == pf[k], k


def test_fused_equals_separate_mixed_lengths(gpu_ctx):
    reads = mixed_lengths()
    sep, fus = both_ways(gpu_ctx, reads)
    assert_same(sep, fus)
    assert np.array_equal(fus[0], oracle.kmer_spectrum(reads, 25))


def test_fused_equals_separate_genome_reads(gpu_ctx):
    g = synth_genome(2_000_000, 11)
    reads = synth_reads(g, 400_000, seed=12)
    sep, fus = both_ways(gpu_ctx, reads)
    assert_same(sep, fus)
    assert fus[1]["n_kmers"] == 76 * reads.n_reads


def test_fused_on_repeats_overflow():
    """Repeat-rich genome: buckets overflow the LDS table in the K+1 pass too
    (global-table path); with record dedup off and on."""
    g = synth_genome(1_000_000, 51, repeats={"tandem_frac": 0.03})
    reads = synth_reads(g, 300_000, seed=52)
    for dedup in (0, 1):
        with Context(device=0, kmer_dedup=dedup) as ctx:
            sep, fus = both_ways(ctx, reads)
            assert_same(sep, fus)
            assert fus[0][1000:].sum() > 0
            assert fus[1]["n_overflow"] > 0


def test_fused_findErrors_cycles(gpu_ctx):
    """n_cycles = 2: the spectrum is the uncorrected reads'; the second cycle
    recounts as apg_precorrect_dev does."""
    g = synth_genome(500_000, 21)
    reads = synth_reads(g, 100_000, seed=22)
    sep, fus = both_ways(gpu_ctx, reads, n_cycles=2)
    assert_same(sep, fus)


def test_not_fusable_falls_back(gpu_ctx):
    """K_spec != K + 1, or K / K+1 walking different m-mers (K = 19: m 11 vs
    12): the two modules in turn, same results."""
    g = synth_genome(300_000, 31)
    reads = synth_reads(g, 60_000, seed=32)
    for K_spec, K in ((31, 24), (20, 19)):
        sep, fus = both_ways(gpu_ctx, reads, K_spec=K_spec, K=K)
        assert_same(sep, fus)


@pytest.mark.parametrize("env", [{"APG_SK_UP_DD": "0"}, {"APG_SK_DEDUP": "none"}, {"APG_SK_UP_SORT": "1"},
                                 {"APG_SK_UP_SORT": "1", "APG_SK_UP_DD": "0"}])
def test_fused_kplus1_record_sources(gpu_ctx, monkeypatch, env):
    """The K+1 pass reads each bucket's distinct records with their
    multiplicity (the solid-set count's dedup output; buckets it handed back
    are read as partitioned).  The same results with the K+1 pass reading
    every record (APG_SK_UP_DD=0), with no record dedup at all, and with the
    LDS counting-sort form of the pass (APG_SK_UP_SORT=1, the A/B of DESIGN
    §4); on a repeat-rich genome, so some buckets take each route."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = synth_genome(1_000_000, 61, repeats={"tandem_frac": 0.03})
    reads = synth_reads(g, 300_000, seed=62)
    sep, fus = both_ways(gpu_ctx, reads)
    assert_same(sep, fus)
    monkeypatch.undo()
    _, fus_dd = both_ways(gpu_ctx, reads)
    assert_same(sep, fus_dd)


@pytest.mark.parametrize("env", [{"APG_SK_PACK": "wide"}, {"APG_SK_PACK": "0"}, {"APG_SK_UNPACK": "1"},
                                 {"APG_SK_PACK": "wide", "APG_SK_UNPACK": "1"}])
def test_solid_count_record_forms(gpu_ctx, monkeypatch, env):
    """The solid-set count's partition records: packed with 32-bit positions
    and read packed by the bucket kernels (the default below 2^32 bases),
    packed wide (34-bit positions, records cut to <= 31 bases: the form of
    read sets of 2^32 .. 2^34 bases, e.g. C4's 50 M reads per GPU;
    APG_SK_PACK=wide forces it), unpacked by the last partition level
    (APG_SK_UNPACK=1) and unpacked 24-byte records throughout (APG_SK_PACK=0)
    give the same spectrum, solid set and corrections, equal to the
    oracle's."""
    g = synth_genome(1_000_000, 71, repeats={"tandem_frac": 0.02})
    reads = synth_reads(g, 200_000, seed=72)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    sep, fus = both_ways(gpu_ctx, reads)
    assert_same(sep, fus)
    monkeypatch.undo()
    _, dflt = both_ways(gpu_ctx, reads)
    assert_same(dflt, fus)
    assert np.array_equal(fus[0], oracle.kmer_spectrum(reads, 25))
    exp, est = oracle.precorrect(reads, K=24, fast=True)
    rf = fus[3]
    assert np.array_equal(rf.packed[: int(rf.byte_off[-1])], exp.packed[: int(exp.byte_off[-1])])
    assert np.array_equal(rf.quals, exp.quals)


@pytest.mark.parametrize("kick", [None, "0", "2", "3", "4"])
def test_spectrum_precorrect_fill_equals_modules(gpu_ctx, monkeypatch, kick):
    """apg_spectrum_precorrect_fill_dev (the bench step's entry point since
    round 6: the fused K+1 count runs beside FillFragments too) equals
    apg_spectrum_precorrect_dev followed by apg_fill_fragments_dev with the
    pass's solid set: spectrum + stats, corrected bases / qualities, every
    fill status, filled fragment and counter — at every kick stage of the
    K+1 pass (APG_SK_UP_AT_FILL; 4 = after PreCorrect, beside the fill only)."""
    import torch

    if kick is not None:
        monkeypatch.setenv("APG_SK_UP_AT", kick)  # read per call (APG_SK_UP_AT_FILL is read once)
    g = synth_genome(2_000_000, 41)
    reads = synth_reads(g, 250_000, seed=42)
    a, b = gpu_ctx.upload(reads), gpu_ctx.upload(reads)
    sa = torch.zeros(reads.n_reads // 2, dtype=torch.uint8, device="cuda")
    sb = torch.zeros(reads.n_reads // 2, dtype=torch.uint8, device="cuda")
    h1, k1, p1 = gpu_ctx.spectrum_precorrect(a, K_spec=25, K=24)
    f1, _, fs1 = gpu_ctx.fill_fragments(a, K=24, last_solid=True, d_status=sa.data_ptr())
    h2, k2, p2, f2, fs2 = gpu_ctx.spectrum_precorrect_fill(b, K_spec=25, K=24, d_status=sb.data_ptr())
    assert np.array_equal(h1, h2) and k1 == k2 and p1 == p2 and fs1 == fs2
    assert np.array_equal(h1, oracle.kmer_spectrum(reads, 25))
    ra, rb = gpu_ctx.download(a, with_quals=True), gpu_ctx.download(b, with_quals=True)
    assert np.array_equal(ra.packed, rb.packed) and np.array_equal(ra.quals, rb.quals)
    assert np.array_equal(sa.cpu().numpy(), sb.cpu().numpy())
    x, y = gpu_ctx.download(f1), gpu_ctx.download(f2)
    assert np.array_equal(x.base_off, y.base_off)
    assert np.array_equal(x.packed[: int(x.byte_off[-1])], y.packed[: int(y.byte_off[-1])])
    assert fs2["n_filled"] > 0
    for d in (a, b, f1, f2):
        d.free()
