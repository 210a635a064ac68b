"""GPU parity on a repeat-rich synthetic genome (apg_synth_repeats: an
Alu-like, an L1-like and a young near-identical family plus tandem arrays):
the bucket skew, high-count K-mers, LDS-table overflow / dedup hand-back and
collapsed or cyclic unipaths the iid genome never produces.  Everything
equals the CPU restatement.  Parity vs real ALLPATHS-LG: unpinned."""
import numpy as np
import pytest

import oracle
from allpathslg_amd import Context, synth_fragments, synth_genome, synth_reads
from tests.test_gpu_unipath import assert_graph_equal

pytestmark = pytest.mark.gpu

G = 1_000_000


@pytest.fixture(scope="module")
def rep_reads():
    g = synth_genome(G, 51, repeats={"tandem_frac": 0.03})
    return g, synth_reads(g, 300_000, seed=52)


@pytest.mark.parametrize("dedup", [0, 1, 2])
def test_spectrum_on_repeats(rep_reads, dedup):
    _, reads = rep_reads
    with Context(device=0, kmer_dedup=dedup) as ctx:
        for K in (24, 25):
            hist, st = ctx.kmer_spectrum(reads, K)
            assert np.array_equal(hist, oracle.kmer_spectrum(reads, K)), (dedup, K)
            assert hist[1000:].sum() > 0  # K-mers seen over a thousand times


def test_precorrect_on_repeats(gpu_ctx, rep_reads):
    _, reads = rep_reads
    got, st = gpu_ctx.precorrect(reads, K=24)
    exp, est = oracle.precorrect(reads, K=24)
    assert np.array_equal(got.packed[: int(got.byte_off[-1])], exp.packed[: int(exp.byte_off[-1])])
    assert np.array_equal(got.quals, exp.quals)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert st[k] == est[k], k


def test_unipaths_on_repeats(gpu_ctx, rep_reads):
    g, _ = rep_reads
    frags = synth_fragments(g, 150_000, seed=53)
    got, st = gpu_ctx.unipaths(frags, 96)
    assert_graph_equal(got, oracle.unipaths(frags, 96))
    # repeats collapse: fewer distinct 96-mers than genome positions
    assert st["n_nodes"] < 0.99 * (G - 95)


@pytest.mark.parametrize("probe", ["1", "4"])
def test_overflow_table_retry_unbounded(rep_reads, monkeypatch, probe):
    """the overflowed buckets' global table (APG_SK_OVF=
    global, for the K pass and the fused K+1 pass) gives up after APG_SK_BIG_PROBE probes
    on its first, small attempt; the full-size retry probes without a limit,
    so a crowded first attempt on tandem-repeat keys still ends in the
    oracle's spectrum, solid set and corrections."""
    monkeypatch.setenv("APG_SK_BIG_PROBE", probe)
    monkeypatch.setenv("APG_SK_OVF", "global")
    _, reads = rep_reads
    with Context(device=0, verbose=True) as ctx:
        for K in (24, 25):
            hist, st = ctx.kmer_spectrum(reads, K)
            assert np.array_equal(hist, oracle.kmer_spectrum(reads, K)), K
            assert st["n_overflow"] > 0  # the global path ran
        got, pst = ctx.precorrect(reads, K=24)
        d = ctx.upload(reads)
        fh, fks, _ = ctx.spectrum_precorrect(d, K_spec=25, K=24)  # the K+1 pass's global table
        d.free()
    assert np.array_equal(fh, oracle.kmer_spectrum(reads, 25))
    assert fks["n_kmers"] == st["n_kmers"] and fks["n_overflow"] > 0
    exp, est = oracle.precorrect(reads, K=24)
    assert np.array_equal(got.packed[: int(got.byte_off[-1])], exp.packed[: int(exp.byte_off[-1])])
    assert np.array_equal(got.quals, exp.quals)
    assert pst["n_solid"] == est["n_solid"]


@pytest.mark.parametrize("mode", ["lds", "bad"])
def test_overflow_sub_buckets(rep_reads, monkeypatch, mode):
    """Overflowed buckets counted by sub-bucket (the default): their K-mer
    instances as entries, one partition level by hash digit inside each
    bucket, an LDS count per sub-bucket and the weak bits from a second read
    of its entries; "bad" sends every sub-bucket through the global-table
    fallback of the ones that fill the LDS table.  Spectrum (K=24, 25, every
    dedup mode's overflow), solid set, corrections and the fused entry point
    (whose K+1 pass counts its overflowed buckets' owned K+1-mers the same
    way) equal the oracle."""
    if mode == "bad":
        monkeypatch.setenv("APG_SK_OVF", "bad")
    else:
        monkeypatch.delenv("APG_SK_OVF", raising=False)
    _, reads = rep_reads
    with Context(device=0) as ctx:
        for K in (24, 25):
            hist, st = ctx.kmer_spectrum(reads, K)
            assert np.array_equal(hist, oracle.kmer_spectrum(reads, K)), K
            assert st["n_overflow"] > 0
        got, pst = ctx.precorrect(reads, K=24)
        d = ctx.upload(reads)
        fh, fks, fps = ctx.spectrum_precorrect(d, K_spec=25, K=24)
        fixed = ctx.download(d, with_quals=True)
        d.free()
    assert fks["n_kmers"] == st["n_kmers"] and fks["n_distinct"] == st["n_distinct"] and fks["n_overflow"] > 0
    exp, est = oracle.precorrect(reads, K=24)
    for g in (got, fixed):
        assert np.array_equal(g.packed[: int(g.byte_off[-1])], exp.packed[: int(exp.byte_off[-1])])
        assert np.array_equal(g.quals, exp.quals)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert pst[k] == est[k] and fps[k] == est[k], k
    assert np.array_equal(fh, oracle.kmer_spectrum(reads, 25))
