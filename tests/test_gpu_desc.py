"""Record descriptors (superkmer.hpp SkDesc): the count pass of the K <= 32
and K = 96 super-k-mer walks keeps one descriptor per record and the scatter
pass replays them instead of walking again; a block whose records overflow
its region walks again.  Every mode must give the same spectrum, PreCorrect
output and unipath graph: descriptors (default), none (APG_SK_DESC=0: every
scatter walks), and a region of one slot per 64 bases (most blocks overflow:
the replay and the walk mixed in one launch).  The default is also checked
against the oracle."""
import os

import numpy as np
import pytest

import oracle
from allpathslg_amd import synth_fragments, synth_genome, synth_reads

pytestmark = pytest.mark.gpu


def _run(ctx, reads, frags):
    h, st = ctx.kmer_spectrum(reads, 25)
    out, pst = ctx.precorrect(reads, K=24)
    g, ust = ctx.unipaths(frags, 96)
    return h, st, out, pst, g, ust


@pytest.fixture(scope="module")
def inputs():
    gen = synth_genome(1_000_000, 51)
    return synth_reads(gen, 100_000, seed=52), synth_fragments(gen, 40_000, seed=53)


@pytest.mark.parametrize("mode", ["0", "64", "1"])
def test_modes_agree(gpu_ctx, inputs, mode):
    reads, frags = inputs
    ref = _run(gpu_ctx, reads, frags)
    old = os.environ.get("APG_SK_DESC")
    os.environ["APG_SK_DESC"] = mode
    try:
        got = _run(gpu_ctx, reads, frags)
    finally:
        if old is None:
            del os.environ["APG_SK_DESC"]
        else:
            os.environ["APG_SK_DESC"] = old
    h0, st0, out0, pst0, g0, ust0 = ref
    h1, st1, out1, pst1, g1, ust1 = got
    assert np.array_equal(h0, h1) and st0 == st1
    assert np.array_equal(out0.packed, out1.packed) and np.array_equal(out0.quals, out1.quals) and pst0 == pst1
    for k in ("len", "id_base", "rc", "unibases", "from", "to", "path_off", "path_start", "path_len"):
        assert np.array_equal(g0[k], g1[k]), k
    assert ust0["n_unipaths"] == ust1["n_unipaths"]


def test_default_matches_oracle(gpu_ctx, inputs):
    reads, _ = inputs
    h, _ = gpu_ctx.kmer_spectrum(reads, 25)
    ho = oracle.kmer_spectrum(reads, 25, len(h))
    assert np.array_equal(h, ho)


def test_reads_past_a_tile_and_past_16_bit_starts(gpu_ctx):
    """Reads longer than an LDS tile are walked from HBM by one thread; a
    record starting past base 65535 cannot be described in 16 bits, so its
    block walks again in the scatter pass.  Spectrum and unipaths = oracle."""
    from allpathslg_amd import ReadSet
    from tests.test_gpu_unipath import assert_graph_equal

    g = synth_genome(300_000, 61)
    rng = np.random.default_rng(62)
    seqs = [g[:150_000], g[100_000:170_000]]  # 150 kb and 70 kb reads: past 65535 and past a tile
    for _ in range(3000):
        s = int(rng.integers(0, len(g) - 200))
        seqs.append(g[s : s + 200])
    reads = ReadSet.from_sequences(seqs)
    h, _ = gpu_ctx.kmer_spectrum(reads, 25)
    assert np.array_equal(h, oracle.kmer_spectrum(reads, 25, len(h)))
    got, _ = gpu_ctx.unipaths(reads, 96)
    assert_graph_equal(got, oracle.unipaths(reads, 96))
