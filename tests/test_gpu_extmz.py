"""GPU parity with APG_EXT_MZ=1: the (K-1)-mer extension table with minimizer
homes (ext_table.hpp: 8-slot lines chosen by a (K-1)-mer's canonical 16-mer
minimizer, large classes at their own hash homes behind a marker).  Every
reader of the table — PreCorrect's decisions, FillFragments' walk and
overlap bridges, ErrorCorrectJump's trim and its reuse of the pass's table —
must give exactly the oracle's results; the repeat-rich genome exercises the
large-class markers, K = 24 / 20 / 27 and a K - 1 below 17 (plain homes)
the boundary."""
import numpy as np
import pytest

import oracle
from allpathslg_amd import Context, synth_fragments, synth_genome, synth_reads
from tests.test_gpu_ecj import run as run_ecj

pytestmark = pytest.mark.gpu


@pytest.fixture
def mz(monkeypatch):
    monkeypatch.setenv("APG_EXT_MZ", "1")


@pytest.mark.parametrize("repeats", [False, True])
@pytest.mark.parametrize("K", [24, 20, 27, 17])
def test_precorrect_and_fill_mz(gpu_ctx, mz, repeats, K):
    g = synth_genome(400_000, 61, repeats=True if repeats else None)
    reads = synth_reads(g, 120_000, seed=62)
    got, st = gpu_ctx.precorrect(reads, K=K)
    exp, est = oracle.precorrect(reads, K=K)
    assert np.array_equal(got.packed[: int(got.byte_off[-1])], exp.packed[: int(exp.byte_off[-1])])
    assert np.array_equal(got.quals, exp.quals)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert st[k] == est[k], k
    solid = oracle.solid_hashes(exp, K=K)
    fr, fs, fst = gpu_ctx.fill_fragments(exp, solid, K=K, status=True)
    er, es, _, est2 = oracle.fill_fragments(exp, solid, K=K)
    assert np.array_equal(fs, es)
    assert np.array_equal(fr.packed[: int(fr.byte_off[-1])], er.packed[: int(er.byte_off[-1])])
    for k in ("n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip"):
        assert fst[k] == est2[k], k


def test_ecj_mz(mz):
    g = synth_genome(300_000, 71, repeats=True)
    frags = synth_reads(g, 90_000, seed=72)
    jumps = synth_reads(g, 30_000, seed=73, insert_mean=3000, insert_sd=300)
    with Context(device=0) as ctx:
        run_ecj(ctx, frags, jumps, K=24)
        # the bench order: a counting PreCorrect pass of the fragments first,
        # whose table (and solid set) ErrorCorrectJump then reuses
        fixed, _ = ctx.precorrect(frags, K=24)
        run_ecj(ctx, fixed, jumps, K=24)
