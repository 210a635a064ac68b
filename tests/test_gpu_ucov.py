"""GPU parity: UnipathCoverage (apg_unipath_coverage, host and device
placements) vs the CPU restatement oracle/ucov_oracle.c — counts, per-K-mer
coverage (bitwise: the same IEEE divisions), c0 and copy numbers exact; and a
known-answer case: a 400-bp repeat present twice in the genome is estimated
at copy number 2, the unique sequence at 1.  Parity vs real ALLPATHS-LG:
unpinned (reference empty)."""
import numpy as np
import pytest

import oracle
from allpathslg_amd import synth_genome, synth_reads
from tests.unipath_cases import noisy_reads, repeat_genome, tiling

pytestmark = pytest.mark.gpu


def check(ctx, g, locs, min_len):
    U = int(g["n_unipaths"])
    exp = oracle.unipath_coverage(g, locs, min_len)
    got, st = ctx.unipath_coverage(locs, U, min_len=min_len)
    assert np.array_equal(got["counts"], exp["counts"])
    assert np.array_equal(got["cov"], exp["cov"])
    assert np.array_equal(got["cn"], exp["cn"])
    assert st["c0"] == exp["c0"] and st["n_long"] == exp["n_long"]
    return got, st


@pytest.mark.parametrize("rc,sorted_", [(True, True), (True, False), (False, False)])
def test_coverage_matches_oracle(gpu_ctx, rc, sorted_):
    reads = noisy_reads(G=60_000, n=30_000, L=100, err=0.003, seed=21)
    g, _ = gpu_ctx.unipaths(reads, 31)
    locs, _ = gpu_ctx.unipath_locs(reads, rc=rc, sorted=sorted_)
    for min_len in (1, 200, 10**9):
        check(gpu_ctx, g, locs, min_len)


def test_device_placements_of_a_full_size_chain(gpu_ctx):
    """Fragments of a 2-Mb genome at 60x through the K=96 graph, placements
    left on the device (apg_unipath_locs_dev -> apg_unipath_coverage_dev)."""
    from allpathslg_amd import synth_fragments

    gen = synth_genome(2_000_000, 22)
    frags = synth_fragments(gen, 600_000, seed=23)
    g, _ = gpu_ctx.unipaths(frags, 96)
    reads = synth_reads(gen, 300_000, seed=24)
    d = gpu_ctx.upload(reads)
    ptr, n, _ = gpu_ctx.unipath_locs(d)
    got, st = gpu_ctx.unipath_coverage(ptr, int(g["n_unipaths"]), n_locs=n)
    host, _ = gpu_ctx.unipath_locs(reads)
    exp = oracle.unipath_coverage(g, host, 500)
    assert np.array_equal(got["counts"], exp["counts"]) and np.array_equal(got["cn"], exp["cn"])
    assert st["c0"] == exp["c0"] > 0
    long_ = g["len"] >= 500
    assert np.mean(got["cn"][long_] == 1) > 0.99  # a repeat-free genome: one copy
    d.free()


def test_repeat_copy_number_known_answer(gpu_ctx):
    gen = repeat_genome(seed=25, unique=3000, rlen=400)  # A R B R C
    reads = tiling(gen, L=150, step=2)
    g, _ = gpu_ctx.unipaths(reads, 96)
    locs, _ = gpu_ctx.unipath_locs(reads)
    got, st = check(gpu_ctx, g, locs, 500)
    lens = g["len"]
    # the repeat's unipath pair: the two shortest multi-K-mer unipaths of ~rlen-K+1 K-mers
    rep = [u for u in range(int(g["n_unipaths"])) if 250 <= lens[u] <= 400]
    uniq = [u for u in range(int(g["n_unipaths"])) if lens[u] >= 2000]
    assert rep and uniq
    assert all(got["cn"][u] == 2 for u in rep), [(int(lens[u]), int(got["cn"][u])) for u in rep]
    assert all(got["cn"][u] == 1 for u in uniq)
