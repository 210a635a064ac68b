"""Known-answer and property tests of the unipath oracle (CPU only; SURVEY
§A.8(3),(4)).  Parity vs real ALLPATHS-LG: unpinned (reference empty)."""
import numpy as np
import pytest

import oracle
from allpathslg_amd import synth_genome
from tests.unipath_cases import (circular_reads, noisy_reads, palindrome_reads, rc_str, repeat_genome, tiling,
                                 unibase_str)


def gstr(g):
    return "".join("ACGT"[x] for x in g)


def check_invariants(u, reads, K):
    U = u["n_unipaths"]
    assert int(u["len"].sum()) == 2 * u["n_nodes"]  # every directed K-mer in exactly one unipath
    for i in range(U):
        j = int(u["rc"][i])
        assert int(u["rc"][j]) == i
        assert unibase_str(u, j) == rc_str(unibase_str(u, i))
        assert int(u["ub_off"][i + 1] - u["ub_off"][i]) == K - 1 + int(u["len"][i])
    assert np.array_equal(u["id_base"], np.concatenate([[0], np.cumsum(u["len"])[:-1]]).astype(np.uint64))
    for r in range(reads.n_reads):
        a, b = int(u["path_off"][r]), int(u["path_off"][r + 1])
        L = int(reads.base_off[r + 1] - reads.base_off[r])
        assert int(u["path_len"][a:b].sum()) == max(0, L - K + 1)


def test_linear_genome_single_pair():
    """§A.8(3): random genome, no K-repeat: one unipath pair of length G-K+1."""
    K, G = 96, 5000
    g = synth_genome(G, 3)
    reads = tiling(g)
    u = oracle.unipaths(reads, K)
    assert u["n_unipaths"] == 2
    assert list(u["len"]) == [G - K + 1] * 2
    s = {unibase_str(u, 0), unibase_str(u, 1)}
    assert s == {gstr(g), rc_str(gstr(g))}
    assert u["n_vertices"] == 4
    check_invariants(u, reads, K)


def test_inserted_repeat_structure():
    """§A.8(4): A R B R C -> A', R, B', C' per strand; junction vertices shared."""
    K = 96
    g = repeat_genome()
    reads = tiling(g, L=200, step=5)
    u = oracle.unipaths(reads, K)
    assert u["n_unipaths"] == 8
    lens = sorted(int(x) for x in u["len"])
    # effective repeat = R extended by the flanks its two copies happen to share
    unique, rlen = 3000, 400
    A, B, C = g[:unique], g[unique + rlen : 2 * unique + rlen], g[2 * unique + 2 * rlen :]
    left = next(i for i in range(1, unique) if A[-i] != B[-i]) - 1
    right = next(i for i in range(unique) if B[i] != C[i])
    assert lens.count(rlen + left + right - K + 1) == 2
    assert u["n_vertices"] == 8
    check_invariants(u, reads, K)


def test_circular_genome_cut_once():
    K, G = 63, 3000
    g = synth_genome(G, 11)
    reads = circular_reads(g)
    u = oracle.unipaths(reads, K)
    assert u["n_unipaths"] == 2
    assert list(u["len"]) == [G, G]
    s0 = unibase_str(u, 0)
    assert len(s0) == G + K - 1
    circ = gstr(g) * 2
    assert s0 in circ or rc_str(s0) in circ
    check_invariants(u, reads, K)


def test_palindromic_kmers():
    K = 4
    reads = palindrome_reads()
    u = oracle.unipaths(reads, K)
    check_invariants(u, reads, K)


@pytest.mark.parametrize("K", [25, 64, 96])
def test_noisy_reads_invariants(K):
    reads = noisy_reads(G=20_000, n=3000)
    u = oracle.unipaths(reads, K)
    assert u["n_unipaths"] > 10
    check_invariants(u, reads, K)


GOLDEN_KEYS = ("len", "id_base", "rc", "ub_off", "unibases", "from", "to", "path_off", "path_start", "path_len")


@pytest.mark.parametrize("threads,parcel", [(1, None), (8, None), (3, "5000"), (8, "777")])
def test_oracle_graph_equals_golden_fixture(threads, parcel, monkeypatch):
    """The restatement (hash-parcelled node fold, hash node index, one-pass
    read paths since round 6) against the committed golden graphs
    (tests/golden/stages_small.npz, written by the round-1 sort-based form):
    at one and several threads, and with parcels forced small so that the
    node fold takes several passes."""
    import os

    from allpathslg_amd import ReadSet

    gold = os.path.join(os.path.dirname(__file__), "golden")
    z = np.load(os.path.join(gold, "stages_small.npz"))
    reads = ReadSet.load(os.path.join(gold, "frag_small.fastb"), os.path.join(gold, "frag_small.qualb"))
    frags = ReadSet.load(os.path.join(gold, "frag_small_fill.fastb"))
    if parcel:
        monkeypatch.setenv("ORU_PARCEL_INSTANCES", parcel)
    before = oracle.threads()
    oracle.set_threads(threads)
    try:
        for K, src in ((31, reads), (96, frags)):
            g = oracle.unipaths(src, K)
            for key in GOLDEN_KEYS:
                assert np.array_equal(np.asarray(g[key]), z[f"u{K}_{key}"]), (K, key)
    finally:
        oracle.set_threads(before)
