"""CPU: the FillFragments restatement (oracle/fill_oracle.c) against known
answers and its committed golden fixture.  Parity vs real ALLPATHS-LG:
unpinned (reference snapshot empty)."""
import os

import numpy as np

import oracle
from allpathslg_amd import ReadSet
from tests.fill_cases import K, branch_cases, genome_cases

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fill_known_answers():
    pairs, solid, exp, _ = genome_cases()
    filled, status, flen, st = oracle.fill_fragments(pairs, solid, K=K)
    assert list(status) == [e[0] for e in exp]
    j = 0
    for i, (s, frag) in enumerate(exp):
        if s == 0:
            assert flen[i] == len(frag)
            assert np.array_equal(filled.read(j), frag), i
            j += 1
        else:
            assert flen[i] == 0
    assert filled.n_reads == j == st["n_filled"]


def test_fill_branches():
    pairs, solid_two, solid_tip, frag1 = branch_cases()
    _, status, _, _ = oracle.fill_fragments(pairs, solid_two, K=K)
    assert list(status) == [2, 2]  # two bridging paths
    filled, status, flen, _ = oracle.fill_fragments(pairs, solid_tip, K=K)
    assert list(status) == [0, 0]  # the dead-end branch is backtracked
    assert np.array_equal(filled.read(0), frag1)
    _, status, _, _ = oracle.fill_fragments(pairs, solid_tip, K=K, max_steps=5)
    assert list(status) == [3, 3]


def test_fill_bounds_and_empty():
    pairs, solid, exp, _ = genome_cases()
    # a window that admits no insert of these pairs
    _, status, _, st = oracle.fill_fragments(pairs, solid, K=K, min_insert=400, max_insert=420)
    assert st["n_filled"] == 0
    empty = ReadSet.from_sequences([])
    f, status, flen, st = oracle.fill_fragments(empty, solid, K=K)
    assert f.n_reads == 0 and len(status) == 0


def test_fill_golden_fixture():
    g = np.load(os.path.join(HERE, "golden", "fill_small.npz"))
    reads = ReadSet.load(os.path.join(HERE, "golden", "frag_small.fastb"), os.path.join(HERE, "golden", "frag_small.qualb"))
    fixed, _ = oracle.precorrect(reads, K=24)
    solid = oracle.solid_hashes(reads, 24, 3)
    assert np.array_equal(np.sort(solid), g["solid"])
    filled, status, flen, st = oracle.fill_fragments(fixed, solid, K=24, min_insert=126, max_insert=234)
    assert np.array_equal(status, g["status"])
    assert np.array_equal(flen, g["flen"])
    assert np.array_equal(filled.base_off, g["base_off"])
    assert np.array_equal(filled.packed[: int(filled.byte_off[-1])], g["packed"])
