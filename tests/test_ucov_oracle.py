"""UnipathCoverage restatement (oracle/ucov_oracle.c) against a pure-Python
statement of the spec in include/apg.h (apg_unipath_coverage): counts,
placements per K-mer, the length-weighted median c0 and copy numbers,
including ties at the median, no long unipath (c0 = 0) and empty input."""
import math

import numpy as np
import pytest

import oracle


def py_cov(lens, locs, min_len):
    U = len(lens)
    counts = np.zeros(U, np.uint64)
    for r in locs:
        counts[r[1]] += 1
    cov = np.array([c / l if l else 0.0 for c, l in zip(counts, lens)])
    items = sorted((cov[u], lens[u]) for u in range(U) if lens[u] >= min_len)
    W = sum(l for _, l in items)
    c0, acc = 0.0, 0
    for c, l in items:
        acc += l
        if 2 * acc >= W:
            c0 = c
            break
    cn = np.array([math.floor(c / c0 + 0.5) if c0 > 0 else 0 for c in cov], np.uint32)
    return counts, cov, cn, c0


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_random_graphs(seed):
    rng = np.random.default_rng(seed)
    U = int(rng.integers(1, 400))
    lens = rng.integers(1, 3000, U).astype(np.uint64)
    n = int(rng.integers(0, 20000))
    locs = np.zeros((n, 4), np.int32)
    locs[:, 0] = rng.integers(0, 5000, n)
    locs[:, 1] = rng.integers(0, U, n)
    locs[:, 2] = rng.integers(-50, 3000, n)
    g = {"n_unipaths": U, "len": lens}
    for min_len in (1, 500, 2500, 10**9):
        got = oracle.unipath_coverage(g, locs, min_len)
        counts, cov, cn, c0 = py_cov(lens, locs, min_len)
        assert np.array_equal(got["counts"], counts)
        assert np.array_equal(got["cov"], cov)
        assert got["c0"] == c0
        assert np.array_equal(got["cn"], cn)


def test_known_answers():
    # two long unique unipaths at 1 placement / K-mer, a 2-copy and a 3-copy
    # repeat, an error path with a tenth of the coverage
    lens = np.array([1000, 1200, 600, 700, 100], np.uint64)
    per_kmer = [1.0, 1.0, 2.0, 3.0, 0.1]
    locs = []
    for u, (l, c) in enumerate(zip(lens, per_kmer)):
        locs += [(0, u, 0, 0)] * int(round(l * c))
    got = oracle.unipath_coverage({"n_unipaths": 5, "len": lens}, np.array(locs, np.int32), 500)
    assert got["c0"] == 1.0 and got["n_long"] == 4
    assert got["cn"].tolist() == [1, 1, 2, 3, 0]
    # the weighted median sits on the 2-copy unipath once it carries half the length
    lens2 = np.array([1000, 600, 5000], np.uint64)
    locs2 = [(0, 0, 0, 0)] * 1000 + [(0, 1, 0, 0)] * 1200 + [(0, 2, 0, 0)] * 10000
    got = oracle.unipath_coverage({"n_unipaths": 3, "len": lens2}, np.array(locs2, np.int32), 500)
    assert got["c0"] == 2.0 and got["cn"].tolist() == [1, 1, 1]


def test_empty_and_no_long_unipath():
    g = {"n_unipaths": 3, "len": np.array([10, 20, 30], np.uint64)}
    got = oracle.unipath_coverage(g, np.zeros((0, 4), np.int32), 500)
    assert got["c0"] == 0.0 and got["n_long"] == 0 and got["cn"].tolist() == [0, 0, 0]
    with pytest.raises(RuntimeError):
        oracle.unipath_coverage(g, np.array([[0, 7, 0, 0]], np.int32), 1)
