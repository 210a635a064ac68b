"""Known-answer and property tests of the UnipathLocs restatement
(oracle/locs_oracle.c; spec include/apg.h apg_unipath_locs).  CPU only.
Parity vs real ALLPATHS-LG: unpinned (reference empty)."""
import numpy as np

import oracle
from allpathslg_amd import ReadSet
from tests.locs_cases import linear_case, repeat_case, sampled_reads


def ub(g, u):
    return g["unibases"][int(g["ub_off"][u]) : int(g["ub_off"][u + 1])]


def assert_locs_consistent(g, reads, locs, K, exact=True):
    """Every location aligns its read (rc read for mirrors) gap-free to the
    unibase over their overlap (exact) or, for reads with errors, on >= K
    consecutive bases of the overlap."""
    for r, u, s, f in locs.tolist():
        seq = reads.read(r)
        if f:
            seq = (3 - seq[::-1]).astype(np.uint8)
        t = ub(g, u)
        lo, hi = max(0, -s), min(len(seq), len(t) - s)
        assert hi - lo >= K, (r, u, s, f)
        eq = seq[lo:hi] == t[s + lo : s + hi]
        if exact:
            assert eq.all(), (r, u, s, f)
        else:
            run = best = 0
            for e in eq.tolist():
                run = run + 1 if e else 0
                best = max(best, run)
            assert best >= K, (r, u, s, f)


def test_linear_error_free_one_location_per_read():
    """Repeat-free genome: one unipath pair; every error-free read gets exactly
    one location (plus its mirror), at its true genome offset on the unipath
    that spells the genome forward."""
    K = 96
    genome, frags = linear_case()
    g = oracle.unipaths(frags, K)
    assert g["n_unipaths"] == 2
    fw = 0 if np.array_equal(ub(g, 0), genome) else 1
    assert np.array_equal(ub(g, fw), genome)
    reads, starts, rcs = sampled_reads(genome, n=300)
    locs, st = oracle.unipath_locs(g, reads, K, rc=True, sorted=False)
    assert st["n_placed"] == reads.n_reads and st["n_missing"] == 0
    assert len(locs) == 2 * reads.n_reads
    own, mirror = locs[0::2], locs[1::2]
    assert np.array_equal(own[:, 0], np.arange(reads.n_reads)) and (own[:, 3] == 0).all() and (mirror[:, 3] == 1).all()
    Lg = len(genome)
    for r in range(reads.n_reads):
        u, s = int(own[r, 1]), int(own[r, 2])
        if not rcs[r]:
            assert (u, s) == (fw, starts[r])
        else:  # rc read on the reverse unipath
            assert (u, s) == (1 - fw, Lg - starts[r] - 100)
        assert int(mirror[r, 1]) == int(g["rc"][u])
    assert_locs_consistent(g, reads, locs, K)


def test_error_in_every_kmer_is_unplaced():
    """A substitution at base 50 of a 100-bp read hits all five 96-mers."""
    K = 96
    genome, frags = linear_case()
    g = oracle.unipaths(frags, K)
    r = genome[1000:1100].copy()
    r[50] = (r[50] + 1) % 4
    locs, st = oracle.unipath_locs(g, ReadSet.from_sequences([r, genome[2000:2100]]), K)
    assert st["n_placed"] == 1 and st["n_missing"] == 5
    assert set(locs[:, 0].tolist()) == {1}


def test_repeat_reads_switch_unipaths():
    """A R B R C: reads crossing a repeat boundary touch two unipaths (one
    location each); the set agrees with the gap-free property."""
    K = 96
    genome, frags = repeat_case()
    g = oracle.unipaths(frags, K)
    reads, _, _ = sampled_reads(genome, n=400, L=150, seed=9)
    locs, st = oracle.unipath_locs(g, reads, K, rc=False, sorted=False)
    per_read = np.bincount(locs[:, 0], minlength=reads.n_reads)
    assert per_read.max() >= 2 and st["n_placed"] == reads.n_reads
    assert_locs_consistent(g, reads, locs, K)


def test_sorted_is_stable_permutation():
    K = 63
    genome, frags = repeat_case()
    g = oracle.unipaths(frags, K)
    reads, _, _ = sampled_reads(genome, n=500, err=0.004, seed=4, ragged=True)
    a, _ = oracle.unipath_locs(g, reads, K, rc=True, sorted=False)
    b, _ = oracle.unipath_locs(g, reads, K, rc=True, sorted=True)
    order = np.lexsort((np.arange(len(a)), a[:, 2], a[:, 1]))
    assert np.array_equal(a[order], b)
    assert_locs_consistent(g, reads, b, K, exact=False)


def test_empty_and_short_reads():
    K = 96
    genome, frags = linear_case(G=5000)
    g = oracle.unipaths(frags, K)
    reads = ReadSet.from_sequences([genome[:50], genome[100:196], np.zeros(0, np.uint8)])
    locs, st = oracle.unipath_locs(g, reads, K)
    assert st["n_placed"] == 1 and len(locs) == 2 and locs[0, 0] == 1


def test_oracle_against_golden_locs_and_ecj():
    """The restatements reproduce the committed fixtures (tests/golden,
    make_golden.py write_locs_ecj_fixture)."""
    import os

    gdir = os.path.join(os.path.dirname(__file__), "golden")
    z = np.load(os.path.join(gdir, "locs_ecj_small.npz"))
    reads = ReadSet.load(os.path.join(gdir, "frag_small.fastb"), os.path.join(gdir, "frag_small.qualb"))
    frags = ReadSet.load(os.path.join(gdir, "frag_small_fill.fastb"))
    g = oracle.unipaths(frags, 96)
    locs, st = oracle.unipath_locs(g, reads, 96, rc=True, sorted=True)
    assert np.array_equal(locs, z["locs"]) and [st["n_placed"], st["n_missing"]] == z["locs_stats"].tolist()
    jumps = ReadSet.load(os.path.join(gdir, "jump_small.fastb"), os.path.join(gdir, "jump_small.qualb"))
    fixed, keep, est = oracle.error_correct_jump(reads, jumps, K=24)
    assert np.array_equal(fixed.packed[: int(fixed.byte_off[-1])], z["ecj_packed"])
    assert np.array_equal(fixed.quals, z["ecj_quals"]) and np.array_equal(keep, z["ecj_keep"])
