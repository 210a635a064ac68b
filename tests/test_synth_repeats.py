"""Repeat injection of the synthetic genome (include/apg.h
apg_synth_repeats): deterministic, covers about the requested fractions,
and produces what the counting and graph stages must survive — K-mers with
counts in the hundreds (young family, tandem arrays) next to unique
sequence."""
import numpy as np

from allpathslg_amd import synth_genome


def kmer_counts(g, K):
    v = np.zeros(len(g) - K + 1, dtype=np.uint64)
    for i in range(K):
        v = (v << np.uint64(2)) | g[i : len(g) - K + 1 + i].astype(np.uint64)
    _, c = np.unique(v, return_counts=True)
    return c


def test_deterministic_and_seeded():
    a = synth_genome(500_000, 7, repeats=True)
    b = synth_genome(500_000, 7, repeats=True)
    c = synth_genome(500_000, 8, repeats=True)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert np.array_equal(synth_genome(500_000, 7), synth_genome(500_000, 7, repeats=False))


def test_fraction_and_multiplicity():
    G = 2_000_000
    plain = synth_genome(G, 9)
    rep = synth_genome(G, 9, repeats=True)
    changed = float(np.mean(plain != rep))
    # ~16 % of the bases overwritten, 3/4 of them by a different base
    assert 0.08 < changed < 0.16, changed
    c = kmer_counts(rep, 24)
    assert c.max() >= 100  # tandem arrays / the young family
    assert np.mean(c == 1) > 0.8  # most of the genome stays unique at K=24
    only_tandem = synth_genome(G, 9, repeats={"n_families": 0, "tandem_frac": 0.02})
    assert 0.01 < float(np.mean(plain != only_tandem)) < 0.03
