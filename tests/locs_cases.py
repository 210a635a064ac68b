"""Shared inputs for the UnipathLocs tests (test infrastructure)."""
import numpy as np

from allpathslg_amd import ReadSet, synth_genome
from tests.unipath_cases import repeat_genome, tiling


def sampled_reads(g, n=400, L=100, err=0.0, seed=3, rc_frac=0.5, ragged=False):
    """n reads drawn from genome g (half reverse-complemented), optional
    substitutions and ragged lengths; returns (ReadSet, starts, rc flags)."""
    rng = np.random.default_rng(seed)
    seqs, quals, starts, rcs = [], [], [], []
    for _ in range(n):
        Lr = int(rng.integers(60, 140)) if ragged else L
        s = int(rng.integers(0, len(g) - Lr + 1))
        r = g[s : s + Lr].copy()
        m = rng.random(Lr) < err
        r[m] = (r[m] + 1 + rng.integers(0, 3, size=int(m.sum()))) % 4
        q = np.where(m, 10, 40).astype(np.uint8)
        rc = bool(rng.random() < rc_frac)
        if rc:
            r = (3 - r[::-1]).copy()
            q = q[::-1].copy()
        seqs.append(r)
        quals.append(q)
        starts.append(s)
        rcs.append(rc)
    return ReadSet.from_sequences(seqs, quals), np.array(starts), np.array(rcs)


def linear_case(G=20_000, seed=3):
    g = synth_genome(G, seed)
    return g, tiling(g)


def repeat_case():
    g = repeat_genome()
    return g, tiling(g, L=200, step=5)
