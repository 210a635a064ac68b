"""Constructed FillFragments cases with known answers (SURVEY §A.8 style):
pairs cut from a random genome whose K-mers are the solid set, plus a second
path (ambiguity), a dead-end branch (backtracking), weak reads, short reads.
Shared by tests/test_fill_oracle.py (CPU) and tests/test_gpu_fill.py."""
import numpy as np

import oracle
from allpathslg_amd import ReadSet

K = 24


def rc(s):
    return (3 - np.asarray(s, np.uint8))[::-1].copy()


def solid_of(seqs, K=K):
    """Hashes of every canonical K-mer of the given sequences (count >= 1)."""
    return oracle.solid_hashes(ReadSet.from_sequences(seqs), K, 1)


def genome_cases(seed=5, glen=6000):
    """(pairs ReadSet, solid hashes, expected list of (status, fragment or None))."""
    rng = np.random.default_rng(seed)
    G = rng.integers(0, 4, glen).astype(np.uint8)
    seqs, exp = [], []

    def pair(s, I, La=100, Lf=100, mutate_a=None):
        A = G[s : s + La].copy()
        F = G[s + I - Lf : s + I].copy()
        if mutate_a is not None:
            A[mutate_a] = (A[mutate_a] + 1) % 4
        seqs.extend([A, rc(F)])

    for j, I in enumerate([120, 126, 130, 150, 176, 177, 180, 190, 199, 200, 201, 215, 234, 235, 250]):
        s = 50 + 300 * j
        pair(s, I)
        ok = 126 <= I <= 234
        exp.append((0, G[s : s + I].copy()) if ok else (1, None))
    # unequal read lengths
    for j, (La, Lf, I) in enumerate([(80, 120, 170), (120, 80, 230), (90, 90, 200), (40, 140, 190)]):
        s = 4700 + 250 * j if j < 3 else 300
        pair(s, I, La, Lf)
        exp.append((0, G[s : s + I].copy()))
    # a weak K-mer inside A (substitution mid-read): no path of solid K-mers
    pair(1000, 180, mutate_a=50)
    exp.append((1, None))
    # reads shorter than K, and a gap longer than the walk allows
    seqs.extend([G[10:30].copy(), rc(G[150:250])])
    exp.append((4, None))
    seqs.extend([G[10:60].copy(), rc(G[150:200])])
    exp.append((4, None))
    return ReadSet.from_sequences(seqs), solid_of([G]), exp, G


def branch_cases(seed=9):
    """Two bridging paths (AMBIGUOUS), a dead-end branch (backtrack, OK), and
    a budget too small for the walk (BUDGET)."""
    rng = np.random.default_rng(seed)
    X = rng.integers(0, 4, 140).astype(np.uint8)
    Y = rng.integers(0, 4, 140).astype(np.uint8)
    g1 = rng.integers(0, 4, 20).astype(np.uint8)
    g2 = rng.integers(0, 4, 27).astype(np.uint8)
    tip = np.concatenate([g1[:6], rng.integers(0, 4, 12).astype(np.uint8)])
    P1 = np.concatenate([X, g1, Y])
    P2 = np.concatenate([X, g2, Y])
    A = X[-100:].copy()
    F = Y[:100].copy()
    seqs = [A, rc(F), A, rc(F)]
    solid_two = solid_of([P1, P2])
    solid_tip = solid_of([P1, np.concatenate([X, tip])])
    frag1 = np.concatenate([A, g1, F])
    return ReadSet.from_sequences(seqs), solid_two, solid_tip, frag1
