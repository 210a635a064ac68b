"""Known-answer tests of the ErrorCorrectJump restatement (correction against
the fragment reads' solid set + prefix trimming; oracle/ecj_oracle.c, spec in
include/apg.h apg_error_correct_jump).  CPU only.  Parity vs real ALLPATHS-LG:
unpinned (reference empty)."""
import numpy as np

import oracle
from allpathslg_amd import ReadSet, synth_genome
from tests.unipath_cases import tiling

K = 24


def frag_set(G=20_000, seed=3):
    g = synth_genome(G, seed)
    # error-free tiling at ~14x: every genome K-mer is solid (count >= 3)
    return g, tiling(g, L=100, step=7)


def read_with(g, start, subs=(), L=100, q_err=10):
    r = g[start : start + L].copy()
    q = np.full(L, 40, np.uint8)
    for p in subs:
        r[p] = (r[p] + 1) % 4
        q[p] = q_err
    return r, q


def test_kats():
    g, frags = frag_set()
    rng = np.random.default_rng(1)
    cases = [
        (read_with(g, 1000, [50], q_err=10), 100),  # low-quality error: corrected, kept whole
        (read_with(g, 2000, [70], q_err=40), 70),   # confident error: not a suspect; trimmed at it
        (read_with(g, 3000, [10], q_err=40), 0),    # trim below min_keep: dropped
        (read_with(g, 4000, []), 100),              # clean
        ((rng.integers(0, 4, 100).astype(np.uint8), np.full(100, 40, np.uint8)), 0),  # novel sequence
        ((g[5000:5020].copy(), np.full(20, 40, np.uint8)), 0),  # shorter than K
    ]
    jumps = ReadSet.from_sequences([c[0][0] for c in cases], [c[0][1] for c in cases])
    fixed, keep, st = oracle.error_correct_jump(frags, jumps, K=K)
    assert keep.tolist() == [c[1] for c in cases]
    assert np.array_equal(fixed.read(0), g[1000:1100])  # the Q10 error was corrected
    assert st["n_corrected"] >= 1


def test_trim_is_first_weak_kmer_plus_k_minus_1():
    g, frags = frag_set(seed=5)
    seqs, quals, expect = [], [], []
    for p in range(30, 100, 7):  # confident error at p: first weak K-mer p-K+1, keep = p
        r, q = read_with(g, 100 + 13 * p, [p], q_err=40)
        seqs.append(r)
        quals.append(q)
        expect.append(p if p >= 40 else 0)
    fixed, keep, _ = oracle.error_correct_jump(frags, ReadSet.from_sequences(seqs, quals), K=K)
    assert keep.tolist() == expect


def test_min_keep_parameter():
    g, frags = frag_set(seed=7)
    r, q = read_with(g, 500, [35], q_err=40)
    _, keep, _ = oracle.error_correct_jump(frags, ReadSet.from_sequences([r], [q]), K=K, min_keep=30)
    assert keep.tolist() == [35]
    _, keep, _ = oracle.error_correct_jump(frags, ReadSet.from_sequences([r], [q]), K=K, min_keep=36)
    assert keep.tolist() == [0]
