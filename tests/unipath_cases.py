"""Shared inputs for the unipath tests (test infrastructure)."""
import numpy as np

from allpathslg_amd import ReadSet, synth_genome


def tiling(g, L=150, step=7):
    seqs = [g[s : s + L] for s in range(0, len(g) - L + 1, step)]
    seqs.append(g[len(g) - L :])
    return ReadSet.from_sequences(seqs)


def circular_reads(g, L=150, step=5):
    gg = np.concatenate([g, g[:L]])
    return ReadSet.from_sequences([gg[s : s + L] for s in range(0, len(g), step)])


def repeat_genome(seed=5, unique=3000, rlen=400):
    g = synth_genome(4 * unique + 2 * rlen, seed)
    A, B, C, R = g[:unique], g[unique : 2 * unique], g[2 * unique : 3 * unique], g[3 * unique : 3 * unique + rlen]
    return np.concatenate([A, R, B, R, C])


def noisy_reads(G=60_000, n=8000, L=100, err=0.01, seed=7):
    rng = np.random.default_rng(seed)
    g = synth_genome(G, seed)
    seqs = []
    for _ in range(n):
        s = int(rng.integers(0, G - L + 1))
        r = g[s : s + L].copy()
        if rng.random() < 0.5:
            r = (3 - r[::-1]).copy()
        m = rng.random(L) < err
        r[m] = (r[m] + 1 + rng.integers(0, 3, size=int(m.sum()))) % 4
        seqs.append(r)
    return ReadSet.from_sequences(seqs)


def palindrome_reads():
    # even K = 4: ACGT, GCGC, AATT ... are their own reverse complements
    code = {"A": 0, "C": 1, "G": 2, "T": 3}
    strs = ["AACGTT", "GACGTC", "ACGTACGT", "TTAATTAA", "CCGCGG", "AAAACGTTTT", "GGCGCC", "ACGCGT"]
    return ReadSet.from_sequences([[code[c] for c in s] for s in strs])


def rc_str(s):
    return "".join("TGCA"["ACGT".index(c)] for c in reversed(s))


def unibase_str(g, i):
    ub = g["unibases"][int(g["ub_off"][i]) : int(g["ub_off"][i + 1])]
    return "".join("ACGT"[x] for x in ub)
