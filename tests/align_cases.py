"""Shared inputs for the aligner / consensus tests (pure numpy)."""
import numpy as np

from allpathslg_amd import ReadSet


def mutate(seq, rng, sub=0.03, ins=0.01, dele=0.01):
    out = []
    for b in seq:
        r = rng.random()
        if r < dele:
            continue
        if r < dele + ins:
            out.append(int(rng.integers(0, 4)))
        out.append(int((b + 1 + rng.integers(0, 3)) % 4) if rng.random() < sub else int(b))
    return np.array(out, dtype=np.uint8)


def sw_case(n_targets=20, n_pairs=400, tlen=600, slen=(60, 160), seed=5, rc_frac=0.5):
    """Targets, queries drawn from them with substitutions/indels, and pairs
    (s, t, offset, flags) with offsets near the true placement."""
    rng = np.random.default_rng(seed)
    targets = [rng.integers(0, 4, size=int(tlen + rng.integers(-100, 100))).astype(np.uint8) for _ in range(n_targets)]
    seqs, quals, pairs = [], [], []
    for k in range(n_pairs):
        t = int(rng.integers(0, n_targets))
        L = int(rng.integers(*slen))
        st = int(rng.integers(-20, len(targets[t]) - L + 20))
        src = targets[t][max(st, 0): max(st, 0) + L]
        s = mutate(src, rng)
        rc = rng.random() < rc_frac
        seqs.append((3 - s)[::-1].copy() if rc else s)
        quals.append(rng.integers(2, 41, size=len(s)).astype(np.uint8))
        off = max(st, 0) + int(rng.integers(-4, 5))
        pairs.append((k, t, off, 1 if rc else 0))
    return ReadSet.from_sequences(seqs, quals), ReadSet.from_sequences(targets), np.array(pairs, dtype=np.int64)


def full_dp_cost(S, T):
    """Semi-global min cost (all of S, free T ends), no band: plain python."""
    INF = 1 << 30
    n, m = len(S), len(T)
    prev = [0] * (m + 1)
    for i in range(1, n + 1):
        cur = [INF] * (m + 1)
        cur[0] = prev[0] + 3
        for j in range(1, m + 1):
            cur[j] = min(prev[j - 1] + (0 if S[i - 1] == T[j - 1] else 2), cur[j - 1] + 3, prev[j] + 3)
        prev = cur
    return min(prev)


def apply_blocks(S, T, t_begin, blocks):
    """Replay blocks: (cost, columns) with mismatch 2, gap 3."""
    i, j, cost = 0, t_begin, 0
    for g, ln in blocks:
        if g > 0:
            j += g
            cost += 3 * g
        elif g < 0:
            i += -g
            cost += 3 * -g
        for _ in range(ln):
            cost += 0 if S[i] == T[j] else 2
            i += 1
            j += 1
    return cost, i, j
