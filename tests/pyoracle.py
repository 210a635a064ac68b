"""Pure-Python restatement of SURVEY §A.3 for SMALL cases — an independent
second implementation used to check the C oracle (test infrastructure)."""
from collections import Counter

import numpy as np


def canonical_kmers(seq, K):
    """Canonical K-mer integer keys of one read (list of 0..3 codes)."""
    out = []
    n = len(seq)
    for i in range(n - K + 1):
        fw = 0
        rc = 0
        for j in range(K):
            fw = fw * 4 + int(seq[i + j])
            rc = rc * 4 + (3 - int(seq[i + K - 1 - j]))
        out.append(min(fw, rc))
    return out


def count(reads, K):
    c = Counter()
    for i in range(reads.n_reads):
        c.update(canonical_kmers(reads.read(i), K))
    return c


def spectrum(counter, hist_len):
    h = np.zeros(hist_len, dtype=np.uint64)
    for v in counter.values():
        h[min(v, hist_len - 1)] += 1
    return h
