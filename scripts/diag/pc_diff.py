"""Diagnose a PreCorrect GPU/oracle mismatch: per-read diff of bases/quals."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import oracle
from allpathslg_amd import Context, synth_genome, synth_reads

g = synth_genome(200_000, 31)
reads = synth_reads(g, 40_000, seed=32)
with Context(device=0, timing=False) as ctx:
    got, st = ctx.precorrect(reads, K=24, n_cycles=1)
exp, est = oracle.precorrect(reads, K=24, n_cycles=1)
print("gpu", st)
print("cpu", est)
nb = 0
for r in range(reads.n_reads):
    a, b = int(reads.byte_off[r]), int(reads.byte_off[r + 1])
    q0, q1 = int(reads.base_off[r]), int(reads.base_off[r + 1])
    if not np.array_equal(got.packed[a:b], exp.packed[a:b]) or not np.array_equal(got.quals[q0:q1], exp.quals[q0:q1]):
        def bases(x):
            return np.array([(x.packed[a + i // 4] >> (2 * (i % 4))) & 3 for i in range(q1 - q0)])
        bo, bg, be = bases(reads), bases(got), bases(exp)
        print("read", r, "L", q1 - q0)
        print("  orig low-q", np.nonzero(reads.quals[q0:q1] < 20)[0].tolist())
        print("  gpu edits", [(int(i), int(bo[i]), int(bg[i])) for i in np.nonzero(bo != bg)[0]])
        print("  cpu edits", [(int(i), int(bo[i]), int(be[i])) for i in np.nonzero(bo != be)[0]])
        print("  qual diff", np.nonzero(got.quals[q0:q1] != exp.quals[q0:q1])[0].tolist())
        nb += 1
        if nb >= 12:
            break
