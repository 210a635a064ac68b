import sys
sys.path.insert(0, ".")
import numpy as np
import torch  # noqa: F401  (one HIP runtime)
import oracle
from allpathslg_amd import Context
from tests.unipath_cases import noisy_reads

ctx = Context(0)
reads = noisy_reads(G=20_000, n=2000, L=100)
g, _ = ctx.unipaths(reads, 15)
got = ctx.make_rc_db(g)["entries"]
exp = oracle.make_rc_db(g)["entries"]
s = got["start"].astype(np.int64)
print("n", len(got), "sorted frac", np.mean(np.diff(s) >= 0))
for bits in (8, 16, 24):
    m = s & ((1 << bits) - 1)
    print(bits, "low-bit sorted frac", np.mean(np.diff(m) >= 0))
ge = np.sort(got, order=["start", "flags", "read", "pos"])
ee = np.sort(exp, order=["start", "flags", "read", "pos"])
print("same multiset", np.array_equal(ge, ee))
print(got[:8])
print(exp[:8])
