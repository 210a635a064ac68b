"""Deferred-walk split vs one pass: per (one-pass status, split status) pair
counts for several APG_FILL_CAP1 values, and the counters of each run."""
import os
import sys
from collections import Counter

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import oracle  # noqa: E402
from allpathslg_amd import Context, synth_genome, synth_reads  # noqa: E402

g = synth_genome(150_000, 5, repeats=True)
reads = synth_reads(g, 15_000, seed=105)
fixed, _ = oracle.precorrect(reads, K=24)
solid = oracle.solid_hashes(reads, 24, 3)
args = dict(K=24, min_insert=100, max_insert=260, max_steps=300, status=True)
with Context(device=0) as ctx:
    ref, rs, rst = ctx.fill_fragments(fixed, solid, **args)
    print("ref", rst, flush=True)
    for c in os.environ.get("SPLIT_CAPS", "0,1,50,299,300").split(","):
        os.environ["APG_FILL_CAP1"] = c
        try:
            got, s, st = ctx.fill_fragments(fixed, solid, **args)
        except Exception as e:  # noqa: BLE001
            print("cap1", c, "error", e, flush=True)
            continue
        diff = np.nonzero(s != rs)[0]
        print("cap1", c, "differ", len(diff), Counter(zip(rs[diff].tolist(), s[diff].tolist())).most_common(6),
              {k: (st[k], rst[k]) for k in st if st[k] != rst[k]}, flush=True)
