"""Run-to-run determinism of FillFragments (one pass, and APG_FILL_CAP1
settings): statuses and counters of repeated identical calls."""
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
ms = int(os.environ.get("DET_STEPS", "300"))
args = dict(K=24, min_insert=100, max_insert=260, max_steps=ms, status=True)
_, es, _, est = oracle.fill_fragments(fixed, solid, K=24, min_insert=100, max_insert=260, max_steps=ms)
print("oracle", est, flush=True)
with Context(device=0) as ctx:
    for r in range(int(os.environ.get("DET_RUNS", "4"))):
        _, s, st = ctx.fill_fragments(fixed, solid, **args)
        diff = np.nonzero(s != es)[0]
        print("run", r, "vs oracle differ", len(diff), Counter(zip(es[diff].tolist(), s[diff].tolist())).most_common(5),
              "budget", st["n_budget"], "lookups", st["lookups"], flush=True)
