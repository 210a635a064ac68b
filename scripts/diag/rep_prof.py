"""Bucket skew and per-phase profile of the K-mer counters on the repeat-rich
chr20-size genome (the bench's repeats line).
  APG_SK_PROF=1 python scripts/diag/rep_prof.py [n_reads] [dedup]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from allpathslg_amd import Context, synth_genome, synth_reads  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 40_000_000
dd = int(sys.argv[2]) if len(sys.argv) > 2 else 0
g = synth_genome(64_444_167, 32, repeats=True)
reads = synth_reads(g, n // 2, seed=33)
with Context(device=0, verbose=True, timing=True, kmer_dedup=dd) as ctx:
    d = ctx.upload(reads)
    for rep in range(2):
        ctx.reset_timing()
        t = time.time()
        h, st = ctx.kmer_spectrum(d, 25)
        print("spectrum", st, f"{(time.time() - t) * 1e3:.1f} ms", flush=True)
        print({k: round(v[0], 2) for k, v in ctx.kernel_times().items() if v[0] > 1}, flush=True)
    ctx.reset_timing()
    t = time.time()
    out, st = ctx.precorrect(d, K=24)
    print("precorrect", st, f"{(time.time() - t) * 1e3:.1f} ms", flush=True)
    print({k: round(v[0], 2) for k, v in ctx.kernel_times().items() if v[0] > 1}, flush=True)
