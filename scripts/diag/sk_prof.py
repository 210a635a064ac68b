"""Per-phase clock64 sums of k_sk_bucket_dd (APG_SK_PROF=1) on the bench's
C2 reads: K=25 spectrum and the K=24 solid set + weak bitmap of PreCorrect.
  APG_SK_PROF=1 python scripts/diag/sk_prof.py [n_reads]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from allpathslg_amd import Context, synth_genome, synth_reads  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 40_000_000
# APG_SK_DEDUP=all counts the spectrum through k_sk_bucket_dd too
g = synth_genome(64_444_167, 1)
reads = synth_reads(g, n // 2, seed=2)
with Context(device=0) as ctx:
    d = ctx.upload(reads)
    for rep in range(3):
        t = time.time()
        h, st = ctx.kmer_spectrum(d, 25)
        print("spectrum", st, f"{(time.time() - t) * 1e3:.1f} ms", flush=True)
    for rep in range(2):
        t = time.time()
        out, st = ctx.precorrect(d, K=24)
        print("precorrect", st, f"{(time.time() - t) * 1e3:.1f} ms", flush=True)
