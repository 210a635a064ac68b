"""The bench's repeats line's counting stage alone: apg_spectrum_precorrect_dev
on the repeat-rich chr20-size genome (bench seeds), for per-kernel traces.
  rocprofv3 --kernel-trace --stats -- python scripts/diag/rep_fused.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import torch  # noqa: E402,F401

from allpathslg_amd import Context, synth_genome, synth_reads  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
seed = 0xA11BA7
g = synth_genome(64_444_167, seed + 31, repeats=True)
reads = synth_reads(g, 20_000_000, seed=seed + 32, with_quals=True, threads=16)
with Context(device=0, timing=True, verbose=True) as ctx:
    src, d = ctx.upload(reads), ctx.upload(reads)
    for r in range(reps):
        ctx.copy_reads(d, src)
        ctx.reset_timing()
        h, k, p = ctx.spectrum_precorrect(d, K_spec=25, K=24)
        print({n: round(v[0], 2) for n, v in ctx.kernel_times().items() if v[0] > 0.5}, flush=True)
