"""A/B of the solid-set count kernel (k_sk_bucket_dd variants, APG_DD_VAR):
the bench's fused entry point on the C2 reads, per-kernel HIP-event times.
  APG_DD_VAR=v python scripts/diag/dd_ab.py [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from allpathslg_amd import Context, synth_genome, synth_reads  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
g = synth_genome(64_444_167, 0xA11BA7)
reads = synth_reads(g, 20_000_000, seed=0xA11BA7 + 1, threads=16)
with Context(device=0, timing=True) as ctx:
    src, d = ctx.upload(reads), ctx.upload(reads)
    ctx.copy_reads(d, src)
    h0, k0, p0 = ctx.spectrum_precorrect(d, K_spec=25, K=24)
    ctx.reset_timing()
    for _ in range(reps):
        ctx.copy_reads(d, src)
        h, k, p = ctx.spectrum_precorrect(d, K_spec=25, K=24)
    kt = ctx.kernel_times()
    sig = int(np.frombuffer(ctx.download(d).packed.tobytes()[: 1 << 24], np.uint64).sum() % (1 << 61))
    out = {n: round(v[0] / reps, 3) for n, v in kt.items() if v[0] / reps > 0.5}
    print(f"DDVAR={os.environ.get('APG_DD_VAR', '0')} sk_bucket_solid={out.get('sk_bucket_solid')} ms", out,
          "same" if np.array_equal(h, h0) and p == p0 else "DIFFERS", p["n_solid"], sig, flush=True)
