"""Where unipaths_with_d2h's time goes (bench file_to_graph leg; VERDICT r02
#9): the bench step's filled fragments through apg_unipaths_dev without the
graph fetch, then with it (timing log of the d2h phase), three times each."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from allpathslg_amd import Context, synth_genome, synth_reads  # noqa: E402

g = synth_genome(64_444_167, 7)
reads = synth_reads(g, 20_000_000, seed=8, threads=16)
with Context(device=0, verbose=True) as ctx:
    d = ctx.upload(reads)
    ctx.kmer_spectrum(d, 25)
    ctx.precorrect(d, K=24)
    filled, _, _ = ctx.fill_fragments(d, K=24, last_solid=True)
    d.free()
    for fetch in (False, True, False, True, True):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        gr, st = ctx.unipaths(filled, 96, read_paths=True, fetch=fetch)
        t1 = time.perf_counter()
        nb = sum(int(v.nbytes) for v in gr.values() if hasattr(v, "nbytes")) if gr else 0
        print(f"fetch={fetch}: {(t1 - t0) * 1e3:.1f} ms, {nb / 1e6:.0f} MB to host", flush=True)
        del gr
