"""Files -> HBM rate of apg_reads_load_dev at the bench size (40 M reads on
/dev/shm), per thread count, three loads each (the first also allocates the
context's pinned staging).  Diagnostic for DESIGN §8 / VERDICT r02 #9."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: F401,E402

from allpathslg_amd import Context, synth_genome, synth_reads  # noqa: E402

n_pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
hog_gb = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0  # device memory held by torch first (the bench holds ~70 GB)
timing = "timing" in sys.argv[3:]
keep = "keep" in sys.argv[3:]
rewrite = "rewrite" in sys.argv[3:]  # write the files again before every load (a module boundary's state)  # hold every loaded set: each load writes fresh device memory
threads = [int(a[1:]) for a in sys.argv[3:] if a[:1] == "t" and a[1:].isdigit()] or [8, 16]
g = synth_genome(64_444_167, 7)
reads = synth_reads(g, n_pairs, seed=8, threads=16)
head = f"/dev/shm/apg_load_rate_{os.getpid()}"
reads.write_fastb(head + ".fastb")
reads.write_qualb(head + ".qualb")
gb = reads.n_bases * 1.25 / 1e9
hog = torch.empty(int(hog_gb * 1e9), dtype=torch.uint8, device="cuda") if hog_gb else None
if hog is not None:
    hog.fill_(1)
try:
    with Context(device=0, verbose=True, timing=timing) as ctx:
        held = []
        for T in threads:
            for rep in range(3):
                if rewrite:
                    reads.write_fastb(head + ".fastb")
                    reads.write_qualb(head + ".qualb")
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                d = ctx.load_reads(head + ".fastb", head + ".qualb", threads=T)
                t1 = time.perf_counter()
                print(f"threads {T:2d} rep {rep}: {(t1 - t0) * 1e3:7.1f} ms  {gb / (t1 - t0):6.1f} GB/s", flush=True)
                if keep:
                    held.append(d)
                else:
                    d.free()
finally:
    for ext in (".fastb", ".qualb"):
        os.unlink(head + ext)
