import os, sys, time
sys.path.insert(0, os.getcwd())
from allpathslg_amd import Context, synth_genome, synth_reads
g = synth_genome(64_444_167, 1)
rs = synth_reads(g, 20_000_000, seed=2)
head = "/dev/shm/apg_lt"
rs.write_fastb(head + ".fastb"); rs.write_qualb(head + ".qualb")
try:
    with Context(device=0, verbose=True) as ctx:
        for th in (0, 4, 2, 0):
            t = time.perf_counter()
            d = ctx.load_reads(head + ".fastb", head + ".qualb", threads=th)
            print(th, f"{(time.perf_counter() - t) * 1e3:.1f} ms", flush=True)
            d.free()
finally:
    for e in (".fastb", ".qualb"): os.unlink(head + e)
