"""FillFragments on the repeat-rich chr20-size genome (the bench's repeats
line) under A/B settings: pass-1-only (max_steps = 96) against the full
budget, free steps per iteration, refill mark.
  [FILL_CASES=base,x0] python scripts/diag/fill_rep.py [n_reads]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
from allpathslg_amd import Context, synth_genome, synth_reads  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 40_000_000
iid = os.environ.get("FILL_GENOME") == "iid"  # the main line's iid genome instead
g = synth_genome(64_444_167, 0xA11BA7 + 31, repeats=None if iid else True)
reads = synth_reads(g, n // 2, seed=0xA11BA7 + 32, with_quals=True, threads=16)
print("reads ready", flush=True)
cases = [("base", 1024, {}), ("pass1", 96, {}), ("x0", 1024, {"APG_FILL_XSTEPS": "0"}),
         ("x64", 1024, {"APG_FILL_XSTEPS": "64"}), ("refill8", 1024, {"APG_FILL_REFILL": "8"}),
         ("refill48", 1024, {"APG_FILL_REFILL": "48"}),
         ("refill24", 1024, {"APG_FILL_REFILL": "24"}), ("refill40", 1024, {"APG_FILL_REFILL": "40"}), ("nocache", 1024, {"APG_FILL_BRANCH_CACHE": "0"}),
         ("x1", 1024, {"APG_FILL_XSTEPS": "1"}), ("x8nc", 1024, {"APG_FILL_XCACHED": "0"}),
         ("x1nc", 1024, {"APG_FILL_XSTEPS": "1", "APG_FILL_XCACHED": "0"}),
         ("p0", 1024, {"APG_FILL_XPCT": "0"}), ("p25", 1024, {"APG_FILL_XPCT": "25"}),
         ("p75", 1024, {"APG_FILL_XPCT": "75"}), ("p90", 1024, {"APG_FILL_XPCT": "90"}),
         ("p50x4", 1024, {"APG_FILL_XSTEPS": "4"}),
         ("c48", 1024, {"APG_FILL_CAP1": "48"}), ("c192", 1024, {"APG_FILL_CAP1": "192"}),
         ("c384", 1024, {"APG_FILL_CAP1": "384"}), ("c1024", 1024, {"APG_FILL_CAP1": "1024"}), ("hash1", 1024, {"APG_EXT_HASH": "1"}), ("nolean", 1024, {"APG_FILL_LEAN": "0"}), ("nofuse", 1024, {"APG_FILL_FUSE_BT": "0"}), ("base2", 1024, {})]
sel = os.environ.get("FILL_CASES")
if sel:
    cases = [c for c in cases if c[0] in sel.split(",")]
with Context(device=0, timing=True) as ctx:
    d = ctx.upload(reads)
    _, pst = ctx.precorrect(d, K=24)
    print("precorrect", pst, flush=True)
    out = None
    for name, ms, env in cases:
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        best = None
        for _ in range(2):
            ctx.reset_timing()
            t = time.time()
            out, _, fst = ctx.fill_fragments(d, K=24, last_solid=True, max_steps=ms, out=out)
            wall = (time.time() - t) * 1e3
            kt = ctx.kernel_times()
            f = kt["fill"][0]
            best = f if best is None else min(best, f)
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        print(f"{name:9s} fill {best:7.2f} ms  wall {wall:7.1f} ms  lookups {fst['lookups']}  budget {fst['n_budget']}"
              f"  amb {fst['n_ambiguous']}  filled {fst['n_filled']}", flush=True)
