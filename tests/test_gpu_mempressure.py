"""Memory pressure (DESIGN.md §7 memory model): a C5-scale
rank cannot hold the counting stages' record buffers, the replicated solid
list and the (K-1)-mer extension table at once, so libapg releases the dead
stage buffers before the correction tables are built (and the correction
tables before the unipath stage) when the device lacks room, and shrinks the
extension table to load <= 0.5 when even that does not fit.  Emulated here
with APG_DEVICE_MEM_LIMIT (the context acts as if the device held only that
much for its workspaces): the chain's results must not change, and the
release path must have run."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

CHAIN = r"""
import json, sys, numpy as np
sys.path.insert(0, {root!r})
import torch
from allpathslg_amd import Context, synth_genome, synth_reads
g = synth_genome(8_000_000, 0x3E3)
reads = synth_reads(g, 1_500_000, seed=0x3E4)
again = None
with Context(device=0, verbose=True) as ctx:
    d = ctx.upload(reads)
    if {fused!r} in ("sharded", "sharded_gather"):  # the driver's per-rank path at world size 1 over RCCL
        from allpathslg_amd.distributed import (Comm, sharded_consensus, sharded_fill, sharded_spectrum_precorrect,
                                                sharded_unipath_locs, sharded_unipaths, unique_id)
        comm = Comm.rccl(ctx, unique_id(), 0, 1)
        hist, st, pst = sharded_spectrum_precorrect(ctx, comm, d, 25, K=24)
        filled, fst = sharded_fill(ctx, comm, d, K=24, last_solid=True)
        graph, ust = sharded_unipaths(ctx, comm, filled, 96, fetch=True, gather_nodes={fused!r} == "sharded_gather")
        ust = {{k: v for k, v in ust.items() if k != "n_shards"}}
        # placement + consensus after the build: under pressure the graph
        # stage's dead temporaries are released first (ws_release_graph_temps)
        pl, nl, lst = sharded_unipath_locs(ctx, comm, d, rc=True, sorted=True)
        locs = torch.empty(max(nl, 1) * 4, dtype=torch.int32, device="cuda")
        if nl:
            ctx.device_copy(locs.data_ptr(), pl, 16 * nl)
        dT = ctx.unibases_dev()
        cb = torch.zeros(max(dT.n_bases, 1), dtype=torch.uint8, device="cuda")
        cq = torch.zeros(max(dT.n_bases, 1), dtype=torch.uint8, device="cuda")
        sharded_consensus(ctx, comm, d, dT, pl, nl, cb.data_ptr(), cq.data_ptr())
        torch.cuda.synchronize()
        again = {{"n_locs": nl, "locs": int(locs[: 4 * nl].cpu().numpy().astype(np.int64).sum()),
                 "cons": int(cb.cpu().numpy().astype(np.uint64).sum()), "consq": int(cq.cpu().numpy().astype(np.uint64).sum())}}
        dT.free()
        comm.close()
    elif {fused!r} == "again":  # the bench loop: a second counting pass after the unipath stage (ADVICE r05)
        d0 = ctx.upload(reads)
        hist, st, pst = ctx.spectrum_precorrect(d, K_spec=25, K=24)
        filled, _, fst = ctx.fill_fragments(d, K=24, last_solid=True)
        graph, ust = ctx.unipaths(filled, 96)
        ctx.copy_reads(d, d0)
        h2, st2, pst2 = ctx.spectrum_precorrect(d, K_spec=25, K=24)
        f2 = ctx.download(d)
        filled2, _, fst2 = ctx.fill_fragments(d, K=24, last_solid=True, out=filled)
        again = {{"hsum": int(h2.astype(np.uint64).sum()), "pst": {{k: pst2[k] for k in ("n_suspect", "n_corrected", "n_solid")}},
                 "fixed": int(np.frombuffer(f2.packed.tobytes(), np.uint64).sum() % (1 << 61)),
                 "filled": fst2["n_filled"], "filled_bases": fst2["filled_bases"]}}
        ctx.copy_reads(d, d0)
        ctx.spectrum_precorrect(d, K_spec=25, K=24)  # leaves d as the first pass did
    else:
      if {fused!r}:  # the bench's entry point: K+1 pass on the side stream (joined before any release)
        hist, st, pst = ctx.spectrum_precorrect(d, K_spec=25, K=24)
      else:
        hist, st = ctx.kmer_spectrum(d, 25)
        _, pst = ctx.precorrect(d, K=24)
      filled, _, fst = ctx.fill_fragments(d, K=24, last_solid=True)
      graph, ust = ctx.unipaths(filled, 96)
    fixed = ctx.download(d)
    fst = {{k: fst[k] for k in ("n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip", "filled_bases")}}
    ust = {{k: ust[k] for k in ("n_nodes", "n_unipaths", "n_vertices", "n_instances", "max_len")}}
    out = {{"hist": hist.tolist()[:200], "hsum": int(hist.astype(np.uint64).sum()), "n_kmers": st["n_kmers"],
           "pst": {{k: pst[k] for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable")}}, "fst": fst, "ust": ust,
           "fixed": int(np.frombuffer(fixed.packed.tobytes(), np.uint64).sum() % (1 << 61)),
           "ub": int(graph["unibases"].astype(np.uint64).sum()), "nu": int(graph["n_unipaths"]),
           "paths": int(graph["path_start"].astype(np.uint64).sum() % (1 << 61)), "again": again}}
print("RESULT " + json.dumps(out))
"""


def run(limit, fused=False, hard=False):
    env = dict(os.environ)
    if limit:
        env["APG_DEVICE_MEM_LIMIT"] = str(limit)
        if hard:
            env["APG_DEVICE_MEM_HARD"] = "1"
    r = subprocess.run([sys.executable, "-c", CHAIN.format(root=ROOT, fused=fused)], capture_output=True, text=True,
                       env=env,
                       timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1]
    return line, r.stderr


@pytest.mark.parametrize("fused", [False, True, "sharded", "sharded_gather"])
def test_release_under_memory_pressure_keeps_results(fused):
    """fused: apg_spectrum_precorrect_dev (the bench's entry point), whose
    K+1 pass on the side stream reads the record buffers the release frees —
    the side stream must be joined first.  "sharded": the driver's per-rank
    path at world size 1 over RCCL, whose replicated solid list is the rank's
    own (the C5-rank rehearsal faulted when the release freed it under the
    extension-table build).  Every form gives the same results."""
    free_run, log0 = run(0, fused)
    assert "dead stage buffers released" not in log0
    # the workspaces this chain reaches without pressure (verbose log)
    peak = max(float(x.split("all workspaces ")[1].split(" GB")[0]) for x in log0.splitlines()
               if "all workspaces" in x)
    tight_run, log1 = run(int(peak * 0.55e9), fused)
    assert "dead stage buffers released" in log1
    if fused in ("sharded", "sharded_gather"):
        assert "dead graph-stage workspaces released" in log1
    assert tight_run == free_run
    if fused in ("sharded", "sharded_gather"):  # the placement outputs are the sharded runs' own
        strip = lambda r: json.dumps(dict(json.loads(r[7:]), again=None))  # noqa: E731
        assert strip(run(0, False)[0]) == strip(free_run)
    elif fused:
        assert run(0, False)[0] == free_run


def _final_sizes(log):
    """Each workspace's last size and the last total (GB) from a verbose log."""
    sizes, total = {}, 0.0
    for x in log.splitlines():
        if "all workspaces" not in x or "] workspace " not in x:
            continue
        name, rest = x.split("] workspace ")[1].split(" -> ")
        sizes[name] = float(rest.split(" GB")[0])
        total = float(x.split("all workspaces ")[1].split(" GB")[0])
    return sizes, total


def test_second_count_after_unipaths_under_a_hard_limit():
    """the unipath stage marks the correction tables dead; a
    counting pass after it (the bench loop's next step) writes its solid list
    into one of them, so a failed allocation inside that count may release the
    previous pass's tables but never the list it has written.
    APG_DEVICE_MEM_HARD makes allocations past the emulated device fail as
    real ones do; the limit sits half the correction tables below the free
    run's final total, so the unipath stage's last allocations fail and
    release them, and the second pass allocates beside the unipath stage's
    workspaces.  Every result equals the unconstrained run's, and the second
    pass's equal the first's."""
    import json

    free_run, log0 = run(0, "again")
    free = json.loads(free_run[7:])
    assert free["again"]["hsum"] == free["hsum"] and free["again"]["pst"]["n_corrected"] == free["pst"]["n_corrected"]
    sizes, total = _final_sizes(log0)
    corr = sum(sizes.get(k, 0.0) for k in ("pc_ext", "fill_ext", "ecj_ext", "fill_solid", "x_solid", "pc_solid"))
    assert corr > 0
    limit = int((total - corr / 2) * 1e9)
    tight_run, log1 = run(limit, "again", hard=True)
    print(f"total {total:.2f} GB, correction tables {corr:.2f} GB, limit {limit / 1e9:.2f} GB")
    print([x for x in log1.splitlines() if "released" in x])
    assert "after a failed allocation" in log1
    assert tight_run == free_run
