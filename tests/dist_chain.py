"""The sharded module chain of one rank and its single-GPU counterpart, shared
by the multi-process GPU tests (test_distributed.py at 250 kb,
test_distributed_scale.py at genome scale).

A rank holds read pairs [PAIRS*r/W, PAIRS*(r+1)/W) of one simulated library
and runs, through the C ABI (include/apg.h apg_sharded_*), with every
exchange inside libapg:

  spectrum (K=25) -> PreCorrect / FindErrors (K=24) -> FillFragments ->
  K=96 unipath graph + KmerPaths (sharded compaction or the replicated build)
  -> UnipathLocs of its corrected reads on that graph -> gap-free alignment
  of the locations against the unibases -> consensus of every rank's
  placements (vote planes summed over the ranks)

The single-GPU chain runs the same entry points on the union of the reads;
check_against_mono() compares every output byte for byte.
"""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

GRAPH_KEYS = ["n_nodes", "n_unipaths", "len", "id_base", "rc", "ub_off", "unibases", "n_vertices", "from", "to"]


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_pairs(pairs, rank, world):
    return pairs * rank // world, pairs * (rank + 1) // world


def _dev_bytes(ctx, ptr, nbytes, dtype):
    """A library-owned device buffer -> host numpy (through a torch buffer)."""
    import torch

    t = torch.empty(max(nbytes, 1), dtype=torch.uint8, device="cuda")
    if nbytes:
        ctx.device_copy(t.data_ptr(), ptr, nbytes)
    torch.cuda.synchronize()
    return t.cpu().numpy()[:nbytes].view(dtype)


def placement_outputs(ctx, d, locs_fn, consensus_fn):
    """Locations (n, 4) int32, their gap-free hits (n, 4) uint32, and the
    consensus (bases, quals) of the context's last graph."""
    import torch

    p, n, lst = locs_fn(d)
    locs = _dev_bytes(ctx, p, 16 * n, np.int32).reshape(n, 4).copy()
    dT = ctx.unibases_dev()
    nt = dT.n_bases
    gf = torch.empty((max(n, 1), 4), dtype=torch.int32, device="cuda")
    ctx.gapfree_dev(d, dT, p, n, gf.data_ptr())
    cb = torch.zeros(max(nt, 1), dtype=torch.uint8, device="cuda")
    cq = torch.zeros(max(nt, 1), dtype=torch.uint8, device="cuda")
    consensus_fn(d, dT, p, n, cb.data_ptr(), cq.data_ptr())
    torch.cuda.synchronize()
    out = {"locs": locs, "hits": gf.cpu().numpy()[:n].view(np.uint32).copy(), "lst": lst,
           "cons_b": cb.cpu().numpy()[:nt].copy(), "cons_q": cq.cpu().numpy()[:nt].copy()}
    dT.free()
    return out


def progress(rank, what):
    """A line per stage (long multi-process runs must show they are alive)."""
    print(f"[rank {rank}] {what}", file=sys.stderr, flush=True)


JUMP_INSERT = (3000, 300)


def jump_reads(g, seed, n_pairs, first_pair=0):
    """A 3-kb jump library (BASELINE configs[2]) of the simulated genome."""
    from allpathslg_amd import synth_reads

    return synth_reads(g, n_pairs, seed=seed + 2, insert_mean=JUMP_INSERT[0], insert_sd=JUMP_INSERT[1],
                       first_pair=first_pair)


def ecj_outputs(ctx, dF, jumps, fn):
    """ErrorCorrectJump of host jump reads against device fragments through
    fn(dF, dJ, d_keep) -> stats: (corrected jumps with quals, keep, stats)."""
    import torch

    dJ = ctx.upload(jumps)
    keep = torch.zeros(max(jumps.n_reads, 1), dtype=torch.int32, device="cuda")
    st = fn(dF, dJ, keep.data_ptr())
    out = (ctx.download(dJ, with_quals=True), keep.cpu().numpy()[: jumps.n_reads].view(np.uint32).copy(), st)
    dJ.free()
    return out


def chain(ctx, comm, reads, n_cycles, gather=False, placement=True, jumps=None):
    """The sharded chain on this rank's reads; host copies of everything.
    jumps: this rank's jump pairs, corrected and trimmed by the sharded
    ErrorCorrectJump after FillFragments (APG_TEST_ECJ_RECOUNT=1: the
    context's solid set dropped first, so the ranks count it again)."""
    from allpathslg_amd.distributed import (sharded_consensus, sharded_error_correct_jump, sharded_fill,
                                            sharded_precorrect, sharded_spectrum, sharded_spectrum_precorrect,
                                            sharded_unipath_locs, sharded_unipaths)

    d = ctx.upload(reads)
    kspec = int(os.environ.get("APG_TEST_KSPEC", "25"))  # != 25: the fused entry point's two-module fallback
    if os.environ.get("APG_TEST_FUSED_SHARDED") == "1":  # one exchange for the K=25 spectrum and the K=24 pass
        hist, st, pst = sharded_spectrum_precorrect(ctx, comm, d, kspec, K=24, n_cycles=n_cycles)
        progress(comm.rank, "spectrum + precorrect")
    else:
        hist, st = sharded_spectrum(ctx, comm, d, kspec)
        progress(comm.rank, "spectrum")
        pst = sharded_precorrect(ctx, comm, d, K=24, n_cycles=n_cycles)
        progress(comm.rank, "precorrect")
    fixed = ctx.download(d)
    filled, fst = sharded_fill(ctx, comm, d, K=24, last_solid=True)
    ffrag = ctx.download(filled)
    progress(comm.rank, "fill")
    ecj = None
    if jumps is not None:
        if os.environ.get("APG_TEST_ECJ_RECOUNT") == "1":
            ctx.trim()
        ecj = ecj_outputs(ctx, d, jumps, lambda dF, dJ, k: sharded_error_correct_jump(ctx, comm, dF, dJ, k))
        progress(comm.rank, "error_correct_jump")
    graph, ust = sharded_unipaths(ctx, comm, filled, 96, fetch=True, gather_nodes=gather)
    progress(comm.rank, "unipaths")
    out = {"hist": hist, "st": st, "pst": pst, "fixed": fixed, "fst": fst, "filled": ffrag, "graph": graph,
           "ust": ust}
    if ecj is not None:
        out["ecj"] = ecj
    if placement:
        out.update(placement_outputs(
            ctx, d, lambda dd: sharded_unipath_locs(ctx, comm, dd, rc=True, sorted=True),
            lambda R, T, p, n, b, q: sharded_consensus(ctx, comm, R, T, p, n, b, q)))
        progress(comm.rank, "placement + consensus")
    d.free()
    filled.free()
    return out


def worker(rank, world, port, cfg, n_cycles, gather, placement, env, q, jump_pairs=0):
    sys.path.insert(0, ROOT)
    os.environ.update(env or {})
    try:
        # one HIP runtime per process: torch's copy first (tests/conftest.py),
        # libapg binds to it; the placement outputs use torch device buffers
        import torch  # noqa: F401

        from allpathslg_amd import Context, synth_genome, synth_reads
        from allpathslg_amd.distributed import Comm

        genome_len, pairs, seed = cfg
        g = synth_genome(genome_len, seed)
        a, b = rank_pairs(pairs, rank, world)
        reads = synth_reads(g, b - a, seed=seed + 1, first_pair=a)
        jumps = None
        if jump_pairs:
            ja, jb = rank_pairs(jump_pairs, rank, world)
            jumps = jump_reads(g, seed, jb - ja, first_pair=ja)
        with Context(device=0) as ctx:
            comm = Comm.tcp(ctx, "127.0.0.1", port, rank, world, timeout_ms=600_000)
            out = chain(ctx, comm, reads, n_cycles, gather, placement, jumps)
            comm.close()
        q.put((rank, out, ""))
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, None, repr(e) + traceback.format_exc()))


def run_world(cfg, world, n_cycles, gather=False, placement=True, timeout=300, env=None, jump_pairs=0):
    """env: extra environment of the rank processes (e.g. APG_CONS_CHUNK, a
    consensus plane smaller than the targets; APG_GRAPH_FLUSH_ROUND).
    jump_pairs: a jump library of that many pairs, split over the ranks."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=worker, args=(r, world, port, cfg, n_cycles, gather, placement, env, q, jump_pairs))
          for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=timeout) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    res.sort(key=lambda x: x[0])
    for rank, out, err in res:
        assert out is not None, (rank, err)
    return [r[1] for r in res]


def mono_chain(gpu_ctx, cfg, n_cycles, placement=True, kspec=25, jump_pairs=0):
    """The single-GPU entry points on the union of the ranks' reads."""
    from allpathslg_amd import synth_genome, synth_reads

    genome_len, pairs, seed = cfg
    g = synth_genome(genome_len, seed)
    reads = synth_reads(g, pairs, seed=seed + 1)
    d = gpu_ctx.upload(reads)
    hist, st = gpu_ctx.kmer_spectrum(d, kspec)
    _, pst = gpu_ctx.precorrect(d, K=24, n_cycles=n_cycles)
    fixed = gpu_ctx.download(d)
    filled, _, fst = gpu_ctx.fill_fragments(d, K=24, last_solid=True)
    ffrag = gpu_ctx.download(filled)
    ecj = None
    if jump_pairs:
        ecj = ecj_outputs(gpu_ctx, d, jump_reads(g, seed, jump_pairs),
                          lambda dF, dJ, k: gpu_ctx.error_correct_jump(dF, dJ, d_keep=k))
    graph, ust = gpu_ctx.unipaths(filled, 96)
    out = {"reads": reads, "hist": hist, "st": st, "pst": pst, "fixed": fixed, "fst": fst, "filled": ffrag,
           "graph": graph, "ust": ust}
    if ecj is not None:
        out["ecj"] = ecj
    if placement:
        out.update(placement_outputs(gpu_ctx, d, lambda dd: gpu_ctx.unipath_locs(dd, rc=True, sorted=True),
                                     gpu_ctx.consensus_dev))
    d.free()
    filled.free()
    return out


def rows(r, a, b):
    """Reads [a, b) of a host read set as (lengths, packed bytes, quals)."""
    s = r.subset(a, b)
    return s.lengths(), s.packed[: int(s.byte_off[-1])], s.quals


def check_ecj_against_mono(parts, m, world, jump_pairs):
    """Each rank's corrected, trimmed jump reads = its slice of the single-GPU
    ErrorCorrectJump of the union; stats summed over ranks equal."""
    mj, mk, ms = m["ecj"]
    for rank, p in enumerate(parts):
        gj, gk, gs = p["ecj"]
        a, b = rank_pairs(jump_pairs, rank, world)
        for x, y in zip(rows(gj, 0, gj.n_reads), rows(mj, 2 * a, 2 * b)):
            assert np.array_equal(x, y), rank
        assert np.array_equal(gk, mk[2 * a : 2 * b]), rank
        for k in ("n_reads", "n_full", "n_trimmed", "n_dropped", "bases_kept"):
            assert gs[k] == ms[k], (rank, k)
        for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
            assert gs["precorrect"][k] == ms["precorrect"][k], (rank, k)
    assert ms["precorrect"]["n_corrected"] > 0 and ms["n_trimmed"] + ms["n_dropped"] > 0


def check_against_mono(parts, m, world, pairs):
    f_off = 0
    all_locs, all_hits = [], []
    for rank, p in enumerate(parts):
        assert np.array_equal(p["hist"], m["hist"])
        for k in ("n_kmers", "n_distinct"):
            assert p["st"][k] == m["st"][k], k
        for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
            assert p["pst"][k] == m["pst"][k], (rank, k)
        a, b = rank_pairs(pairs, rank, world)
        got, exp = rows(p["fixed"], 0, p["fixed"].n_reads), rows(m["fixed"], 2 * a, 2 * b)
        for x, y in zip(got, exp):
            assert np.array_equal(x, y), rank
        for k in ("n_pairs", "n_filled", "n_none", "n_ambiguous", "filled_bases"):
            assert p["fst"][k] == m["fst"][k], (rank, k)
        nf = p["filled"].n_reads
        gl, gp, _ = rows(p["filled"], 0, nf)
        el, ep, _ = rows(m["filled"], f_off, f_off + nf)
        assert np.array_equal(gl, el) and np.array_equal(gp, ep), rank
        for k in GRAPH_KEYS:
            a_, b_ = p["graph"][k], m["graph"][k]
            assert (np.array_equal(a_, b_) if isinstance(a_, np.ndarray) else a_ == b_), (rank, k)
        # this rank's fragments' KmerPaths = its slice of the monolithic ones
        mo, po = m["graph"]["path_off"], p["graph"]["path_off"]
        lo, hi = int(mo[f_off]), int(mo[f_off + nf])
        assert np.array_equal(po - po[0], mo[f_off : f_off + nf + 1] - lo)
        assert np.array_equal(p["graph"]["path_start"], m["graph"]["path_start"][lo:hi])
        assert np.array_equal(p["graph"]["path_len"], m["graph"]["path_len"][lo:hi])
        assert p["ust"]["n_instances"] == m["ust"]["n_instances"]
        f_off += nf
        if "locs" in p:
            for k in ("n_reads", "n_placed", "n_locs", "n_missing"):
                assert p["lst"][k] == m["lst"][k], (rank, k)
            loc = p["locs"].copy()
            loc[:, 0] += 2 * a  # this rank's reads start at read 2a of the union
            all_locs.append(loc)
            all_hits.append(p["hits"])
            assert np.array_equal(p["cons_b"], m["cons_b"]) and np.array_equal(p["cons_q"], m["cons_q"]), rank
    assert f_off == m["filled"].n_reads
    if all_locs:
        loc = np.concatenate(all_locs)
        hit = np.concatenate(all_hits)
        # the union's by-unipath order: stable by (unipath, offset); ranks
        # hold consecutive read ranges, so rank order is read order
        order = np.lexsort((loc[:, 2], loc[:, 1]))
        assert np.array_equal(loc[order], m["locs"])
        assert np.array_equal(hit[order], m["hits"])
        assert len(m["locs"]) > 0 and (m["cons_q"] > 0).any()
