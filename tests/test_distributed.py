"""Sharded module entry points through the C ABI (include/apg.h
apg_sharded_*), one process per rank, every exchange inside libapg:

  * world 2 and 4: ranks share GPU 0 and talk over the TCP communicator;
    spectrum, PreCorrect (1 and 2 passes), FillFragments and the K=96
    unipath graph + KmerPaths (sharded compaction, and once the replicated
    build) equal the single-GPU entry points on the union of the ranks'
    reads (the compaction's hard cases: tests/test_sharded_graph.py);
  * world 1 over RCCL with the segment to self routed through ncclSend /
    ncclRecv (APG_COMM_SELF_P2P): the same stages, and one alltoallv of
    2^31 + 4 KiB bytes compared byte for byte (the size at which the old
    torch-level exchange once lost data).
"""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

GENOME, PAIRS, SEED = 250_000, 48_000, 0xD157


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def rank_pairs(rank, world):
    return PAIRS * rank // world, PAIRS * (rank + 1) // world


def chain(ctx, comm, reads, n_cycles, gather=False):
    """The sharded chain on this rank's reads; host copies of everything."""
    from allpathslg_amd.distributed import (sharded_fill, sharded_precorrect, sharded_spectrum,
                                            sharded_unipaths)

    d = ctx.upload(reads)
    hist, st = sharded_spectrum(ctx, comm, d, 25)
    pst = sharded_precorrect(ctx, comm, d, K=24, n_cycles=n_cycles)
    fixed = ctx.download(d)
    filled, fst = sharded_fill(ctx, comm, d, K=24, last_solid=True)
    ffrag = ctx.download(filled)
    graph, ust = sharded_unipaths(ctx, comm, filled, 96, fetch=True, gather_nodes=gather)
    d.free()
    filled.free()
    return {"hist": hist, "st": st, "pst": pst, "fixed": fixed, "fst": fst, "filled": ffrag, "graph": graph,
            "ust": ust}


def worker(rank, world, port, n_cycles, gather, q):
    sys.path.insert(0, ROOT)
    try:
        from allpathslg_amd import Context, synth_genome, synth_reads
        from allpathslg_amd.distributed import Comm

        g = synth_genome(GENOME, SEED)
        a, b = rank_pairs(rank, world)
        reads = synth_reads(g, b - a, seed=SEED + 1, first_pair=a)
        with Context(device=0) as ctx:
            comm = Comm.tcp(ctx, "127.0.0.1", port, rank, world, timeout_ms=240_000)
            out = chain(ctx, comm, reads, n_cycles, gather)
            comm.close()
        q.put((rank, out, ""))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


def run_world(world, n_cycles, gather=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=worker, args=(r, world, port, n_cycles, gather, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=300) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    res.sort(key=lambda x: x[0])
    for rank, out, err in res:
        assert out is not None, (rank, err)
    return [r[1] for r in res]


@pytest.fixture(scope="module")
def mono(gpu_ctx):
    """The single-GPU entry points on the union of the ranks' reads."""
    from allpathslg_amd import synth_genome, synth_reads

    g = synth_genome(GENOME, SEED)
    reads = synth_reads(g, PAIRS, seed=SEED + 1)
    out = {}
    for n_cycles in (1, 2):
        d = gpu_ctx.upload(reads)
        hist, st = gpu_ctx.kmer_spectrum(d, 25)
        _, pst = gpu_ctx.precorrect(d, K=24, n_cycles=n_cycles)
        fixed = gpu_ctx.download(d)
        filled, _, fst = gpu_ctx.fill_fragments(d, K=24, last_solid=True)
        ffrag = gpu_ctx.download(filled)
        graph, ust = gpu_ctx.unipaths(filled, 96)
        out[n_cycles] = {"reads": reads, "hist": hist, "st": st, "pst": pst, "fixed": fixed, "fst": fst,
                         "filled": ffrag, "graph": graph, "ust": ust}
        d.free()
        filled.free()
    return out


def rows(r, a, b):
    """Reads [a, b) of a host read set as (lengths, packed bytes, quals)."""
    s = r.subset(a, b)
    return s.lengths(), s.packed[: int(s.byte_off[-1])], s.quals


def check_against_mono(parts, m, world):
    graph_keys = ["n_nodes", "n_unipaths", "len", "id_base", "rc", "ub_off", "unibases", "n_vertices", "from", "to"]
    f_off = 0
    for rank, p in enumerate(parts):
        assert np.array_equal(p["hist"], m["hist"])
        for k in ("n_kmers", "n_distinct"):
            assert p["st"][k] == m["st"][k], k
        for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
            assert p["pst"][k] == m["pst"][k], (rank, k)
        a, b = rank_pairs(rank, world)
        got, exp = rows(p["fixed"], 0, p["fixed"].n_reads), rows(m["fixed"], 2 * a, 2 * b)
        for x, y in zip(got, exp):
            assert np.array_equal(x, y), rank
        for k in ("n_pairs", "n_filled", "n_none", "n_ambiguous", "filled_bases"):
            assert p["fst"][k] == m["fst"][k], (rank, k)
        nf = p["filled"].n_reads
        gl, gp, _ = rows(p["filled"], 0, nf)
        el, ep, _ = rows(m["filled"], f_off, f_off + nf)
        assert np.array_equal(gl, el) and np.array_equal(gp, ep), rank
        for k in graph_keys:
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
    assert f_off == m["filled"].n_reads


@pytest.mark.parametrize("world,n_cycles,gather", [(2, 1, False), (4, 1, False), (2, 2, False), (2, 1, True)])
def test_sharded_chain_tcp_equals_single_gpu(mono, world, n_cycles, gather):
    """gather=False: sharded unipath compaction; True: the replicated build
    (APG_UNIPATH_GATHER_NODES)."""
    check_against_mono(run_world(world, n_cycles, gather), mono[n_cycles], world)


def test_sharded_chain_rccl_world1_equals_single_gpu(gpu_ctx, mono):
    from allpathslg_amd.distributed import Comm, unique_id

    comm = Comm.rccl(gpu_ctx, unique_id(), 0, 1, self_p2p=True)
    try:
        out = chain(gpu_ctx, comm, mono[1]["reads"], 1)
        check_against_mono([out], mono[1], 1)
    finally:
        comm.close()


def test_rccl_exchange_above_2gib_bytewise(gpu_ctx):
    import torch

    from allpathslg_amd.distributed import Comm, unique_id

    n = (1 << 31) + 4096
    comm = Comm.rccl(gpu_ctx, unique_id(), 0, 1, self_p2p=True)
    try:
        g = torch.Generator(device="cuda")
        g.manual_seed(5)
        src = torch.randint(-(2**31), 2**31 - 1, (n // 4,), dtype=torch.int32, device="cuda", generator=g)
        dst = torch.zeros_like(src)
        torch.cuda.synchronize()
        comm.alltoallv(src.data_ptr(), [n], dst.data_ptr(), [n])
        assert torch.equal(src, dst)
        # the same through allgatherv
        dst.zero_()
        torch.cuda.synchronize()
        comm.allgatherv(src.data_ptr(), n, dst.data_ptr(), [n])
        assert torch.equal(src, dst)
    finally:
        comm.close()
