"""Sharded unipath compaction (apg_sharded_unipaths, ushard_graph.inc): each
rank holds only its minimizer shard's nodes, links and ranks them into chain
fragments, the fragments' end records are gathered and stitched into the
global graph.  The graph (unipaths, ids, rc partners, unibases,
HyperKmerPath) and each rank's KmerPaths must equal the single-GPU
apg_unipaths on the union of the reads, on inputs chosen for the stitch's
hard cases: a circular genome (a cycle that crosses shards and is cut before
its minimum K-mer, possibly inside a fragment), a genome folded onto its own
reverse complement (palindromic junctions), repeats with branching, noisy
reads (many short unipaths), small K with palindromic K-mers, and the
repeat-rich synthetic genome (apg_synth_repeats).  Ranks share
GPU 0 and talk over the TCP communicator."""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu

GRAPH_KEYS = ["n_nodes", "n_unipaths", "len", "id_base", "rc", "ub_off", "unibases", "n_vertices", "from", "to"]


def case_reads(name):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from unipath_cases import circular_reads, noisy_reads, palindrome_reads, repeat_genome, tiling

    from allpathslg_amd import ReadSet, synth_genome

    if name == "circular":
        return circular_reads(synth_genome(20_000, 31), L=150, step=3), 96
    if name == "circular_k31":
        return circular_reads(synth_genome(4_000, 32), L=120, step=2), 31
    if name == "folded":
        s = synth_genome(3_000, 33)
        circ = np.concatenate([s, (3 - s[::-1]).astype(np.uint8)])
        return circular_reads(circ, L=150, step=3), 96
    if name == "repeats":
        return tiling(repeat_genome(seed=34), L=150, step=2), 96
    if name == "noisy":
        return noisy_reads(G=40_000, n=12_000, L=100, err=0.01, seed=35), 25
    if name == "repeat_genome":  # apg_synth_repeats: collapsed repeats, tandem arrays
        from allpathslg_amd import synth_fragments

        g = synth_genome(300_000, 36, repeats={"tandem_frac": 0.03})
        return synth_fragments(g, 60_000, seed=37), 96
    if name == "palindromes":
        r = palindrome_reads()
        return ReadSet.from_sequences([r.read(i) for i in range(r.n_reads)] * 3), 4
    raise ValueError(name)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, name, q, flush_round=None):
    sys.path.insert(0, ROOT)
    if flush_round is not None:  # KmerPaths: the all-at-once last round from this round on
        os.environ["APG_GRAPH_FLUSH_ROUND"] = str(flush_round)
    try:
        from allpathslg_amd import Context
        from allpathslg_amd.distributed import Comm, sharded_unipaths

        reads, K = case_reads(name)
        n = reads.n_reads
        a, b = n * rank // world, n * (rank + 1) // world
        with Context(device=0) as ctx:
            comm = Comm.tcp(ctx, "127.0.0.1", port, rank, world, timeout_ms=120_000)
            d = ctx.upload(reads.subset(a, b))
            graph, st = sharded_unipaths(ctx, comm, d, K, fetch=True)
            d.free()
            comm.close()
        q.put((rank, (graph, st, a, b), ""))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


def run_world(world, name, flush_round=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=worker, args=(r, world, port, name, q, flush_round)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    res.sort(key=lambda x: x[0])
    for rank, out, err in res:
        assert out is not None, (rank, err)
    return [r[1] for r in res]


CASES = [(w, n, None) for w in (2, 4) for n in ("circular", "circular_k31", "folded", "repeats", "noisy",
                                                 "palindromes", "repeat_genome")]
CASES += [(2, "noisy", 1), (4, "repeat_genome", 2)]  # KmerPaths resolved by the flush round


@pytest.mark.parametrize("world,name,flush_round", CASES)
def test_sharded_graph_equals_single_gpu(gpu_ctx, world, name, flush_round):
    reads, K = case_reads(name)
    mono, mst = gpu_ctx.unipaths(reads, K)
    parts = run_world(world, name, flush_round)
    for rank, (g, st, a, b) in enumerate(parts):
        for k in GRAPH_KEYS:
            x, y = g[k], mono[k]
            assert (np.array_equal(x, y) if isinstance(x, np.ndarray) else x == y), (name, world, rank, k)
        mo = mono["path_off"]
        lo, hi = int(mo[a]), int(mo[b])
        assert np.array_equal(g["path_off"] - g["path_off"][0], mo[a : b + 1] - lo), (name, rank)
        assert np.array_equal(g["path_start"], mono["path_start"][lo:hi]), (name, rank)
        assert np.array_equal(g["path_len"], mono["path_len"][lo:hi]), (name, rank)
        assert st["n_unipaths"] == mst["n_unipaths"] and st["n_nodes"] == mst["n_nodes"]
        assert st["n_links"] == mst["n_links"], (name, rank)
        assert st["n_cycles_cut"] == mst["n_cycles_cut"], (name, rank)
    if name.startswith("circular"):
        assert mst["n_cycles_cut"] >= 1
