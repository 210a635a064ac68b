"""Sharded == single-GPU at genome scale (BASELINE configs[3]/[4] are 8-GPU
runs; VERDICT r02 "next" #1): the sharded module chain through the C ABI
(apg_sharded_*) with ranks sharing GPU 0 over the TCP communicator, on a
20-Mb genome at 30x (3 M pairs = 6 M reads), compared byte for byte with the
single-GPU entry points on the union of the reads — spectrum, corrected
reads, FillFragments, unipaths, unibases, HyperKmerPath, every rank's
KmerPaths, UnipathLocs, gap-free hits and consensus (tests/dist_chain.py).

A second case forces the rare paths at that size: error-free 150-bp tiles of
a circular 20-Mb genome (one cycle pair, which crosses every shard and is cut
by the stitch before its minimum K-mer) with every KmerPath resolved by the
all-at-once flush round (APG_GRAPH_FLUSH_ROUND=1).
"""
import multiprocessing as mp
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dist_chain import GRAPH_KEYS, check_against_mono, free_port, mono_chain, run_world  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

CFG = (20_000_000, 3_000_000, 0x5CA1E)


@pytest.fixture(scope="module")
def mono(gpu_ctx):
    out = mono_chain(gpu_ctx, CFG, 1)
    gpu_ctx.trim()
    return out


@pytest.mark.parametrize("world,fused", [(2, False), (4, False), (2, True), (4, True)])
def test_sharded_chain_genome_scale_equals_single_gpu(mono, world, fused):
    """fused: the N > 1 bench step's entry point, apg_sharded_spectrum_precorrect
    (one exchange of K=24 records for the K=25 spectrum and the solid set)."""
    env = {"APG_TEST_FUSED_SHARDED": "1"} if fused else None
    parts = run_world(CFG, world, 1, timeout=800, env=env)
    check_against_mono(parts, mono, world, CFG[1])
    # the workload is what it claims: 6 M reads, most pairs filled, a real graph
    assert mono["st"]["n_kmers"] == 2 * CFG[1] * 76
    assert mono["fst"]["n_filled"] > CFG[1] // 2
    assert mono["graph"]["n_unipaths"] > 1000 and int(mono["graph"]["len"].max()) > 10_000


CIRC_G, CIRC_L, CIRC_STEP, CIRC_SEED = 20_000_000, 150, 10, 0xC1C


def circular_tiles():
    from allpathslg_amd import ReadSet, synth_genome

    g = synth_genome(CIRC_G, CIRC_SEED)
    gg = np.concatenate([g, g[:CIRC_L]])
    win = np.lib.stride_tricks.sliding_window_view(gg, CIRC_L)[: CIRC_G : CIRC_STEP]
    return ReadSet.from_matrix(win)


def circ_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    os.environ["APG_GRAPH_FLUSH_ROUND"] = "1"  # every KmerPath through the flush round
    try:
        from allpathslg_amd import Context
        from allpathslg_amd.distributed import Comm, sharded_unipaths

        reads = circular_tiles()
        n = reads.n_reads
        a, b = n * rank // world, n * (rank + 1) // world
        with Context(device=0) as ctx:
            comm = Comm.tcp(ctx, "127.0.0.1", port, rank, world, timeout_ms=600_000)
            d = ctx.upload(reads.subset(a, b))
            graph, st = sharded_unipaths(ctx, comm, d, 96, fetch=True)
            d.free()
            comm.close()
        q.put((rank, (graph, st, a, b), ""))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_cycle_cut_and_flush_genome_scale(gpu_ctx, world):
    reads = circular_tiles()
    mono, mst = gpu_ctx.unipaths(reads, 96)
    assert mst["n_cycles_cut"] == 1 and mst["n_unipaths"] == 2  # the circle and its reverse complement
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=circ_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=800) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    res.sort(key=lambda x: x[0])
    for rank, out, err in res:
        assert out is not None, (rank, err)
        g, st, a, b = out
        for k in GRAPH_KEYS:
            x, y = g[k], mono[k]
            assert (np.array_equal(x, y) if isinstance(x, np.ndarray) else x == y), (world, rank, k)
        mo = mono["path_off"]
        lo, hi = int(mo[a]), int(mo[b])
        assert np.array_equal(g["path_off"] - g["path_off"][0], mo[a : b + 1] - lo), rank
        assert np.array_equal(g["path_start"], mono["path_start"][lo:hi]), rank
        assert np.array_equal(g["path_len"], mono["path_len"][lo:hi]), rank
        assert st["n_cycles_cut"] == mst["n_cycles_cut"] and st["n_links"] == mst["n_links"], rank
    gpu_ctx.trim()
