"""GPU parity: the unipath graph (nodes, unipaths in emitted order, ids,
rc partners, unibases, HyperKmerPath vertices/edges, read KmerPaths) from
libapg's HIP kernels vs oracle/unipath_oracle.cpp — exact equality."""
import numpy as np
import pytest

import oracle
from allpathslg_amd import synth_genome, synth_reads
from tests.unipath_cases import circular_reads, noisy_reads, palindrome_reads, repeat_genome, tiling

pytestmark = pytest.mark.gpu

KEYS = ["n_nodes", "n_unipaths", "len", "id_base", "rc", "ub_off", "unibases", "n_vertices", "from", "to",
        "path_off", "path_start", "path_len"]


def assert_graph_equal(got, exp):
    for k in KEYS:
        a, b = got[k], exp[k]
        if isinstance(a, np.ndarray):
            assert a.shape == b.shape, (k, a.shape, b.shape)
            if not np.array_equal(a, b):
                bad = np.nonzero(a != b)[0][:5]
                raise AssertionError(f"{k} differs at {bad.tolist()}: got {a[bad]} expected {b[bad]}")
        else:
            assert a == b, (k, a, b)


def run(ctx, reads, K):
    got, st = ctx.unipaths(reads, K)
    exp = oracle.unipaths(reads, K)
    assert_graph_equal(got, exp)
    assert st["n_unipaths"] == exp["n_unipaths"] and st["n_nodes"] == exp["n_nodes"]
    return got, st


def test_linear_genome(gpu_ctx):
    g = synth_genome(20_000, 3)
    got, st = run(gpu_ctx, tiling(g), 96)
    assert got["n_unipaths"] == 2 and st["max_len"] == 20_000 - 96 + 1


def test_repeat_genome(gpu_ctx):
    run(gpu_ctx, tiling(repeat_genome(), L=200, step=5), 96)


@pytest.mark.parametrize("K", [31, 63, 96])
def test_circular_genome_cycles(gpu_ctx, K):
    got, st = run(gpu_ctx, circular_reads(synth_genome(3000, 11)), K)
    assert st["n_cycles_cut"] >= 1


def test_palindromes_small_k(gpu_ctx):
    for K in (2, 4, 6):
        run(gpu_ctx, palindrome_reads(), K)


@pytest.mark.parametrize("K", [1, 5, 25, 32, 33, 64, 65, 95, 96])
def test_noisy_reads(gpu_ctx, K):
    run(gpu_ctx, noisy_reads(G=30_000, n=6000), K)


def test_synthetic_library_and_device_path(gpu_ctx):
    g = synth_genome(300_000, 51)
    reads = synth_reads(g, 40_000, seed=52)
    run(gpu_ctx, reads, 96)
    d = gpu_ctx.upload(reads)
    none, st = gpu_ctx.unipaths(d, 96, read_paths=False, fetch=False)
    assert none is None and st["n_unipaths"] > 0
    again, _ = gpu_ctx.unipaths(d, 96)
    assert_graph_equal(again, oracle.unipaths(reads, 96))
    d.free()


def test_reads_longer_than_a_walk_tile(gpu_ctx):
    """Reads past the K=96 walk's LDS tile (6 KiB = 24,576 bases) are walked
    from HBM by one thread of the block (superkmer.hpp sk_walk_global) — with
    the register-column count walk, on a one-column stride of its own — beside
    tiles of ordinary reads walked by every lane."""
    from allpathslg_amd import ReadSet

    g = synth_genome(90_000, 17)
    seqs = [g[0:30_000], g[20_000:55_000]]
    seqs += [g[s : s + 150] for s in range(30_000, 90_000 - 150, 9)]
    seqs.append(g[60_000:90_000])
    run(gpu_ctx, ReadSet.from_sequences(seqs), 96)


def test_empty_and_short(gpu_ctx):
    from allpathslg_amd import ReadSet

    for reads in (ReadSet.from_sequences([]), ReadSet.from_sequences([[0, 1, 2], [], [3] * 50])):
        run(gpu_ctx, reads, 96)


@pytest.mark.parametrize("P", [1, 2, 4])
def test_shard_path_loopback(gpu_ctx, P):
    """Multi-GPU unipath data path on one GPU: P read slices -> ushard_count /
    ushard_scatter -> loopback all_to_all -> ushard_nodes per shard -> gather
    -> unipaths_from_nodes == single-call build (graph and read paths)."""
    import torch

    K = 96
    reads = noisy_reads(G=40_000, n=8000)
    B = 32 // P
    parts = np.array_split(np.arange(reads.n_reads), P)
    subs = [reads.subset(int(ix[0]), int(ix[-1]) + 1) for ix in parts]
    dsubs = [gpu_ctx.upload(s) for s in subs]
    sends, counts = [], []
    for d in dsubs:
        c, _ = gpu_ctx.ushard_count(d, K, P)
        buf = torch.empty(max(4 * int(c.sum()), 1), dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        gpu_ctx.ushard_scatter(d, K, P, buf.data_ptr())
        sends.append(buf)
        counts.append(c.reshape(P, B))
    node_chunks = []
    for s in range(P):
        pieces, rc = [], []
        for p in range(P):
            starts = np.concatenate([[0], np.cumsum(counts[p].reshape(-1))]).astype(np.int64)
            a, b = starts[s * B], starts[(s + 1) * B]
            pieces.append(sends[p][4 * a : 4 * b])
            rc.append(counts[p][s])
        recv = torch.cat(pieces) if sum(x.numel() for x in pieces) else torch.empty(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        n = gpu_ctx.ushard_nodes(recv.data_ptr(), np.concatenate(rc), K, P)
        out = torch.empty(max(4 * n, 1), dtype=torch.int64, device="cuda")
        gpu_ctx.ushard_export(out.data_ptr())
        node_chunks.append(out[: 4 * n])
    nodes = torch.cat(node_chunks)
    torch.cuda.synchronize()
    exp = oracle.unipaths(reads, K)
    lo = 0
    for i, d in enumerate(dsubs):
        g, st = gpu_ctx.unipaths_from_nodes(nodes.data_ptr(), nodes.numel() // 4, d, K, fetch=True)
        for k in ("n_nodes", "n_unipaths", "len", "id_base", "rc", "ub_off", "unibases", "n_vertices", "from", "to"):
            a = g[k]
            assert (np.array_equal(a, exp[k]) if isinstance(a, np.ndarray) else a == exp[k]), k
        a, b = int(parts[i][0]), int(parts[i][-1]) + 1
        assert np.array_equal(g["path_start"], exp["path_start"][int(exp["path_off"][a]) : int(exp["path_off"][b])])
        d.free()


@pytest.mark.parametrize("P", [1, 2, 4, 8])
def test_urec_path_loopback(gpu_ctx, P):
    """Multi-GPU unipath nodes through minimizer partitions on one GPU: P read
    slices -> urec_count / urec_scatter (48-byte records by minimizer shard)
    -> loopback all_to_all -> urec_nodes per shard -> gather ->
    unipaths_from_nodes == single-call build (graph and read paths)."""
    import torch

    K = 96
    reads = noisy_reads(G=40_000, n=8000)
    B = 32
    parts = np.array_split(np.arange(reads.n_reads), P)
    subs = [reads.subset(int(ix[0]), int(ix[-1]) + 1) for ix in parts]
    dsubs = [gpu_ctx.upload(s) for s in subs]
    sends, counts, n_inst = [], [], 0
    for d in dsubs:
        c, ni = gpu_ctx.urec_count(d, K, P)
        n_inst += ni
        buf = torch.empty(max(6 * int(c.sum()), 1), dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        gpu_ctx.urec_scatter(d, K, P, buf.data_ptr())
        sends.append(buf)
        counts.append(c.reshape(P, B))
    assert n_inst == reads.n_reads * (100 - K + 1)
    node_chunks = []
    for s in range(P):
        pieces, rc = [], []
        for p in range(P):
            starts = np.concatenate([[0], np.cumsum(counts[p].reshape(-1))]).astype(np.int64)
            a, b = starts[s * B], starts[(s + 1) * B]
            pieces.append(sends[p][6 * a : 6 * b])
            rc.append(counts[p][s])
        recv = torch.cat(pieces) if sum(x.numel() for x in pieces) else torch.empty(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        n = gpu_ctx.urec_nodes(recv.data_ptr(), np.concatenate(rc), K, P)
        out = torch.empty(max(4 * n, 1), dtype=torch.int64, device="cuda")
        gpu_ctx.urec_export(out.data_ptr())
        node_chunks.append(out[: 4 * n])
    nodes = torch.cat(node_chunks)
    torch.cuda.synchronize()
    exp = oracle.unipaths(reads, K)
    assert nodes.numel() // 4 == exp["n_nodes"]
    for i, d in enumerate(dsubs):
        g, st = gpu_ctx.unipaths_from_nodes(nodes.data_ptr(), nodes.numel() // 4, d, K, fetch=True)
        for k in ("n_nodes", "n_unipaths", "len", "id_base", "rc", "ub_off", "unibases", "n_vertices", "from", "to"):
            a = g[k]
            assert (np.array_equal(a, exp[k]) if isinstance(a, np.ndarray) else a == exp[k]), k
        a, b = int(parts[i][0]), int(parts[i][-1]) + 1
        assert np.array_equal(g["path_start"], exp["path_start"][int(exp["path_off"][a]) : int(exp["path_off"][b])])
        d.free()


@pytest.mark.parametrize("tab", ["512", "512w6"])
def test_node_buckets_small_table(gpu_ctx, monkeypatch, tab):
    """APG_USK_TAB=512: the node buckets' first pass on a 512-slot LDS table,
    the buckets it overflows rerun through the bucket list with the full
    table, the rest through the global table — same graph."""
    monkeypatch.setenv("APG_USK_TAB", tab)
    g = synth_genome(300_000, 51, repeats=True)
    run(gpu_ctx, synth_reads(g, 40_000, seed=52), 96)
    run(gpu_ctx, noisy_reads(G=30_000, n=6000), 96)
    run(gpu_ctx, tiling(repeat_genome(), L=200, step=5), 96)
