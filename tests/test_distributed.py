"""World-size-2 (and 4) gloo tests of the multi-GPU exchange logic on CPU.

The driver (allpathslg_amd.distributed.sharded_spectrum) is run with an
oracle-backed shard backend: same contract as libapg's shard_* stages
(records = k-mer hashes grouped by (owner shard, L1 group)), computed on the
CPU.  The GPU stages themselves are covered by test_gpu_kmer.py's loopback
shard test; this covers splits, count-matrix exchange and the all_reduce.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from allpathslg_amd import shard_bins, synth_genome, synth_reads
from allpathslg_amd.distributed import sharded_spectrum


class OracleShardBackend:
    def __init__(self):
        self.cache = {}

    def alloc(self, n):
        return torch.empty(max(n, 1), dtype=torch.int64)

    def _digits(self, reads, K, P):
        key = (id(reads), K, P)
        if key not in self.cache:
            h = oracle.extract_hashes(reads, K)
            D = int(np.log2(P)) + int(np.log2(shard_bins(K, P)))
            d = (h >> np.uint64(2 * K - D)).astype(np.int64) if D else np.zeros(len(h), np.int64)
            self.cache[key] = (h, d)
        return self.cache[key]

    def shard_count(self, reads, K, P):
        h, d = self._digits(reads, K, P)
        return np.bincount(d, minlength=P * shard_bins(K, P)).astype(np.uint64)

    def shard_scatter(self, reads, K, P, send):
        h, d = self._digits(reads, K, P)
        order = np.argsort(d, kind="stable")
        send[: len(h)] = torch.from_numpy(h[order].view(np.int64))

    def shard_spectrum(self, recv, recv_counts, K, P, hist_len):
        n = int(recv_counts.sum())
        h = recv[:n].numpy().view(np.uint64)
        rank = dist.get_rank()
        pbits = int(np.log2(P))
        if n and pbits:
            assert np.all((h >> np.uint64(2 * K - pbits)) == rank), "record delivered to the wrong shard"
        _, c = np.unique(h, return_counts=True)
        hist = oracle.spectrum_from_counts(c.astype(np.uint32), hist_len)
        return hist, {"n_kmers": n, "n_distinct": len(c), "n_overflow": 0}

    # correction stages: solid set of the received records, pass on own reads
    def shard_solid(self, recv, recv_counts, K, P, min_solid):
        n = int(recv_counts.sum())
        u, c = np.unique(recv[:n].numpy().view(np.uint64), return_counts=True)
        self.solid = u[c >= min_solid]
        return len(self.solid)

    def solid_export(self, out):
        out[: len(self.solid)] = torch.from_numpy(self.solid.view(np.int64))

    def precorrect_solid(self, reads, solid, n_solid, prm):
        fixed, st = oracle.precorrect_solid(reads, solid[:n_solid].numpy().view(np.uint64), prm["K"],
                                            prm["max_q_suspect"])
        reads.packed[:] = fixed.packed  # in place, like the device path
        reads.quals[:] = fixed.quals
        self.cache.clear()  # bases changed
        return st

    def fill(self, reads, solid, n_solid, prm, out=None):
        filled, _, _, st = oracle.fill_fragments(reads, solid[:n_solid].numpy().view(np.uint64), **prm)
        st["n_pairs"] = reads.n_reads // 2
        return filled, st


class OracleWeakBackend(OracleShardBackend):
    """OracleShardBackend + the weak-mask return contract (apg_shard_scatter_pos
    / apg_shard_solid_weak / apg_precorrect_weak): records are single K-mer
    hashes, so a record's mask is one bit.  precorrect_weak checks that the
    bitmap rebuilt from the returned masks is exactly the set of this rank's
    K-mer instances outside the global solid set, then corrects."""

    def _pos(self, reads, K):
        L = reads.lengths().astype(np.int64)
        nk = np.maximum(L - K + 1, 0)
        start = np.repeat(reads.base_off[:-1].astype(np.int64), nk)
        return start + (np.arange(int(nk.sum())) - np.repeat(np.cumsum(nk) - nk, nk))

    def shard_scatter_pos(self, reads, K, P, send, pos):
        h, d = self._digits(reads, K, P)
        order = np.argsort(d, kind="stable")
        send[: len(h)] = torch.from_numpy(h[order].view(np.int64))
        pos[: len(h)] = torch.from_numpy(self._pos(reads, K)[order])

    def alloc_mask(self, n):
        return torch.zeros(max(n, 1), dtype=torch.int32)

    def shard_solid_weak(self, recv, recv_counts, K, P, min_solid, mask):
        n = int(recv_counts.sum())
        h = recv[:n].numpy().view(np.uint64)
        u, inv, c = np.unique(h, return_inverse=True, return_counts=True)
        self.solid = u[c >= min_solid]
        mask[:n] = torch.from_numpy((c[inv] < min_solid).astype(np.int32))
        return len(self.solid)

    def precorrect_weak(self, reads, solid, n_solid, pos, mask, n_records, prm):
        K = prm["K"]
        weak = np.zeros(reads.n_bases + 1, dtype=bool)
        m = mask[:n_records].numpy() != 0
        weak[pos[:n_records].numpy()[m]] = True
        h = oracle.extract_hashes(reads, K)
        sol = np.isin(h, solid[:n_solid].numpy().view(np.uint64))
        exp = np.zeros(reads.n_bases + 1, dtype=bool)
        exp[self._pos(reads, K)[~sol]] = True
        assert np.array_equal(weak, exp), "weak bitmap from the returned masks differs"
        self.weak_checked = getattr(self, "weak_checked", 0) + 1
        return self.precorrect_solid(reads, solid, n_solid, prm)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _small_chunks():
    """Force the chunked collectives through many rounds (odd-sized chunks)."""
    import allpathslg_amd.distributed as D

    D.CHUNK_ELEMS = 4093


def _worker(rank, world, port, K, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _small_chunks()
    try:
        g = synth_genome(100_000, 21)
        reads = synth_reads(g, 4000, seed=22)
        parts = np.array_split(np.arange(reads.n_reads), world)
        mine = reads.subset(int(parts[rank][0]), int(parts[rank][-1]) + 1)
        hist, st = sharded_spectrum(OracleShardBackend(), mine, K, hist_len=1 << 12)
        q.put((rank, hist, st))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_spectrum_gloo(world):
    K = 25
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, K, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = synth_genome(100_000, 21)
    reads = synth_reads(g, 4000, seed=22)
    expect = oracle.kmer_spectrum(reads, K, 1 << 12)
    for rank, hist, st in res:
        assert np.array_equal(hist, expect)
        assert st["n_kmers"] == reads.n_reads * (100 - K + 1)
        assert st["n_distinct"] == int(expect.sum())


class OracleUnipathBackend(OracleShardBackend):
    """CPU stand-in for libapg's ushard_* stages (same record layout:
    4 x int64 = canonical key limbs + (56-bit hash | ext bits))."""

    def _inst(self, reads, K):
        key = ("u", id(reads), K)
        if key not in self.cache:
            self.cache[key] = oracle.instances(reads, K)
        return self.cache[key]

    def _local(self, reads, K):
        """This rank's distinct local nodes (key, ext, hash) in digit order."""
        key = ("n", id(reads), K)
        if key not in self.cache:
            k, e, h = self._inst(reads, K)
            nk, ne = oracle.group_nodes(k.copy(), e.astype(np.uint8))
            # hash of each distinct key = the hash of any of its instances
            uk, first = np.unique(k, axis=0, return_index=True)
            assert np.array_equal(uk, nk)
            hh = h[first]
            d = (hh >> np.uint64(59)).astype(np.int64)
            o = np.argsort(d, kind="stable")
            out = np.zeros((len(ne), 4), dtype=np.uint64)
            out[:, :3] = nk[o]
            out[:, 3] = hh[o] | ne[o].astype(np.uint64)
            self.cache[key] = (out, np.bincount(d, minlength=32).astype(np.uint64), len(h))
        return self.cache[key]

    def ushard_count(self, reads, K, P):
        out, counts, n_inst = self._local(reads, K)
        return counts, n_inst

    def ushard_scatter(self, reads, K, P, send):
        out, _, _ = self._local(reads, K)
        send[: 4 * len(out)] = torch.from_numpy(out.reshape(-1).view(np.int64))

    def ushard_nodes(self, recv, recv_counts, K, P):
        n = int(recv_counts.sum())
        rec = recv[: 4 * n].numpy().view(np.uint64).reshape(n, 4)
        pbits = int(np.log2(P))
        if n and pbits:
            assert np.all((rec[:, 3] >> np.uint64(64 - pbits)) == dist.get_rank())
        self.nodes = oracle.group_nodes(rec[:, :3].copy(), (rec[:, 3] & np.uint64(0xFF)).astype(np.uint8))
        return len(self.nodes[1])

    def ushard_export(self, out):
        k, e = self.nodes
        rec = np.zeros((len(e), 4), dtype=np.uint64)
        rec[:, :3] = k
        rec[:, 3] = e.astype(np.uint64)
        out[: 4 * len(e)] = torch.from_numpy(rec.reshape(-1).view(np.int64))

    def graph_from_nodes(self, nodes, n_nodes, reads, K, fetch):
        rec = nodes[: 4 * n_nodes].numpy().view(np.uint64).reshape(n_nodes, 4)
        g = oracle.graph_from_nodes(rec[:, :3].copy(), (rec[:, 3] & np.uint64(0xFF)).astype(np.uint8), reads, K)
        return g, {"n_unipaths": g["n_unipaths"], "n_nodes": g["n_nodes"]}


class OracleRecBackend(OracleUnipathBackend):
    """OracleUnipathBackend with the minimizer-record contract (urec_*):
    6-word records, counts per (shard, 32 digits).  The oracle's records are
    K-mer instances (key limbs, hash | ext, padding) grouped by the top
    log2(P) + 5 hash bits — any grouping every instance of a K-mer shares
    satisfies the contract."""

    urec_words = 6

    def _recs(self, reads, K, P):
        key = ("r", id(reads), K, P)
        if key not in self.cache:
            k, e, h = self._inst(reads, K)
            D = int(np.log2(P)) + 5
            d = (h >> np.uint64(64 - D)).astype(np.int64)
            o = np.argsort(d, kind="stable")
            out = np.zeros((len(h), 6), dtype=np.uint64)
            out[:, :3] = k[o]
            out[:, 3] = h[o] | e[o].astype(np.uint64)
            self.cache[key] = (out, np.bincount(d, minlength=P * 32).astype(np.uint64), len(h))
        return self.cache[key]

    def urec_count(self, reads, K, P):
        out, counts, n_inst = self._recs(reads, K, P)
        return counts, n_inst

    def urec_scatter(self, reads, K, P, send):
        out, _, _ = self._recs(reads, K, P)
        send[: 6 * len(out)] = torch.from_numpy(out.reshape(-1).view(np.int64))

    def urec_nodes(self, recv, recv_counts, K, P):
        n = int(recv_counts.sum())
        rec = recv[: 6 * n].numpy().view(np.uint64).reshape(n, 6)
        pbits = int(np.log2(P))
        if n and pbits:
            assert np.all((rec[:, 3] >> np.uint64(64 - pbits)) == dist.get_rank())
        self.nodes = oracle.group_nodes(rec[:, :3].copy(), (rec[:, 3] & np.uint64(0xFF)).astype(np.uint8))
        return len(self.nodes[1])

    def urec_export(self, out):
        self.ushard_export(out)


def _uworker(rank, world, port, K, q, rec=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _small_chunks()
    try:
        from allpathslg_amd.distributed import sharded_unipaths
        from tests.unipath_cases import noisy_reads

        reads = noisy_reads(G=15_000, n=2000)
        parts = np.array_split(np.arange(reads.n_reads), world)
        mine = reads.subset(int(parts[rank][0]), int(parts[rank][-1]) + 1)
        g, st = sharded_unipaths(OracleRecBackend() if rec else OracleUnipathBackend(), mine, K, fetch=True)
        q.put((rank, int(parts[rank][0]), int(parts[rank][-1]) + 1, g, st))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,rec", [(2, False), (4, False), (2, True), (4, True)])
def test_sharded_unipaths_gloo(world, rec):
    """Sharded unipath graph == single-process graph, with distinct-local-node
    records or with minimizer-partition records (rec)."""
    from tests.unipath_cases import noisy_reads

    K = 63
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_uworker, args=(r, world, port, K, q, rec)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    reads = noisy_reads(G=15_000, n=2000)
    exp = oracle.unipaths(reads, K)
    for rank, a, b, g, st in res:
        for k in ("len", "id_base", "rc", "ub_off", "unibases", "from", "to"):
            assert np.array_equal(g[k], exp[k]), k
        assert st["n_instances"] == reads.n_reads * (100 - K + 1)
        lo, hi = int(exp["path_off"][a]), int(exp["path_off"][b])
        assert np.array_equal(g["path_start"], exp["path_start"][lo:hi])
        assert np.array_equal(g["path_len"], exp["path_len"][lo:hi])


def _pcworker(rank, world, port, n_cycles, q, weak=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _small_chunks()
    try:
        from allpathslg_amd.distributed import sharded_precorrect

        reads = synth_reads(synth_genome(30_000, 31), 3000, seed=32)
        parts = np.array_split(np.arange(reads.n_reads), world)
        mine = reads.subset(int(parts[rank][0]), int(parts[rank][-1]) + 1)
        be = OracleWeakBackend() if weak else OracleShardBackend()
        st = sharded_precorrect(be, mine, K=24, n_cycles=n_cycles)
        if weak:
            assert getattr(be, "weak_checked", 0) == n_cycles
        q.put((rank, mine.packed[: int(mine.byte_off[-1])].copy(), mine.quals.copy(), st))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_cycles,weak", [(2, 1, False), (4, 2, False), (2, 1, True), (4, 2, True)])
def test_sharded_precorrect_gloo(world, n_cycles, weak):
    """Replicated-solid-set correction == single-process PreCorrect/FindErrors
    (weak: with the weak-mask return, whose bitmap the backend verifies)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pcworker, args=(r, world, port, n_cycles, q, weak)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    reads = synth_reads(synth_genome(30_000, 31), 3000, seed=32)
    exp, est = oracle.precorrect(reads, K=24, n_cycles=n_cycles)
    assert est["n_corrected"] > 0
    assert np.array_equal(np.concatenate([r[1] for r in res]), exp.packed[: int(exp.byte_off[-1])])
    assert np.array_equal(np.concatenate([r[2] for r in res]), exp.quals)
    for _, _, _, st in res:
        for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
            assert st[k] == est[k], k


def _fillworker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    _small_chunks()
    try:
        from allpathslg_amd.distributed import sharded_fill, sharded_precorrect

        reads = synth_reads(synth_genome(30_000, 41), 3000, seed=42)
        pairs = np.array_split(np.arange(reads.n_reads // 2), world)  # ranks hold whole pairs
        mine = reads.subset(2 * int(pairs[rank][0]), 2 * int(pairs[rank][-1]) + 2)
        be = OracleShardBackend()
        _, solid, ns = sharded_precorrect(be, mine, K=24, keep_solid=True)
        filled, st = sharded_fill(be, mine, solid, ns, K=24)
        q.put((rank, filled.base_off.copy(), filled.packed[: int(filled.byte_off[-1])].copy(), st))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_fill_gloo(world):
    """Precorrect with the replicated solid set, then FillFragments per rank
    == single-process PreCorrect + FillFragments, fragments in pair order."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fillworker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    reads = synth_reads(synth_genome(30_000, 41), 3000, seed=42)
    fixed, _ = oracle.precorrect(reads, K=24)
    exp, es, _, est = oracle.fill_fragments(fixed, oracle.solid_hashes(reads, 24, 3), K=24)
    assert est["n_filled"] > 0
    lens = np.concatenate([np.diff(r[1]) for r in res])
    assert np.array_equal(lens, np.diff(exp.base_off))
    assert np.array_equal(np.concatenate([r[2] for r in res]), exp.packed[: int(exp.byte_off[-1])])
    for _, _, _, st in res:
        for k in ("n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip", "filled_bases"):
            assert st[k] == est[k], k
        assert st["n_pairs"] == reads.n_reads // 2
