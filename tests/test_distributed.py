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


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, K, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
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
