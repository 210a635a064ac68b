"""Multi-process CPU baseline for bench.py (TEST INFRASTRUCTURE: only bench.py's
cpu_baseline leg imports this; never part of the product path).

The CPU restatement in oracle/ is single-threaded.  This runs W copies of the
bench's per-stage samples — spectrum, PreCorrect, FillFragments against the
full-size solid set, K=96 unipaths of the filled fragments — on disjoint
slices of the same synthetic read stream in W spawned processes at once, and
reports the aggregate rate: the host's throughput with W cores busy on this
restatement, not a parallel implementation of it.
"""
from __future__ import annotations

import os
import time
from concurrent.futures import ProcessPoolExecutor
from multiprocessing import get_context

import numpy as np


def _worker(args):
    (root, genome_len, seed, first_pair, n_spec, n_pc, n_pairs, K, Kc, Ku, solid_path) = args
    import sys

    if root not in sys.path:
        sys.path.insert(0, root)
    import oracle
    from allpathslg_amd.reads import synth_genome, synth_reads  # host-only simulator (no device calls)

    g = synth_genome(genome_len, seed)
    reads = synth_reads(g, n_spec // 2, seed=seed + 1, first_pair=first_pair, threads=1)
    oracle.lib()
    t = time.perf_counter()
    oracle.kmer_spectrum(reads, K)
    ts = time.perf_counter() - t
    pcs = reads.subset(0, n_pc)
    t = time.perf_counter()
    fixed, _ = oracle.precorrect(pcs, K=Kc)
    tp = time.perf_counter() - t
    solid = np.load(solid_path, mmap_mode="r")
    pairs = fixed.subset(0, 2 * n_pairs)
    t = time.perf_counter()
    frags, _, _, _ = oracle.fill_fragments(pairs, np.ascontiguousarray(solid), K=Kc)
    tf = time.perf_counter() - t
    t = time.perf_counter()
    oracle.unipaths(frags, Ku)
    tu = time.perf_counter() - t
    return n_spec / ts, n_pc / tp, 2 * n_pairs / tf, 2 * n_pairs / tu


def parallel_baseline(root: str, genome_len: int, seed: int, solid: np.ndarray, workers: int, K: int = 25,
                      Kc: int = 24, Ku: int = 96, n_spec: int = 1_000_000, n_pc: int = 500_000,
                      n_pairs: int = 10_000, tmpdir: str = "/tmp") -> dict:
    """Aggregate reads/s of `workers` concurrent single-threaded oracle
    processes; per stage the sum of the workers' rates, combined like the
    single-core baseline as 1 / sum(1 / stage rate)."""
    solid_path = os.path.join(tmpdir, f"apg_solid_{os.getpid()}.npy")
    np.save(solid_path, np.ascontiguousarray(solid, dtype=np.uint64))
    try:
        jobs = [(root, genome_len, seed, 10_000_000 * (w + 1), n_spec, n_pc, n_pairs, K, Kc, Ku, solid_path)
                for w in range(workers)]
        t = time.perf_counter()
        with ProcessPoolExecutor(max_workers=workers, mp_context=get_context("spawn")) as ex:
            res = list(ex.map(_worker, jobs))
        wall = time.perf_counter() - t
    finally:
        os.unlink(solid_path)
    agg = np.array(res).sum(axis=0)
    value = 1.0 / float((1.0 / agg).sum())
    names = ("spectrum", "precorrect", "fill", "unipaths")
    return {"value": value, "unit": "reads/s", "cores": workers, "kind": "port",
            "stage_reads_per_s": dict(zip(names, agg.tolist())), "wall_s": wall,
            "sample": (f"{workers} concurrent single-threaded oracle/ processes, each on its own slice of the "
                       f"same synthetic read stream: spectrum {n_spec} reads K={K}, PreCorrect {n_pc} reads "
                       f"K={Kc}, FillFragments {n_pairs} oracle-corrected pairs against the full-size solid set, "
                       f"unipaths K={Ku} of the filled fragments; aggregate = sum of the workers' rates per stage, "
                       f"value = 1/(sum of 1/stage rate)")}
