"""bench.py's host-cores CPU baseline (oracle/baseline.py): the OpenMP
restatement's per-stage and combined rates, threaded and single-threaded, and
the same results whatever the thread count."""
import numpy as np

import oracle
from allpathslg_amd import synth_genome, synth_reads


def test_cpu_baseline_small():
    from oracle.baseline import cpu_baseline

    g = synth_genome(300_000, 5)
    reads = synth_reads(g, 60_000, seed=6)
    solid = oracle.solid_hashes(reads, 24, 3)
    out = cpu_baseline(reads, solid, threads=2, n_spec=40_000, n_pc=20_000, n_pairs=2_000,
                       single=(20_000, 10_000, 500))
    assert out["cores"] == 2 and out["kind"] == "port" and out["value"] > 0
    r = out["stage_reads_per_s"]
    assert set(r) == {"spectrum", "precorrect", "fill", "unipaths"} and min(r.values()) > 0
    assert out["value"] <= min(r.values())
    assert out["single_core"]["cores"] == 1 and out["single_core"]["value"] > 0
    assert out["host"]["logical_cpus"] >= 1


def test_restatement_thread_count_invariant():
    g = synth_genome(200_000, 9)
    reads = synth_reads(g, 30_000, seed=10)
    before = oracle.threads()
    try:
        res = []
        for t in (1, 4):
            oracle.set_threads(t)
            h, c = oracle.kmer_count(reads, 25)
            fixed, st = oracle.precorrect(reads, K=24)
            solid = np.sort(oracle.solid_hashes(fixed, 24, 3))
            filled, status, _, fst = oracle.fill_fragments(fixed, solid, K=24)
            gr = oracle.unipaths(filled, 96)
            res.append((h, c, fixed.packed, fixed.quals, st, status, filled.packed, fst, gr["unibases"],
                        gr["path_start"]))
        for a, b in zip(*res):
            if isinstance(a, np.ndarray):
                assert np.array_equal(a, b)
            else:
                assert a == b
    finally:
        oracle.set_threads(before)
