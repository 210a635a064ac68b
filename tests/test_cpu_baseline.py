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


def test_fast_baseline_forms_equal_the_restatement():
    """ork_precorrect_fast (rolling keys, hash-table lookups) and
    orf_fill_fast give the restatement's outputs exactly: the CPU baseline
    times the same algorithm, only faster structures."""
    g = synth_genome(150_000, 21)
    reads = synth_reads(g, 40_000, seed=22)
    for n_cycles in (1, 2):
        a, sa = oracle.precorrect(reads, K=24, n_cycles=n_cycles)
        b, sb = oracle.precorrect(reads, K=24, n_cycles=n_cycles, fast=True)
        assert sa == sb and sa["n_corrected"] > 0
        assert np.array_equal(a.packed, b.packed) and np.array_equal(a.quals, b.quals)
    solid = oracle.solid_hashes(a, 24, 3)
    fa, st_a, la, xa = oracle.fill_fragments(a, solid, K=24)
    fb, st_b, lb, xb = oracle.fill_fragments(a, solid, K=24, fast=True)
    assert xa == xb and xa["n_filled"] > 0
    assert np.array_equal(st_a, st_b) and np.array_equal(la, lb)
    assert np.array_equal(fa.base_off, fb.base_off) and np.array_equal(fa.packed, fb.packed)


def test_fast_precorrect_solid_equals_restatement():
    g = synth_genome(120_000, 23)
    reads = synth_reads(g, 30_000, seed=24)
    solid = oracle.solid_hashes(reads, 24, 3)
    a, sa = oracle.precorrect_solid(reads, solid, K=24)
    b, sb = oracle.precorrect_solid(reads, solid, K=24, fast=True)
    assert sa == sb and sa["n_corrected"] > 0
    assert np.array_equal(a.packed, b.packed) and np.array_equal(a.quals, b.quals)
