"""Host-cores CPU baseline for bench.py (TEST INFRASTRUCTURE: only bench.py's
cpu_baseline leg imports this; never part of the product path).

Times the CPU restatement (oracle/, OpenMP over its independent per-read /
per-pair loops and per-partition sorts) on bounded samples of the bench's own
synthetic reads, stage by stage — K=25 spectrum (extraction + parallel radix
sort + run-length), K=24 PreCorrect (count + correct), FillFragments against
the full-size solid set, K=96 unipaths of the filled fragments — once with
every thread it is given and once on one thread, and names the host CPU.
value = 1 / sum(1 / stage rate), as for the GPU step.

PreCorrect and FillFragments run their baseline forms (ork_precorrect_fast,
orf_fill_fast: rolling K-mer keys and hash-table solid lookups instead of the
checker's per-position re-hash and binary search; outputs identical,
tests/test_cpu_baseline.py), so the baseline is not slowed by the checker's
deliberately simple structures.

Threads: the GPU box allots 16 host CPUs per GPU and sets OMP_NUM_THREADS=16
for that share (the pool's rule: leave it); os.sched_getaffinity() there
reports the whole machine, which other jobs share.  The baseline therefore
runs at OMP_NUM_THREADS threads and reports that count in `cores`, with the
one-thread figure beside it (`single_core`).
"""
from __future__ import annotations

import os
import time

import numpy as np


def host_cpu() -> dict:
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    return {"model": model, "logical_cpus": os.cpu_count(), "affinity_cpus": aff,
            "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def _stages(reads, solid, n_spec, n_pc, n_pairs, K=25, Kc=24, Ku=96):
    import oracle

    spec = reads.subset(0, min(n_spec, reads.n_reads))
    t = time.perf_counter()
    oracle.kmer_count(spec, K)
    ts = time.perf_counter() - t
    pcs = reads.subset(0, min(n_pc, reads.n_reads))
    t = time.perf_counter()
    fixed, _ = oracle.precorrect(pcs, K=Kc, fast=True)
    tp = time.perf_counter() - t
    npairs = min(n_pairs, fixed.n_reads // 2)
    # FillFragments' fixed setup (the hash table over the full-size solid set,
    # built once per call whatever the sample) timed apart: one pair
    t = time.perf_counter()
    oracle.fill_fragments(fixed.subset(0, 2), solid, K=Kc, fast=True)
    tf0 = time.perf_counter() - t
    t = time.perf_counter()
    frags, _, _, _ = oracle.fill_fragments(fixed.subset(0, 2 * npairs), solid, K=Kc, fast=True)
    tf = time.perf_counter() - t
    tfp = max(tf - tf0, 1e-9)  # per-pair work
    t = time.perf_counter()
    oracle.unipaths(frags, Ku)
    tu = time.perf_counter() - t
    rates = {"spectrum": spec.n_reads / ts, "precorrect": pcs.n_reads / tp, "fill": 2 * npairs / tfp,
             "unipaths": 2 * npairs / tu}
    desc = (f"spectrum {spec.n_reads} reads K={K} ({ts:.2f} s); PreCorrect {pcs.n_reads} reads K={Kc}, own "
            f"solid set, rolling keys + hash table ({tp:.2f} s); FillFragments {npairs} restatement-corrected pairs "
            f"against the full-size solid set ({len(solid)} K-mers, hash table): {tf:.2f} s of which {tf0:.2f} s "
            f"table setup (timed on one pair, excluded from the rate); unipaths K={Ku} of the "
            f"{frags.n_reads} filled fragments ({tu:.2f} s)")
    return rates, desc, ts + tp + tf + tu, {"fill_setup_s": tf0}


def _median_runs(n_runs, *args):
    """Each stage's median rate over n_runs runs (median of 3)."""
    runs = [_stages(*args) for _ in range(n_runs)]
    rates = {k: float(np.median([r[0][k] for r in runs])) for k in runs[0][0]}
    return rates, runs[-1][1], sum(r[2] for r in runs), {
        "runs": n_runs, "stage_reads_per_s_runs": {k: [r[0][k] for r in runs] for k in runs[0][0]},
        "fill_setup_s": [r[3]["fill_setup_s"] for r in runs]}


def cpu_baseline(reads, solid: np.ndarray, threads: int = 0, n_spec: int = 4_000_000, n_pc: int = 2_000_000,
                 n_pairs: int = 200_000, single=(500_000, 250_000, 20_000), runs: int = 3) -> dict:
    """The restatement on `threads` OpenMP threads (0: OMP_NUM_THREADS or
    every CPU of the process), then on one thread with the smaller `single`
    samples (spectrum reads, PreCorrect reads, Fill pairs); each stage's rate
    is the median of `runs` runs."""
    import oracle

    solid = np.sort(np.ascontiguousarray(solid, dtype=np.uint64))
    before = oracle.threads()
    if threads:
        oracle.set_threads(threads)
    used = oracle.threads()
    try:
        rates, desc, wall, ex = _median_runs(runs, reads, solid, n_spec, n_pc, n_pairs)
        oracle.set_threads(1)
        r1, d1, w1, ex1 = _median_runs(runs, reads, solid, *single)
    finally:
        oracle.set_threads(before)
    value = 1.0 / sum(1.0 / r for r in rates.values())
    v1 = 1.0 / sum(1.0 / r for r in r1.values())
    return {"value": value, "unit": "reads/s", "cores": used, "kind": "port",
            "stage_reads_per_s": rates, "wall_s": wall, "host": host_cpu(), **ex,
            "sample": (f"oracle/ CPU restatement (OpenMP, {used} threads) on the bench's own synthetic reads, each "
                       f"stage's median rate of {runs} runs: " + desc + "; value = 1/(sum of 1/stage rate)"),
            "single_core": {"value": v1, "unit": "reads/s", "cores": 1, "kind": "port",
                            "stage_reads_per_s": r1, "wall_s": w1, **ex1,
                            "sample": f"one thread, median of {runs} runs: " + d1}}
