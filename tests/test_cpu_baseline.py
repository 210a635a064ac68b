"""bench.py's host-cores CPU baseline (oracle/parallel.py): W concurrent
single-threaded oracle processes report per-stage and combined rates."""
import os

import numpy as np

import oracle
from allpathslg_amd import synth_genome, synth_reads

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parallel_baseline_small(tmp_path):
    from oracle.parallel import parallel_baseline

    g = synth_genome(300_000, 5)
    solid = np.sort(oracle.solid_hashes(synth_reads(g, 60_000, seed=6), 24, 3))
    out = parallel_baseline(ROOT, 300_000, 5, solid, 2, n_spec=20_000, n_pc=10_000, n_pairs=500,
                            tmpdir=str(tmp_path))
    assert out["cores"] == 2 and out["kind"] == "port" and out["value"] > 0
    r = out["stage_reads_per_s"]
    assert set(r) == {"spectrum", "precorrect", "fill", "unipaths"} and min(r.values()) > 0
    assert out["value"] <= min(r.values())
    assert not list(tmp_path.iterdir())  # the solid-set file is removed
