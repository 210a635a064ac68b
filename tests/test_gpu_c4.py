"""BASELINE.json configs[3] (C4, D. melanogaster, 200 M pairs on 8 x MI355X)
at its per-rank size on one GPU: 50 M x 100-bp reads (25 M pairs, 5.0 G
bases) of a 143,726,002-bp genome — what each of the driver's 8 ranks holds
(VERDICT r04 #1).

Two paths over the same reads:
  * the single-GPU entry points (the bench's apg_spectrum_precorrect_dev,
    FillFragments, K=96 unipaths): 5.0 G bases >= 2^32, so the solid-set count
    takes the wide 34-bit-position SKP records by itself
    (apg_pc_stats.record_form = 2), never forced;
  * the sharded per-rank path of the driver's N > 1 bench at world size 1 over
    RCCL (apg_sharded_spectrum_precorrect -> sharded fill -> sharded unipath
    compaction): the owner count packs received records by receive index
    (record_form = 3).

Checks: the whole K=25 spectrum (3.8 G instances) and the whole K=24 solid
set of all 50 M reads equal the oracle (oracle/, parity unpinned vs
ALLPATHS-LG); PreCorrect of a 2 M-read slice against that solid set equals
the oracle; the bench's size-independent properties; and the sharded path
equals the single-GPU path everywhere (spectrum, solid set, every corrected
base and quality, fill statuses and counters, the whole graph, unibases,
HyperKmerPath and KmerPaths); and the whole single-GPU graph equals the
oracle's graph of the same filled fragments (round 6)."""
import numpy as np
import pytest
import torch

import oracle
from allpathslg_amd import Context, synth_genome, synth_reads
from allpathslg_amd.distributed import Comm, sharded_fill, sharded_spectrum_precorrect, sharded_unipaths, unique_id
from tests.test_gpu_configs import assert_precorrect_equal, solid_sorted
from tests.test_gpu_unipath import assert_graph_equal

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(1200)]

DMEL = 143_726_002
PAIRS = 25_000_000
K96 = 96


def _chain_single(ctx, dsrc, dwork, status):
    ctx.copy_reads(dwork, dsrc)
    h, ks, ps = ctx.spectrum_precorrect(dwork, K_spec=25, K=24)
    out = {"hist": h, "st": ks, "pst": ps, "solid": solid_sorted(ctx), "fixed": ctx.download(dwork)}
    filled, _, fst = ctx.fill_fragments(dwork, K=24, last_solid=True, d_status=status.data_ptr())
    out["fst"], out["status"] = fst, status.cpu().numpy().copy()
    out["graph"], out["ust"] = ctx.unipaths(filled, K96, fetch=True)
    out["mem"] = ctx.mem_stats()
    out["filled"] = ctx.download(filled)
    filled.free()
    return out


def _chain_sharded(ctx, comm, dsrc, dwork, status):
    ctx.copy_reads(dwork, dsrc)
    h, ks, ps = sharded_spectrum_precorrect(ctx, comm, dwork, 25, K=24)
    out = {"hist": h, "st": ks, "pst": ps, "solid": solid_sorted(ctx), "fixed": ctx.download(dwork)}
    filled, fst = sharded_fill(ctx, comm, dwork, K=24, last_solid=True, d_status=status.data_ptr())
    out["fst"], out["status"] = fst, status.cpu().numpy().copy()
    out["graph"], out["ust"] = sharded_unipaths(ctx, comm, filled, K96, fetch=True)
    out["mem"] = ctx.mem_stats()
    filled.free()
    return out


@pytest.fixture(scope="module")
def c4(gpu_ctx):
    gpu_ctx.trim()  # this module's context needs the device to itself
    torch.cuda.empty_cache()
    seed = 0xA11BA7 + 3
    g = synth_genome(DMEL, seed)
    reads = synth_reads(g, PAIRS, seed=seed + 100, threads=16)
    assert reads.n_bases >= 1 << 32
    ctx = Context(device=0)
    dsrc, dwork = ctx.upload(reads), ctx.upload(reads)
    status = torch.zeros(PAIRS, dtype=torch.uint8, device="cuda")
    single = _chain_single(ctx, dsrc, dwork, status)
    comm = Comm.rccl(ctx, unique_id(), 0, 1)
    try:
        shard = _chain_sharded(ctx, comm, dsrc, dwork, status)
    finally:
        comm.close()
    for d in (dsrc, dwork):
        d.free()
    ctx.close()
    del status
    torch.cuda.empty_cache()
    yield {"genome": g, "reads": reads, "single": single, "sharded": shard}


@pytest.fixture(scope="module")
def c4_oracle(c4):
    reads = c4["reads"]
    return {"hist": oracle.kmer_spectrum(reads, 25), "solid": np.sort(oracle.solid_hashes(reads, 24, 3))}


def test_c4_wide_records_engage_by_themselves(c4):
    assert c4["single"]["pst"]["record_form"] == 2  # packed wide SKP, 34-bit positions
    assert c4["sharded"]["pst"]["record_form"] == 3  # the owner's records by receive index


def test_c4_full_spectrum_matches_oracle(c4, c4_oracle):
    """The whole K=25 spectrum of the 50 M reads (3.8 G instances), both paths."""
    for path in ("single", "sharded"):
        r = c4[path]
        assert np.array_equal(r["hist"], c4_oracle["hist"]), path
        m = np.arange(len(r["hist"]), dtype=np.uint64)
        assert int((r["hist"] * m).sum()) == r["st"]["n_kmers"] == c4["reads"].n_reads * 76
        assert int(r["hist"].sum()) == r["st"]["n_distinct"]


def test_c4_full_solid_set_matches_oracle(c4, c4_oracle):
    """The whole K=24 solid set (count >= 3), both paths."""
    assert len(c4_oracle["solid"]) > 130_000_000
    for path in ("single", "sharded"):
        assert np.array_equal(c4[path]["solid"], c4_oracle["solid"]), path
        assert c4[path]["pst"]["n_solid"] == len(c4_oracle["solid"])


def test_c4_precorrect_slice_matches_oracle(c4, c4_oracle):
    """PreCorrect of the first 2 M reads against the whole-table-checked solid
    set (per-read independent: a slice is an exact check)."""
    n = 2_000_000
    exp, est = oracle.precorrect_solid(c4["reads"].subset(0, n), c4_oracle["solid"], K=24, fast=True)
    got = c4["single"]["fixed"].subset(0, n)
    assert np.array_equal(got.packed[: int(got.byte_off[-1])], exp.packed[: int(exp.byte_off[-1])])
    assert np.array_equal(got.quals, exp.quals)
    assert est["n_corrected"] > 0


def test_c4_sharded_equals_single_gpu(c4):
    a, b = c4["single"], c4["sharded"]
    fa, fb = a["fixed"], b["fixed"]
    assert np.array_equal(fa.packed[: int(fa.byte_off[-1])], fb.packed[: int(fb.byte_off[-1])])
    assert np.array_equal(fa.quals, fb.quals)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert a["pst"][k] == b["pst"][k], k
    assert np.array_equal(a["status"], b["status"])
    for k in ("n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip", "filled_bases"):
        assert a["fst"][k] == b["fst"][k], k
    assert_graph_equal(b["graph"], a["graph"])


def test_c4_whole_graph_matches_oracle(c4):
    """The whole single-GPU K=96 graph of the rank's filled fragments (2 G
    instances, 143.6 M nodes) against the oracle's graph of the same
    fragments (C4 had been checked only sharded against
    single); the sharded graph equals it by test_c4_sharded_equals_single_gpu."""
    og = oracle.unipaths(c4["single"]["filled"], K96)
    assert og["n_nodes"] >= DMEL - K96 + 1 - 1000
    assert_graph_equal(c4["single"]["graph"], og)


def test_c4_properties(c4):
    """The bench's size-independent checks at C4's per-rank size (35x)."""
    a = c4["single"]
    f, u = a["fst"], a["ust"]
    assert a["pst"]["n_corrected"] > 0.5 * a["pst"]["n_suspect"]
    assert sum(int(f[k]) for k in ("n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip")) == PAIRS
    assert f["n_filled"] > 0.5 * PAIRS
    assert u["n_instances"] == int(f["filled_bases"]) - (K96 - 1) * int(f["n_filled"])
    assert u["n_nodes"] >= DMEL - K96 + 1 - 1000
    assert u["max_len"] >= 10_000
    g = a["graph"]
    rc = g["rc"].astype(np.int64)
    assert np.array_equal(rc[rc], np.arange(len(rc))) and np.array_equal(g["len"][rc], g["len"])
    for path in ("single", "sharded"):  # what a C4 rank holds, and nothing was released
        m = c4[path]["mem"]
        assert m["releases"] == 0
        print(f"C4 {path}: workspace peak {m['workspace_peak'] / 1e9:.1f} GB, device used {m['device_used'] / 1e9:.1f} GB")
