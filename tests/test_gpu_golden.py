"""GPU stages against the committed golden fixtures (tests/golden/, produced by
the oracle from deterministic synthetic inputs; parity vs real ALLPATHS-LG
unpinned).  Exact equality."""
import os

import numpy as np
import pytest

from allpathslg_amd import ReadSet

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _load():
    z = np.load(os.path.join(GOLDEN, "stages_small.npz"))
    reads = ReadSet.load(os.path.join(GOLDEN, "frag_small.fastb"), os.path.join(GOLDEN, "frag_small.qualb"))
    frags = ReadSet.load(os.path.join(GOLDEN, "frag_small_fill.fastb"))
    S = ReadSet.load(os.path.join(GOLDEN, "aln_queries.fastb"), os.path.join(GOLDEN, "aln_queries.qualb"))
    T = ReadSet.load(os.path.join(GOLDEN, "aln_targets.fastb"))
    return z, reads, frags, S, T


def test_precorrect_golden(gpu_ctx):
    z, reads, _, _, _ = _load()
    for cyc in (1, 2):
        fixed, st = gpu_ctx.precorrect(reads, K=24, n_cycles=cyc)
        assert np.array_equal(fixed.packed[: int(fixed.byte_off[-1])], z[f"pc{cyc}_packed"])
        assert np.array_equal(fixed.quals, z[f"pc{cyc}_quals"])
        keys = ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid")
        assert [st[k] for k in keys] == z[f"pc{cyc}_stats"].tolist()


def test_unipaths_golden(gpu_ctx):
    z, reads, frags, _, _ = _load()
    for K, src in ((31, reads), (96, frags)):
        g, _ = gpu_ctx.unipaths(src, K)
        for key in ("len", "id_base", "rc", "ub_off", "unibases", "from", "to", "path_off", "path_start", "path_len"):
            assert np.array_equal(np.asarray(g[key]), z[f"u{K}_{key}"]), (K, key)


def test_aligners_golden(gpu_ctx):
    z, _, _, S, T = _load()
    pairs = z["aln_pairs"]
    assert np.array_equal(gpu_ctx.gapfree(S, T, pairs), z["aln_gapfree"])
    res, blk = gpu_ctx.banded_sw(S, T, pairs, band_w=8, max_blocks=16)
    assert np.array_equal(res, z["aln_sw"]) and np.array_equal(blk, z["aln_sw_blocks"])
    b, q = gpu_ctx.consensus(S, T, pairs)
    assert np.array_equal(b, z["aln_cons_bases"]) and np.array_equal(q, z["aln_cons_quals"])


def test_locs_and_ecj_golden(gpu_ctx):
    z = np.load(os.path.join(GOLDEN, "locs_ecj_small.npz"))
    _, reads, frags, _, _ = _load()
    gpu_ctx.unipaths(frags, 96)
    locs, st = gpu_ctx.unipath_locs(reads, rc=True, sorted=True)
    assert np.array_equal(locs, z["locs"]) and [st["n_placed"], st["n_missing"]] == z["locs_stats"].tolist()
    jumps = ReadSet.load(os.path.join(GOLDEN, "jump_small.fastb"), os.path.join(GOLDEN, "jump_small.qualb"))
    fixed, keep, est = gpu_ctx.error_correct_jump(reads, jumps, K=24)
    assert np.array_equal(fixed.packed[: int(fixed.byte_off[-1])], z["ecj_packed"])
    assert np.array_equal(fixed.quals, z["ecj_quals"]) and np.array_equal(keep, z["ecj_keep"])
    keys = ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid")
    assert [est["precorrect"][k] for k in keys] == z["ecj_stats"].tolist()
