"""GPU parity: gap-free aligner, banded Smith-Waterman (cost, ends,
counts, blocks) and column consensus through libapg vs
oracle/align_oracle.c — exact equality (integer costs: tolerance 0)."""
import numpy as np
import pytest

import oracle
from allpathslg_amd import ReadSet
from tests.align_cases import sw_case

pytestmark = pytest.mark.gpu


def test_gapfree_parity(gpu_ctx):
    S, T, pairs = sw_case(n_targets=30, n_pairs=3000, seed=21)
    rng = np.random.default_rng(22)
    pairs = pairs.copy()
    pairs[::7, 2] += rng.integers(-300, 300, size=len(pairs[::7]))  # partial / empty overlaps
    got = gpu_ctx.gapfree(S, T, pairs)
    exp = oracle.gapfree(S, T, pairs)
    assert np.array_equal(got, exp)
    noq = ReadSet(S.base_off, S.byte_off, S.packed, None)
    assert np.array_equal(gpu_ctx.gapfree(noq, T, pairs), oracle.gapfree(noq, T, pairs))


@pytest.mark.parametrize("w", [0, 1, 5, 7, 8, 11, 12, 15, 16, 31, 32, 63, 64, 100, 127])
def test_banded_sw_parity(gpu_ctx, w):
    S, T, pairs = sw_case(n_targets=12, n_pairs=500, seed=30 + w)
    got, gb = gpu_ctx.banded_sw(S, T, pairs, band_w=w, max_blocks=16)
    exp, eb = oracle.banded_sw(S, T, pairs, band_w=w, max_blocks=16)
    bad = np.nonzero(np.any(got != exp, axis=1))[0]
    assert len(bad) == 0, (bad[:5].tolist(), got[bad[:3]].tolist(), exp[bad[:3]].tolist())
    assert np.array_equal(gb, eb)
    got2, _ = gpu_ctx.banded_sw(S, T, pairs, band_w=w)  # without a block buffer
    assert np.array_equal(got2[:, :7], exp[:, :7])


def _interior_first(S, T, pairs, w):
    """Pairs whose whole band stays inside the target first (whole waves of
    them take the LDS kernel's unchecked rows), the rest after."""
    Ls = np.diff(S.base_off.astype(np.int64))[pairs[:, 0]]
    Lt = np.diff(T.base_off.astype(np.int64))[pairs[:, 1]]
    dmin = pairs[:, 2] - w
    inside = (dmin >= 0) & (Ls + dmin + 2 * w <= Lt)
    return np.concatenate([pairs[inside], pairs[~inside]]), int(inside.sum())


def test_banded_sw_parity_every_w(gpu_ctx):
    """Every band width 0..127 (LDS kernel w <= 9, lane kernel w <= 15, wave
    kernel above), pairs ordered so that both the unchecked and the checked
    rows of the LDS kernel run; exact equality with the oracle, and with the
    HBM-direction kernels (APG_SW_NO_LDS) for w <= 9."""
    import os

    for w in range(128):
        S, T, pairs = sw_case(n_targets=6, n_pairs=200 if w < 16 else 64, seed=1000 + w)
        rng = np.random.default_rng(w)
        pairs = pairs.copy()
        pairs[::9, 2] += rng.integers(-2 * w - 3, 2 * w + 4, size=len(pairs[::9]))
        pairs, n_in = _interior_first(S, T, pairs, w)
        got, gb = gpu_ctx.banded_sw(S, T, pairs, band_w=w, max_blocks=12)
        exp, eb = oracle.banded_sw(S, T, pairs, band_w=w, max_blocks=12)
        bad = np.nonzero(np.any(got != exp, axis=1))[0]
        assert len(bad) == 0, (w, n_in, bad[:5].tolist(), got[bad[:3]].tolist(), exp[bad[:3]].tolist())
        assert np.array_equal(gb, eb), w
        if w <= 9:
            os.environ["APG_SW_NO_LDS"] = "1"
            try:
                got2, gb2 = gpu_ctx.banded_sw(S, T, pairs, band_w=w, max_blocks=12)
            finally:
                del os.environ["APG_SW_NO_LDS"]
            assert np.array_equal(got2, got) and np.array_equal(gb2, gb), w


def test_banded_sw_lds_rows_above_64k(gpu_ctx):
    """Queries of 300-550 bases at w = 8 and 9: the LDS kernel's direction
    rows need more than 64 KiB per workgroup (the raised dynamic-LDS limit)."""
    S, T, pairs = sw_case(n_targets=4, n_pairs=300, tlen=2000, slen=(300, 550), seed=46)
    for w in (8, 9):
        p2, _ = _interior_first(S, T, pairs, w)
        got, gb = gpu_ctx.banded_sw(S, T, p2, band_w=w, max_blocks=40)
        exp, eb = oracle.banded_sw(S, T, p2, band_w=w, max_blocks=40)
        assert np.array_equal(got, exp) and np.array_equal(gb, eb), w


@pytest.mark.parametrize("w", [3, 8, 40])
def test_banded_sw_block_overflow(gpu_ctx, w):
    """More blocks than max_blocks: status 2, n_blocks exact, the first
    max_blocks blocks written (LDS kernel for w <= 9, lane-per-pair kernel
    for w <= 15, wave kernel above)."""
    S, T, pairs = sw_case(n_targets=8, n_pairs=400, seed=70 + w)
    got, gb = gpu_ctx.banded_sw(S, T, pairs, band_w=w, max_blocks=2)
    exp, eb = oracle.banded_sw(S, T, pairs, band_w=w, max_blocks=2)
    assert np.array_equal(got, exp) and np.array_equal(gb, eb)
    assert (got[:, 7] == 2).any()


def test_banded_sw_long_queries(gpu_ctx):
    S, T, pairs = sw_case(n_targets=4, n_pairs=120, tlen=3000, slen=(800, 1500), seed=44)
    for w in (20, 9):  # wave kernel, lane-per-pair kernel (1000+ direction rows per lane: too many for LDS)
        got, gb = gpu_ctx.banded_sw(S, T, pairs, band_w=w, max_blocks=40)
        exp, eb = oracle.banded_sw(S, T, pairs, band_w=w, max_blocks=40)
        assert np.array_equal(got, exp) and np.array_equal(gb, eb)


def test_consensus_parity(gpu_ctx):
    S, T, pairs = sw_case(n_targets=10, n_pairs=4000, seed=50)
    plc = pairs.copy()
    got_b, got_q = gpu_ctx.consensus(S, T, plc)
    exp_b, exp_q = oracle.consensus(S, T, plc)
    assert np.array_equal(got_b, exp_b) and np.array_equal(got_q, exp_q)
    e_b, e_q = gpu_ctx.consensus(S, T, plc[:0])
    assert np.array_equal(e_b, np.concatenate([T.read(i) for i in range(T.n_reads)])) and not e_q.any()


def test_aligner_argument_errors(gpu_ctx):
    from allpathslg_amd import ApgError

    S, T, pairs = sw_case(n_targets=2, n_pairs=4, seed=60)
    with pytest.raises(ApgError):
        gpu_ctx.banded_sw(S, T, pairs, band_w=128)
    bad = pairs.copy()
    bad[0, 1] = 99
    with pytest.raises(ApgError):
        gpu_ctx.gapfree(S, T, bad)
