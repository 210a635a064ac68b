"""GPU parity at small odd K on palindrome-dense genomes,
and ErrorCorrectJump's solid-set reuse against a fresh recount (ADVICE r04
medium + low).

For odd K the (K-1)-mers have even length, so palindromic (K-1)-mers exist.
The extension table stores a palindrome's two orientations in one slot, and a
K-mer around it is recorded as a successor bit or a predecessor bit depending
on which orientation is canonical; every reader must OR both readings
(ext_table.hpp ext_masks_lsb / ext_masks2_lsb).  PreCorrect's decisions
(pc_all_solid2, two-level table, the default link-ahead path) and
ErrorCorrectJump's trim (k_ecj_trim) both go through ext_masks2_lsb."""
import ctypes as C

import numpy as np
import pytest

import oracle
from allpathslg_amd import ReadSet, synth_genome, synth_reads
from allpathslg_amd._lib import lib

pytestmark = pytest.mark.gpu


def palindrome_genome(n: int, K: int, every: int, seed: int) -> np.ndarray:
    """iid genome with a palindromic (K-1)-mer planted every `every` bases."""
    rng = np.random.default_rng(seed)
    g = rng.integers(0, 4, n).astype(np.uint8)
    h = (K - 1) // 2
    for s in range(5, n - K, every):
        half = rng.integers(0, 4, h).astype(np.uint8)
        g[s : s + h] = half
        g[s + h : s + 2 * h] = 3 - half[::-1]
    return g


def assert_same(a: ReadSet, b: ReadSet):
    assert np.array_equal(a.packed[: int(a.byte_off[-1])], b.packed[: int(b.byte_off[-1])])
    assert np.array_equal(a.quals, b.quals)


@pytest.mark.parametrize("K", [11, 13, 21, 25])
def test_precorrect_palindromes_odd_K(gpu_ctx, K):
    g = palindrome_genome(60_000, K, 23, seed=K)
    reads = synth_reads(g, 15_000, seed=K + 1)  # 50x, errors with low Q
    got, st = gpu_ctx.precorrect(reads, K=K)
    exp, est = oracle.precorrect(reads, K=K)
    assert_same(got, exp)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert st[k] == est[k], (k, st[k], est[k])
    assert st["n_corrected"] > 0


@pytest.mark.parametrize("K", [11, 13, 25])
def test_ecj_palindromes_odd_K(gpu_ctx, K):
    g = palindrome_genome(60_000, K, 23, seed=100 + K)
    frags = synth_reads(g, 15_000, seed=K + 2)
    jumps = synth_reads(g, 3_000, seed=K + 3, insert_mean=3000, insert_sd=300)
    got, keep, st = gpu_ctx.error_correct_jump(frags, jumps, K=K, min_keep=30)
    exp, ekeep, est = oracle.error_correct_jump(frags, jumps, K=K, min_keep=30)
    assert np.array_equal(got.packed[: exp.byte_off[-1]], exp.packed[: exp.byte_off[-1]])
    assert np.array_equal(got.quals, exp.quals)
    assert np.array_equal(keep, ekeep)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert st["precorrect"][k] == est[k], k


def _download_solid(ctx) -> np.ndarray:
    L = lib()
    n = C.c_uint64()
    assert L.apg_solid_download(ctx._h, None, C.byref(n)) == 0
    out = np.empty(n.value, dtype=np.uint64)
    assert L.apg_solid_download(ctx._h, out.ctypes.data_as(C.POINTER(C.c_uint64)), C.byref(n)) == 0
    return out


@pytest.mark.parametrize("K", [24, 13])
def test_ecj_reuse_equals_recount(gpu_ctx, K):
    """PreCorrect, then ErrorCorrectJump on the same context twice: once
    reusing the correction pass's solid list (pc_self), once after an
    apg_solid_upload (which must end the reuse: the fragments are recounted).
    Jump reads, keep lengths and counters equal; the recounted solid set equals
    the reused one (a pass leaves its reads' solid set unchanged)."""
    import torch

    g = synth_genome(150_000, 40 + K)
    frags = synth_reads(g, 30_000, seed=41)
    jumps = synth_reads(g, 4_000, seed=42, insert_mean=3000, insert_sd=300)
    ctx = gpu_ctx
    dF = ctx.upload(frags)
    ctx.precorrect(dF, K=K)
    reused = np.sort(_download_solid(ctx))
    runs = []
    for upload in (False, True):
        if upload:  # same hashes, installed by upload: no longer the reads' own count
            assert lib().apg_solid_upload(ctx._h, K, reused.ctypes.data_as(C.POINTER(C.c_uint64)), len(reused)) == 0
        dJ = ctx.upload(jumps)
        keep = torch.empty(jumps.n_reads, dtype=torch.int32, device="cuda")
        st = ctx.error_correct_jump(dF, dJ, K=K, d_keep=keep.data_ptr())
        torch.cuda.synchronize()
        runs.append((ctx.download(dJ, with_quals=True), keep.cpu().numpy().copy(), st,
                     np.sort(_download_solid(ctx))))
        dJ.free()
    (j0, k0, s0, l0), (j1, k1, s1, l1) = runs
    assert_same(j0, j1)
    assert np.array_equal(k0, k1)
    for k in ("n_full", "n_trimmed", "n_dropped", "bases_kept"):
        assert s0[k] == s1[k], k
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert s0["precorrect"][k] == s1["precorrect"][k], k
    assert np.array_equal(l0, reused)
    assert np.array_equal(l1, reused)  # the recount of the corrected fragments
    # and the corrected fragments' fresh count equals the list too
    exp = oracle.precorrect(frags, K=K)[0]
    ctx2_hist, _ = ctx.kmer_spectrum(exp, K)
    assert int(ctx2_hist[3:].sum()) == len(reused)
    dF.free()
