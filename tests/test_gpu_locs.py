"""GPU parity: UnipathLocs (apg_unipath_locs, read placement on the unipaths
of the context's last build) from libapg's HIP kernels vs
oracle/locs_oracle.c — exact equality of every location, in both orders,
with and without rc mirrors; the device variant feeds the aligners."""
import numpy as np
import pytest
import torch

import oracle
from allpathslg_amd import ReadSet
from tests.locs_cases import linear_case, repeat_case, sampled_reads
from tests.unipath_cases import noisy_reads

pytestmark = pytest.mark.gpu


def check(ctx, frags, reads, K, rc=True, sorted=True):
    g, _ = ctx.unipaths(frags, K)
    got, st = ctx.unipath_locs(reads, rc=rc, sorted=sorted)
    exp, est = oracle.unipath_locs(g, reads, K, rc=rc, sorted=sorted)
    assert got.shape == exp.shape, (got.shape, exp.shape)
    if not np.array_equal(got, exp):
        bad = np.nonzero((got != exp).any(axis=1))[0][:5]
        raise AssertionError(f"locations differ at {bad.tolist()}: got {got[bad]} expected {exp[bad]}")
    assert st["n_placed"] == est["n_placed"] and st["n_missing"] == est["n_missing"]
    assert st["n_locs"] == len(exp) and st["n_reads"] == reads.n_reads
    return g, got, st


@pytest.mark.parametrize("rc,sorted", [(False, False), (True, False), (False, True), (True, True)])
def test_linear(gpu_ctx, rc, sorted):
    genome, frags = linear_case()
    reads, _, _ = sampled_reads(genome, n=2000)
    _, got, st = check(gpu_ctx, frags, reads, 96, rc, sorted)
    assert st["n_placed"] == reads.n_reads


@pytest.mark.parametrize("K", [31, 63, 96])
def test_repeat_ragged_errors(gpu_ctx, K):
    genome, frags = repeat_case()
    reads, _, _ = sampled_reads(genome, n=3000, err=0.005, seed=5, ragged=True)
    check(gpu_ctx, frags, reads, K)


def test_noisy_graph(gpu_ctx):
    """Graph built from noisy reads (error K-mers make short unipaths); other
    noisy reads placed on it."""
    frags = noisy_reads(G=30_000, n=6000, L=150, err=0.004, seed=2)
    reads = noisy_reads(G=30_000, n=4000, L=100, err=0.01, seed=2)
    check(gpu_ctx, frags, reads, 63)


def test_edge_cases(gpu_ctx):
    genome, frags = linear_case(G=5000)
    reads = ReadSet.from_sequences([genome[:50], genome[100:196], np.zeros(0, np.uint8), genome[4900:5000]])
    check(gpu_ctx, frags, reads, 96)
    check(gpu_ctx, frags, ReadSet.from_sequences([]), 96)


def test_device_locs_feed_aligners(gpu_ctx):
    """Device locations + device unibases -> gap-free (error-free reads: 0
    mismatches) and consensus equal to the oracle's consensus of the oracle's
    locations."""
    K = 96
    genome, frags = repeat_case()
    g, _ = gpu_ctx.unipaths(frags, K)
    reads, _, _ = sampled_reads(genome, n=1500, seed=8, err=0.003)
    dR = gpu_ctx.upload(reads)
    p, n, st = gpu_ctx.unipath_locs(dR, rc=True, sorted=True)
    exp, _ = oracle.unipath_locs(g, reads, K, rc=True, sorted=True)
    assert n == len(exp) and st["n_locs"] == n
    dT = gpu_ctx.unibases_dev()
    assert dT.n_reads == g["n_unipaths"]
    T = ReadSet.from_sequences([g["unibases"][int(g["ub_off"][u]) : int(g["ub_off"][u + 1])]
                                for u in range(g["n_unipaths"])])
    nt = T.n_bases
    dl = gpu_ctx.download(dT)  # device-produced set: shape from the device
    assert np.array_equal(dl.base_off, T.base_off) and np.array_equal(dl.packed[: T.byte_off[-1]],
                                                                        T.packed[: T.byte_off[-1]])
    cb = torch.empty(max(nt, 1), dtype=torch.uint8, device="cuda")
    cq = torch.empty(max(nt, 1), dtype=torch.uint8, device="cuda")
    gpu_ctx.consensus_dev(dR, dT, p, n, cb.data_ptr(), cq.data_ptr())
    torch.cuda.synchronize()
    eb, eq = oracle.consensus(reads, T, exp)
    assert np.array_equal(cb.cpu().numpy()[:nt], eb) and np.array_equal(cq.cpu().numpy()[:nt], eq)
    gf = torch.empty((max(n, 1), 4), dtype=torch.int32, device="cuda")
    gpu_ctx.gapfree_dev(dR, dT, p, n, gf.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(gf.cpu().numpy()[:n].view(np.uint32), oracle.gapfree(reads, T, exp))
    dR.free()
    dT.free()
