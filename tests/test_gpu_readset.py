"""GPU: all_reads assembly (apg_reads_concat_dev) and the K=96 unipath build
over filled fragments + corrected, trimmed jump reads (BASELINE configs[2],
SURVEY §3(1) / §8f #3) against host-built sets and oracle/unipath_oracle.cpp
— exact equality."""
import numpy as np
import pytest
import torch

import oracle
from allpathslg_amd import ReadSet, synth_genome, synth_reads
from tests.test_gpu_unipath import assert_graph_equal

pytestmark = pytest.mark.gpu


def truncated(r: ReadSet, keep) -> ReadSet:
    """Host restatement of one input's part of the concatenation."""
    seqs, quals = [], []
    for i in range(r.n_reads):
        L = int(r.base_off[i + 1] - r.base_off[i])
        k = L if keep is None else min(L, int(keep[i]))
        seqs.append(r.read(i)[:k])
        if r.quals is not None:
            quals.append(r.quals[int(r.base_off[i]) : int(r.base_off[i]) + k])
    return seqs, quals


def host_concat(parts, keeps):
    seqs, quals = [], []
    for r, k in zip(parts, keeps):
        s, q = truncated(r, k)
        seqs += s
        quals += q
    return ReadSet.from_sequences(seqs, quals if len(quals) == len(seqs) else None)


def ragged(n, seed, with_quals=True, max_len=300):
    rng = np.random.default_rng(seed)
    seqs = [rng.integers(0, 4, int(rng.integers(0, max_len))).astype(np.uint8) for _ in range(n)]
    q = [rng.integers(2, 41, len(s)).astype(np.uint8) for s in seqs] if with_quals else None
    return ReadSet.from_sequences(seqs, q)


def test_concat_matches_host(gpu_ctx):
    A, B, Cs = ragged(700, 1), ragged(900, 2), ragged(5, 3)
    rng = np.random.default_rng(4)
    keepB = rng.integers(0, 320, B.n_reads).astype(np.uint32)
    keepB[::7] = 0  # reads trimmed away stay as empty reads
    dA, dB, dC = gpu_ctx.upload(A), gpu_ctx.upload(B), gpu_ctx.upload(Cs)
    dk = torch.from_numpy(keepB.astype(np.int32)).cuda()
    out = gpu_ctx.concat_reads([dA, dB, dC], [None, dk.data_ptr(), None])
    got = gpu_ctx.download(out, with_quals=True)
    exp = host_concat([A, B, Cs], [None, keepB, None])
    assert np.array_equal(got.base_off, exp.base_off)
    assert np.array_equal(got.byte_off, exp.byte_off)
    assert np.array_equal(got.packed[: int(exp.byte_off[-1])], exp.packed[: int(exp.byte_off[-1])])
    assert np.array_equal(got.quals[: exp.n_bases], exp.quals)
    # reuse of the output object with a different shape
    out = gpu_ctx.concat_reads([dB], [dk.data_ptr()], out=out)
    got = gpu_ctx.download(out, with_quals=True)
    exp = host_concat([B], [keepB])
    assert np.array_equal(got.base_off, exp.base_off)
    assert np.array_equal(got.packed[: int(exp.byte_off[-1])], exp.packed[: int(exp.byte_off[-1])])
    # an input without qualities: the output has none
    noq = ragged(50, 5, with_quals=False)
    dn = gpu_ctx.upload(noq)
    out2 = gpu_ctx.concat_reads([dA, dn])
    got = gpu_ctx.download(out2)
    exp = host_concat([A, noq], [None, None])
    assert np.array_equal(got.packed[: int(exp.byte_off[-1])], exp.packed[: int(exp.byte_off[-1])])
    for d in (dA, dB, dC, dn, out, out2):
        d.free()


def test_concat_empty_and_errors(gpu_ctx):
    from allpathslg_amd import ApgError

    out = gpu_ctx.concat_reads([])
    assert out.n_reads == 0
    dA = gpu_ctx.upload(ragged(10, 6))
    with pytest.raises(ApgError):  # the output must be a concat result
        gpu_ctx.concat_reads([dA], out=dA)
    out.free()
    dA.free()


def test_all_reads_unipaths_match_oracle(gpu_ctx):
    """Frag library -> PreCorrect -> FillFragments (device) ++ jump library ->
    ErrorCorrectJump (device, keep lengths) -> concat -> K=96 unipaths +
    HKP + KmerPaths of every read == the oracle graph of the host-built
    all_reads set."""
    g = synth_genome(120_000, 61)
    frags = synth_reads(g, 30_000, seed=62)
    jumps = synth_reads(g, 8_000, seed=63, insert_mean=3000, insert_sd=300)
    dF, dJ = gpu_ctx.upload(frags), gpu_ctx.upload(jumps)
    gpu_ctx.precorrect(dF, K=24)
    filled, _, fst = gpu_ctx.fill_fragments(dF, K=24, last_solid=True)
    keep = torch.empty(jumps.n_reads, dtype=torch.int32, device="cuda")
    gpu_ctx.error_correct_jump(dF, dJ, d_keep=keep.data_ptr())
    allr = gpu_ctx.concat_reads([filled, dJ], [None, keep.data_ptr()])
    got, st = gpu_ctx.unipaths(allr, 96)
    host = gpu_ctx.download(allr)
    # the host-built all_reads equals the concatenation of the parts
    exp_set = host_concat([gpu_ctx.download(filled), gpu_ctx.download(dJ)],
                          [None, keep.cpu().numpy().astype(np.uint32)])
    assert np.array_equal(host.base_off, exp_set.base_off)
    assert np.array_equal(host.packed[: int(exp_set.byte_off[-1])], exp_set.packed[: int(exp_set.byte_off[-1])])
    exp = oracle.unipaths(exp_set, 96)
    assert_graph_equal(got, exp)
    assert got["n_unipaths"] > 0 and int(got["path_off"].shape[0]) == host.n_reads + 1
    for d in (dF, dJ, filled, allr):
        d.free()
