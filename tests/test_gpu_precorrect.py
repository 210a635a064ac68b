"""GPU parity: PreCorrect / FindErrors through libapg vs the
CPU restatement oracle/precorrect_oracle.c — bit-identical bases, quals and
counters.  Semantics vs real ALLPATHS-LG: unpinned (reference empty)."""
import numpy as np
import pytest

import oracle
from allpathslg_amd import ReadSet, synth_genome, synth_reads

pytestmark = pytest.mark.gpu


def assert_same(a: ReadSet, b: ReadSet):
    assert np.array_equal(a.packed[: int(a.byte_off[-1])], b.packed[: int(b.byte_off[-1])])
    assert np.array_equal(a.quals, b.quals)


@pytest.mark.parametrize("n_cycles", [1, 2])
def test_precorrect_matches_oracle(gpu_ctx, n_cycles):
    g = synth_genome(200_000, 31)
    reads = synth_reads(g, 40_000, seed=32)
    got, st = gpu_ctx.precorrect(reads, K=24, n_cycles=n_cycles)
    exp, est = oracle.precorrect(reads, K=24, n_cycles=n_cycles)
    assert_same(got, exp)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert st[k] == est[k], k
    if n_cycles == 1:  # later cycles re-examine the uncorrectable suspects
        assert st["n_corrected"] > 0.5 * st["n_suspect"]


@pytest.mark.parametrize("glen,pairs", [(3_000, 20_000), (40_000, 60_000)])
def test_precorrect_deep_coverage(gpu_ctx, glen, pairs):
    """Very deep coverage (1300x / 300x): a bucket's K-mer instances exceed
    the per-wave recorded-slot capacity of the weak pass, which then takes
    the probing fallback; a few buckets see counts in the thousands."""
    g = synth_genome(glen, 77)
    reads = synth_reads(g, pairs, seed=78)
    got, st = gpu_ctx.precorrect(reads, K=24)
    exp, est = oracle.precorrect(reads, K=24)
    assert_same(got, exp)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert st[k] == est[k], k
    h, _ = gpu_ctx.kmer_spectrum(reads, 24)
    assert np.array_equal(h, oracle.kmer_spectrum(reads, 24))


def test_precorrect_identical_copies(gpu_ctx):
    """3000 copies of each of a few reads among ordinary ones: buckets of
    more records than the dedup kernel records slots for in its weak pass
    are handed back to the per-instance kernel; the rest dedup to
    multiplicity 3000.  Both must give the oracle's corrections."""
    rng = np.random.default_rng(12)
    g = synth_genome(100_000, 13)
    base = synth_reads(g, 20_000, seed=14)
    B = np.stack([base.read(i) for i in range(base.n_reads)])
    Q = base.quals.reshape(base.n_reads, -1)
    rep = np.concatenate([np.arange(base.n_reads), np.repeat(np.arange(3), 3000)])
    rep = rep[rng.permutation(len(rep))]
    reads = ReadSet.from_matrix(B[rep], Q[rep])
    got, st = gpu_ctx.precorrect(reads, K=24)
    exp, est = oracle.precorrect(reads, K=24)
    assert_same(got, exp)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert st[k] == est[k], k


def test_precorrect_ragged_and_params(gpu_ctx):
    rng = np.random.default_rng(8)
    g = synth_genome(20_000, 9)
    seqs, quals = [], []
    for _ in range(5000):
        L = int(rng.integers(0, 150))
        s = int(rng.integers(0, 20_000 - 150))
        r = g[s : s + L].copy()
        q = rng.integers(2, 41, size=L).astype(np.uint8)
        flip = rng.random(L) < 0.02
        r[flip] = (r[flip] + 1) % 4
        seqs.append(r)
        quals.append(q)
    reads = ReadSet.from_sequences(seqs, quals)
    for K, ms, mq in [(24, 3, 20), (16, 2, 30), (31, 4, 41)]:
        got, st = gpu_ctx.precorrect(reads, K=K, min_solid=ms, max_q_suspect=mq)
        exp, est = oracle.precorrect(reads, K=K, min_solid=ms, max_q=mq)
        assert_same(got, exp)
        assert st == {**st, **est}


def test_precorrect_device_inplace_then_spectrum(gpu_ctx):
    g = synth_genome(100_000, 41)
    reads = synth_reads(g, 30_000, seed=42)
    d = gpu_ctx.upload(reads)
    h0, _ = gpu_ctx.kmer_spectrum(d, 25)
    gpu_ctx.precorrect(d, K=24)
    h1, _ = gpu_ctx.kmer_spectrum(d, 25)
    fixed = gpu_ctx.download(d)
    exp, _ = oracle.precorrect(reads, K=24)
    assert_same(fixed, exp)
    assert np.array_equal(h1, oracle.kmer_spectrum(exp, 25))
    assert h1[1] < h0[1]  # correction removes singleton error k-mers
    d.free()


def test_precorrect_requires_quals(gpu_ctx):
    from allpathslg_amd import ApgError

    reads = ReadSet.from_sequences([[0, 1, 2, 3] * 10])
    with pytest.raises((ApgError, ValueError)):
        gpu_ctx.precorrect(reads)


@pytest.mark.parametrize("P", [1, 2, 4])
def test_sharded_solid_loopback(gpu_ctx, P):
    """Multi-GPU correction data path on one GPU: P read slices -> shard_count /
    shard_scatter at K=24 -> loopback all_to_all -> shard_solid per shard ->
    gathered solid set -> precorrect_solid on every slice == monolithic
    PreCorrect (bases, quals, counters); the union of shard solid sets is the
    oracle's solid set."""
    import torch

    from allpathslg_amd import shard_bins

    K = 24
    reads = synth_reads(synth_genome(150_000, 61), 30_000, seed=62)
    B = shard_bins(K, P)
    parts = np.array_split(np.arange(reads.n_reads), P)
    subs = [reads.subset(int(ix[0]), int(ix[-1]) + 1) for ix in parts]
    dsubs = [gpu_ctx.upload(s) for s in subs]
    sends, counts = [], []
    for d in dsubs:
        c = gpu_ctx.shard_count(d, K, P)
        buf = torch.empty(max(2 * int(c.sum()), 1), dtype=torch.int64, device="cuda")  # 16-byte records
        torch.cuda.synchronize()
        gpu_ctx.shard_scatter(d, K, P, buf.data_ptr())
        sends.append(buf)
        counts.append(c.reshape(P, B))
    solids = []
    for s in range(P):
        pieces, rc = [], []
        for p in range(P):
            starts = np.concatenate([[0], np.cumsum(counts[p].reshape(-1))]).astype(np.int64)
            pieces.append(sends[p][2 * starts[s * B] : 2 * starts[(s + 1) * B]])
            rc.append(counts[p][s])
        recv = torch.cat(pieces) if sum(x.numel() for x in pieces) else torch.empty(1, dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        n = gpu_ctx.shard_solid(recv.data_ptr(), np.concatenate(rc), K, P, 3)
        out = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
        gpu_ctx.solid_export(out.data_ptr())
        solids.append(out[:n])
    solid = torch.cat(solids)
    keys, cnt = oracle.kmer_count(reads, K)
    assert np.array_equal(np.sort(solid.cpu().numpy().view(np.uint64)), keys[cnt >= 3])
    exp, est = oracle.precorrect(reads, K=K)
    tot = {"n_suspect": 0, "n_corrected": 0, "n_ambiguous": 0, "n_uncorrectable": 0}
    fixed = []
    for d in dsubs:
        st = gpu_ctx.precorrect_solid(d, solid.data_ptr(), solid.numel(), K=K)
        assert st["n_solid"] == est["n_solid"]
        for k in tot:
            tot[k] += st[k]
        fixed.append(gpu_ctx.download(d))
        d.free()
    assert tot == {k: est[k] for k in tot}
    assert np.array_equal(np.concatenate([f.packed[: int(f.byte_off[-1])] for f in fixed]),
                          exp.packed[: int(exp.byte_off[-1])])
    assert np.array_equal(np.concatenate([f.quals for f in fixed]), exp.quals)


def test_copy_reads_restores(gpu_ctx):
    reads = synth_reads(synth_genome(50_000, 71), 8000, seed=72)
    src = gpu_ctx.upload(reads)
    work = gpu_ctx.upload(reads)
    exp, _ = oracle.precorrect(reads, K=24)
    for _ in range(2):  # correct, restore, correct again: same result
        gpu_ctx.copy_reads(work, src)
        gpu_ctx.precorrect(work, K=24)
        assert_same(gpu_ctx.download(work), exp)
    assert_same(gpu_ctx.download(src), reads)
    src.free()
    work.free()


def test_precorrect_long_and_boundary_reads(gpu_ctx):
    """Reads around the wave kernel's 1024-base limit (longer ones take the
    thread-per-read kernel) and K from 1 to 32 (1 or 2 lane rounds)."""
    rng = np.random.default_rng(81)
    g = synth_genome(30_000, 82)
    seqs, quals = [], []
    for L in [1023, 1024, 1025, 1500, 64, 65, 128, 2000] * 6 + list(rng.integers(20, 300, size=300)):
        s = int(rng.integers(0, 30_000 - int(L)))
        r = g[s : s + int(L)].copy()
        q = np.full(int(L), 40, np.uint8)
        flip = rng.random(int(L)) < 0.01
        r[flip] = (r[flip] + 1 + rng.integers(0, 3, size=int(flip.sum()))) % 4
        q[flip] = rng.integers(2, 20, size=int(flip.sum()))
        low = rng.random(int(L)) < 0.01
        q[low] = 10
        seqs.append(r)
        quals.append(q)
    reads = ReadSet.from_sequences(seqs, quals)
    for K in (1, 12, 21, 22, 24, 32):
        got, st = gpu_ctx.precorrect(reads, K=K, min_solid=2)
        exp, est = oracle.precorrect(reads, K=K, min_solid=2)
        assert_same(got, exp)
        assert st == {**st, **est}


@pytest.mark.gpu
def test_precorrect_extension_path_short_reads(gpu_ctx):
    """Reads <= 1024 bases take the (K-1)-mer extension-table path for
    2 <= K <= 29 (weak tests by lookups below K = 9, by the counted weak
    bitmap above); reads as short as K and shorter than 2K-1 exercise the
    clipped covering ranges (no K-mer on one or both sides of a suspect)."""
    rng = np.random.default_rng(91)
    g = synth_genome(20_000, 92)
    seqs, quals = [], []
    for L in list(rng.integers(2, 120, size=400)) + [1024, 1000, 512] * 4:
        s = int(rng.integers(0, 20_000 - int(L)))
        r = g[s : s + int(L)].copy()
        q = np.full(int(L), 40, np.uint8)
        flip = rng.random(int(L)) < 0.02
        r[flip] = (r[flip] + 1 + rng.integers(0, 3, size=int(flip.sum()))) % 4
        q[flip] = rng.integers(2, 20, size=int(flip.sum()))
        low = rng.random(int(L)) < 0.02
        q[low] = 10
        seqs.append(r)
        quals.append(q)
    # the genome itself, tiled, keeps most K-mers solid
    for s in range(0, 20_000 - 100, 7):
        seqs.append(g[s : s + 100].copy())
        quals.append(np.full(100, 40, np.uint8))
    reads = ReadSet.from_sequences(seqs, quals)
    for K in (2, 3, 5, 8, 9, 13, 24, 28, 29):
        got, st = gpu_ctx.precorrect(reads, K=K, min_solid=2)
        exp, est = oracle.precorrect(reads, K=K, min_solid=2)
        assert_same(got, exp)
        assert st == {**st, **est}


@pytest.mark.parametrize("P", [1, 2, 4])
def test_sharded_weak_return_loopback(gpu_ctx, P):
    """The multi-GPU weak-mask return on one GPU: shard_scatter_pos per slice ->
    loopback all_to_all -> shard_solid_weak per shard (solid set + per-record
    weak masks) -> masks routed back in send order -> precorrect_weak on every
    slice == monolithic PreCorrect (bases, quals, counters)."""
    import torch

    from allpathslg_amd import shard_bins

    K = 24
    reads = synth_reads(synth_genome(150_000, 71), 30_000, seed=72)
    B = shard_bins(K, P)
    parts = np.array_split(np.arange(reads.n_reads), P)
    subs = [reads.subset(int(ix[0]), int(ix[-1]) + 1) for ix in parts]
    dsubs = [gpu_ctx.upload(s) for s in subs]
    sends, poss, counts = [], [], []
    for d in dsubs:
        c = gpu_ctx.shard_count(d, K, P)
        n = int(c.sum())
        buf = torch.empty(max(2 * n, 1), dtype=torch.int64, device="cuda")
        pos = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
        torch.cuda.synchronize()
        gpu_ctx.shard_scatter_pos(d, K, P, buf.data_ptr(), pos.data_ptr())
        sends.append(buf)
        poss.append(pos)
        counts.append(c.reshape(P, B))
    solids, masks = [], []  # masks[s][p]: shard s's masks for source p's records
    for s in range(P):
        pieces, rc, sizes = [], [], []
        for p in range(P):
            starts = np.concatenate([[0], np.cumsum(counts[p].reshape(-1))]).astype(np.int64)
            pieces.append(sends[p][2 * starts[s * B] : 2 * starts[(s + 1) * B]])
            rc.append(counts[p][s])
            sizes.append(int(starts[(s + 1) * B] - starts[s * B]))
        recv = torch.cat(pieces) if sum(x.numel() for x in pieces) else torch.empty(1, dtype=torch.int64, device="cuda")
        mask = torch.empty(max(sum(sizes), 1), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        n = gpu_ctx.shard_solid_weak(recv.data_ptr(), np.concatenate(rc), K, P, 3, mask.data_ptr())
        out = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
        gpu_ctx.solid_export(out.data_ptr())
        solids.append(out[:n])
        offs = np.concatenate([[0], np.cumsum(sizes)])
        masks.append([mask[int(offs[p]) : int(offs[p + 1])] for p in range(P)])
    solid = torch.cat(solids)
    exp, est = oracle.precorrect(reads, K=K)
    tot = {"n_suspect": 0, "n_corrected": 0, "n_ambiguous": 0, "n_uncorrectable": 0}
    fixed = []
    for p, d in enumerate(dsubs):
        back = torch.cat([masks[s][p] for s in range(P)])  # send order: by destination shard
        n_rec = int(counts[p].sum())
        assert back.numel() == n_rec
        st = gpu_ctx.precorrect_weak(d, solid.data_ptr(), solid.numel(), poss[p].data_ptr(), back.data_ptr(), n_rec,
                                     K=K)
        assert st["n_solid"] == est["n_solid"]
        for k in tot:
            tot[k] += st[k]
        fixed.append(gpu_ctx.download(d))
        d.free()
    assert tot == {k: est[k] for k in tot}
    assert np.array_equal(np.concatenate([f.packed[: int(f.byte_off[-1])] for f in fixed]),
                          exp.packed[: int(exp.byte_off[-1])])
    assert np.array_equal(np.concatenate([f.quals for f in fixed]), exp.quals)
