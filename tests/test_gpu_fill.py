"""GPU parity: FillFragments through libapg (apg_fill_fragments / _dev, HIP
kernels in csrc/fill.hip) vs the CPU restatement oracle/fill_oracle.c —
identical status per pair and bit-identical filled fragments.  Semantics vs
real ALLPATHS-LG: unpinned (reference snapshot empty)."""
import os

import numpy as np
import pytest

import oracle
from allpathslg_amd import ApgError, ReadSet, synth_fragments, synth_genome, synth_reads
from tests.fill_cases import K, branch_cases, genome_cases

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def same_reads(a: ReadSet, b: ReadSet):
    assert a.n_reads == b.n_reads
    assert np.array_equal(a.base_off, b.base_off)
    assert np.array_equal(a.packed[: int(a.byte_off[-1])], b.packed[: int(b.byte_off[-1])])


def test_fill_known_answers_gpu(gpu_ctx):
    pairs, solid, exp, _ = genome_cases()
    got, status, st = gpu_ctx.fill_fragments(pairs, solid, K=K, status=True)
    ef, es, _, est = oracle.fill_fragments(pairs, solid, K=K)
    assert list(status) == [e[0] for e in exp]
    assert np.array_equal(status, es)
    same_reads(got, ef)
    for k in ("n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip", "filled_bases"):
        assert st[k] == est[k], k


def test_fill_branches_gpu(gpu_ctx):
    pairs, solid_two, solid_tip, frag1 = branch_cases()
    _, status, _ = gpu_ctx.fill_fragments(pairs, solid_two, K=K, status=True)
    assert list(status) == [2, 2]
    got, status, _ = gpu_ctx.fill_fragments(pairs, solid_tip, K=K, status=True)
    assert list(status) == [0, 0]
    assert np.array_equal(got.read(0), frag1)
    _, status, _ = gpu_ctx.fill_fragments(pairs, solid_tip, K=K, max_steps=5, status=True)
    assert list(status) == [3, 3]


# K <= 25: two-level extension slots (successor's successors, a free walk
# step); K >= 26: the one-level layout.  rep: a repeat-rich genome (branching
# walks, budget pairs).
@pytest.mark.parametrize("seed,K,lo,hi,rep", [(3, 24, 126, 234, False), (4, 20, 150, 220, False),
                                              (5, 28, 100, 260, False), (6, 25, 126, 234, False),
                                              (7, 26, 126, 234, False), (8, 24, 126, 234, True)])
def test_fill_matches_oracle_synthetic(gpu_ctx, seed, K, lo, hi, rep):
    g = synth_genome(150_000, seed, repeats=True if rep else None)
    reads = synth_reads(g, 15_000, seed=seed + 100)
    fixed, _ = oracle.precorrect(reads, K=24)
    solid = oracle.solid_hashes(reads, K, 3)
    got, status, st = gpu_ctx.fill_fragments(fixed, solid, K=K, min_insert=lo, max_insert=hi, status=True)
    ef, es, _, est = oracle.fill_fragments(fixed, solid, K=K, min_insert=lo, max_insert=hi)
    assert np.array_equal(status, es)
    same_reads(got, ef)
    assert st["n_filled"] == est["n_filled"] > 0


def test_fill_golden_gpu(gpu_ctx):
    gz = np.load(os.path.join(HERE, "golden", "fill_small.npz"))
    reads = ReadSet.load(os.path.join(HERE, "golden", "frag_small.fastb"), os.path.join(HERE, "golden", "frag_small.qualb"))
    fixed, _ = gpu_ctx.precorrect(reads, K=24)
    got, status, st = gpu_ctx.fill_fragments(fixed, gz["solid"], K=24, status=True)
    assert np.array_equal(status, gz["status"])
    assert np.array_equal(got.base_off, gz["base_off"])
    assert np.array_equal(got.packed[: int(got.byte_off[-1])], gz["packed"])


def test_fill_device_last_solid_and_reuse(gpu_ctx):
    """PreCorrect on the device, then fill with the pass's own solid set
    (APG_FILL_LAST_SOLID) into a reused device read set; equals the host API
    with the solid set given explicitly, and feeds the unipath stage."""
    g = synth_genome(120_000, 61)
    reads = synth_reads(g, 12_000, seed=62)
    d = gpu_ctx.upload(reads)
    gpu_ctx.precorrect(d, K=24)
    fixed = gpu_ctx.download(d)
    solid = oracle.solid_hashes(reads, 24, 3)
    exp, es, _, _ = oracle.fill_fragments(fixed, solid, K=24)
    out = None
    for _ in range(2):  # second round reuses the buffers of the first
        out, _, st = gpu_ctx.fill_fragments(d, K=24, last_solid=True, out=out)
        assert st["n_filled"] == int((es == 0).sum()) == out.n_reads
    gpu_ctx_unipaths, ust = gpu_ctx.unipaths(out, 96)
    eg = oracle.unipaths(exp, 96)
    for k in ("len", "id_base", "rc", "unibases", "from", "to", "path_off", "path_start", "path_len"):
        assert np.array_equal(gpu_ctx_unipaths[k], eg[k]), k
    out.free()
    d.free()


def test_fill_own_count_mode(gpu_ctx):
    """No solid set given: the pairs' own K-mers with count >= min_solid."""
    g = synth_genome(80_000, 71)
    reads = synth_reads(g, 10_000, seed=72)
    got, status, _ = gpu_ctx.fill_fragments(reads, None, K=24, min_solid=2, status=True)
    exp, es, _, _ = oracle.fill_fragments(reads, oracle.solid_hashes(reads, 24, 2), K=24)
    assert np.array_equal(status, es)
    same_reads(got, exp)


def test_fill_errors(gpu_ctx):
    odd = ReadSet.from_sequences([np.zeros(100, np.uint8)] * 3)
    with pytest.raises(ApgError):
        gpu_ctx.fill_fragments(odd, np.zeros(1, np.uint64), K=24)
    pairs, solid, _, _ = genome_cases()
    with pytest.raises(ApgError):
        gpu_ctx.fill_fragments(pairs, solid, K=31)  # K > 29
    with pytest.raises(ApgError):
        gpu_ctx.fill_fragments(pairs, solid, K=24, min_insert=300, max_insert=200)
    empty = ReadSet.from_sequences([])
    got, status, st = gpu_ctx.fill_fragments(empty, solid, K=24, status=True)
    assert got.n_reads == 0 and st["n_pairs"] == 0


def test_fill_full_size_properties(gpu_ctx):
    """2 M pairs (too many for the oracle): size-independent properties —
    every filled fragment starts with A, ends with rc(B), has a length in the
    insert window, statuses add up; the device path agrees with the host
    path on the same corrected reads."""
    n = 2_000_000
    g = synth_genome(5_000_000, 81)
    reads = synth_reads(g, n, seed=82, threads=16)
    d = gpu_ctx.upload(reads)
    gpu_ctx.precorrect(d, K=24)
    fixed = gpu_ctx.download(d)
    out, _, st = gpu_ctx.fill_fragments(d, K=24, min_solid=3)  # own count of the corrected reads
    host, status, st2 = gpu_ctx.fill_fragments(fixed, None, K=24, min_solid=3, status=True)
    assert st == {**st, **{k: v for k, v in st2.items() if k != "lookups"}}
    assert out.n_reads == host.n_reads == int((status == 0).sum()) > n // 2
    assert sum(int((status == s).sum()) for s in range(5)) == n
    lens = np.diff(host.base_off).astype(np.int64)
    assert lens.min() >= 126 and lens.max() <= 234
    idx = np.nonzero(status == 0)[0]
    # A = the first 25 bytes of each fragment (both byte-aligned, 100 bases)
    fo = host.byte_off[:-1].astype(np.int64)[:, None] + np.arange(25)
    ao = fixed.byte_off[2 * idx].astype(np.int64)[:, None] + np.arange(25)
    assert np.array_equal(host.packed[fo], fixed.packed[ao])
    rng = np.random.default_rng(0)
    for j in rng.choice(len(idx), 2000, replace=False):
        frag = host.read(int(j))
        b = fixed.read(2 * int(idx[j]) + 1)
        assert np.array_equal(frag[-100:], (3 - b)[::-1])
    truth = synth_fragments(g, n, seed=82, threads=16)
    tl = np.diff(truth.base_off).astype(np.int64)[idx]
    assert (tl == lens).mean() > 0.999  # filled lengths are the true inserts
    out.free()
    d.free()


def test_fill_last_solid_long_and_short_reads(gpu_ctx):
    """Clean flags of the correction pass (weak-bitmap path, reads <= 1024)
    and the thread-per-read path (longer reads, flags not derived: the fill
    looks their K-mers up) give the oracle's fill."""
    rng = np.random.default_rng(17)
    G = synth_genome(60_000, 18)
    seqs, quals = [], []
    for i in range(1200):
        La = 1100 if i % 3 == 0 else 100
        I = int(rng.integers(2 * La - 40, 2 * La + 40))
        s = int(rng.integers(0, len(G) - I))
        A = G[s : s + La].copy()
        F = G[s + I - La : s + I].copy()
        for r in (A, F):
            flip = rng.random(La) < 0.01
            r[flip] = (r[flip] + 1) % 4
        qa = np.where(rng.random(La) < 0.05, 10, 40).astype(np.uint8)
        qb = np.where(rng.random(La) < 0.05, 10, 40).astype(np.uint8)
        seqs += [A, (3 - F)[::-1].copy()]
        quals += [qa, qb]
    reads = ReadSet.from_sequences(seqs, quals)
    fixed, _ = oracle.precorrect(reads, K=24)
    solid = oracle.solid_hashes(reads, 24, 3)
    for lo, hi in ((160, 240), (2160, 2240)):
        d = gpu_ctx.upload(reads)
        gpu_ctx.precorrect(d, K=24)
        assert np.array_equal(gpu_ctx.download(d).packed[: int(fixed.byte_off[-1])], fixed.packed[: int(fixed.byte_off[-1])])
        out, _, st = gpu_ctx.fill_fragments(d, K=24, last_solid=True, min_insert=lo, max_insert=hi)
        exp, es, _, est = oracle.fill_fragments(fixed, solid, K=24, min_insert=lo, max_insert=hi)
        assert st["n_filled"] == est["n_filled"] and st["n_skip"] == est["n_skip"]
        host, hs, _ = gpu_ctx.fill_fragments(fixed, solid, K=24, min_insert=lo, max_insert=hi, status=True)
        assert np.array_equal(hs, es)
        same_reads(host, exp)
        out.free()
        d.free()


# The general (non-LEAN) k_fill form runs whenever an APG_FILL_* A/B knob is
# set; round 5 never tested it against the oracle (a two-pass
# split had diverged).  Every form must give the oracle's statuses and bases.
@pytest.mark.parametrize("env", [{"APG_FILL_LEAN": "0"}, {"APG_FILL_CAP1": "50"}, {"APG_FILL_CAP1": "1"},
                                 {"APG_FILL_XSTEPS": "0"}, {"APG_FILL_FUSE_BT": "0"},
                                 {"APG_FILL_BRANCH_CACHE": "0"}, {"APG_FILL_BRIDGE_FILTER": "0"},
                                 {"APG_FILL_REFILL": "8"}])
def test_fill_general_forms_match_oracle(gpu_ctx, monkeypatch, env):
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    g = synth_genome(150_000, 5, repeats=True)
    reads = synth_reads(g, 15_000, seed=105)
    fixed, _ = oracle.precorrect(reads, K=24)
    solid = oracle.solid_hashes(reads, 24, 3)
    args = dict(K=24, min_insert=100, max_insert=260, max_steps=300)
    got, status, st = gpu_ctx.fill_fragments(fixed, solid, status=True, **args)
    ef, es, _, est = oracle.fill_fragments(fixed, solid, **args)
    bad = np.nonzero(status != es)[0]
    assert len(bad) == 0, (len(bad), list(zip(es[bad[:8]].tolist(), status[bad[:8]].tolist())))
    same_reads(got, ef)
    for k in ("n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip", "filled_bases"):
        assert st[k] == est[k], k
