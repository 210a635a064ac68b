"""apg_reads_load_dev: .fastb / .qualb straight into HBM must give the same
device read set as apg_fastb_read + apg_qualb_read + apg_reads_upload —
bases, qualities and offsets byte for byte — for ragged and empty reads, for
payloads of many 16 MiB chunks spread over an odd number of workers, and it
must refuse the inputs apg_fastb_read refuses (bad magic, truncated payload,
qualb lengths that do not match the fastb)."""
import os

import numpy as np
import pytest

from allpathslg_amd import ApgError, ReadSet, synth_genome, synth_reads

pytestmark = pytest.mark.gpu


def _same(ctx, d, ref, quals):
    a = ctx.download(d, with_quals=quals)
    assert a.n_reads == ref.n_reads
    assert np.array_equal(a.base_off, ref.base_off)
    assert np.array_equal(a.byte_off, ref.byte_off)
    nb = int(ref.byte_off[-1])
    assert np.array_equal(a.packed[:nb], ref.packed[:nb])
    if quals:
        assert np.array_equal(a.quals[: ref.n_bases], ref.quals[: ref.n_bases])


def _write(tmp_path, rs, tag):
    fb, qb = str(tmp_path / f"{tag}.fastb"), str(tmp_path / f"{tag}.qualb")
    rs.write_fastb(fb)
    if rs.quals is not None:
        rs.write_qualb(qb)
    return fb, qb


def test_ragged_reads(gpu_ctx, tmp_path):
    rng = np.random.default_rng(3)
    lens = [0, 1, 3, 4, 5, 31, 32, 33, 99, 100, 250, 0, 7]
    seqs = [rng.integers(0, 4, size=n) for n in lens]
    quals = [rng.integers(2, 41, size=n) for n in lens]
    rs = ReadSet.from_sequences(seqs, quals)
    fb, qb = _write(tmp_path, rs, "ragged")
    ref = ReadSet.load(fb, qb)
    for threads in (0, 1, 3):
        d = gpu_ctx.load_reads(fb, qb, threads=threads)
        _same(gpu_ctx, d, ref, True)
        d.free()
    d = gpu_ctx.load_reads(fb)  # bases only
    _same(gpu_ctx, d, ReadSet.load(fb), False)
    d.free()


def test_many_chunks(gpu_ctx, tmp_path):
    """2 M reads: 50 MB of bases (4 chunks) and 200 MB of qualities (12
    chunks) over 3 and 8 workers; the loaded set runs the K=25 spectrum to
    the same histogram as the uploaded one."""
    g = synth_genome(2_000_000, 41)
    rs = synth_reads(g, 1_000_000, seed=42)
    fb, qb = _write(tmp_path, rs, "big")
    try:
        ref = ReadSet.load(fb, qb)
        for threads in (3, 8):
            d = gpu_ctx.load_reads(fb, qb, threads=threads)
            _same(gpu_ctx, d, ref, True)
            h1, s1 = gpu_ctx.kmer_spectrum(d, 25)
            d.free()
        du = gpu_ctx.upload(ref)
        h2, s2 = gpu_ctx.kmer_spectrum(du, 25)
        du.free()
        assert np.array_equal(h1, h2) and s1 == s2
    finally:
        for p in (fb, qb):
            os.unlink(p)


def test_empty_set(gpu_ctx, tmp_path):
    rs = ReadSet.from_sequences([], [])
    fb, qb = _write(tmp_path, rs, "empty")
    d = gpu_ctx.load_reads(fb, qb)
    assert d.n_reads == 0
    d.free()


def test_refuses_bad_inputs(gpu_ctx, tmp_path):
    rng = np.random.default_rng(4)
    seqs = [rng.integers(0, 4, size=n) for n in (50, 60, 70)]
    rs = ReadSet.from_sequences(seqs, [rng.integers(0, 41, size=len(s)) for s in seqs])
    fb, qb = _write(tmp_path, rs, "ok")
    bad = tmp_path / "bad.fastb"
    bad.write_bytes(b"NOTAFASTB" * 10)
    with pytest.raises(ApgError):
        gpu_ctx.load_reads(str(bad))
    trunc = tmp_path / "trunc.fastb"
    trunc.write_bytes(open(fb, "rb").read()[:-5])
    with pytest.raises(ApgError):
        gpu_ctx.load_reads(str(trunc))
    other = ReadSet.from_sequences([s[:-1] for s in seqs], [rng.integers(0, 41, size=len(s) - 1) for s in seqs])
    _, qo = _write(tmp_path, other, "other")
    with pytest.raises(ApgError):
        gpu_ctx.load_reads(fb, qo)
    with pytest.raises(ApgError):
        gpu_ctx.load_reads(str(tmp_path / "missing.fastb"))


def test_background_qualities_equal_uploaded(gpu_ctx, tmp_path):
    """apg_reads_load_dev returns once bases and offsets are in HBM; the
    qualities stream in on a host thread while the next module counts the
    bases, and every reader of them joins the load first.  The fused K=25
    spectrum + K=24 PreCorrect called right after the load (the bench's
    file_to_graph order) gives the uploaded set's spectrum, corrected bases,
    qualities and counters byte for byte; a set freed, copied or reloaded
    while its qualities stream is safe."""
    g = synth_genome(3_000_000, 43)
    rs = synth_reads(g, 1_500_000, seed=44)  # 300 MB of qualities: many chunks after the call returns
    fb, qb = _write(tmp_path, rs, "bg")
    try:
        d = gpu_ctx.load_reads(fb, qb)
        h1, k1, p1 = gpu_ctx.spectrum_precorrect(d, K_spec=25, K=24)
        got = gpu_ctx.download(d, with_quals=True)
        d.free()
        du = gpu_ctx.upload(rs)
        h2, k2, p2 = gpu_ctx.spectrum_precorrect(du, K_spec=25, K=24)
        exp = gpu_ctx.download(du, with_quals=True)
        assert np.array_equal(h1, h2) and k1 == k2 and p1 == p2
        nb = int(exp.byte_off[-1])
        assert np.array_equal(got.packed[:nb], exp.packed[:nb])
        assert np.array_equal(got.quals, exp.quals)
        # freed while streaming; reloaded while the previous load streams;
        # copied while streaming
        gpu_ctx.load_reads(fb, qb).free()
        a = gpu_ctx.load_reads(fb, qb)
        b = gpu_ctx.load_reads(fb, qb)
        gpu_ctx.copy_reads(du, b)
        _same(gpu_ctx, du, ReadSet.load(fb, qb), True)
        _same(gpu_ctx, a, ReadSet.load(fb, qb), True)
        for x in (a, b, du):
            x.free()
    finally:
        for p in (fb, qb):
            os.unlink(p)


def test_qualb_offsets_checked_beside_the_load(gpu_ctx, tmp_path):
    """A .qualb whose per-read lengths differ from the .fastb's at the same
    total passes the header checks; its offset table is compared with the
    fastb's beside the background qualities load, and the first reader of
    the qualities fails with APG_E_IO (a download, or PreCorrect)."""
    rng = np.random.default_rng(5)
    seqs = [rng.integers(0, 4, size=n) for n in (50, 60, 70)]
    rs = ReadSet.from_sequences(seqs, [rng.integers(0, 41, size=len(s)) for s in seqs])
    fb, _ = _write(tmp_path, rs, "okq")
    swapped = ReadSet.from_sequences([s for s in (seqs[1], seqs[0], seqs[2])],
                                     [rng.integers(0, 41, size=len(s)) for s in (seqs[1], seqs[0], seqs[2])])
    _, qb = _write(tmp_path, swapped, "swapped")
    d = gpu_ctx.load_reads(fb, qb)
    with pytest.raises(ApgError):
        gpu_ctx.download(d, with_quals=True)
    d.free()
    d = gpu_ctx.load_reads(fb, qb)
    with pytest.raises(ApgError):
        gpu_ctx.precorrect(d, K=24)
    d.free()
    # a good pair still loads on the same context
    fb2, qb2 = _write(tmp_path, rs, "good")
    d = gpu_ctx.load_reads(fb2, qb2)
    _same(gpu_ctx, d, ReadSet.load(fb2, qb2), True)
    d.free()
    # the bad set's error sticks to it.  A second load on the
    # context joins the first (without failing itself), and every later
    # reader of the bad set's qualities still fails.
    bad = gpu_ctx.load_reads(fb, qb)
    good = gpu_ctx.load_reads(fb2, qb2)
    _same(gpu_ctx, good, ReadSet.load(fb2, qb2), True)
    for _ in range(2):
        with pytest.raises(ApgError):
            gpu_ctx.precorrect(bad, K=24)
    with pytest.raises(ApgError):
        gpu_ctx.download(bad, with_quals=True)
    # overwriting its qualities from a good set clears it
    gpu_ctx.copy_reads(bad, good)
    _same(gpu_ctx, bad, ReadSet.load(fb2, qb2), True)
    bad.free()
    good.free()
