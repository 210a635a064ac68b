"""CPU checks of the drop-in boundary: libapg.so loads, exports every entry
point declared in include/apg.h, and its host-only functions (hash, synth,
file formats) behave; no GPU compute here."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
from allpathslg_amd import ApgError, ReadSet, kmer_hash, kmer_unhash, lib, synth_genome, synth_reads
from allpathslg_amd._lib import LIB_PATH, SIGNATURES

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in os.listdir(os.path.join(ROOT, "include")):
        if not h.endswith(".h"):
            continue
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        names |= set(re.findall(r"\b(apg_[a-z0-9_]+)\s*\(", src))
    return names


def test_every_declared_symbol_is_exported():
    names = declared_functions()
    assert len(names) > 20
    out = subprocess.run(["nm", "-D", "--defined-only", LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = sorted(n for n in names if n not in exported)
    assert not missing, f"declared but not exported: {missing}"
    L = lib()
    for n in names:
        assert hasattr(L, n)


def test_binding_covers_header():
    assert declared_functions() == set(SIGNATURES)


def test_abi_version():
    assert lib().apg_abi_version() == 1


@pytest.mark.parametrize("K", [1, 7, 16, 24, 25, 31, 32])
def test_library_hash_matches_oracle(K):
    rng = np.random.default_rng(K)
    for x in rng.integers(0, 2**62, size=200, dtype=np.uint64):
        x = int(x) & ((1 << (2 * K)) - 1)
        h = kmer_hash(K, x)
        assert h == oracle.kmer_hash(K, x)
        assert kmer_unhash(K, h) == x


def test_synth_deterministic_and_sliceable():
    g = synth_genome(100_000, 42)
    assert np.array_equal(g, synth_genome(100_000, 42))
    assert not np.array_equal(g, synth_genome(100_000, 43))
    assert set(np.unique(g)) <= {0, 1, 2, 3}
    a = synth_reads(g, 1000, seed=9, threads=1)
    b = synth_reads(g, 1000, seed=9, threads=8)
    assert np.array_equal(a.packed, b.packed) and np.array_equal(a.quals, b.quals)
    # pairs [400, 1000) regenerated independently equal the tail of the full set
    c = synth_reads(g, 600, seed=9, first_pair=400)
    assert np.array_equal(c.packed[: 1200 * 25], a.packed[800 * 25 : 2000 * 25])


def test_synth_error_model():
    g = synth_genome(200_000, 1)
    r = synth_reads(g, 5000, seed=2)
    q = r.quals.reshape(-1, 100)
    err = q < 40
    rate = err.mean()
    assert 0.007 < rate < 0.014  # mean of 0.2%..2% ramp = 1.1%
    assert err[:, :10].mean() < err[:, -10:].mean()
    assert q[err].min() >= 2 and q[err].max() <= 20


def test_synth_reads_come_from_genome():
    g = synth_genome(20_000, 5)
    r = synth_reads(g, 200, seed=6, err_lo=0.0, err_hi=0.0)
    gs = "".join("ACGT"[x] for x in g)
    rcs = "".join("ACGT"[3 - x] for x in g[::-1])
    for i in range(0, 40):
        s = "".join("ACGT"[x] for x in r.read(i))
        assert s in gs or s in rcs


def test_fastb_qualb_roundtrip(tmp_path):
    rng = np.random.default_rng(0)
    seqs = [rng.integers(0, 4, size=int(n)) for n in [0, 1, 3, 4, 5, 99, 100, 250]]
    quals = [rng.integers(0, 60, size=len(s)) for s in seqs]
    rs = ReadSet.from_sequences(seqs, quals)
    fb, qb = str(tmp_path / "x.fastb"), str(tmp_path / "x.qualb")
    rs.write_fastb(fb)
    rs.write_qualb(qb)
    back = ReadSet.load(fb, qb)
    assert back.n_reads == len(seqs)
    for i, s in enumerate(seqs):
        assert np.array_equal(back.read(i), s)
    assert np.array_equal(back.quals, rs.quals)
    assert not os.path.exists(fb + ".tmp")


def test_fastb_bad_magic(tmp_path):
    p = tmp_path / "bad.fastb"
    p.write_bytes(b"NOTAFASTB" * 10)
    with pytest.raises(ApgError) as e:
        ReadSet.load(str(p))
    assert e.value.code == -3


def test_create_fails_loudly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from allpathslg_amd import Context

    with pytest.raises(ApgError) as e:
        Context(0)
    assert e.value.code == -2
    assert "HIP" in str(e.value) or "device" in str(e.value)


def test_synth_fragments_are_the_pairs_inserts():
    """Each fragment starts with read A and ends with rc(read B) (error-free
    reads), so the oracle fill is exactly the simulated insert."""
    from allpathslg_amd import synth_fragments

    g = synth_genome(20_000, 5)
    reads = synth_reads(g, 500, seed=6, err_lo=0.0, err_hi=0.0)
    frags = synth_fragments(g, 500, seed=6)
    assert frags.n_reads == 500
    lens = np.diff(frags.base_off)
    assert lens.min() >= 100 and abs(lens.mean() - 180) < 5
    for k in range(500):
        f = frags.read(k)
        a, b = reads.read(2 * k), reads.read(2 * k + 1)
        assert np.array_equal(f[:100], a)
        assert np.array_equal(f[-100:], (3 - b)[::-1])
    part = synth_fragments(g, 100, seed=6, first_pair=200)
    assert np.array_equal(part.read(7), frags.read(207))


def test_lib_variant_name_is_validated():
    """APG_LIB_VARIANT only selects libapg_<[A-Za-z0-9_]+>.so in the package
    directory, and a missing variant fails loudly."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = "import sys; sys.path.insert(0, %r); import allpathslg_amd._lib as L; print(L.LIB_PATH)" % root
    for bad, err in (("../x", "ValueError"), ("a/b", "ValueError"), ("nope_not_built", "FileNotFoundError")):
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, APG_LIB_VARIANT=bad),
                           capture_output=True, text=True)
        assert r.returncode != 0 and err in r.stderr, (bad, r.stderr[-500:])
    env = dict(os.environ)
    env.pop("APG_LIB_VARIANT", None)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True)
    assert r.returncode == 0 and r.stdout.strip().endswith("libapg.so")
