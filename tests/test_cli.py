"""Drop-in command-line modules (bin/<Module>, tools/apg_modules.cpp):
KEY=VALUE parsing and error exits on CPU; on the GPU the whole chain
KmerSpectrum -> PreCorrect / FindErrors -> CommonPather -> Unipather ->
MakeRcDb on files, checked against the oracle."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "bin")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def _ensure_bin():
    if not os.path.exists(os.path.join(BIN, "MakeRcDb")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tools")], check=True)


def run(module, *args):
    _ensure_bin()
    return subprocess.run([os.path.join(BIN, module), *args], capture_output=True, text=True, timeout=600)


def test_cli_argument_errors(tmp_path):
    p = run("KmerSpectrum", f"RUN={tmp_path}", "READS=none")
    assert p.returncode == 1 and "missing input" in p.stderr
    p = run("PreCorrect", "BOGUS=1")
    assert p.returncode == 1 and "unknown argument BOGUS" in p.stderr
    p = run("FindErrors", "K=abc")
    assert p.returncode == 1 and "not an integer" in p.stderr
    p = run("Unipather", "notkeyvalue")
    assert p.returncode == 1 and "KEY=VALUE" in p.stderr
    p = run("MakeRcDb", f"RUN={tmp_path}")
    assert p.returncode == 1 and "CommonPather" in p.stderr


def _stage(tmp_path, name):
    import shutil

    for ext in ("fastb", "qualb"):
        shutil.copy(os.path.join(GOLDEN, f"frag_small.{ext}"), tmp_path / f"{name}.{ext}")


@pytest.mark.gpu
def test_cli_pipeline_matches_oracle(tmp_path):
    import oracle
    from allpathslg_amd import ReadSet, read_graph, read_kmerpaths

    _stage(tmp_path, "frag_reads_filt")
    reads = ReadSet.load(str(tmp_path / "frag_reads_filt.fastb"), str(tmp_path / "frag_reads_filt.qualb"))
    p = run("KmerSpectrum", f"RUN={tmp_path}", "K=25")
    assert p.returncode == 0, p.stderr
    exp = oracle.kmer_spectrum(reads, 25)
    got = {}
    for line in open(tmp_path / "frag_reads_filt.kspec.k25"):
        if line.strip() and not line.startswith("#"):
            m, c = line.split()[:2]
            got[int(m)] = int(c)
    assert got == {m: int(c) for m, c in enumerate(exp) if c}
    for mod, cyc, out in (("PreCorrect", 1, "frag_reads_edit"), ("FindErrors", 2, "frag_reads_corr")):
        p = run(mod, f"RUN={tmp_path}", "K=24")
        assert p.returncode == 0, p.stderr
        fixed = ReadSet.load(str(tmp_path / f"{out}.fastb"), str(tmp_path / f"{out}.qualb"))
        e, _ = oracle.precorrect(reads, K=24, n_cycles=cyc)
        assert np.array_equal(fixed.packed[: int(fixed.byte_off[-1])], e.packed[: int(e.byte_off[-1])])
        assert np.array_equal(fixed.quals, e.quals)
    # unipaths on the corrected reads
    import shutil

    shutil.copy(tmp_path / "frag_reads_corr.fastb", tmp_path / "all_reads.fastb")
    for mod in ("CommonPather", "Unipather", "MakeRcDb"):
        p = run(mod, f"RUN={tmp_path}", "READS=all_reads", "K=31")
        assert p.returncode == 0, (mod, p.stderr)
    corr = ReadSet.load(str(tmp_path / "all_reads.fastb"))
    g = oracle.unipaths(corr, 31)
    back = read_graph(str(tmp_path / "all_reads"), 31)
    for k in ("len", "id_base", "rc", "ub_off", "unibases", "from", "to", "path_off", "path_start", "path_len"):
        assert np.array_equal(np.asarray(back[k]), np.asarray(g[k])), k
    db = oracle.make_rc_db(g)
    K, off, st, ln = read_kmerpaths(str(tmp_path / "all_reads.paths_rc.k31"))
    assert np.array_equal(off, db["rc_path_off"]) and np.array_equal(st, db["rc_start"])
    raw = np.fromfile(tmp_path / "all_reads.pathsdb.k31", dtype=np.uint8)[48:]
    assert np.array_equal(raw, db["entries"].view(np.uint8))


@pytest.mark.gpu
def test_cli_error_correct_jump_matches_oracle(tmp_path):
    """ErrorCorrectJump module: jump reads corrected against the frag reads'
    solid set and written trimmed (one read per input read) = restatement."""
    import oracle
    from allpathslg_amd import ReadSet, synth_genome, synth_reads

    g = synth_genome(100_000, 21)
    frags = synth_reads(g, 20_000, seed=22)
    jumps = synth_reads(g, 1_500, seed=23, insert_mean=3000, insert_sd=300)
    frags.write_fastb(str(tmp_path / "frag_reads_edit.fastb"))
    jumps.write_fastb(str(tmp_path / "jump_reads_filt.fastb"))
    jumps.write_qualb(str(tmp_path / "jump_reads_filt.qualb"))
    p = run("ErrorCorrectJump", f"RUN={tmp_path}", "K=24")
    assert p.returncode == 0, p.stderr
    out = ReadSet.load(str(tmp_path / "jump_reads_ec.fastb"), str(tmp_path / "jump_reads_ec.qualb"))
    fixed, keep, _ = oracle.error_correct_jump(frags, jumps, K=24)
    assert out.n_reads == jumps.n_reads
    assert np.array_equal(out.lengths(), keep.astype(out.lengths().dtype))
    for r in range(0, jumps.n_reads, 7):
        k = int(keep[r])
        assert np.array_equal(out.read(r), fixed.read(r)[:k])
        assert np.array_equal(out.quals[int(out.base_off[r]) : int(out.base_off[r + 1])],
                              fixed.quals[int(fixed.base_off[r]) : int(fixed.base_off[r]) + k])


def test_cli_shard_argument_errors(tmp_path):
    _stage(tmp_path, "frag_reads_filt")
    p = run("KmerSpectrum", f"RUN={tmp_path}", "WORLD=2", "RANK=2")
    assert p.returncode == 1 and "RANK / WORLD" in p.stderr
    p = run("KmerSpectrum", f"RUN={tmp_path}", "WORLD=2", "RANK=0", "COMM=mpi")
    assert p.returncode == 1 and "COMM must be" in p.stderr


def _free_port():
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_ranks(module, world, *args):
    """`world` processes of one module (WORLD/RANK/COMM=tcp on 127.0.0.1),
    sharing GPU 0; returns their completed processes."""
    _ensure_bin()
    port = _free_port()
    ps = [subprocess.Popen([os.path.join(BIN, module), *args, f"WORLD={world}", f"RANK={r}", "COMM=tcp",
                            "MASTER_ADDR=127.0.0.1", f"MASTER_PORT={port}"],
                           stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True) for r in range(world)]
    out = []
    for p in ps:
        o, e = p.communicate(timeout=300)
        out.append((p.returncode, o, e))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4])
def test_cli_sharded_matches_single_process(tmp_path, world):
    """RunAllPathsLG-style modules one process per rank (WORLD=N RANK=r): the
    files they write are byte-identical to the single-process modules'."""
    import shutil

    one, many = tmp_path / "one", tmp_path / "many"
    for d in (one, many):
        d.mkdir()
        _stage(d, "frag_reads_filt")
    steps = [("KmerSpectrum", ["K=25"]), ("PreCorrect", ["K=24"]), ("FindErrors", ["K=24"])]
    for mod, args in steps:
        p = run(mod, f"RUN={one}", *args)
        assert p.returncode == 0, p.stderr
        for rc, o, e in _run_ranks(mod, world, f"RUN={many}", *args):
            assert rc == 0, (mod, e)
    for d in (one, many):
        shutil.copy(d / "frag_reads_corr.fastb", d / "all_reads.fastb")
    for mod in ("CommonPather", "Unipather"):
        p = run(mod, f"RUN={one}", "READS=all_reads", "K=96")
        assert p.returncode == 0, p.stderr
        for rc, o, e in _run_ranks(mod, world, f"RUN={many}", "READS=all_reads", "K=96"):
            assert rc == 0, (mod, e)
        names = sorted(f for f in os.listdir(one) if not f.startswith("all_reads.fastb"))
        assert names == sorted(f for f in os.listdir(many) if not f.startswith("all_reads.fastb"))
        for f in names:
            assert (one / f).read_bytes() == (many / f).read_bytes(), (mod, f)
