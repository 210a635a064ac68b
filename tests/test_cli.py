"""Drop-in command-line modules (bin/<Module>, tools/apg_modules.cpp):
KEY=VALUE parsing and error exits on CPU; on the GPU the RunAllPathsLG module
chain of SURVEY.md:126-131 from files — KmerSpectrum -> PreCorrect /
FindErrors -> FillFragments -> ErrorCorrectJump -> MergeReadSets (all_reads)
-> CommonPather -> Unipather -> MakeRcDb -> UnipathLocs -> UnipathCoverage —
every output file checked against the oracle chain, and the sharded
(WORLD=N RANK=r) modules byte-identical to the single-process ones."""
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
    p = run("FillFragments", f"RUN={tmp_path}", "SOLID=nosuch")
    assert p.returncode == 1 and "missing solid set" in p.stderr
    p = run("MergeReadSets", f"RUN={tmp_path}", "HEADS=,")
    assert p.returncode == 1 and "names no read set" in p.stderr
    p = run("UnipathCoverage", f"RUN={tmp_path}")
    assert p.returncode == 1 and "run UnipathLocs first" in p.stderr


def test_cli_merge_read_sets(tmp_path):
    """MergeReadSets is host-only file work: all_reads = the inputs in order,
    0-length reads kept; qualities only when every input has them."""
    from allpathslg_amd import ReadSet

    rng = np.random.default_rng(5)
    a = ReadSet.from_sequences([rng.integers(0, 4, n) for n in (180, 0, 7, 150)])
    b = ReadSet.from_sequences([rng.integers(0, 4, n) for n in (100, 0, 40)], [rng.integers(2, 41, n) for n in (100, 0, 40)])
    a.write_fastb(str(tmp_path / "filled_reads.fastb"))
    b.write_fastb(str(tmp_path / "jump_reads_ec.fastb"))
    b.write_qualb(str(tmp_path / "jump_reads_ec.qualb"))
    p = run("MergeReadSets", f"RUN={tmp_path}")
    assert p.returncode == 0, p.stderr
    m = ReadSet.load(str(tmp_path / "all_reads.fastb"))
    assert m.n_reads == 7 and not (tmp_path / "all_reads.qualb").exists()
    for i in range(4):
        assert np.array_equal(m.read(i), a.read(i))
    for i in range(3):
        assert np.array_equal(m.read(4 + i), b.read(i))
    p = run("MergeReadSets", f"RUN={tmp_path}", "HEADS=jump_reads_ec,jump_reads_ec", "HEAD_OUT=jj")
    assert p.returncode == 0, p.stderr
    jj = ReadSet.load(str(tmp_path / "jj.fastb"), str(tmp_path / "jj.qualb"))
    assert np.array_equal(jj.quals, np.concatenate([b.quals[: int(b.base_off[-1])]] * 2))


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
    # sharded (WORLD=2 / 4 over TCP): the same files byte for byte
    # (apg_sharded_error_correct_jump: the frags' solid set counted across ranks)
    ref = {e: (tmp_path / f"jump_reads_ec.{e}").read_bytes() for e in ("fastb", "qualb")}
    for world in (2, 4):
        for e in ("fastb", "qualb"):
            (tmp_path / f"jump_reads_ec.{e}").unlink()
        for rc, o, e in _run_ranks("ErrorCorrectJump", world, f"RUN={tmp_path}", "K=24"):
            assert rc == 0, (world, e)
        for e in ("fastb", "qualb"):
            assert (tmp_path / f"jump_reads_ec.{e}").read_bytes() == ref[e], (world, e)


@pytest.mark.gpu
def test_cli_module_chain_from_files_matches_oracle(tmp_path):
    """SURVEY.md:126-131's chain on files with GPU modules only, checked file
    by file against the oracle chain: the spectrum (and its genome-size
    estimate), FindErrors' corrected reads and solid set, FillFragments
    against that set, ErrorCorrectJump against the corrected frags, all_reads
    = filled ++ trimmed jumps, the K=96 graph files, UnipathLocs of the
    corrected frag reads and UnipathCoverage of those placements."""
    import oracle
    from allpathslg_amd import (ReadSet, read_graph, read_solid, read_unilocs, read_unipath_coverage, synth_genome,
                                synth_reads)

    G = 200_000
    g = synth_genome(G, 31)
    frags = synth_reads(g, 30_000, seed=32)
    jumps = synth_reads(g, 2_000, seed=33, insert_mean=3000, insert_sd=300)
    for r, h in ((frags, "frag_reads_filt"), (jumps, "jump_reads_filt")):
        r.write_fastb(str(tmp_path / f"{h}.fastb"))
        r.write_qualb(str(tmp_path / f"{h}.qualb"))
    R = f"RUN={tmp_path}"
    # KmerSpectrum: h[m] and the genome-size estimate in its header
    p = run("KmerSpectrum", R, "K=25")
    assert p.returncode == 0, p.stderr
    spec = oracle.kmer_spectrum(frags, 25)
    lines = open(tmp_path / "frag_reads_filt.kspec.k25").read().splitlines()
    kv = dict(x.split("=") for x in lines[1][1:].split())
    est = oracle.kspec_estimate(spec)
    assert int(kv["genome_size_estimate"]) == est["genome_size"] and abs(est["genome_size"] - G) < 0.02 * G
    assert {int(a): int(b) for a, b in (x.split() for x in lines[2:])} == {m: int(c) for m, c in enumerate(spec) if c}
    # FindErrors (2 cycles): corrected reads + the last pass's solid set
    p = run("FindErrors", R, "K=24")
    assert p.returncode == 0, p.stderr
    fixed, _ = oracle.precorrect(frags, K=24, n_cycles=2)
    e1, _ = oracle.precorrect(frags, K=24, n_cycles=1)
    solid = np.sort(oracle.solid_hashes(e1, 24, 3))
    corr = ReadSet.load(str(tmp_path / "frag_reads_corr.fastb"), str(tmp_path / "frag_reads_corr.qualb"))
    assert np.array_equal(corr.packed[: int(corr.byte_off[-1])], fixed.packed[: int(fixed.byte_off[-1])])
    assert np.array_equal(corr.quals, fixed.quals)
    K, got_solid = read_solid(str(tmp_path / "frag_reads_corr.solid.k24"))
    assert K == 24 and np.array_equal(got_solid, solid)
    # FillFragments against that solid set
    p = run("FillFragments", R, "K=24")
    assert p.returncode == 0, p.stderr
    ofill, ostatus, _, _ = oracle.fill_fragments(fixed, solid, K=24)
    filled = ReadSet.load(str(tmp_path / "filled_reads.fastb"))
    assert np.array_equal(filled.base_off, ofill.base_off)
    assert np.array_equal(filled.packed[: int(filled.byte_off[-1])], ofill.packed[: int(ofill.byte_off[-1])])
    assert (ostatus == 0).sum() > 0.5 * len(ostatus)
    # ErrorCorrectJump against the corrected frag reads, then all_reads
    p = run("ErrorCorrectJump", R, "K=24", "FRAG_IN=frag_reads_corr")
    assert p.returncode == 0, p.stderr
    jfix, keep, _ = oracle.error_correct_jump(fixed, jumps, K=24)
    p = run("MergeReadSets", R)
    assert p.returncode == 0, p.stderr
    allr = ReadSet.load(str(tmp_path / "all_reads.fastb"))
    exp_all = ReadSet.from_sequences([ofill.read(i) for i in range(ofill.n_reads)] +
                                     [jfix.read(i)[: int(keep[i])] for i in range(jfix.n_reads)])
    assert np.array_equal(allr.base_off, exp_all.base_off)
    assert np.array_equal(allr.packed[: int(allr.byte_off[-1])], exp_all.packed[: int(exp_all.byte_off[-1])])
    # the K=96 graph files
    for mod in ("CommonPather", "Unipather", "MakeRcDb"):
        p = run(mod, R, "READS=all_reads", "K=96")
        assert p.returncode == 0, (mod, p.stderr)
    og = oracle.unipaths(exp_all, 96)
    back = read_graph(str(tmp_path / "all_reads"), 96)
    for k in ("len", "id_base", "rc", "ub_off", "unibases", "from", "to", "path_off", "path_start", "path_len"):
        assert np.array_equal(np.asarray(back[k]), np.asarray(og[k])), k
    # UnipathLocs of the corrected frag reads, UnipathCoverage of them
    p = run("UnipathLocs", R, "READS=all_reads", "HEAD_IN=frag_reads_corr", "K=96")
    assert p.returncode == 0, p.stderr
    olocs, _ = oracle.unipath_locs(og, fixed, 96, rc=True, sorted=True)
    K, nr, locs = read_unilocs(str(tmp_path / "frag_reads_corr.unilocs.k96"))
    assert K == 96 and nr == fixed.n_reads and len(locs) > fixed.n_reads
    assert np.array_equal(locs, olocs)
    p = run("UnipathCoverage", R, "READS=all_reads", "HEAD_IN=frag_reads_corr", "K=96")
    assert p.returncode == 0, p.stderr
    oc = oracle.unipath_coverage(og, olocs, 500)
    cov = read_unipath_coverage(str(tmp_path / "all_reads.unipath_cov.k96"))
    assert cov["c0"] == oc["c0"] and oc["c0"] > 0
    for k in ("counts", "cov", "cn"):
        assert np.array_equal(cov[k], oc[k]), k


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
    p = run("FillFragments", f"RUN={one}", "K=24")
    assert p.returncode == 0, p.stderr
    for rc, o, e in _run_ranks("FillFragments", world, f"RUN={many}", "K=24"):
        assert rc == 0, ("FillFragments", e)
    for d in (one, many):
        shutil.copy(d / "frag_reads_corr.fastb", d / "all_reads.fastb")
    for mod, args in (("CommonPather", ["READS=all_reads", "K=96"]), ("Unipather", ["READS=all_reads", "K=96"]),
                      ("UnipathLocs", ["READS=all_reads", "HEAD_IN=frag_reads_corr", "K=96"])):
        p = run(mod, f"RUN={one}", *args)
        assert p.returncode == 0, p.stderr
        for rc, o, e in _run_ranks(mod, world, f"RUN={many}", *args):
            assert rc == 0, (mod, e)
        names = sorted(f for f in os.listdir(one) if not f.startswith("all_reads.fastb"))
        assert names == sorted(f for f in os.listdir(many) if not f.startswith("all_reads.fastb"))
        for f in names:
            assert (one / f).read_bytes() == (many / f).read_bytes(), (mod, f)
    assert (one / "filled_reads.fastb").exists() and (one / "frag_reads_corr.unilocs.k96").exists()
