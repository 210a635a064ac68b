"""MakeRcDb: rc read paths and the sorted interval index.
CPU: the numpy restatement against first-principles properties; GPU: libapg
against the restatement (exact)."""
import numpy as np
import pytest

import oracle
from tests.unipath_cases import noisy_reads


def _kmer_seq(g, K, kid):
    u = int(np.searchsorted(g["id_base"], kid, side="right") - 1)
    o = int(kid - g["id_base"][u])
    a = int(g["ub_off"][u]) + o
    return g["unibases"][a : a + K]


def _spell(g, K, starts, lens):
    ids = [int(s) + t for s, l in zip(starts, lens) for t in range(int(l))]
    if not ids:
        return np.zeros(0, np.uint8)
    seq = list(_kmer_seq(g, K, ids[0]))
    for kid in ids[1:]:
        seq.append(int(_kmer_seq(g, K, kid)[-1]))
    return np.array(seq, np.uint8)


def test_rc_paths_spell_reverse_complements_and_index_is_sorted():
    K = 15
    reads = noisy_reads(G=3000, n=300, L=60)
    g = oracle.unipaths(reads, K)
    db = oracle.make_rc_db(g)
    for r in range(0, reads.n_reads, 7):
        a, b = int(db["rc_path_off"][r]), int(db["rc_path_off"][r + 1])
        rd = reads.read(r)
        assert np.array_equal(_spell(g, K, db["rc_start"][a:b], db["rc_len"][a:b]), (3 - rd)[::-1])
    e = db["entries"]
    assert len(e) == len(g["path_start"]) + len(db["rc_start"])
    assert np.all(np.diff(e["start"].astype(np.int64)) >= 0)
    # rc of rc is the forward path
    g2 = dict(g, path_off=db["rc_path_off"], path_start=db["rc_start"], path_len=db["rc_len"])
    back = oracle.make_rc_db(g2)
    assert np.array_equal(back["rc_start"], g["path_start"]) and np.array_equal(back["rc_len"], g["path_len"])


@pytest.mark.gpu
@pytest.mark.parametrize("K", [15, 31, 96])
def test_make_rc_db_gpu_parity(gpu_ctx, K):
    reads = noisy_reads(G=20_000, n=2000 if K < 96 else 4000, L=100 if K < 96 else 150)
    g, _ = gpu_ctx.unipaths(reads, K)
    got = gpu_ctx.make_rc_db(g)
    exp = oracle.make_rc_db(g)
    for k in ("rc_path_off", "rc_start", "rc_len"):
        assert np.array_equal(got[k], exp[k]), k
    assert np.array_equal(got["entries"], exp["entries"])


def test_graph_and_rcdb_files_round_trip(tmp_path):
    """.unipaths/.unibases/.hkp/.paths and .paths_rc/.pathsdb writers and
    readers (CPU only: no device needed)."""
    from allpathslg_amd import read_graph, read_kmerpaths, write_graph, write_rc_db

    K = 21
    reads = noisy_reads(G=4000, n=400, L=80)
    g = oracle.unipaths(reads, K)
    head = str(tmp_path / "all_reads")
    write_graph(head, g, K)
    back = read_graph(head, K)
    for k in ("len", "id_base", "rc", "ub_off", "unibases", "from", "to", "path_off", "path_start", "path_len"):
        assert np.array_equal(np.asarray(back[k]), np.asarray(g[k])), k
    assert back["n_vertices"] == g["n_vertices"]
    db = oracle.make_rc_db(g)
    write_rc_db(head, K, db)
    k2, off, st, ln = read_kmerpaths(head + f".paths_rc.k{K}")
    assert k2 == K and np.array_equal(off, db["rc_path_off"]) and np.array_equal(st, db["rc_start"])
    raw = open(head + f".pathsdb.k{K}", "rb").read()
    assert raw[:5] == b"APGDB" and len(raw) == 32 + 16 + 24 * len(db["entries"])
    bad = tmp_path / "bad.paths.k21"
    bad.write_bytes(b"garbage!" * 8)
    from allpathslg_amd import ApgError

    with pytest.raises(ApgError):
        read_kmerpaths(str(bad))
