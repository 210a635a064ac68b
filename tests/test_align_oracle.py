"""Known-answer tests of the CPU restatement of the aligners and consensus
(oracle/align_oracle.c; SURVEY §A.7, §A.8 KAT 6).  Parity vs real ALLPATHS-LG
is unpinned (reference snapshot empty)."""
import itertools

import numpy as np

import oracle
from allpathslg_amd import ReadSet
from tests.align_cases import apply_blocks, full_dp_cost, sw_case


def rs(*seqs, quals=None):
    return ReadSet.from_sequences([np.asarray(s, np.uint8) for s in seqs], quals)


def test_gapfree_known_answers():
    T = rs([0, 1, 2, 3] * 10)
    S = rs([0, 1, 2, 3, 0, 1, 2, 3], [0, 1, 2, 2, 0, 1, 2, 3], [3, 2, 1, 0, 3, 2, 1, 0],
           quals=[[30] * 8, [5, 6, 7, 8, 9, 10, 11, 12], [20] * 8])
    pairs = [(0, 0, 0, 0), (0, 0, 4, 0), (1, 0, 0, 0), (0, 0, 1, 0), (0, 0, -3, 0), (0, 0, 36, 0), (0, 0, 40, 0),
             (2, 0, 0, 1)]
    out = oracle.gapfree(S, T, pairs)
    assert out[0].tolist() == [8, 0, 0, 0]
    assert out[1].tolist() == [8, 0, 0, 4]
    assert out[2].tolist() == [8, 1, 8, 0]  # S[3]=2 vs T[3]=3, Q 8
    assert out[3][1] == 8 and out[3][2] == 8 * 30  # shifted by one: every base differs
    assert out[4][0] == 5  # overlap at negative offset
    assert out[5][0] == 4 and out[6][0] == 0
    assert out[7][1] == 8  # TGCA is its own reverse complement: every base faces a different one


def test_gapfree_reverse_complement_and_quals():
    rng = np.random.default_rng(3)
    T = rng.integers(0, 4, size=300).astype(np.uint8)
    src = T[40:140].copy()
    q = rng.integers(2, 41, size=100).astype(np.uint8)
    src[[3, 50, 97]] = (src[[3, 50, 97]] + 1) % 4
    rcs = (3 - src)[::-1].copy()
    S = rs(src, rcs, quals=[q, q[::-1].copy()])
    out = oracle.gapfree(S, rs(T), [(0, 0, 40, 0), (1, 0, 40, 1)])
    for row in out:
        assert row[0] == 100 and row[1] == 3 and row[2] == int(q[3]) + int(q[50]) + int(q[97])


def test_banded_equals_full_dp_exhaustive_small():
    """SURVEY §A.8 KAT 6: with a band covering every diagonal, banded SW is the
    full DP; exhaustive over all S of length <= 4 against fixed T."""
    T = np.array([0, 1, 1, 2, 3, 0, 2], np.uint8)
    Ts = rs(T)
    for L in range(1, 5):
        seqs = [np.array(x, np.uint8) for x in itertools.product(range(4), repeat=L)]
        S = ReadSet.from_sequences(seqs)
        pairs = [(i, 0, 0, 0) for i in range(len(seqs))]
        res, blk = oracle.banded_sw(S, Ts, pairs, band_w=len(T) + L, max_blocks=8)
        for i, sq in enumerate(seqs):
            r = res[i]
            assert r[7] == 0
            assert r[0] == full_dp_cost(sq, T), (sq, r)
            assert r[0] == 2 * r[3] + 3 * (r[4] + r[5])
            nb = r[6]
            cost, si, tj = apply_blocks(sq, T, r[1], blk[i][:nb])
            assert cost == r[0] and si == L and tj == r[2]


def test_banded_known_indels():
    rng = np.random.default_rng(9)
    T = rng.integers(0, 4, size=200).astype(np.uint8)
    S_del = np.delete(T[50:150], 40)  # one T base missing from S: gap in S
    S_ins = np.insert(T[50:150], 40, (T[90] + 1) % 4)  # one extra S base: gap in T
    S = rs(S_del, S_ins, T[50:150])
    res, blk = oracle.banded_sw(S, rs(T), [(0, 0, 50, 0), (1, 0, 50, 0), (2, 0, 50, 0)], band_w=5, max_blocks=4)
    assert res[0][0] == 3 and res[0][4] == 1 and res[0][5] == 0 and res[0][1] == 50 and res[0][2] == 150
    assert res[1][0] == 3 and res[1][4] == 0 and res[1][5] == 1
    assert res[2][0] == 0 and res[2][6] == 1 and blk[2][0].tolist() == [0, 100]


def test_banded_band_limits_and_status():
    rng = np.random.default_rng(10)
    T = rng.integers(0, 4, size=120).astype(np.uint8)
    S = rs(T[30:80])
    # the true placement (offset 30) outside a band around offset 0: worse cost
    res_far, _ = oracle.banded_sw(S, rs(T), [(0, 0, 0, 0)], band_w=3)
    res_ok, _ = oracle.banded_sw(S, rs(T), [(0, 0, 28, 0)], band_w=3)
    assert res_ok[0][0] == 0 and res_far[0][0] > 0
    # band entirely right of T: no cell reaches the end of S
    res_none, _ = oracle.banded_sw(S, rs(T[:10]), [(0, 0, 500, 0)], band_w=2)
    assert res_none[0][7] == 1


def test_banded_random_consistency():
    S, T, pairs = sw_case(n_targets=5, n_pairs=60, tlen=250, slen=(30, 90))
    res, blk = oracle.banded_sw(S, T, pairs, band_w=12, max_blocks=64)
    for k, (s, t, off, fl) in enumerate(pairs):
        r = res[k]
        if r[7]:
            continue
        sq = S.read(int(s))
        if fl:
            sq = (3 - sq)[::-1]
        cost, si, tj = apply_blocks(sq, T.read(int(t)), r[1], blk[k][: r[6]])
        assert cost == r[0] and si == len(sq) and tj == r[2]


def test_consensus_votes_ties_and_quality():
    T = rs([0, 0, 0, 0, 0, 0])
    R = rs([1, 1, 1, 1], [2, 2, 0, 0], [1, 2], quals=[[10, 10, 10, 10], [10, 30, 5, 70], [5, 5]])
    plc = [(0, 0, 0, 0), (1, 0, 0, 0), (2, 0, 4, 0)]
    b, q = oracle.consensus(R, T, plc)
    # col0: C10 vs G10 -> tie between non-target bases -> smaller code (C); Q 0
    # col1: C10 vs G30 -> G, Q 20; col2: C10 vs A5 -> C, Q 5; col3: C10 vs A70 -> A (target), Q 60
    # col4: C5 -> C, Q 5; col5: G5 -> G, Q 5
    assert b.tolist() == [1, 2, 1, 0, 1, 2]
    assert q.tolist() == [0, 20, 5, 60, 5, 5]
    b2, q2 = oracle.consensus(R, T, [])
    assert b2.tolist() == [0] * 6 and q2.tolist() == [0] * 6
    # a tie that includes the target base keeps it
    b3, q3 = oracle.consensus(rs([1], [0], quals=[[7], [7]]), rs([0]), [(0, 0, 0, 0), (1, 0, 0, 0)])
    assert b3.tolist() == [0] and q3.tolist() == [0]
