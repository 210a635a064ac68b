"""ctypes binding of the CPU restatement (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg, never by the product package.  Parity is
UNPINNED against the real ALLPATHS-LG (reference snapshot empty).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None

_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)
_u8p = C.POINTER(C.c_uint8)


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return LIB_PATH


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.ork_hash.restype = C.c_uint64
        L.ork_hash.argtypes = [C.c_int, C.c_uint64]
        L.ork_unhash.restype = C.c_uint64
        L.ork_unhash.argtypes = [C.c_int, C.c_uint64]
        L.ork_count_instances.restype = C.c_uint64
        L.ork_count_instances.argtypes = [C.c_uint64, _u64p, C.c_int]
        L.ork_extract_hashes.restype = C.c_uint64
        L.ork_extract_hashes.argtypes = [C.c_uint64, _u64p, _u64p, _u8p, C.c_int, _u64p]
        L.ork_kmer_count.restype = C.c_uint64
        L.ork_kmer_count.argtypes = [C.c_uint64, _u64p, _u64p, _u8p, C.c_int, C.POINTER(_u64p), C.POINTER(_u32p)]
        L.ork_kmer_count_range.restype = C.c_uint64
        L.ork_kmer_count_range.argtypes = [C.c_uint64, _u64p, _u64p, _u8p, C.c_int, C.c_uint64, C.c_uint64,
                                           C.POINTER(_u64p), C.POINTER(_u32p)]
        L.ork_set_threads.restype = None
        L.ork_set_threads.argtypes = [C.c_int]
        L.ork_threads.restype = C.c_int
        L.ork_threads.argtypes = []
        L.ork_spectrum.restype = None
        L.ork_spectrum.argtypes = [_u32p, C.c_uint64, _u64p, C.c_uint64]
        L.ork_precorrect.restype = C.c_int
        L.ork_precorrect.argtypes = [C.c_uint64, _u64p, _u64p, _u8p, _u8p, C.c_int, C.c_uint32, C.c_uint32,
                                     C.c_uint32, _u64p]
        L.ork_precorrect_solid.restype = C.c_int
        L.ork_precorrect_solid.argtypes = [C.c_uint64, _u64p, _u64p, _u8p, _u8p, C.c_int, C.c_uint32, _u64p,
                                           C.c_uint64, _u64p]
        L.ork_kspec_estimate.restype = None
        L.ork_kspec_estimate.argtypes = [_u64p, C.c_uint64, _u64p, C.POINTER(C.c_double)]
        L.ork_free.restype = None
        L.ork_free.argtypes = [C.c_void_p]
        _lib = L
    return _lib


def _rp(reads):
    return (
        reads.n_reads,
        reads.base_off.ctypes.data_as(_u64p),
        reads.byte_off.ctypes.data_as(_u64p),
        reads.packed.ctypes.data_as(_u8p),
    )


def kmer_hash(K: int, x: int) -> int:
    return int(lib().ork_hash(K, x))


def kmer_unhash(K: int, h: int) -> int:
    return int(lib().ork_unhash(K, h))


def extract_hashes(reads, K: int) -> np.ndarray:
    L = lib()
    n, bo, yo, pk = _rp(reads)
    m = int(L.ork_count_instances(n, bo, K))
    out = np.empty(max(m, 1), dtype=np.uint64)
    L.ork_extract_hashes(n, bo, yo, pk, K, out.ctypes.data_as(_u64p))
    return out[:m]


def kmer_count(reads, K: int):
    """(hashes, counts) in ascending hash order."""
    L = lib()
    n, bo, yo, pk = _rp(reads)
    hp, cp = _u64p(), _u32p()
    nd = int(L.ork_kmer_count(n, bo, yo, pk, K, C.byref(hp), C.byref(cp)))
    if nd == 2**64 - 1:
        raise MemoryError("oracle kmer_count allocation failed")
    try:
        h = np.ctypeslib.as_array(hp, shape=(nd,)).copy() if nd else np.zeros(0, np.uint64)
        c = np.ctypeslib.as_array(cp, shape=(nd,)).copy() if nd else np.zeros(0, np.uint32)
    finally:
        L.ork_free(C.cast(hp, C.c_void_p))
        L.ork_free(C.cast(cp, C.c_void_p))
    return h, c


def kmer_count_range(reads, K: int, lo: int, hi: int):
    """(hashes, counts) of the parcel lo <= hash < hi, ascending (the CPU
    side of the sampled full-size parity tests)."""
    L = lib()
    n, bo, yo, pk = _rp(reads)
    hp, cp = _u64p(), _u32p()
    nd = int(L.ork_kmer_count_range(n, bo, yo, pk, K, lo, hi, C.byref(hp), C.byref(cp)))
    if nd == 2**64 - 1:
        raise MemoryError("oracle kmer_count_range allocation failed")
    try:
        h = np.ctypeslib.as_array(hp, shape=(nd,)).copy() if nd else np.zeros(0, np.uint64)
        c = np.ctypeslib.as_array(cp, shape=(nd,)).copy() if nd else np.zeros(0, np.uint32)
    finally:
        L.ork_free(C.cast(hp, C.c_void_p))
        L.ork_free(C.cast(cp, C.c_void_p))
    return h, c


def set_threads(n: int) -> None:
    """OpenMP threads of the restatement's parallel loops (0: leave as is)."""
    lib().ork_set_threads(int(n))


def threads() -> int:
    return int(lib().ork_threads())


def spectrum_from_counts(counts: np.ndarray, hist_len: int) -> np.ndarray:
    hist = np.zeros(hist_len, dtype=np.uint64)
    c = np.ascontiguousarray(counts, dtype=np.uint32)
    lib().ork_spectrum(c.ctypes.data_as(_u32p), len(c), hist.ctypes.data_as(_u64p), hist_len)
    return hist


def kmer_spectrum(reads, K: int, hist_len: int = 1 << 16) -> np.ndarray:
    _, c = kmer_count(reads, K)
    return spectrum_from_counts(c, hist_len)


def kspec_estimate(hist) -> dict:
    """Genome-size estimate of a spectrum (ork_kspec_estimate)."""
    h = np.ascontiguousarray(hist, dtype=np.uint64)
    u = np.zeros(7, np.uint64)
    d = np.zeros(3, np.float64)
    lib().ork_kspec_estimate(h.ctypes.data_as(_u64p), len(h), u.ctypes.data_as(_u64p),
                             d.ctypes.data_as(C.POINTER(C.c_double)))
    names = ("valley", "peak", "genome_size", "genomic_kmers", "genomic_instances", "error_kmers", "error_instances")
    out = {k: int(x) for k, x in zip(names, u)}
    out.update(coverage=float(d[0]), repeat_fraction=float(d[1]), het_ratio=float(d[2]))
    return out


def precorrect(reads, K=24, min_solid=3, max_q=20, n_cycles=1, fast=False):
    """Corrected copy of `reads` (needs quals) and stats dict.
    fast=True: ork_precorrect_fast (bench.py's CPU baseline: rolling keys,
    hash-table solid lookups; same outputs)."""
    from allpathslg_amd.reads import ReadSet  # plain data container

    L = lib()
    if fast and not hasattr(L, "_ork_fast"):
        L.ork_precorrect_fast.restype = C.c_int
        L.ork_precorrect_fast.argtypes = L.ork_precorrect.argtypes
        L._ork_fast = True
    fn = L.ork_precorrect_fast if fast else L.ork_precorrect
    pk = reads.packed.copy()
    q = reads.quals.copy()
    st = np.zeros(5, dtype=np.uint64)
    rc = fn(reads.n_reads, reads.base_off.ctypes.data_as(_u64p), reads.byte_off.ctypes.data_as(_u64p),
                              pk.ctypes.data_as(_u8p), q.ctypes.data_as(_u8p), K, min_solid, max_q, n_cycles,
                              st.ctypes.data_as(_u64p))
    if rc:
        raise MemoryError("oracle precorrect failed")
    keys = ["n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"]
    return ReadSet(reads.base_off.copy(), reads.byte_off.copy(), pk, q), {k: int(v) for k, v in zip(keys, st)}


def precorrect_solid(reads, solid_hashes, K=24, max_q=20, fast=False):
    """One correction pass of `reads` against a given solid hash set
    (fast=True: rolling keys + hash table, same outputs; for full-size
    parity checks and the CPU baseline)."""
    from allpathslg_amd.reads import ReadSet

    L = lib()
    if fast and not hasattr(L, "_ork_sfast"):
        L.ork_precorrect_solid_fast.restype = C.c_int
        L.ork_precorrect_solid_fast.argtypes = L.ork_precorrect_solid.argtypes
        L._ork_sfast = True
    pk = reads.packed.copy()
    q = reads.quals.copy()
    st = np.zeros(5, dtype=np.uint64)
    sh = np.ascontiguousarray(solid_hashes, dtype=np.uint64)
    rc = (L.ork_precorrect_solid_fast if fast else L.ork_precorrect_solid)(reads.n_reads, reads.base_off.ctypes.data_as(_u64p),
                                    reads.byte_off.ctypes.data_as(_u64p), pk.ctypes.data_as(_u8p),
                                    q.ctypes.data_as(_u8p), K, max_q, sh.ctypes.data_as(_u64p), len(sh),
                                    st.ctypes.data_as(_u64p))
    if rc:
        raise MemoryError("oracle precorrect failed")
    keys = ["n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"]
    return ReadSet(reads.base_off.copy(), reads.byte_off.copy(), pk, q), {k: int(v) for k, v in zip(keys, st)}


FILL_STATUS = {0: "filled", 1: "none", 2: "ambiguous", 3: "budget", 4: "skip"}


def solid_hashes(reads, K: int = 24, min_solid: int = 3) -> np.ndarray:
    """Hashes of the canonical K-mers of `reads` seen >= min_solid times."""
    h, c = kmer_count(reads, K)
    return h[c >= min_solid]


def fill_fragments(reads, solid, K: int = 24, min_insert: int = 126, max_insert: int = 234,
                   max_steps: int = 1024, fast: bool = False):
    """FillFragments restated (oracle/fill_oracle.c): pairs (2i, 2i+1) closed
    through the solid K-mer set (fast=True: hash-table lookups, bench.py's
    CPU baseline; same outputs).  Returns (filled ReadSet in pair order,
    status uint8[n_pairs], length uint32[n_pairs], stats dict)."""
    from allpathslg_amd.reads import ReadSet

    L = lib()
    if not hasattr(L, "_orf"):
        L.orf_fill.restype = C.c_int
        L.orf_fill.argtypes = [C.c_uint64, _u64p, _u64p, _u8p, C.c_int, _u64p, C.c_uint64, C.c_uint32, C.c_uint32,
                               C.c_uint32, _u8p, _u32p, C.POINTER(_u8p), _u64p]
        L.orf_fill_fast.restype = C.c_int
        L.orf_fill_fast.argtypes = L.orf_fill.argtypes
        L._orf = True
    n, bo, yo, pk = _rp(reads)
    npairs = n // 2
    status = np.zeros(max(npairs, 1), np.uint8)
    flen = np.zeros(max(npairs, 1), np.uint32)
    st = np.zeros(7, np.uint64)
    sh = np.ascontiguousarray(solid, dtype=np.uint64)
    outp = _u8p()
    rc = (L.orf_fill_fast if fast else L.orf_fill)(n, bo, yo, pk, K, sh.ctypes.data_as(_u64p), len(sh), min_insert, max_insert, max_steps,
                    status.ctypes.data_as(_u8p), flen.ctypes.data_as(_u32p), C.byref(outp), st.ctypes.data_as(_u64p))
    if rc:
        raise RuntimeError("oracle fill_fragments failed (odd read count, bad K or allocation)")
    try:
        nb = int(st[5])
        codes = np.ctypeslib.as_array(outp, shape=(nb,)).copy() if nb else np.zeros(0, np.uint8)
    finally:
        L.ork_free(C.cast(outp, C.c_void_p))
    status, flen = status[:npairs], flen[:npairs]
    lens = flen[status == 0].astype(np.uint64)
    base_off = np.zeros(len(lens) + 1, np.uint64)
    base_off[1:] = np.cumsum(lens)
    byte_off = np.zeros(len(lens) + 1, np.uint64)
    byte_off[1:] = np.cumsum((lens + 3) // 4)
    packed = np.zeros(int(byte_off[-1]) + 64, np.uint8)
    for i in range(len(lens)):  # pack each fragment byte-aligned (numpy, small cases)
        a = codes[int(base_off[i]):int(base_off[i + 1])]
        a4 = np.concatenate([a, np.zeros((-len(a)) % 4, np.uint8)]).reshape(-1, 4)
        b = (a4[:, 0] | (a4[:, 1] << 2) | (a4[:, 2] << 4) | (a4[:, 3] << 6)).astype(np.uint8)
        packed[int(byte_off[i]):int(byte_off[i]) + len(b)] = b
    keys = ["n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip", "filled_bases", "lookups"]
    return ReadSet(base_off, byte_off, packed, None), status, flen, {k: int(v) for k, v in zip(keys, st)}


class _OruResult(C.Structure):
    _fields_ = [
        ("n_nodes", C.c_uint64),
        ("n_unipaths", C.c_uint64),
        ("len", _u64p),
        ("id_base", _u64p),
        ("rc", _u64p),
        ("ub_off", _u64p),
        ("unibases", _u8p),
        ("n_vertices", C.c_uint64),
        ("frm", _u64p),
        ("to", _u64p),
        ("n_reads", C.c_uint64),
        ("path_off", _u64p),
        ("n_intervals", C.c_uint64),
        ("path_start", _u64p),
        ("path_len", _u64p),
    ]


def _arr(p, n, dt):
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dt).copy() if n else np.zeros(0, dt)


def unipaths(reads, K: int = 96) -> dict:
    """The unipath graph of `reads` as numpy arrays."""
    L = lib()
    if not hasattr(L, "_oru"):
        L.oru_build.restype = C.c_int
        L.oru_build.argtypes = [C.c_uint64, _u64p, _u64p, _u8p, C.c_int, C.POINTER(_OruResult)]
        L.oru_free.restype = None
        L.oru_free.argtypes = [C.POINTER(_OruResult)]
        L._oru = True
    res = _OruResult()
    n, bo, yo, pk = _rp(reads)
    rc = L.oru_build(n, bo, yo, pk, K, C.byref(res))
    if rc:
        raise RuntimeError(f"oracle unipaths failed ({rc})")
    try:
        U = int(res.n_unipaths)
        out = {
            "n_nodes": int(res.n_nodes),
            "n_unipaths": U,
            "len": _arr(res.len, U, np.uint64),
            "id_base": _arr(res.id_base, U, np.uint64),
            "rc": _arr(res.rc, U, np.uint64),
            "ub_off": _arr(res.ub_off, U + 1, np.uint64),
            "n_vertices": int(res.n_vertices),
            "from": _arr(res.frm, U, np.uint64),
            "to": _arr(res.to, U, np.uint64),
            "path_off": _arr(res.path_off, int(res.n_reads) + 1, np.uint64),
            "path_start": _arr(res.path_start, int(res.n_intervals), np.uint64),
            "path_len": _arr(res.path_len, int(res.n_intervals), np.uint64),
        }
        out["unibases"] = _arr(res.unibases, int(out["ub_off"][-1]) if U else 0, np.uint8)
        return out
    finally:
        L.oru_free(C.byref(res))


def instances(reads, K: int = 96):
    """All K-mer instances: (keys [n,3] u64, ext [n] u8, hash [n] u64)."""
    L = lib()
    if not hasattr(L, "_oi"):
        L.oru_instances.restype = C.c_uint64
        L.oru_instances.argtypes = [C.c_uint64, _u64p, _u64p, _u8p, C.c_int, _u64p, _u8p, _u64p]
        L.oru_graph_from_nodes.restype = C.c_int
        L.oru_graph_from_nodes.argtypes = [C.c_uint64, _u64p, _u8p, C.c_uint64, _u64p, _u64p, _u8p, C.c_int,
                                           C.POINTER(_OruResult)]
        L._oi = True
    n, bo, yo, pk = _rp(reads)
    m = int(L.oru_instances(n, bo, yo, pk, K, None, None, None))
    keys = np.zeros((max(m, 1), 3), dtype=np.uint64)
    ext = np.zeros(max(m, 1), dtype=np.uint8)
    h = np.zeros(max(m, 1), dtype=np.uint64)
    L.oru_instances(n, bo, yo, pk, K, keys.ctypes.data_as(_u64p), ext.ctypes.data_as(_u8p), h.ctypes.data_as(_u64p))
    return keys[:m], ext[:m], h[:m]


def group_nodes(keys, ext):
    """Distinct keys with the OR of their instances' extension bits."""
    if len(keys) == 0:
        return np.zeros((0, 3), np.uint64), np.zeros(0, np.uint8)
    order = np.lexsort((keys[:, 2], keys[:, 1], keys[:, 0]))
    k = keys[order]
    e = ext[order]
    new = np.ones(len(k), dtype=bool)
    new[1:] = np.any(k[1:] != k[:-1], axis=1)
    gid = np.cumsum(new) - 1
    out_e = np.zeros(int(gid[-1]) + 1, dtype=np.uint8)
    np.bitwise_or.at(out_e, gid, e)
    return k[new], out_e


def graph_from_nodes(keys, ext, reads, K: int = 96) -> dict:
    instances(reads, K)  # binds the entry points
    L = lib()
    res = _OruResult()
    kk = np.ascontiguousarray(keys, dtype=np.uint64)
    ee = np.ascontiguousarray(ext, dtype=np.uint8)
    n, bo, yo, pk = _rp(reads)
    rc = L.oru_graph_from_nodes(len(ee), kk.ctypes.data_as(_u64p), ee.ctypes.data_as(_u8p), n, bo, yo, pk, K,
                                C.byref(res))
    if rc:
        raise RuntimeError(f"oracle graph_from_nodes failed ({rc})")
    try:
        U = int(res.n_unipaths)
        out = {
            "n_nodes": int(res.n_nodes), "n_unipaths": U,
            "len": _arr(res.len, U, np.uint64), "id_base": _arr(res.id_base, U, np.uint64),
            "rc": _arr(res.rc, U, np.uint64), "ub_off": _arr(res.ub_off, U + 1, np.uint64),
            "n_vertices": int(res.n_vertices), "from": _arr(res.frm, U, np.uint64), "to": _arr(res.to, U, np.uint64),
            "path_off": _arr(res.path_off, int(res.n_reads) + 1, np.uint64),
            "path_start": _arr(res.path_start, int(res.n_intervals), np.uint64),
            "path_len": _arr(res.path_len, int(res.n_intervals), np.uint64),
        }
        out["unibases"] = _arr(res.unibases, int(out["ub_off"][-1]) if U else 0, np.uint8)
        return out
    finally:
        L.oru_free(C.byref(res))


def _rs(reads):
    return (reads.base_off.ctypes.data_as(_u64p), reads.byte_off.ctypes.data_as(_u64p),
            reads.packed.ctypes.data_as(_u8p))


def _bind_align():
    L = lib()
    if not hasattr(L, "_al"):
        L.ora_gapfree.restype = None
        L.ora_gapfree.argtypes = [_u64p, _u64p, _u8p, _u8p, _u64p, _u64p, _u8p, _u32p, C.c_uint64, _u32p]
        L.ora_banded_sw.restype = None
        L.ora_banded_sw.argtypes = [_u64p, _u64p, _u8p, _u64p, _u64p, _u8p, _u32p, C.c_uint64, C.c_int,
                                    C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_uint32]
        L.ora_consensus.restype = None
        L.ora_consensus.argtypes = [_u64p, _u64p, _u8p, _u8p, _u64p, _u64p, _u8p, C.c_uint64, _u32p, C.c_uint64,
                                    _u8p, _u8p]
        L._al = True
    return L


def _pairs(pairs):
    return np.ascontiguousarray(np.asarray(pairs, dtype=np.int64).reshape(-1, 4).astype(np.int32).view(np.uint32))


def gapfree(S, T, pairs):
    """(n, 4) uint32 [overlap, mismatches, qsum, offset]."""
    L = _bind_align()
    p = _pairs(pairs)
    out = np.zeros((len(p), 4), dtype=np.uint32)
    sq = S.quals.ctypes.data_as(_u8p) if S.quals is not None else None
    L.ora_gapfree(*_rs(S), sq, *_rs(T), p.ctypes.data_as(_u32p), len(p), out.ctypes.data_as(_u32p))
    return out


def banded_sw(S, T, pairs, band_w, max_blocks=0):
    """((n, 8) int32 results, (n, max_blocks, 2) blocks or None)."""
    L = _bind_align()
    p = _pairs(pairs)
    res = np.zeros((len(p), 8), dtype=np.int32)
    blk = np.zeros((len(p), max_blocks, 2), dtype=np.int32) if max_blocks else None
    L.ora_banded_sw(*_rs(S), *_rs(T), p.ctypes.data_as(_u32p), len(p), band_w,
                    res.ctypes.data_as(C.POINTER(C.c_int32)),
                    blk.ctypes.data_as(C.POINTER(C.c_int32)) if blk is not None else None, max_blocks)
    return res, blk


def consensus(R, T, placements):
    """(bases, quals), one per base of T."""
    L = _bind_align()
    p = _pairs(placements)
    nt = T.n_bases
    b = np.zeros(max(nt, 1), dtype=np.uint8)
    q = np.zeros(max(nt, 1), dtype=np.uint8)
    L.ora_consensus(*_rs(R), R.quals.ctypes.data_as(_u8p), *_rs(T), T.n_reads, p.ctypes.data_as(_u32p), len(p),
                    b.ctypes.data_as(_u8p), q.ctypes.data_as(_u8p))
    return b[:nt], q[:nt]


def make_rc_db(g):
    """MakeRcDb restated in numpy / python loops (small cases): rc paths and
    the stable start-sorted index of fw then rc intervals (include/apg.h)."""
    ub = np.asarray(g["id_base"], np.int64)
    ul = np.asarray(g["len"], np.int64)
    urc = np.asarray(g["rc"], np.int64)
    off = np.asarray(g["path_off"], np.int64)
    ps = np.asarray(g["path_start"], np.int64)
    pl = np.asarray(g["path_len"], np.int64)
    R = len(off) - 1
    rc_off, rc_s, rc_l = [0], [], []
    for r in range(R):
        ids = []
        for q in range(off[r], off[r + 1]):
            ids.extend(range(ps[q], ps[q] + pl[q]))
        mapped = []
        for x in reversed(ids):
            u = int(np.searchsorted(ub, x, side="right") - 1)
            mapped.append(ub[urc[u]] + ul[u] - 1 - (x - ub[u]))
        for x in mapped:
            if rc_l and len(rc_s) > rc_off[-1] and rc_s[-1] + rc_l[-1] == x:
                rc_l[-1] += 1
            else:
                rc_s.append(x)
                rc_l.append(1)
        rc_off.append(len(rc_s))
    ent = []
    for r in range(R):
        for q in range(off[r], off[r + 1]):
            ent.append((ps[q], pl[q], r, q - off[r], 0))
    for r in range(R):
        for q in range(rc_off[r], rc_off[r + 1]):
            ent.append((rc_s[q], rc_l[q], r, q - rc_off[r], 1))
    order = sorted(range(len(ent)), key=lambda i: ent[i][0])  # stable
    from allpathslg_amd.engine import RPINT_DTYPE

    arr = np.array([ent[i] for i in order], dtype=RPINT_DTYPE) if ent else np.zeros(0, RPINT_DTYPE)
    return {"rc_path_off": np.array(rc_off, np.uint64), "rc_start": np.array(rc_s, np.uint64),
            "rc_len": np.array(rc_l, np.uint64), "entries": arr}


def unipath_locs(g: dict, reads, K: int = 96, rc: bool = True, sorted: bool = True):
    """UnipathLocs restated (oracle/locs_oracle.c): placements of `reads` on
    graph `g` (dict as returned by unipaths()).  Returns ((n, 4) int32
    [read, unipath, start, flags], {"n_placed", "n_missing"})."""
    L = lib()
    if not hasattr(L, "_orl"):
        L.orl_locs.restype = C.c_int
        L.orl_locs.argtypes = [C.c_uint64, _u64p, _u64p, _u64p, _u8p, C.c_int, C.c_uint64, _u64p, _u64p, _u8p,
                               C.c_uint32, C.POINTER(_u32p), _u64p, _u64p]
        L._orl = True
    U = int(g["n_unipaths"])
    ulen = np.ascontiguousarray(g["len"], dtype=np.uint64)
    urc = np.ascontiguousarray(g["rc"], dtype=np.uint64)
    uoff = np.ascontiguousarray(g["ub_off"], dtype=np.uint64)
    ub = np.ascontiguousarray(g["unibases"], dtype=np.uint8)
    if ub.size == 0:
        ub = np.zeros(1, np.uint8)
    out = _u32p()
    n = C.c_uint64(0)
    stats = np.zeros(2, dtype=np.uint64)
    flags = (1 if rc else 0) | (2 if sorted else 0)
    rn, bo, yo, pk = _rp(reads)
    rcode = L.orl_locs(U, ulen.ctypes.data_as(_u64p), urc.ctypes.data_as(_u64p), uoff.ctypes.data_as(_u64p),
                       ub.ctypes.data_as(_u8p), K, rn, bo, yo, pk, flags, C.byref(out), C.byref(n),
                       stats.ctypes.data_as(_u64p))
    if rcode:
        raise RuntimeError(f"oracle unipath_locs failed ({rcode})")
    try:
        k = int(n.value)
        res = np.ctypeslib.as_array(out, shape=(4 * k,)).view(np.int32).reshape(k, 4).copy() if k else \
            np.zeros((0, 4), np.int32)
    finally:
        L.ork_free(out)
    return res, {"n_placed": int(stats[0]), "n_missing": int(stats[1])}


def error_correct_jump(frags, jumps, K: int = 24, min_solid: int = 3, max_q: int = 20, min_keep: int = 40):
    """ErrorCorrectJump restated: the fragment reads' solid set, one PreCorrect
    pass of the jump reads against it, prefix trimming (oracle/ecj_oracle.c).
    Returns (corrected jumps ReadSet (untrimmed layout), keep u32[n], pc stats)."""
    L = lib()
    if not hasattr(L, "_oje"):
        L.oje_trim.restype = None
        L.oje_trim.argtypes = [C.c_uint64, _u64p, _u64p, _u8p, C.c_int, _u64p, C.c_uint64, C.c_uint32, _u32p]
        L._oje = True
    solid = np.sort(solid_hashes(frags, K, min_solid)).astype(np.uint64)
    return error_correct_jump_solid(jumps, solid, K, max_q, min_keep)


def error_correct_jump_solid(jumps, solid, K: int = 24, max_q: int = 20, min_keep: int = 40, fast: bool = False):
    """error_correct_jump against a given solid hash set (e.g. the GPU's
    frag-read set, itself checked against kmer_count_range parcels).
    fast=True: the correction pass in precorrect_solid's rolling-key form
    (same outputs; full-size inputs)."""
    L = lib()
    if not hasattr(L, "_oje"):
        L.oje_trim.restype = None
        L.oje_trim.argtypes = [C.c_uint64, _u64p, _u64p, _u8p, C.c_int, _u64p, C.c_uint64, C.c_uint32, _u32p]
        L._oje = True
    solid = np.sort(np.ascontiguousarray(solid, dtype=np.uint64))
    fixed, st = precorrect_solid(jumps, solid, K, max_q, fast=fast) if fast else precorrect_solid(jumps, solid, K, max_q)
    keep = np.zeros(max(fixed.n_reads, 1), dtype=np.uint32)
    n, bo, yo, pk = _rp(fixed)
    L.oje_trim(n, bo, yo, pk, K, solid.ctypes.data_as(_u64p), len(solid), min_keep, keep.ctypes.data_as(_u32p))
    return fixed, keep[: fixed.n_reads], st


def unipath_coverage(g: dict, locs: np.ndarray, min_len: int = 500):
    """UnipathCoverage restated (oracle/ucov_oracle.c): placements per
    unipath, per K-mer, genome-wide coverage c0 and copy numbers on graph
    `g` from (n, 4) int32 placements [read, unipath, start, flags].
    Returns {"counts", "cov", "cn", "c0", "n_long"}."""
    L = lib()
    if not hasattr(L, "_ouc"):
        L.ouc_coverage.restype = C.c_int
        L.ouc_coverage.argtypes = [C.c_uint64, _u64p, _u32p, C.c_uint64, C.c_uint64, _u64p,
                                   C.POINTER(C.c_double), _u32p, C.POINTER(C.c_double), _u64p]
        L._ouc = True
    U = int(g["n_unipaths"])
    ulen = np.ascontiguousarray(g["len"], dtype=np.uint64)
    pairs = np.ascontiguousarray(locs, dtype=np.int32).view(np.uint32).reshape(-1)
    if pairs.size == 0:
        pairs = np.zeros(4, np.uint32)
    n = len(locs)
    counts = np.zeros(max(U, 1), np.uint64)
    cov = np.zeros(max(U, 1), np.float64)
    cn = np.zeros(max(U, 1), np.uint32)
    c0 = C.c_double(0)
    nl = C.c_uint64(0)
    rc = L.ouc_coverage(U, ulen.ctypes.data_as(_u64p), pairs.ctypes.data_as(_u32p), n, min_len,
                        counts.ctypes.data_as(_u64p), cov.ctypes.data_as(C.POINTER(C.c_double)),
                        cn.ctypes.data_as(_u32p), C.byref(c0), C.byref(nl))
    if rc:
        raise RuntimeError(f"oracle unipath_coverage failed ({rc})")
    return {"counts": counts[:U], "cov": cov[:U], "cn": cn[:U], "c0": c0.value, "n_long": int(nl.value)}
