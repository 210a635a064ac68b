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
        L.ork_spectrum.restype = None
        L.ork_spectrum.argtypes = [_u32p, C.c_uint64, _u64p, C.c_uint64]
        L.ork_precorrect.restype = C.c_int
        L.ork_precorrect.argtypes = [C.c_uint64, _u64p, _u64p, _u8p, _u8p, C.c_int, C.c_uint32, C.c_uint32,
                                     C.c_uint32, _u64p]
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


def spectrum_from_counts(counts: np.ndarray, hist_len: int) -> np.ndarray:
    hist = np.zeros(hist_len, dtype=np.uint64)
    c = np.ascontiguousarray(counts, dtype=np.uint32)
    lib().ork_spectrum(c.ctypes.data_as(_u32p), len(c), hist.ctypes.data_as(_u64p), hist_len)
    return hist


def kmer_spectrum(reads, K: int, hist_len: int = 1 << 16) -> np.ndarray:
    _, c = kmer_count(reads, K)
    return spectrum_from_counts(c, hist_len)


def precorrect(reads, K=24, min_solid=3, max_q=20, n_cycles=1):
    """Corrected copy of `reads` (needs quals) and stats dict."""
    from allpathslg_amd.reads import ReadSet  # plain data container

    pk = reads.packed.copy()
    q = reads.quals.copy()
    st = np.zeros(5, dtype=np.uint64)
    rc = lib().ork_precorrect(reads.n_reads, reads.base_off.ctypes.data_as(_u64p), reads.byte_off.ctypes.data_as(_u64p),
                              pk.ctypes.data_as(_u8p), q.ctypes.data_as(_u8p), K, min_solid, max_q, n_cycles,
                              st.ctypes.data_as(_u64p))
    if rc:
        raise MemoryError("oracle precorrect failed")
    keys = ["n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"]
    return ReadSet(reads.base_off.copy(), reads.byte_off.copy(), pk, q), {k: int(v) for k, v in zip(keys, st)}
