"""Read sets: the in-memory form of vecbasevector/vecqualvector ([R:M]
src/Basevector.h, src/Qualvector.h) backed by numpy arrays, plus the
synthetic generator and .fastb/.qualb I/O — all through libapg.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

from ._lib import apg_reads, apg_synth_params, check, lib

_u64p = C.POINTER(C.c_uint64)
_u8p = C.POINTER(C.c_uint8)


def _ptr(a: Optional[np.ndarray], t):
    if a is None:
        return C.cast(None, C.POINTER(t))
    return a.ctypes.data_as(C.POINTER(t))


@dataclass
class ReadSet:
    """2-bit packed reads (A=0 C=1 G=2 T=3, 4 bases/byte LSB-first, each read
    byte-aligned) with optional Phred qualities."""

    base_off: np.ndarray  # uint64[n+1]
    byte_off: np.ndarray  # uint64[n+1]
    packed: np.ndarray  # uint8[byte_off[n] (+ slack)]
    quals: Optional[np.ndarray] = None  # uint8[base_off[n]]

    def __post_init__(self):
        self.base_off = np.ascontiguousarray(self.base_off, dtype=np.uint64)
        self.byte_off = np.ascontiguousarray(self.byte_off, dtype=np.uint64)
        self.packed = np.ascontiguousarray(self.packed, dtype=np.uint8)
        if self.quals is not None:
            self.quals = np.ascontiguousarray(self.quals, dtype=np.uint8)

    @property
    def n_reads(self) -> int:
        return len(self.base_off) - 1

    @property
    def n_bases(self) -> int:
        return int(self.base_off[-1] - self.base_off[0])

    def lengths(self) -> np.ndarray:
        return np.diff(self.base_off)

    def c_struct(self) -> apg_reads:
        r = apg_reads()
        r.n_reads = self.n_reads
        r.base_off = _ptr(self.base_off, C.c_uint64)
        r.byte_off = _ptr(self.byte_off, C.c_uint64)
        r.packed = _ptr(self.packed, C.c_uint8)
        r.quals = _ptr(self.quals, C.c_uint8)
        return r

    # -- conversions -------------------------------------------------------
    @classmethod
    def from_sequences(cls, seqs: Sequence[Sequence[int]], quals: Optional[Sequence[Sequence[int]]] = None):
        """Build from per-read base codes (0..3)."""
        lens = np.array([len(s) for s in seqs], dtype=np.uint64)
        base_off = np.zeros(len(seqs) + 1, dtype=np.uint64)
        base_off[1:] = np.cumsum(lens)
        byte_off = np.zeros(len(seqs) + 1, dtype=np.uint64)
        byte_off[1:] = np.cumsum((lens + 3) // 4)
        packed = np.zeros(int(byte_off[-1]) + 64, dtype=np.uint8)
        for i, s in enumerate(seqs):
            a = np.asarray(s, dtype=np.uint8)
            if a.size and a.max() > 3:
                raise ValueError("base codes must be 0..3")
            pad = (-len(a)) % 4
            a4 = np.concatenate([a, np.zeros(pad, np.uint8)]).reshape(-1, 4)
            b = (a4[:, 0] | (a4[:, 1] << 2) | (a4[:, 2] << 4) | (a4[:, 3] << 6)).astype(np.uint8)
            packed[int(byte_off[i]) : int(byte_off[i]) + len(b)] = b
        q = None
        if quals is not None:
            q = np.concatenate([np.asarray(x, dtype=np.uint8) for x in quals]) if len(quals) else np.zeros(0, np.uint8)
        return cls(base_off, byte_off, packed, q)

    @classmethod
    def from_matrix(cls, bases: np.ndarray, quals: Optional[np.ndarray] = None):
        """Build from an (n, L) matrix of base codes (equal-length reads),
        vectorised; quals (n, L) uint8 or None."""
        b = np.ascontiguousarray(bases, dtype=np.uint8)
        n, L = b.shape
        pad = (-L) % 4
        if pad:
            b = np.concatenate([b, np.zeros((n, pad), np.uint8)], axis=1)
        packed = np.zeros(n * ((L + 3) // 4) + 64, dtype=np.uint8)
        packed[: n * ((L + 3) // 4)] = (b[:, 0::4] | (b[:, 1::4] << 2) | (b[:, 2::4] << 4) | (b[:, 3::4] << 6)).reshape(-1)
        base_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(L)
        byte_off = np.arange(n + 1, dtype=np.uint64) * np.uint64((L + 3) // 4)
        q = None if quals is None else np.ascontiguousarray(quals, dtype=np.uint8).reshape(-1)
        return cls(base_off, byte_off, packed, q)

    @classmethod
    def from_strings(cls, seqs: Sequence[str]):
        code = {"A": 0, "C": 1, "G": 2, "T": 3, "N": 0}
        return cls.from_sequences([[code[c] for c in s.upper()] for s in seqs])

    def read(self, i: int) -> np.ndarray:
        """Base codes of read i."""
        n = int(self.base_off[i + 1] - self.base_off[i])
        b0 = int(self.byte_off[i])
        raw = self.packed[b0 : b0 + (n + 3) // 4]
        out = np.stack([(raw >> s) & 3 for s in (0, 2, 4, 6)], axis=1).reshape(-1)[:n]
        return out.astype(np.uint8)

    def subset(self, start: int, stop: int) -> "ReadSet":
        """Reads [start, stop) as a standalone set (copies)."""
        bo = self.base_off[start : stop + 1] - self.base_off[start]
        yo = self.byte_off[start : stop + 1] - self.byte_off[start]
        pk = np.zeros(int(yo[-1]) + 64, dtype=np.uint8)
        pk[: int(yo[-1])] = self.packed[int(self.byte_off[start]) : int(self.byte_off[stop])]
        q = None
        if self.quals is not None:
            q = self.quals[int(self.base_off[start]) : int(self.base_off[stop])].copy()
        return ReadSet(bo, yo, pk, q)

    # -- files -------------------------------------------------------------
    def write_fastb(self, path: str) -> None:
        r = self.c_struct()
        check(lib().apg_fastb_write(path.encode(), C.byref(r)), "apg_fastb_write")

    def write_qualb(self, path: str) -> None:
        if self.quals is None:
            raise ValueError("read set has no qualities")
        r = self.c_struct()
        check(lib().apg_qualb_write(path.encode(), C.byref(r)), "apg_qualb_write")

    @classmethod
    def load(cls, fastb: str, qualb: Optional[str] = None) -> "ReadSet":
        r = apg_reads()
        L = lib()
        check(L.apg_fastb_read(fastb.encode(), C.byref(r)), "apg_fastb_read")
        try:
            if qualb:
                check(L.apg_qualb_read(qualb.encode(), C.byref(r)), "apg_qualb_read")
            n = int(r.n_reads)
            bo = np.ctypeslib.as_array(r.base_off, shape=(n + 1,)).copy()
            yo = np.ctypeslib.as_array(r.byte_off, shape=(n + 1,)).copy()
            nb = int(yo[-1])
            pk = np.zeros(nb + 64, dtype=np.uint8)
            if nb:
                pk[:nb] = np.ctypeslib.as_array(r.packed, shape=(nb,))
            q = None
            if qualb:
                nq = int(bo[-1])
                q = np.ctypeslib.as_array(r.quals, shape=(nq,)).copy() if nq else np.zeros(0, np.uint8)
            return cls(bo, yo, pk, q)
        finally:
            L.apg_reads_release(C.byref(r))


def synth_genome(length: int, seed: int, repeats=None) -> np.ndarray:
    """Uniform iid genome; repeats=True injects apg_repeat_defaults' human-like
    mix (include/apg.h apg_synth_repeats), or pass a dict of
    apg_repeat_params fields to override it."""
    g = np.empty(length, dtype=np.uint8)
    check(lib().apg_synth_genome(length, seed, _ptr(g, C.c_uint8)), "apg_synth_genome")
    if repeats:
        from ._lib import apg_repeat_params

        p = apg_repeat_params()
        lib().apg_repeat_defaults(C.byref(p))
        if isinstance(repeats, dict):
            for k, v in repeats.items():
                if isinstance(v, (list, tuple)):
                    arr = getattr(p, k)
                    for i, x in enumerate(v):
                        arr[i] = x
                else:
                    setattr(p, k, v)
        check(lib().apg_synth_repeats(length, seed, C.byref(p), _ptr(g, C.c_uint8)), "apg_synth_repeats")
    return g


def synth_reads(
    genome: np.ndarray,
    n_pairs: int,
    seed: int,
    read_len: int = 100,
    insert_mean: int = 180,
    insert_sd: int = 18,
    err_lo: float = 0.002,
    err_hi: float = 0.02,
    first_pair: int = 0,
    threads: int = 0,
    with_quals: bool = True,
) -> ReadSet:
    """Paired frag reads from `genome`: reads 2i, 2i+1 are mates."""
    p = apg_synth_params()
    p.genome_len = len(genome)
    p.seed = seed
    p.n_pairs = n_pairs
    p.read_len = read_len
    p.insert_mean = insert_mean
    p.insert_sd = insert_sd
    p.threads = threads
    p.err_lo = err_lo
    p.err_hi = err_hi
    p.first_pair = first_pair
    nr, nb, npk = C.c_uint64(), C.c_uint64(), C.c_uint64()
    L = lib()
    check(L.apg_synth_sizes(C.byref(p), C.byref(nr), C.byref(nb), C.byref(npk)), "apg_synth_sizes")
    base_off = np.empty(nr.value + 1, dtype=np.uint64)
    byte_off = np.empty(nr.value + 1, dtype=np.uint64)
    packed = np.zeros(npk.value + 64, dtype=np.uint8)
    quals = np.empty(nb.value, dtype=np.uint8) if with_quals else None
    g = np.ascontiguousarray(genome, dtype=np.uint8)
    check(
        L.apg_synth_reads(
            C.byref(p),
            _ptr(g, C.c_uint8),
            _ptr(base_off, C.c_uint64),
            _ptr(byte_off, C.c_uint64),
            _ptr(packed, C.c_uint8),
            _ptr(quals, C.c_uint8),
        ),
        "apg_synth_reads",
    )
    return ReadSet(base_off, byte_off, packed, quals)


def synth_layout(genome_len: int, n_pairs: int, seed: int, read_len: int = 100, insert_mean: int = 180,
                 insert_sd: int = 18, first_pair: int = 0, threads: int = 0):
    """Simulator truth of synth_reads' pairs: (start u64[n], flen u32[n],
    flip u8[n]) — each fragment's genome interval and strand."""
    p = apg_synth_params()
    p.genome_len = genome_len
    p.seed = seed
    p.n_pairs = n_pairs
    p.read_len = read_len
    p.insert_mean = insert_mean
    p.insert_sd = insert_sd
    p.threads = threads
    p.first_pair = first_pair
    start = np.empty(max(n_pairs, 1), dtype=np.uint64)
    flen = np.empty(max(n_pairs, 1), dtype=np.uint32)
    flip = np.empty(max(n_pairs, 1), dtype=np.uint8)
    check(lib().apg_synth_layout(C.byref(p), _ptr(start, C.c_uint64), _ptr(flen, C.c_uint32), _ptr(flip, C.c_uint8)),
          "apg_synth_layout")
    return start[:n_pairs], flen[:n_pairs], flip[:n_pairs]


def synth_fragments(
    genome: np.ndarray,
    n_pairs: int,
    seed: int,
    read_len: int = 100,
    insert_mean: int = 180,
    insert_sd: int = 18,
    first_pair: int = 0,
    threads: int = 0,
) -> ReadSet:
    """The error-free insert of each pair synth_reads(genome, n_pairs, seed, ...)
    generates, in read A's orientation — the "oracle fill" that stands in for
    FillFragments as K=96 unipath input.  No qualities."""
    p = apg_synth_params()
    p.genome_len = len(genome)
    p.seed = seed
    p.n_pairs = n_pairs
    p.read_len = read_len
    p.insert_mean = insert_mean
    p.insert_sd = insert_sd
    p.threads = threads
    p.first_pair = first_pair
    L = lib()
    base_off = np.empty(n_pairs + 1, dtype=np.uint64)
    byte_off = np.empty(n_pairs + 1, dtype=np.uint64)
    check(L.apg_synth_fragments(C.byref(p), _ptr(base_off, C.c_uint64), _ptr(byte_off, C.c_uint64), None, None),
          "apg_synth_fragments")
    packed = np.zeros(int(byte_off[-1]) + 64, dtype=np.uint8)
    g = np.ascontiguousarray(genome, dtype=np.uint8)
    check(L.apg_synth_fragments(C.byref(p), _ptr(base_off, C.c_uint64), _ptr(byte_off, C.c_uint64),
                                _ptr(g, C.c_uint8), _ptr(packed, C.c_uint8)), "apg_synth_fragments")
    return ReadSet(base_off, byte_off, packed, None)
