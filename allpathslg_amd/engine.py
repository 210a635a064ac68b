"""Python face of libapg: a device context and the k-mer operations.

Mirrors the reference's module operations ([R:M] KmerSpectrum / naif_kmerize /
KernelKmerStorer): same argument meaning (K, histogram length), same error
behaviour (an exception where the module would FatalErr and exit non-zero).
All compute runs in libapg's HIP kernels; nothing here computes k-mers.
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, Optional, Tuple

import numpy as np

from ._lib import apg_config, apg_kstats, apg_pc_params, apg_pc_stats, check, lib
from .reads import ReadSet

_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)

DEFAULT_HIST_LEN = 1 << 16  # bins 0..65535, last bin = count >= 65535


def kmer_hash(K: int, canonical: int) -> int:
    return int(lib().apg_kmer_hash(K, canonical))


def kmer_unhash(K: int, h: int) -> int:
    return int(lib().apg_kmer_unhash(K, h))


def shard_bins(K: int, n_shards: int) -> int:
    b = lib().apg_shard_bins(K, n_shards)
    check(0 if b > 0 else b, "apg_shard_bins")
    return int(b)


class DeviceReads:
    """A read set resident in HBM (apg_dreads)."""

    def __init__(self, ctx: "Context", reads: Optional[ReadSet]):
        self.ctx = ctx
        self.reads = reads
        self._h = C.c_void_p()
        if reads is None:  # filled in by a device-side producer (apg_fill_fragments_dev)
            return
        r = reads.c_struct()
        check(lib().apg_reads_upload(ctx.handle, C.byref(r), C.byref(self._h)), "apg_reads_upload")

    @property
    def n_reads(self) -> int:
        return int(lib().apg_dreads_count(self._h)) if self._h else 0

    @property
    def n_bases(self) -> int:
        if not self._h:
            return 0
        nr, nb, ny = C.c_uint64(), C.c_uint64(), C.c_uint64()
        check(lib().apg_dreads_shape(self.ctx.handle, self._h, C.byref(nr), C.byref(nb), C.byref(ny), None, None),
              "apg_dreads_shape")
        return int(nb.value)

    @property
    def handle(self):
        return self._h

    def free(self):
        if self._h:
            lib().apg_reads_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class Context:
    """One HIP device + stream (apg_ctx).  One per host thread."""

    def __init__(self, device: int = 0, timing: bool = False, verbose: bool = False, kmer_dedup: int = 0):
        cfg = apg_config()
        cfg.device = device
        cfg.timing = int(timing)
        cfg.verbose = int(verbose)
        cfg.kmer_dedup = int(kmer_dedup)
        self._h = C.c_void_p()
        check(lib().apg_create(C.byref(cfg), C.byref(self._h)), "apg_create")
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            lib().apg_destroy(self._h)
            self._h = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- timing ------------------------------------------------------------
    def kernel_times(self) -> Dict[str, Tuple[float, int, int]]:
        """name -> (total_ms, launches, algorithmic_bytes)."""
        out = {}
        L = lib()
        i = 0
        name = C.create_string_buffer(128)
        ms, n, b = C.c_double(), C.c_uint64(), C.c_uint64()
        while L.apg_timing_get(self._h, i, name, 128, C.byref(ms), C.byref(n), C.byref(b)) == 0:
            out[name.value.decode()] = (ms.value, int(n.value), int(b.value))
            i += 1
        return out

    def overlapped_kernels(self) -> Dict[str, int]:
        """name -> launches that ran on the side / auxiliary stream (beside the
        main stream's kernels, so their event time is not a standalone time)."""
        out = {}
        L = lib()
        i = 0
        name = C.create_string_buffer(128)
        ov = C.c_uint64()
        while L.apg_timing_get(self._h, i, name, 128, None, None, None) == 0:
            check(L.apg_timing_overlapped(self._h, i, C.byref(ov)), "apg_timing_overlapped")
            if ov.value:
                out[name.value.decode()] = int(ov.value)
            i += 1
        return out

    def mem_stats(self, reset_peak: bool = False) -> dict:
        """Device memory of the context (include/apg.h apg_mem_stats_get)."""
        from ._lib import apg_mem_stats

        m = apg_mem_stats()
        check(lib().apg_mem_stats_get(self._h, 1 if reset_peak else 0, C.byref(m)), "apg_mem_stats_get")
        return m.as_dict()

    def reset_timing(self):
        check(lib().apg_timing_reset(self._h), "apg_timing_reset")

    def trim(self):
        check(lib().apg_trim(self._h), "apg_trim")

    # -- k-mers --------------------------------------------------------------
    def upload(self, reads: ReadSet) -> DeviceReads:
        return DeviceReads(self, reads)

    def load_reads(self, fastb: str, qualb: Optional[str] = None, threads: int = 0) -> DeviceReads:
        """.fastb (+ .qualb) files straight into HBM (apg_reads_load_dev):
        the same device read set as upload(ReadSet.load(fastb, qualb))."""
        d = DeviceReads(self, None)
        check(lib().apg_reads_load_dev(self._h, fastb.encode(), qualb.encode() if qualb else None, int(threads),
                                       C.byref(d._h)), "apg_reads_load_dev")
        return d

    def kmer_spectrum(self, reads, K: int, hist_len: int = DEFAULT_HIST_LEN):
        """Spectrum h[m] of canonical K-mers (K <= 32).  `reads` is a ReadSet
        (host; includes H2D) or DeviceReads (HBM-resident).  Returns
        (hist, stats)."""
        hist = np.zeros(hist_len, dtype=np.uint64)
        st = apg_kstats()
        L = lib()
        if isinstance(reads, DeviceReads):
            rc = L.apg_kmer_spectrum_dev(self._h, reads.handle, K, hist.ctypes.data_as(_u64p), hist_len, C.byref(st))
        else:
            r = reads.c_struct()
            rc = L.apg_kmer_spectrum(self._h, C.byref(r), K, hist.ctypes.data_as(_u64p), hist_len, C.byref(st))
        check(rc, "apg_kmer_spectrum")
        return hist, st.as_dict()

    def kmer_count(self, reads, K: int, hash_range: Optional[Tuple[int, int]] = None):
        """(keys, counts, stats): distinct canonical K-mers in ascending
        kmer_hash order and their multiplicities.  `reads`: ReadSet (host) or
        DeviceReads; hash_range=(lo, hi): only the parcel lo <= hash < hi
        (hi = 0: no upper bound; device reads only)."""
        L = lib()
        kp, cp = _u64p(), _u32p()
        nd = C.c_uint64()
        st = apg_kstats()
        if isinstance(reads, DeviceReads):
            lo, hi = hash_range if hash_range is not None else (0, 0)
            check(L.apg_kmer_count_dev(self._h, reads.handle, K, lo, hi, C.byref(kp), C.byref(cp), C.byref(nd),
                                       C.byref(st)), "apg_kmer_count_dev")
        else:
            if hash_range is not None:
                raise ValueError("hash_range needs a DeviceReads input")
            r = reads.c_struct()
            check(L.apg_kmer_count(self._h, C.byref(r), K, C.byref(kp), C.byref(cp), C.byref(nd), C.byref(st)),
                  "apg_kmer_count")
        try:
            n = int(nd.value)
            keys = np.ctypeslib.as_array(kp, shape=(n,)).copy() if n else np.zeros(0, np.uint64)
            counts = np.ctypeslib.as_array(cp, shape=(n,)).copy() if n else np.zeros(0, np.uint32)
        finally:
            L.apg_free(C.cast(kp, C.c_void_p))
            L.apg_free(C.cast(cp, C.c_void_p))
        return keys, counts, st.as_dict()

    # -- error correction ------------------------------------------------------
    @staticmethod
    def pc_params(K: int = 24, min_solid: int = 3, max_q_suspect: int = 20, n_cycles: int = 1) -> apg_pc_params:
        p = apg_pc_params()
        lib().apg_pc_defaults(C.byref(p))
        p.K, p.min_solid, p.max_q_suspect, p.n_cycles = K, min_solid, max_q_suspect, n_cycles
        return p

    def precorrect(self, reads, K: int = 24, min_solid: int = 3, max_q_suspect: int = 20, n_cycles: int = 1):
        """PreCorrect (n_cycles=1) / FindErrors (n_cycles=2), SURVEY §A.4.
        ReadSet -> (corrected ReadSet, stats); DeviceReads -> corrected in
        place, returns (same DeviceReads, stats)."""
        p = self.pc_params(K, min_solid, max_q_suspect, n_cycles)
        st = apg_pc_stats()
        if isinstance(reads, DeviceReads):
            check(lib().apg_precorrect_dev(self._h, reads.handle, C.byref(p), C.byref(st)), "apg_precorrect_dev")
            return reads, st.as_dict()
        if reads.quals is None:
            raise ValueError("precorrect needs qualities")
        pk = reads.packed.copy()
        q = reads.quals.copy()
        r = reads.c_struct()
        check(lib().apg_precorrect(self._h, C.byref(r), C.byref(p), pk.ctypes.data_as(C.POINTER(C.c_uint8)),
                                   q.ctypes.data_as(C.POINTER(C.c_uint8)), C.byref(st)), "apg_precorrect")
        return ReadSet(reads.base_off.copy(), reads.byte_off.copy(), pk, q), st.as_dict()

    def spectrum_precorrect(self, dreads: DeviceReads, K_spec: int = 25, K: int = 24, min_solid: int = 3,
                            max_q_suspect: int = 20, n_cycles: int = 1, hist_len: int = DEFAULT_HIST_LEN):
        """KmerSpectrum at K_spec, then PreCorrect at K, of one device read
        set in one counting pass (apg_spectrum_precorrect_dev; the same
        results as kmer_spectrum + precorrect).  Returns (hist, spectrum
        stats, correction stats); the reads are corrected in place."""
        p = self.pc_params(K, min_solid, max_q_suspect, n_cycles)
        hist = np.zeros(hist_len, dtype=np.uint64)
        ks, ps = apg_kstats(), apg_pc_stats()
        check(lib().apg_spectrum_precorrect_dev(self._h, dreads.handle, K_spec, hist.ctypes.data_as(_u64p), hist_len,
                                                C.byref(ks), C.byref(p), C.byref(ps)), "apg_spectrum_precorrect_dev")
        return hist, ks.as_dict(), ps.as_dict()

    def spectrum_precorrect_fill(self, dreads: DeviceReads, K_spec: int = 25, K: int = 24, min_solid: int = 3,
                                 max_q_suspect: int = 20, hist_len: int = DEFAULT_HIST_LEN, min_insert: int = 126,
                                 max_insert: int = 234, max_steps: int = 1024, out: Optional[DeviceReads] = None,
                                 d_status: Optional[int] = None):
        """spectrum_precorrect, then fill_fragments of the corrected pairs
        against the pass's solid set, in one call
        (apg_spectrum_precorrect_fill_dev: the fused K+1 count also runs
        beside FillFragments).  Returns (hist, spectrum stats, correction
        stats, filled DeviceReads (reusing `out`), fill stats)."""
        from ._lib import apg_fill_stats

        p = self.pc_params(K, min_solid, max_q_suspect, 1)
        fp = self.fill_params(K, min_insert, max_insert, max_steps, min_solid, True)
        hist = np.zeros(hist_len, dtype=np.uint64)
        ks, ps, fs = apg_kstats(), apg_pc_stats(), apg_fill_stats()
        fd = out if out is not None else DeviceReads(self, None)
        check(lib().apg_spectrum_precorrect_fill_dev(self._h, dreads.handle, K_spec, hist.ctypes.data_as(_u64p),
                                                     hist_len, C.byref(ks), C.byref(p), C.byref(ps), C.byref(fp),
                                                     C.byref(fd._h), C.c_void_p(d_status) if d_status else None,
                                                     C.byref(fs)), "apg_spectrum_precorrect_fill_dev")
        return hist, ks.as_dict(), ps.as_dict(), fd, fs.as_dict()

    def copy_reads(self, dst: DeviceReads, src: DeviceReads) -> None:
        """dst := src (device-to-device; same read lengths)."""
        check(lib().apg_reads_copy_dev(self._h, dst.handle, src.handle), "apg_reads_copy_dev")

    def concat_reads(self, sets, keeps=None, out: Optional[DeviceReads] = None) -> DeviceReads:
        """all_reads: the device read sets concatenated in order, set s's reads
        truncated to the device u32 keep lengths keeps[s] (a device pointer or
        None) — include/apg.h apg_reads_concat_dev.  `out`: an earlier result
        to reuse (its buffers are recycled)."""
        n = len(sets)
        arr = (C.c_void_p * max(n, 1))(*[d.handle.value for d in sets])
        karr = None
        if keeps is not None:
            karr = (C.c_void_p * max(n, 1))(*[(k if k else None) for k in keeps])
        if out is None:
            out = DeviceReads(self, None)
        check(lib().apg_reads_concat_dev(self._h, C.cast(arr, C.POINTER(C.c_void_p)),
                                         C.cast(karr, C.POINTER(C.c_void_p)) if karr is not None else None, n,
                                         C.byref(out._h)), "apg_reads_concat_dev")
        return out

    # multi-GPU correction stages (allpathslg_amd.distributed.sharded_precorrect)
    def shard_solid(self, d_recv_ptr: int, recv_counts: np.ndarray, K: int, n_shards: int, min_solid: int) -> int:
        rc = np.ascontiguousarray(recv_counts, dtype=np.uint64)
        n = C.c_uint64()
        check(lib().apg_shard_solid(self._h, C.c_void_p(d_recv_ptr), rc.ctypes.data_as(_u64p), K, n_shards,
                                    min_solid, C.byref(n)), "apg_shard_solid")
        return int(n.value)

    def shard_solid_weak(self, d_recv_ptr: int, recv_counts: np.ndarray, K: int, n_shards: int, min_solid: int,
                         d_mask_ptr: int) -> int:
        """apg_shard_solid + the weak mask (u32) of every received record."""
        rc = np.ascontiguousarray(recv_counts, dtype=np.uint64)
        n = C.c_uint64()
        check(lib().apg_shard_solid_weak(self._h, C.c_void_p(d_recv_ptr), rc.ctypes.data_as(_u64p), K, n_shards,
                                         min_solid, C.c_void_p(d_mask_ptr), C.byref(n)), "apg_shard_solid_weak")
        return int(n.value)

    def precorrect_weak(self, dreads: DeviceReads, d_solid_ptr: int, n_solid: int, d_pos_ptr: int, d_mask_ptr: int,
                        n_records: int, K: int = 24, min_solid: int = 3, max_q_suspect: int = 20) -> dict:
        """One correction pass through the weak bitmap built from the returned
        per-record masks (apg_precorrect_weak)."""
        p = self.pc_params(K, min_solid, max_q_suspect, 1)
        st = apg_pc_stats()
        check(lib().apg_precorrect_weak(self._h, dreads.handle, C.byref(p), C.c_void_p(d_solid_ptr), n_solid,
                                        C.c_void_p(d_pos_ptr), C.c_void_p(d_mask_ptr), n_records, C.byref(st)),
              "apg_precorrect_weak")
        return st.as_dict()

    def solid_export(self, d_out_ptr: int) -> None:
        check(lib().apg_solid_export(self._h, C.c_void_p(d_out_ptr)), "apg_solid_export")

    def solid_copy(self, d_out_ptr: Optional[int] = None) -> int:
        """Copy the last correction pass's solid hashes to a device buffer
        (None: size only); returns their number."""
        n = C.c_uint64()
        check(lib().apg_solid_copy(self._h, C.c_void_p(d_out_ptr) if d_out_ptr else None, C.byref(n)),
              "apg_solid_copy")
        return int(n.value)

    def precorrect_solid(self, dreads: DeviceReads, d_solid_ptr: int, n_solid: int, K: int = 24, min_solid: int = 3,
                         max_q_suspect: int = 20) -> dict:
        p = self.pc_params(K, min_solid, max_q_suspect, 1)
        st = apg_pc_stats()
        check(lib().apg_precorrect_solid(self._h, dreads.handle, C.byref(p), C.c_void_p(d_solid_ptr), n_solid,
                                         C.byref(st)), "apg_precorrect_solid")
        return st.as_dict()

    def download(self, dreads: DeviceReads, with_quals: bool = False) -> ReadSet:
        """Host copy of a device read set.  Sets produced on the device
        (FillFragments, concat) come back without qualities unless
        with_quals (the set must then have them)."""
        r = dreads.reads
        if r is None:  # produced on the device: take the shape from the device set
            n, nb, ny = C.c_uint64(), C.c_uint64(), C.c_uint64()
            check(lib().apg_dreads_shape(self._h, dreads.handle, C.byref(n), C.byref(nb), C.byref(ny), None, None),
                  "apg_dreads_shape")
            bo = np.zeros(n.value + 1, dtype=np.uint64)
            yo = np.zeros(n.value + 1, dtype=np.uint64)
            check(lib().apg_dreads_shape(self._h, dreads.handle, None, None, None, bo.ctypes.data_as(_u64p),
                                         yo.ctypes.data_as(_u64p)), "apg_dreads_shape")
            r = ReadSet(bo, yo, np.zeros(max(int(ny.value), 1), dtype=np.uint8),
                        np.zeros(max(int(nb.value), 1), dtype=np.uint8) if with_quals else None)
        pk = np.zeros_like(r.packed)
        q = np.zeros_like(r.quals) if r.quals is not None else None
        check(lib().apg_reads_download(self._h, dreads.handle, pk.ctypes.data_as(C.POINTER(C.c_uint8)),
                                       q.ctypes.data_as(C.POINTER(C.c_uint8)) if q is not None else None),
              "apg_reads_download")
        return ReadSet(r.base_off.copy(), r.byte_off.copy(), pk, q)

    # -- FillFragments ---------------------------------------------------------
    @staticmethod
    def fill_params(K: int = 24, min_insert: int = 126, max_insert: int = 234, max_steps: int = 1024,
                    min_solid: int = 3, last_solid: bool = False):
        from ._lib import APG_FILL_LAST_SOLID, apg_fill_params

        p = apg_fill_params()
        lib().apg_fill_defaults(C.byref(p))
        p.K, p.min_insert, p.max_insert, p.max_steps, p.min_solid = K, min_insert, max_insert, max_steps, min_solid
        p.flags = APG_FILL_LAST_SOLID if last_solid else 0
        return p

    def fill_fragments(self, pairs, solid=None, K: int = 24, min_insert: int = 126, max_insert: int = 234,
                       max_steps: int = 1024, min_solid: int = 3, last_solid: bool = False, out=None,
                       status: bool = False, d_status: Optional[int] = None):
        """FillFragments (include/apg.h): pairs (2i, 2i+1) closed through the
        solid K-mer graph.  `solid`: hashes of solid canonical K-mers (numpy
        u64 for host pairs; (device pointer, count) for DeviceReads), or None
        = last correction pass's set (last_solid=True) / the pairs' own
        count.  ReadSet -> (filled ReadSet, status u8 or None, stats);
        DeviceReads -> (DeviceReads of the filled fragments (reusing `out`),
        None, stats); d_status: a device u8[n_pairs] buffer for the
        per-pair statuses."""
        from ._lib import apg_fill_stats

        p = self.fill_params(K, min_insert, max_insert, max_steps, min_solid, last_solid)
        st = apg_fill_stats()
        L = lib()
        if isinstance(pairs, DeviceReads):
            dptr, ns = solid if solid is not None else (None, 0)
            fd = out if out is not None else DeviceReads(self, None)
            check(L.apg_fill_fragments_dev(self._h, pairs.handle, C.byref(p), C.c_void_p(dptr) if dptr else None, ns,
                                           C.byref(fd._h), C.c_void_p(d_status) if d_status else None,
                                           C.byref(st)), "apg_fill_fragments_dev")
            return fd, None, st.as_dict()
        from ._lib import apg_reads

        sh = None if solid is None else np.ascontiguousarray(solid, dtype=np.uint64)
        r = pairs.c_struct()
        o = apg_reads()
        np_ = pairs.n_reads // 2
        stat = np.zeros(max(np_, 1), dtype=np.uint8) if status else None
        check(L.apg_fill_fragments(self._h, C.byref(r), C.byref(p), sh.ctypes.data_as(_u64p) if sh is not None else None,
                                   0 if sh is None else len(sh), C.byref(o),
                                   stat.ctypes.data_as(C.POINTER(C.c_uint8)) if stat is not None else None,
                                   C.byref(st)), "apg_fill_fragments")
        try:
            n = int(o.n_reads)
            bo = np.ctypeslib.as_array(o.base_off, shape=(n + 1,)).copy()
            yo = np.ctypeslib.as_array(o.byte_off, shape=(n + 1,)).copy()
            nb = int(yo[-1])
            pk = np.zeros(nb + 64, dtype=np.uint8)
            if nb:
                pk[:nb] = np.ctypeslib.as_array(o.packed, shape=(nb,))
        finally:
            L.apg_reads_release(C.byref(o))
        return ReadSet(bo, yo, pk, None), (stat[:np_] if stat is not None else None), st.as_dict()

    # -- unipaths -------------------------------------------------------------
    def unipaths(self, reads, K: int = 96, read_paths: bool = True, fetch: bool = True):
        """Unipath graph (Unipather + HyperKmerPath).
        Returns (graph dict of numpy arrays or None if fetch=False, stats)."""
        from ._lib import APG_UNIPATH_READ_PATHS, apg_unipath_graph, apg_unipath_params, apg_unipath_stats

        p = apg_unipath_params()
        lib().apg_unipath_defaults(C.byref(p))
        p.K = K
        p.flags = APG_UNIPATH_READ_PATHS if read_paths else 0
        g = apg_unipath_graph()
        st = apg_unipath_stats()
        gp = C.byref(g) if fetch else None
        L = lib()
        if isinstance(reads, DeviceReads):
            check(L.apg_unipaths_dev(self._h, reads.handle, C.byref(p), gp, C.byref(st)), "apg_unipaths_dev")
        else:
            if not fetch:
                raise ValueError("host read sets always fetch the graph")
            r = reads.c_struct()
            check(L.apg_unipaths(self._h, C.byref(r), C.byref(p), gp, C.byref(st)), "apg_unipaths")
        if not fetch:
            return None, st.as_dict()
        try:
            return graph_arrays(g), st.as_dict()
        finally:
            L.apg_unipath_graph_free(C.byref(g))

    def error_correct_jump(self, frags, jumps, K: int = 24, min_solid: int = 3, max_q_suspect: int = 20,
                           min_keep: int = 40, d_keep: Optional[int] = None):
        """ErrorCorrectJump (include/apg.h apg_error_correct_jump; [R:M]
        src/paths/ErrorCorrectJump.cc): correct `jumps` against the solid set of
        `frags`, then trim each to its all-solid prefix.

        Host ReadSets -> (corrected jumps ReadSet (untrimmed layout), keep u32[n],
        stats).  DeviceReads (jumps corrected in place, keep lengths written to
        the device buffer d_keep) -> stats."""
        from ._lib import apg_ecj_params, apg_ecj_stats

        p = apg_ecj_params()
        lib().apg_ecj_defaults(C.byref(p))
        p.K, p.min_solid, p.max_q_suspect, p.min_keep = K, min_solid, max_q_suspect, min_keep
        st = apg_ecj_stats()
        if isinstance(jumps, DeviceReads):
            check(lib().apg_error_correct_jump_dev(self._h, frags.handle, jumps.handle, C.byref(p),
                                                   C.c_void_p(d_keep), C.byref(st)), "apg_error_correct_jump_dev")
            return st.as_dict()
        f, j = frags.c_struct(), jumps.c_struct()
        pk = np.zeros_like(jumps.packed)
        q = np.zeros_like(jumps.quals)
        keep = np.zeros(max(jumps.n_reads, 1), dtype=np.uint32)
        check(lib().apg_error_correct_jump(self._h, C.byref(f), C.byref(j), C.byref(p), pk.ctypes.data_as(C.POINTER(C.c_uint8)),
                                           q.ctypes.data_as(C.POINTER(C.c_uint8)), keep.ctypes.data_as(_u32p),
                                           C.byref(st)), "apg_error_correct_jump")
        return ReadSet(jumps.base_off.copy(), jumps.byte_off.copy(), pk, q), keep[: jumps.n_reads], st.as_dict()

    def unipath_coverage(self, locs, n_unipaths: int, n_locs: Optional[int] = None, min_len: int = 500):
        """UnipathCoverage (include/apg.h apg_unipath_coverage): placements per
        unipath, placements per K-mer, genome-wide coverage c0 and copy-number
        estimates on this context's last unipath build.  `locs`: (n, 4) int32
        host placements, or a device pointer from unipath_locs(DeviceReads)
        with n_locs.  Returns ({"counts", "cov", "cn"}, stats)."""
        from ._lib import apg_aln_pair, apg_ucov_params, apg_ucov_stats

        p = apg_ucov_params()
        lib().apg_ucov_defaults(C.byref(p))
        p.min_len = min_len
        U = int(n_unipaths)
        counts = np.zeros(max(U, 1), np.uint64)
        cov = np.zeros(max(U, 1), np.float64)
        cn = np.zeros(max(U, 1), np.uint32)
        st = apg_ucov_stats()
        outs = (counts.ctypes.data_as(C.POINTER(C.c_uint64)), cov.ctypes.data_as(C.POINTER(C.c_double)),
                cn.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(st))
        if isinstance(locs, np.ndarray):
            a = np.ascontiguousarray(locs, dtype=np.int32)
            n = len(a)
            check(lib().apg_unipath_coverage(self._h, a.ctypes.data_as(C.POINTER(apg_aln_pair)) if n else None, n,
                                             C.byref(p), *outs), "apg_unipath_coverage")
        else:
            check(lib().apg_unipath_coverage_dev(self._h, C.c_void_p(int(locs)), int(n_locs), C.byref(p), *outs),
                  "apg_unipath_coverage_dev")
        return {"counts": counts[:U], "cov": cov[:U], "cn": cn[:U]}, st.as_dict()

    def unipath_locs(self, reads, rc: bool = True, sorted: bool = True):
        """UnipathLocs: placements of `reads` (host ReadSet or DeviceReads) on
        the unipaths of this context's last unipath build (include/apg.h
        apg_unipath_locs; [R:M] BuildUnipathLocs / ReadLocationLG).

        Host reads -> ((n, 4) int32 [read, unipath, start, flags], stats).
        DeviceReads -> (device pointer to n apg_aln_pair, n, stats); the
        pointer is valid until the next unipath_locs call."""
        from ._lib import APG_ULOCS_RC, APG_ULOCS_SORTED, apg_aln_pair, apg_uloc_stats

        flags = (APG_ULOCS_RC if rc else 0) | (APG_ULOCS_SORTED if sorted else 0)
        st = apg_uloc_stats()
        n = C.c_uint64(0)
        L = lib()
        if isinstance(reads, DeviceReads):
            p = C.c_void_p()
            check(L.apg_unipath_locs_dev(self._h, reads.handle, flags, C.byref(p), C.byref(n), C.byref(st)),
                  "apg_unipath_locs_dev")
            return int(p.value or 0), int(n.value), st.as_dict()
        r = reads.c_struct()
        p = C.POINTER(apg_aln_pair)()
        check(L.apg_unipath_locs(self._h, C.byref(r), flags, C.byref(p), C.byref(n), C.byref(st)),
              "apg_unipath_locs")
        try:
            k = int(n.value)
            buf = C.cast(p, C.POINTER(C.c_int32 * (4 * k))).contents if k else None
            out = np.frombuffer(buf, dtype=np.int32).reshape(k, 4).copy() if k else np.zeros((0, 4), np.int32)
        finally:
            L.apg_free(p)
        return out, st.as_dict()

    def device_copy(self, d_dst: int, d_src: int, nbytes: int) -> None:
        """Device-to-device copy on libapg's stream (library output -> caller buffer)."""
        check(lib().apg_device_copy(self._h, C.c_void_p(d_dst), C.c_void_p(d_src), nbytes), "apg_device_copy")

    def unibases_dev(self) -> "DeviceReads":
        """The last build's unibases as a device read set (aligner targets)."""
        d = DeviceReads(self, None)
        check(lib().apg_unibases_dev(self._h, C.byref(d._h)), "apg_unibases_dev")
        return d

    # -- sharded unipath stages (multi-GPU) -------------------------------------
    def ushard_count(self, dreads: DeviceReads, K: int, n_shards: int) -> Tuple[np.ndarray, int]:
        """(distinct local nodes per digit [32, shard-major], K-mer instances)."""
        counts = np.zeros(32, dtype=np.uint64)
        n = C.c_uint64()
        check(lib().apg_ushard_count(self._h, dreads.handle, K, n_shards, counts.ctypes.data_as(_u64p), C.byref(n)),
              "apg_ushard_count")
        return counts, int(n.value)

    def ushard_scatter(self, dreads: DeviceReads, K: int, n_shards: int, d_send_ptr: int) -> None:
        check(lib().apg_ushard_scatter(self._h, dreads.handle, K, n_shards, C.c_void_p(d_send_ptr)),
              "apg_ushard_scatter")

    def ushard_nodes(self, d_recv_ptr: int, recv_counts: np.ndarray, K: int, n_shards: int) -> int:
        rc = np.ascontiguousarray(recv_counts, dtype=np.uint64)
        n = C.c_uint64()
        check(lib().apg_ushard_nodes(self._h, C.c_void_p(d_recv_ptr), rc.ctypes.data_as(_u64p), K, n_shards,
                                     C.byref(n)), "apg_ushard_nodes")
        return int(n.value)

    def urec_count(self, dreads: DeviceReads, K: int, n_shards: int) -> Tuple[np.ndarray, int]:
        """Sharded node build through minimizer partitions, step 1: 48-byte
        records per (shard, digit) (n_shards * 32, dest-major) and the reads'
        K-mer instances."""
        counts = np.zeros(n_shards * 32, dtype=np.uint64)
        ni = C.c_uint64()
        check(lib().apg_urec_count(self._h, dreads.handle, K, n_shards, counts.ctypes.data_as(_u64p), C.byref(ni)),
              "apg_urec_count")
        return counts, int(ni.value)

    def urec_scatter(self, dreads: DeviceReads, K: int, n_shards: int, d_send_ptr: int) -> None:
        check(lib().apg_urec_scatter(self._h, dreads.handle, K, n_shards, C.c_void_p(d_send_ptr)), "apg_urec_scatter")

    def urec_nodes(self, d_recv_ptr: int, recv_counts: np.ndarray, K: int, n_shards: int) -> int:
        rc = np.ascontiguousarray(recv_counts, dtype=np.uint64)
        n = C.c_uint64()
        check(lib().apg_urec_nodes(self._h, C.c_void_p(d_recv_ptr), rc.ctypes.data_as(_u64p), K, n_shards,
                                   C.byref(n)), "apg_urec_nodes")
        return int(n.value)

    def urec_export(self, d_out_ptr: int) -> None:
        check(lib().apg_urec_export(self._h, C.c_void_p(d_out_ptr)), "apg_urec_export")

    def ushard_export(self, d_out_ptr: int) -> None:
        check(lib().apg_ushard_export(self._h, C.c_void_p(d_out_ptr)), "apg_ushard_export")

    def unipaths_from_nodes(self, d_nodes_ptr: int, n_nodes: int, dreads, K: int = 96, read_paths: bool = True,
                            fetch: bool = False):
        from ._lib import APG_UNIPATH_READ_PATHS, apg_unipath_graph, apg_unipath_params, apg_unipath_stats

        p = apg_unipath_params()
        lib().apg_unipath_defaults(C.byref(p))
        p.K = K
        p.flags = APG_UNIPATH_READ_PATHS if read_paths else 0
        g = apg_unipath_graph()
        st = apg_unipath_stats()
        check(lib().apg_unipaths_from_nodes(self._h, C.c_void_p(d_nodes_ptr), n_nodes,
                                            dreads.handle if dreads is not None else None, C.byref(p),
                                            C.byref(g) if fetch else None, C.byref(st)), "apg_unipaths_from_nodes")
        if not fetch:
            return None, st.as_dict()
        try:
            return graph_arrays(g), st.as_dict()
        finally:
            lib().apg_unipath_graph_free(C.byref(g))

    # -- MakeRcDb ------------------------------------------------------------------
    def make_rc_db(self, g: dict) -> dict:
        """rc read paths + the sorted (fw + rc) interval index of a graph dict
        with read paths (as returned by unipaths()).  entries: structured array
        (start, len, read, pos, flags)."""
        from ._lib import apg_rc_db, apg_unipath_graph

        keep = {k: np.ascontiguousarray(g[k], dtype=np.uint64)
                for k in ("len", "id_base", "rc", "path_off", "path_start", "path_len")}
        gg = apg_unipath_graph()
        gg.n_unipaths = len(keep["len"])
        gg.len = keep["len"].ctypes.data_as(_u64p)
        gg.id_base = keep["id_base"].ctypes.data_as(_u64p)
        gg.rc = keep["rc"].ctypes.data_as(_u64p)
        gg.n_reads = len(keep["path_off"]) - 1
        gg.path_off = keep["path_off"].ctypes.data_as(_u64p)
        gg.n_intervals = len(keep["path_start"])
        gg.path_start = keep["path_start"].ctypes.data_as(_u64p)
        gg.path_len = keep["path_len"].ctypes.data_as(_u64p)
        db = apg_rc_db()
        L = lib()
        check(L.apg_make_rc_db(self._h, C.byref(gg), C.byref(db)), "apg_make_rc_db")
        try:
            n = int(db.n_entries)
            ent = np.zeros(n, dtype=RPINT_DTYPE)
            if n:
                C.memmove(ent.ctypes.data, C.cast(db.entries, C.c_void_p), n * RPINT_DTYPE.itemsize)
            return {
                "rc_path_off": _arr(db.rc_path_off, int(db.n_reads) + 1, np.uint64),
                "rc_start": _arr(db.rc_start, int(db.n_rc_intervals), np.uint64),
                "rc_len": _arr(db.rc_len, int(db.n_rc_intervals), np.uint64),
                "entries": ent,
            }
        finally:
            L.apg_rc_db_free(C.byref(db))

    # -- alignment and consensus ----------------------------------
    @staticmethod
    def _pairs(pairs) -> np.ndarray:
        """(n, 4) [s_id, t_id, offset, flags] -> contiguous int32 rows (= apg_aln_pair)."""
        a = np.ascontiguousarray(np.asarray(pairs, dtype=np.int64).reshape(-1, 4).astype(np.int32))
        return a

    def gapfree(self, S: ReadSet, T: ReadSet, pairs) -> np.ndarray:
        """Gap-free alignments: (n, 4) uint32 rows [overlap, mismatches, qsum, offset]."""
        from ._lib import apg_aln_pair, apg_gapfree_hit

        p = self._pairs(pairs)
        out = np.zeros((len(p), 4), dtype=np.uint32)
        rs, rt = S.c_struct(), T.c_struct()
        check(lib().apg_gapfree(self._h, C.byref(rs), C.byref(rt), p.ctypes.data_as(C.POINTER(apg_aln_pair)), len(p),
                                out.ctypes.data_as(C.POINTER(apg_gapfree_hit))), "apg_gapfree")
        return out

    def banded_sw(self, S: ReadSet, T: ReadSet, pairs, band_w: int, max_blocks: int = 0):
        """Banded Smith-Waterman: ((n, 8) int32 rows [cost, t_begin, t_end,
        mismatches, gaps_s, gaps_t, n_blocks, status], blocks (n, max_blocks, 2)
        int32 or None)."""
        from ._lib import apg_aln_pair, apg_sw_hit

        p = self._pairs(pairs)
        out = np.zeros((len(p), 8), dtype=np.int32)
        blk = np.zeros((len(p), max_blocks, 2), dtype=np.int32) if max_blocks else None
        rs, rt = S.c_struct(), T.c_struct()
        check(lib().apg_banded_sw(self._h, C.byref(rs), C.byref(rt), p.ctypes.data_as(C.POINTER(apg_aln_pair)),
                                  len(p), band_w, out.ctypes.data_as(C.POINTER(apg_sw_hit)),
                                  blk.ctypes.data_as(C.POINTER(C.c_int32)) if blk is not None else None, max_blocks),
              "apg_banded_sw")
        return out, blk

    def consensus(self, R: ReadSet, T: ReadSet, placements) -> Tuple[np.ndarray, np.ndarray]:
        """Column consensus of R placed gap-free on T: (bases, quals), one per T base."""
        from ._lib import apg_aln_pair

        p = self._pairs(placements)
        nt = T.n_bases
        b = np.zeros(max(nt, 1), dtype=np.uint8)
        q = np.zeros(max(nt, 1), dtype=np.uint8)
        rr, rt = R.c_struct(), T.c_struct()
        check(lib().apg_consensus(self._h, C.byref(rr), C.byref(rt), p.ctypes.data_as(C.POINTER(apg_aln_pair)), len(p),
                                  b.ctypes.data_as(C.POINTER(C.c_uint8)), q.ctypes.data_as(C.POINTER(C.c_uint8))),
              "apg_consensus")
        return b[:nt], q[:nt]

    # device-resident variants (pairs / outputs are device pointers, e.g.
    # torch tensors' data_ptr(); ids must be in range)
    def gapfree_dev(self, dS: DeviceReads, dT: DeviceReads, d_pairs: int, n: int, d_out: int) -> None:
        check(lib().apg_gapfree_dev(self._h, dS.handle, dT.handle, C.c_void_p(d_pairs), n, C.c_void_p(d_out)),
              "apg_gapfree_dev")

    def banded_sw_dev(self, dS: DeviceReads, dT: DeviceReads, d_pairs: int, n: int, band_w: int, d_out: int,
                      d_blocks: int = 0, max_blocks: int = 0) -> None:
        check(lib().apg_banded_sw_dev(self._h, dS.handle, dT.handle, C.c_void_p(d_pairs), n, band_w,
                                      C.c_void_p(d_out), C.c_void_p(d_blocks or None), max_blocks),
              "apg_banded_sw_dev")

    def consensus_dev(self, dR: DeviceReads, dT: DeviceReads, d_plc: int, n: int, d_bases: int, d_quals: int) -> None:
        check(lib().apg_consensus_dev(self._h, dR.handle, dT.handle, C.c_void_p(d_plc), n, C.c_void_p(d_bases),
                                      C.c_void_p(d_quals)), "apg_consensus_dev")

    # -- sharded (multi-GPU) stages ------------------------------------------
    def shard_count(self, dreads: DeviceReads, K: int, n_shards: int) -> np.ndarray:
        B = shard_bins(K, n_shards)
        counts = np.zeros(n_shards * B, dtype=np.uint64)
        check(lib().apg_shard_count(self._h, dreads.handle, K, n_shards, counts.ctypes.data_as(_u64p)),
              "apg_shard_count")
        return counts

    def shard_scatter(self, dreads: DeviceReads, K: int, n_shards: int, d_send_ptr: int) -> None:
        check(lib().apg_shard_scatter(self._h, dreads.handle, K, n_shards, C.c_void_p(d_send_ptr)),
              "apg_shard_scatter")

    def shard_scatter_pos(self, dreads: DeviceReads, K: int, n_shards: int, d_send_ptr: int, d_pos_ptr: int) -> None:
        check(lib().apg_shard_scatter_pos(self._h, dreads.handle, K, n_shards, C.c_void_p(d_send_ptr),
                                          C.c_void_p(d_pos_ptr)), "apg_shard_scatter_pos")

    def shard_spectrum(self, d_recv_ptr: int, recv_counts: np.ndarray, K: int, n_shards: int,
                       hist_len: int = DEFAULT_HIST_LEN):
        rc_arr = np.ascontiguousarray(recv_counts, dtype=np.uint64)
        hist = np.zeros(hist_len, dtype=np.uint64)
        st = apg_kstats()
        check(lib().apg_shard_spectrum(self._h, C.c_void_p(d_recv_ptr), rc_arr.ctypes.data_as(_u64p), K, n_shards,
                                       hist.ctypes.data_as(_u64p), hist_len, C.byref(st)),
              "apg_shard_spectrum")
        return hist, st.as_dict()


RPINT_DTYPE = np.dtype([("start", "<u8"), ("len", "<u4"), ("read", "<u4"), ("pos", "<u4"), ("flags", "<u4")])


def _arr(p, n, dt):
    return np.ctypeslib.as_array(p, shape=(n,)).astype(dt).copy() if n else np.zeros(0, dt)


class _HostArray:
    """Owns one library-allocated host array (apg_free on release); numpy views
    keep it alive, so the graph's arrays need no copy."""

    def __init__(self, addr: int):
        self.addr = addr

    def __del__(self):
        try:
            lib().apg_free(C.c_void_p(self.addr))
        except Exception:
            pass


def _take(g, field: str, n: int, dt) -> np.ndarray:
    """Take ownership of graph field `field` (n elements): a numpy array over
    the library's buffer, the struct's pointer cleared (so
    apg_unipath_graph_free leaves it alone)."""
    p = getattr(g, field)
    addr = C.cast(p, C.c_void_p).value if p else None
    setattr(g, field, type(p)())
    if not addr:
        return np.zeros(0, dt)
    owner = _HostArray(addr)
    if n == 0:
        return np.zeros(0, dt)
    buf = (C.c_uint8 * (n * np.dtype(dt).itemsize)).from_address(addr)
    buf._owner = owner
    return np.frombuffer(buf, dtype=dt)


def graph_arrays(g) -> dict:
    """apg_unipath_graph -> dict of numpy arrays (same keys as oracle.unipaths).
    The arrays take over the library's host buffers (no copy of the graph,
    which is ~0.4 GB at the bench config)."""
    U = int(g.n_unipaths)
    out = {
        "n_nodes": int(g.n_nodes),
        "n_unipaths": U,
        "len": _take(g, "len", U, np.uint64),
        "id_base": _take(g, "id_base", U, np.uint64),
        "rc": _take(g, "rc", U, np.uint64),
        "ub_off": _take(g, "ub_off", U + 1, np.uint64),
        "n_vertices": int(g.n_vertices),
        "from": _take(g, "frm", U, np.uint64),
        "to": _take(g, "to", U, np.uint64),
    }
    out["unibases"] = _take(g, "unibases", int(out["ub_off"][-1]) if U else 0, np.uint8)
    nr = int(g.n_reads)
    if g.path_off:
        out["path_off"] = _take(g, "path_off", nr + 1, np.uint64)
        out["path_start"] = _take(g, "path_start", int(g.n_intervals), np.uint64)
        out["path_len"] = _take(g, "path_len", int(g.n_intervals), np.uint64)
    return out


def write_kspec(path: str, K: int, hist: np.ndarray) -> None:
    h = np.ascontiguousarray(hist, dtype=np.uint64)
    check(lib().apg_kspec_write(path.encode(), K, h.ctypes.data_as(_u64p), len(h)), "apg_kspec_write")


def _graph_struct(g: dict, K: int):
    """dict of numpy arrays -> (apg_unipath_graph, arrays kept alive)."""
    from ._lib import apg_unipath_graph

    keep = {k: np.ascontiguousarray(g[k], dtype=np.uint64)
            for k in ("len", "id_base", "rc", "ub_off", "from", "to", "path_off", "path_start", "path_len") if k in g}
    keep["unibases"] = np.ascontiguousarray(g["unibases"], dtype=np.uint8)
    s = apg_unipath_graph()
    s.K = K
    s.n_nodes = int(g.get("n_nodes", 0))
    s.n_unipaths = len(keep["len"])
    s.len = keep["len"].ctypes.data_as(_u64p)
    s.id_base = keep["id_base"].ctypes.data_as(_u64p)
    s.rc = keep["rc"].ctypes.data_as(_u64p)
    s.ub_off = keep["ub_off"].ctypes.data_as(_u64p)
    s.unibases = keep["unibases"].ctypes.data_as(C.POINTER(C.c_uint8))
    s.n_vertices = int(g.get("n_vertices", 0))
    s.frm = keep["from"].ctypes.data_as(_u64p)
    s.to = keep["to"].ctypes.data_as(_u64p)
    if "path_off" in keep:
        s.n_reads = len(keep["path_off"]) - 1
        s.path_off = keep["path_off"].ctypes.data_as(_u64p)
        s.n_intervals = len(keep["path_start"])
        s.path_start = keep["path_start"].ctypes.data_as(_u64p)
        s.path_len = keep["path_len"].ctypes.data_as(_u64p)
    return s, keep


def write_graph(head: str, g: dict, K: int) -> None:
    """<head>.unipaths/.unibases/.hkp(/.paths).k<K> (include/apg.h)."""
    s, _keep = _graph_struct(g, K)
    check(lib().apg_graph_write(head.encode(), C.byref(s)), "apg_graph_write")


def read_graph(head: str, K: int) -> dict:
    from ._lib import apg_unipath_graph

    s = apg_unipath_graph()
    check(lib().apg_graph_read(head.encode(), K, C.byref(s)), "apg_graph_read")
    try:
        return graph_arrays(s)
    finally:
        lib().apg_unipath_graph_free(C.byref(s))


def write_rc_db(head: str, K: int, db: dict) -> None:
    """<head>.paths_rc.k<K> and <head>.pathsdb.k<K>."""
    from ._lib import apg_rc_db, apg_rpint

    off = np.ascontiguousarray(db["rc_path_off"], dtype=np.uint64)
    st = np.ascontiguousarray(db["rc_start"], dtype=np.uint64)
    ln = np.ascontiguousarray(db["rc_len"], dtype=np.uint64)
    ent = np.ascontiguousarray(db["entries"], dtype=RPINT_DTYPE)
    s = apg_rc_db()
    s.n_reads = len(off) - 1
    s.rc_path_off = off.ctypes.data_as(_u64p)
    s.n_rc_intervals = len(st)
    s.rc_start = st.ctypes.data_as(_u64p)
    s.rc_len = ln.ctypes.data_as(_u64p)
    s.n_entries = len(ent)
    s.entries = ent.ctypes.data_as(C.POINTER(apg_rpint))
    check(lib().apg_rc_db_write(head.encode(), K, C.byref(s)), "apg_rc_db_write")


def read_kmerpaths(path: str):
    """(K, path_off, start, len) of a .paths / .paths_rc file."""
    K = C.c_int()
    n, ni = C.c_uint64(), C.c_uint64()
    po, ps, pl = _u64p(), _u64p(), _u64p()
    L = lib()
    check(L.apg_kmerpaths_read(path.encode(), C.byref(K), C.byref(n), C.byref(po), C.byref(ni), C.byref(ps),
                               C.byref(pl)), "apg_kmerpaths_read")
    try:
        return (int(K.value), _arr(po, int(n.value) + 1, np.uint64), _arr(ps, int(ni.value), np.uint64),
                _arr(pl, int(ni.value), np.uint64))
    finally:
        for p in (po, ps, pl):
            L.apg_free(C.cast(p, C.c_void_p))


def kspec_estimate(hist) -> dict:
    """Genome-size estimate of a spectrum (include/apg.h apg_kspec_estimate)."""
    from ._lib import apg_kspec_summary

    h = np.ascontiguousarray(hist, dtype=np.uint64)
    out = apg_kspec_summary()
    check(lib().apg_kspec_estimate(h.ctypes.data_as(_u64p), len(h), C.byref(out)), "apg_kspec_estimate")
    return out.as_dict()


def read_solid(path: str):
    """(K, hashes) of a <head>.solid.k<K> file (ascending apg_kmer_hash values)."""
    K, n, p = C.c_int(), C.c_uint64(), _u64p()
    L = lib()
    check(L.apg_solid_read(path.encode(), C.byref(K), C.byref(p), C.byref(n)), "apg_solid_read")
    try:
        return int(K.value), _arr(p, int(n.value), np.uint64)
    finally:
        L.apg_free(C.cast(p, C.c_void_p))


def read_unilocs(path: str):
    """(K, n_reads, locs) of a <head>.unilocs.k<K> file; locs (n, 4) int32
    [read, unipath, start, flags] as Context.unipath_locs returns them."""
    from ._lib import apg_aln_pair

    K, nr, n = C.c_int(), C.c_uint64(), C.c_uint64()
    p = C.POINTER(apg_aln_pair)()
    L = lib()
    check(L.apg_ulocs_read(path.encode(), C.byref(K), C.byref(nr), C.byref(p), C.byref(n)), "apg_ulocs_read")
    try:
        m = int(n.value)
        locs = (np.ctypeslib.as_array(C.cast(p, C.POINTER(C.c_int32)), shape=(m * 4,)).reshape(m, 4).copy()
                if m else np.zeros((0, 4), np.int32))
        return int(K.value), int(nr.value), locs
    finally:
        L.apg_free(C.cast(p, C.c_void_p))


def read_unipath_coverage(path: str) -> dict:
    """A <head>.unipath_cov.k<K> file: {K, c0, counts, cov, cn}."""
    K, c0, n = C.c_int(), C.c_double(), C.c_uint64()
    pc, pv, pn = _u64p(), C.POINTER(C.c_double)(), C.POINTER(C.c_uint32)()
    L = lib()
    check(L.apg_ucov_read(path.encode(), C.byref(K), C.byref(c0), C.byref(n), C.byref(pc), C.byref(pv), C.byref(pn)),
          "apg_ucov_read")
    try:
        U = int(n.value)
        return {"K": int(K.value), "c0": float(c0.value), "counts": _arr(pc, U, np.uint64),
                "cov": _arr(pv, U, np.float64), "cn": _arr(pn, U, np.uint32)}
    finally:
        for p in (pc, pv, pn):
            L.apg_free(C.cast(p, C.c_void_p))
