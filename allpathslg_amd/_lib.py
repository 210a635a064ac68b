"""ctypes binding of libapg.so (the C ABI declared in include/apg.h).

The shared library is built in-tree (``allpathslg_amd/libapg.so``) by
``__graft_entry__.build()`` / ``make -C allpathslg_amd/csrc``.  There is no
fallback: if the library is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))


def _lib_path() -> str:
    """libapg.so, or libapg_<name>.so for APG_LIB_VARIANT=name (diagnostics
    builds, scripts/build_fill_variants.sh): the name is [A-Za-z0-9_]+ only,
    so the variant always comes from this directory."""
    v = os.environ.get("APG_LIB_VARIANT")
    if not v:
        return os.path.join(_HERE, "libapg.so")
    if not re.fullmatch(r"[A-Za-z0-9_]+", v):
        raise ValueError(f"APG_LIB_VARIANT={v!r}: only [A-Za-z0-9_] is allowed")
    path = os.path.join(_HERE, f"libapg_{v}.so")
    if not os.path.exists(path):
        raise FileNotFoundError(f"APG_LIB_VARIANT={v!r}: {path} is not built")
    return path


LIB_PATH = _lib_path()

APG_OK = 0
ERRORS = {
    -1: "APG_E_ARG",
    -2: "APG_E_HIP",
    -3: "APG_E_IO",
    -4: "APG_E_STATE",
    -5: "APG_E_NOMEM",
    -6: "APG_E_UNSUPPORTED",
}


class ApgError(RuntimeError):
    def __init__(self, code: int, where: str, msg: str):
        super().__init__(f"{where}: {ERRORS.get(code, code)}: {msg}")
        self.code = code


class apg_config(C.Structure):
    _fields_ = [
        ("device", C.c_int32),
        ("timing", C.c_int32),
        ("verbose", C.c_int32),
        ("kmer_dedup", C.c_int32),
        ("reserved", C.c_uint64 * 6),
    ]


class apg_reads(C.Structure):
    _fields_ = [
        ("n_reads", C.c_uint64),
        ("base_off", C.POINTER(C.c_uint64)),
        ("byte_off", C.POINTER(C.c_uint64)),
        ("packed", C.POINTER(C.c_uint8)),
        ("quals", C.POINTER(C.c_uint8)),
    ]


class apg_kstats(C.Structure):
    _fields_ = [
        ("n_kmers", C.c_uint64),
        ("n_distinct", C.c_uint64),
        ("n_buckets", C.c_uint64),
        ("n_overflow", C.c_uint64),
        ("max_bucket", C.c_uint64),
        ("n_redo", C.c_uint64),
        ("reserved", C.c_uint64 * 2),
    ]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_ if f != "reserved"}


class apg_pc_params(C.Structure):
    _fields_ = [
        ("K", C.c_int32),
        ("min_solid", C.c_uint32),
        ("max_q_suspect", C.c_uint32),
        ("n_cycles", C.c_uint32),
        ("reserved", C.c_uint64 * 4),
    ]


class apg_mem_stats(C.Structure):
    _fields_ = [
        ("workspace_bytes", C.c_uint64),
        ("workspace_peak", C.c_uint64),
        ("releases", C.c_uint64),
        ("device_used", C.c_uint64),
        ("device_total", C.c_uint64),
        ("reserved", C.c_uint64 * 3),
    ]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_ if f != "reserved"}


class apg_pc_stats(C.Structure):
    _fields_ = [
        ("n_suspect", C.c_uint64),
        ("n_corrected", C.c_uint64),
        ("n_ambiguous", C.c_uint64),
        ("n_uncorrectable", C.c_uint64),
        ("n_solid", C.c_uint64),
        ("record_form", C.c_uint64),
        ("reserved", C.c_uint64 * 2),
    ]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_ if f != "reserved"}


class apg_ecj_params(C.Structure):
    _fields_ = [("K", C.c_int32), ("min_solid", C.c_uint32), ("max_q_suspect", C.c_uint32), ("min_keep", C.c_uint32),
                ("reserved", C.c_uint64 * 4)]


class apg_ecj_stats(C.Structure):
    _fields_ = [("pc", apg_pc_stats), ("n_reads", C.c_uint64), ("n_full", C.c_uint64), ("n_trimmed", C.c_uint64),
                ("n_dropped", C.c_uint64), ("bases_kept", C.c_uint64), ("reserved", C.c_uint64 * 3)]

    def as_dict(self) -> dict:
        d = {f: int(getattr(self, f)) for f, _ in self._fields_ if f not in ("pc", "reserved")}
        d["precorrect"] = self.pc.as_dict()
        return d


APG_FILL_LAST_SOLID = 1
FILL_STATUS = {0: "filled", 1: "none", 2: "ambiguous", 3: "budget", 4: "skip"}


class apg_fill_params(C.Structure):
    _fields_ = [
        ("K", C.c_int32),
        ("min_insert", C.c_uint32),
        ("max_insert", C.c_uint32),
        ("max_steps", C.c_uint32),
        ("min_solid", C.c_uint32),
        ("flags", C.c_uint32),
        ("reserved", C.c_uint64 * 3),
    ]


class apg_fill_stats(C.Structure):
    _fields_ = [
        ("n_pairs", C.c_uint64),
        ("n_filled", C.c_uint64),
        ("n_none", C.c_uint64),
        ("n_ambiguous", C.c_uint64),
        ("n_budget", C.c_uint64),
        ("n_skip", C.c_uint64),
        ("filled_bases", C.c_uint64),
        ("n_solid", C.c_uint64),
        ("lookups", C.c_uint64),
        ("reserved", C.c_uint64 * 3),
    ]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_ if f != "reserved"}


class apg_unipath_params(C.Structure):
    _fields_ = [("K", C.c_int32), ("flags", C.c_uint32), ("reserved", C.c_uint64 * 4)]


class apg_unipath_stats(C.Structure):
    _fields_ = [
        ("n_instances", C.c_uint64),
        ("n_nodes", C.c_uint64),
        ("n_links", C.c_uint64),
        ("n_cycles_cut", C.c_uint64),
        ("n_unipaths", C.c_uint64),
        ("n_vertices", C.c_uint64),
        ("n_intervals", C.c_uint64),
        ("max_len", C.c_uint64),
    ]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class apg_unipath_graph(C.Structure):
    _fields_ = [
        ("K", C.c_int32),
        ("reserved0", C.c_int32),
        ("n_nodes", C.c_uint64),
        ("n_unipaths", C.c_uint64),
        ("len", C.POINTER(C.c_uint64)),
        ("id_base", C.POINTER(C.c_uint64)),
        ("rc", C.POINTER(C.c_uint64)),
        ("ub_off", C.POINTER(C.c_uint64)),
        ("unibases", C.POINTER(C.c_uint8)),
        ("n_vertices", C.c_uint64),
        ("frm", C.POINTER(C.c_uint64)),
        ("to", C.POINTER(C.c_uint64)),
        ("n_reads", C.c_uint64),
        ("path_off", C.POINTER(C.c_uint64)),
        ("n_intervals", C.c_uint64),
        ("path_start", C.POINTER(C.c_uint64)),
        ("path_len", C.POINTER(C.c_uint64)),
    ]


APG_UNIPATH_READ_PATHS = 1
APG_UNIPATH_GATHER_NODES = 2


APG_RPINT_RC = 1


class apg_rpint(C.Structure):
    _fields_ = [("start", C.c_uint64), ("len", C.c_uint32), ("read", C.c_uint32), ("pos", C.c_uint32),
                ("flags", C.c_uint32)]


class apg_rc_db(C.Structure):
    _fields_ = [
        ("n_reads", C.c_uint64),
        ("rc_path_off", C.POINTER(C.c_uint64)),
        ("n_rc_intervals", C.c_uint64),
        ("rc_start", C.POINTER(C.c_uint64)),
        ("rc_len", C.POINTER(C.c_uint64)),
        ("n_entries", C.c_uint64),
        ("entries", C.POINTER(apg_rpint)),
    ]


APG_ALN_RC = 1


class apg_aln_pair(C.Structure):
    _fields_ = [("s_id", C.c_uint32), ("t_id", C.c_uint32), ("offset", C.c_int32), ("flags", C.c_uint32)]


APG_ULOCS_RC = 1
APG_ULOCS_SORTED = 2


class apg_repeat_params(C.Structure):
    _fields_ = [("n_families", C.c_uint32), ("tandem_unit_max", C.c_uint32), ("family_len", C.c_uint32 * 8),
                ("family_frac", C.c_double * 8), ("family_div", C.c_double * 8), ("tandem_frac", C.c_double),
                ("tandem_array_max", C.c_uint32), ("reserved0", C.c_uint32)]


class apg_ucov_params(C.Structure):
    _fields_ = [("min_len", C.c_uint64), ("reserved", C.c_uint64 * 3)]


class apg_ucov_stats(C.Structure):
    _fields_ = [("c0", C.c_double), ("n_long", C.c_uint64), ("n_locs", C.c_uint64), ("n_bad", C.c_uint64)]

    def as_dict(self) -> dict:
        return {"c0": float(self.c0), "n_long": int(self.n_long), "n_locs": int(self.n_locs), "n_bad": int(self.n_bad)}


class apg_uloc_stats(C.Structure):
    _fields_ = [("n_reads", C.c_uint64), ("n_placed", C.c_uint64), ("n_locs", C.c_uint64), ("n_missing", C.c_uint64)]

    def as_dict(self) -> dict:
        return {f: int(getattr(self, f)) for f, _ in self._fields_}


class apg_kspec_summary(C.Structure):
    _fields_ = [("valley", C.c_uint64), ("peak", C.c_uint64), ("genome_size", C.c_uint64),
                ("genomic_kmers", C.c_uint64), ("genomic_instances", C.c_uint64), ("error_kmers", C.c_uint64),
                ("error_instances", C.c_uint64), ("coverage", C.c_double), ("repeat_fraction", C.c_double),
                ("het_ratio", C.c_double), ("reserved", C.c_uint64 * 2)]

    def as_dict(self) -> dict:
        return {f: (float(getattr(self, f)) if t is C.c_double else int(getattr(self, f)))
                for f, t in self._fields_ if f != "reserved"}


class apg_gapfree_hit(C.Structure):
    _fields_ = [("overlap", C.c_uint32), ("mismatches", C.c_uint32), ("qsum", C.c_uint32), ("offset", C.c_int32)]


class apg_sw_hit(C.Structure):
    _fields_ = [(f, C.c_int32) for f in ("cost", "t_begin", "t_end", "mismatches", "gaps_s", "gaps_t", "n_blocks",
                                         "status")]


class apg_synth_params(C.Structure):
    _fields_ = [
        ("genome_len", C.c_uint64),
        ("seed", C.c_uint64),
        ("n_pairs", C.c_uint64),
        ("read_len", C.c_uint32),
        ("insert_mean", C.c_uint32),
        ("insert_sd", C.c_uint32),
        ("threads", C.c_uint32),
        ("err_lo", C.c_double),
        ("err_hi", C.c_double),
        ("first_pair", C.c_uint64),
    ]


_P = C.c_void_p
_u64p = C.POINTER(C.c_uint64)
_u32p = C.POINTER(C.c_uint32)
_u8p = C.POINTER(C.c_uint8)

# name -> (restype, argtypes).  Every symbol of include/apg.h is listed here;
# tests/test_abi.py checks the two stay in sync.
SIGNATURES = {
    "apg_abi_version": (C.c_int, []),
    "apg_last_error": (C.c_char_p, []),
    "apg_create": (C.c_int, [C.POINTER(apg_config), C.POINTER(_P)]),
    "apg_destroy": (None, [_P]),
    "apg_trim": (C.c_int, [_P]),
    "apg_timing_get": (C.c_int, [_P, C.c_int, C.c_char_p, C.c_size_t, C.POINTER(C.c_double), _u64p, _u64p]),
    "apg_timing_overlapped": (C.c_int, [_P, C.c_int, _u64p]),
    "apg_mem_stats_get": (C.c_int, [_P, C.c_int, C.POINTER(apg_mem_stats)]),
    "apg_timing_reset": (C.c_int, [_P]),
    "apg_reads_upload": (C.c_int, [_P, C.POINTER(apg_reads), C.POINTER(_P)]),
    "apg_reads_free": (None, [_P]),
    "apg_dreads_count": (C.c_uint64, [_P]),
    "apg_reads_copy_dev": (C.c_int, [_P, _P, _P]),
    "apg_reads_concat_dev": (C.c_int, [_P, C.POINTER(_P), C.POINTER(_P), C.c_uint32, C.POINTER(_P)]),
    "apg_byte_offsets": (C.c_int, [_u64p, C.c_uint64, _u64p]),
    "apg_kmer_hash": (C.c_uint64, [C.c_int, C.c_uint64]),
    "apg_kmer_unhash": (C.c_uint64, [C.c_int, C.c_uint64]),
    "apg_kmer_spectrum": (C.c_int, [_P, C.POINTER(apg_reads), C.c_int, _u64p, C.c_size_t, C.POINTER(apg_kstats)]),
    "apg_kmer_spectrum_dev": (C.c_int, [_P, _P, C.c_int, _u64p, C.c_size_t, C.POINTER(apg_kstats)]),
    "apg_kmer_count": (
        C.c_int,
        [_P, C.POINTER(apg_reads), C.c_int, C.POINTER(_u64p), C.POINTER(_u32p), _u64p, C.POINTER(apg_kstats)],
    ),
    "apg_free": (None, [_P]),
    "apg_kmer_count_dev": (
        C.c_int,
        [_P, _P, C.c_int, C.c_uint64, C.c_uint64, C.POINTER(_u64p), C.POINTER(_u32p), _u64p, C.POINTER(apg_kstats)],
    ),
    "apg_shard_bins": (C.c_int, [C.c_int, C.c_int]),
    "apg_shard_count": (C.c_int, [_P, _P, C.c_int, C.c_int, _u64p]),
    "apg_shard_scatter": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_void_p]),
    "apg_shard_spectrum": (
        C.c_int,
        [_P, C.c_void_p, _u64p, C.c_int, C.c_int, _u64p, C.c_size_t, C.POINTER(apg_kstats)],
    ),
    "apg_pc_defaults": (None, [C.POINTER(apg_pc_params)]),
    "apg_precorrect": (C.c_int, [_P, C.POINTER(apg_reads), C.POINTER(apg_pc_params), _u8p, _u8p, C.POINTER(apg_pc_stats)]),
    "apg_precorrect_dev": (C.c_int, [_P, _P, C.POINTER(apg_pc_params), C.POINTER(apg_pc_stats)]),
    "apg_spectrum_precorrect_dev": (C.c_int, [_P, _P, C.c_int, _u64p, C.c_size_t, C.POINTER(apg_kstats),
                                              C.POINTER(apg_pc_params), C.POINTER(apg_pc_stats)]),
    "apg_reads_download": (C.c_int, [_P, _P, _u8p, _u8p]),
    "apg_shard_solid": (C.c_int, [_P, C.c_void_p, _u64p, C.c_int, C.c_int, C.c_uint32, _u64p]),
    "apg_partition_u64": (C.c_int, [_P, C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    "apg_solid_export": (C.c_int, [_P, C.c_void_p]),
    "apg_solid_copy": (C.c_int, [_P, C.c_void_p, _u64p]),
    "apg_solid_download": (C.c_int, [_P, _u64p, _u64p]),
    "apg_solid_upload": (C.c_int, [_P, C.c_int, _u64p, C.c_uint64]),
    "apg_precorrect_solid": (
        C.c_int, [_P, _P, C.POINTER(apg_pc_params), C.c_void_p, C.c_uint64, C.POINTER(apg_pc_stats)]
    ),
    "apg_fill_defaults": (None, [C.POINTER(apg_fill_params)]),
    "apg_fill_fragments": (
        C.c_int, [_P, C.POINTER(apg_reads), C.POINTER(apg_fill_params), _u64p, C.c_uint64, C.POINTER(apg_reads), _u8p,
                  C.POINTER(apg_fill_stats)]),
    "apg_fill_fragments_dev": (
        C.c_int, [_P, _P, C.POINTER(apg_fill_params), C.c_void_p, C.c_uint64, C.POINTER(_P), C.c_void_p,
                  C.POINTER(apg_fill_stats)]),
    "apg_spectrum_precorrect_fill_dev": (
        C.c_int, [_P, _P, C.c_int, _u64p, C.c_size_t, C.POINTER(apg_kstats), C.POINTER(apg_pc_params),
                  C.POINTER(apg_pc_stats), C.POINTER(apg_fill_params), C.POINTER(_P), C.c_void_p,
                  C.POINTER(apg_fill_stats)]),
    "apg_unipath_defaults": (None, [C.POINTER(apg_unipath_params)]),
    "apg_unipaths": (
        C.c_int,
        [_P, C.POINTER(apg_reads), C.POINTER(apg_unipath_params), C.POINTER(apg_unipath_graph),
         C.POINTER(apg_unipath_stats)],
    ),
    "apg_unipaths_dev": (
        C.c_int,
        [_P, _P, C.POINTER(apg_unipath_params), C.POINTER(apg_unipath_graph), C.POINTER(apg_unipath_stats)],
    ),
    "apg_unipath_graph_free": (None, [C.POINTER(apg_unipath_graph)]),
    "apg_ushard_bins": (C.c_int, [C.c_int]),
    "apg_ushard_count": (C.c_int, [_P, _P, C.c_int, C.c_int, _u64p, _u64p]),
    "apg_ushard_scatter": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_void_p]),
    "apg_ushard_nodes": (C.c_int, [_P, C.c_void_p, _u64p, C.c_int, C.c_int, _u64p]),
    "apg_ushard_export": (C.c_int, [_P, C.c_void_p]),
    "apg_unipaths_from_nodes": (
        C.c_int,
        [_P, C.c_void_p, C.c_uint64, _P, C.POINTER(apg_unipath_params), C.POINTER(apg_unipath_graph),
         C.POINTER(apg_unipath_stats)],
    ),
    "apg_make_rc_db": (C.c_int, [_P, C.POINTER(apg_unipath_graph), C.POINTER(apg_rc_db)]),
    "apg_rc_db_free": (None, [C.POINTER(apg_rc_db)]),
    "apg_gapfree": (
        C.c_int, [_P, C.POINTER(apg_reads), C.POINTER(apg_reads), C.POINTER(apg_aln_pair), C.c_uint64,
                  C.POINTER(apg_gapfree_hit)]),
    "apg_gapfree_dev": (C.c_int, [_P, _P, _P, C.c_void_p, C.c_uint64, C.c_void_p]),
    "apg_banded_sw": (
        C.c_int, [_P, C.POINTER(apg_reads), C.POINTER(apg_reads), C.POINTER(apg_aln_pair), C.c_uint64, C.c_int,
                  C.POINTER(apg_sw_hit), C.POINTER(C.c_int32), C.c_uint32]),
    "apg_banded_sw_dev": (C.c_int, [_P, _P, _P, C.c_void_p, C.c_uint64, C.c_int, C.c_void_p, C.c_void_p, C.c_uint32]),
    "apg_consensus": (
        C.c_int, [_P, C.POINTER(apg_reads), C.POINTER(apg_reads), C.POINTER(apg_aln_pair), C.c_uint64, _u8p, _u8p]),
    "apg_consensus_dev": (C.c_int, [_P, _P, _P, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
    "apg_urec_count": (C.c_int, [_P, _P, C.c_int, C.c_int, _u64p, _u64p]),
    "apg_urec_scatter": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_void_p]),
    "apg_urec_nodes": (C.c_int, [_P, C.c_void_p, _u64p, C.c_int, C.c_int, _u64p]),
    "apg_urec_export": (C.c_int, [_P, C.c_void_p]),
    "apg_shard_scatter_pos": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    "apg_shard_solid_weak": (C.c_int, [_P, C.c_void_p, _u64p, C.c_int, C.c_int, C.c_uint32, C.c_void_p, _u64p]),
    "apg_precorrect_weak": (
        C.c_int, [_P, _P, C.POINTER(apg_pc_params), C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                  C.POINTER(apg_pc_stats)]),
    "apg_ecj_defaults": (None, [C.POINTER(apg_ecj_params)]),
    "apg_error_correct_jump": (
        C.c_int, [_P, C.POINTER(apg_reads), C.POINTER(apg_reads), C.POINTER(apg_ecj_params), _u8p, _u8p,
                  C.POINTER(C.c_uint32), C.POINTER(apg_ecj_stats)]),
    "apg_error_correct_jump_dev": (
        C.c_int, [_P, _P, _P, C.POINTER(apg_ecj_params), C.c_void_p, C.POINTER(apg_ecj_stats)]),
    "apg_unipath_locs": (
        C.c_int, [_P, C.POINTER(apg_reads), C.c_uint32, C.POINTER(C.POINTER(apg_aln_pair)), _u64p,
                  C.POINTER(apg_uloc_stats)]),
    "apg_unipath_locs_dev": (
        C.c_int, [_P, _P, C.c_uint32, C.POINTER(C.c_void_p), _u64p, C.POINTER(apg_uloc_stats)]),
    "apg_unibases_dev": (C.c_int, [_P, C.POINTER(_P)]),
    "apg_ucov_defaults": (None, [C.POINTER(apg_ucov_params)]),
    "apg_unipath_coverage_dev": (
        C.c_int, [_P, C.c_void_p, C.c_uint64, C.POINTER(apg_ucov_params), _u64p, C.POINTER(C.c_double),
                  C.POINTER(C.c_uint32), C.POINTER(apg_ucov_stats)]),
    "apg_unipath_coverage": (
        C.c_int, [_P, C.POINTER(apg_aln_pair), C.c_uint64, C.POINTER(apg_ucov_params), _u64p,
                  C.POINTER(C.c_double), C.POINTER(C.c_uint32), C.POINTER(apg_ucov_stats)]),
    "apg_device_copy": (C.c_int, [_P, C.c_void_p, C.c_void_p, C.c_uint64]),
    "apg_device_alloc": (C.c_int, [_P, C.c_uint64, C.POINTER(C.c_void_p)]),
    "apg_device_free": (None, [_P, C.c_void_p]),
    "apg_device_to_host": (C.c_int, [_P, C.c_void_p, C.c_void_p, C.c_uint64]),
    "apg_dreads_shape": (C.c_int, [_P, _P, _u64p, _u64p, _u64p, _u64p, _u64p]),
    "apg_synth_genome": (C.c_int, [C.c_uint64, C.c_uint64, _u8p]),
    "apg_repeat_defaults": (None, [C.POINTER(apg_repeat_params)]),
    "apg_synth_repeats": (C.c_int, [C.c_uint64, C.c_uint64, C.POINTER(apg_repeat_params), _u8p]),
    "apg_synth_sizes": (C.c_int, [C.POINTER(apg_synth_params), _u64p, _u64p, _u64p]),
    "apg_synth_reads": (C.c_int, [C.POINTER(apg_synth_params), _u8p, _u64p, _u64p, _u8p, _u8p]),
    "apg_synth_layout": (C.c_int, [C.POINTER(apg_synth_params), _u64p, _u32p, C.POINTER(C.c_uint8)]),
    "apg_synth_fragments": (C.c_int, [C.POINTER(apg_synth_params), _u64p, _u64p, _u8p, _u8p]),
    "apg_fastb_write": (C.c_int, [C.c_char_p, C.POINTER(apg_reads)]),
    "apg_qualb_write": (C.c_int, [C.c_char_p, C.POINTER(apg_reads)]),
    "apg_fastb_read": (C.c_int, [C.c_char_p, C.POINTER(apg_reads)]),
    "apg_qualb_read": (C.c_int, [C.c_char_p, C.POINTER(apg_reads)]),
    "apg_reads_release": (None, [C.POINTER(apg_reads)]),
    "apg_reads_load_dev": (C.c_int, [C.c_void_p, C.c_char_p, C.c_char_p, C.c_int, C.POINTER(C.c_void_p)]),
    "apg_kspec_write": (C.c_int, [C.c_char_p, C.c_int, _u64p, C.c_size_t]),
    "apg_kspec_estimate": (C.c_int, [_u64p, C.c_size_t, C.POINTER(apg_kspec_summary)]),
    "apg_solid_write": (C.c_int, [C.c_char_p, C.c_int, _u64p, C.c_uint64]),
    "apg_solid_read": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.POINTER(_u64p), _u64p]),
    "apg_ulocs_write": (C.c_int, [C.c_char_p, C.c_int, C.c_uint64, C.POINTER(apg_aln_pair), C.c_uint64]),
    "apg_ulocs_read": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), _u64p, C.POINTER(C.POINTER(apg_aln_pair)), _u64p]),
    "apg_ucov_write": (C.c_int, [C.c_char_p, C.c_int, C.c_double, C.c_uint64, _u64p, C.POINTER(C.c_double), _u32p]),
    "apg_ucov_read": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_double), _u64p, C.POINTER(_u64p),
                                C.POINTER(C.POINTER(C.c_double)), C.POINTER(_u32p)]),
    "apg_graph_write": (C.c_int, [C.c_char_p, C.POINTER(apg_unipath_graph)]),
    "apg_graph_read": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(apg_unipath_graph)]),
    "apg_kmerpaths_write": (C.c_int, [C.c_char_p, C.c_int, C.c_uint64, _u64p, _u64p, _u64p]),
    "apg_kmerpaths_read": (
        C.c_int, [C.c_char_p, C.POINTER(C.c_int), _u64p, C.POINTER(_u64p), _u64p, C.POINTER(_u64p), C.POINTER(_u64p)]),
    "apg_rc_db_write": (C.c_int, [C.c_char_p, C.c_int, C.POINTER(apg_rc_db)]),
    # communicators + sharded module entry points
    "apg_comm_unique_id": (C.c_int, [_P]),
    "apg_comm_init_rccl": (C.c_int, [_P, _P, C.c_int, C.c_int, C.c_uint32, C.POINTER(_P)]),
    "apg_comm_init_tcp": (C.c_int, [_P, C.c_char_p, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_P)]),
    "apg_comm_destroy": (None, [_P]),
    "apg_comm_abort": (C.c_int, [_P]),
    "apg_comm_rank": (C.c_int, [_P]),
    "apg_comm_world": (C.c_int, [_P]),
    "apg_comm_alltoallv": (C.c_int, [_P, _P, _u64p, _P, _u64p]),
    "apg_comm_allgatherv": (C.c_int, [_P, _P, C.c_uint64, _P, _u64p]),
    "apg_comm_allreduce_u64": (C.c_int, [_P, _u64p, C.c_uint64, C.c_int]),
    "apg_comm_barrier": (C.c_int, [_P]),
    "apg_sharded_spectrum": (C.c_int, [_P, _P, _P, C.c_int, _u64p, C.c_size_t, C.POINTER(apg_kstats)]),
    "apg_sharded_precorrect": (C.c_int, [_P, _P, _P, C.POINTER(apg_pc_params), C.POINTER(apg_pc_stats)]),
    "apg_sharded_spectrum_precorrect": (C.c_int, [_P, _P, _P, C.c_int, _u64p, C.c_size_t, C.POINTER(apg_kstats),
                                                  C.POINTER(apg_pc_params), C.POINTER(apg_pc_stats)]),
    "apg_sharded_fill": (C.c_int, [_P, _P, _P, C.POINTER(apg_fill_params), _P, C.c_uint64, C.POINTER(_P), _P,
                                   C.POINTER(apg_fill_stats)]),
    "apg_sharded_unipaths": (C.c_int, [_P, _P, _P, C.POINTER(apg_unipath_params), C.POINTER(apg_unipath_graph),
                                       C.POINTER(apg_unipath_stats)]),
    "apg_sharded_error_correct_jump": (
        C.c_int, [_P, _P, _P, _P, C.POINTER(apg_ecj_params), C.c_void_p, C.POINTER(apg_ecj_stats)]),
    "apg_sharded_unipath_locs": (
        C.c_int, [_P, _P, _P, C.c_uint32, C.POINTER(C.c_void_p), _u64p, C.POINTER(apg_uloc_stats)]),
    "apg_sharded_consensus": (C.c_int, [_P, _P, _P, _P, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
}

APG_COMM_SELF_P2P = 1
APG_COMM_SUM = 0
APG_COMM_MAX = 1

_lock = threading.Lock()
_lib = None


def lib() -> C.CDLL:
    """Load libapg.so (once).  Raises if it has not been built."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"libapg.so not found at {LIB_PATH}: build it with "
                    "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)"
                )
            handle = C.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
            _lib = handle
    return _lib


def check(rc: int, where: str) -> None:
    if rc != APG_OK:
        msg = lib().apg_last_error()
        raise ApgError(rc, where, msg.decode() if msg else "")
