"""allpathslg_amd — MI355X-native k-mer spectrum / correction / unipath engine.

The compute lives in libapg.so (HIP kernels for gfx950 behind the C ABI of
include/apg.h).  This package is the Python host layer used by tests, the
benchmark and the multi-GPU driver.
"""
from ._lib import ApgError, lib  # noqa: F401
from .engine import (  # noqa: F401
    DEFAULT_HIST_LEN, Context, DeviceReads, kmer_hash, kmer_unhash, kspec_estimate, read_graph, read_kmerpaths,
    read_solid, read_unilocs, read_unipath_coverage, shard_bins, write_graph, write_kspec, write_rc_db)
from .reads import ReadSet, synth_fragments, synth_genome, synth_layout, synth_reads  # noqa: F401

__all__ = [
    "ApgError",
    "Context",
    "DeviceReads",
    "DEFAULT_HIST_LEN",
    "ReadSet",
    "kmer_hash",
    "kmer_unhash",
    "lib",
    "shard_bins",
    "synth_genome",
    "synth_reads",
    "synth_fragments",
    "synth_layout",
    "read_graph",
    "read_kmerpaths",
    "kspec_estimate",
    "read_solid",
    "read_unilocs",
    "read_unipath_coverage",
    "write_graph",
    "write_kspec",
    "write_rc_db",
]
