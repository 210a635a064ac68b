"""Multi-GPU host mirror: one process per GPU, every exchange inside libapg.

The sharded module entry points (include/apg.h apg_sharded_*) run the whole
exchange — super-k-mer records to their owner shards, weak masks back, solid
sets and node sets gathered, spectra and counters summed — through a libapg
communicator (csrc/exchange.cpp):

  Comm.rccl(ctx, uid, rank, world)   RCCL over xGMI (device buffers); every
                                     rank passes the same 128-byte id from
                                     unique_id(), made on one rank
  Comm.tcp(ctx, addr, port, rank, world)
                                     host sockets; several ranks may share a
                                     GPU (the multi-process tests)

Nothing here imports torch or moves data: these are ctypes calls that mirror
the C ABI, like engine.py does for the single-GPU entry points.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Tuple

import numpy as np

from ._lib import (APG_COMM_MAX, APG_COMM_SELF_P2P, APG_COMM_SUM, apg_fill_stats, apg_kstats, apg_pc_stats,
                   apg_unipath_graph, apg_unipath_params, apg_unipath_stats, check, lib)
from .engine import DEFAULT_HIST_LEN, Context, DeviceReads, graph_arrays

_u64p = C.POINTER(C.c_uint64)


def unique_id() -> bytes:
    """A fresh RCCL communicator id (128 bytes), made on one rank and passed
    to every rank by the launcher."""
    buf = C.create_string_buffer(128)
    check(lib().apg_comm_unique_id(buf), "apg_comm_unique_id")
    return buf.raw


class Comm:
    """A libapg communicator (apg_comm): this rank's view of a sharded run."""

    def __init__(self, handle: C.c_void_p, ctx: Optional[Context]):
        self._h = handle
        self.ctx = ctx
        self.rank = int(lib().apg_comm_rank(handle))
        self.world = int(lib().apg_comm_world(handle))

    @classmethod
    def rccl(cls, ctx: Context, uid: bytes, rank: int, world: int, self_p2p: bool = False) -> "Comm":
        h = C.c_void_p()
        buf = C.create_string_buffer(uid, 128)
        check(lib().apg_comm_init_rccl(ctx.handle, buf, rank, world, APG_COMM_SELF_P2P if self_p2p else 0,
                                       C.byref(h)), "apg_comm_init_rccl")
        return cls(h, ctx)

    @classmethod
    def tcp(cls, ctx: Optional[Context], addr: str, port: int, rank: int, world: int,
            timeout_ms: int = 0) -> "Comm":
        """ctx=None: a host-memory communicator (buffers are host memory)."""
        h = C.c_void_p()
        check(lib().apg_comm_init_tcp(ctx.handle if ctx is not None else None, addr.encode(), port, rank, world,
                                      timeout_ms, C.byref(h)), "apg_comm_init_tcp")
        return cls(h, ctx)

    @property
    def handle(self):
        return self._h

    def abort(self) -> None:
        """After a local failure: peers blocked in a collective with this rank
        error out instead of waiting (apg_comm_abort)."""
        check(lib().apg_comm_abort(self._h), "apg_comm_abort")

    def close(self):
        if self._h:
            lib().apg_comm_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- primitives (pointers: device memory for a ctx communicator, host
    #    memory otherwise) --------------------------------------------------
    def alltoallv(self, send_ptr: int, send_bytes, recv_ptr: int, recv_bytes) -> None:
        sb = np.ascontiguousarray(send_bytes, dtype=np.uint64)
        rb = np.ascontiguousarray(recv_bytes, dtype=np.uint64)
        check(lib().apg_comm_alltoallv(self._h, C.c_void_p(send_ptr), sb.ctypes.data_as(_u64p),
                                       C.c_void_p(recv_ptr), rb.ctypes.data_as(_u64p)), "apg_comm_alltoallv")

    def allgatherv(self, send_ptr: int, send_bytes: int, recv_ptr: int, recv_bytes) -> None:
        rb = np.ascontiguousarray(recv_bytes, dtype=np.uint64)
        check(lib().apg_comm_allgatherv(self._h, C.c_void_p(send_ptr), send_bytes, C.c_void_p(recv_ptr),
                                        rb.ctypes.data_as(_u64p)), "apg_comm_allgatherv")

    def allreduce(self, values, op: str = "sum") -> np.ndarray:
        v = np.array(values, dtype=np.uint64).reshape(-1)
        check(lib().apg_comm_allreduce_u64(self._h, v.ctypes.data_as(_u64p), len(v),
                                           APG_COMM_MAX if op == "max" else APG_COMM_SUM), "apg_comm_allreduce_u64")
        return v

    def barrier(self) -> None:
        check(lib().apg_comm_barrier(self._h), "apg_comm_barrier")


# -- sharded module entry points ----------------------------------------------
def sharded_spectrum(ctx: Context, comm: Comm, reads: DeviceReads, K: int,
                     hist_len: int = DEFAULT_HIST_LEN) -> Tuple[np.ndarray, dict]:
    """The global spectrum of every rank's reads (same on every rank)."""
    hist = np.zeros(hist_len, dtype=np.uint64)
    st = apg_kstats()
    check(lib().apg_sharded_spectrum(ctx.handle, comm.handle, reads.handle, K, hist.ctypes.data_as(_u64p), hist_len,
                                     C.byref(st)), "apg_sharded_spectrum")
    out = st.as_dict()
    out["n_shards"] = comm.world
    return hist, out


def sharded_precorrect(ctx: Context, comm: Comm, reads: DeviceReads, K: int = 24, min_solid: int = 3,
                       max_q_suspect: int = 20, n_cycles: int = 1) -> dict:
    """PreCorrect (n_cycles=1) / FindErrors (2) of every rank's reads in place
    against the global solid set, which stays on ctx for
    sharded_fill(last_solid=True)."""
    p = ctx.pc_params(K, min_solid, max_q_suspect, n_cycles)
    st = apg_pc_stats()
    check(lib().apg_sharded_precorrect(ctx.handle, comm.handle, reads.handle, C.byref(p), C.byref(st)),
          "apg_sharded_precorrect")
    return st.as_dict()


def sharded_spectrum_precorrect(ctx: Context, comm: Comm, reads: DeviceReads, K_spec: int = 25, K: int = 24,
                                min_solid: int = 3, max_q_suspect: int = 20, n_cycles: int = 1,
                                hist_len: int = DEFAULT_HIST_LEN) -> Tuple[np.ndarray, dict, dict]:
    """sharded_spectrum(K_spec) of the uncorrected reads and
    sharded_precorrect(K) from one exchange of K-records
    (apg_sharded_spectrum_precorrect; K_spec = K + 1 fuses, else the two in
    turn).  Returns (hist, spectrum stats, PreCorrect stats)."""
    hist = np.zeros(hist_len, dtype=np.uint64)
    kst = apg_kstats()
    p = ctx.pc_params(K, min_solid, max_q_suspect, n_cycles)
    pst = apg_pc_stats()
    check(lib().apg_sharded_spectrum_precorrect(ctx.handle, comm.handle, reads.handle, K_spec,
                                                hist.ctypes.data_as(_u64p), hist_len, C.byref(kst), C.byref(p),
                                                C.byref(pst)), "apg_sharded_spectrum_precorrect")
    out = kst.as_dict()
    out["n_shards"] = comm.world
    return hist, out, pst.as_dict()


def sharded_fill(ctx: Context, comm: Comm, reads: DeviceReads, K: int = 24, min_insert: int = 126,
                 max_insert: int = 234, max_steps: int = 1024, last_solid: bool = True, out=None,
                 d_status: Optional[int] = None):
    """FillFragments of this rank's pairs (no exchange); stats summed.
    Returns (this rank's filled fragments, stats)."""
    p = ctx.fill_params(K, min_insert, max_insert, max_steps, 3, last_solid)
    st = apg_fill_stats()
    fd = out if out is not None else DeviceReads(ctx, None)
    check(lib().apg_sharded_fill(ctx.handle, comm.handle, reads.handle, C.byref(p), None, 0, C.byref(fd._h),
                                 C.c_void_p(d_status) if d_status else None, C.byref(st)), "apg_sharded_fill")
    return fd, st.as_dict()


def sharded_unipaths(ctx: Context, comm: Comm, reads: DeviceReads, K: int = 96, read_paths: bool = True,
                     fetch: bool = False, gather_nodes: bool = False):
    """The global unipath graph (identical on every rank) + KmerPaths of this
    rank's reads.  Default: sharded compaction (no rank holds every node);
    gather_nodes=True: every rank gathers all nodes and builds the whole graph.
    Returns (graph dict or None, stats)."""
    from ._lib import APG_UNIPATH_GATHER_NODES, APG_UNIPATH_READ_PATHS

    p = apg_unipath_params()
    lib().apg_unipath_defaults(C.byref(p))
    p.K = K
    p.flags = (APG_UNIPATH_READ_PATHS if read_paths else 0) | (APG_UNIPATH_GATHER_NODES if gather_nodes else 0)
    g = apg_unipath_graph()
    st = apg_unipath_stats()
    check(lib().apg_sharded_unipaths(ctx.handle, comm.handle, reads.handle, C.byref(p),
                                     C.byref(g) if fetch else None, C.byref(st)), "apg_sharded_unipaths")
    out = st.as_dict()
    out["n_shards"] = comm.world
    if not fetch:
        return None, out
    try:
        return graph_arrays(g), out
    finally:
        lib().apg_unipath_graph_free(C.byref(g))


def sharded_error_correct_jump(ctx: Context, comm: Comm, frags: DeviceReads, jumps: DeviceReads, d_keep: int,
                               K: int = 24, min_solid: int = 3, max_q_suspect: int = 20, min_keep: int = 40) -> dict:
    """ErrorCorrectJump of this rank's jump reads against the global solid set
    of every rank's fragment reads (include/apg.h
    apg_sharded_error_correct_jump): the replicated set of their sharded
    correction pass when `frags` are its output, else counted across the
    ranks.  Jumps corrected in place, keep lengths into device d_keep (u32
    per read); stats summed over ranks."""
    from ._lib import apg_ecj_params, apg_ecj_stats

    p = apg_ecj_params()
    lib().apg_ecj_defaults(C.byref(p))
    p.K, p.min_solid, p.max_q_suspect, p.min_keep = K, min_solid, max_q_suspect, min_keep
    st = apg_ecj_stats()
    check(lib().apg_sharded_error_correct_jump(ctx.handle, comm.handle, frags.handle, jumps.handle, C.byref(p),
                                               C.c_void_p(d_keep), C.byref(st)), "apg_sharded_error_correct_jump")
    return st.as_dict()


def sharded_unipath_locs(ctx: Context, comm: Comm, reads: DeviceReads, rc: bool = True, sorted: bool = True):
    """UnipathLocs of this rank's reads on the global graph of the last
    sharded_unipaths on ctx (include/apg.h apg_sharded_unipath_locs): every
    K-mer this rank does not own is resolved by one query to its owner shard.
    Returns (device pointer to n apg_aln_pair, n, stats summed over ranks);
    s_id = the read's index in `reads`; valid until the next locs call."""
    from ._lib import APG_ULOCS_RC, APG_ULOCS_SORTED, apg_uloc_stats

    flags = (APG_ULOCS_RC if rc else 0) | (APG_ULOCS_SORTED if sorted else 0)
    st = apg_uloc_stats()
    n = C.c_uint64(0)
    p = C.c_void_p()
    check(lib().apg_sharded_unipath_locs(ctx.handle, comm.handle, reads.handle, flags, C.byref(p), C.byref(n),
                                         C.byref(st)), "apg_sharded_unipath_locs")
    return int(p.value or 0), int(n.value), st.as_dict()


def sharded_consensus(ctx: Context, comm: Comm, R: DeviceReads, T: DeviceReads, d_placements: int, n: int,
                      d_bases: int, d_quals: int) -> None:
    """Column consensus of every rank's placements on the replicated targets
    T (include/apg.h apg_sharded_consensus): the vote planes are summed over
    the ranks; every rank gets every column (device outputs, T.n_bases each)."""
    check(lib().apg_sharded_consensus(ctx.handle, comm.handle, R.handle, T.handle, C.c_void_p(d_placements), n,
                                      C.c_void_p(d_bases), C.c_void_p(d_quals)), "apg_sharded_consensus")
