"""Multi-GPU k-mer spectrum: one process per GPU, canonical k-mers
hash-partitioned across ranks.

  rank r:  local reads --shard_count/shard_scatter--> records grouped by
           (owner shard, L1 group)
           all_to_all(count matrix)        (P x B u64 per rank)
           all_to_all(records)             (the one real exchange; RCCL/xGMI)
           shard_spectrum(received)        (this shard's distinct k-mers)
           all_reduce(spectrum)            (<= 64 Ki u64)

torch.distributed is plumbing here (device buffers + collectives; backend
"nccl" is RCCL on ROCm, "gloo" on CPU for tests); all k-mer compute is in
libapg.  `backend` is any object with shard_count / shard_scatter /
shard_spectrum taking torch tensors — `HipShardBackend` in production; the
CPU tests plug in an oracle-backed one to exercise the exchange logic.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .engine import DEFAULT_HIST_LEN, Context, DeviceReads, shard_bins


class HipShardBackend:
    """libapg's sharded stages on this rank's GPU."""

    record_words = 2  # K <= 32 exchange records: 16-byte super-k-mers

    def __init__(self, ctx: Context):
        self.ctx = ctx
        self.device = torch.device("cuda", ctx.device)

    def alloc(self, n: int) -> torch.Tensor:
        return torch.empty(max(n, 1), dtype=torch.int64, device=self.device)

    def shard_count(self, dreads: DeviceReads, K: int, P: int) -> np.ndarray:
        return self.ctx.shard_count(dreads, K, P)

    def shard_scatter(self, dreads: DeviceReads, K: int, P: int, send: torch.Tensor) -> None:
        torch.cuda.synchronize(self.device)  # libapg runs on its own stream
        self.ctx.shard_scatter(dreads, K, P, send.data_ptr())

    def shard_spectrum(self, recv: torch.Tensor, recv_counts: np.ndarray, K: int, P: int, hist_len: int):
        torch.cuda.synchronize(self.device)
        return self.ctx.shard_spectrum(recv.data_ptr(), recv_counts, K, P, hist_len)

    # correction stages
    def shard_solid(self, recv: torch.Tensor, recv_counts: np.ndarray, K: int, P: int, min_solid: int) -> int:
        torch.cuda.synchronize(self.device)
        return self.ctx.shard_solid(recv.data_ptr(), recv_counts, K, P, min_solid)

    # weak-mask return (apg_shard_scatter_pos / apg_shard_solid_weak / apg_precorrect_weak)
    def shard_scatter_pos(self, dreads: DeviceReads, K: int, P: int, send: torch.Tensor, pos: torch.Tensor) -> None:
        torch.cuda.synchronize(self.device)
        self.ctx.shard_scatter_pos(dreads, K, P, send.data_ptr(), pos.data_ptr())

    def alloc_mask(self, n: int) -> torch.Tensor:
        return torch.empty(max(n, 1), dtype=torch.int32, device=self.device)

    def shard_solid_weak(self, recv: torch.Tensor, recv_counts: np.ndarray, K: int, P: int, min_solid: int,
                         mask: torch.Tensor) -> int:
        torch.cuda.synchronize(self.device)
        return self.ctx.shard_solid_weak(recv.data_ptr(), recv_counts, K, P, min_solid, mask.data_ptr())

    def precorrect_weak(self, dreads: DeviceReads, solid: torch.Tensor, n_solid: int, pos: torch.Tensor,
                        mask: torch.Tensor, n_records: int, prm: dict) -> dict:
        torch.cuda.synchronize(self.device)
        return self.ctx.precorrect_weak(dreads, solid.data_ptr(), n_solid, pos.data_ptr(), mask.data_ptr(), n_records,
                                        **prm)

    def solid_export(self, out: torch.Tensor) -> None:
        torch.cuda.synchronize(self.device)
        self.ctx.solid_export(out.data_ptr())

    def precorrect_solid(self, dreads: DeviceReads, solid: torch.Tensor, n_solid: int, prm: dict) -> dict:
        torch.cuda.synchronize(self.device)
        return self.ctx.precorrect_solid(dreads, solid.data_ptr(), n_solid, **prm)

    def fill(self, dreads: DeviceReads, solid: torch.Tensor, n_solid: int, prm: dict, out=None,
             last_solid: bool = False):
        """last_solid: `solid` is the set the last correction pass on this
        context used — reuse its extension table and clean flags."""
        torch.cuda.synchronize(self.device)
        if last_solid:
            filled, _, st = self.ctx.fill_fragments(dreads, K=prm["K"], min_insert=prm["min_insert"],
                                                    max_insert=prm["max_insert"], max_steps=prm["max_steps"],
                                                    last_solid=True, out=out)
        else:
            filled, _, st = self.ctx.fill_fragments(dreads, (solid.data_ptr(), n_solid), out=out, **prm)
        return filled, st

    # unipath stages
    def ushard_count(self, dreads: DeviceReads, K: int, P: int) -> Tuple[np.ndarray, int]:
        return self.ctx.ushard_count(dreads, K, P)

    def ushard_scatter(self, dreads: DeviceReads, K: int, P: int, send: torch.Tensor) -> None:
        torch.cuda.synchronize(self.device)
        self.ctx.ushard_scatter(dreads, K, P, send.data_ptr())

    def ushard_nodes(self, recv: torch.Tensor, recv_counts: np.ndarray, K: int, P: int) -> int:
        torch.cuda.synchronize(self.device)
        return self.ctx.ushard_nodes(recv.data_ptr(), recv_counts, K, P)

    def ushard_export(self, out: torch.Tensor) -> None:
        torch.cuda.synchronize(self.device)
        self.ctx.ushard_export(out.data_ptr())

    # minimizer-partition records (apg_urec_*)
    urec_words = 6  # 48-byte super-k-mer records

    def urec_count(self, dreads: DeviceReads, K: int, P: int) -> Tuple[np.ndarray, int]:
        return self.ctx.urec_count(dreads, K, P)

    def urec_scatter(self, dreads: DeviceReads, K: int, P: int, send: torch.Tensor) -> None:
        torch.cuda.synchronize(self.device)
        self.ctx.urec_scatter(dreads, K, P, send.data_ptr())

    def urec_nodes(self, recv: torch.Tensor, recv_counts: np.ndarray, K: int, P: int) -> int:
        torch.cuda.synchronize(self.device)
        return self.ctx.urec_nodes(recv.data_ptr(), recv_counts, K, P)

    def urec_export(self, out: torch.Tensor) -> None:
        torch.cuda.synchronize(self.device)
        self.ctx.urec_export(out.data_ptr())

    def graph_from_nodes(self, nodes: torch.Tensor, n_nodes: int, dreads, K: int, fetch: bool):
        torch.cuda.synchronize(self.device)
        return self.ctx.unipaths_from_nodes(nodes.data_ptr(), n_nodes, dreads, K, read_paths=True, fetch=fetch)


# Largest message per peer per collective call, in int64 elements (256 MiB).
# Single RCCL all_to_all messages around 1 GiB were observed to deliver only
# part of the data on this stack (sharded unipath exchange, 2 GB to self: the
# second half arrived as zeros), so every bulk exchange is cut into rounds.
CHUNK_ELEMS = 1 << 25


def _rounds(n_max: int, group, dev) -> int:
    """Number of chunk rounds every rank agrees on."""
    r = torch.tensor([(n_max + CHUNK_ELEMS - 1) // CHUNK_ELEMS], dtype=torch.int64, device=dev)
    dist.all_reduce(r, op=dist.ReduceOp.MAX, group=group)
    return int(r.item())


def all_to_all_chunked(recv: torch.Tensor, send: torch.Tensor, out_splits, in_splits, group=None) -> None:
    """all_to_all_single(recv, send, out_splits, in_splits) in rounds of at
    most CHUNK_ELEMS elements per peer, as grouped point-to-point transfers
    straight between the peer segments of send and recv (no staging copies;
    the segment to self is one local copy).  Round r moves elements
    [r*C, (r+1)*C) of every peer segment.  APG_A2A=collective selects staged
    all_to_all_single rounds instead."""
    C = CHUNK_ELEMS
    P = len(in_splits)
    me = dist.get_rank(group)
    in_off = np.concatenate([[0], np.cumsum(in_splits)]).astype(np.int64)
    out_off = np.concatenate([[0], np.cumsum(out_splits)]).astype(np.int64)
    if int(in_splits[me]) != int(out_splits[me]):
        raise ValueError("all_to_all_chunked: the segment to self must have equal send and receive sizes")
    R = _rounds(max(max(in_splits), max(out_splits), 0), group, send.device)
    if os.environ.get("APG_A2A", "p2p") == "collective":  # staged all_to_all_single rounds
        for r in range(R):
            lo = r * C
            ins = [int(min(max(in_splits[d] - lo, 0), C)) for d in range(P)]
            outs = [int(min(max(out_splits[q] - lo, 0), C)) for q in range(P)]
            pieces = [send[int(in_off[d]) + lo : int(in_off[d]) + lo + ins[d]] for d in range(P) if ins[d]]
            sbuf = torch.cat(pieces) if pieces else send.new_empty(0)
            rbuf = recv.new_empty(sum(outs))
            dist.all_to_all_single(rbuf, sbuf, outs, ins, group=group)
            pos = 0
            for q in range(P):
                if outs[q]:
                    recv[int(out_off[q]) + lo : int(out_off[q]) + lo + outs[q]].copy_(rbuf[pos : pos + outs[q]])
                    pos += outs[q]
        return
    peer = (lambda q: q) if group is None else (lambda q: dist.get_global_rank(group, q))
    for r in range(R):
        lo = r * C
        ops = []
        for q in range(P):
            ni = int(min(max(in_splits[q] - lo, 0), C))
            no = int(min(max(out_splits[q] - lo, 0), C))
            if q == me:
                if ni:
                    recv[int(out_off[q]) + lo : int(out_off[q]) + lo + ni].copy_(
                        send[int(in_off[q]) + lo : int(in_off[q]) + lo + ni])
                continue
            if ni:
                ops.append(dist.P2POp(dist.isend, send[int(in_off[q]) + lo : int(in_off[q]) + lo + ni], peer(q), group))
            if no:
                ops.append(dist.P2POp(dist.irecv, recv[int(out_off[q]) + lo : int(out_off[q]) + lo + no], peer(q), group))
        if ops:
            for req in dist.batch_isend_irecv(ops):
                req.wait()


def all_gather_var(local: torch.Tensor, n_local: int, group=None):
    """Concatenation over ranks (rank order) of each rank's first n_local
    elements of `local`, gathered in rounds of at most CHUNK_ELEMS per rank.
    Returns (tensor, sizes)."""
    P = dist.get_world_size(group)
    dev = local.device
    sizes_t = torch.tensor([n_local], dtype=torch.int64, device=dev)
    all_sizes = [torch.empty_like(sizes_t) for _ in range(P)]
    dist.all_gather(all_sizes, sizes_t, group=group)
    sizes = [int(x.item()) for x in all_sizes]
    out = local.new_empty(max(sum(sizes), 1))
    off = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    C = CHUNK_ELEMS
    R = _rounds(max(sizes), group, dev)
    for r in range(R):
        lo = r * C
        m = min(C, max(max(sizes) - lo, 0))
        part = local.new_zeros(m)
        mine = min(max(n_local - lo, 0), m)
        if mine:
            part[:mine].copy_(local[lo : lo + mine])
        buf = local.new_empty(m * P)
        dist.all_gather_into_tensor(buf, part, group=group)
        for q in range(P):
            k = min(max(sizes[q] - lo, 0), m)
            if k:
                out[int(off[q]) + lo : int(off[q]) + lo + k].copy_(buf[q * m : q * m + k])
    return out[: sum(sizes)], sizes


def _exchange_kmers(backend, reads, K: int, P: int, group, pos=None):
    """K <= 32 records of this rank's reads -> their owner shards.  A record
    is backend.record_words int64 words (libapg: 16-byte super-k-mers).
    pos: a one-element list to receive the sent records' base positions
    (weak-mask return); the record splits are then appended to it.
    Returns (recv tensor, recv_counts [src * B + l1], records sent, received)."""
    B = shard_bins(K, P)
    W = getattr(backend, "record_words", 1)
    dev = backend.alloc(1).device
    counts = backend.shard_count(reads, K, P)  # [dest * B + l1]
    send = backend.alloc(W * int(counts.sum()))
    if pos is not None:
        pos[0] = backend.alloc(int(counts.sum()))
        backend.shard_scatter_pos(reads, K, P, send, pos[0])
    else:
        backend.shard_scatter(reads, K, P, send)

    cnt_t = torch.from_numpy(counts.astype(np.int64)).to(dev)
    recv_cnt_t = torch.empty_like(cnt_t)
    dist.all_to_all_single(recv_cnt_t, cnt_t, group=group)  # equal splits of B
    recv_counts = recv_cnt_t.cpu().numpy().astype(np.uint64)  # [src * B + l1]

    in_splits = (counts.reshape(P, B).sum(axis=1) * W).astype(np.int64).tolist()
    out_splits = (recv_counts.reshape(P, B).sum(axis=1) * W).astype(np.int64).tolist()
    recv = backend.alloc(int(sum(out_splits)))
    n_in, n_out = int(sum(in_splits)) // W, int(sum(out_splits)) // W
    all_to_all_chunked(recv, send, out_splits, in_splits, group=group)
    if pos is not None:
        pos.append([x // W for x in in_splits])
        pos.append([x // W for x in out_splits])
    return recv, recv_counts, n_in, n_out


def _check_pow2(P: int) -> None:
    if P & (P - 1):
        raise ValueError(f"world size {P} must be a power of two (k-mer hash shards)")


def sharded_spectrum(backend, reads, K: int, hist_len: int = DEFAULT_HIST_LEN,
                     group: Optional[dist.ProcessGroup] = None) -> Tuple[np.ndarray, dict]:
    """Global spectrum of the union of every rank's reads.  Returns the same
    (hist, stats) on every rank; stats are summed over ranks."""
    P = dist.get_world_size(group)
    _check_pow2(P)
    dev = backend.alloc(1).device
    recv, recv_counts, n_in, n_out = _exchange_kmers(backend, reads, K, P, group)
    hist, st = backend.shard_spectrum(recv, recv_counts, K, P, hist_len)
    hist_t = torch.from_numpy(hist.astype(np.int64)).to(dev)
    dist.all_reduce(hist_t, group=group)
    keys = ["n_kmers", "n_distinct", "n_overflow"]
    st_t = torch.tensor([int(st[k]) for k in keys], dtype=torch.int64, device=dev)
    dist.all_reduce(st_t, group=group)
    out = dict(st)
    out.update({k: int(v) for k, v in zip(keys, st_t.cpu().tolist())})
    out["n_shards"] = P
    out["records_sent"] = n_in
    out["records_received"] = n_out
    return hist_t.cpu().numpy().astype(np.uint64), out


def sharded_precorrect(backend, reads, K: int = 24, min_solid: int = 3, max_q_suspect: int = 20, n_cycles: int = 1,
                       group: Optional[dist.ProcessGroup] = None, keep_solid: bool = False):
    """PreCorrect / FindErrors over every rank's reads: per pass,
    K-mers are counted on their owner shards, each shard's solid set is
    all_gathered (the replicated solid set), and every rank corrects its own
    reads in place.  Returns stats summed over ranks (n_solid = global); with
    keep_solid, (stats, solid tensor, n_solid) — the last pass's replicated
    solid set, for sharded_fill."""
    P = dist.get_world_size(group)
    _check_pow2(P)
    dev = backend.alloc(1).device
    tot = {"n_suspect": 0, "n_corrected": 0, "n_ambiguous": 0, "n_uncorrectable": 0, "n_solid": 0}
    weak = hasattr(backend, "shard_solid_weak") and 9 <= K <= 29
    prm = {"K": K, "min_solid": min_solid, "max_q_suspect": max_q_suspect}
    for _ in range(n_cycles):
        if weak:
            # weak-mask return: owners report the weak K-mers of every record
            # they received, so the correction needs no weak-test lookups
            pos = [None]
            recv, recv_counts, n_in, n_out = _exchange_kmers(backend, reads, K, P, group, pos=pos)
            rmask = backend.alloc_mask(n_out)
            n_local = backend.shard_solid_weak(recv, recv_counts, K, P, min_solid, rmask)
            del recv
            smask = backend.alloc_mask(n_in)
            all_to_all_chunked(smask, rmask, pos[1], pos[2], group=group)  # splits reversed
            del rmask
        else:
            recv, recv_counts, _, _ = _exchange_kmers(backend, reads, K, P, group)
            n_local = backend.shard_solid(recv, recv_counts, K, P, min_solid)
            del recv
        local = backend.alloc(n_local)
        backend.solid_export(local)
        solid, sizes = all_gather_var(local, n_local, group=group)
        del local
        if weak:
            st = backend.precorrect_weak(reads, solid, sum(sizes), pos[0], smask, n_in, prm)
            del smask, pos
        else:
            st = backend.precorrect_solid(reads, solid, sum(sizes), prm)
        for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable"):
            tot[k] += int(st[k])
        tot["n_solid"] = sum(sizes)
    keys = ["n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable"]
    st_t = torch.tensor([tot[k] for k in keys], dtype=torch.int64, device=dev)
    dist.all_reduce(st_t, group=group)
    tot.update({k: int(v) for k, v in zip(keys, st_t.cpu().tolist())})
    return (tot, solid, tot["n_solid"]) if keep_solid else tot


FILL_KEYS = ("n_pairs", "n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip", "filled_bases")


def sharded_fill(backend, reads, solid, n_solid: int, K: int = 24, min_insert: int = 126, max_insert: int = 234,
                 max_steps: int = 1024, out=None, group: Optional[dist.ProcessGroup] = None,
                 last_solid: bool = False):
    """FillFragments on every rank's own pairs (ranks hold whole pairs)
    against the replicated solid set of sharded_precorrect(keep_solid=True):
    no exchange ("reads sharded, no exchange").  Returns this
    rank's filled fragments and the stats summed over ranks.  last_solid:
    `solid` is what the last correction pass on this rank's context used
    (sharded_precorrect(keep_solid=True) right before) — its extension table
    and per-read clean flags are reused."""
    prm = {"K": K, "min_insert": min_insert, "max_insert": max_insert, "max_steps": max_steps}
    if last_solid:
        filled, st = backend.fill(reads, solid, n_solid, prm, out, last_solid=True)
    else:
        filled, st = backend.fill(reads, solid, n_solid, prm, out)
    dev = backend.alloc(1).device
    t = torch.tensor([int(st[k]) for k in FILL_KEYS], dtype=torch.int64, device=dev)
    dist.all_reduce(t, group=group)
    tot = dict(st)
    tot.update({k: int(v) for k, v in zip(FILL_KEYS, t.cpu().tolist())})
    tot["n_solid"] = n_solid
    return filled, tot


def sharded_unipaths(backend, reads, K: int = 96, group: Optional[dist.ProcessGroup] = None,
                     fetch: bool = False):
    """Global unipath graph of every rank's reads ("shard the
    counting, replicate the compaction"):

      rank r: reads -> 48-byte super-k-mer records by minimizer shard
              (urec_*; backends without them: distinct local nodes, 32 B)
              all_to_all(records)          records of this shard's K-mers
              urec_nodes                   this shard's distinct nodes
              all_gather(nodes)            the full node set on every rank
              unipaths_from_nodes          graph (identical on every rank) +
                                           KmerPaths of this rank's reads

    Returns (graph dict or None, stats); graph stats are per rank (identical),
    n_instances is summed over ranks."""
    P = dist.get_world_size(group)
    if P & (P - 1) or P > 32:
        raise ValueError(f"world size {P} must be a power of two <= 32")
    # minimizer-partition records (48-byte super-k-mers, P <= 8) when the
    # backend has them, else distinct local nodes (32-byte records)
    rec = hasattr(backend, "urec_count") and P <= 8
    B = 32 if rec else 32 // P
    W = getattr(backend, "urec_words", 6) if rec else 4
    dev = backend.alloc(1).device
    if rec:
        counts, n_inst = backend.urec_count(reads, K, P)  # [dest * 32 + digit]
    else:
        counts, n_inst = backend.ushard_count(reads, K, P)  # [dest * B + group]
    n_send = int(counts.sum())
    send = backend.alloc(W * n_send)
    if rec:
        backend.urec_scatter(reads, K, P, send)
    else:
        backend.ushard_scatter(reads, K, P, send)

    cnt_t = torch.from_numpy(counts.astype(np.int64)).to(dev)
    recv_cnt_t = torch.empty_like(cnt_t)
    dist.all_to_all_single(recv_cnt_t, cnt_t, group=group)
    recv_counts = recv_cnt_t.cpu().numpy().astype(np.uint64)  # [src * B + group]
    in_splits = (counts.reshape(P, B).sum(axis=1) * W).astype(np.int64).tolist()
    out_splits = (recv_counts.reshape(P, B).sum(axis=1) * W).astype(np.int64).tolist()
    n_in, n_out = int(sum(in_splits)), int(sum(out_splits))
    recv = backend.alloc(n_out)
    all_to_all_chunked(recv, send, out_splits, in_splits, group=group)
    del send

    if rec:
        n_local = backend.urec_nodes(recv, recv_counts, K, P)
    else:
        n_local = backend.ushard_nodes(recv, recv_counts, K, P)
    del recv
    local = backend.alloc(4 * n_local)
    if rec:
        backend.urec_export(local)
    else:
        backend.ushard_export(local)
    nodes, sizes4 = all_gather_var(local, 4 * n_local, group=group)
    del local
    graph, st = backend.graph_from_nodes(nodes, sum(sizes4) // 4, reads, K, fetch)
    inst = torch.tensor([n_inst], dtype=torch.int64, device=dev)
    dist.all_reduce(inst, group=group)
    st = dict(st)
    st["n_instances"] = int(inst.item())
    st["n_shards"] = P
    return (graph, st) if fetch else st
