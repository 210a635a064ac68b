"""libapg's exchange layer on CPU (csrc/exchange.cpp, the TCP transport with
host buffers): world sizes 2 and 4 in separate processes, bytewise checks of
alltoallv / allgatherv / allreduce, a single peer segment above 2^31 bytes,
empty segments, and the errors a size mismatch or a missing peer raise."""
import multiprocessing as mp
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def seg(src: int, dst: int, n: int) -> np.ndarray:
    """The bytes rank src sends to rank dst: deterministic from (src, dst)."""
    return np.random.default_rng(1000 * src + dst).integers(0, 256, n, dtype=np.uint8)


def sizes(world: int, big: int):
    """send sizes [src][dst] (bytes): irregular, some empty; one pair `big`."""
    rng = np.random.default_rng(7)
    s = rng.integers(0, 300_000, (world, world))
    s[rng.random((world, world)) < 0.2] = 0
    if big:
        s[0, 1 % world] = big
    return s


def worker(rank, world, port, big, q):
    sys.path.insert(0, ROOT)
    try:
        from allpathslg_amd.distributed import Comm

        c = Comm.tcp(None, "127.0.0.1", port, rank, world, timeout_ms=120_000)
        S = sizes(world, big)
        send = np.concatenate([seg(rank, d, int(S[rank, d])) for d in range(world)] + [np.zeros(1, np.uint8)])
        recv = np.zeros(int(S[:, rank].sum()) + 1, np.uint8)
        c.alltoallv(send.ctypes.data, S[rank], recv.ctypes.data, S[:, rank])
        off = 0
        ok = True
        for s_ in range(world):
            n = int(S[s_, rank])
            ok &= bool(np.array_equal(recv[off : off + n], seg(s_, rank, n)))
            off += n
        # allgatherv: rank r contributes r*1000 + 17 bytes
        mine = seg(rank, 99, rank * 1000 + 17)
        rb = np.array([r * 1000 + 17 for r in range(world)], np.uint64)
        allg = np.zeros(int(rb.sum()), np.uint8)
        c.allgatherv(mine.ctypes.data, len(mine), allg.ctypes.data, rb)
        exp = np.concatenate([seg(r, 99, r * 1000 + 17) for r in range(world)])
        ok &= bool(np.array_equal(allg, exp))
        tot = c.allreduce([rank + 1, 2**40 + rank], "sum")
        mx = c.allreduce([rank, 5], "max")
        ok &= int(tot[0]) == world * (world + 1) // 2 and int(tot[1]) == world * 2**40 + world * (world - 1) // 2
        ok &= int(mx[0]) == world - 1 and int(mx[1]) == 5
        c.barrier()
        # a receive size that disagrees with the sender's: an error, not a hang
        err = ""
        if world >= 2:
            bad = S[:, rank].copy()
            peer = (rank + 1) % world
            bad[peer] += 1
            recv2 = np.zeros(int(bad.sum()) + 1, np.uint8)
            try:
                c.alltoallv(send.ctypes.data, S[rank], recv2.ctypes.data, bad)
                err = "no error"
            except Exception as e:  # noqa: BLE001
                err = str(e)
        c.close()
        q.put((rank, ok, err))
    except Exception as e:  # noqa: BLE001
        q.put((rank, False, repr(e)))


def run_world(world, big=0, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=worker, args=(r, world, port, big, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = [q.get(timeout=timeout) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    return sorted(out)


@pytest.mark.parametrize("world", [1, 2, 4])
def test_tcp_exchange(world):
    res = run_world(world)
    for rank, ok, err in res:
        assert ok, (rank, err)
        if world >= 2:  # the mismatch (or a peer dropping out over it) is reported
            assert err and err != "no error", err


def test_tcp_exchange_segment_above_2gib():
    """One peer segment of 2^31 + 4097 bytes (0 -> 1): every byte arrives,
    the sizes and offsets are u64 end to end."""
    res = run_world(2, big=(1 << 31) + 4097, timeout=600)
    for rank, ok, err in res:
        assert ok, (rank, err)


def test_tcp_missing_peer_times_out():
    from allpathslg_amd import ApgError
    from allpathslg_amd.distributed import Comm

    with pytest.raises(ApgError):
        Comm.tcp(None, "127.0.0.1", free_port(), 1, 2, timeout_ms=1500)


def abort_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    try:
        import time

        from allpathslg_amd.distributed import Comm

        c = Comm.tcp(None, "127.0.0.1", port, rank, world, timeout_ms=600_000)
        c.barrier()
        t0 = time.time()
        if rank == world - 1:  # a local failure on the last rank
            time.sleep(0.5)
            c.abort()
            try:
                c.barrier()
                err = "no error"
            except Exception as e:  # noqa: BLE001
                err = str(e)
        else:
            try:
                c.barrier()
                err = "no error"
            except Exception as e:  # noqa: BLE001
                err = str(e)
        q.put((rank, time.time() - t0, err))
        c.close()
    except Exception as e:  # noqa: BLE001
        q.put((rank, -1.0, repr(e)))


def test_tcp_abort_releases_peers():
    """apg_comm_abort on one rank (tools/apg_modules.cpp does it before a FATAL
    exit): its peers, blocked in a barrier with it, get an error within seconds
    rather than waiting out the 600 s timeout; the aborted communicator refuses
    further calls."""
    world = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=abort_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for rank, dt, err in out:
        assert err != "no error" and dt >= 0, (rank, err)
        assert dt < 30, (rank, dt, err)
        if rank == world - 1:
            assert "aborted" in err, err
