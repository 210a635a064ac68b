"""Sharded module entry points through the C ABI (include/apg.h
apg_sharded_*), one process per rank, every exchange inside libapg:

  * world 2 and 4: ranks share GPU 0 and talk over the TCP communicator;
    spectrum, PreCorrect (1 and 2 passes), FillFragments, the K=96
    unipath graph + KmerPaths (sharded compaction, and once the replicated
    build), UnipathLocs of the corrected reads, their gap-free hits and the
    consensus of every rank's placements equal the single-GPU entry points
    on the union of the ranks' reads (tests/dist_chain.py; the compaction's
    hard cases: tests/test_sharded_graph.py; genome scale:
    tests/test_distributed_scale.py);
  * world 1 over RCCL with the segment to self routed through ncclSend /
    ncclRecv (APG_COMM_SELF_P2P): the same stages, and one alltoallv of
    2^31 + 4 KiB bytes compared byte for byte (the size at which the old
    torch-level exchange once lost data).
"""
import os
import sys

import numpy as np
import pytest

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from dist_chain import chain, check_against_mono, mono_chain, run_world  # noqa: E402

pytestmark = pytest.mark.gpu

GENOME, PAIRS, SEED = 250_000, 48_000, 0xD157
CFG = (GENOME, PAIRS, SEED)


@pytest.fixture(scope="module")
def mono(gpu_ctx):
    """The single-GPU entry points on the union of the ranks' reads."""
    return {n_cycles: mono_chain(gpu_ctx, CFG, n_cycles) for n_cycles in (1, 2)}


@pytest.mark.parametrize("world,n_cycles,gather,chunk", [(2, 1, False, None), (4, 1, False, 100_003),
                                                         (2, 2, False, None), (2, 1, True, None)])
def test_sharded_chain_tcp_equals_single_gpu(mono, world, n_cycles, gather, chunk):
    """gather=False: sharded unipath compaction; True: the replicated build
    (APG_UNIPATH_GATHER_NODES).  chunk: consensus vote planes of that many
    columns (chunk boundaries inside unipaths)."""
    env = {"APG_CONS_CHUNK": str(chunk)} if chunk else None
    check_against_mono(run_world(CFG, world, n_cycles, gather, env=env), mono[n_cycles], world, PAIRS)


@pytest.mark.parametrize("world,n_cycles,extra", [(2, 1, None), (4, 2, None), (2, 1, {"APG_SK_UP_DD": "0"}),
                                                   (2, 1, {"APG_SK_DEDUP": "none"})])
def test_sharded_fused_spectrum_precorrect_equals_single_gpu(mono, world, n_cycles, extra):
    """apg_sharded_spectrum_precorrect: the K=25 spectrum rides on the K=24
    owner count (one exchange; the records cut to <= 32 bases so the owner's
    partition levels carry them packed); spectrum, corrected reads and
    everything downstream equal the single-GPU entry points on the union.
    extra: the K+1 pass reading every received record instead of the dedup's
    distinct records (APG_SK_UP_DD=0), and no record dedup at all."""
    env = {"APG_TEST_FUSED_SHARDED": "1", **(extra or {})}
    check_against_mono(run_world(CFG, world, n_cycles, env=env), mono[n_cycles], world, PAIRS)


JUMP_PAIRS = 6_000


@pytest.fixture(scope="module")
def mono_jumps(gpu_ctx):
    return mono_chain(gpu_ctx, CFG, 1, placement=False, jump_pairs=JUMP_PAIRS)


@pytest.mark.parametrize("world,extra", [(2, {"APG_TEST_FUSED_SHARDED": "1"}), (4, None),
                                         (2, {"APG_TEST_ECJ_RECOUNT": "1"})])
def test_sharded_error_correct_jump_equals_single_gpu(mono_jumps, world, extra):
    """apg_sharded_error_correct_jump (BASELINE configs[2]/[4]'s jump library
    on N ranks): every rank's corrected and trimmed jump reads equal its slice
    of the single-GPU ErrorCorrectJump of the union — against the replicated
    solid set of the fragments' sharded correction pass, and (RECOUNT) with
    that set dropped, counted across the ranks again."""
    from dist_chain import check_ecj_against_mono

    env = {"APG_CONS_CHUNK": "100003"} if extra is None else dict(extra)
    parts = run_world(CFG, world, 1, placement=False, env=env, jump_pairs=JUMP_PAIRS)
    check_against_mono(parts, mono_jumps, world, PAIRS)
    check_ecj_against_mono(parts, mono_jumps, world, JUMP_PAIRS)


@pytest.fixture(scope="module")
def mono31(gpu_ctx):
    return mono_chain(gpu_ctx, CFG, 1, placement=False, kspec=31)


def test_sharded_fused_fallback_equals_single_gpu(mono31):
    """K_spec != K + 1: apg_sharded_spectrum_precorrect falls back to the two
    sharded entry points (K=31 spectrum exchange, K=24 correction exchange)."""
    env = {"APG_TEST_FUSED_SHARDED": "1", "APG_TEST_KSPEC": "31"}
    check_against_mono(run_world(CFG, 2, 1, placement=False, env=env), mono31, 2, PAIRS)


@pytest.mark.parametrize("fused", [False, True])
def test_sharded_chain_rccl_world1_equals_single_gpu(gpu_ctx, mono, monkeypatch, fused):
    """fused: the bench's N > 1 step entry point (apg_sharded_spectrum_precorrect)."""
    from allpathslg_amd.distributed import Comm, unique_id

    if fused:
        monkeypatch.setenv("APG_TEST_FUSED_SHARDED", "1")
    comm = Comm.rccl(gpu_ctx, unique_id(), 0, 1, self_p2p=True)
    try:
        out = chain(gpu_ctx, comm, mono[1]["reads"], 1)
        check_against_mono([out], mono[1], 1, PAIRS)
    finally:
        comm.close()


def test_rccl_exchange_above_2gib_bytewise(gpu_ctx):
    import torch

    from allpathslg_amd.distributed import Comm, unique_id

    n = (1 << 31) + 4096
    comm = Comm.rccl(gpu_ctx, unique_id(), 0, 1, self_p2p=True)
    try:
        g = torch.Generator(device="cuda")
        g.manual_seed(5)
        src = torch.randint(-(2**31), 2**31 - 1, (n // 4,), dtype=torch.int32, device="cuda", generator=g)
        dst = torch.zeros_like(src)
        torch.cuda.synchronize()
        comm.alltoallv(src.data_ptr(), [n], dst.data_ptr(), [n])
        assert torch.equal(src, dst)
        # the same through allgatherv
        dst.zero_()
        torch.cuda.synchronize()
        comm.allgatherv(src.data_ptr(), n, dst.data_ptr(), [n])
        assert torch.equal(src, dst)
    finally:
        comm.close()


def _mismatch_worker(rank, world, port, q):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        import torch

        from allpathslg_amd import ApgError, Context, ReadSet
        from allpathslg_amd.distributed import Comm, sharded_consensus

        rng = np.random.default_rng(rank)
        T = ReadSet.from_sequences([rng.integers(0, 4, 500) for _ in range(2 + rank)])  # rank 1 holds one more target
        R = ReadSet.from_sequences([rng.integers(0, 4, 100)], [np.full(100, 30)])
        with Context(device=0) as ctx:
            comm = Comm.tcp(ctx, "127.0.0.1", port, rank, world, timeout_ms=120_000)
            dT, dR = ctx.upload(T), ctx.upload(R)
            b = torch.zeros(int(T.base_off[-1]), dtype=torch.uint8, device="cuda")
            qq = torch.zeros_like(b)
            try:
                sharded_consensus(ctx, comm, dR, dT, 0, 0, b.data_ptr(), qq.data_ptr())
                q.put((rank, "no error"))
            except ApgError as e:
                q.put((rank, str(e)))
            comm.close()
    except Exception as e:  # noqa: BLE001
        q.put((rank, "worker failed: " + repr(e)))


def test_sharded_consensus_target_mismatch_fails_every_rank():
    """Ranks holding different target sets all fail at the shape check
    (max and min reduced), none waits in the vote-plane collectives."""
    import multiprocessing as mp

    from dist_chain import free_port

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_mismatch_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all("different target sets" in res[r] for r in range(2)), res
