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


@pytest.mark.parametrize("world,n_cycles", [(2, 1), (4, 2)])
def test_sharded_fused_spectrum_precorrect_equals_single_gpu(mono, world, n_cycles):
    """apg_sharded_spectrum_precorrect: the K=25 spectrum rides on the K=24
    owner count (one exchange); spectrum, corrected reads and everything
    downstream equal the single-GPU entry points on the union."""
    check_against_mono(run_world(CFG, world, n_cycles, env={"APG_TEST_FUSED_SHARDED": "1"}), mono[n_cycles], world,
                       PAIRS)


def test_sharded_chain_rccl_world1_equals_single_gpu(gpu_ctx, mono):
    from allpathslg_amd.distributed import Comm, unique_id

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
