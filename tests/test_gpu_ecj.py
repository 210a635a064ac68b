"""GPU parity: ErrorCorrectJump (apg_error_correct_jump) from libapg's HIP
kernels vs the restatement (oracle precorrect_solid + ecj_oracle.c) — exact
equality of corrected bases, qualities, keep lengths and counters."""
import numpy as np
import pytest
import torch

import oracle
from allpathslg_amd import ReadSet, synth_genome, synth_reads
from tests.test_ecj_oracle import frag_set, read_with

pytestmark = pytest.mark.gpu


def run(ctx, frags, jumps, **kw):
    got, keep, st = ctx.error_correct_jump(frags, jumps, **kw)
    exp, ekeep, est = oracle.error_correct_jump(frags, jumps, **kw)
    assert np.array_equal(got.packed[: exp.byte_off[-1]], exp.packed[: exp.byte_off[-1]])
    assert np.array_equal(got.quals, exp.quals)
    if not np.array_equal(keep, ekeep):
        bad = np.nonzero(keep != ekeep)[0][:5]
        raise AssertionError(f"keep differs at {bad.tolist()}: got {keep[bad]} expected {ekeep[bad]}")
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert st["precorrect"][k] == est[k], (k, st["precorrect"][k], est[k])
    assert st["n_full"] + st["n_trimmed"] + st["n_dropped"] == jumps.n_reads
    assert st["bases_kept"] == int(ekeep.sum())
    return keep, st


def test_kats(gpu_ctx):
    g, frags = frag_set()
    cases = [read_with(g, 1000, [50], q_err=10), read_with(g, 2000, [70], q_err=40),
             read_with(g, 3000, [10], q_err=40), read_with(g, 4000, [])]
    keep, _ = run(gpu_ctx, frags, ReadSet.from_sequences([c[0] for c in cases], [c[1] for c in cases]), K=24)
    assert keep.tolist() == [100, 70, 0, 100]


@pytest.mark.parametrize("K,min_keep", [(24, 40), (20, 30), (27, 60)])
def test_synthetic_libraries(gpu_ctx, K, min_keep):
    g = synth_genome(200_000, 9)
    frags = synth_reads(g, 40_000, seed=10)                                   # 40x frag pairs
    jumps = synth_reads(g, 6_000, seed=11, insert_mean=3000, insert_sd=300)   # 3 kb jumps
    keep, st = run(gpu_ctx, frags, jumps, K=K, min_keep=min_keep)
    assert st["n_full"] > 0.5 * jumps.n_reads and st["n_trimmed"] > 0


def test_device_variant_and_empty(gpu_ctx):
    g = synth_genome(100_000, 4)
    frags = synth_reads(g, 20_000, seed=5)
    jumps = synth_reads(g, 2_000, seed=6, insert_mean=3000, insert_sd=300)
    _, hkeep, _ = gpu_ctx.error_correct_jump(frags, jumps)
    dF, dJ = gpu_ctx.upload(frags), gpu_ctx.upload(jumps)
    dk = torch.empty(jumps.n_reads, dtype=torch.int32, device="cuda")
    st = gpu_ctx.error_correct_jump(dF, dJ, d_keep=dk.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(dk.cpu().numpy().view(np.uint32), hkeep)
    assert st["n_reads"] == jumps.n_reads
    dF.free()
    dJ.free()
    _, keep, st = gpu_ctx.error_correct_jump(frags, ReadSet.from_sequences([], []))
    assert len(keep) == 0 and st["n_reads"] == 0
