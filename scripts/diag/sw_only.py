"""The bench's aligner workload (bench.align_workload: 4 M placed 100-bp
reads on 50-kb genome pieces) through banded SW only, for rocprofv3 runs
(kernel trace / PMC passes of k_banded_sw_*).  Diagnostic for DESIGN §5."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
from allpathslg_amd import Context, synth_genome  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
w = int(sys.argv[2]) if len(sys.argv) > 2 else 8
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
g = synth_genome(64_444_167, 7)
S, T, pairs, plain, nsub = bench.align_workload(g, n, 50_000, 15)
with Context(device=0, timing=True) as ctx:
    dS, dT = ctx.upload(S), ctx.upload(T)
    dp = torch.from_numpy(pairs).cuda()
    sw = torch.empty((n, 8), dtype=torch.int32, device="cuda")
    for _ in range(reps + 1):
        ctx.banded_sw_dev(dS, dT, dp.data_ptr(), n, w, sw.data_ptr())
    torch.cuda.synchronize()
    kt = ctx.kernel_times()
    t = kt["banded_sw"]
    print(f"banded_sw w={w}: {t[0] / t[1]:.3f} ms/launch over {t[1]} launches", flush=True)
    dS.free()
    dT.free()
