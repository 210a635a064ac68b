import os
import sys
sys.path.insert(0, ".")
import numpy as np
import torch
import torch.distributed as dist
from allpathslg_amd import Context, synth_fragments, synth_genome
from allpathslg_amd.distributed import HipShardBackend, sharded_unipaths


def fmix64(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


class Checked(HipShardBackend):
    def ushard_nodes(self, recv, recv_counts, K, P):
        torch.cuda.synchronize()
        n = int(recv_counts.sum())
        rec = recv[: 4 * n].cpu().numpy().view(np.uint64).reshape(n, 4)
        with np.errstate(over="ignore"):
            kh = fmix64(rec[:, 0] ^ fmix64(rec[:, 1] ^ fmix64(rec[:, 2] ^ np.uint64(0x5851f42d4c957f2d)))) & ~np.uint64(0xff)
        ok = kh == (rec[:, 3] & ~np.uint64(0xff))
        print("recv", n, "consistent", ok.mean(), "distinct h", len(np.unique(rec[:, 3] >> np.uint64(8))), flush=True)
        bad = np.nonzero(~ok)[0]
        if len(bad):
            print("first bad idx", bad[:5], rec[bad[:3]], flush=True)
        return super().ushard_nodes(recv, recv_counts, K, P)


local = int(os.environ.get("LOCAL_RANK", "0"))
torch.cuda.set_device(local)
dist.init_process_group("nccl", device_id=torch.device("cuda", local))
ctx = Context(local, verbose=True)
nf = int(sys.argv[1]) if len(sys.argv) > 1 else 20_000_000
g = synth_genome(64_444_167, 0xA11BA7)
fr = synth_fragments(g, nf, seed=0xA11BA7 + 1, threads=16)
d = ctx.upload(fr)
st = sharded_unipaths(Checked(ctx), d, 96)
print(st, flush=True)
dist.destroy_process_group()
