import sys
sys.path.insert(0, ".")
import numpy as np
import torch
from allpathslg_amd import Context, synth_fragments, synth_genome

M64 = (1 << 64) - 1


def fmix64(z):
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xbf58476d1ce4e5b9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94d049bb133111eb)
    return z ^ (z >> np.uint64(31))


ctx = Context(0, verbose=True)
g = synth_genome(8_000_000, 5)
fr = synth_fragments(g, 2_000_000, seed=6)
d = ctx.upload(fr)
counts, ninst = ctx.ushard_count(d, 96, 1)
n = int(counts.sum())
print("local nodes", n, "instances", ninst)
send = torch.empty(4 * n, dtype=torch.int64, device="cuda")
torch.cuda.synchronize()
ctx.ushard_scatter(d, 96, 1, send.data_ptr())
rec = send.cpu().numpy().view(np.uint64).reshape(n, 4)
with np.errstate(over="ignore"):
    kh = fmix64(rec[:, 0] ^ fmix64(rec[:, 1] ^ fmix64(rec[:, 2] ^ np.uint64(0x5851f42d4c957f2d)))) & ~np.uint64(0xff)
ok = kh == (rec[:, 3] & ~np.uint64(0xff))
print("meta hash consistent", ok.mean(), "first bad", np.nonzero(~ok)[0][:5], rec[~ok][:3])
print("distinct hashes", len(np.unique(kh)), "distinct keys", len(np.unique(rec[:, :3], axis=0)))
print("digits", counts[:8])
m = ctx.ushard_nodes(send.data_ptr(), counts, 96, 1)
print("owner nodes", m)
