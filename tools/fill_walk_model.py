"""Inputs for tools/fill_walk_model.c: a synthetic genome (iid, or with
apg_repeat_defaults' repeats), paired 100-bp reads at the bench's 62x read
coverage, and the canonical K-mers seen >= 3 times in them (the solid set of
the uncorrected reads — a model input, not FillFragments' own).

    python tools/fill_walk_model.py OUTDIR GENOME_LEN [--repeats] [--K 24]
    gcc -O2 -o /tmp/fwm tools/fill_walk_model.c && /tmp/fwm 24 OUTDIR/solid.bin OUTDIR/reads.bin
"""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from allpathslg_amd import synth_genome, synth_reads  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out")
    ap.add_argument("genome_len", type=int)
    ap.add_argument("--repeats", action="store_true")
    ap.add_argument("--K", type=int, default=24)
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    g = synth_genome(a.genome_len, 51, repeats=True if a.repeats else None)
    reads = synth_reads(g, int(a.genome_len * 0.31), seed=52)
    n, L, K = len(reads.base_off) - 1, 100, a.K
    idx = reads.byte_off[:-1].astype(np.int64)[:, None] + np.arange(L // 4)[None, :]
    by = reads.packed[idx]
    b = np.stack([(by >> (2 * i)) & 3 for i in range(4)], axis=2).reshape(n, L).astype(np.uint8)
    with open(os.path.join(a.out, "reads.bin"), "wb") as f:
        f.write(np.uint64(n).tobytes() + np.uint32(L).tobytes() + b.tobytes())
    fw = np.zeros((n, L - K + 1), np.uint64)
    rc = np.zeros_like(fw)
    for t in range(K):
        fw = (fw << np.uint64(2)) | b[:, t:t + L - K + 1].astype(np.uint64)
        rc |= (3 - b[:, t:t + L - K + 1]).astype(np.uint64) << np.uint64(2 * t)
    u, c = np.unique(np.minimum(fw, rc).ravel(), return_counts=True)
    sol = u[c >= 3]
    with open(os.path.join(a.out, "solid.bin"), "wb") as f:
        f.write(np.uint64(len(sol)).tobytes() + sol.tobytes())
    print(f"{n} reads, {len(sol)} solid {K}-mers -> {a.out}")


if __name__ == "__main__":
    main()
