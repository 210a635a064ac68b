#!/usr/bin/env python3
"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes to per-launch HBM
traffic per timed kernel (the `traffic` field of bench.py's roofline).

FETCH_SIZE corrections (MI355X_MICROARCH.md, HBM section): wide coalesced
streaming reads are tallied at half their bytes on gfx950 (x2); random 64-byte
line reads are tallied exactly — calibrated here on tools/microbench/randread
(2^28 random lines = 16 GiB read, FETCH_SIZE = 16.0 GiB per launch; see
calibration_randread.csv).  Kernels are tagged with their access pattern.

  python scripts/pmc_traffic.py profiles/r01_pmc_v7
writes <dir>/traffic.json.
"""
import collections
import csv
import json
import os
import sys

# HIP symbol prefix -> (bench timing label, read pattern).  Several symbols may
# share a label in two ways: one timed region launching two kernels (REGIONS:
# their traffic adds, the label's launches are the most frequent symbol's), or
# separate launches of template instantiations under one label (sk_scatter's
# SK16 spectrum and SK24 solid-set launches: launches add too).
KERNELS = [
    ("void apg::k_sk_bucket_dd<true, apg::SK24>", "sk_bucket_solid", "stream"),
    ("void apg::k_sk_bucket_dd<true, apg::SKP>", "sk_bucket_solid", "stream"),  # round 4: packed records read directly
    ("void apg::k_sk_bucket<true, apg::SKP>", "sk_bucket_solid", "stream"),
    ("void apg::k_sk_bucket<false, apg::SKP>", "sk_bucket", "stream"),  # the fused K+1 pass on packed records
    ("void apg::k_sk_bucket<true, apg::SK24>", "sk_bucket_solid", "stream"),
    ("void apg::k_sk_bucket<false, apg::SK16>", "sk_bucket", "stream"),
    ("void apg::k_sk_bucket<false, apg::SK24>", "sk_bucket", "stream"),  # the fused K+1 pass (UP)
    ("apg::k_sk_count", "sk_count", "stream"),
    ("void apg::k_sk_scatter<apg::SK16*>", "sk_scatter", "stream"),
    ("void apg::k_sk_scatter<apg::SK24*>", "sk_scatter", "stream"),
    ("void apg::k_sk_replay<apg::SK16*>", "sk_scatter", "stream"),
    ("void apg::k_sk_replay<apg::SK24*>", "sk_scatter", "stream"),
    ("void apg::k_sk_scatter<apg::SKP*>", "sk_scatter", "stream"),
    ("void apg::k_sk_replay<apg::SKP*>", "sk_scatter", "stream"),
    ("void apg::k_sk_scatter<apg::SkpOut>", "sk_scatter", "stream"),  # round 4: packed output with the wide form
    ("void apg::k_sk_replay<apg::SkpOut>", "sk_scatter", "stream"),
    ("void apg::k_sk_scatter<apg::SplitOut>", "sk_scatter", "stream"),  # multi-GPU: records + positions
    ("void apg::k_sk_replay<apg::SplitOut>", "sk_scatter", "stream"),
    ("void apg::k_part_scatter<apg::SKP>", "s24_part_scatter", "stream"),  # packed levels (SKP -> SKP / SK24)
    ("void apg::k_part_scatter<apg::SK16, apg::SKP>", "s24_part_scatter", "stream"),  # multi-GPU owner: packing level
    ("void apg::k_part_count<apg::SKP>", "s24_part_count", "stream"),
    ("void apg::k_part_scatter<apg::SK16>", "s_part_scatter", "stream"),
    ("void apg::k_part_scatter<apg::SK24>", "s24_part_scatter", "stream"),
    ("void apg::k_part_count<apg::SK16>", "s_part_count", "stream"),
    ("void apg::k_part_count<apg::SK24>", "s24_part_count", "stream"),
    ("apg::k_fill(", "fill", "random"),
    ("void apg::k_fill<16>", "fill", "random"),  # round 4: the slot layout as a template parameter
    ("void apg::k_fill<8>", "fill", "random"),
    ("apg::k_ext_link", "ext_link", "random"),
    ("apg::k_fill_write", "fill_write", "stream"),
    ("apg::k_pc_decide", "precorrect", "random"),
    ("void apg::k_pc_candidates<true>", "pc_cand_write", "stream"),  # the bench's timed-region name
    ("apg::k_pc_apply", "pc_apply", "stream"),
    ("apg::k_fill_ext_insert", "solid_insert", "random"),
    ("void apg::k_read_paths<false>", "u_read_paths_count", "random"),
    ("void apg::k_read_paths<true>", "u_read_paths_write", "random"),
    ("apg::k_unibases", "u_unibases", "random"),
    ("apg::k_usk_count", "usk_count", "stream"),
    ("apg::k_usk_scatter", "usk_scatter", "stream"),
    ("apg::k_usk_bucket", "usk_bucket", "stream"),
    ("void apg::k_usk_bucket<1024u>", "usk_bucket", "stream"),  # round 4: table size (and waves) as template arguments
    ("void apg::k_usk_bucket<512u>", "usk_bucket", "stream"),
    ("void apg::k_part_scatter<apg::SK48>", "usk_part_scatter", "stream"),
    ("apg::k_links", "u_links", "random"),
    ("apg::k_walk", "u_walk", "random"),
]


REGIONS = {"sk_bucket_solid"}  # k_sk_bucket_dd + the hand-back k_sk_bucket in one timed region
# symbols whose traffic adds to their label but whose launches do not: the
# walk kernel launched after k_sk_replay in the same timed region (it walks
# only the blocks whose descriptors overflowed)
NO_LAUNCHES = ("void apg::k_sk_scatter<",)


def load(path):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1024.0)  # KB -> bytes
    return agg


def matches(sym, prefix):
    if prefix.endswith("("):
        return sym.startswith(prefix)
    base = sym.split("(")[0]
    return base == prefix or (prefix.endswith(">") and base.startswith(prefix[:-1] + ","))


def main(d):
    f = load(os.path.join(d, "fetch.csv"))
    w = load(os.path.join(d, "write.csv"))
    out = {}
    for prefix, label, pattern in KERNELS:
        corr = 2.0 if pattern == "stream" else 1.0
        for sym in f:
            if not matches(sym, prefix):
                continue
            e = out.setdefault(label, {"symbols": [], "pattern": pattern, "launches": 0, "fetch_size_bytes": 0.0,
                                       "fetch_correction": corr, "write_size_bytes": 0.0})
            e["symbols"].append(sym.split("(")[0])
            if sym.startswith(NO_LAUNCHES):
                pass
            elif label in REGIONS:
                e["launches"] = max(e["launches"], len(f[sym]))
            else:
                e["launches"] += len(f[sym])
            e["fetch_size_bytes"] += sum(f[sym])
            e["write_size_bytes"] += sum(w.get(sym, [0.0]))
    for e in out.values():
        n = max(e["launches"], 1)
        e["fetch_size_bytes"] /= n
        e["write_size_bytes"] /= n
        e["traffic_bytes_per_launch"] = e["fetch_size_bytes"] * e["fetch_correction"] + e["write_size_bytes"]
    json.dump(out, open(os.path.join(d, "traffic.json"), "w"), indent=1)
    for k, v in out.items():
        print(f"{k:18s} {v['traffic_bytes_per_launch'] / 1e9:9.2f} GB/launch ({v['pattern']}; "
              f"fetch {v['fetch_size_bytes'] / 1e9:.2f} x{v['fetch_correction']:.0f}, write {v['write_size_bytes'] / 1e9:.2f})")


if __name__ == "__main__":
    main(sys.argv[1])
