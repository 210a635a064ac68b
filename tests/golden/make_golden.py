"""Regenerate the golden fixtures in this directory (test infrastructure).

The reference snapshot is empty, so these vectors are produced
by this repo's CPU restatement (oracle/) from the deterministic synthetic
generator; they pin the oracle against regressions and give the GPU path a
fixed known answer.  Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

import oracle  # noqa: E402
from allpathslg_amd import synth_genome, synth_reads  # noqa: E402


def main():
    g = synth_genome(10_000, 0xA11A7)
    reads = synth_reads(g, 500, seed=0xA11A7 + 1)
    reads.write_fastb(os.path.join(HERE, "frag_small.fastb"))
    reads.write_qualb(os.path.join(HERE, "frag_small.qualb"))
    out = {}
    for K in (16, 25):
        h, c = oracle.kmer_count(reads, K)
        out[f"hash_k{K}"] = h
        out[f"count_k{K}"] = c
        out[f"spec_k{K}"] = oracle.spectrum_from_counts(c, 1 << 16)[:4096]
    np.savez_compressed(os.path.join(HERE, "kmer_small.npz"), **out)
    print({k: v.shape for k, v in out.items()})
    write_stage_fixtures(g, reads)
    write_fill_fixture(reads)
    write_locs_ecj_fixture()


def write_fill_fixture(reads):
    """FillFragments of the PreCorrect'ed pairs through the raw reads' solid
    K=24 set (the bench pipeline's order): status, length and bases."""
    fixed, _ = oracle.precorrect(reads, K=24)
    solid = oracle.solid_hashes(reads, 24, 3)
    filled, status, flen, st = oracle.fill_fragments(fixed, solid, K=24, min_insert=126, max_insert=234)
    out = {"solid": np.sort(solid), "status": status, "flen": flen,
           "packed": filled.packed[: int(filled.byte_off[-1])], "base_off": filled.base_off,
           "stats": np.array([st[k] for k in ("n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip",
                                              "filled_bases")], np.uint64)}
    np.savez_compressed(os.path.join(HERE, "fill_small.npz"), **out)
    print({k: v.shape for k, v in out.items()}, st)


def write_stage_fixtures(g, reads):
    """PreCorrect / FindErrors, unipaths (K = 31, 96) and aligner outputs of
    the same inputs (+ the pairs' fragments and a small alignment case)."""
    from allpathslg_amd import synth_fragments
    from tests.align_cases import sw_case

    out = {}
    for cyc in (1, 2):
        fixed, st = oracle.precorrect(reads, K=24, n_cycles=cyc)
        out[f"pc{cyc}_packed"] = fixed.packed[: int(fixed.byte_off[-1])]
        out[f"pc{cyc}_quals"] = fixed.quals
        out[f"pc{cyc}_stats"] = np.array([st[k] for k in ("n_suspect", "n_corrected", "n_ambiguous",
                                                           "n_uncorrectable", "n_solid")], np.uint64)
    frags = synth_fragments(g, 500, seed=0xA11A7 + 1)
    frags.write_fastb(os.path.join(HERE, "frag_small_fill.fastb"))
    for K, src in ((31, reads), (96, frags)):
        gr = oracle.unipaths(src, K)
        for key in ("len", "id_base", "rc", "ub_off", "unibases", "from", "to", "path_off", "path_start",
                    "path_len"):
            out[f"u{K}_{key}"] = np.asarray(gr[key])
    S, T, pairs = sw_case(n_targets=6, n_pairs=200, tlen=300, slen=(40, 120), seed=7)
    S.write_fastb(os.path.join(HERE, "aln_queries.fastb"))
    S.write_qualb(os.path.join(HERE, "aln_queries.qualb"))
    T.write_fastb(os.path.join(HERE, "aln_targets.fastb"))
    out["aln_pairs"] = pairs
    out["aln_gapfree"] = oracle.gapfree(S, T, pairs)
    res, blk = oracle.banded_sw(S, T, pairs, band_w=8, max_blocks=16)
    out["aln_sw"] = res
    out["aln_sw_blocks"] = blk
    b, q = oracle.consensus(S, T, pairs)
    out["aln_cons_bases"] = b
    out["aln_cons_quals"] = q
    np.savez_compressed(os.path.join(HERE, "stages_small.npz"), **out)
    print({k: v.shape for k, v in out.items()})


def write_locs_ecj_fixture():
    """UnipathLocs of the raw small reads on the K=96 graph of the fixture
    fragments (rc mirrors, by-unipath order), and ErrorCorrectJump of a small
    3-kb jump library against the small frag reads."""
    from allpathslg_amd import ReadSet

    reads = ReadSet.load(os.path.join(HERE, "frag_small.fastb"), os.path.join(HERE, "frag_small.qualb"))
    frags = ReadSet.load(os.path.join(HERE, "frag_small_fill.fastb"))
    g = oracle.unipaths(frags, 96)
    locs, lst = oracle.unipath_locs(g, reads, 96, rc=True, sorted=True)
    genome = synth_genome(10_000, 0xA11A7)
    jumps = synth_reads(genome, 150, seed=0xA11A7 + 3, insert_mean=3000, insert_sd=300)
    jumps.write_fastb(os.path.join(HERE, "jump_small.fastb"))
    jumps.write_qualb(os.path.join(HERE, "jump_small.qualb"))
    fixed, keep, st = oracle.error_correct_jump(reads, jumps, K=24)
    out = {"locs": locs, "locs_stats": np.array([lst["n_placed"], lst["n_missing"]], np.uint64),
           "ecj_packed": fixed.packed[: int(fixed.byte_off[-1])], "ecj_quals": fixed.quals, "ecj_keep": keep,
           "ecj_stats": np.array([st[k] for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable",
                                                  "n_solid")], np.uint64)}
    np.savez_compressed(os.path.join(HERE, "locs_ecj_small.npz"), **out)
    print({k: v.shape for k, v in out.items()}, lst, st)


if __name__ == "__main__":
    if sys.argv[1:] == ["locs_ecj"]:
        write_locs_ecj_fixture()
    elif sys.argv[1:] == ["fill"]:
        from allpathslg_amd import ReadSet

        write_fill_fixture(ReadSet.load(os.path.join(HERE, "frag_small.fastb"), os.path.join(HERE, "frag_small.qualb")))
    else:
        main()
