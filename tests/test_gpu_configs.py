"""Full-size GPU tests of BASELINE.json's single-GPU configs (C1, C2, C3).

The HIP path runs at the configs' own sizes; parity against the CPU
restatement (oracle/, parity unpinned vs ALLPATHS-LG: SURVEY §0.1) is checked
where the oracle finishes in seconds:

  C1  E. coli 4.64 Mb, 1 M reads: the whole chain (K=25 spectrum, K=24
      PreCorrect, FillFragments, K=96 unipaths + HyperKmerPath + KmerPaths)
      against the oracle end to end.
  C2  chr20 64.4 Mb, 40 M reads: the chain twice (byte-identical), the
      bench's size-independent properties, and whole-table parity of the
      counting stages: the complete K=25 spectrum of all 40 M reads, the
      complete K=24 solid set, and PreCorrect of all 40 M reads against it
      (the oracle's rolling-key form, ork_precorrect_solid_fast, equal to the
      checker by tests/test_cpu_baseline.py); one 1/256 hash parcel of the
      K=25 counted table (keys and counts); FillFragments of all 20 M pairs
      (every status and filled byte); the whole K=96 graph of all filled
      fragments (round 6: unipaths, ids, rc partners, unibases, HKP,
      every KmerPath); and, as a fast smoke, both directions of the unipath
      graph inside five 400-kb genome windows.
  C3  chr20 40 M frag + 20 M 3-kb jump reads: ErrorCorrectJump, all_reads =
      filled fragments ++ trimmed jumps, K=96 graph over all of them, run
      twice, ECJ parity on all 20 M jump reads (bases, qualities, trim
      lengths, counters), the whole all_reads graph against the oracle
      (round 6), window parity with the window's jump reads included.
"""
import numpy as np
import pytest
import torch

import oracle
from allpathslg_amd import ReadSet, synth_genome, synth_layout, synth_reads
from tests.test_gpu_unipath import assert_graph_equal

pytestmark = [pytest.mark.gpu, pytest.mark.timeout(900)]

CHR20 = 64_444_167
ECOLI = 4_641_652
K96 = 96


# -- helpers ---------------------------------------------------------------
def khash_np(K: int, x: np.ndarray) -> np.ndarray:
    """apg_kmer_hash / ork_hash (SURVEY §A.3 bijection on 2K bits), vectorised."""
    w = 2 * K
    m = np.uint64((1 << w) - 1) if w < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)

    def sh(num):
        return np.uint64(max(1, (w * num) // 64))

    c1 = np.uint64((0xBF58476D1CE4E5B9 & int(m)) | 1)
    c2 = np.uint64((0x94D049BB133111EB & int(m)) | 1)
    x = x.astype(np.uint64) & m
    with np.errstate(over="ignore"):
        x ^= x >> sh(30)
        x = (x * c1) & m
        x ^= x >> sh(27)
        x = (x * c2) & m
        x ^= x >> sh(31)
    return x


def parcel(K: int, idx: int, bits: int = 8):
    """[lo, hi) of the idx-th of 2^bits hash parcels of 2K-bit hashes."""
    s = 2 * K - bits
    return idx << s, (idx + 1) << s


def solid_sorted(ctx) -> np.ndarray:
    n = ctx.solid_copy(None)
    t = torch.empty(max(n, 1), dtype=torch.int64, device="cuda")
    ctx.solid_copy(t.data_ptr())
    return np.sort(t[:n].cpu().numpy().view(np.uint64))


def run_chain(ctx, dsrc, dwork, fill_out, status_t, with_graph=True):
    """restore -> K=25 spectrum -> K=24 PreCorrect -> FillFragments -> K=96
    unipaths (graph fetched)."""
    ctx.copy_reads(dwork, dsrc)
    hist, st = ctx.kmer_spectrum(dwork, 25)
    _, pst = ctx.precorrect(dwork, K=24)
    solid = solid_sorted(ctx)
    filled, _, fst = ctx.fill_fragments(dwork, K=24, last_solid=True, out=fill_out, d_status=status_t.data_ptr())
    graph, ust = ctx.unipaths(filled, K96, fetch=True) if with_graph else (None, None)
    return {"hist": hist, "st": st, "pst": pst, "solid": solid, "filled": filled, "fst": fst,
            "status": status_t.cpu().numpy().copy(), "graph": graph, "ust": ust}


def check_chain_properties(r, n_reads, genome_len, node_frac=None):
    """The bench's size-independent checks.  node_frac: the genome K-mers the
    filled fragments must cover (None: all but 1000, as at 62x)."""
    hist, st = r["hist"], r["st"]
    m = np.arange(len(hist), dtype=np.uint64)
    assert int(hist[-1]) == 0 and int((hist * m).sum()) == st["n_kmers"] == n_reads * 76
    assert int(hist.sum()) == st["n_distinct"]
    assert r["pst"]["n_corrected"] > 0.5 * r["pst"]["n_suspect"]
    f = r["fst"]
    assert sum(int(f[k]) for k in ("n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip")) == n_reads // 2
    assert int((r["status"] == 0).sum()) == f["n_filled"]
    g, u = r["graph"], r["ust"]
    gk = genome_len - K96 + 1
    assert u["n_nodes"] >= (gk - 1000 if node_frac is None else node_frac * gk)
    # ids are contiguous in emitted order; rc partners pair up with equal lengths
    assert np.array_equal(g["id_base"][1:], np.cumsum(g["len"])[:-1])
    rc = g["rc"].astype(np.int64)
    assert np.array_equal(rc[rc], np.arange(len(rc))) and np.array_equal(g["len"][rc], g["len"])


def same_chain(a, b, ctx):
    assert np.array_equal(a["hist"], b["hist"])
    assert a["st"] == b["st"] and a["pst"] == b["pst"] and a["fst"] == b["fst"]
    assert np.array_equal(a["solid"], b["solid"])
    assert np.array_equal(a["status"], b["status"])
    assert_graph_equal(a["graph"], b["graph"])


def kmer_set(seq: np.ndarray, K: int):
    """Both orientations of every K-mer of seq, as bytes."""
    out = set()
    rc = (3 - seq[::-1]).astype(np.uint8)
    b, r = seq.astype(np.uint8).tobytes(), rc.tobytes()
    for i in range(len(seq) - K + 1):
        out.add(b[i : i + K])
        out.add(r[i : i + K])
    return out


def unipath_seqs(g):
    """unibases of every unipath as bytes (one per emitted unipath)."""
    ub, off = g["unibases"], g["ub_off"]
    return [ub[int(off[i]) : int(off[i + 1])].tobytes() for i in range(g["n_unipaths"])]


def window_parity(gpu_graph, oracle_reads, genome, w0, w1, margin=20_000):
    """Both directions inside the window interior (the window minus `margin`
    at each end, so every unipath counted lies wholly inside the window and
    is built from the window's reads only):
      - every oracle unipath (of the window's reads) shorter than the margin
        that holds an interior K-mer is a unipath of the full-size GPU graph,
        and such unipaths cover most of the interior;
      - every GPU unipath shorter than the margin that holds an interior
        K-mer is an oracle unipath (same bases)."""
    og = oracle.unipaths(oracle_reads, K96)
    interior = kmer_set(genome[w0 + margin : w1 - margin], K96)

    def touching(g):
        out = []
        for s, L in zip(unipath_seqs(g), g["len"]):
            if L >= margin:
                continue
            ks = [s[i : i + K96] for i in range(len(s) - K96 + 1)]
            hit = [k for k in ks if k in interior]
            if hit:
                out.append((s, hit))
        return out

    gpu_all = set(s for s, L in zip(unipath_seqs(gpu_graph), gpu_graph["len"]) if L < 2 * margin)
    ora_all = set(unipath_seqs(og))
    covered, compared = set(), 0
    for s, hit in touching(og):
        assert s in gpu_all, "an oracle unipath of the window is not a GPU unipath"
        covered.update(hit)
        compared += 1
    assert compared > 0
    assert len(covered) >= 0.9 * len(interior), (len(covered), len(interior))
    back = 0
    for s, _ in touching(gpu_graph):
        assert s in ora_all, "a GPU unipath of the window interior is not an oracle unipath"
        back += 1
    assert back == compared, (back, compared)
    return compared


def pairs_in_window(start, flen, w0, w1, pad=500):
    return np.nonzero((start.astype(np.int64) + flen < w1 + pad) & (start.astype(np.int64) > w0 - pad))[0]


def filled_subset(filled: ReadSet, status: np.ndarray, pairs: np.ndarray) -> ReadSet:
    """The filled fragments of the given pairs (filled sets are in pair order)."""
    fidx = np.cumsum(status == 0) - 1
    sel = pairs[status[pairs] == 0]
    return ReadSet.from_sequences([filled.read(int(fidx[p])) for p in sel])


# -- C1: E. coli, 1 M reads, whole chain vs the oracle ---------------------
def test_c1_ecoli_whole_chain_matches_oracle(gpu_ctx):
    g = synth_genome(ECOLI, 0xA11BA7 + 0)
    reads = synth_reads(g, 500_000, seed=0xA11BA7 + 100, threads=16)
    dsrc, dwork = gpu_ctx.upload(reads), gpu_ctx.upload(reads)
    status = torch.zeros(reads.n_reads // 2, dtype=torch.uint8, device="cuda")
    r = run_chain(gpu_ctx, dsrc, dwork, None, status)
    # K=25 spectrum
    assert np.array_equal(r["hist"], oracle.kmer_spectrum(reads, 25))
    # K=24 PreCorrect: solid set, corrected bases / quals, counters
    assert np.array_equal(r["solid"], np.sort(oracle.solid_hashes(reads, 24, 3)))
    fixed, est = oracle.precorrect(reads, K=24)
    got = gpu_ctx.download(dwork)
    assert np.array_equal(got.packed[: int(got.byte_off[-1])], fixed.packed[: int(fixed.byte_off[-1])])
    assert np.array_equal(got.quals, fixed.quals)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable", "n_solid"):
        assert r["pst"][k] == est[k], k
    # FillFragments against that solid set
    ofill, ostatus, _, ost = oracle.fill_fragments(fixed, r["solid"], K=24)
    assert np.array_equal(r["status"], ostatus)
    hf = gpu_ctx.download(r["filled"])
    assert np.array_equal(hf.base_off, ofill.base_off)
    assert np.array_equal(hf.packed[: int(hf.byte_off[-1])], ofill.packed[: int(ofill.byte_off[-1])])
    # K=96 unipaths, unibases, HKP, KmerPaths of every filled fragment
    assert_graph_equal(r["graph"], oracle.unipaths(ofill, K96))
    check_chain_properties(r, reads.n_reads, ECOLI, node_frac=0.98)  # 21.5x: a few K-mers uncovered
    for d in (dsrc, dwork, r["filled"]):
        d.free()


# -- C2: chr20, 40 M reads ---------------------------------------------------
@pytest.fixture(scope="module")
def c2(gpu_ctx):
    seed = 0xA11BA7 + 1
    g = synth_genome(CHR20, seed)
    reads = synth_reads(g, 20_000_000, seed=seed + 100, threads=16)
    dsrc, dwork = gpu_ctx.upload(reads), gpu_ctx.upload(reads)
    status = torch.zeros(reads.n_reads // 2, dtype=torch.uint8, device="cuda")
    a = run_chain(gpu_ctx, dsrc, dwork, None, status)
    fixed_a = gpu_ctx.download(dwork)
    filled_a = gpu_ctx.download(a["filled"])
    b = run_chain(gpu_ctx, dsrc, dwork, a["filled"], status)
    filled_b = gpu_ctx.download(b["filled"])
    # the bench's timed entry point with its defaults (bench.py step():
    # apg_spectrum_precorrect_dev — side-stream K+1 pass with the deferred
    # kick, extension table on the auxiliary stream, packed SKP records, the
    # K+1 pass fed by the record dedup)
    gpu_ctx.copy_reads(dwork, dsrc)
    fh, fks, fps = gpu_ctx.spectrum_precorrect(dwork, K_spec=25, K=24)
    fused = {"hist": fh, "st": fks, "pst": fps, "solid": solid_sorted(gpu_ctx), "fixed": gpu_ctx.download(dwork)}
    # ... and the step's entry point since round 6, with FillFragments in the
    # same call (apg_spectrum_precorrect_fill_dev)
    gpu_ctx.copy_reads(dwork, dsrc)
    ffh, ffks, ffps, ffd, ffst = gpu_ctx.spectrum_precorrect_fill(dwork, K_spec=25, K=24, d_status=status.data_ptr())
    fused_fill = {"hist": ffh, "st": ffks, "pst": ffps, "fst": ffst, "status": status.cpu().numpy().copy(),
                  "filled": gpu_ctx.download(ffd), "fixed": gpu_ctx.download(dwork)}
    ffd.free()
    yield {"genome": g, "reads": reads, "a": a, "b": b, "fixed": fixed_a, "filled_a": filled_a,
           "filled_b": filled_b, "seed": seed, "dsrc": dsrc, "fused": fused, "fused_fill": fused_fill}
    for d in (dsrc, dwork, a["filled"]):
        d.free()


def test_c2_deterministic_and_properties(c2, gpu_ctx):
    same_chain(c2["a"], c2["b"], gpu_ctx)
    fa, fb = c2["filled_a"], c2["filled_b"]
    assert np.array_equal(fa.base_off, fb.base_off)
    assert np.array_equal(fa.packed[: int(fa.byte_off[-1])], fb.packed[: int(fb.byte_off[-1])])
    check_chain_properties(c2["a"], c2["reads"].n_reads, CHR20)
    assert c2["a"]["ust"]["max_len"] >= 10_000


def test_c2_parcel_counts_match_oracle(c2, gpu_ctx):
    reads = c2["reads"]
    lo, hi = parcel(25, 0x5A)
    keys, counts, _ = gpu_ctx.kmer_count(c2["dsrc"], 25, hash_range=(lo, hi))
    oh, oc = oracle.kmer_count_range(reads, 25, lo, hi)
    assert len(oh) > 1_000_000
    assert np.array_equal(khash_np(25, keys), oh)
    assert np.array_equal(counts, oc)


@pytest.fixture(scope="module")
def c2_oracle(c2):
    """The oracle's whole-table results for all 40 M reads, computed once:
    K=25 spectrum, K=24 solid set, PreCorrect against that solid set."""
    reads = c2["reads"]
    spec = oracle.kmer_spectrum(reads, 25)
    solid = np.sort(oracle.solid_hashes(reads, 24, 3))
    fixed, est = oracle.precorrect_solid(reads, solid, K=24, fast=True)
    return {"hist": spec, "solid": solid, "fixed": fixed, "est": est}


def assert_precorrect_equal(fixed, pst, exp, est):
    assert np.array_equal(fixed.packed[: int(fixed.byte_off[-1])], exp.packed[: int(exp.byte_off[-1])])
    assert np.array_equal(fixed.quals, exp.quals)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable"):
        assert pst[k] == est[k], k


def test_c2_full_spectrum_matches_oracle(c2, c2_oracle):
    """The complete K=25 spectrum of all 40 M reads (3.04 G K-mer instances)."""
    assert np.array_equal(c2["a"]["hist"], c2_oracle["hist"])


def test_c2_full_solid_set_matches_oracle(c2, c2_oracle):
    """The complete K=24 solid set (count >= 3) of all 40 M reads."""
    assert len(c2_oracle["solid"]) > 60_000_000
    assert np.array_equal(c2["a"]["solid"], c2_oracle["solid"])


def test_c2_full_precorrect_matches_oracle(c2, c2_oracle):
    """PreCorrect of all 40 M reads against the (whole-table-checked) solid
    set: every base, quality and counter."""
    assert_precorrect_equal(c2["fixed"], c2["a"]["pst"], c2_oracle["fixed"], c2_oracle["est"])


def test_c2_bench_entry_point_matches_oracle(c2, c2_oracle):
    """The bench's own timed entry point (apg_spectrum_precorrect_dev at its
    defaults) at full C2 size against the oracle: the whole K=25 spectrum,
    the whole K=24 solid set, and every corrected base, quality and counter
    of the 40 M reads."""
    f = c2["fused"]
    assert np.array_equal(f["hist"], c2_oracle["hist"])
    m = np.arange(len(f["hist"]), dtype=np.uint64)
    assert int((f["hist"] * m).sum()) == f["st"]["n_kmers"] == c2["reads"].n_reads * 76
    assert int(f["hist"].sum()) == f["st"]["n_distinct"]
    assert np.array_equal(f["solid"], c2_oracle["solid"])
    assert f["pst"]["n_solid"] == len(c2_oracle["solid"])
    assert_precorrect_equal(f["fixed"], f["pst"], c2_oracle["fixed"], c2_oracle["est"])


def test_c2_fused_fill_entry_point_equals_modules(c2, c2_oracle):
    """apg_spectrum_precorrect_fill_dev at full C2 size (the bench's timed
    entry point since round 6): spectrum = oracle, corrected reads = oracle,
    and every fill status, filled fragment and counter equal the modules' run
    (which test_c2_full_fill_matches_oracle checks against the oracle)."""
    f = c2["fused_fill"]
    assert np.array_equal(f["hist"], c2_oracle["hist"])
    assert_precorrect_equal(f["fixed"], f["pst"], c2_oracle["fixed"], c2_oracle["est"])
    assert np.array_equal(f["status"], c2["a"]["status"])
    assert f["fst"] == c2["a"]["fst"]
    hf, hb = f["filled"], c2["filled_a"]
    assert np.array_equal(hf.base_off, hb.base_off)
    assert np.array_equal(hf.packed[: int(hf.byte_off[-1])], hb.packed[: int(hb.byte_off[-1])])


def test_c2_full_fill_matches_oracle(c2, c2_oracle):
    """FillFragments of all 20 M pairs (the whole-table-checked corrected
    reads and solid set) against the oracle's hash-table form: every status,
    every filled fragment byte for byte, every counter."""
    fixed, solid = c2["fixed"], c2["a"]["solid"]
    assert np.array_equal(solid, c2_oracle["solid"])
    ofill, ostatus, _, ost = oracle.fill_fragments(fixed, solid, K=24, fast=True)
    status = c2["a"]["status"]
    assert np.array_equal(status, ostatus)
    hf = c2["filled_a"]
    assert np.array_equal(hf.base_off, ofill.base_off)
    assert np.array_equal(hf.packed[: int(hf.byte_off[-1])], ofill.packed[: int(ofill.byte_off[-1])])
    for k in ("n_filled", "n_none", "n_ambiguous", "n_budget", "n_skip", "filled_bases"):
        assert c2["a"]["fst"][k] == ost[k], k


def test_c2_whole_graph_matches_oracle(c2):
    """The whole K=96 graph of all filled fragments of the 40 M reads (SURVEY
    §8a a8-a11): node count, every unipath's length, id
    base and rc partner, every unibase, the HyperKmerPath's vertices and
    edges, and every fragment's KmerPath, against the oracle's graph of the
    same (whole-table-checked) filled fragments."""
    og = oracle.unipaths(c2["filled_a"], K96)
    assert og["n_nodes"] >= CHR20 - K96 + 1 - 1000
    assert_graph_equal(c2["a"]["graph"], og)


# five windows of 400 kb spread over the chromosome (2 Mb, 3 % of it; round 4
# checked one 200-kb window)
C2_WINDOWS = [int(CHR20 * f) for f in (0.07, 0.29, 0.5, 0.71, 0.9)]


@pytest.mark.parametrize("w0", C2_WINDOWS)
def test_c2_window_unipaths_match_oracle(c2, w0):
    g = c2["genome"]
    w1 = w0 + 400_000
    start, flen, _ = synth_layout(CHR20, 20_000_000, seed=c2["seed"] + 100, threads=16)
    pairs = pairs_in_window(start, flen, w0, w1)
    sub = filled_subset(c2["filled_a"], c2["a"]["status"], pairs)
    assert window_parity(c2["a"]["graph"], sub, g, w0, w1) > 0


# -- C3: chr20, frag + 3 kb jump library, unipaths over all_reads -------------
def test_c3_frag_plus_jump_graph(gpu_ctx):
    seed = 0xA11BA7 + 2
    g = synth_genome(CHR20, seed)
    frags = synth_reads(g, 20_000_000, seed=seed + 100, threads=16)
    jumps = synth_reads(g, 10_000_000, seed=seed + 200, insert_mean=3000, insert_sd=300, threads=16)
    dF0, dF, dJ0, dJ = gpu_ctx.upload(frags), gpu_ctx.upload(frags), gpu_ctx.upload(jumps), gpu_ctx.upload(jumps)
    status = torch.zeros(frags.n_reads // 2, dtype=torch.uint8, device="cuda")
    keep = torch.zeros(jumps.n_reads, dtype=torch.int32, device="cuda")
    runs = []
    filled = allr = None
    for _ in range(2):
        gpu_ctx.copy_reads(dF, dF0)
        gpu_ctx.copy_reads(dJ, dJ0)
        gpu_ctx.precorrect(dF, K=24)
        filled, _, fst = gpu_ctx.fill_fragments(dF, K=24, last_solid=True, out=filled, d_status=status.data_ptr())
        est = gpu_ctx.error_correct_jump(dF, dJ, d_keep=keep.data_ptr())
        ecj_solid = solid_sorted(gpu_ctx)
        allr = gpu_ctx.concat_reads([filled, dJ], [None, keep.data_ptr()], out=allr)
        graph, ust = gpu_ctx.unipaths(allr, K96, fetch=True)
        runs.append((graph, ust, fst, est, keep.cpu().numpy().astype(np.uint32), status.cpu().numpy().copy()))
    (ga, ua, fa, ea, ka, sa), (gb, ub, fb, eb, kb, sb) = runs
    assert_graph_equal(ga, gb)
    assert ua == ub and fa == fb and ea == eb
    assert np.array_equal(ka, kb) and np.array_equal(sa, sb)
    # all_reads = filled fragments ++ trimmed jumps; every read's KmerPath
    n_all = fa["n_filled"] + jumps.n_reads
    assert allr.n_reads == n_all and int(ga["path_off"].shape[0]) == n_all + 1
    jl = np.minimum(ka, 100).astype(np.int64)
    inst = int(fa["filled_bases"]) - (K96 - 1) * fa["n_filled"] + int(np.maximum(jl - K96 + 1, 0).sum())
    assert ua["n_instances"] == inst
    assert ua["n_nodes"] >= CHR20 - K96 + 1 - 1000
    # ErrorCorrectJump parity on all 20 M jump reads (the fragments' solid set):
    # every corrected base and quality, every trim length, every counter
    dJ_host = gpu_ctx.download(dJ)
    fixed, okeep, ost = oracle.error_correct_jump_solid(jumps, ecj_solid, K=24, fast=True)
    assert np.array_equal(dJ_host.packed[: int(dJ_host.byte_off[-1])], fixed.packed[: int(fixed.byte_off[-1])])
    assert np.array_equal(dJ_host.quals, fixed.quals)
    assert np.array_equal(ka, okeep)
    for k in ("n_suspect", "n_corrected", "n_ambiguous", "n_uncorrectable"):
        assert ea["precorrect"][k] == ost[k], k
    assert ea["bases_kept"] == int(okeep.astype(np.uint64).sum())
    # the whole all_reads graph (filled fragments ++ trimmed jumps) against the
    # oracle's graph of the same reads: every unipath, unibase, HKP vertex /
    # edge and every read's KmerPath
    allr_host = gpu_ctx.download(allr)
    assert allr_host.n_reads == n_all
    assert_graph_equal(ga, oracle.unipaths(allr_host, K96))
    del allr_host
    # window parity with the window's jump reads in the oracle's input
    w0 = CHR20 // 3
    w1 = w0 + 200_000
    fs, fl, _ = synth_layout(CHR20, 20_000_000, seed=seed + 100, threads=16)
    js, jlen, _ = synth_layout(CHR20, 10_000_000, seed=seed + 200, insert_mean=3000, insert_sd=300, threads=16)
    fpairs = pairs_in_window(fs, fl, w0, w1)
    sub = filled_subset(gpu_ctx.download(filled), sa, fpairs)
    # a jump read lies at either end of its 3-kb fragment: take reads whose
    # 100 bases fall in the window
    js = js.astype(np.int64)
    ends = np.concatenate([np.stack([js, 2 * np.arange(len(js))], 1),
                           np.stack([js + jlen - 100, 2 * np.arange(len(js)) + 1], 1)])
    inwin = ends[(ends[:, 0] > w0 - 500) & (ends[:, 0] + 100 < w1 + 500)]
    jr = set()
    for _, pair_read in inwin:  # the pair's two reads, either orientation
        p = int(pair_read) // 2
        jr.update((2 * p, 2 * p + 1))
    jr = sorted(jr)
    jseqs = [dJ_host.read(i)[: int(ka[i])] for i in jr]
    win = ReadSet.from_sequences([sub.read(i) for i in range(sub.n_reads)] + jseqs)
    assert window_parity(ga, win, g, w0, w1) > 0
    for d in (dF0, dF, dJ0, dJ, filled, allr):
        d.free()
