"""The unipath pair-key sort (U7, unipath.hip `u_sort_keys`): the one-pass
form (keys binned on their most significant varying bits, each bin ranked in
LDS, ties by input position) and the stable LSD passes it replaced must give
the same unipath order.  Each form runs in its own process (the knobs are
read once per process): the default, `APG_U_SORT=lsd`, and
`APG_U_SORT_BINMAX=1` — every bin over one key sends the sort to the LSD
passes after the binning ran.  Graphs are compared with the CPU restatement
and with each other, on inputs whose keys live in one word (K <= 32), two
(K <= 64) and three (K = 96), with palindromes and cycles."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = [pytest.mark.gpu, pytest.mark.timeout(600)]

CHILD = r"""
import hashlib, json, sys
sys.path.insert(0, {root!r})
import torch  # noqa: F401  (loads the HIP runtime libapg binds to, as bench.py and the other tests do)
import numpy as np
import oracle
from allpathslg_amd import Context, synth_genome, synth_reads
from tests.unipath_cases import circular_reads, noisy_reads, palindrome_reads
from tests.test_gpu_unipath import KEYS, assert_graph_equal

cases = [("palindromes", palindrome_reads(), 4), ("noisy25", noisy_reads(G=30_000, n=6000), 25),
         ("noisy33", noisy_reads(G=30_000, n=6000), 33), ("circular63", circular_reads(synth_genome(3000, 11)), 63),
         ("synth96", synth_reads(synth_genome(300_000, 61), 40_000, seed=62), 96)]
out = {{}}
with Context(device=0) as ctx:
    for name, reads, K in cases:
        got, st = ctx.unipaths(reads, K)
        assert_graph_equal(got, oracle.unipaths(reads, K))
        h = hashlib.sha256()
        for k in KEYS:
            v = got[k]
            h.update(np.ascontiguousarray(v).tobytes() if isinstance(v, np.ndarray) else str(v).encode())
        out[name] = [h.hexdigest(), int(st["n_unipaths"])]
print("RESULT " + json.dumps(out))
"""


def run(env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    r = subprocess.run([sys.executable, "-c", CHILD.format(root=ROOT)], capture_output=True, text=True, env=env,
                       cwd=ROOT, timeout=500)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([x for x in r.stdout.splitlines() if x.startswith("RESULT ")][-1][7:])


def test_pair_key_sort_forms_agree():
    one_pass = run({})
    lsd = run({"APG_U_SORT": "lsd"})
    fallback = run({"APG_U_SORT_BINMAX": "1"})
    assert one_pass == lsd == fallback
    assert all(v[1] > 0 for v in one_pass.values())
