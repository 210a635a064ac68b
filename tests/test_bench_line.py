"""bench.py's result line stays driver-parseable (the r04
line grew to ~21 KB and the driver's bounded stdout tail could not parse it).

Runs the line builder on a recorded full result (profiles/r04_v4's bench
output, ~90 kernels and every sub-benchmark) and checks the compact line's
size, its contract fields, and that side-stream kernels never become the
roofline kernel.  CPU only."""
import argparse
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REC = os.path.join(ROOT, "profiles", "r04_v4", "bench_final.json")


def _bench():
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _recorded():
    if not os.path.exists(REC):
        pytest.skip("recorded bench output absent")
    out = json.load(open(REC))
    steps = out["steps"]
    # kernel_times() form: name -> (total ms, launches, algorithmic bytes)
    kt = {k: (v["ms_per_launch"] * v["launches"], v["launches"],
              v["GBps"] * 1e9 * v["ms_per_launch"] * 1e-3 * v["launches"]) for k, v in out["kernels"].items()}
    return out, kt, steps


def test_result_line_under_limit_and_complete():
    b = _bench()
    out, kt, steps = _recorded()
    a = argparse.Namespace(steps=steps, traffic_json=os.path.join(ROOT, "profiles", "current", "pmc", "traffic.json"),
                           lds_json=os.path.join(ROOT, "profiles", "current", "pmc", "lds.json"))
    tj = json.load(open(a.traffic_json))
    lj = json.load(open(a.lds_json))
    ov = {"sk_bucket": steps}  # the fused K+1 pass runs on the side stream
    out["roofline"] = b.roofline_summary(kt, ov, tj, lj, a)
    line = b.result_line(out, "gpurun_out/bench_detail.json")
    assert len(line) < 8192
    assert len(line) < 5000, len(line)  # headroom for the driver's tail (stderr follows stdout there)
    d = json.loads(line)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config", "roofline",
              "cpu_baseline", "checks"):
        assert k in d
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r
    assert r["kernel"] != "sk_bucket"  # overlapped kernels are reported apart
    assert [e["kernel"] for e in r["overlapped"]] == ["sk_bucket"]
    assert len(r["next"]) <= 3
    assert d["cpu_baseline"]["cores"] >= 1 and d["cpu_baseline"]["kind"] == "port"
    assert d["end_to_end"]["reads_per_s"] > 0
    assert "workload" in d["config"]
    assert d["traffic_source" if False else "roofline"]["traffic_source"].startswith("profiles/")


def test_result_line_refuses_oversized():
    b = _bench()
    out, kt, steps = _recorded()
    a = argparse.Namespace(steps=steps, traffic_json="/nonexistent", lds_json="/nonexistent")
    out["roofline"] = b.roofline_summary(kt, {}, {}, {}, a)
    out["config"]["workload"] = "x" * 9000
    with pytest.raises(RuntimeError):
        b.result_line(out, None)
