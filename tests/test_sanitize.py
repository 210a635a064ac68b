"""The host-side code under the sanitizers (SURVEY §5 "race detection /
sanitizers"): `make sanitize` (tests/sanitize/Makefile) builds libapg's host
sources and the CPU restatement with -fsanitize=address,undefined and
-fsanitize=thread and runs their drivers (formats and their rejected headers,
graph files, simulator worker threads, the TCP communicator at world 1/2/4
with ranks as threads, the oracle's known-answer tests).  CPU only."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_make_sanitize_green():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "sanitize"), "all"], capture_output=True,
                       text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.count("san_host: ok") == 2 and "san_oracle: ok" in out, out[-2000:]
