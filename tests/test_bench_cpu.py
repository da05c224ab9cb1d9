"""CPU: bench.py's CPU comparison legs (no GPU).

oracle/cpu_best.py is the "best CPU" line of SURVEY.md §8(d): the reference
on W cores, observations split.  Bar: it runs as a child process, reports the
fields bench.py copies into its JSON line, and scales its sample to the full
N it was asked about.
"""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_best_line():
    cmd = [sys.executable, "-m", "oracle.cpu_best", "--n", "3", "--N", "4000", "--workers", "2", "--seconds", "0.5"]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stderr[-2000:]
    d = json.loads(p.stdout.strip().splitlines()[-1])
    assert set(d) >= {"value", "unit", "cores", "kind", "sample"}
    assert d["value"] > 0 and d["cores"] == 2 and d["unit"] == "iterations/s"
    assert d["kind"] in ("reference", "port")
    assert "N=4000" in d["sample"]


def test_bench_help():
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--help"], capture_output=True, text=True,
                       timeout=120)
    assert p.returncode == 0 and "--no-cpu-baseline" in p.stdout
