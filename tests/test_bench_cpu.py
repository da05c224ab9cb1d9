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


def test_counters_fail_closed(tmp_path):
    """VERDICT r05 Weak 7: bench.py reports PMC traffic / FP64 flops only
    when profiles/traffic_latest.json was measured on the library this run
    loaded (its source key, phasetype_amd.lib_key) and on the same workload; otherwise null."""
    sys.path.insert(0, REPO)
    import bench

    f = tmp_path / "t.json"
    rec = {"n": 10, "N_local": 1000000, "method": "ECS", "hbm_bytes_per_launch": 1.5e7,
           "fp64_flops_per_launch": 1.1e10, "lib_key": "ab" * 32, "pmc_dir": "profiles/r06/x"}
    f.write_text(json.dumps(rec))
    t, fl, why = bench.load_counters(str(f), 10, 1000000, "ECS", "ab" * 32)
    assert (t, fl) == (1.5e7, 1.1e10) and "profiles/r06/x" in why
    t, fl, why = bench.load_counters(str(f), 10, 1000000, "ECS", "cd" * 32)
    assert t is None and fl is None and "not reported" in why
    t, fl, _ = bench.load_counters(str(f), 10, 125000, "ECS", "ab" * 32)
    assert t is None and fl is None
    del rec["lib_key"]
    f.write_text(json.dumps(rec))
    assert bench.load_counters(str(f), 10, 1000000, "ECS", "ab" * 32)[:2] == (None, None)
    assert bench.load_counters(str(tmp_path / "missing.json"), 10, 1000000, "ECS", "ab" * 32)[:2] == (None, None)


def test_committed_counters_name_a_library():
    """The committed counter file carries the library hash and its PMC directory."""
    d = json.load(open(os.path.join(REPO, "profiles", "traffic_latest.json")))
    assert (d.get("lib_key") or "").startswith(("src:", "file:")) and os.path.isdir(os.path.join(REPO, d["pmc_dir"]))
