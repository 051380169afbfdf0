"""bench/_watchdog.py: the guard that keeps bench.py's one JSON line from being lost.

CPU only: a stand-in parent streams snapshots into the watchdog exactly as bench.py's
``Phases`` does, and each of the three endings is checked -- DONE (silent), EOF before
DONE (prints the last snapshot, ``aborted``) and the deadline (prints the last snapshot with
the phase it hung in, then SIGKILLs the parent).
"""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WD = os.path.join(ROOT, "bench", "_watchdog.py")

PARENT = r"""
import json, os, subprocess, sys, time
mode, marker, deadline = sys.argv[1], sys.argv[2], float(sys.argv[3])
w = subprocess.Popen([sys.executable, %r, repr(deadline), marker, str(os.getpid())], stdin=subprocess.PIPE)
snap = {"metric": "m", "value": 1.5, "phase_s": {}}
w.stdin.write((json.dumps(snap) + "\n").encode()); w.stdin.flush()
w.stdin.write(b"PHASE slow_side\n"); w.stdin.flush()
snap["phase_s"]["infer"] = 0.1
w.stdin.write((json.dumps(snap) + "\n").encode()); w.stdin.flush()
if mode == "done":
    fd = os.open(marker, os.O_CREAT | os.O_EXCL | os.O_WRONLY); os.close(fd)
    print(json.dumps(dict(snap, final=True)), flush=True)
    w.stdin.write(b"DONE\n"); w.stdin.flush(); w.wait()
elif mode == "crash":
    os._exit(3)                       # dies after the headline without printing
else:
    time.sleep(60)                    # a hung side measurement
""" % WD


def _run(mode, tmp_path, deadline_in=30.0):
    marker = str(tmp_path / f"marker_{mode}")
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", PARENT, mode, marker, repr(time.time() + deadline_in)],
                       capture_output=True, text=True, timeout=90)
    time.sleep(0.3)   # the watchdog may print just after the parent exits (EOF path)
    return r, time.time() - t0


def _lines(r):
    return [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_done_prints_exactly_one_line(tmp_path):
    r, _ = _run("done", tmp_path)
    ls = _lines(r)
    assert r.returncode == 0 and len(ls) == 1 and ls[0]["final"] is True, r.stdout + r.stderr


def test_parent_crash_keeps_the_headline(tmp_path):
    marker = str(tmp_path / "marker_crash")
    out = tmp_path / "out.txt"
    with open(out, "w") as f:   # the watchdog outlives the parent: read its output from a file
        p = subprocess.run([sys.executable, "-c", PARENT, "crash", marker, repr(time.time() + 30)], stdout=f,
                           stderr=subprocess.PIPE, timeout=60)
    for _ in range(50):
        ls = [json.loads(ln) for ln in out.read_text().splitlines() if ln.startswith("{")]
        if ls:
            break
        time.sleep(0.1)
    assert p.returncode == 3
    assert len(ls) == 1 and ls[0]["value"] == 1.5 and ls[0]["phase_s"] == {"infer": 0.1}, ls
    assert "aborted" in ls[0]["budget"] and ls[0]["budget"]["last_phase"] == "slow_side"


def test_deadline_prints_snapshot_and_ends_the_job(tmp_path):
    r, dt = _run("hang", tmp_path, deadline_in=2.0)
    ls = _lines(r)
    assert r.returncode == -9, (r.returncode, r.stderr)        # SIGKILLed instead of sleeping 60 s
    assert dt < 30
    assert len(ls) == 1 and ls[0]["budget"]["exceeded_in"] == "slow_side", r.stdout


def test_line_order_ends_with_summary():
    """bench.py's line: the contract's keys first, scalar secondaries next, detail objects, then
    a compact ``summary`` LAST (a stored tail of a long line still carries the secondary metric)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("sml_bench_main", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    out = {"infer": {"runs": [1, 2]}, "metric": "m", "value": 48447797557.72098, "unit": "rows/s", "n_gpus": 1,
           "p50_infer_us": 4.37612, "keras_batch32": {"rows_per_s": 16829151.4, "vs_baseline": 268.57},
           "config": {"model": "ae"}, "steps": 20, "kafka_e2e_p50_us": 8.973}
    line = bench.ordered_line(out)
    keys = list(line)
    assert keys[:3] == ["metric", "value", "unit"] and keys[-1] == "summary"
    assert keys.index("p50_infer_us") < keys.index("infer")
    s = line["summary"]
    assert s["headline_rows_per_s"] == 4.845e10 and s["ae_infer_p50_us"] == 4.376
    assert s["vs_baseline_same_batch32"] == 268.6 and s["ae_kafka_e2e_p50_us"] == 8.973
    assert "lstm_seq50_windows_per_s" not in s
    json.dumps(line)
