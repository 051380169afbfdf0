"""Per-step kernel timeline from a rocprofv3 --kernel-trace SQLite db: for the launches
between consecutive dispatches of a step-marker kernel (default: the Adam launch), the
median duration of each launch position and the median idle gap before it, so a step's
wall time splits into kernel time and launch / dependency gaps.

    python tools/probes/kernel_gaps.py gpurun_out/lstmtrace/.../lt_results.db [--marker adam]
"""
import argparse
import json
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="adam")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    con = sqlite3.connect(a.db)
    rows = con.execute("select name, start, end from kernels order by start").fetchall()
    marks = [i for i, r in enumerate(rows) if a.marker in r[0].lower()]
    steps = [rows[marks[j] + 1: marks[j + 1] + 1] for j in range(len(marks) - 1)]
    if not steps:
        raise SystemExit("no step marker kernels found")
    # keep the modal step shape (warmup / eval steps differ)
    shape = statistics.mode(tuple(r[0] for r in s) for s in steps)
    steps = [s for s in steps if tuple(r[0] for r in s) == shape]
    pos = []
    for k in range(len(shape)):
        durs = [(s[k][2] - s[k][1]) / 1e3 for s in steps]
        gaps = [(s[k][1] - (s[k - 1][2] if k else s[k][1])) / 1e3 for s in steps]
        pos.append({"kernel": shape[k][:70], "dur_us": round(statistics.median(durs), 2),
                    "gap_before_us": round(statistics.median(gaps), 2)})
    walls = [(s[-1][2] - s[0][1]) / 1e3 for s in steps]
    out = {"steps": len(steps), "launches_per_step": len(shape),
           "wall_us_median": round(statistics.median(walls), 1),
           "kernel_us_sum": round(sum(p["dur_us"] for p in pos), 1),
           "gap_us_sum": round(sum(p["gap_before_us"] for p in pos), 1), "positions": pos}
    print(json.dumps({k: v for k, v in out.items() if k != "positions"}))
    for p in pos:
        print(f'{p["dur_us"]:9.2f} {p["gap_before_us"]:7.2f}  {p["kernel"]}')
    if a.json:
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
