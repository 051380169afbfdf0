#!/usr/bin/env python3
"""Summarise rocprofv3 kernel-stats CSVs into a markdown table (for profiles/*.md).

    python tools/prof_summary.py gpurun_out/prof_lstm/run_kernel_stats.csv [--top 15]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from streamml.obs.profile import load_kernel_stats, stats_markdown  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    for p in a.csv:
        rows = load_kernel_stats(p)
        tot = sum(r["total_us"] for r in rows)
        print(f"### {p}\n\ntotal device time {tot / 1e3:.2f} ms over {sum(r['calls'] for r in rows)} launches\n")
        print(stats_markdown(rows, a.top))
        print()


if __name__ == "__main__":
    main()
