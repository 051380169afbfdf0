#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc counter_collection CSVs per kernel: median over the dispatches
of each kernel name (optionally only dispatches whose grid is at least --min-grid), one row
per kernel, one column per counter; plus per-wave and derived ratios used in profiles/.

usage: pmc_table.py <pass_dir> [<pass_dir> ...] [--min-grid N] [--json]"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import statistics


def load(dirs, min_grid=0):
    rows = collections.defaultdict(lambda: collections.defaultdict(list))
    meta = {}
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if int(r["Grid_Size"]) < min_grid:
                        continue
                    k = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"])[:110]
                    rows[k][(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
                    meta[k] = {"grid": int(r["Grid_Size"]), "wg": int(r["Workgroup_Size"]),
                               "vgpr": int(r["VGPR_Count"]), "agpr": int(r["Accum_VGPR_Count"]),
                               "lds": int(r["LDS_Block_Size"]), "scratch": int(r["Scratch_Size"])}
    out = {}
    for k, d in rows.items():
        per = collections.defaultdict(list)
        for (disp, cn), vals in d.items():
            per[cn].append(sum(vals))        # a dispatch's value summed over its XCD / SE rows
        out[k] = {cn: statistics.median(v) for cn, v in per.items()}
        out[k]["_meta"] = meta[k]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--min-grid", type=int, default=0)
    ap.add_argument("--json", action="store_true")
    a = ap.parse_args()
    t = load(a.dirs, a.min_grid)
    if a.json:
        print(json.dumps(t, indent=1))
        return
    for k, d in sorted(t.items()):
        print(k)
        print("   ", d["_meta"])
        print("   ", {cn: v for cn, v in sorted(d.items()) if cn != "_meta"})


if __name__ == "__main__":
    main()
