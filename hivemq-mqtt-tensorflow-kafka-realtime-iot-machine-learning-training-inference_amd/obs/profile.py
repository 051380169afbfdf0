"""Profiling helpers.

The reference profiles with the Keras ``TensorBoard`` callback (TF profiler
trace of batch 2, CPU only, python-scripts/autoencoder-anomaly-detection/logs/
plugins/profile/*/local.trace).  On MI355X the tools are:

* ``rocprofv3 --kernel-trace --stats`` for per-kernel device time, and a
  separate ``--pmc`` run for counters (MFMA / VALU / LDS / HBM) --
  :func:`rocprof_command` builds both command lines the way the GPU pool
  requires (program directly after ``--``, counters never combined with
  runtime / system tracing);
* :func:`load_kernel_stats` / :func:`stats_markdown` turn the
  ``*_kernel_stats.csv`` into the tables committed under ``profiles/``;
* :class:`DeviceTimer` -- HIP-event section timing without host syncs inside
  the timed region;
* :func:`torch_trace` -- ``torch.profiler`` host + device timeline exported as a
  chrome trace (``roctx`` ranges via :func:`range_push` / :func:`range_pop`).
"""
from __future__ import annotations

import contextlib
import csv
import os
import re
from typing import Dict, List, Optional, Sequence

PMC_DEFAULT = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
               "SQ_INSTS_VMEM_WR", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES"]


def rocprof_command(program: Sequence[str], out_dir: str, name: str = "run", pmc: Optional[Sequence[str]] = None,
                    csv_out: bool = True) -> List[str]:
    """``rocprofv3`` argv: kernel trace + stats, or a counter run when ``pmc`` is given.

    The program (e.g. ``["python3", "bench.py", "--steps", "5"]``) goes directly
    after ``--``: wrappers such as ``env`` / ``bash -c`` would exec from a
    process the profiler already attached to the GPU.
    """
    if program and os.path.basename(program[0]) in ("env", "bash", "sh", "taskset", "numactl"):
        raise ValueError("put the program itself after '--' (no env / shell / launcher)")
    cmd = ["rocprofv3", "--kernel-trace"]
    if pmc:
        cmd += ["--pmc", *pmc]
    else:
        cmd += ["--stats"]
    if csv_out:
        cmd += ["--output-format", "csv"]
    cmd += ["-d", out_dir, "-o", name, "--", *program]
    return cmd


def load_kernel_stats(path: str) -> List[Dict]:
    """Rows of a rocprofv3 ``*_kernel_stats.csv`` (Name, Calls, TotalDurationNs, AverageNs, Percentage...)."""
    rows = []
    with open(path, newline="") as f:
        for r in csv.DictReader(f):
            rows.append({"name": r.get("Name", ""), "calls": int(float(r.get("Calls", 0) or 0)),
                         "total_us": float(r.get("TotalDurationNs", 0) or 0) / 1e3,
                         "avg_us": float(r.get("AverageNs", 0) or 0) / 1e3,
                         "pct": float(r.get("Percentage", 0) or 0)})
    rows.sort(key=lambda r: -r["total_us"])
    return rows


def short_kernel_name(name: str, width: int = 70) -> str:
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    n = n.replace("sml::", "")
    # drop the argument list, keep template args
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            n = n[:i]
            break
    return n if len(n) <= width else n[:width - 3] + "..."


def stats_markdown(rows: List[Dict], top: int = 15) -> str:
    out = ["| kernel | calls | avg us | total us | % |", "|---|---:|---:|---:|---:|"]
    for r in rows[:top]:
        out.append(f"| `{short_kernel_name(r['name'])}` | {r['calls']} | {r['avg_us']:.1f} | "
                   f"{r['total_us']:.0f} | {r['pct']:.1f} |")
    return "\n".join(out)


class DeviceTimer:
    """Accumulating HIP-event timer: ``with t.section("fwd"): ...``; read with :meth:`summary`
    (one synchronize at read time, none inside the timed code)."""

    def __init__(self, enabled: bool = True):
        import torch
        self.enabled = enabled and torch.cuda.is_available()
        self._events: Dict[str, List] = {}

    @contextlib.contextmanager
    def section(self, name: str):
        if not self.enabled:
            yield
            return
        import torch
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        try:
            yield
        finally:
            e.record()
            self._events.setdefault(name, []).append((s, e))

    def summary(self) -> Dict[str, Dict[str, float]]:
        if not self.enabled:
            return {}
        import torch
        torch.cuda.synchronize()
        out = {}
        for k, evs in self._events.items():
            ts = [s.elapsed_time(e) * 1e3 for s, e in evs]
            out[k] = {"calls": len(ts), "total_us": sum(ts), "avg_us": sum(ts) / len(ts)}
        return out


def range_push(name: str) -> None:
    import torch
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_push(name)   # roctx on ROCm builds


def range_pop() -> None:
    import torch
    if torch.cuda.is_available():
        torch.cuda.nvtx.range_pop()


@contextlib.contextmanager
def torch_trace(out_path: str, with_stack: bool = False):
    """Chrome-trace of host ops + device kernels for the enclosed region."""
    import torch
    acts = [torch.profiler.ProfilerActivity.CPU]
    if torch.cuda.is_available():
        acts.append(torch.profiler.ProfilerActivity.CUDA)
    with torch.profiler.profile(activities=acts, with_stack=with_stack) as prof:
        yield prof
    os.makedirs(os.path.dirname(os.path.abspath(out_path)), exist_ok=True)
    prof.export_chrome_trace(out_path)
