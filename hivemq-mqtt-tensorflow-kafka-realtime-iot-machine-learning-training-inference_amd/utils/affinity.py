"""CPU placement for the latency-critical host threads (the ``serve --low-latency`` loop, a
paced producer, the in-process broker's connection threads).

A loopback TCP hop between two threads costs ~2.3 us when both run in one core complex (one
L3) and ~4.7 us across complexes; unpinned, the scheduler picks either, run to run
(profiles/r04/SUMMARY.md §7).  ``l3_cpus`` returns distinct physical cores of one L3 domain
from this process's affinity set; ``parse_cpus`` reads taskset's list syntax.
"""
from __future__ import annotations

import os
from typing import List, Optional, Set


def parse_cpus(spec: str) -> Set[int]:
    """'4', '4-7,12' -> {4, 5, 6, 7, 12} (taskset's list syntax)."""
    out: Set[int] = set()
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        lo, _, hi = part.partition("-")
        lo_i, hi_i = int(lo), int(hi) if hi else int(lo)
        if lo_i < 0 or hi_i < lo_i:
            raise ValueError(f"bad CPU range {part!r}")
        out.update(range(lo_i, hi_i + 1))
    if not out:
        raise ValueError(f"no CPUs in {spec!r}")
    return out


def _read(path: str) -> str:
    with open(path) as f:
        return f.read().strip()


def cpu_busy(sample_s: float = 0.05) -> Optional[dict]:
    """Per-CPU busy fraction over ``sample_s`` from /proc/stat (None where unreadable)."""
    import time

    def snap():
        out = {}
        with open("/proc/stat") as f:
            for line in f:
                if line.startswith("cpu") and line[3:4].isdigit():
                    v = line.split()
                    t = [int(x) for x in v[1:]]
                    idle = t[3] + (t[4] if len(t) > 4 else 0)
                    out[int(v[0][3:])] = (sum(t), idle)
        return out
    try:
        a = snap()
        time.sleep(sample_s)
        b = snap()
    except (OSError, ValueError, IndexError):
        return None
    busy = {}
    for c, (tot, idle) in b.items():
        if c in a:
            dt = tot - a[c][0]
            busy[c] = 0.0 if dt <= 0 else 1.0 - (idle - a[c][1]) / dt
    return busy


def l3_cpus(k: int, slot: int = 0, avoid_busy: bool = True) -> Optional[List[int]]:
    """``k`` CPUs of this process's affinity set sharing one L3, one per physical core (None:
    cache topology not readable, or no L3 domain with ``k`` allowed cores).

    ``slot`` (e.g. a replica's rank) picks the domain round-robin in a DETERMINISTIC order (by
    first CPU): replicas started one after another each sample the load on their own, so an
    order derived from that sample would differ between them and two replicas could land on one
    domain while another stays unused.  Inside the chosen domain, spinning latency-critical
    threads lose whole scheduler slices (ms) to any other runnable thread on their CPU, so with
    ``avoid_busy`` the ``k`` least-busy cores are taken (a 50 ms /proc/stat sample; CPU 0, which
    services most housekeeping, last)."""
    groups = {}
    for c in sorted(os.sched_getaffinity(0)):
        try:
            l3 = _read(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list")
            core = _read(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list")
        except OSError:
            return None
        groups.setdefault(l3, {}).setdefault(core, c)   # first allowed CPU of each core
    cands = sorted((sorted(g.values()) for g in groups.values() if len(g) >= k), key=lambda cs: cs[0])
    if not cands:
        return None
    dom = cands[slot % len(cands)]
    busy = cpu_busy() if avoid_busy else None
    if busy:
        def load(c):
            return busy.get(c, 0.0) + (0.5 if c == 0 else 0.0)
        return sorted(sorted(dom, key=lambda c: (load(c), c))[:k])
    return dom[:k]


def resolve_cpus(spec: Optional[str], slot: int = 0) -> Optional[Set[int]]:
    """``--cpus`` value -> CPU set: None / '' = leave placement alone, 'auto' = one core of an L3
    domain chosen by ``slot`` (None when the topology is unknown), else taskset syntax."""
    if not spec:
        return None
    if spec == "auto":
        cs = l3_cpus(1, slot)
        return set(cs) if cs else None
    return parse_cpus(spec)
