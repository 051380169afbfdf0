#!/usr/bin/env python3
"""Deadline guard for bench.py's one JSON line (rank 0 only; no torch, no GPU).

bench.py starts this as a CHILD process with a pipe on stdin and the same stdout.  After the
timed headline, rank 0 streams a snapshot of its result line (one JSON object per line) after
every measurement phase.  Three endings:

* ``DONE``  -- rank 0 printed the line itself; exit silently.
* EOF without ``DONE`` -- rank 0 died after the headline (exception, signal): print the last
  snapshot with ``"aborted"`` set, so the measured headline is not lost.
* the deadline passes (a side measurement hung inside a GPU or native call, where no Python
  thread of rank 0 could run): print the last snapshot with ``budget.exceeded_in`` set, then
  SIGKILL rank 0 so the job ends inside the driver's window.

Whoever prints first claims ``marker`` with O_CREAT|O_EXCL, so exactly one line appears.
usage: _watchdog.py <deadline_unix_s> <marker_path> <parent_pid>
"""
import json
import os
import select
import signal
import sys
import time


def claim(marker: str) -> bool:
    try:
        os.close(os.open(marker, os.O_CREAT | os.O_EXCL | os.O_WRONLY, 0o600))
        return True
    except FileExistsError:
        return False


def emit(snap: bytes, marker: str, **flags) -> None:
    if snap is None or not claim(marker):
        return
    d = json.loads(snap)
    b = d.setdefault("budget", {})
    b.update(flags)
    sys.stdout.write(json.dumps(d) + "\n")
    sys.stdout.flush()


def main() -> int:
    deadline, marker, parent = float(sys.argv[1]), sys.argv[2], int(sys.argv[3])
    fd = sys.stdin.fileno()
    snap, buf, phase = None, b"", None
    while True:
        left = deadline - time.time()
        if left <= 0:
            break
        r, _, _ = select.select([fd], [], [], min(left, 0.5))
        if not r:
            continue
        chunk = os.read(fd, 1 << 20)
        if not chunk:                      # rank 0 is gone without DONE
            emit(snap, marker, aborted="rank 0 exited before printing its line", last_phase=phase)
            return 0
        buf += chunk
        while b"\n" in buf:
            line, buf = buf.split(b"\n", 1)
            if line == b"DONE":
                return 0
            if line.startswith(b"PHASE "):
                phase = line[6:].decode()
            elif line.startswith(b"{"):
                snap = line
    emit(snap, marker, exceeded_in=phase, watchdog="deadline passed; rank 0 killed")
    try:
        os.kill(parent, signal.SIGKILL)
    except ProcessLookupError:
        pass
    return 0


if __name__ == "__main__":
    sys.exit(main())
