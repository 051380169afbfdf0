#!/usr/bin/env python3
"""Instruction-issue bound of one kernel's hot loop, from its gfx950 assembly (no GPU).

    hipcc --offload-arch=gfx950 -O3 -S --offload-device-only <flags of _build.py> k.hip -o k.s
    python tools/isa_bound.py k.s '<demangled-name substring>' [--per-trip N]

Splits the kernel into basic blocks, finds the loops (a branch back to an earlier label),
and for the loop body prints the instruction mix and the per-trip SIMD issue cycles under the
measured gfx950 issue costs (MI355X_MICROARCH.md, constants table, row 'vector-instruction
ISSUE cost', one wave's stream on one SIMD): VALU 4, transcendental 8, v_cvt_pk_bf16_f32 4,
an MFMA holds vector issue for 8 cycles (16x16x32 bf16 paces at 16, 32x32x16 at 32), LDS /
VMEM / SALU counted at their issue slot (4).  With W waves per SIMD the vector pipe is shared:
the bound of the SIMD is the SUM over its waves of the VALU + transcendental cycles at the
2-cycle dual-wave VALU rate -- both figures are printed.
"""
import re
import subprocess
import sys
from collections import Counter, OrderedDict

TRANS = ("v_exp_", "v_log_", "v_rcp_", "v_rsq_", "v_sqrt_", "v_sin_", "v_cos_")


def demangle(name):
    try:
        return subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    except Exception:
        return name


def kernel_body(lines, sub):
    start = None
    for i, ln in enumerate(lines):
        m = re.match(r"^(_Z\S+):", ln)
        if m:
            if start is not None:
                return lines[start:i]
            if sub in demangle(m.group(1)):
                start = i
    if start is None:
        raise SystemExit("kernel not found: " + sub)
    return lines[start:]


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith(TRANS):
        return "trans"
    if op.startswith("v_cvt_pk_bf16"):
        return "cvt_bf16"
    if op.startswith("v_accvgpr"):
        return "accvgpr"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_")):
        return "vmem"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_nop"):
        return "nop"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    with open(path) as f:
        lines = f.read().splitlines()
    body = kernel_body(lines, sub)
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = []
    for ln in body:
        s = ln.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            cur = m.group(1)
            blocks[cur] = []
            continue
        if not s or s.startswith((";", ".", "_Z")):
            continue
        blocks[cur].append(s.split()[0])
    names = list(blocks)
    loops = []   # back edges: a branch in block i to a label at index <= i
    targets = {}
    cur = "entry"
    for ln in body:
        s = ln.strip()
        m = re.match(r"^(\.LBB\S+):", s)
        if m:
            cur = m.group(1)
            continue
        m = re.match(r"^s_(cbranch_\w+|branch)\s+(\.LBB\S+)", s)
        if m:
            targets.setdefault(cur, []).append(m.group(2))
    for i, b in enumerate(names):
        for t in targets.get(b, []):
            if t in blocks and names.index(t) <= i:
                loops.append((names.index(t), i))
    if not loops:
        raise SystemExit("no loop found")
    # the hot loop: the one with the most MFMAs
    def mix(lo, hi):
        c = Counter()
        for b in names[lo:hi + 1]:
            for op in blocks[b]:
                c[classify(op)] += 1
        return c
    best = max(loops, key=lambda lh: mix(*lh)["mfma"])
    c = mix(*best)
    mf_ops = Counter(op for b in names[best[0]:best[1] + 1] for op in blocks[b] if op.startswith("v_mfma"))
    print("kernel:", sub)
    print("hot loop: blocks %s .. %s (%d blocks)" % (names[best[0]], names[best[1]], best[1] - best[0] + 1))
    for k in ("mfma", "valu", "trans", "cvt_bf16", "accvgpr", "lds", "vmem", "salu", "waitcnt", "nop", "other"):
        print("  %-9s %5d" % (k, c[k]))
    for op, n in mf_ops.items():
        print("  %-40s %d" % (op, n))
    mfma_pace = sum(n * (32 if "32x32" in op else 16) for op, n in mf_ops.items())
    issue_one = 8 * c["mfma"] + 4 * (c["valu"] + c["cvt_bf16"] + c["accvgpr"]) + 8 * c["trans"] + \
        4 * (c["lds"] + c["vmem"] + c["salu"] + c["nop"])
    valu_pipe = 2 * (c["valu"] + c["cvt_bf16"] + c["accvgpr"]) + 8 * c["trans"]
    print("per trip, one wave alone: issue %d cyc, MFMA pacing %d cyc -> bound max = %d cyc" %
          (issue_one, mfma_pace, max(issue_one, mfma_pace)))
    print("per trip, SIMD vector pipe (VALU at the 2-cycle rate, trans 8): %d cyc + MFMA %d cyc" % (valu_pipe, mfma_pace))


if __name__ == "__main__":
    main()
