"""Instruction mix of one kernel in a hipcc device-assembly dump, per basic block.

    hipcc ... --cuda-device-only -S -o step.s rl_rocket_amd/csrc/rocket_hip.hip
    python tools/isa_count.py step.s 'step_kernelILi6ELi0ELb0ELb1ELi4'   [--blocks]

Classes: valu (v_*, excluding v_readfirstlane / v_writelane / MFMA), trans (v_exp / v_log /
v_rcp / v_rsq / v_sqrt / v_sin / v_cos: 8 issue cycles for a lone wave, 2x a plain VALU op),
vmem (buffer_ / global_), lds (ds_), salu (s_*, excluding waitcnt / branches), waitcnt, branch.
A lone wave per SIMD issues one VALU op per 4 cycles (MI355X_MICROARCH.md, 'vector-instruction
ISSUE cost'), so 4 x valu + 8 x trans approximates its VALU issue cycles.
"""
import re
import sys

TRANS = re.compile(r"^v_(exp|log|rcp|rsq|sqrt|sin|cos)_")


def classify(op):
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("s_cbranch") or op.startswith("s_branch"):
        return "branch"
    if op.startswith("v_mfma"):
        return "mfma"
    if TRANS.match(op):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("buffer_") or op.startswith("global_"):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    blocks = "--blocks" in sys.argv
    lines = open(path).read().split("\n")
    start = None
    for k, ln in enumerate(lines):
        if re.match(r"^_Z\w*:", ln) and pat in ln.split(":")[0]:
            start = k
            break
    if start is None:
        sys.exit("kernel not found")
    tot, bb, name = {}, {}, "entry"
    out = []
    for ln in lines[start + 1:]:
        s = ln.strip()
        if s.startswith(".Lfunc_end"):
            break
        if re.match(r"^\.LBB\w+:", s):
            out.append((name, bb))
            name, bb = s.split(":")[0], {}
            continue
        if not s or s.startswith(";") or s.startswith("."):
            continue
        op = s.split()[0]
        c = classify(op)
        tot[c] = tot.get(c, 0) + 1
        bb[c] = bb.get(c, 0) + 1
    out.append((name, bb))
    if blocks:
        for name, b in out:
            print("%-16s %s" % (name, " ".join("%s=%d" % kv for kv in sorted(b.items()))))
    print("TOTAL", " ".join("%s=%d" % kv for kv in sorted(tot.items())))
    print("lone-wave VALU issue cycles ~ %d" % (4 * tot.get("valu", 0) + 8 * tot.get("trans", 0)))


if __name__ == "__main__":
    main()
