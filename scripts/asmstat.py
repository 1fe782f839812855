"""Instruction mix of one kernel's basic blocks in a hipcc -S listing (tuning aid, not product).
usage: python scripts/asmstat.py file.s <kernel-substring> [--body]"""
import re
import sys
from collections import Counter


def kernel_lines(path, sub):
    out, on = [], False
    for ln in open(path):
        if re.match(r"^_Z\S*:", ln):
            on = sub in ln
            continue
        if on:
            if ln.startswith("\t.section") or ln.strip().startswith(".Lfunc_end"):
                break
            out.append(ln.rstrip("\n"))
    return out


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_exp") or op.startswith("v_log") or op.startswith("v_rcp"):
        return "trans"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "ds"
    if op.startswith(("global_", "buffer_")):
        return "vmem"
    if op == "s_waitcnt":
        return "wait"
    if op == "s_barrier":
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, sub = sys.argv[1], sys.argv[2]
    lines = kernel_lines(path, sub)
    blocks, cur, name = [], [], "entry"
    for ln in lines:
        m = re.match(r"^(\.LBB\S+):", ln)
        if m:
            blocks.append((name, cur))
            name, cur = m.group(1), []
            continue
        s = ln.strip()
        if not s or s.startswith((";", ".", "//")):
            continue
        cur.append(s.split()[0])
    blocks.append((name, cur))
    tot = Counter()
    for name, ops in blocks:
        c = Counter(classify(o) for o in ops)
        tot += c
        if len(ops) > int(__import__("os").environ.get("MINOPS", "40")):
            print(f"{name:16s} n={len(ops):5d} " + " ".join(f"{k}={c[k]}" for k in
                  ("mfma", "valu", "trans", "ds", "vmem", "wait", "barrier", "salu")))
    print("total", dict(tot))
    if "--body" in sys.argv:
        big = max(blocks, key=lambda b: len(b[1]))
        print(big[0])


if __name__ == "__main__":
    main()
