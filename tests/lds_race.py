"""Static check of the gfx950 code objects for the "fill overtakes read" LDS hazard (test infrastructure).

The hazard (found in the exchange main loop): a wave issues ds_read* from an LDS
stage, passes a raw ``s_barrier`` before those reads have returned (no covering ``s_waitcnt lgkmcnt``),
and another wave, released by that barrier, refills the stage by LDS-DMA (``global_load_lds_*`` /
``buffer_load_* ... lds``, untracked by the compiler when issued from inline asm).  A read still queued
behind that traffic returns the NEW bytes.  ``__syncthreads()`` is safe (the compiler drains lgkmcnt before
its barrier); raw barriers in LDS-DMA kernels are not, unless the stage read before the barrier is not the
one refilled after it.

The check: extract every amdgcn code object from the library's clang offload bundles, disassemble it with
ROCm's llvm-objdump, build each kernel's control-flow graph from the branch instructions, and propagate
"LDS reads possibly in flight" (a ds_read* adds one; ``s_waitcnt lgkmcnt(N)`` bounds the count by N) to a
fixed point.  In kernels that issue LDS-DMA, every ``s_barrier`` reached with a possibly-outstanding LDS
read and followed (on some path) by an LDS-DMA instruction is reported.
"""
import os
import re
import struct
import subprocess
import tempfile
from collections import defaultdict

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_SAT = 64  # the count saturates (lgkmcnt is 4 bits on gfx9; any positive count is a finding)


def code_objects(path):
    """The amdgcn code objects (ELF bytes) bundled in a shared library or object file."""
    data = open(path, "rb").read()
    out = []
    i = data.find(_MAGIC)
    while i >= 0:
        n = struct.unpack_from("<Q", data, i + len(_MAGIC))[0]
        off = i + len(_MAGIC) + 8
        for _ in range(n):
            o, sz, tl = struct.unpack_from("<QQQ", data, off)
            triple = data[off + 24:off + 24 + tl].decode(errors="replace")
            off += 24 + tl
            if "amdgcn" in triple and sz:
                out.append(data[i + o:i + o + sz])
        i = data.find(_MAGIC, i + 1)
    return out


def disassemble(path):
    """llvm-objdump -d text of every code object in ``path`` (concatenated)."""
    texts = []
    with tempfile.TemporaryDirectory() as td:
        for k, co in enumerate(code_objects(path)):
            f = os.path.join(td, f"co{k}.elf")
            open(f, "wb").write(co)
            texts.append(subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", "--no-show-raw-insn", f], check=True,
                                        capture_output=True, text=True).stdout)
    return "\n".join(texts)


_FUNC = re.compile(r"^([0-9a-f]+) <(.+)>:\s*$")
_INSN = re.compile(r"^\s+([a-z_0-9]+)\b(.*?)(?://\s*([0-9A-F]+):(.*))?$")
_TARGET = re.compile(r"<(.+?)\+0x([0-9a-f]+)>")


def kernels(text):
    """{symbol: [(offset, mnemonic, operand text)]} of the functions in an llvm-objdump listing."""
    out = {}
    cur = None
    for ln in text.splitlines():
        m = _FUNC.match(ln)
        if m:
            cur = m.group(2)
            out[cur] = []
            continue
        if cur is None or not ln.strip() or ln.lstrip().startswith(";"):
            continue
        m = _INSN.match(ln)
        if m and m.group(3):
            ops = m.group(2).strip()
            t = _TARGET.search(m.group(4) or "")  # a branch's target, printed in the trailing comment
            out[cur].append((int(m.group(3), 16), m.group(1), ops + (f" {t.group(0)}" if t else "")))
    return {k: v for k, v in out.items() if v}


def _lgkm(ops):
    m = re.search(r"lgkmcnt\((\d+)\)", ops)
    return int(m.group(1)) if m else None


def _is_dma(mn, ops):
    return mn.startswith("global_load_lds") or (mn.startswith("buffer_load") and re.search(r"\blds\b", ops))


def uses_lds_dma(insns):
    return any(_is_dma(mn, ops) for _, mn, ops in insns)


def barriers_with_reads_in_flight(insns, depth=1):
    """Offsets of the s_barrier instructions that may be reached with LDS reads outstanding (depth 1), or
    with reads outstanding that were issued before the PREVIOUS barrier (depth 2: kernels whose stages
    are refilled only two barriers after their last read, the 8-wave phased GEMMs)."""
    if not insns:
        return []
    base = insns[0][0]
    idx = {off: i for i, (off, _, _) in enumerate(insns)}
    # basic-block leaders: entry, branch targets, instructions after a branch
    succ = defaultdict(list)
    leaders = {0}
    for i, (off, mn, ops) in enumerate(insns):
        if mn.startswith("s_branch") or mn.startswith("s_cbranch"):
            t = _TARGET.search(ops)
            if t:  # llvm-objdump prints <symbol+0xOFF>, relative to the function symbol
                tgt = base + int(t.group(2), 16)
                if tgt in idx:
                    leaders.add(idx[tgt])
                    succ[i].append(idx[tgt])
            if i + 1 < len(insns):
                leaders.add(i + 1)
                if mn.startswith("s_cbranch"):
                    succ[i].append(i + 1)
        elif mn in ("s_endpgm", "s_setpc_b64") and i + 1 < len(insns):
            leaders.add(i + 1)
    order = sorted(leaders)
    blocks = []
    for k, s in enumerate(order):
        e = order[k + 1] if k + 1 < len(order) else len(insns)
        blocks.append((s, e))
    start_of = {s: k for k, (s, _) in enumerate(blocks)}
    bsucc = defaultdict(set)
    for k, (s, e) in enumerate(blocks):
        last = e - 1
        mn = insns[last][1]
        for t in succ.get(last, []):
            bsucc[k].add(start_of[t])
        if not (mn.startswith("s_branch") or mn in ("s_endpgm", "s_setpc_b64")) and e < len(insns):
            if not succ.get(last) or mn.startswith("s_cbranch"):
                bsucc[k].add(start_of[e])
    # blocks from which an LDS-DMA instruction is reachable (a barrier after which no wave fills LDS any
    # more — the epilogue's staging passes, whose ds_writes queue behind earlier reads — is no hazard)
    has_dma = {k for k, (s, e) in enumerate(blocks) if any(_is_dma(insns[i][1], insns[i][2]) for i in range(s, e))}
    reach = set(has_dma)
    changed = True
    while changed:
        changed = False
        for k in range(len(blocks)):
            if k not in reach and bsucc[k] & reach:
                reach.add(k)
                changed = True

    def dma_after(k, i):
        s, e = blocks[k]
        return any(_is_dma(insns[j][1], insns[j][2]) for j in range(i + 1, e)) or bool(bsucc[k] & reach)

    # state: (LDS reads possibly outstanding, of which issued before the last barrier); LDS returns in
    # order, so lgkmcnt(N) leaves at most the N youngest
    state_in = {0: (0, 0)}
    work = [0]
    flagged = set()
    while work:
        k = work.pop()
        cur, old = state_in[k]
        s, e = blocks[k]
        for i in range(s, e):
            off, mn, ops = insns[i]
            if mn == "s_barrier":
                if (old if depth == 2 else cur + old) > 0 and dma_after(k, i):
                    flagged.add(off - base)
                cur, old = 0, min(cur + old, _SAT)
            elif mn.startswith("ds_read") or mn.startswith("ds_load"):
                cur = min(cur + 1, _SAT)
            elif mn.startswith("s_waitcnt"):
                c = _lgkm(ops)
                if c is not None:
                    cur = min(cur, c)
                    old = min(old, max(c - cur, 0))
        for t in bsucc[k]:
            a, b = state_in.get(t, (-1, -1))
            if cur > a or old > b:
                state_in[t] = (max(cur, a), max(old, b))
                work.append(t)
    return sorted(flagged)


# The 8-wave phased 256-row GEMMs (gemm8_kernel, and wgrad8_grouped_kernel on the same main loop) leave
# LDS reads in flight across a raw barrier by design: a K-tile's B images are refilled only in phase 3 and
# its A images in phase 0 of the next K-tile, two barriers after their last read (the slot-reuse invariant
# at repurpose_amd/csrc/rp_gemm.hip, "Slot reuse ... INVARIANT", above gemm8_tile).  Their check is depth
# 2: no read may still be in flight at the second barrier after it was issued.
DEPTH2 = ("gemm8_kernel", "wgrad8_grouped_kernel")


def scan(text):
    """{kernel: [barrier offsets]} for the LDS-DMA kernels of a listing that pass a barrier with LDS reads
    possibly in flight (depth 2 for the DEPTH2 kernels)."""
    out = {}
    for name, insns in kernels(text).items():
        if not uses_lds_dma(insns):
            continue
        bad = barriers_with_reads_in_flight(insns, 2 if any(d in name for d in DEPTH2) else 1)
        if bad:
            out[name] = bad
    return out
