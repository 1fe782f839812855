"""Summarise rocprofv3 --pmc CSVs (one directory per pass) per kernel: the median over a kernel's
dispatches of each counter, plus derived per-wave-tile figures for the attention kernels.
usage: python scripts/sqsum.py gpurun_out/sq3_p1 gpurun_out/sq3_p2 ... [--match attn]"""
import csv
import re
import statistics
import sys
from collections import defaultdict


def short(name):
    name = re.sub(r"\(.*", "", name)
    m = re.search(r"(attn_\w+|gemm\w*|ln_\w+|wgrad\w*|adam\w*)", name)
    return (m.group(1) if m else name[:60]) + ("<drop>" if "Lb1E" in name.split("(")[0][:80] or "<true" in name else "")


def main():
    argv = sys.argv[1:]
    match = argv[argv.index("--match") + 1] if "--match" in argv else ""
    dirs = [a for a in argv if not a.startswith("--") and a != match]
    vals = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values]
    dur = defaultdict(list)
    for d in dirs:
        for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
            k = r["Kernel_Name"]
            if match and match not in k:
                continue
            vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            if r["Counter_Name"] == "SQ_WAVE_CYCLES":
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, cs in vals.items():
        med = {c: statistics.median(v) for c, v in cs.items()}
        print(f"== {k[:110]}")
        if dur.get(k):
            print(f"   dispatches {len(dur[k])}, median duration {statistics.median(dur[k]):.1f} us (profiled)")
        for c in sorted(med):
            print(f"   {c:30s} {med[c]:16.0f}")
        wc = med.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_ACTIVE_INST_VMEM", "SQ_WAIT_INST_LDS"):
                if c in med:
                    print(f"   {c + ' / WAVE_CYCLES':44s} {med[c] / wc:6.3f}")


if __name__ == "__main__":
    main()
