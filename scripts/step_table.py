"""Per-kernel table of ONE graph-replayed training step from a rocprofv3 kernel trace (steps delimited
by the Adam kernel; the step with the smallest span, i.e. a replay, is taken).
usage: python scripts/step_table.py gpurun_out/<tag>/run_kernel_trace.csv [top]"""
import collections
import csv
import re
import sys


def short(n):
    n = re.sub(r'^void ', '', n)
    n = re.sub(r'\(anonymous namespace\)::', '', n)
    n = re.sub(r'_ZN12_GLOBAL__N_1\d+', '', n)
    return re.sub(r'\(.*', '', n)[:72]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 24
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if 'adam_kernel' in r['Kernel_Name']]
    best = None
    for a, b in zip(idx, idx[1:]):
        seq = rows[a + 1:b + 1]
        span = int(seq[-1]['End_Timestamp']) - int(seq[0]['Start_Timestamp'])
        if best is None or span < best[0]:
            best = (span, seq)
    span, seq = best
    d = collections.defaultdict(lambda: [0, 0.0])
    for r in seq:
        k = short(r['Kernel_Name'])
        d[k][0] += 1
        d[k][1] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    busy = sum(v[1] for v in d.values())
    print(f"one replayed step: span {span / 1e3:.0f} us, busy {busy:.0f} us, {len(seq)} launches")
    for k, (n, t) in sorted(d.items(), key=lambda x: -x[1][1])[:top]:
        print(f"{t:8.1f} us  n={n:3d}  avg={t / n:7.1f}  {k}")


if __name__ == "__main__":
    main()
