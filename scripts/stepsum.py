"""Per-kernel time of one training step from a rocprofv3 kernel trace (steps delimited by the Adam
kernel): python scripts/stepsum.py TRACE_CSV [step_index]"""
import collections
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(rows) if 'adam_kernel' in r['Kernel_Name']]
k = int(sys.argv[2]) if len(sys.argv) > 2 else len(idx) // 2
a, b = idx[k - 1], idx[k]
d = collections.defaultdict(lambda: [0, 0.0])
for i in range(a + 1, b + 1):
    n = rows[i]['Kernel_Name']
    n = re.sub(r'^void ', '', n)
    n = re.sub(r'\(anonymous namespace\)::', '', n)
    n = re.sub(r'_ZN12_GLOBAL__N_1\d+', '', n)
    key = re.sub(r'\((?!anon).*$', '', n)[:80] + ' g=' + rows[i]['Grid_Size_X']
    d[key][0] += 1
    d[key][1] += (int(rows[i]['End_Timestamp']) - int(rows[i]['Start_Timestamp'])) / 1e3
tot = sum(v[1] for v in d.values())
span = (int(rows[b]['End_Timestamp']) - int(rows[a]['End_Timestamp'])) / 1e3
print(f'step {k}: busy {tot:.0f} us, span {span:.0f} us, {b - a} launches')
for key, v in sorted(d.items(), key=lambda kv: -kv[1][1]):
    print(f"{v[1]:8.1f} us  n={v[0]:3d}  avg={v[1] / v[0]:7.1f}  {key}")
