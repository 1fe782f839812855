"""Per-dispatch timeline of one training step from a rocprofv3 kernel_trace.csv:
python scripts/steptrace.py TRACE.csv [step_index]  (steps delimited by adam_kernel launches)"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
steps, cur = [], []
for r in rows:
    cur.append(r)
    if "adam_kernel" in r["Kernel_Name"]:
        steps.append(cur)
        cur = []
st = steps[which]
t0 = int(st[0]["Start_Timestamp"])
tot = 0.0
agg = {}
for r in st:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][:60]
    g = f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}/{r["Workgroup_Size_X"]}'
    key = (n, g)
    a = agg.setdefault(key, [0, 0.0])
    a[0] += 1
    a[1] += d
span = (int(st[-1]["End_Timestamp"]) - t0) / 1e3
print(f"step span {span:.1f} us, kernel sum {tot:.1f} us, {len(st)} dispatches, gaps {span - tot:.1f} us")
for (n, g), (c, d) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{d:9.1f} us  n={c:4d}  avg={d / c:7.1f}  {g:>18s}  {n}")
