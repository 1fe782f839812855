"""Summarise rocprofv3 --pmc counter_collection.csv files: mean counter value per kernel name.
usage: python scripts/pmcsum.py DIR [DIR ...]"""
import csv
import sys
from collections import defaultdict

tot = defaultdict(lambda: defaultdict(list))
for d in sys.argv[1:]:
    with open(f"{d}/run_counter_collection.csv") as f:
        for row in csv.DictReader(f):
            k = row["Kernel_Name"]
            tot[k][row["Counter_Name"]].append((row["Dispatch_Id"], float(row["Counter_Value"])))
for k, cs in tot.items():
    short = k.split("(")[0][-70:]
    print(short)
    for c, vals in sorted(cs.items()):
        per = defaultdict(float)
        for d, v in vals:
            per[d] += v
        mean = sum(per.values()) / len(per)
        print(f"   {c:28s} {mean:16.0f}")
