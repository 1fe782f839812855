#!/bin/bash
# kernel trace of the metric bench (per-dispatch timeline) + the config-2 / config-4 shapes
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/s5tr -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/s5tr.log 2>&1 || exit 1
python3 scripts/steptrace.py gpurun_out/s5tr/run_kernel_trace.csv -1 > gpurun_out/s5tr_step.txt
python3 - <<'PY' > gpurun_out/s5tr_copies.txt
import csv
rows = sorted(csv.DictReader(open("gpurun_out/s5tr/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
for i, r in enumerate(rows):
    if "copyBuffer" in r["Kernel_Name"] or "FillFunctor" in r["Kernel_Name"]:
        prev = rows[i-1]["Kernel_Name"][:70] if i else ""
        nxt = rows[i+1]["Kernel_Name"][:70] if i + 1 < len(rows) else ""
        print(i, r["Kernel_Name"][:40], r.get("Grid_Size", ""), "| prev:", prev, "| next:", nxt)
PY
rm -rf gpurun_out/s5tr
timeout -k 10 300 python3 -u bench.py --seq-len 4096 --batch 1 --no-cpu-baseline > gpurun_out/s5_cfg4.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --seq-len 1024 --batch 8 --no-cpu-baseline > gpurun_out/s5_cfg2.log 2>&1 || exit 1
grep '"metric"' gpurun_out/s5_cfg4.log gpurun_out/s5_cfg2.log
