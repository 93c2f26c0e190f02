#!/bin/bash
# Where the B = 1 value+gradient device chain goes: kernel trace of 200 value_and_grad_host calls, and the
# per-workgroup phase stamps of the gradient kernels at B = 1.
set -uo pipefail
out=${1:-gpurun_out/r06_b1trace}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 tools/b1_kernels.py > "$out/trace.log" 2>&1 || { tail -5 "$out/trace.log"; exit 1; }
f=$(find "$out/trace" -name "*kernel_stats.csv" | head -1)
cp "$f" "$out/kernel_stats.csv"
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:8]:
    print(f'{float(r["AverageNs"])/1e3:9.2f} us avg  {int(r["Calls"]):6d} calls  {r["Name"][:90]}')
PY
timeout -k 10 120 python3 -u tools/kstamps_grad.py headline 1 > "$out/kstamps_b1.txt" 2>&1 || { tail -5 "$out/kstamps_b1.txt"; exit 1; }
grep -v amdgpu.ids "$out/kstamps_b1.txt"
