#!/bin/bash
# rocprofv3 kernel statistics of tools/stage_probe.py (every kernel of the three stages, launched alone).
# usage: tools/gpu/trace_stage.sh <out> <workload> <groups...>
set -uo pipefail
out=${1:-gpurun_out/ts}; wl=${2:-stress}; shift 2 || true
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$wl" -o run -- python3 tools/stage_probe.py --workload "$wl" --groups ${*:-1} --reps 20 > "$out/$wl.log" 2>&1 || { tail -5 "$out/$wl.log"; exit 1; }
f=$(find "$out/$wl" -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f'{float(r["AverageNs"])/1e3:9.2f} us avg  {int(r["Calls"]):6d} calls  {r["Name"][:110]}')
PY
