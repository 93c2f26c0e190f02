#!/bin/bash
# rocprofv3 kernel trace + stats of the driver's bench command (the line's roofline durations against the trace's).
# usage: tools/gpu/trace_bench.sh <out> [bench args]
set -uo pipefail
out=${1:-gpurun_out/tb}; shift || true
mkdir -p "$out"
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 bench.py ${*:---steps 20 --warmup 5} > "$out/bench.json" 2> "$out/bench.err" || { tail -5 "$out/bench.err"; exit 1; }
f=$(find "$out/trace" -name "*kernel_stats.csv" | head -1)
cp "$f" "$out/kernel_stats.csv"
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:10]:
    print(f'{float(r["AverageNs"])/1e3:9.2f} us avg  {int(r["Calls"]):6d} calls  {r["Name"][:100]}')
PY
