#!/bin/bash
# B = 1 value+gradient: per-kernel durations (kernel trace of the probe)
set -uo pipefail
out=gpurun_out/r02zq
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o b1 -- python3 tools/b1_probe.py headline 300 > "$out/prof.log" 2>&1
rc=$?; echo "prof rc=$rc"; tail -2 "$out/prof.log"
f=$(find "$out/prof" -name "*kernel_stats.csv" | head -1); cat "$f"
