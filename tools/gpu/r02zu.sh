#!/bin/bash
# timeline of the driver's short run (--steps 20 --warmup 5): kernel trace of the timed region
set -uo pipefail
out=gpurun_out/r02zu
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$out/t20" -o run -- python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --profile-reps 2 > "$out/t20.json" 2> "$out/t20.err"
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find "$out/t20" -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 45 20
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$out/t1k" -o run -- python3 bench.py --steps 1024 --warmup 50 --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --profile-reps 2 > "$out/t1k.json" 2> "$out/t1k.err"
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find "$out/t1k" -name "*kernel_trace.csv" | head -1)
python3 tools/trace_window.py "$f" 562 1024
