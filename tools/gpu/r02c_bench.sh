#!/bin/bash
# Bench on the current tree + rocprofv3 kernel stats of a short bench run.
set -uo pipefail
out=gpurun_out/r02c
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
cat "$out/bench.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 bench.py --steps 512 --cpu-seconds 0 --grad-steps 0 > "$out/prof.log" 2>&1
rc=$?; echo "prof rc=$rc"
exit $rc
