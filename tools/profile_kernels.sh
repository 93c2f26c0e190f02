#!/bin/bash
# Kernel-trace profile of the headline bench (run on the GPU box from the repo root).
# usage: tools/profile_kernels.sh <tag> [extra bench args]
set -euo pipefail
tag=${1:-r01}; shift || true
out=gpurun_out/prof_${tag}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
  python3 bench.py --steps 200 --warmup 20 --cpu-seconds 0 --profile-reps 20 "$@" > "$out/bench.json" 2> "$out/bench.err"
find "$out" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats.csv" \;
cat "$out/kernel_stats.csv"
