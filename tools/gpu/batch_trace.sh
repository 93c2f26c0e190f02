#!/bin/bash
# Kernel trace of batched launches (tools/batch_probe.py: 20 steps as G batches per launch, one stream).
set -uo pipefail
out=${1:-gpurun_out/bt}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for G in 20 1; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/g$G" -o run -- \
    python3 tools/batch_probe.py --steps 20 --groups $G --streams 1 --reps 3 --graph 0 > "$out/g$G.log" 2>&1 \
    || { tail -5 "$out/g$G.log"; exit 1; }
done
find "$out" -name "*kernel_stats.csv"
