#!/bin/bash
# Split-envelope probe (tools/split_probe.py), bounded; then the split parity suites and A/B (env_split.sh).
set -uo pipefail
out=${1:-gpurun_out/sp}
mkdir -p "$out"
timeout -k 10 90 python3 -u tools/split_probe.py > "$out/s1.txt" 2>&1 || { cat "$out/s1.txt"; exit 1; }
cat "$out/s1.txt"
