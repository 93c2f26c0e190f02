#!/bin/bash
# Per-stage launch times of batched launches (tools/stage_probe.py), both covariance block shapes.
set -uo pipefail
out=${1:-gpurun_out/sp}
mkdir -p "$out"
for wide in 0 1; do
  DKG_COV_WIDE=$wide timeout -k 10 200 python3 -u tools/stage_probe.py --groups 1 10 20 40 > "$out/headline_w$wide.txt" 2>&1 || { tail -5 "$out/headline_w$wide.txt"; exit 1; }
  cat "$out/headline_w$wide.txt" | grep '^{'
done
timeout -k 10 200 python3 -u tools/stage_probe.py --workload headline_nd --groups 1 20 > "$out/nd.txt" 2>&1 || { tail -5 "$out/nd.txt"; exit 1; }
grep '^{' "$out/nd.txt"
