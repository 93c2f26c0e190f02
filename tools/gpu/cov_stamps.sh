#!/bin/bash
# Covariance-stage workgroup stamps of batched launches, both block shapes (tools/cov_stamps.py).
set -uo pipefail
out=${1:-gpurun_out/covst}
mkdir -p "$out"
for big in 0 1; do
  for G in 1 20; do
    DKG_COV_BIG=$big timeout -k 10 120 python3 -u tools/cov_stamps.py $G > "$out/b${big}_g$G.txt" 2>&1 || { tail -5 "$out/b${big}_g$G.txt"; exit 1; }
    grep -v amdgpu.ids "$out/b${big}_g$G.txt"
  done
done
