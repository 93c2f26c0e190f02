#!/bin/bash
set -uo pipefail
out=${1:-gpurun_out/envst}
mkdir -p "$out"
for G in 1 4; do
  timeout -k 10 120 python3 -u tools/cov_stamps.py $G headline --env > "$out/env_g$G.txt" 2>&1 || { tail -5 "$out/env_g$G.txt"; exit 1; }
  grep -v amdgpu.ids "$out/env_g$G.txt"
done
