#!/bin/bash
# Headline covariance stage at 1 / 5 / 10 batches per launch, big (64 x 64) vs narrow (32 x 32) blocks, and the
# workgroup stamps of both at 5 batches.
set -uo pipefail
out=${1:-gpurun_out/r06_cov}
mkdir -p "$out"
for big in 1 0; do
  DKG_COV_BIG=$big timeout -k 10 150 python3 -u tools/stage_probe.py --workload headline --groups 1 5 10 > "$out/h_big$big.txt" 2>&1 || { tail -5 "$out/h_big$big.txt"; exit 1; }
  grep '^{' "$out/h_big$big.txt"
done
for big in 1 0; do
  DKG_COV_BIG=$big timeout -k 10 120 python3 -u tools/cov_stamps.py 5 > "$out/covst_b${big}_g5.txt" 2>&1 || { tail -5 "$out/covst_b${big}_g5.txt"; exit 1; }
  grep -v amdgpu.ids "$out/covst_b${big}_g5.txt"
done
