#!/bin/bash
# Covariance-kernel iteration: bit tests of batched launches, then stamps and stage times at G = 1 / 20.
set -uo pipefail
out=${1:-gpurun_out/ci}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batches.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for G in 1 20; do
  DKG_COV_BIG=1 timeout -k 10 120 python3 -u tools/cov_stamps.py $G > "$out/st_g$G.txt" 2>&1 || { tail -5 "$out/st_g$G.txt"; exit 1; }
  grep -v amdgpu.ids "$out/st_g$G.txt"
done
timeout -k 10 200 python3 -u tools/stage_probe.py --groups 10 20 > "$out/headline.txt" 2>&1 || { tail -5 "$out/headline.txt"; exit 1; }
grep '^{' "$out/headline.txt"
timeout -k 10 200 python3 -u tools/stage_probe.py --workload headline_nd --groups 20 > "$out/nd.txt" 2>&1 || { tail -5 "$out/nd.txt"; exit 1; }
grep '^{' "$out/nd.txt"
timeout -k 10 200 python3 -u tools/stage_probe.py --workload stress --groups 1 --reps 5 > "$out/stress.txt" 2>&1 || { tail -5 "$out/stress.txt"; exit 1; }
grep '^{' "$out/stress.txt"
