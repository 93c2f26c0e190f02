#!/bin/bash
# Batched-launch bit tests + parity + per-stage times (headline, headline_nd, stress).
set -uo pipefail
out=${1:-gpurun_out/qs}
mkdir -p "$out"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batches.py tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_api.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for big in 0 1; do
  DKG_COV_BIG=$big timeout -k 10 200 python3 -u tools/stage_probe.py --groups 1 10 20 > "$out/headline_b$big.txt" 2>&1 || { tail -5 "$out/headline_b$big.txt"; exit 1; }
  grep '^{' "$out/headline_b$big.txt"
done
timeout -k 10 200 python3 -u tools/stage_probe.py --workload headline_nd --groups 1 20 > "$out/nd.txt" 2>&1 || { tail -5 "$out/nd.txt"; exit 1; }
grep '^{' "$out/nd.txt"
timeout -k 10 200 python3 -u tools/stage_probe.py --workload stress --groups 1 --reps 5 > "$out/stress.txt" 2>&1 || { tail -5 "$out/stress.txt"; exit 1; }
grep '^{' "$out/stress.txt"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_bo_smoke.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/tests_smoke.log" 2>&1 || { tail -30 "$out/tests_smoke.log"; exit 1; }
tail -1 "$out/tests_smoke.log"
