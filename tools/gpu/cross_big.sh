#!/bin/bash
# Big cross blocks (cross_big_kernel): batched-launch bits and parity suites, then the stage times with and
# without them (DKG_CROSS_BIG), stress (one forward per launch) and headline (10 / 20 batches per launch).
set -uo pipefail
out=${1:-gpurun_out/xb}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batches.py tests/test_gpu_parity.py tests/test_golden.py -m gpu -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -40 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for xb in 1 0; do
  DKG_CROSS_BIG=$xb timeout -k 10 150 python3 -u tools/stage_probe.py --workload stress --groups 1 > "$out/s_x$xb.txt" 2>&1 || { tail -5 "$out/s_x$xb.txt"; exit 1; }
  grep '^{' "$out/s_x$xb.txt"
  DKG_CROSS_BIG=$xb timeout -k 10 150 python3 -u tools/stage_probe.py --workload headline --groups 10 20 > "$out/h_x$xb.txt" 2>&1 || { tail -5 "$out/h_x$xb.txt"; exit 1; }
  grep '^{' "$out/h_x$xb.txt"
done
