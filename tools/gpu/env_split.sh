#!/bin/bash
# Split envelope: forward parity suites, batched bits, stage times with and without the split.
set -uo pipefail
out=${1:-gpurun_out/es}
mkdir -p "$out"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batches.py tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_api.py tests/test_gpu_epigraph.py tests/test_gpu_fused.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -40 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for sp in 0 1; do
  DKG_ENV_SPLIT=$sp timeout -k 10 200 python3 -u tools/stage_probe.py --groups 1 10 20 > "$out/h_s$sp.txt" 2>&1 || { tail -5 "$out/h_s$sp.txt"; exit 1; }
  grep '^{' "$out/h_s$sp.txt"
  DKG_ENV_SPLIT=$sp timeout -k 10 200 python3 -u tools/stage_probe.py --workload headline_nd --groups 1 20 > "$out/nd_s$sp.txt" 2>&1 || { tail -5 "$out/nd_s$sp.txt"; exit 1; }
  grep '^{' "$out/nd_s$sp.txt"
done
