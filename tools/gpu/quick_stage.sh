#!/bin/bash
# Batched-launch bit tests + per-stage times (headline, headline_nd).
set -uo pipefail
out=${1:-gpurun_out/qs}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batches.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
timeout -k 10 200 python3 -u tools/stage_probe.py --groups 1 10 20 > "$out/headline.txt" 2>&1 || { tail -5 "$out/headline.txt"; exit 1; }
grep '^{' "$out/headline.txt"
timeout -k 10 200 python3 -u tools/stage_probe.py --workload headline_nd --groups 1 20 > "$out/nd.txt" 2>&1 || { tail -5 "$out/nd.txt"; exit 1; }
grep '^{' "$out/nd.txt"
