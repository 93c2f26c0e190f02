#!/bin/bash
# Round-4: coincident-candidate tests first, then the GPU suite, then the measurement pass (r04b's).
set -uo pipefail
out=${1:-gpurun_out/r04d}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_grad.py tests/test_gpu_bo_smoke.py -m gpu -v -k "discretisation_points or oracle_run" \
  --timeout 300 --timeout-method thread > "$out/focus.log" 2>&1
rc=$?; tail -30 "$out/focus.log"; [ $rc -ne 0 ] && exit $rc
bash tools/gpu/r04b.sh "$out"
