#!/bin/bash
# After a covariance-kernel change: batched bits, forward parity, smoke loop, then stamps and stage times.
set -uo pipefail
out=${1:-gpurun_out/cf}
mkdir -p "$out"
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_batches.py tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_grad.py tests/test_gpu_epigraph.py tests/test_gpu_bo_smoke.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
bash tools/gpu/cov_iter.sh "$out/iter" | grep -v "passed"
