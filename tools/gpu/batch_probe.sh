#!/bin/bash
# Forward batches per launch: bit check + rates (tools/batch_probe.py), then the forward parity suites.
set -uo pipefail
out=${1:-gpurun_out/batch}
mkdir -p "$out"
timeout -k 10 300 python3 -u tools/batch_probe.py > "$out/probe.txt" 2>&1 || { tail -20 "$out/probe.txt"; exit 1; }
tail -3 "$out/probe.txt"
DKG_COV_WIDE=1 timeout -k 10 300 python3 -u tools/batch_probe.py --groups 10 20 32 64 > "$out/probe_wide.txt" 2>&1 || { tail -20 "$out/probe_wide.txt"; exit 1; }
tail -2 "$out/probe_wide.txt"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_grad.py tests/test_gpu_api.py \
  -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
