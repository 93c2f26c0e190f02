#!/bin/bash
# The host B = 1 paths: API tests, b1_probe.
set -uo pipefail
out=${1:-gpurun_out/r06_b1}
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_api.py tests/test_gpu_grad.py -x -q --timeout 120 --timeout-method thread > "$out/api.log" 2>&1 || { tail -30 "$out/api.log"; exit 1; }
tail -n1 "$out/api.log"
timeout -k 10 120 python3 -u tools/b1_probe.py headline 400 > "$out/b1_probe.txt" 2>&1 || { tail -5 "$out/b1_probe.txt"; exit 1; }
tail -n1 "$out/b1_probe.txt"
timeout -k 10 400 python3 -u tools/parity_report.py "$out/r06_parity.json" > "$out/parity.log" 2>&1 || { tail -5 "$out/parity.log"; exit 1; }
tail -n1 "$out/parity.log"
