#!/bin/bash
# Streaming-envelope change check: stress parity + the parity-heavy suites, stress stamps, the stress bench leg.
set -uo pipefail
out=${1:-gpurun_out/stress}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_epigraph.py tests/test_gpu_grad.py \
  -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
timeout -k 10 200 python3 -u tools/kstamps.py stress > "$out/kst_stress.txt" 2>&1 || { tail -5 "$out/kst_stress.txt"; exit 1; }
grep -A7 "^envelope" "$out/kst_stress.txt"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$out/b20.json" 2> "$out/b20.err" || { tail -5 "$out/b20.err"; exit 1; }
python3 tools/bench_summary.py "$out/b20.json"
