#!/bin/bash
# Forward-kernel change check: parity suites, stamps (headline), bench at the driver shape.
set -uo pipefail
out=${1:-gpurun_out/qb}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fused.py tests/test_gpu_grad.py \
  -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
timeout -k 10 200 python3 -u tools/kstamps.py headline > "$out/kst.txt" 2>&1 || { tail -5 "$out/kst.txt"; exit 1; }
cat "$out/kst.txt"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$out/b20.json" 2> "$out/b20.err" || { tail -5 "$out/b20.err"; exit 1; }
python3 tools/bench_summary.py "$out/b20.json"
