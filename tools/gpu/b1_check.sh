#!/bin/bash
# B = 1 route check: API tests (host route bit-identity), the B = 1 probe, grad-kernel stamps at B = 1,
# then the bench at the driver's shape and at the default.
set -uo pipefail
out=${1:-gpurun_out/b1}
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_api.py -x -q --timeout 120 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
timeout -k 10 120 python3 -u tools/b1_probe.py headline 300 > "$out/b1_probe.txt" 2>&1 || { tail -5 "$out/b1_probe.txt"; exit 1; }
tail -1 "$out/b1_probe.txt"
timeout -k 10 120 python3 -u tools/kstamps_grad.py headline 1 > "$out/kst_grad_b1.txt" 2>&1 || { tail -5 "$out/kst_grad_b1.txt"; exit 1; }
cat "$out/kst_grad_b1.txt"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 > "$out/b20.json" 2> "$out/b20.err" || { tail -5 "$out/b20.err"; exit 1; }
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 > "$out/b1024.json" 2> "$out/b1024.err" || { tail -5 "$out/b1024.err"; exit 1; }
python3 tools/bench_summary.py "$out/b20.json" "$out/b1024.json"
