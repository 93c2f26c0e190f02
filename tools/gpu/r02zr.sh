#!/bin/bash
# gradient cross stage on a side stream (independent of the forward cross stage): grad/api/optim/bo tests, B=1 probe
set -uo pipefail
out=gpurun_out/r02zr
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_grad.py tests/test_gpu_api.py tests/test_gpu_optim.py tests/test_gpu_bo_smoke.py tests/test_gpu_dist.py -x -v --timeout 200 --timeout-method thread -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$out/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/b1_probe.py headline 300 > "$out/b1_probe.txt" 2>&1
rc=$?; echo "probe rc=$rc"; cat "$out/b1_probe.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 -u tools/bench_optimize.py --cpu-seconds 0 > "$out/bench_optimize.json" 2>&1
rc=$?; echo "opt rc=$rc"; tail -1 "$out/bench_optimize.json"
