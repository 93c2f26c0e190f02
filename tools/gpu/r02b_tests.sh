#!/bin/bash
# GPU tests: the new epigraph suite first, then the whole -m gpu suite.
set -uo pipefail
out=gpurun_out/r02b
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_epigraph.py -x -v --timeout 180 --timeout-method thread -m gpu > "$out/epigraph.log" 2>&1
rc=$?
echo "epigraph rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > "$out/gpu_all.log" 2>&1
rc=$?
echo "all rc=$rc"
exit $rc
