#!/bin/bash
# GPU test suite on the box (repo root): every -m gpu test, one process, per-test timeouts.
# usage: bash tools/gpu/tests.sh <out_dir> [pytest args...]
set -uo pipefail
out=${1:-gpurun_out/tests}
shift || true
mkdir -p "$out"
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
  > "$out/gpu_tests.log" 2>&1
rc=$?
tail -15 "$out/gpu_tests.log"
exit $rc
