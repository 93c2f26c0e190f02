#!/bin/bash
# rec2 covariance blocks (m = 2): bits, then headline stage times for rec2 (default) / 64 x 32 blocks, G = 5 stamps.
set -uo pipefail
out=${1:-gpurun_out/r06_rec2b}
mkdir -p "$out"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batches.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
probe() {
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 180 python3 -u tools/stage_probe.py "$@" > "$out/$name.txt" 2>&1 || { tail -5 "$out/$name.txt"; exit 1; }
  grep '^{' "$out/$name.txt"
}
probe h_rec2 X=1 -- --workload headline --groups 2 5 10 16 32
probe h_blk DKG_COV_REC2=0 -- --workload headline --groups 2 5 10 16 32
timeout -k 10 120 python3 -u tools/cov_stamps.py 5 > "$out/covst_g5.txt" 2>&1 || { tail -5 "$out/covst_g5.txt"; exit 1; }
grep -v amdgpu.ids "$out/covst_g5.txt"
