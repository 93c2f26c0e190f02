#!/bin/bash
# Round 6: the whole GPU suite, then the fp32 plan's big blocks (posterior_cov_big32 / cross_big32) against the
# narrow fp32 kernels (DKG_COV_BIG32=0, DKG_CROSS_BIG=0) and the fp64 plan at BASELINE configs[4]'s shape, and
# the headline stage times at 1 and 5 batches per launch.
# usage: bash tools/gpu/r06_f32.sh <out_dir> [skip_tests]
set -uo pipefail
out=${1:-gpurun_out/r06_f32}
mkdir -p "$out"
if [ "${2:-}" != "skip_tests" ]; then
  bash tools/gpu/tests.sh "$out" || exit 1
fi
run() {  # name, env..., then the probe's arguments after --
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 180 python3 -u tools/stage_probe.py "$@" > "$out/$name.txt" 2>&1 || { tail -5 "$out/$name.txt"; exit 1; }
  grep '^{' "$out/$name.txt"
}
run s32_big DKG_COV_BIG32=1 -- --workload stress32 --precision fp32 --groups 1
run s32_narrow DKG_COV_BIG32=0 DKG_CROSS_BIG=0 -- --workload stress32 --precision fp32 --groups 1
run s32_f64 DKG_COV_BIG32=1 -- --workload stress32 --precision fp64 --groups 1
run h_f64 DKG_COV_BIG32=1 -- --workload headline --precision fp64 --groups 1 5 10
for big in 1 0; do
  DKG_COV_BIG=$big timeout -k 10 120 python3 -u tools/cov_stamps.py 5 > "$out/covst_b${big}_g5.txt" 2>&1 || { tail -5 "$out/covst_b${big}_g5.txt"; exit 1; }
  grep -v amdgpu.ids "$out/covst_b${big}_g5.txt"
done
