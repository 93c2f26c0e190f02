#!/bin/bash
# 64 x 32 covariance blocks (posterior_cov_blk_kernel): the GPU suite, then headline stage times at 1/5/10/32
# batches per launch with them (default), with the 64 x 64 blocks (DKG_COV_BLK=0) and, for one forward, the
# narrow kernel unconstrained (the pcw2 build: waves_per_eu 2, 130 VGPRs); stress stage times; G = 5 stamps.
set -uo pipefail
out=${1:-gpurun_out/r06_blk}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
probe() {  # name, then env assignments, then -- and the probe's arguments
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 180 python3 -u tools/stage_probe.py "$@" > "$out/$name.txt" 2>&1 || { tail -5 "$out/$name.txt"; exit 1; }
  grep '^{' "$out/$name.txt"
}
probe h_blk X=1 -- --workload headline --groups 1 5 10 32
probe h_big64 DKG_COV_BLK=0 -- --workload headline --groups 5 10 32
probe h_pcw2 DKG_LIB=decoupled-kg_amd/dkg_amd/_native/ab/libdkg_pcw2.so -- --workload headline --groups 1
probe h_nd X=1 -- --workload headline_nd --groups 1 5
probe s_blk X=1 -- --workload stress --groups 1
probe s_big64 DKG_COV_BLK=0 -- --workload stress --groups 1
timeout -k 10 120 python3 -u tools/cov_stamps.py 5 > "$out/covst_blk_g5.txt" 2>&1 || { tail -5 "$out/covst_blk_g5.txt"; exit 1; }
grep -v amdgpu.ids "$out/covst_blk_g5.txt"
