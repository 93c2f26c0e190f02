#!/bin/bash
# fp32 block kernels: per-candidate slope errors against fp64 with each block kernel switched off in turn.
set -uo pipefail
out=${1:-gpurun_out/r06_f32dbg}
mkdir -p "$out"
for cfg in "1 1" "0 1" "1 0" "0 0"; do
  set -- $cfg
  DKG_COV_BIG32=$1 DKG_CROSS_BIG=$2 timeout -k 10 150 python3 -u tools/f32_debug.py stress32 > "$out/dbg_c$1_x$2.txt" 2>&1 || { tail -5 "$out/dbg_c$1_x$2.txt"; exit 1; }
  grep -v amdgpu.ids "$out/dbg_c$1_x$2.txt"
done
