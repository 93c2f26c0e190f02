#!/bin/bash
# fp32 block kernels: slope errors against fp64 (default kernels and the narrow ones), the fp32 / batch tests,
# then stage times of the fp32 and fp64 plans at BASELINE configs[4]'s shape.
set -uo pipefail
out=${1:-gpurun_out/r06_f32b}
mkdir -p "$out"
for cfg in "1 1" "0 0"; do
  set -- $cfg
  DKG_COV_BIG32=$1 DKG_CROSS_BIG=$2 timeout -k 10 150 python3 -u tools/f32_debug.py stress32 > "$out/dbg_c$1_x$2.txt" 2>&1 || { tail -5 "$out/dbg_c$1_x$2.txt"; exit 1; }
  grep -v amdgpu.ids "$out/dbg_c$1_x$2.txt"
done
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_batches.py tests/test_gpu_parity.py -m gpu -x -q -k "f32 or fp32 or batched" --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -3 "$out/tests.log"
for prec in fp32 fp64; do
  timeout -k 10 150 python3 -u tools/stage_probe.py --workload stress32 --precision $prec --groups 1 > "$out/s32_$prec.txt" 2>&1 || { tail -5 "$out/s32_$prec.txt"; exit 1; }
  grep '^{' "$out/s32_$prec.txt"
done
DKG_COV_BIG32=0 DKG_CROSS_BIG=0 timeout -k 10 150 python3 -u tools/stage_probe.py --workload stress32 --precision fp32 --groups 1 > "$out/s32_fp32_narrow.txt" 2>&1 || { tail -5 "$out/s32_fp32_narrow.txt"; exit 1; }
grep '^{' "$out/s32_fp32_narrow.txt"
