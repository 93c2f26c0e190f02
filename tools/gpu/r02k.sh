#!/bin/bash
# parity report, fp32 accuracy survey, non-degenerate pair stamps
set -uo pipefail
out=gpurun_out/r02k
mkdir -p "$out"
timeout -k 10 300 python3 -u tools/parity_report.py $out/r02_parity.json > "$out/parity.log" 2>&1
rc=$?; echo "parity rc=$rc"; tail -2 "$out/parity.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/f32_check.py > "$out/f32.log" 2>&1
rc=$?; echo "f32 rc=$rc"; cat "$out/f32.log" | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/pair_stamps.py headline_nd > "$out/pairs_nd.txt" 2>&1 || exit $?
cat $out/pairs_nd.txt
