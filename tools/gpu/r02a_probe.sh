#!/bin/bash
# Round-2 probe: measured f64 MFMA / VALU peaks, forward phase stamps, available PMC counters.
set -euo pipefail
out=gpurun_out/r02a
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 90 tools/ubench/rates > "$out/rates.txt" 2>&1
timeout -k 10 180 python3 tools/kstamps.py headline > "$out/kstamps.txt" 2>&1
timeout -k 10 90 rocprofv3 --list-avail > "$out/avail.txt" 2>&1 || true
grep -i -E "MFMA|VALU|FLOP|F64" "$out/avail.txt" > "$out/avail_mfma.txt" || true
echo done
