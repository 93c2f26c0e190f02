#!/bin/bash
set -uo pipefail
out=gpurun_out/r02t
mkdir -p "$out"
timeout -k 10 200 python3 -u tools/launch_probe.py > "$out/probe.txt" 2>&1; rc=$?
cat "$out/probe.txt"; [ $rc -eq 0 ] || exit $rc
DKG_DEBUG_COV_FLAGS=3 DKG_DEBUG_ENV_FLAGS=2 timeout -k 10 200 python3 -u tools/launch_probe.py > "$out/probe_empty.txt" 2>&1; rc=$?
echo "--- empty kernels"; cat "$out/probe_empty.txt"
