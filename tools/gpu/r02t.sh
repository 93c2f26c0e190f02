#!/bin/bash
set -uo pipefail
out=gpurun_out/r02t
mkdir -p "$out"
PROBE_STREAMS=1,4,8 timeout -k 10 200 python3 -u tools/launch_probe.py > "$out/probe2.txt" 2>&1; rc=$?
cat "$out/probe2.txt"; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=8 PROBE_MODES=2 PROBE_STREAMS=4,8 timeout -k 10 200 python3 -u tools/launch_probe.py > "$out/probe2_q8.txt" 2>&1; rc=$?
echo "--- 8 queues"; cat "$out/probe2_q8.txt"; [ $rc -eq 0 ] || exit $rc
DKG_DEBUG_COV_FLAGS=3 DKG_DEBUG_ENV_FLAGS=2 PROBE_MODES=2 PROBE_STREAMS=1,4 timeout -k 10 200 python3 -u tools/launch_probe.py > "$out/probe2_empty.txt" 2>&1; rc=$?
echo "--- empty kernels"; cat "$out/probe2_empty.txt"
