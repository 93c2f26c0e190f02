#!/bin/bash
set -uo pipefail
out=gpurun_out/r02zd
mkdir -p "$out"
PROBE_MODES=1,2 PROBE_STREAMS=2,3,4,6,8 timeout -k 10 300 python3 -u tools/launch_probe.py > "$out/probe.txt" 2>&1; rc=$?
cat "$out/probe.txt"; [ $rc -eq 0 ] || exit $rc
GPU_MAX_HW_QUEUES=8 PROBE_MODES=1,2 PROBE_STREAMS=6,8 timeout -k 10 300 python3 -u tools/launch_probe.py > "$out/probe_q8.txt" 2>&1; rc=$?
echo "--- 8 queues"; cat "$out/probe_q8.txt"
