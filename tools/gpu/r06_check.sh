#!/bin/bash
# The GPU suite, the headline stage times at the driver's launch shape, then the bench line at the driver's shape
# (--steps 20 --warmup 5) and its default.
set -uo pipefail
out=${1:-gpurun_out/r06_check}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
timeout -k 10 180 python3 -u tools/stage_probe.py --workload headline --groups 1 5 > "$out/h_stage.txt" 2>&1 || { tail -5 "$out/h_stage.txt"; exit 1; }
grep '^{' "$out/h_stage.txt"
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > "$out/b20.json" 2> "$out/b20.err" || { tail -20 "$out/b20.err"; exit 1; }
python3 tools/bench_summary.py "$out/b20.json" 2>/dev/null || tail -c 1500 "$out/b20.json"
