#!/bin/bash
# Whole GPU suite, smoke(), the default bench line and one driver-shape run.
set -uo pipefail
out=${1:-gpurun_out/full}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -2 "$out/smoke.log"
timeout -k 10 400 python3 -u bench.py > "$out/bench_default.json" 2> "$out/bench_default.err" || { tail -5 "$out/bench_default.err"; exit 1; }
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$out/bench20.json" 2> "$out/bench20.err" || { tail -5 "$out/bench20.err"; exit 1; }
python3 tools/bench_summary.py "$out"/bench_default.json "$out"/bench20.json
