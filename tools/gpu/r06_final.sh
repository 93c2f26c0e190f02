#!/bin/bash
# Round-6 final tree: the GPU suite, smoke, the bench line at the driver's shape and its default, and the
# rocprofv3 kernel statistics of the driver-shaped command.
set -uo pipefail
out=${1:-gpurun_out/r06_final}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 || { tail -5 "$out/smoke.txt"; exit 1; }
tail -n1 "$out/smoke.txt"
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > "$out/b20.json" 2> "$out/b20.err" || { tail -20 "$out/b20.err"; exit 1; }
python3 tools/bench_summary.py "$out/b20.json" 2>/dev/null | cut -c1-400
timeout -k 10 500 python3 -u bench.py > "$out/bdef.json" 2> "$out/bdef.err" || { tail -20 "$out/bdef.err"; exit 1; }
python3 tools/bench_summary.py "$out/bdef.json" 2>/dev/null | cut -c1-400
bash tools/gpu/trace_bench.sh "$out/tb" > "$out/tb.txt" 2>&1 || { tail -5 "$out/tb.txt"; exit 1; }
cat "$out/tb.txt"
