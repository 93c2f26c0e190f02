#!/bin/bash
# Round-6 main check: the GPU suite, smoke, headline stage times, the bench line at the driver's shape and its
# default, and the B = 1 breakdown.
set -uo pipefail
out=${1:-gpurun_out/r06_main}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
timeout -k 10 120 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$out/smoke.txt" 2>&1 || { tail -5 "$out/smoke.txt"; exit 1; }
timeout -k 10 180 python3 -u tools/stage_probe.py --workload headline --groups 1 5 > "$out/h_stage.txt" 2>&1 || { tail -5 "$out/h_stage.txt"; exit 1; }
grep '^{' "$out/h_stage.txt"
timeout -k 10 120 python3 -u tools/b1_probe.py headline 400 > "$out/b1_probe.txt" 2>&1 || { tail -5 "$out/b1_probe.txt"; exit 1; }
cat "$out/b1_probe.txt"
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > "$out/b20.json" 2> "$out/b20.err" || { tail -20 "$out/b20.err"; exit 1; }
python3 tools/bench_summary.py "$out/b20.json" 2>/dev/null || tail -c 1500 "$out/b20.json"
timeout -k 10 500 python3 -u bench.py > "$out/bdef.json" 2> "$out/bdef.err" || { tail -20 "$out/bdef.err"; exit 1; }
python3 tools/bench_summary.py "$out/bdef.json" 2>/dev/null || tail -c 1500 "$out/bdef.json"
