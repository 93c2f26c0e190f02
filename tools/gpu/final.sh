#!/bin/bash
# Final check of the tree: every GPU test, smoke(), the default bench line, and the B = 1 probe.
set -uo pipefail
out=${1:-gpurun_out/final}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -2 "$out/smoke.log"
timeout -k 10 400 python3 -u bench.py > "$out/bench_default.json" 2> "$out/bench_default.err" || { tail -5 "$out/bench_default.err"; exit 1; }
python3 tools/bench_summary.py "$out"/bench_default.json
timeout -k 10 200 python3 -u tools/b1_probe.py > "$out/b1_probe.txt" 2>&1 || { tail -5 "$out/b1_probe.txt"; exit 1; }
grep -v amdgpu.ids "$out/b1_probe.txt" | cut -c1-400
