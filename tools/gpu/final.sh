#!/bin/bash
# The round-end driver's sequence on the final tree: every -m gpu test, smoke(), the driver-shaped bench, the default bench.
set -uo pipefail
out=${1:-gpurun_out/final}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || { tail -5 "$out/smoke.txt"; exit 1; }
tail -2 "$out/smoke.txt"
timeout -k 10 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$out/b20.json" 2> "$out/b20.err" || { tail -5 "$out/b20.err"; exit 1; }
timeout -k 10 500 python3 -u bench.py > "$out/b1024.json" 2> "$out/b1024.err" || { tail -5 "$out/b1024.err"; exit 1; }
python3 tools/bench_summary.py "$out"/b*.json
