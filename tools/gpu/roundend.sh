#!/bin/bash
# Round-end evidence on one box: the GPU suite, smoke(), the default bench line (CPU baseline included),
# three runs at the driver's shape, and the rocprofv3 kernel statistics of a driver-shape run.
set -uo pipefail
out=${1:-gpurun_out/end}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1 || { tail -20 "$out/smoke.log"; exit 1; }
tail -2 "$out/smoke.log"
timeout -k 10 400 python3 -u bench.py > "$out/bench_default.json" 2> "$out/bench_default.err" || { tail -5 "$out/bench_default.err"; exit 1; }
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$out/bench20_$i.json" 2> "$out/bench20_$i.err" || { tail -5 "$out/bench20_$i.err"; exit 1; }
done
python3 tools/bench_summary.py "$out"/bench_default.json "$out"/bench20_*.json
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/rocprof" -o run -- \
  python3 bench.py --steps 20 --warmup 5 --cpu-seconds 0 --b1-calls 20 --grad-steps 5 --nd-steps 20 --stress-steps 4 \
  > "$out/rocprof_bench.json" 2> "$out/rocprof_bench.err" || { tail -5 "$out/rocprof_bench.err"; exit 1; }
ls "$out/rocprof"
