#!/bin/bash
# Batched launches: bit tests, driver-shape bench A/B (streams x batches per launch), default bench, kernel trace.
set -uo pipefail
out=${1:-gpurun_out/bb}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_batches.py -m gpu -x -q --timeout 300 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
lite="--cpu-seconds 0 --nd-steps 0 --stress-steps 0 --b1-calls 0 --grad-steps 0 --prep-reps 0 --profile-reps 20"
for cfg in "--streams 2" "--streams 1 --batches-per-launch 20" "--streams 4 --batches-per-launch 1" "--streams 2" \
           "--streams 4 --batches-per-launch 5" "--streams 2 --batches-per-launch 5"; do
  tag=$(echo "$cfg" | tr -d ' -')
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 $lite $cfg > "$out/b20_$tag.json" 2> "$out/b20_$tag.err" \
    || { tail -5 "$out/b20_$tag.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['value']/1e6,3), d['config']['batches_per_launch'], d['region_breakdown'] and d['region_breakdown']['last_stream_done_us'])" "$out/b20_$tag.json" "$cfg"
done
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 > "$out/b1024.json" 2> "$out/b1024.err" || { tail -5 "$out/b1024.err"; exit 1; }
python3 tools/bench_summary.py "$out/b1024.json"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run -- python3 tools/batch_probe.py --steps 20 --groups 20 --streams 1 --reps 3 > "$out/prof.log" 2>&1 || { tail -5 "$out/prof.log"; exit 1; }
find "$out/prof" -name "*kernel_stats.csv" | head -3
