#!/bin/bash
# Driver-shape bench over more stream counts (light legs), two passes.
set -uo pipefail
out=${1:-gpurun_out/b20cfg2}
mkdir -p "$out"
lite="--cpu-seconds 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --b1-calls 0 --grad-steps 0 --prep-reps 0 --profile-reps 5"
for rep in 1 2; do
for cfg in "--streams 4" "--streams 5" "--streams 4 --batches-per-launch 2" "--streams 8 --batches-per-launch 2" "--streams 4 --graph-head 1"; do
  tag=$(echo "$cfg" | tr -d ' -')_$rep
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 $lite $cfg > "$out/b20_$tag.json" 2> "$out/b20_$tag.err" \
    || { tail -5 "$out/b20_$tag.err"; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], round(d['value']/1e6,3), d['config']['batches_per_launch'], d['ms_per_step'])" "$out/b20_$tag.json" "$cfg"
done
done
