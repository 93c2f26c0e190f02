#!/bin/bash
# Forward batches in flight: streams x hardware queues at the driver shape (20 steps) and at 1024 steps.
set -uo pipefail
out=${1:-gpurun_out/streams}
mkdir -p "$out"
run() {  # name queues streams steps
  GPU_MAX_HW_QUEUES=$2 timeout -k 10 200 python3 -u bench.py --steps $4 --warmup 5 --streams $3 --cpu-seconds 0 --b1-calls 0 \
    --grad-steps 0 --nd-steps 0 --stress-steps 0 --prep-reps 0 > "$out/$1.json" 2> "$out/$1.err" || { tail -5 "$out/$1.err"; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step')" "$out/$1.json" "$1"
}
for i in 1 2; do
  run q4s4_20_$i 4 4 20 || exit 1
  run q8s8_20_$i 8 8 20 || exit 1
  run q8s6_20_$i 8 6 20 || exit 1
  run q4s8_20_$i 4 8 20 || exit 1
done
run q4s4_1024 4 4 1024 || exit 1
run q8s8_1024 8 8 1024 || exit 1
run q8s6_1024 8 6 1024 || exit 1
