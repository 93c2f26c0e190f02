#!/bin/bash
# Launch-mode A/B at the driver's shape and the 1024-step line: --graph 2 (per-stream graphs) vs --graph 3
# (one native call enqueues the period's forwards round-robin over the streams), interleaved; optional
# extra bench arguments per mode after "--".
set -uo pipefail
out=${1:-gpurun_out/modes}
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -k "forward_many or concurrent" -q --timeout 120 \
  --timeout-method thread > "$out/tests.log" 2>&1 || { tail -20 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
opts="--cpu-seconds 0 --grad-steps 0 --b1-calls 0 --nd-steps 0 --stress-steps 0 --prep-reps 0"
for rep in 1 2 3; do
  for g in 2 3; do
    timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --graph $g $opts > "$out/b20_g${g}_$rep.json" 2> "$out/b20_g${g}_$rep.err" || { tail -5 "$out/b20_g${g}_$rep.err"; exit 1; }
    [ $rep -le 2 ] && { timeout -k 10 200 python3 -u bench.py --steps 1024 --warmup 50 --graph $g $opts > "$out/b1k_g${g}_$rep.json" 2> "$out/b1k_g${g}_$rep.err" || { tail -5 "$out/b1k_g${g}_$rep.err"; exit 1; }; }
  done
done
for f in "$out"/*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), round(d['ms_per_step']*1e3,2), 'host/step', round(d['host_launch_us_per_step'],2), 'compute', d['per_rank']['compute_ms'])" "$f"; done
