#!/bin/bash
# B = 1 host entry: hipStreamSynchronize against polling the stream (DKG_HOSTX_SPIN=1): b1_probe and the bench's
# latency_b1 leg (interleaved calls), two runs each.
set -uo pipefail
out=${1:-gpurun_out/r06_spin}
mkdir -p "$out"
Q="--cpu-seconds 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --grad-steps 0 --prep-reps 0 --profile-reps 2 --single-rank-pg 0 --b1-calls 400"
for rep in 1 2; do
  for sp in 0 1; do
    DKG_HOSTX_SPIN=$sp timeout -k 10 120 python3 -u tools/b1_probe.py headline 400 > "$out/probe_${sp}_$rep.txt" 2>&1 || { tail -5 "$out/probe_${sp}_$rep.txt"; exit 1; }
    echo "spin=$sp probe: $(tail -n1 $out/probe_${sp}_$rep.txt | cut -c1-400)"
    DKG_HOSTX_SPIN=$sp timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $Q > "$out/b_${sp}_$rep.json" 2> "$out/b_${sp}_$rep.err" || { tail -20 "$out/b_${sp}_$rep.err"; exit 1; }
    python3 -c "
import json; d=json.loads([l for l in open('$out/b_${sp}_$rep.json') if l.startswith('{')][-1]); b=d['latency_b1']
print('spin=$sp bench: vgh', round(b['median_us'],1), 'autograd', round(b['autograd_route']['median_us'],1), 'eager', round(b['eager_two_copies_median_us'],1))"
  done
done
