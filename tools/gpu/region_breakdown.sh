#!/bin/bash
# The driver-shaped region (--steps 20 --warmup 5): its breakdown (bench.py region_breakdown) under the launch
# variants (graph head 0/1/2, 3 or 4 streams), two runs each, interleaved.
set -uo pipefail
out=${1:-gpurun_out/region}
mkdir -p "$out"
opts="--steps 20 --warmup 5 --cpu-seconds 0 --grad-steps 0 --b1-calls 0 --nd-steps 0 --stress-steps 0 --prep-reps 0"
for rep in 1 2; do
  for v in "h1:--graph-head 1" "h0:--graph-head 0" "h2:--graph-head 2" "s3:--streams 3" "s2:--streams 2"; do
    name=${v%%:*}; extra=${v#*:}
    timeout -k 10 200 python3 -u bench.py $opts $extra > "$out/b20_${name}_$rep.json" 2> "$out/b20_${name}_$rep.err" || { tail -5 "$out/b20_${name}_$rep.err"; exit 1; }
  done
done
for f in "$out"/b20_*.json; do python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); b=d.get('region_breakdown') or {}
print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), round(d['ms_per_step']*1e3,1), 'host', b.get('host_launch_done_us'), 'done', b.get('stream_piece_done_us'), 'wall', b.get('wall_us'))" "$f"; done
