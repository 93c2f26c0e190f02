#!/bin/bash
# Driver-shaped region under stream skews (--stream-skew 0/1/2, graph head 1; skew 2 with head 0), three runs each.
set -uo pipefail
out=${1:-gpurun_out/skew}
mkdir -p "$out"
opts="--steps 20 --warmup 5 --cpu-seconds 0 --grad-steps 0 --b1-calls 0 --nd-steps 0 --stress-steps 0 --prep-reps 0"
for rep in 1 2 3; do
  for v in "k0:--stream-skew 0" "k1:--stream-skew 1" "k2:--stream-skew 2" "k2h0:--stream-skew 2 --graph-head 0" "k3:--stream-skew 3"; do
    name=${v%%:*}; extra=${v#*:}
    timeout -k 10 200 python3 -u bench.py $opts $extra > "$out/b20_${name}_$rep.json" 2> "$out/b20_${name}_$rep.err" || { tail -5 "$out/b20_${name}_$rep.err"; exit 1; }
  done
done
for f in "$out"/b20_*.json; do python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); b=d.get('region_breakdown') or {}
print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), b.get('forwards_per_stream'), 'host', b.get('host_launch_done_us'), 'done', b.get('stream_piece_done_us'), 'wall', b.get('wall_us'))" "$f"; done
