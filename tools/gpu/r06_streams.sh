#!/bin/bash
# The driver-shaped line (--steps 20 --warmup 5, main legs only) at 1, 2 and 4 streams (G = 20, 10, 5), and the
# default 1,024-step run at 1, 2, 4 streams; two runs each, interleaved.
set -uo pipefail
out=${1:-gpurun_out/r06_streams}
mkdir -p "$out"
Q="--cpu-seconds 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --grad-steps 0 --b1-calls 0 --prep-reps 0 --profile-reps 10 --single-rank-pg 0"
for rep in 1 2; do
  for s in 1 2 4; do
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --streams $s $Q > "$out/b20_s${s}_$rep.json" 2> "$out/b20_s${s}_$rep.err" || { tail -20 "$out/b20_s${s}_$rep.err"; exit 1; }
  done
done
for s in 1 2 4; do
  timeout -k 10 300 python3 -u bench.py --streams $s $Q > "$out/bdef_s${s}.json" 2> "$out/bdef_s${s}.err" || { tail -20 "$out/bdef_s${s}.err"; exit 1; }
done
python3 tools/bench_summary.py $out/b*.json | cut -c1-140
for f in $out/b20_s*_1.json; do python3 -c "
import json,sys; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); r=d['region_breakdown']; print('$f', r['host_launch_done_us'], r['stream_piece_done_us'], r['wall_us'])"; done
