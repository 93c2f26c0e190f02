#!/bin/bash
# forwards-in-flight launch modes: one forked graph vs per-stream graphs; streams 4 / 6 / 8
set -uo pipefail
out=gpurun_out/r02ze
mkdir -p "$out"
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 150 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 "$@" > "$out/$name.json" 2> "$out/$name.err" || exit $?
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step; host', round(d['host_launch_us_per_step'],2))"
}
run g1_s4 --graph 1 --streams 4
run g2_s4 --graph 2 --streams 4
run g1_s6 --graph 1 --streams 6
run g2_s6 --graph 2 --streams 6
run g2_s8 --graph 2 --streams 8
run g1_s2 --graph 1 --streams 2
run g2_s2 --graph 2 --streams 2
