#!/bin/bash
# stage ablations under the 4-stream throughput: which kernel bounds the forwards in flight
set -uo pipefail
out=gpurun_out/r02s
mkdir -p "$out"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/$name.json" 2> "$out/$name.err" || exit $?
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step; single', round(d['single_stream']['ms_per_step']*1e3,2), {k: round(v['avg_launch_us'],2) for k,v in d['roofline']['stages'].items()})"
}
for sp in 2 1; do
  run s${sp}_all DKG_ENV_SPLIT=$sp
  run s${sp}_noenv DKG_ENV_SPLIT=$sp DKG_DEBUG_ENV_FLAGS=2
  run s${sp}_nocov DKG_ENV_SPLIT=$sp DKG_DEBUG_COV_FLAGS=1
  run s${sp}_nocross DKG_ENV_SPLIT=$sp DKG_DEBUG_COV_FLAGS=2
done
run s1_none DKG_ENV_SPLIT=1 DKG_DEBUG_COV_FLAGS=3 DKG_DEBUG_ENV_FLAGS=2
