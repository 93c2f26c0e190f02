#!/bin/bash
# forwards in flight: HIP hardware queues x streams, envelope split 2 vs 1
set -uo pipefail
out=gpurun_out/r02q
mkdir -p "$out"
for sp in 2 1; do
  for q in 4 8 16; do
    DKG_ENV_SPLIT=$sp GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 --streams $q > "$out/b_s${sp}_q$q.json" 2>"$out/b_s${sp}_q$q.err" || exit $?
    python3 -c "import json; d=json.load(open('$out/b_s${sp}_q$q.json')); print('split $sp queues/streams $q', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step')"
  done
done
