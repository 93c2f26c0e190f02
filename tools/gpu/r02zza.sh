#!/bin/bash
# HIP runtime knobs vs the default: kernel arguments in device memory
set -uo pipefail
out=gpurun_out/r02zza
mkdir -p "$out"
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/$name.json" 2> "$out/$name.err" || exit 1
  env "$@" timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 20 --warmup 5 > "$out/${name}_20.json" 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$out/$name.json')); e=json.load(open('$out/${name}_20.json')); print('$name', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step; single', round(d['single_stream']['ms_per_step']*1e3,2), '; 20 steps', round(e['value']))"
}
run base
run devka1 HIP_FORCE_DEV_KERNARG=1
run devka0 HIP_FORCE_DEV_KERNARG=0
run base2
run devka1b HIP_FORCE_DEV_KERNARG=1
