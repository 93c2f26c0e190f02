#!/bin/bash
# configs[4] stress shape at the final tree (fp64; fp32-contraction opt-in)
set -uo pipefail
out=gpurun_out/r02zzc
mkdir -p "$out"
timeout -k 10 300 python3 -u bench.py --workload stress --steps 256 --exchange-every 64 --cpu-seconds 0 --grad-steps 0 --b1-calls 0 --nd-steps 0 > "$out/stress64.json" 2> "$out/stress64.err" || { tail -5 "$out/stress64.err"; exit 1; }
timeout -k 10 300 python3 -u bench.py --workload stress32 --precision fp32 --steps 256 --exchange-every 64 --cpu-seconds 0 --grad-steps 0 --b1-calls 0 --nd-steps 0 > "$out/stress32.json" 2> "$out/stress32.err" || { tail -5 "$out/stress32.err"; exit 1; }
python3 -c "
import json
for f in ('stress64','stress32'):
    d=json.load(open('$out/'+f+'.json')); print(f, round(d['value']), round(d['ms_per_step']*1e3,1), 'us/step', {k: round(v['avg_launch_us'],1) for k,v in d['roofline']['stages'].items()})"
