#!/bin/bash
# Driver-shape bench A/B: per-stream head graphs (bench.py --graph-head) and the walked-pair issue priority
# (DKG_DEBUG_ENV_FLAGS=4 turns it off), alternated; then the default 1024-step run with and without priority.
set -uo pipefail
out=${1:-gpurun_out/head}
mkdir -p "$out"
summ() { python3 -c "import json,sys; d=json.load(open(sys.argv[1])); nd=d.get('nondegenerate') or {}; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step host', round(d['host_launch_us_per_step'],2), 'nd', round(nd.get('value',0)/1e6,2))" "$1"; }
for i in 1 2 3; do
  for v in h0 h1 h2 h1np; do
    case $v in h0) h=0; f=0;; h1) h=1; f=0;; h2) h=2; f=0;; h1np) h=1; f=4;; esac
    DKG_DEBUG_ENV_FLAGS=$f timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --graph-head $h \
      --b1-calls 0 --grad-steps 0 --nd-steps 20 --stress-steps 0 --prep-reps 0 > "$out/b20_${v}_$i.json" 2> "$out/b20_${v}_$i.err" \
      || { tail -5 "$out/b20_${v}_$i.err"; exit 1; }
    summ "$out/b20_${v}_$i.json"
  done
done
for f in 0 4; do
  DKG_DEBUG_ENV_FLAGS=$f timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --stress-steps 0 \
    --prep-reps 0 > "$out/b1024_f$f.json" 2> "$out/b1024_f$f.err" || { tail -5 "$out/b1024_f$f.err"; exit 1; }
  summ "$out/b1024_f$f.json"
done
