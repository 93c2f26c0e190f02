#!/bin/bash
# The driver's shape (--steps 20 --warmup 5) at other stream counts / batches per launch, two runs each.
set -uo pipefail
out=${1:-gpurun_out/r06_sg}
mkdir -p "$out"
Q="--cpu-seconds 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --grad-steps 0 --b1-calls 0 --prep-reps 0 --profile-reps 2 --single-rank-pg 0"
for rep in 1 2; do
  for cfg in "4 5" "5 4" "10 2" "4 4" "8 2"; do
    set -- $cfg
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --streams $1 --batches-per-launch $2 $Q > "$out/b20_s$1_g$2_$rep.json" 2> "$out/b20_s$1_g$2_$rep.err" || { tail -20 "$out/b20_s$1_g$2_$rep.err"; exit 1; }
  done
done
python3 tools/bench_summary.py $out/b20_*.json | cut -c1-100
