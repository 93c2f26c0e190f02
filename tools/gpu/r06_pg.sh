#!/bin/bash
# The driver-shaped line (--steps 20 --warmup 5) with and without the one-rank RCCL process group, main legs only.
set -uo pipefail
out=${1:-gpurun_out/r06_pg}
mkdir -p "$out"
Q="--cpu-seconds 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --grad-steps 0 --b1-calls 0 --prep-reps 0 --profile-reps 10"
n=0
for pg in 1 0 1 0; do
  n=$((n+1))
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --single-rank-pg $pg $Q > "$out/b20_pg${pg}_$n.json" 2> "$out/b20_pg${pg}_$n.err" || { tail -20 "$out/b20_pg${pg}_$n.err"; exit 1; }
done
python3 tools/bench_summary.py $out/b20_*.json
