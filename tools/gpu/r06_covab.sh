#!/bin/bash
# The driver-shaped line (--steps 20 --warmup 5, main legs only) with each covariance block kernel at its 5-batch
# launches: rec2 (default), the 64 x 32 blocks, the 64 x 64 blocks (round 5); two runs each, interleaved.
set -uo pipefail
out=${1:-gpurun_out/r06_covab}
mkdir -p "$out"
Q="--cpu-seconds 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --grad-steps 0 --b1-calls 0 --prep-reps 0 --profile-reps 10 --single-rank-pg 0"
for rep in 1 2; do
  for cfg in rec2 blk big64; do
    case $cfg in rec2) E="X=1";; blk) E="DKG_COV_REC2=0";; big64) E="DKG_COV_REC2=0 DKG_COV_BLK=0";; esac
    env $E timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $Q > "$out/b20_${cfg}_$rep.json" 2> "$out/b20_${cfg}_$rep.err" || { tail -20 "$out/b20_${cfg}_$rep.err"; exit 1; }
  done
done
python3 tools/bench_summary.py $out/b20_*.json | cut -c1-200
