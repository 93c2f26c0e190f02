#!/bin/bash
# Multi-candidate envelope workgroups (DKG_ENV_IPW): bit tests, headline / headline_nd stage times, envelope
# stamps at 5 batches, and the driver-shaped line per ipw (two runs each, interleaved).
set -uo pipefail
out=${1:-gpurun_out/r06_ipw}
mkdir -p "$out"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_env_items.py -x -q --timeout 120 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -n1 "$out/tests.log"
for v in 1 2 4; do
  DKG_ENV_IPW=$v timeout -k 10 150 python3 -u tools/stage_probe.py --workload headline --groups 1 5 20 > "$out/h_$v.txt" 2>&1 || { tail -5 "$out/h_$v.txt"; exit 1; }
  grep '^{' "$out/h_$v.txt" | cut -c1-190
  DKG_ENV_IPW=$v timeout -k 10 150 python3 -u tools/stage_probe.py --workload headline_nd --groups 1 5 > "$out/nd_$v.txt" 2>&1 || { tail -5 "$out/nd_$v.txt"; exit 1; }
  grep '^{' "$out/nd_$v.txt" | cut -c1-190
done
Q="--cpu-seconds 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --grad-steps 0 --b1-calls 0 --prep-reps 0 --profile-reps 10 --single-rank-pg 0"
for rep in 1 2; do
  for v in 1 2 4; do
    DKG_ENV_IPW=$v timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $Q > "$out/b20_${v}_$rep.json" 2> "$out/b20_${v}_$rep.err" || { tail -20 "$out/b20_${v}_$rep.err"; exit 1; }
  done
done
for v in 1 2 4; do
  DKG_ENV_IPW=$v timeout -k 10 300 python3 -u bench.py $Q > "$out/bdef_${v}.json" 2> "$out/bdef_${v}.err" || { tail -20 "$out/bdef_${v}.err"; exit 1; }
done
python3 tools/bench_summary.py $out/b*.json | cut -c1-110
