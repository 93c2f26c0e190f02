#!/bin/bash
# K(x, X) fill workgroup size (DKG_KF_KB = 16 default; variants k-blocks per workgroup): batch-test bits, headline
# stage times, and the driver-shaped line (two runs each, interleaved).
set -uo pipefail
out=${1:-gpurun_out/r06_kf}
mkdir -p "$out"
AB=decoupled-kg_amd/dkg_amd/_native/ab
for v in kf8 kf4; do
  DKG_LIB=$AB/libdkg_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_batches.py -x -q --timeout 120 --timeout-method thread -k "per_batch_bits or stress or fp32" > "$out/tests_$v.log" 2>&1 || { tail -20 "$out/tests_$v.log"; exit 1; }
  tail -n1 "$out/tests_$v.log"
done
for v in def kf8 kf4; do
  L=""; [ $v != def ] && L=$AB/libdkg_$v.so
  DKG_LIB=$L timeout -k 10 150 python3 -u tools/stage_probe.py --workload headline --groups 1 5 20 > "$out/h_$v.txt" 2>&1 || { tail -5 "$out/h_$v.txt"; exit 1; }
  grep '^{' "$out/h_$v.txt" | cut -c1-150
done
Q="--cpu-seconds 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --grad-steps 0 --b1-calls 0 --prep-reps 0 --profile-reps 10 --single-rank-pg 0"
for rep in 1 2; do
  for v in def kf8 kf4; do
    L=""; [ $v != def ] && L=$AB/libdkg_$v.so
    DKG_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $Q > "$out/b20_${v}_$rep.json" 2> "$out/b20_${v}_$rep.err" || { tail -20 "$out/b20_${v}_$rep.err"; exit 1; }
  done
done
python3 tools/bench_summary.py $out/b20_*.json | cut -c1-110
