#!/bin/bash
# posterior_cov_big_kernel with the kernel terms in registers (DKG_PB_KVREG=1) at two and three stage buffers
# (kv2, kv3) against the default build: batch-test bits, stage times, stamps at 5 batches, the driver-shaped line.
set -uo pipefail
out=${1:-gpurun_out/r06_kv}
mkdir -p "$out"
AB=decoupled-kg_amd/dkg_amd/_native/ab
for v in kv2 kv3; do
  DKG_LIB=$AB/libdkg_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_batches.py -x -q --timeout 120 --timeout-method thread > "$out/tests_$v.log" 2>&1 || { tail -20 "$out/tests_$v.log"; exit 1; }
  tail -n1 "$out/tests_$v.log"
done
for v in def kv2 kv3; do
  L=""; [ $v != def ] && L=$AB/libdkg_$v.so
  DKG_LIB=$L timeout -k 10 150 python3 -u tools/stage_probe.py --workload headline --groups 1 5 10 > "$out/h_$v.txt" 2>&1 || { tail -5 "$out/h_$v.txt"; exit 1; }
  grep '^{' "$out/h_$v.txt" | cut -c1-200
  DKG_LIB=$L timeout -k 10 150 python3 -u tools/stage_probe.py --workload stress --groups 1 > "$out/s_$v.txt" 2>&1 || { tail -5 "$out/s_$v.txt"; exit 1; }
  grep '^{' "$out/s_$v.txt" | cut -c1-200
  DKG_LIB=$L timeout -k 10 120 python3 -u tools/cov_stamps.py 5 > "$out/covst_$v.txt" 2>&1 || { tail -5 "$out/covst_$v.txt"; exit 1; }
  grep -v amdgpu.ids "$out/covst_$v.txt"
done
Q="--cpu-seconds 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --grad-steps 0 --b1-calls 0 --prep-reps 0 --profile-reps 10 --single-rank-pg 0"
for rep in 1 2; do
  for v in def kv2 kv3; do
    L=""; [ $v != def ] && L=$AB/libdkg_$v.so
    DKG_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $Q > "$out/b20_${v}_$rep.json" 2> "$out/b20_${v}_$rep.err" || { tail -20 "$out/b20_${v}_$rep.err"; exit 1; }
  done
done
python3 tools/bench_summary.py $out/b20_*.json | cut -c1-160
