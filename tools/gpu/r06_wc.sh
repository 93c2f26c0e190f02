#!/bin/bash
# posterior_cov_big_kernel with 4 words per chunk (32 MFMAs per barrier; kernel terms in registers, DKG_PB_WC=4
# DKG_PB_KVREG=1; wc4s: three stage buffers) against the default (2 words): batch-test bits, stage times, and the
# driver-shaped line (two runs each, interleaved).
set -uo pipefail
out=${1:-gpurun_out/r06_wc}
mkdir -p "$out"
AB=decoupled-kg_amd/dkg_amd/_native/ab
for v in def wc4; do
  L=""; [ $v != def ] && L=$AB/libdkg_$v.so
  DKG_LIB=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_batches.py -x -q --timeout 120 --timeout-method thread > "$out/tests_$v.log" 2>&1 || { tail -20 "$out/tests_$v.log"; exit 1; }
  echo "$v: $(tail -n1 $out/tests_$v.log)"
done
for v in def wc4; do
  L=""; [ $v != def ] && L=$AB/libdkg_$v.so
  DKG_LIB=$L timeout -k 10 150 python3 -u tools/stage_probe.py --workload headline --groups 1 5 20 > "$out/h_$v.txt" 2>&1 || { tail -5 "$out/h_$v.txt"; exit 1; }
  DKG_LIB=$L timeout -k 10 150 python3 -u tools/stage_probe.py --workload stress --groups 1 > "$out/s_$v.txt" 2>&1 || { tail -5 "$out/s_$v.txt"; exit 1; }
  for f in "$out/h_$v.txt" "$out/s_$v.txt"; do grep '^{' "$f" | python3 -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$v', d['workload'], d['G'], 'cov', round(d['cov_us'],2), 'fwd', round(d['forward_us'],2))"; done
done
Q="--cpu-seconds 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --grad-steps 0 --b1-calls 0 --prep-reps 0 --profile-reps 10 --single-rank-pg 0"
for rep in 1 2; do
  for v in def wc4; do
    L=""; [ $v != def ] && L=$AB/libdkg_$v.so
    DKG_LIB=$L timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 $Q > "$out/b20_${v}_$rep.json" 2> "$out/b20_${v}_$rep.err" || { tail -20 "$out/b20_${v}_$rep.err"; exit 1; }
  done
done
for v in def wc4; do
  L=""; [ $v != def ] && L=$AB/libdkg_$v.so
  DKG_LIB=$L timeout -k 10 300 python3 -u bench.py $Q > "$out/bdef_${v}.json" 2> "$out/bdef_${v}.err" || { tail -20 "$out/bdef_${v}.err"; exit 1; }
done
python3 tools/bench_summary.py $out/b*.json | cut -c1-100
