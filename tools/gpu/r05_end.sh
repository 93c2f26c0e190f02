#!/bin/bash
# Round-5 end-of-work check on the box: every -m gpu test, the cross-stage A/B, the driver-shaped bench twice and
# the default bench once.  usage: tools/gpu/r05_end.sh <out>
set -uo pipefail
out=${1:-gpurun_out/r05end}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
for xb in 1 0; do
  DKG_CROSS_BIG=$xb timeout -k 10 150 python3 -u tools/stage_probe.py --workload stress --groups 1 > "$out/cross_s_x$xb.txt" 2>&1 || exit 1
  DKG_CROSS_BIG=$xb timeout -k 10 150 python3 -u tools/stage_probe.py --workload headline --groups 1 10 20 > "$out/cross_h_x$xb.txt" 2>&1 || exit 1
done
grep -h '^{' "$out"/cross_*.txt | cut -c1-150
for i in 1 2; do
  timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > "$out/b20_$i.json" 2> "$out/b20_$i.err" || { tail -5 "$out/b20_$i.err"; exit 1; }
done
timeout -k 10 500 python3 -u bench.py > "$out/b1024.json" 2> "$out/b1024.err" || { tail -5 "$out/b1024.err"; exit 1; }
python3 tools/bench_summary.py "$out"/b*.json
