#!/bin/bash
# Round-4 first check: GPU suite, fp32 probe at configs[4]'s shape, driver-shape bench with the side-by-side
# graph launcher (dkg_launcher) and without it (--launch-threads 1).
set -uo pipefail
out=${1:-gpurun_out/r04a}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
timeout -k 10 300 python3 -u tools/f32_stress_probe.py "$out/f32_stress.json" > "$out/f32.log" 2>&1 || { tail -5 "$out/f32.log"; exit 1; }
for i in 1 2; do
  for lt in -1 1; do
    timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --launch-threads $lt --grad-steps 0 \
      --b1-calls 0 --nd-steps 0 --stress-steps 0 --prep-reps 0 > "$out/b20_lt${lt}_$i.json" 2> "$out/b20_lt${lt}_$i.err" || { tail -5 "$out/b20_lt${lt}_$i.err"; exit 1; }
  done
done
python3 tools/bench_summary.py "$out"/b20_*.json
