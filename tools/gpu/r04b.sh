#!/bin/bash
# Round-4 measurement pass: GPU suite, driver-shape and default bench lines, per-workgroup and per-pair envelope
# stamps (headline, headline_nd), B = 1 breakdown, state-preparation kernel statistics.
set -uo pipefail
out=${1:-gpurun_out/r04b}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
timeout -k 10 300 python3 -u tools/f32_stress_probe.py "$out/f32_stress.json" > "$out/f32.log" 2>&1 || { tail -5 "$out/f32.log"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$out/b20_$i.json" 2> "$out/b20_$i.err" || { tail -5 "$out/b20_$i.err"; exit 1; }
done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --launch-threads 1 --grad-steps 0 --b1-calls 0 \
  --nd-steps 0 --stress-steps 0 --prep-reps 0 > "$out/b20_lt1.json" 2> "$out/b20_lt1.err" || { tail -5 "$out/b20_lt1.err"; exit 1; }
timeout -k 10 400 python3 -u bench.py --cpu-seconds 3 > "$out/bench_default.json" 2> "$out/bench_default.err" || { tail -5 "$out/bench_default.err"; exit 1; }
python3 tools/bench_summary.py "$out"/b20_*.json "$out/bench_default.json"
for wl in headline headline_nd; do
  timeout -k 10 120 python3 -u tools/kstamps.py $wl > "$out/kst_$wl.txt" 2>&1 || { tail -5 "$out/kst_$wl.txt"; exit 1; }
  timeout -k 10 120 python3 -u tools/pair_stamps.py $wl > "$out/pairs_$wl.txt" 2>&1 || { tail -5 "$out/pairs_$wl.txt"; exit 1; }
done
timeout -k 10 200 python3 -u tools/b1_probe.py > "$out/b1_probe.txt" 2>&1 || { tail -5 "$out/b1_probe.txt"; exit 1; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prep" -o prep -- python3 tools/prep_kernels.py \
  > "$out/prep.log" 2>&1 || { tail -5 "$out/prep.log"; exit 1; }
ls "$out"
