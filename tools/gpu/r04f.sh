#!/bin/bash
# GPU suite, stamps (headline), bench at the driver shape (x2) and the default bench line.
set -uo pipefail
out=${1:-gpurun_out/r04f}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kst_headline.txt" 2>&1 || { tail -5 "$out/kst_headline.txt"; exit 1; }
timeout -k 10 120 python3 -u tools/pair_stamps.py headline > "$out/pairs_headline.txt" 2>&1 || { tail -5 "$out/pairs_headline.txt"; exit 1; }
for i in 1 2; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$out/b20_$i.json" 2> "$out/b20_$i.err" || { tail -5 "$out/b20_$i.err"; exit 1; }
done
timeout -k 10 400 python3 -u bench.py --cpu-seconds 3 > "$out/bench_default.json" 2> "$out/bench_default.err" || { tail -5 "$out/bench_default.err"; exit 1; }
python3 tools/bench_summary.py "$out"/b20_*.json "$out/bench_default.json"
grep -v amdgpu.ids "$out/kst_headline.txt" | sed -n '/^envelope/,$p' | head -8
