#!/bin/bash
# Driver-shape bench runs (--steps 20 --warmup 5) and the default run.
set -uo pipefail
out=${1:-gpurun_out/b20}
mkdir -p "$out"
for i in 1 2 3; do
  timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$out/b20_$i.json" 2> "$out/b20_$i.err" || { tail -5 "$out/b20_$i.err"; exit 1; }
  python3 tools/bench_summary.py "$out/b20_$i.json"
done
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --graph 0 --nd-steps 0 --stress-steps 0 --b1-calls 0 --grad-steps 0 > "$out/b20_eager.json" 2> "$out/b20_eager.err" || { tail -5 "$out/b20_eager.err"; exit 1; }
python3 tools/bench_summary.py "$out/b20_eager.json"
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 > "$out/b1024.json" 2> "$out/b1024.err" || { tail -5 "$out/b1024.err"; exit 1; }
python3 tools/bench_summary.py "$out/b1024.json"
