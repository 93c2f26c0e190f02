#!/bin/bash
# final tree: full GPU suite, smoke(), driver-shaped bench
set -uo pipefail
out=gpurun_out/r02zzb
mkdir -p "$out"
timeout -k 10 900 python3 -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > "$out/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$out/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 "$out/smoke.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$out/b20.json" 2> "$out/b20.err" || exit 1
python3 -c "import json; d=json.load(open('$out/b20.json')); print('steps20', round(d['value']), d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 400 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err" || exit 1
python3 -c "import json; d=json.load(open('$out/bench.json')); print('default', round(d['value']), d['latency_b1']['median_us'], d['value_and_grad']['value'], d['nondegenerate']['value'])"
