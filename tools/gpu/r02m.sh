#!/bin/bash
# headline gradient vs oracle, full GPU suite, stress bench lines (fp64, fp32)
set -uo pipefail
out=gpurun_out/r02m
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_grad.py -x -v --timeout 250 --timeout-method thread -m gpu -k "headline" > "$out/grad_headline.log" 2>&1
rc=$?; echo "grad rc=$rc"; grep -E "PASS|FAIL|Error|assert" "$out/grad_headline.log" | head -20
timeout -k 10 900 python3 -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > "$out/gpu_tests.log" 2>&1
rc2=$?; echo "tests rc=$rc2"; tail -3 "$out/gpu_tests.log"
timeout -k 10 300 python3 -u bench.py --workload stress --steps 256 --exchange-every 64 --cpu-seconds 0 --grad-steps 0 --b1-calls 0 --nd-steps 0 > "$out/stress64.json" 2> "$out/stress64.err"
echo "stress fp64 rc=$?"
timeout -k 10 300 python3 -u bench.py --workload stress32 --precision fp32 --steps 256 --exchange-every 64 --cpu-seconds 0 --grad-steps 0 --b1-calls 0 --nd-steps 0 > "$out/stress32.json" 2> "$out/stress32.err"
echo "stress fp32 rc=$?"
for f in stress64 stress32; do python3 -c "import json; d=json.load(open('$out/$f.json')); print('$f', d['value'], d['ms_per_step'], {k: round(v['avg_launch_us'],1) for k,v in d['roofline']['stages'].items()})"; done
exit $rc
