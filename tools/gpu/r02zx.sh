#!/bin/bash
# GRAD envelope flat early-out: grad/api/optim/parity tests, value+gradient timing, B=1 probe, scratch check
set -uo pipefail
out=gpurun_out/r02zx
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_grad.py tests/test_gpu_api.py tests/test_gpu_optim.py tests/test_gpu_dist.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$out/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 --nd-steps 0 --steps 256 > "$out/bench.json" 2> "$out/bench.err" || { tail -5 "$out/bench.err"; exit 1; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(round(d['value']), d['value_and_grad'], d['latency_b1']['median_us'])"
timeout -k 10 200 python3 -u tools/b1_probe.py headline 300 > "$out/b1_probe.txt" 2>&1 || exit 1
tail -1 "$out/b1_probe.txt"
timeout -k 10 200 python3 -u tools/bench_optimize.py --cpu-seconds 0 > "$out/bench_optimize.json" 2>&1 || exit 1
tail -1 "$out/bench_optimize.json"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$out/tr" -o run -- python3 tools/b1_probe.py headline 20 > /dev/null 2>&1 || exit 1
python3 -c "
import csv,glob
f=glob.glob('$out/tr/**/*kernel_trace.csv', recursive=True)[0]
seen={}
for r in csv.DictReader(open(f)):
    n=r['Kernel_Name'].split('(')[0]
    if 'envelope' in n or 'cross' in n: seen[n]=(r['Scratch_Size'], r['VGPR_Count'], r['Accum_VGPR_Count'])
print(seen)"
