#!/bin/bash
# A/B: forward envelope at 3 waves/SIMD (<=168 VGPRs, main build) vs 2 (256 VGPRs, ab build)
set -uo pipefail
out=gpurun_out/r02o
mkdir -p "$out"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_epigraph.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$out/tests.log"; [ $rc -eq 0 ] || exit $rc
for v in main wpe3; do
  if [ $v = wpe3 ]; then export DKG_LIB=$PWD/decoupled-kg_amd/dkg_amd/_native/ab/libdkg_wpe3.so; fi
  timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 > "$out/bench_$v.json" 2> "$out/bench_$v.err" || exit $?
  python3 -c "import json; d=json.load(open('$out/bench_$v.json')); print('$v', d['value'], d['single_stream']['value'], {k: round(v['avg_launch_us'],2) for k,v in d['roofline']['stages'].items()}, d['nondegenerate']['value'], round(d['nondegenerate']['envelope_us'],2))"
  timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/bench4k_$v.json" 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$out/bench4k_$v.json')); print('$v 4096 steps', d['value'])"
done
export DKG_LIB=$PWD/decoupled-kg_amd/dkg_amd/_native/ab/libdkg_wpe3.so
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --profile-reps 2 --grad-steps 0 --b1-calls 0 --nd-steps 0 --streams 1 --graph 0 > /dev/null 2>&1
echo "write rc=$?"
python3 - <<PY
import csv, glob
v=[float(r['Counter_Value']) for f in glob.glob('$out/write/**/*counter_collection.csv', recursive=True) for r in csv.DictReader(open(f)) if 'envelope_kernel' in r['Kernel_Name'] and ', true,' not in r['Kernel_Name']]
print('envelope WRITE_SIZE KB per launch', sum(v)/max(1,len(v)))
PY
