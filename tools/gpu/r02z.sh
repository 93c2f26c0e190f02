#!/bin/bash
# psi by rational approximations, envelope at 4 waves/SIMD; cross stage with 4 tile pairs per workgroup
set -uo pipefail
out=gpurun_out/${OUT:-r02z}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$out/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 > "$out/bench.json" 2> "$out/bench.err" || exit $?
python3 -c "import json; d=json.load(open('$out/bench.json')); print('bench', round(d['value']), d['single_stream']['value'], {k: round(v['avg_launch_us'],2) for k,v in d['roofline']['stages'].items()}, d['nondegenerate']['value'], round(d['nondegenerate']['envelope_us'],2))"
timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/bench4k.json" 2>/dev/null || exit $?
python3 -c "import json; d=json.load(open('$out/bench4k.json')); print('4096 steps', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step')"
timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps.txt" 2>&1 || exit $?
grep -E "WGs|lifetime" "$out/kstamps.txt"
timeout -k 10 120 python3 -u tools/pair_stamps.py headline > "$out/pairs_headline.txt" 2>&1 || exit $?
head -12 "$out/pairs_headline.txt"
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --profile-reps 2 --grad-steps 0 --b1-calls 0 --nd-steps 0 --streams 1 --graph 0 > /dev/null 2>&1
echo "write rc=$?"
python3 - <<PY
import csv, glob
v=[float(r['Counter_Value']) for f in glob.glob('$out/write/**/*counter_collection.csv', recursive=True) for r in csv.DictReader(open(f)) if 'envelope_kernel' in r['Kernel_Name'] and ', true,' not in r['Kernel_Name']]
print('envelope WRITE_SIZE KB per launch', sum(v)/max(1,len(v)))
PY
