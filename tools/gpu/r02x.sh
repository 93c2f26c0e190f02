#!/bin/bash
# covariance stage: operand and epilogue loads in one round trip, one 32-k-block batch
set -uo pipefail
out=gpurun_out/r02x
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$out/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps.txt" 2>&1 || exit $?
grep -E "WGs|lifetime|loads|LDS" "$out/kstamps.txt"
for v in 2 1; do
  export DKG_ENV_SPLIT=$v
  timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/bench4k_s$v.json" 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$out/bench4k_s$v.json')); print('split $v 4096 steps', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step', {k: round(v['avg_launch_us'],2) for k,v in d['roofline']['stages'].items()})"
done
