#!/bin/bash
# forward envelope: 8 vs 16 scalarisation waves per workgroup (one workgroup per candidate at S = 16)
set -uo pipefail
out=gpurun_out/r02zh
mkdir -p "$out"
DKG_ENV_FWD_WAVES=16 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_epigraph.py -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests_w16.log" 2>&1
rc=$?; echo "tests w16 rc=$rc"; tail -1 "$out/tests_w16.log"; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/$name.json" 2> "$out/$name.err" || exit $?
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step; single', round(d['single_stream']['ms_per_step']*1e3,2), {k: round(v['avg_launch_us'],2) for k,v in d['roofline']['stages'].items()})"
}
run w8
run w16 DKG_ENV_FWD_WAVES=16
run w8b
run w16b DKG_ENV_FWD_WAVES=16
DKG_ENV_FWD_WAVES=16 timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps_w16.txt" 2>&1 || exit $?
grep -E "WGs|lifetime" "$out/kstamps_w16.txt"
