#!/bin/bash
# covariance stage at 16 waves (K quarters); cross stage 8 vs 16 waves (A/B lib)
set -uo pipefail
out=gpurun_out/r02zc
mkdir -p "$out"
AB=$PWD/decoupled-kg_amd/dkg_amd/_native/ab
timeout -k 10 600 python3 -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -1 "$out/tests.log"; [ $rc -eq 0 ] || exit $rc
DKG_LIB=$AB/libdkg_cr16.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_grad.py tests/test_gpu_api.py -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests_cr16.log" 2>&1
rc=$?; echo "tests cr16 rc=$rc"; tail -1 "$out/tests_cr16.log"; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/$name.json" 2> "$out/$name.err" || exit $?
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step; single', round(d['single_stream']['ms_per_step']*1e3,2), {k: round(v['avg_launch_us'],2) for k,v in d['roofline']['stages'].items()})"
}
run main
run cr16 DKG_LIB=$AB/libdkg_cr16.so
run main2
run cr16b DKG_LIB=$AB/libdkg_cr16.so
timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps.txt" 2>&1 || exit $?
DKG_LIB=$AB/libdkg_cr16.so timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps_cr16.txt" 2>&1 || exit $?
grep -E "WGs|lifetime" "$out/kstamps.txt" "$out/kstamps_cr16.txt"
