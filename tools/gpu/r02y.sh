#!/bin/bash
# envelope occupancy A/B: one-shot at 3 waves/SIMD (168 VGPRs) with 4- or 2-wave workgroups
set -uo pipefail
out=gpurun_out/r02y
mkdir -p "$out"
AB=$PWD/decoupled-kg_amd/dkg_amd/_native/ab
DKG_LIB=$AB/libdkg_os3.so DKG_ENV_WAVES=4 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests_os3_w4.log" 2>&1
rc=$?; echo "tests os3 w4 rc=$rc"; tail -1 "$out/tests_os3_w4.log"; [ $rc -eq 0 ] || exit $rc
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/$name.json" 2> "$out/$name.err" || exit $?
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step; single', round(d['single_stream']['ms_per_step']*1e3,2), {k: round(v['avg_launch_us'],2) for k,v in d['roofline']['stages'].items()})"
}
run main_s2
run main_s1 DKG_ENV_SPLIT=1
run os2_w8 DKG_LIB=$AB/libdkg_os2.so
run os3_w8 DKG_LIB=$AB/libdkg_os3.so
run os3_w4 DKG_LIB=$AB/libdkg_os3.so DKG_ENV_WAVES=4
run os3_w2 DKG_LIB=$AB/libdkg_os3.so DKG_ENV_WAVES=2
run os2_w4 DKG_LIB=$AB/libdkg_os2.so DKG_ENV_WAVES=4
DKG_LIB=$AB/libdkg_os3.so DKG_ENV_WAVES=4 timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps_os3_w4.txt" 2>&1 || exit $?
grep -E "WGs|lifetime" "$out/kstamps_os3_w4.txt"
