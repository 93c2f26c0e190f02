#!/bin/bash
# fill stage for the fp64 forward: bit identity vs the previous build, tests, A/B throughput, stamps
set -uo pipefail
out=gpurun_out/r02zz
mkdir -p "$out"
NEW=decoupled-kg_amd/dkg_amd/_native/libdkg.so
OLD=decoupled-kg_amd/dkg_amd/_native/ab/libdkg_old.so
timeout -k 10 400 python3 -u tools/ab_bits.py $OLD $NEW > "$out/ab_bits.txt" 2>&1
rc=$?; tail -3 "$out/ab_bits.txt"; echo "ab rc=$rc"; [ $rc -eq 0 ] || { cat "$out/ab_bits.txt" | tail -40; exit $rc; }
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_golden.py tests/test_gpu_dist.py -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$out/tests.log"; [ $rc -eq 0 ] || exit $rc
for v in old new old new; do
  lib=$NEW; [ $v = old ] && lib=$OLD
  DKG_LIB=$lib timeout -k 10 200 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/b4k_$v.json" 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$out/b4k_$v.json')); print('$v', round(d['value']), round(d['ms_per_step']*1e3,2), 'us/step; single', round(d['single_stream']['ms_per_step']*1e3,2), {k: round(v['avg_launch_us'],2) for k,v in d['roofline']['stages'].items()})"
done
for i in 1 2; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 > "$out/b20_$i.json" 2>/dev/null || exit 1
  python3 -c "import json; d=json.load(open('$out/b20_$i.json')); print('steps20 new', round(d['value']))"
done
timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps.txt" 2>&1 || exit 1
grep -E "WGs|lifetime" "$out/kstamps.txt"
