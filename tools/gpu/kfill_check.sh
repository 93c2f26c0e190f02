#!/bin/bash
# Cross-stage K(x, X) fill (large n): bit-identity against the build without it, the stress parity suite,
# the stress leg.
set -uo pipefail
out=${1:-gpurun_out/kfill}
mkdir -p "$out"
timeout -k 10 400 python3 -u tools/ab_bits.py decoupled-kg_amd/dkg_amd/_native/libdkg.so \
  decoupled-kg_amd/dkg_amd/_native/ab/libdkg_nokfill.so > "$out/ab.txt" 2>&1 || { tail -20 "$out/ab.txt"; exit 1; }
tail -25 "$out/ab.txt"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -k "stress or f32" -x -q --timeout 300 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for v in on off; do
  lib=decoupled-kg_amd/dkg_amd/_native/libdkg.so; [ $v = off ] && lib=decoupled-kg_amd/dkg_amd/_native/ab/libdkg_nokfill.so
  DKG_LIB=$PWD/$lib timeout -k 10 300 python3 -u bench.py --workload stress --steps 16 --warmup 4 --cpu-seconds 0 --b1-calls 0 \
    --grad-steps 0 --nd-steps 0 --stress-steps 0 --prep-reps 0 > "$out/bs_$v.json" 2> "$out/bs_$v.err" || { tail -5 "$out/bs_$v.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e3,1), 'K/s', {k: round(v['avg_launch_us'],1) for k,v in d['roofline']['stages'].items()})" "$out/bs_$v.json" $v
done
