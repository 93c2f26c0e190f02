#!/bin/bash
# Covariance block A/B at the stress shape (DKG_COV_WIDE=0: 32 x 32 blocks, 1: 64 x 64): parity of the
# stress suites with the wide blocks, then the kernel stamps and the stress leg with each.
set -uo pipefail
out=${1:-gpurun_out/cov}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -k "stress" -x -q --timeout 300 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for w in 0 1; do
  DKG_COV_WIDE=$w timeout -k 10 200 python3 -u tools/kstamps.py stress > "$out/kst_w$w.txt" 2>&1 || { tail -5 "$out/kst_w$w.txt"; exit 1; }
  echo "== wide=$w"; grep -A5 "^posterior_cov" "$out/kst_w$w.txt"
  DKG_COV_WIDE=$w timeout -k 10 300 python3 -u bench.py --workload stress --steps 16 --warmup 4 --cpu-seconds 0 --b1-calls 0 \
    --grad-steps 0 --nd-steps 0 --stress-steps 0 --prep-reps 0 > "$out/bs_w$w.json" 2> "$out/bs_w$w.err" || { tail -5 "$out/bs_w$w.err"; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(round(d['value']/1e3,1), 'K/s', {k: round(v['avg_launch_us'],1) for k,v in d['roofline']['stages'].items()})" "$out/bs_w$w.json"
done
