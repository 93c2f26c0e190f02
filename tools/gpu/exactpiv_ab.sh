#!/bin/bash
# The SMOKE loop against the oracle run, default build and the exact-pivot Cholesky variant; state tests; prep time.
set -uo pipefail
out=${1:-gpurun_out/exactpiv}
mkdir -p "$out"
ab=$GRAFT_REPO_ROOT/decoupled-kg_amd/dkg_amd/_native/ab
for v in cur exactpiv; do
  lib=""; [ "$v" != cur ] && lib=$ab/libdkg_$v.so
  DKG_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_bo_smoke.py tests/test_gpu_state.py -m gpu -q --timeout 240 --timeout-method thread > "$out/tests_$v.log" 2>&1
  echo "$v rc=$?"; tail -4 "$out/tests_$v.log"
  DKG_LIB=$lib timeout -k 10 120 python3 -u tools/smoke_probe.py 0 > "$out/smoke_probe_$v.txt" 2>&1 || true
  DKG_LIB=$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --grad-steps 0 --b1-calls 0 --nd-steps 0 --stress-steps 0 > "$out/bench_$v.json" 2> "$out/bench_$v.err" || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], d['state_prep'])" "$out/bench_$v.json"
done
