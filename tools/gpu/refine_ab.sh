#!/bin/bash
# Envelope list refinement (DKG_ENV_REFINE, DKG_REFINE_OVERFLOW): forward + gradient parity suites, headline /
# headline_nd pair and kernel stamps of the default build and each variant, then the variant A/B.
set -uo pipefail
out=${1:-gpurun_out/refine_ab}
mkdir -p "$out"
ab=$GRAFT_REPO_ROOT/decoupled-kg_amd/dkg_amd/_native/ab
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fused.py tests/test_gpu_epigraph.py \
  tests/test_gpu_grad.py -m gpu -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
for w in headline headline_nd; do
  for v in cur $(ls "$ab" | sed 's/libdkg_\(.*\)\.so/\1/'); do
    lib=""; [ "$v" != cur ] && lib=$ab/libdkg_$v.so
    DKG_LIB=$lib timeout -k 10 120 python3 -u tools/pair_stamps.py $w > "$out/pairs_${w}_$v.txt" 2>&1 || { tail -5 "$out/pairs_${w}_$v.txt"; exit 1; }
    DKG_LIB=$lib timeout -k 10 120 python3 -u tools/kstamps.py $w > "$out/kst_${w}_$v.txt" 2>&1 || { tail -5 "$out/kst_${w}_$v.txt"; exit 1; }
    echo "== $w $v"; sed -n 3,10p "$out/pairs_${w}_$v.txt"; grep -A2 "^envelope" "$out/kst_${w}_$v.txt"
  done
done
bash tools/gpu/ab_variants.sh "$out/ab"
