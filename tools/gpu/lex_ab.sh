#!/bin/bash
# DKG_ENV_LEX variant: forward parity suites on it, headline pair stamps of both builds, then the variant A/B.
set -uo pipefail
out=${1:-gpurun_out/lex}
mkdir -p "$out"
lib=$GRAFT_REPO_ROOT/decoupled-kg_amd/dkg_amd/_native/ab/libdkg_lex.so
DKG_LIB=$lib timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fused.py tests/test_gpu_epigraph.py \
  tests/test_gpu_grad.py -m gpu -x -q --timeout 300 --timeout-method thread > "$out/tests_lex.log" 2>&1 || { tail -30 "$out/tests_lex.log"; exit 1; }
tail -1 "$out/tests_lex.log"
for w in headline headline_nd; do
  timeout -k 10 120 python3 -u tools/pair_stamps.py $w > "$out/pairs_${w}_cur.txt" 2>&1 || exit 1
  DKG_LIB=$lib timeout -k 10 120 python3 -u tools/pair_stamps.py $w > "$out/pairs_${w}_lex.txt" 2>&1 || exit 1
  echo "== $w"; sed -n 4,8p "$out/pairs_${w}_cur.txt"; sed -n 4,8p "$out/pairs_${w}_lex.txt"
done
bash tools/gpu/ab_variants.sh "$out/ab"
