#!/bin/bash
# Envelope change: forward parity suites, pair stamps, then the variant A/B (tools/gpu/ab_variants.sh).
set -uo pipefail
out=${1:-gpurun_out/r04h}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_fused.py tests/test_gpu_epigraph.py \
  tests/test_gpu_grad.py -m gpu -x -q --timeout 300 --timeout-method thread > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
timeout -k 10 120 python3 -u tools/pair_stamps.py headline > "$out/pairs_headline.txt" 2>&1 || { tail -5 "$out/pairs_headline.txt"; exit 1; }
DKG_LIB=$GRAFT_REPO_ROOT/decoupled-kg_amd/dkg_amd/_native/ab/libdkg_nohint.so timeout -k 10 120 python3 -u tools/pair_stamps.py headline > "$out/pairs_headline_nohint.txt" 2>&1 || exit 1
head -12 "$out/pairs_headline.txt"; head -12 "$out/pairs_headline_nohint.txt"
bash tools/gpu/ab_variants.sh "$out/ab"
