#!/bin/bash
# The covariance stage's workgroup phases: this tree against the round-3 build (kstamps, headline), twice each.
set -uo pipefail
out=${1:-gpurun_out/covcmp}
mkdir -p "$out"
for rep in 1 2; do
  timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kst_cur_$rep.txt" 2>&1 || exit 1
  (cd .ab/f96856c && timeout -k 10 120 python3 -u tools/kstamps.py headline) > "$out/kst_r03_$rep.txt" 2>&1 || exit 1
done
for f in "$out"/kst_*.txt; do echo "== $f"; grep -A4 "^posterior_cov" "$f"; grep -A1 "^cross_root" "$f"; done
