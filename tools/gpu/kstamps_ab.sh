#!/bin/bash
# Per-workgroup phase stamps of the forward, fused launch vs the three stage kernels (tools/kstamps.py).
set -uo pipefail
out=${1:-gpurun_out/kst}
mkdir -p "$out"
for wl in headline headline_nd; do
  DKG_FUSED=1 timeout -k 10 120 python3 -u tools/kstamps.py $wl > "$out/kst_fused_$wl.txt" 2>&1 || { tail -5 "$out/kst_fused_$wl.txt"; exit 1; }
  timeout -k 10 120 python3 -u tools/kstamps.py $wl > "$out/kst_split_$wl.txt" 2>&1 || { tail -5 "$out/kst_split_$wl.txt"; exit 1; }
done
cat "$out"/kst_fused_headline.txt "$out"/kst_split_headline.txt
