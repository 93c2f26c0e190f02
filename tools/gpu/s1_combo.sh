#!/bin/bash
# Session check: streaming-envelope parity + stress stamps/bench, then the head-graph / priority A/B.
set -uo pipefail
out=${1:-gpurun_out/combo}
mkdir -p "$out"
bash tools/gpu/stress_check.sh "$out/stress" || exit 1
timeout -k 10 120 python3 -u tools/pair_stamps.py headline > "$out/pairs_headline.txt" 2>&1 || { tail -5 "$out/pairs_headline.txt"; exit 1; }
tail -25 "$out/pairs_headline.txt"
bash tools/gpu/head_check.sh "$out/head"
