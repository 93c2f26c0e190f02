#!/bin/bash
set -uo pipefail
out=gpurun_out/r02d
mkdir -p "$out"
timeout -k 10 120 python3 -u tools/pair_stamps.py headline > "$out/pairs_headline.txt" 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/pair_stamps.py headline 0 > "$out/pairs_headline_t0.txt" 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/pair_stamps.py parity6d > "$out/pairs_parity6d.txt" 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps.txt" 2>&1
cat $out/*.txt
