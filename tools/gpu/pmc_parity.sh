#!/bin/bash
# Round-4 PMC passes (headline, headline_nd, stress) and the parity report (profiles/r04_parity.json).
set -uo pipefail
out=${1:-gpurun_out/pmc_parity}
mkdir -p "$out"
timeout -k 10 600 python3 -u tools/parity_report.py "$out/r04_parity.json" > "$out/parity.log" 2>&1 || { tail -20 "$out/parity.log"; exit 1; }
tail -12 "$out/parity.log"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu/pmc_all.sh "$out/pmc"
