#!/bin/bash
# PMC passes (tools/pmc_passes.sh) for each benched workload, aggregated into <out>/pmc_<workload>.json (copied into profiles/r04/).
set -uo pipefail
out=${1:-gpurun_out/pmc}
for wl in headline headline_nd stress; do
  bash tools/pmc_passes.sh "$out/$wl" --workload "$wl" || exit 1
  python3 tools/pmc_report.py "$out/$wl" "$out/${wl}_report.json" "$out/pmc_${wl}.json" > "$out/${wl}_report.txt" || exit 1
done
ls -la "$out"
