#!/bin/bash
# PMC passes (tools/pmc_passes.sh) for each benched workload at the launch shape of the driver's run
# (--steps 20, two streams: 10 forward batches per launch), aggregated into <out>/pmc_<workload>.json (copied
# into profiles/r05/).  The stress leg runs one forward per launch (bench.py), so its passes use 1.
set -uo pipefail
out=${1:-gpurun_out/pmc}
for wl in headline headline_nd stress; do
  g=10; [ "$wl" = stress ] && g=1
  bash tools/pmc_passes.sh "$out/$wl" --workload "$wl" --batches-per-launch $g || exit 1
  python3 tools/pmc_report.py "$out/$wl" "$out/${wl}_report.json" "$out/pmc_${wl}.json" > "$out/${wl}_report.txt" || exit 1
done
ls -la "$out"
