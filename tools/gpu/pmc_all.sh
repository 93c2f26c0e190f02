#!/bin/bash
# PMC passes (tools/pmc_passes.sh) for each benched workload at the launch shape of the driver's run
# (--steps 20, four streams: 5 forward batches per launch), aggregated into <out>/pmc_<workload>.json (copied
# into profiles/r05/).  The stress legs run one forward per launch (bench.py), so their passes use 1.
# usage: tools/gpu/pmc_all.sh <out> [workload[:fp32] ...]   (default: headline headline_nd stress)
set -uo pipefail
out=${1:-gpurun_out/pmc}; shift || true
wls=${*:-headline headline_nd stress}
for spec in $wls; do
  wl=${spec%%:*}; prec=fp64; tag=$wl
  [ "$spec" != "$wl" ] && { prec=${spec#*:}; tag=${wl}_$prec; }
  g=5; case $wl in stress*) g=1;; esac
  bash tools/pmc_passes.sh "$out/$tag" --workload "$wl" --precision "$prec" --batches-per-launch $g || exit 1
  python3 tools/pmc_report.py "$out/$tag" "$out/${tag}_report.json" "$out/pmc_${tag}.json" > "$out/${tag}_report.txt" || exit 1
done
ls -la "$out"
