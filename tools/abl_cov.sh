#!/bin/bash
set -uo pipefail
export TMPDIR=/tmp
for f in 0 1 2 4 7; do
  out=gpurun_out/ablcov/f$f
  mkdir -p $out
  DKG_DEBUG_COV_FLAGS=$f timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 --profile-reps 2 > /dev/null 2>&1 || exit 1
  echo "flags $f: $(grep posterior_cov $(find $out -name '*kernel_stats.csv' | head -1) | cut -d, -f4)"
done
