#!/bin/bash
# Envelope-kernel ablations (run on the GPU box from the repo root): kernel-trace
# stats of the bench for each DKG_DEBUG_ENV_FLAGS value given.
#   1: skip the hull (lines + a max)  2: atomic WG combine  8: skip the LDS staging  16: skip the line build
set -uo pipefail
tag=${1:-abl}; shift
out=gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
for f in "$@"; do
  DKG_DEBUG_ENV_FLAGS=$f timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/f$f" -o run -- \
    python3 bench.py --steps 100 --warmup 5 --cpu-seconds 0 --profile-reps 2 > "$out/f$f.json" 2>/dev/null || exit 1
  printf "flags=%s " "$f"; grep -h envelope "$out"/f$f/*kernel_stats.csv | cut -d, -f1,4
done
