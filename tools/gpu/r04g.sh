#!/bin/bash
# Covariance-kernel change: the GPU suite, then the variant A/B (tools/gpu/ab_variants.sh).
set -uo pipefail
out=${1:-gpurun_out/r04g}
mkdir -p "$out"
bash tools/gpu/tests.sh "$out" || exit 1
bash tools/gpu/ab_variants.sh "$out/ab"
