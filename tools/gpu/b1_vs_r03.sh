#!/bin/bash
# B = 1 value + gradient: this tree's latency breakdown and kernels (tools/gpu/b1.sh), then the round-3 build's probe.
set -uo pipefail
out=${1:-gpurun_out/b1cmp}
mkdir -p "$out"
bash tools/gpu/b1.sh "$out/cur" || exit 1
(cd .ab/f96856c && timeout -k 10 200 python3 -u tools/b1_probe.py) > "$out/b1_probe_r03.txt" 2>&1 || { tail -5 "$out/b1_probe_r03.txt"; exit 1; }
echo "== round-3 build"; grep -v amdgpu.ids "$out/b1_probe_r03.txt"
