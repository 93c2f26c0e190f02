#!/bin/bash
# B = 1 value + gradient: the latency breakdown (tools/b1_probe.py) and its kernels' statistics.
set -uo pipefail
out=${1:-gpurun_out/b1}
mkdir -p "$out"
timeout -k 10 200 python3 -u tools/b1_probe.py > "$out/b1_probe.txt" 2>&1 || { tail -5 "$out/b1_probe.txt"; exit 1; }
grep -v amdgpu.ids "$out/b1_probe.txt"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o b1 -- python3 tools/b1_kernels.py \
  > "$out/b1k.log" 2>&1 || { tail -5 "$out/b1k.log"; exit 1; }
cut -d, -f1-4,6,7 $(find "$out/prof" -name "*kernel_stats.csv") | head -12
for v in $(ls decoupled-kg_amd/dkg_amd/_native/ab/ 2>/dev/null | sed 's/libdkg_\(.*\)\.so/\1/'); do
  DKG_LIB=$GRAFT_REPO_ROOT/decoupled-kg_amd/dkg_amd/_native/ab/libdkg_$v.so timeout -k 10 200 python3 -u tools/b1_probe.py > "$out/b1_probe_$v.txt" 2>&1 || exit 1
  echo "== $v"; grep -v amdgpu.ids "$out/b1_probe_$v.txt"
  DKG_LIB=$GRAFT_REPO_ROOT/decoupled-kg_amd/dkg_amd/_native/ab/libdkg_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof_$v" -o b1 -- python3 tools/b1_kernels.py > "$out/b1k_$v.log" 2>&1 || exit 1
  cut -d, -f1,2,4 $(find "$out/prof_$v" -name "*kernel_stats.csv") | head -4
done
