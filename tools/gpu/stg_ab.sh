#!/bin/bash
# Staged streaming envelope variants (tools/build_variant.sh builds under decoupled-kg_amd/dkg_amd/_native/ab/):
# phase stamps and the envelope launch span at the stress shape, per variant.
set -uo pipefail
out=${1:-gpurun_out/stg}; shift
mkdir -p "$out"
for v in "$@"; do
  lib=$PWD/decoupled-kg_amd/dkg_amd/_native/ab/libdkg_$v.so
  DKG_LIB=$lib timeout -k 10 120 python3 -u tools/stg_stamps.py stress > "$out/stg_$v.txt" 2>&1 || { tail -5 "$out/stg_$v.txt"; exit 1; }
  DKG_LIB=$lib timeout -k 10 120 python3 -u tools/kstamps.py stress > "$out/kst_$v.txt" 2>&1 || { tail -5 "$out/kst_$v.txt"; exit 1; }
  echo "== $v"; grep -v amdgpu.ids "$out/stg_$v.txt"; grep -A2 "^envelope" "$out/kst_$v.txt"
done
