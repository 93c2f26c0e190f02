#!/bin/bash
# Build an A/B variant of libdkg.so with extra defines into dkg_amd/_native/ab/libdkg_<name>.so
# usage: tools/build_variant.sh <name> -DFOO=1 ...   (load it with DKG_LIB=...)
set -euo pipefail
name=$1; shift
cd "$(dirname "$0")/../decoupled-kg_amd"
mkdir -p build/ab_$name dkg_amd/_native/ab
pids=()
for f in csrc/*.hip; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I../include -Icsrc -Wno-unused-result -Wno-pass-failed "$@" \
    -c "$f" -o "build/ab_$name/$(basename "$f" .hip).o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared build/ab_$name/*.o -o dkg_amd/_native/ab/libdkg_$name.so
echo "dkg_amd/_native/ab/libdkg_$name.so"
