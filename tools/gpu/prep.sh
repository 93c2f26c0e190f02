#!/bin/bash
# State preparation: its tests, the kernel statistics of tools/prep_kernels.py, the bench leg alone.
set -uo pipefail
out=${1:-gpurun_out/prep}
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_state.py tests/test_gpu_api.py -m gpu -x -q --timeout 120 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -1 "$out/tests.log"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/prof" -o prep -- python3 tools/prep_kernels.py \
  > "$out/prep.log" 2>&1 || { tail -5 "$out/prep.log"; exit 1; }
cut -d, -f1-4 $(find "$out/prof" -name "*kernel_stats.csv") | head -14
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 --grad-steps 0 --b1-calls 0 --nd-steps 0 --stress-steps 0 \
  --prep-reps 9 > "$out/b.json" 2> "$out/b.err" || { tail -5 "$out/b.err"; exit 1; }
python3 -c "import json; print(json.load(open('$out/b.json'))['state_prep'])"
for v in $(ls decoupled-kg_amd/dkg_amd/_native/ab/ 2>/dev/null | sed 's/libdkg_\(.*\)\.so/\1/'); do
  DKG_LIB=$GRAFT_REPO_ROOT/decoupled-kg_amd/dkg_amd/_native/ab/libdkg_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats \
    --output-format csv -d "$out/prof_$v" -o prep -- python3 tools/prep_kernels.py > "$out/prep_$v.log" 2>&1 || exit 1
  echo "== variant $v"; cut -d, -f1-4 $(find "$out/prof_$v" -name "*kernel_stats.csv") | head -4
done
