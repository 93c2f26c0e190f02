#!/bin/bash
# rocprofv3 PMC passes over a short headline bench (GPU box, repo root).
# usage: tools/pmc_passes.sh <outdir> [extra bench args]
# One pass per counter group (MI355X_MICROARCH.md "rocprofv3 PMC slots": <= 8 SQ,
# FETCH_SIZE and WRITE_SIZE in separate passes); aggregate with tools/pmc_report.py.
set -uo pipefail
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --profile-reps 2 --grad-steps 0 --b1-calls 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --streams 1 --graph 0 $*"
timeout -s KILL 60 rocprofv3 -L > "$out/counters_list.txt" 2>&1 || true
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$out/$name" -o run -- $B > "$out/$name.log" 2>&1
  local rc=$?
  echo "pass $name rc=$rc"
  return $rc
}
pass sqA SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 || exit 1
pass sqB SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS || exit 1
pass fetch FETCH_SIZE || exit 1
pass write WRITE_SIZE || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- $B > "$out/trace.log" 2>&1
echo "trace rc=$?"
