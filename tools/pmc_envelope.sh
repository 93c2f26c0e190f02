#!/bin/bash
# PMC counters + ablations of the headline forward (run on the GPU box from the repo root).
set -uo pipefail
out=gpurun_out/pmc_${1:-r01}
mkdir -p "$out"
export TMPDIR=/tmp
B="python3 bench.py --steps 50 --warmup 5 --cpu-seconds 0 --profile-reps 2"
for f in 0 1 2 3; do
  DKG_DEBUG_ENV_FLAGS=$f timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/abl$f" -o run -- $B > "$out/abl$f.json" 2>/dev/null || exit 1
done
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d "$out/pmc1" -o run -- $B > /dev/null 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_MFMA_F64 SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE --output-format csv -d "$out/pmc2" -o run -- $B > /dev/null 2>&1 || exit 1
echo done
