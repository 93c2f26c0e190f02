#!/bin/bash
# Where posterior_cov_big_kernel's waves wait at 5 headline batches per launch: one PMC pass of SQ wait / LDS
# counters and one of TA busy over tools/stage_probe.py (the stage launched back to back).
set -uo pipefail
out=${1:-gpurun_out/r06_covwait}
mkdir -p "$out"
export TMPDIR=/tmp
P="python3 tools/stage_probe.py --workload headline --groups 5"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_VMEM --output-format csv -d "$out/sq" -o run -- $P > "$out/sq.log" 2>&1 || { tail -5 "$out/sq.log"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d "$out/ta" -o run -- $P > "$out/ta.log" 2>&1 || { tail -5 "$out/ta.log"; exit 1; }
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for tag in ("sq", "ta"):
    f = glob.glob(f"{out}/{tag}/**/*counter_collection.csv", recursive=True)
    if not f:
        print(tag, "no counter file"); continue
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        name = r.get("Kernel_Name", "")
        for k in ("posterior_cov_big_kernel", "envelope_kernel", "cross_big_kernel"):
            if k in name:
                acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(f"{tag} {k:28s} {c:26s} per dispatch {sum(v) / len(v):.4g}  (n={len(v)})")
PY
