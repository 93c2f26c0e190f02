#!/bin/bash
# Per-wave instruction mix of the envelope kernel (PMC counters, two passes).
# usage (GPU box, repo root): tools/pmc_env_insts.sh <tag>
set -uo pipefail
out=gpurun_out/${1:-pmcins}
mkdir -p "$out"
export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --profile-reps 1 --grad-steps 0"
for f in 0; do
  DKG_DEBUG_ENV_FLAGS=$f timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH --output-format csv -d "$out/a$f" -o run -- $B > /dev/null 2>&1 || exit 1
  DKG_DEBUG_ENV_FLAGS=$f timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --output-format csv -d "$out/b$f" -o run -- $B > /dev/null 2>&1 || exit 1
done
python3 - "$out" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
for f in (0,):
    agg = collections.defaultdict(list)
    for p in (f"{out}/a{f}", f"{out}/b{f}"):
        for fn in glob.glob(p + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(fn)):
                if "envelope" in r["Kernel_Name"]:
                    agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    avg = {k: sum(v) / len(v) for k, v in agg.items()}
    w = avg.get("SQ_WAVES", 1)
    print(f"flags={f} waves={w:.0f} " + " ".join(f"{k[3:]}={v / w:.0f}" for k, v in sorted(avg.items()) if k != "SQ_WAVES"))
PY
