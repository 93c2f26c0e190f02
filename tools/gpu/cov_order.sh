#!/bin/bash
# Big covariance blocks' order (DKG_COV_ORDER, block_order): L2 fetch / write bytes per launch of
# posterior_cov_big_kernel (FETCH_SIZE x2 read-side correction, WRITE_SIZE; MI355X_MICROARCH.md) and the
# covariance stage time, stress (one forward per launch) and headline (10 batches per launch).
set -uo pipefail
out=${1:-gpurun_out/co}
mkdir -p "$out"
export TMPDIR=/tmp
B="python3 bench.py --steps 20 --warmup 2 --cpu-seconds 0 --profile-reps 2 --grad-steps 0 --b1-calls 0 --nd-steps 0 --stress-steps 0 --stress32-steps 0 --streams 1 --graph 0"
for wl in ${WLS:-stress headline}; do
  g=10; [ "$wl" = stress ] && g=1
  for o in ${ORDERS:-0 1 2}; do
    for c in FETCH_SIZE WRITE_SIZE; do
      DKG_COV_ORDER=$o timeout -s KILL 90 rocprofv3 --pmc $c --output-format csv -d "$out/${wl}_o${o}_$c" -o run -- $B --workload $wl --batches-per-launch $g > "$out/${wl}_o${o}_$c.log" 2>&1 || { echo "pass $wl $o $c failed"; tail -5 "$out/${wl}_o${o}_$c.log"; exit 1; }
    done
    python3 - "$out" "$wl" "$o" <<'PY'
import csv, glob, sys, json
out, wl, o = sys.argv[1:4]
res = {}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = []
    for f in glob.glob(f"{out}/{wl}_o{o}_{c}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "posterior_cov_big_kernel" in r["Kernel_Name"] and r["Counter_Name"] == c:
                g = int(float(r.get("Grid_Size") or 0))
                rows.append((g, r.get("Dispatch_Id"), float(r["Counter_Value"])))
    gmax = max(g for g, _, _ in rows)
    per = {}
    for g, dsp, v in rows:
        if g == gmax:
            per[dsp] = per.get(dsp, 0.0) + v
    vals = list(per.values())
    res[c] = sum(vals) / len(vals) * 1024 * (2 if c == "FETCH_SIZE" else 1)
print(json.dumps({"workload": wl, "order": int(o), "fetch_MB_x2": res["FETCH_SIZE"] / 1e6, "write_MB": res["WRITE_SIZE"] / 1e6}))
PY
    DKG_COV_ORDER=$o timeout -k 10 120 python3 -u tools/stage_probe.py --workload $wl --groups $g > "$out/${wl}_o${o}_stage.txt" 2>&1 || { tail -5 "$out/${wl}_o${o}_stage.txt"; exit 1; }
    grep '^{' "$out/${wl}_o${o}_stage.txt"
  done
done
