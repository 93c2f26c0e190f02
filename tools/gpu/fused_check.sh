#!/bin/bash
# Fused one-launch forward: hand-off tests, then the bench at the driver's shape and the default, fused vs split.
set -uo pipefail
out=${1:-gpurun_out/fused}
mkdir -p "$out"
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fused.py -x -v --timeout 120 --timeout-method thread \
  > "$out/fused_tests.log" 2>&1 || { tail -30 "$out/fused_tests.log"; exit 1; }
tail -3 "$out/fused_tests.log"
for mode in fused split; do
  env_fused=1; [ "$mode" = split ] && env_fused=0
  DKG_FUSED=$env_fused timeout -k 10 240 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 \
    > "$out/b20_$mode.json" 2> "$out/b20_$mode.err" || { tail -5 "$out/b20_$mode.err"; exit 1; }
  DKG_FUSED=$env_fused timeout -k 10 240 python3 -u bench.py --cpu-seconds 0 --grad-steps 0 --b1-calls 0 \
    > "$out/b1024_$mode.json" 2> "$out/b1024_$mode.err" || { tail -5 "$out/b1024_$mode.err"; exit 1; }
done
python3 - "$out" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("b20_fused", "b20_split", "b1024_fused", "b1024_split"):
    d = json.load(open(f"{o}/{f}.json"))
    nd = d.get("nondegenerate") or {}
    print(f, round(d["value"] / 1e6, 2), "M/s", round(d["ms_per_step"] * 1e3, 2), "us/step single",
          round(d["single_stream"]["ms_per_step"] * 1e3, 2), "us  nd", round(nd.get("value", 0) / 1e6, 2))
PY
