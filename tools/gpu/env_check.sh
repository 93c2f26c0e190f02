#!/bin/bash
# Envelope change check: parity-heavy GPU tests, phase stamps, bench (driver shape and default).
set -uo pipefail
out=${1:-gpurun_out/env}
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_gpu_epigraph.py \
  tests/test_gpu_fused.py tests/test_gpu_api.py -x -q --timeout 300 --timeout-method thread \
  > "$out/tests.log" 2>&1 || { tail -30 "$out/tests.log"; exit 1; }
tail -2 "$out/tests.log"
for wl in headline headline_nd; do
  timeout -k 10 120 python3 -u tools/kstamps.py $wl > "$out/kst_$wl.txt" 2>&1 || { tail -5 "$out/kst_$wl.txt"; exit 1; }
done
cat "$out/kst_headline.txt"
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --cpu-seconds 0 > "$out/b20.json" 2> "$out/b20.err" || { tail -5 "$out/b20.err"; exit 1; }
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 > "$out/b1024.json" 2> "$out/b1024.err" || { tail -5 "$out/b1024.err"; exit 1; }
python3 - "$out" <<'PY'
import json, sys
o = sys.argv[1]
for f in ("b20", "b1024"):
    d = json.load(open(f"{o}/{f}.json"))
    nd = d.get("nondegenerate") or {}
    st = d["roofline"]["stages"]
    print(f, round(d["value"] / 1e6, 2), "M/s", round(d["ms_per_step"] * 1e3, 2), "us/step; single",
          round(d["single_stream"]["ms_per_step"] * 1e3, 2), "us; nd", round(nd.get("value", 0) / 1e6, 2), "M/s env",
          round(nd.get("envelope_us", 0), 1), "us; stages", {k: round(v["avg_launch_us"], 2) for k, v in st.items()},
          "b1", d.get("latency_b1", {}) and round(d["latency_b1"]["median_us"], 1))
PY
