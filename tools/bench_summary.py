"""One-line summaries of bench.py JSON lines:  python tools/bench_summary.py a.json [b.json ...]"""
import json
import sys

for f in sys.argv[1:]:
    # the last JSON line of the file (gloo and torchrun may print other lines to stdout)
    d = json.loads([ln for ln in open(f) if ln.startswith("{")][-1])
    nd = d.get("nondegenerate") or {}
    st = d.get("stress") or {}
    b1 = d.get("latency_b1") or {}
    r = d["roofline"]
    print(f, {"M/s": round(d["value"] / 1e6, 2), "us/step": round(d["ms_per_step"] * 1e3, 2),
              "single_us": round((d.get("single_stream") or {}).get("ms_per_step", 0) * 1e3, 2),
              "nd M/s": round(nd.get("value", 0) / 1e6, 2), "nd env us": round(nd.get("envelope_us", 0), 1),
              "stress K/s": round(st.get("value", 0) / 1e3, 1), "stress ms": round(st.get("ms_per_step", 0), 3),
              "stress stages": {k: round(v["avg_launch_us"], 1) for k, v in (st.get("stages") or {}).items()},
              "stages": {k: round(v["avg_launch_us"], 2) for k, v in r["stages"].items()},
              "roof": (r["kernel"], round(r["frac"], 4), r.get("valu_busy_frac")),
              "b1": round(b1.get("median_us", 0), 1), "b1 autograd": round((b1.get("autograd_route") or {}).get("median_us", 0), 1),
              "exposed_ms": (d.get("per_rank") or {}).get("exposed_collective_ms"),
              "prep_ms": round((d.get("state_prep") or {}).get("ms_median", 0), 3),
              "cpu": (d.get("cpu_baseline") or {}).get("value")})
