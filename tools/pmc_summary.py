"""Per-kernel HBM traffic of the headline forward from rocprofv3 PMC passes.

Run on the GPU box (from the repo root):
    python tools/pmc_summary.py --tag r01
It runs the bench under rocprofv3 twice, once per counter (FETCH_SIZE and
WRITE_SIZE each need most of the TCC counter slots, so they get separate
passes, as MI355X_MICROARCH.md "rocprofv3 PMC slots" prescribes), plus one
kernel-trace/stats pass, and writes:
  profiles/pmc_headline.json  per-kernel {fetch_kb, write_kb, hbm_bytes_per_launch, ...}
  profiles/<tag>_kernel_stats.csv, profiles/<tag>_pmc_raw.csv
Correction applied (MI355X_MICROARCH.md "HBM"): on gfx950 FETCH_SIZE reports
half the bytes of a 16-byte-per-lane coalesced streaming read; the kernels'
bulk reads are 16 B/lane (LDS-DMA dwordx4) or 8 B/lane fragment loads, so the
reported fetch is doubled for the read side and flagged as an estimate.
"""

import argparse
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"cross_root_plan_kernel": "cross_root_kernel", "posterior_cov_kernel": "posterior_cov_kernel",
           "envelope_kernel": "envelope_kernel"}


def run(cmd, env=None):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True, cwd=REPO, env=env, timeout=600)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", default="r01")
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--collect", action="store_true",
                    help="only aggregate gpurun_out/pmc_<tag> (merged back from the box) into profiles/")
    args = ap.parse_args()
    out = os.path.join(REPO, "gpurun_out", f"pmc_{args.tag}")
    os.makedirs(out, exist_ok=True)
    env = dict(os.environ, TMPDIR="/tmp")
    bench = [sys.executable, "bench.py", "--steps", str(args.steps), "--warmup", "5", "--cpu-seconds", "0",
             "--profile-reps", "2"]
    if not args.collect:
        profile(out, env, bench)
    collect(args, out)


def profile(out, env, bench):
    run(["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", f"{out}/trace", "-o", "run", "--"]
        + bench, env)
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        run(["rocprofv3", "--pmc", ctr, "--output-format", "csv", "-d", f"{out}/{ctr}", "-o", "run", "--"] + bench,
            env)


def collect(args, out):
    agg = {}
    raw_rows = []
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        for f in glob.glob(f"{out}/{ctr}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                raw_rows.append(r)
                for k, name in KERNELS.items():
                    # the forward instantiation only (envelope_kernel<MAXL, M, GRAD=false, ...>)
                    if k in r["Kernel_Name"] and not (k == "envelope_kernel" and ", true," in r["Kernel_Name"]):
                        agg.setdefault(name, {}).setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    summary = {}
    for name, d in agg.items():
        fetch_kb = sum(d.get("FETCH_SIZE", [0])) / max(1, len(d.get("FETCH_SIZE", [1])))
        write_kb = sum(d.get("WRITE_SIZE", [0])) / max(1, len(d.get("WRITE_SIZE", [1])))
        summary[name] = {
            "fetch_kb_reported": fetch_kb,
            "write_kb_reported": write_kb,
            "hbm_bytes_per_launch": (2.0 * fetch_kb + write_kb) * 1024.0,
            "note": "FETCH_SIZE x2 (gfx950 wide-read correction, estimate) + WRITE_SIZE, KiB units -> bytes",
        }
    os.makedirs(os.path.join(REPO, "profiles"), exist_ok=True)
    json.dump(summary, open(os.path.join(REPO, "profiles", "pmc_headline.json"), "w"), indent=2)
    stats = glob.glob(f"{out}/trace/**/*kernel_stats.csv", recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(REPO, "profiles", f"{args.tag}_kernel_stats.csv"))
    with open(os.path.join(REPO, "profiles", f"{args.tag}_pmc_raw.csv"), "w", newline="") as fh:
        if raw_rows:
            w = csv.DictWriter(fh, fieldnames=list(raw_rows[0].keys()))
            w.writeheader()
            w.writerows(raw_rows)
    print(json.dumps(summary, indent=2))


if __name__ == "__main__":
    main()
