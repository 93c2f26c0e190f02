#!/bin/bash
# A/B of earlier commits' builds (git worktrees under .ab/, built in-tree) against the working tree: the driver-shape
# bench (20 steps) and the 1024-step line, interleaved, envelope-free legs skipped.
set -uo pipefail
out=${1:-gpurun_out/ab}
mkdir -p "$out"
root=$GRAFT_REPO_ROOT
opts="--cpu-seconds 0 --grad-steps 0 --b1-calls 0 --nd-steps 0 --stress-steps 0 --prep-reps 0"
for rep in 1 2; do
  for v in cur $(ls .ab); do
    d=$root; [ "$v" != cur ] && d=$root/.ab/$v
    (cd "$d" && timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 $opts) > "$out/b20_${v}_$rep.json" 2> "$out/b20_${v}_$rep.err" || { tail -5 "$out/b20_${v}_$rep.err"; exit 1; }
    (cd "$d" && timeout -k 10 200 python3 -u bench.py --steps 1024 --warmup 50 $opts) > "$out/b1k_${v}_$rep.json" 2> "$out/b1k_${v}_$rep.err" || { tail -5 "$out/b1k_${v}_$rep.err"; exit 1; }
  done
done
for f in "$out"/*.json; do python3 -c "import json,sys; d=json.load(open(sys.argv[1])); st=d['roofline']['stages']; print(sys.argv[1].split('/')[-1], round(d['value']/1e6,2), round(d['single_stream']['ms_per_step']*1e3,2), [round(v['avg_launch_us'],2) for v in st.values()])" "$f"; done
