#!/bin/bash
# extremes: T's tie first, chord ends after the flat test
set -uo pipefail
out=gpurun_out/r02v
mkdir -p "$out"
timeout -k 10 120 tools/ubench/env_phases > "$out/phases.txt" 2>&1 || exit $?
head -4 "$out/phases.txt"; grep -E "ends|tie" "$out/phases.txt"
timeout -k 10 600 python3 -u -m pytest tests -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$out/tests.log"; [ $rc -eq 0 ] || exit $rc
for v in 2 1; do
  export DKG_ENV_SPLIT=$v
  timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 > "$out/bench_s$v.json" 2> "$out/bench_s$v.err" || exit $?
  python3 -c "import json; d=json.load(open('$out/bench_s$v.json')); print('split $v', d['value'], d['single_stream']['value'], {k: round(v['avg_launch_us'],2) for k,v in d['roofline']['stages'].items()}, d['nondegenerate']['value'], round(d['nondegenerate']['envelope_us'],2))"
  timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/bench4k_s$v.json" 2>/dev/null || exit $?
  python3 -c "import json; d=json.load(open('$out/bench4k_s$v.json')); print('split $v 4096 steps', d['value'])"
done
unset DKG_ENV_SPLIT
timeout -k 10 120 python3 -u tools/pair_stamps.py headline > "$out/pairs_headline.txt" 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps.txt" 2>&1 || exit $?
cat "$out/pairs_headline.txt"; tail -6 "$out/kstamps.txt"
