#!/bin/bash
# round-2 measurement bundle: full default bench (all legs, CPU baseline), PMC passes, kernel trace
set -uo pipefail
out=gpurun_out/r02zf
mkdir -p "$out"
timeout -k 10 500 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json; d=json.load(open('$out/bench.json')); print(round(d['value']), d['single_stream'], {k: round(v['avg_launch_us'],2) for k,v in d['roofline']['stages'].items()}, d['nondegenerate']['value'], d['latency_b1'], d['value_and_grad'], d['cpu_baseline'])"
bash tools/pmc_passes.sh $out/pmc || exit $?
python3 tools/pmc_report.py $out/pmc $out/pmc_report.json $out/pmc_headline.json || exit $?
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --pmc $out/pmc_headline.json > "$out/bench_pmc.json" 2> "$out/bench_pmc.err" || exit $?
