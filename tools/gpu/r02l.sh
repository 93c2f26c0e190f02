#!/bin/bash
# mov_dpp + grouped compaction: tests, stamps, bench, PMC passes
set -uo pipefail
out=gpurun_out/r02l
mkdir -p "$out"
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_epigraph.py tests/test_gpu_parity.py tests/test_gpu_grad.py -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$out/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/pair_stamps.py headline > "$out/pairs_headline.txt" 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps.txt" 2>&1 || exit $?
head -8 $out/pairs*.txt; grep -A6 "^envelope" $out/kstamps.txt
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 -c "import json,sys; d=json.load(open('$out/bench.json')); print(d['value'], d['single_stream'], d['roofline']['stages_us'], d['value_and_grad'])"
bash tools/pmc_passes.sh $out/pmc || exit $?
python3 tools/pmc_report.py $out/pmc $out/pmc_report.json
