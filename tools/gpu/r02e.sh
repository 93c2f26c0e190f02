#!/bin/bash
# walk_table + refilter: epigraph/parity tests, pair stamps, bench
set -uo pipefail
out=gpurun_out/r02e
mkdir -p "$out"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_epigraph.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > "$out/tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$out/tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -u tools/pair_stamps.py headline > "$out/pairs_headline.txt" 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/pair_stamps.py headline 0 > "$out/pairs_headline_t0.txt" 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps.txt" 2>&1 || exit $?
cat $out/pairs*.txt; grep -A6 "^envelope" $out/kstamps.txt
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$out/bench.json" | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['value'], d['single_stream'], d['roofline']['stages_us'], d['value_and_grad'])"
exit $rc
