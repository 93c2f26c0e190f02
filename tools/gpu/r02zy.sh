#!/bin/bash
# round-2 final bundle (catalog, fused value+gradient cross stage): full GPU suite, parity report, default bench (all legs), gloo 2-rank rehearsal,
# PMC passes + kernel trace, bench with the refreshed PMC
set -uo pipefail
out=gpurun_out/r02zy
mkdir -p "$out"
timeout -k 10 900 python3 -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > "$out/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -2 "$out/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/parity_report.py "$out/parity.json" > "$out/parity.log" 2>&1
rc=$?; echo "parity rc=$rc"; tail -3 "$out/parity.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/bench.err"; exit $rc; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(round(d['value']), d['single_stream'], {k: round(v['avg_launch_us'],2) for k,v in d['roofline']['stages'].items()}, d['nondegenerate']['value'], d['latency_b1']['median_us'], d['value_and_grad']['value'], d['cpu_baseline']['value'])"
timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/bench4k.json" 2>/dev/null || exit $?
timeout -k 10 120 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 20 --warmup 5 > "$out/bench20.json" 2>/dev/null || exit $?
python3 -c "import json; [print(f, round(json.load(open('$out/'+f))['value'])) for f in ('bench4k.json','bench20.json')]"
for sh in scalarisations candidates; do
  DKG_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --steps 512 --cpu-seconds 0 --nd-steps 0 --b1-calls 0 --grad-steps 0 --shard $sh > "$out/rehearsal_$sh.json" 2> "$out/rehearsal_$sh.err"
  rc=$?; echo "rehearsal $sh rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/rehearsal_$sh.err"; exit $rc; }
done
bash tools/pmc_passes.sh $out/pmc || exit $?
python3 tools/pmc_report.py $out/pmc $out/pmc_report.json $out/pmc_headline.json > /dev/null || exit $?
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --pmc $out/pmc_headline.json > "$out/bench_pmc.json" 2> "$out/bench_pmc.err" || exit $?
timeout -k 10 120 python3 -u tools/kstamps.py headline > "$out/kstamps.txt" 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/pair_stamps.py headline > "$out/pairs_headline.txt" 2>&1 || exit $?
timeout -k 10 120 python3 -u tools/pair_stamps.py headline_nd > "$out/pairs_nd.txt" 2>&1 || exit $?
timeout -k 10 200 python3 -u tools/b1_probe.py headline 300 > "$out/b1_probe.txt" 2>&1 || exit $?
echo done
