#!/bin/bash
# full GPU suite (new: api, sharded HIP), bench with the new legs, gloo 2-rank rehearsal
set -uo pipefail
out=gpurun_out/r02j
mkdir -p "$out"
timeout -k 10 900 python3 -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > "$out/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 "$out/gpu_tests.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py > "$out/bench.json" 2> "$out/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/bench.err"; exit $rc; }
python3 -c "import json; d=json.load(open('$out/bench.json')); print(d['value'], d['single_stream'], {k: v['avg_launch_us'] for k, v in d['roofline']['stages'].items()}, d['roofline']['frac'], d['latency_b1'], d['nondegenerate']['value'], d['nondegenerate']['envelope_us'], d['cpu_baseline']['cores'], d['cpu_baseline']['cpu_model'])"
for sh in scalarisations candidates; do
  DKG_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --steps 512 --cpu-seconds 0 --nd-steps 0 --b1-calls 0 --grad-steps 0 --shard $sh > "$out/rehearsal_$sh.json" 2> "$out/rehearsal_$sh.err"
  rc=$?; echo "rehearsal $sh rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/rehearsal_$sh.err"; exit $rc; }
done
