#!/bin/bash
# bench with per-stream graphs launched by hipGraphLaunch: driver's short run, default, 4096 steps, gloo rehearsal
set -uo pipefail
out=gpurun_out/r02zv
mkdir -p "$out"
for i in 1 2 3; do
  timeout -k 10 200 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > "$out/b20_$i.json" 2> "$out/b20_$i.err" || { tail -5 "$out/b20_$i.err"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/b20_$i.json')); print('steps20', round(d['value']), round(d['ms_per_step']*1e3,2), d['host_launch_us_per_step'], d['latency_b1']['median_us'], d['latency_b1']['eager_two_copies_median_us'])"
done
timeout -k 10 300 python3 -u bench.py --cpu-seconds 0 > "$out/bench.json" 2> "$out/bench.err" || { tail -5 "$out/bench.err"; exit 1; }
timeout -k 10 200 python3 -u bench.py --cpu-seconds 0 --b1-calls 0 --grad-steps 0 --nd-steps 0 --steps 4096 > "$out/bench4k.json" 2>/dev/null || exit 1
python3 -c "import json; [print(f, round(json.load(open('$out/'+f))['value']), json.load(open('$out/'+f))['host_launch_us_per_step']) for f in ('bench.json','bench4k.json')]"
DKG_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29533 bench.py --gpus 2 --steps 512 --cpu-seconds 0 --nd-steps 0 --b1-calls 0 --grad-steps 0 > "$out/rehearsal.json" 2> "$out/rehearsal.err"
rc=$?; echo "rehearsal rc=$rc"; [ $rc -eq 0 ] || { tail -20 "$out/rehearsal.err"; exit $rc; }
