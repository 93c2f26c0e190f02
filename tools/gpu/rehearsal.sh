#!/bin/bash
# The driver's N > 1 command shape over 2 ranks on this box's one GPU (gloo: RCCL will not put two ranks on
# one device), then the parity report.
set -uo pipefail
out=${1:-gpurun_out/reh}
mkdir -p "$out"
for shard in scalarisations candidates; do
  DKG_BENCH_BACKEND=gloo timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 2 --steps 20 --warmup 5 --shard $shard \
    > "$out/gloo2_$shard.json" 2> "$out/gloo2_$shard.err" || { tail -20 "$out/gloo2_$shard.err"; exit 1; }
  python3 tools/bench_summary.py "$out/gloo2_$shard.json"
done
timeout -k 10 600 python3 -u tools/parity_report.py "$out/r03_parity.json" > "$out/parity.log" 2>&1 || { tail -20 "$out/parity.log"; exit 1; }
tail -3 "$out/parity.log"
