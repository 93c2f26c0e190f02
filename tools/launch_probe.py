"""Where the forwards-in-flight throughput goes: host launch cost vs GPU time.

Modes: 0 plain launches, 1 one graph forked over the streams, 2 one single-stream
graph per stream replayed side by side.

Run on the GPU box from the repo root:  python tools/launch_probe.py
For one headline plan: E = 256 forwards captured as one HIP graph over 1 or 4
streams, replayed R times; prints the host time spent inside replay() and the
GPU time (events) per forward, and the same for plain (uncaptured) launches.
A host time per forward close to the GPU time means the launches, not the
kernels, bound the throughput.
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]
import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402

w = WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "headline"]
model, D, X, W = make_problem(w)
acq = DiscreteKnowledgeGradient(model, D, W)
dev = torch.device("cuda")
Xd = X.to(dev).contiguous()
E, R = 256, 8


def probe(ns, graph):
    plans = [acq._plan_for(w.B)] + [acq._state.plan(acq._W, acq._target, w.B) for _ in range(ns - 1)]
    main = torch.cuda.current_stream()
    streams = [main] + [torch.cuda.Stream() for _ in range(ns - 1)]
    outs = torch.zeros(E, w.B, dtype=torch.double, device=dev)

    def issue():
        for s in streams[1:]:
            s.wait_stream(torch.cuda.current_stream())
        cs = torch.cuda.current_stream()
        lanes = [cs] + streams[1:]
        for r in range(E):
            with torch.cuda.stream(lanes[r % ns]):
                plans[r % ns].forward_into(Xd, outs[r])
        for s in lanes[1:]:
            cs.wait_stream(s)

    issue()
    torch.cuda.synchronize()
    if graph == 2:
        # one single-stream graph per stream (rows r = i mod ns), replayed side by side
        gs = []
        for i in range(ns):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=streams[i] if i else torch.cuda.Stream()):
                for r in range(i, E, ns):
                    plans[i].forward_into(Xd, outs[r])
            gs.append(g)
        torch.cuda.synchronize()

        def run():
            cs = torch.cuda.current_stream()
            for s in streams[1:]:
                s.wait_stream(cs)
            for i in range(ns):
                with torch.cuda.stream(streams[i]):
                    gs[i].replay()
            for s in streams[1:]:
                cs.wait_stream(s)
    elif graph:
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            issue()
        torch.cuda.synchronize()
        run = g.replay
    else:
        run = issue
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host = 0.0
    e0.record()
    for _ in range(R):
        t = time.perf_counter()
        run()
        host += time.perf_counter() - t
    e1.record()
    t = time.perf_counter()
    torch.cuda.synchronize()
    tail = time.perf_counter() - t
    gpu = e0.elapsed_time(e1) / 1e3
    n = E * R
    print(f"streams {ns} graph {int(graph)}: host in launch {host / n * 1e6:7.2f} us/forward, "
          f"GPU {gpu / n * 1e6:7.2f} us/forward, sync tail {tail * 1e3:7.2f} ms", flush=True)


modes = [int(v) for v in os.environ.get("PROBE_MODES", "0,1,2").split(",")]
for ns in [int(v) for v in os.environ.get("PROBE_STREAMS", "1,4").split(",")]:
    for graph in modes:
        probe(ns, graph)
