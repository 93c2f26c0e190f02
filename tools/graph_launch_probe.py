"""Short-run launch cost: per-stream HIP graphs (bench.py --graph 2) launched one after another by torch,
one after another by hipGraphLaunch, or by one host thread per stream at once (tools/ubench/graphpar.hip).

Run on the GPU box from the repo root (after `make -C tools/ubench libgraphpar.so`):
    python tools/graph_launch_probe.py [forwards per run ...]
Prints, per mode and run length: median wall time of a run (stream fork, the launches, join, sync) per forward,
and the median host span of the launches.
"""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]
import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402

lib = ctypes.CDLL(os.path.join(REPO, "tools", "ubench", "libgraphpar.so"))
lib.graphpar_launch.restype = ctypes.c_double
lib.graphpar_launch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]

w = WORKLOADS["headline"]
model, D, X, W = make_problem(w)
acq = DiscreteKnowledgeGradient(model, D, W)
dev = torch.device("cuda")
Xd = X.to(dev).contiguous()
ns = 4
plans = [acq._plan_for(w.B)] + [acq._state.plan(acq._W, acq._target, w.B) for _ in range(ns - 1)]
streams = [torch.cuda.Stream() for _ in range(ns)]


def med(v):
    v = sorted(v)
    return v[len(v) // 2]


for E in [int(a) for a in sys.argv[1:]] or [20, 64, 256]:
    outs = torch.zeros(E, w.B, dtype=torch.double, device=dev)
    gs = []
    for i in range(ns):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=streams[i]):
            for r in range(i, E, ns):
                plans[i].forward_into(Xd, outs[r])
        gs.append(g)
    torch.cuda.synchronize()
    execs = (ctypes.c_void_p * ns)(*[g.raw_cuda_graph_exec() for g in gs])
    sps = (ctypes.c_void_p * ns)(*[s.cuda_stream for s in streams])
    calls = (ctypes.c_double * ns)()
    ref = None
    for mode in ("torch", "hip_seq", "hip_threads"):
        walls, spans = [], []
        for rep in range(25):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            main = torch.cuda.current_stream()
            for s in streams:
                s.wait_stream(main)
            if mode == "torch":
                h0 = time.perf_counter()
                for i in range(ns):
                    with torch.cuda.stream(streams[i]):
                        gs[i].replay()
                span = (time.perf_counter() - h0) * 1e6
            else:
                span = lib.graphpar_launch(execs, sps, ns, 1 if mode == "hip_threads" else 0, calls)
            for s in streams:
                main.wait_stream(s)
            torch.cuda.synchronize()
            if rep >= 5:
                walls.append(time.perf_counter() - t0)
                spans.append(span)
        if ref is None:
            ref = outs.clone()
        same = torch.equal(outs, ref)
        print(f"E {E:4d} {mode:12s}: wall {med(walls) / E * 1e6:7.2f} us/forward ({med(walls) * 1e6:8.1f} us/run), "
              f"launch span {med(spans):7.1f} us, last calls {[round(c, 1) for c in calls]}, same {same}", flush=True)
