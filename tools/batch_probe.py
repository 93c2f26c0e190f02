"""Forward batches per launch (dkg_plan_forward_batches): rate at the driver's shape and at long runs.

usage: python tools/batch_probe.py [--steps 20] [--reps 5]
For every (batches per launch G, streams) a region of `steps` headline forwards (B = 128 each) is timed
with HIP events after a synchronize, as bench.py times its region; also checks that the batched launch
writes the same bits as one forward_into per batch.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]

import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="headline")
    ap.add_argument("--steps", type=int, nargs="+", default=[20, 1024])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--groups", type=int, nargs="+", default=[1, 2, 4, 5, 10, 20, 32, 64])
    ap.add_argument("--streams", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--graph", type=int, default=1)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    w = WORKLOADS[args.workload]
    model, D, X0, W = make_problem(w)
    acq = DiscreteKnowledgeGradient(model, D, W, device=dev)
    B = w.B
    gmax = max(args.groups)
    # bit check: gmax distinct batches, one batched launch against one forward_into per batch
    Xs = torch.quasirandom.SobolEngine(w.d, scramble=True, seed=7).draw(gmax * B, dtype=torch.double).to(dev)
    big = acq._state.plan(acq._W, acq._target, gmax * B)
    one = acq._state.plan(acq._W, acq._target, B)
    kg_b = torch.empty(gmax * B, dtype=torch.double, device=dev)
    big.forward_batches_into(Xs, kg_b, B)
    kg_s = torch.empty_like(kg_b)
    for k in range(gmax):
        one.forward_into(Xs[k * B:(k + 1) * B], kg_s[k * B:(k + 1) * B])
    torch.cuda.synchronize()
    same = bool(torch.equal(kg_b, kg_s))
    print(json.dumps({"bits_equal": same, "batches": gmax, "kg_max": float(kg_b.max())}), flush=True)

    X = X0.to(dev).repeat(gmax, 1).contiguous()
    res = []
    for steps in args.steps:
        for G in args.groups:
            if steps % G:
                continue
            for ns in args.streams:
                units = steps // G
                if ns > units:
                    continue
                streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(ns - 1)]
                plans = [acq._state.plan(acq._W, acq._target, G * B) for _ in range(ns)]
                out = torch.empty(steps, B, dtype=torch.double, device=dev)
                xg = X[:G * B]

                def region():
                    main = streams[0]
                    for s in streams[1:]:
                        s.wait_stream(main)
                    for u in range(units):
                        i = u % ns
                        with torch.cuda.stream(streams[i]):
                            plans[i].forward_batches_into(xg, out[u * G:(u + 1) * G].view(-1), B)
                    for s in streams[1:]:
                        main.wait_stream(s)

                g = None
                if args.graph:
                    # one graph per stream of its units, launched side by side (bench.py --graph 2)
                    g = []
                    for i in range(ns):
                        gi = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(gi, stream=torch.cuda.Stream(dev), capture_error_mode="thread_local"):
                            for u in range(i, units, ns):
                                plans[i].forward_batches_into(xg, out[u * G:(u + 1) * G].view(-1), B)
                        g.append(gi)
                    for gi in g:
                        gi.replay()
                for _ in range(2):
                    region()
                torch.cuda.synchronize()
                ts = []
                for _ in range(args.reps):
                    torch.cuda.synchronize()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    t0 = time.perf_counter()
                    e0.record()
                    if g is None:
                        region()
                    else:
                        main = streams[0]
                        for s in streams[1:]:
                            s.wait_stream(main)
                        for i, gi in enumerate(g):
                            with torch.cuda.stream(streams[i]):
                                gi.replay()
                        for s in streams[1:]:
                            main.wait_stream(s)
                    e1.record()
                    torch.cuda.synchronize()
                    wall = time.perf_counter() - t0
                    ts.append(max(wall, e0.elapsed_time(e1) / 1e3))
                ts.sort()
                r = {"steps": steps, "G": G, "streams": ns, "graph": bool(g), "median_us": ts[len(ts) // 2] * 1e6,
                     "min_us": ts[0] * 1e6, "rate_M": steps * B / ts[len(ts) // 2] / 1e6}
                res.append(r)
                print(json.dumps(r), flush=True)
                del plans, g
    best = {}
    for r in res:
        k = r["steps"]
        if k not in best or r["rate_M"] > best[k]["rate_M"]:
            best[k] = r
    print(json.dumps({"best": best}))


if __name__ == "__main__":
    main()
