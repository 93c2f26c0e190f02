"""Why the bench line's B = 1 figures exceed tools/b1_probe.py's: the bench interleaves three routes call by call
(value_and_grad_host, the eager plan call + two copies, forward() + autograd).  Medians per route for the bench's
loop and for variants that drop one route or disable Python's garbage collector.

Run on the GPU box from the repo root:  python tools/b1_interleave.py [calls]
"""
import gc
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]
import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
w = WORKLOADS["headline"]
model, D, X, W = make_problem(w)
acq = DiscreteKnowledgeGradient(model, D, W)
Xd = X.cuda().contiguous()
xh = Xd.cpu()
p1 = acq._plan_for(1, grad=True)
for i in range(10):
    p1.forward_grad(Xd[:1].contiguous())
    acq.value_and_grad_host(xh[i:i + 1])
    xa = xh[i:i + 1].unsqueeze(-2).requires_grad_(True)
    torch.autograd.grad(-acq(xa).sum(), xa)
torch.cuda.synchronize()


def med(ts):
    return round(sorted(ts)[len(ts) // 2] * 1e6, 1) if ts else None


def loop(vgh=True, eager=True, auto=True, inner=True):
    ts, te, ta = [], [], []
    for i in range(calls):
        x1 = xh[i % w.B:i % w.B + 1]
        if vgh:
            t0 = time.perf_counter()
            acq.value_and_grad_host(x1)
            ts.append(time.perf_counter() - t0)
        if eager:
            xd = Xd[i % w.B:i % w.B + 1].contiguous()
            t0 = time.perf_counter()
            kg1, g1 = p1.forward_grad(xd)
            kg1.cpu(), g1.cpu()
            te.append(time.perf_counter() - t0)
        if auto:
            if inner:
                t0 = time.perf_counter()
                xa = x1.unsqueeze(-2).requires_grad_(True)
            else:
                xa = x1.unsqueeze(-2).requires_grad_(True)
                t0 = time.perf_counter()
            loss = -acq(xa).sum()
            (ga,) = torch.autograd.grad(loss, xa)
            if inner:
                float(loss.detach()), ga.numpy()
            ta.append(time.perf_counter() - t0)
    return {"vgh": med(ts), "eager": med(te), "autograd": med(ta)}


print("bench loop          ", loop())
print("bench loop, no gc   ", (gc.disable(), loop(), gc.enable())[1])
print("no eager            ", loop(eager=False))
print("no vgh              ", loop(vgh=False))
print("autograd only       ", loop(vgh=False, eager=False))
print("autograd only, probe", loop(vgh=False, eager=False, inner=False))
print("vgh only            ", loop(eager=False, auto=False))
