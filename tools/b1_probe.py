"""Where the B = 1 value+gradient latency goes (the reference's optimize_acqf call shape, bo_loop.py:127-129).

Run on the GPU box from the repo root:  python tools/b1_probe.py [workload] [calls]
Prints median microseconds per call for:
  launch   -- host time of the C call alone (3 launches), no sync
  device   -- back-to-back calls, HIP events on the stream (device-bound per-call time)
  bench    -- forward_grad + kg.cpu() + dkg.cpu() (bench.py's latency_b1 leg)
  fused    -- forward_grad_host(): one pinned H2D, the C call, one pinned D2H of [kg, dkg], one event sync
  graph    -- the same with the three launches replayed from a captured HIP graph
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]
import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402


def med(ts):
    ts = sorted(ts)
    return round(ts[len(ts) // 2] * 1e6, 1)


w = WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "headline"]
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 200
model, D, X, W = make_problem(w)
acq = DiscreteKnowledgeGradient(model, D, W)
p1 = acq._plan_for(1, grad=True)
Xd = X.cuda().contiguous()
xs = [Xd[i % w.B:i % w.B + 1].contiguous() for i in range(calls)]
xh = [x.cpu() for x in xs]
for i in range(10):
    p1.forward_grad(xs[i])
torch.cuda.synchronize()

res = {}
ts = []
for i in range(calls):
    t0 = time.perf_counter()
    p1.forward_grad(xs[i])
    ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
res["launch"] = med(ts)

e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for i in range(calls):
    p1.forward_grad(xs[i])
e1.record()
torch.cuda.synchronize()
res["device"] = round(e0.elapsed_time(e1) * 1e3 / calls, 1)

ts = []
for i in range(calls):
    t0 = time.perf_counter()
    kg, g = p1.forward_grad(xs[i])
    kg.cpu(), g.cpu()
    ts.append(time.perf_counter() - t0)
res["bench"] = med(ts)

# the round trip's parts: the C call + stream sync; + a pinned H2D copy of x first; + a pinned D2H copy after
stream = torch.cuda.current_stream()
hx = torch.empty(w.d, dtype=torch.double).pin_memory()
hout = torch.empty(1 + w.d, dtype=torch.double).pin_memory()
dout = torch.empty(1 + w.d, dtype=torch.double, device="cuda")
dx = torch.empty(1, w.d, dtype=torch.double, device="cuda")
for name, h2d, d2h in (("sync_only", False, False), ("h2d+sync", True, False), ("d2h+sync", False, True),
                       ("h2d+d2h+sync", True, True)):
    ts = []
    for i in range(calls):
        t0 = time.perf_counter()
        if h2d:
            dx.copy_(hx.view(1, w.d), non_blocking=True)
            kg, g = p1.forward_grad(dx)
        else:
            kg, g = p1.forward_grad(xs[i])
        if d2h:
            hout.copy_(dout, non_blocking=True)
        stream.synchronize()
        ts.append(time.perf_counter() - t0)
    res[name] = med(ts)
# the kernel-argument entry alone: without and with the pinned output written by the envelope kernel
from dkg_amd import _lib  # noqa: E402
lib = _lib.load()
p1._host_buffers(w.d)
xc = [x.cpu().contiguous() for x in xs]
kgb = torch.empty(1, dtype=torch.double, device="cuda")
dkgb = torch.empty(1, w.d, dtype=torch.double, device="cuda")
outp = torch.empty(1 + w.d, dtype=torch.double).pin_memory()
sptr = torch.cuda.current_stream().cuda_stream
for name, hout in (("hostx+sync", 0), ("hostx+hout+sync", outp.data_ptr())):
    ts = []
    for i in range(calls):
        t0 = time.perf_counter()
        lib.dkg_plan_forward_grad_hostx(p1.host, p1._dev_ptr, xc[i].data_ptr(), dx.data_ptr(), 1, kgb.data_ptr(),
                                        dkgb.data_ptr(), hout, sptr)
        stream.synchronize()
        ts.append(time.perf_counter() - t0)
    res[name] = med(ts)
# host overhead of the pieces alone
ts = []
for i in range(calls):
    t0 = time.perf_counter()
    torch.cuda.current_stream()
    ts.append(time.perf_counter() - t0)
res["current_stream_call"] = med(ts)
ts = []
for i in range(calls):
    t0 = time.perf_counter()
    with torch.cuda.device(0):
        pass
    ts.append(time.perf_counter() - t0)
res["device_ctx"] = med(ts)
ts = []
for i in range(calls):
    xa = xh[i].unsqueeze(-2).requires_grad_(True)
    t0 = time.perf_counter()
    loss = -acq(xa).sum()
    (ga,) = torch.autograd.grad(loss, xa)
    ts.append(time.perf_counter() - t0)
res["autograd_route"] = med(ts)
ts = []
for i in range(calls):
    t0 = time.perf_counter()
    acq.value_and_grad_host(xh[i])
    ts.append(time.perf_counter() - t0)
res["value_and_grad_host"] = med(ts)


class _Trivial(torch.autograd.Function):  # the same autograd call shape with no device work: torch's own cost
    @staticmethod
    def forward(ctx, X, a):
        ctx.save_for_backward(X)
        return X.detach().sum(-1).reshape(X.shape[:-2])

    @staticmethod
    def backward(ctx, g):
        (X,) = ctx.saved_tensors
        return torch.ones_like(X), None


ts = []
for i in range(calls):
    xa = xh[i].unsqueeze(-2).requires_grad_(True)
    t0 = time.perf_counter()
    loss = -_Trivial.apply(xa, None).sum()
    (ga,) = torch.autograd.grad(loss, xa)
    ts.append(time.perf_counter() - t0)
res["autograd_floor_no_device"] = med(ts)

ref = [p1.forward_grad(xs[i]) for i in range(8)]
ref = [(a.cpu(), b.cpu()) for a, b in ref]
if hasattr(p1, "forward_grad_host"):
    for graph in (False, True):
        for i in range(10):
            p1.forward_grad_host(xh[i], graph=graph)
        ok = all(torch.equal(p1.forward_grad_host(xh[i], graph=graph)[0], ref[i][0])
                 and torch.equal(p1.forward_grad_host(xh[i], graph=graph)[1], ref[i][1]) for i in range(8))
        ts = []
        for i in range(calls):
            t0 = time.perf_counter()
            p1.forward_grad_host(xh[i], graph=graph)
            ts.append(time.perf_counter() - t0)
        res["graph" if graph else "fused"] = med(ts)
        res[("graph" if graph else "fused") + "_bit_identical"] = ok
print(res)
