"""The fused one-launch forward (dkg_fused.h, DKG_PLAN_FUSED) against the three stage kernels (the default).

Both run the same arithmetic (the same stage bodies, the same reduction orders), so every KG must be the
same bits; what differs is how the stages meet: two kernel boundaries, or arrival counters inside one
launch (write-through stores, one acquire per consumer workgroup, counters re-zeroed by the launch's last
workgroup).  So these check the hand-offs: shapes with partial row tiles / row blocks, one output to eight,
S below 8 and above 16 (more than two envelope workgroups per candidate), repeated launches on one plan,
HIP-graph replay, plans on four streams at once, and launches next to a heavy kernel on another stream
(uneven load, MI355X_MICROARCH.md "test every hand-off under uneven load").  Every in-launch wait must have
matched (dkg_plan_status == 0).
"""

import pytest
import torch

from dkg_amd.gp_state import DeviceGPState
from dkg_amd.model import ModelListGPState, SingleTaskGPState
from dkg_amd.synthetic import WORKLOADS, make_problem

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _pair(model, D, W, target, max_B):
    st = DeviceGPState(model, D, DEV)
    fused = st.plan(W, target, max_B, fused=True)
    split = st.plan(W, target, max_B)
    assert fused.fused and not split.fused
    return fused, split


def _random_model(m, d, n, seed):
    g = torch.Generator().manual_seed(seed)
    outs = []
    for i in range(m):
        X = torch.rand(n + 3 * i, d, generator=g, dtype=torch.double)
        y = torch.sin(3 * X.sum(-1) + i) + 0.1 * torch.randn(X.shape[0], generator=g, dtype=torch.double)
        outs.append(SingleTaskGPState(X, y, 0.3 + 0.1 * i, 1.0 + i, 1e-3, 0.1 * i,
                                      kernel=["matern", "rbf"][i % 2], nu=[2.5, None][i % 2]))
    return ModelListGPState(*outs), g


@pytest.mark.parametrize("workload", ["small", "headline", "headline_nd", "parity6d"])
@pytest.mark.parametrize("target", [None, 1])
def test_fused_is_the_split_forward_bit_for_bit(workload, target):
    model, D, X, W = make_problem(WORKLOADS[workload])
    fused, split = _pair(model, D, W, target, X.shape[0])
    Xd = X.to(DEV).contiguous()
    a, b = fused.forward(Xd), split.forward(Xd)
    assert torch.equal(a, b)
    assert fused.status() == 0


@pytest.mark.parametrize("m,d,N,S,B", [(1, 2, 37, 1, 1), (2, 3, 77, 5, 17), (3, 3, 200, 24, 33), (8, 2, 60, 8, 48),
                                       (2, 6, 1000, 16, 100), (4, 2, 513, 40, 7)])
def test_fused_odd_shapes(m, d, N, S, B):
    """Partial row tiles and row blocks (B not a multiple of 16 / 32), one to eight outputs, S < 8 and S > 16
    (three to five envelope workgroups per candidate, the ticketed combine), d = 6, N + 1 across slot buckets."""
    model, g = _random_model(m, d, 40, 100 * m + N)
    D = torch.rand(N, d, generator=g, dtype=torch.double)
    W = torch.rand(S, m, generator=g, dtype=torch.double)
    W = W / W.sum(-1, keepdim=True)
    Xc = torch.rand(B, d, generator=g, dtype=torch.double).to(DEV)
    for target in (None, m - 1):
        fused, split = _pair(model, D, W, target, B)
        assert torch.equal(fused.forward(Xc), split.forward(Xc))
        assert fused.status() == 0


def test_fused_repeated_graph_and_streams():
    """Many launches on one plan (the counters re-zeroed in-launch every time), replays of a captured graph of
    eight forwards, and four plans on four streams, all equal to the split forward's bits."""
    w = WORKLOADS["headline"]
    model, D, X, W = make_problem(w)
    st = DeviceGPState(model, D, DEV)
    split = st.plan(W, None, w.B)
    batches = [torch.quasirandom.SobolEngine(2, scramble=True, seed=30 + k).draw(w.B, dtype=torch.double)
               .to(DEV).contiguous() for k in range(8)]
    want = [split.forward(x) for x in batches]
    plans = [st.plan(W, None, w.B, fused=True) for _ in range(4)]
    out = torch.full((len(batches), w.B), float("nan"), dtype=torch.double, device=DEV)
    for rep in range(40):
        plans[0].forward_into(batches[rep % 8], out[rep % 8])
    torch.cuda.synchronize()
    assert all(torch.equal(out[k], want[k]) for k in range(8))
    # graph replay
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for k in range(8):
            plans[1].forward_into(batches[k], out[k])
    for _ in range(3):
        out.fill_(float("nan"))
        g.replay()
        torch.cuda.synchronize()
        assert all(torch.equal(out[k], want[k]) for k in range(8))
    # four plans on four streams, interleaved
    main = torch.cuda.current_stream(DEV)
    streams = [main] + [torch.cuda.Stream(DEV) for _ in range(3)]
    for s in streams[1:]:
        s.wait_stream(main)
    out.fill_(float("nan"))
    for rep in range(32):
        with torch.cuda.stream(streams[rep % 4]):
            plans[rep % 4].forward_into(batches[rep % 8], out[rep % 8])
    for s in streams[1:]:
        main.wait_stream(s)
    torch.cuda.synchronize()
    assert all(torch.equal(out[k], want[k]) for k in range(8))
    assert all(p.status() == 0 for p in plans)


def test_fused_under_uneven_load():
    """Fused forwards while a long matrix multiply occupies CUs from another stream: the hand-offs meet
    workgroups that start late and run slow; every result is the split forward's."""
    w = WORKLOADS["headline_nd"]
    model, D, X, W = make_problem(w)
    fused, split = _pair(model, D, W, None, w.B)
    Xd = X.to(DEV).contiguous()
    want = split.forward(Xd)
    big = torch.randn(4096, 4096, device=DEV)
    other = torch.cuda.Stream(DEV)
    outs = torch.empty(24, w.B, dtype=torch.double, device=DEV)
    for k in range(24):
        if k % 6 == 0:
            with torch.cuda.stream(other):
                big = (big @ big).tanh_()
        fused.forward_into(Xd, outs[k])
    torch.cuda.synchronize()
    assert all(torch.equal(outs[k], want) for k in range(24))
    assert fused.status() == 0
