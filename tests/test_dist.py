"""Sharded Discrete KG over 2 ranks (gloo, CPU) vs the unsharded oracle.

SURVEY.md §8(e): the (candidate x scalarisation) pairs are split across ranks
and combined with one collective (all-reduce over scalarisations, or
all-gather over candidates).  Each rank's local evaluation is the oracle
(injected), so this checks the partitioning and the exchange, not the kernels.
Tolerance: the stated one (tests/helpers.py: 1e-6 |KG| + 64 eps max|a|) — the
oracle's batched matmuls round differently for a candidate slice than for the
whole batch.
"""

import os
import socket
import subprocess
import sys

import pytest
import torch

from dkg_amd.dist import shard_range
from dkg_amd.synthetic import WORKLOADS, make_problem
from helpers import assert_within, stated_tol, to_oracle
from oracle.discretekg import discrete_kg_batched, lines_batched

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(tmp_path, axis, B, S, target):
    out = str(tmp_path / f"{axis}_{B}_{S}.pt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "dist_worker.py"),
           axis, str(B), str(S), str(-1 if target is None else target), out]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    return torch.load(out, weights_only=True)


def test_shard_range_covers():
    for total in (0, 1, 3, 16, 17):
        for world in (1, 2, 3, 8):
            got = [shard_range(total, r, world) for r in range(world)]
            assert got[0][0] == 0 and got[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(got, got[1:]))


@pytest.mark.parametrize("axis,B,S,target", [
    ("scalarisations", 8, 8, None),
    ("scalarisations", 5, 3, 1),
    ("scalarisations", 4, 1, None),   # S < world: rank 1 holds no scalarisation
    ("candidates", 8, 8, None),
    ("candidates", 5, 8, 0),          # ragged candidate split
])
def test_sharded_matches_unsharded(tmp_path, axis, B, S, target):
    res = _launch(tmp_path, axis, B, S, target)
    model, D, X, W = make_problem(WORKLOADS["small"])
    om = to_oracle(model)
    ref = discrete_kg_batched(om, X[:B], D, W[:S], target)[0]
    amax = lines_batched(om, X[:B], D, W[:S], target)[0].abs().amax((-1, -2))
    assert_within(res["kg"], ref, stated_tol(ref, amax))
    calls = res["calls"]
    if axis == "scalarisations":
        assert sum(c[0][1] for c in calls if c) == S and all(c[0][0] == B for c in calls if c)
    else:
        assert sum(c[0][0] for c in calls if c) == B and all(c[0][1] == S for c in calls if c)
    # gradient: every rank holds the full d(sum_b w_b KG_b)/dX of the unsharded oracle
    Xr = X[:B].clone().requires_grad_(True)
    wts = torch.arange(1.0, B + 1.0, dtype=torch.double)
    (discrete_kg_batched(om, Xr, D, W[:S], target)[0] * wts).sum().backward()
    g_ref = Xr.grad
    for g in res["grads"]:
        assert g is not None and g.shape == g_ref.shape
        # the gradient floor of tests/test_gpu_grad.py: 1e-9 of the largest component (cancellation in E - max a)
        torch.testing.assert_close(g, g_ref, rtol=1e-9, atol=1e-9 * float(g_ref.abs().max()))
    assert torch.equal(res["grads"][0], res["grads"][1])
    assert torch.equal(res["kg_async"], res["kg"])
    assert_within(res["kg_async_flip"], ref.flip(0), stated_tol(ref.flip(0), amax.flip(0)))


def test_idle_rank_zeros_keep_nonfinite_inputs_out():
    """A rank with no local work joins the backward through zeros connected to X: an inf / NaN coordinate in X
    gives an exact zero gradient there, not NaN (which the all-reduce would spread to every candidate)."""
    from dkg_amd.dist import _zeros_like_graph

    x = torch.tensor([[0.5, float("inf")], [float("nan"), 0.1]], dtype=torch.double, requires_grad=True)
    z = _zeros_like_graph(x, 3, torch.device("cpu"))
    assert torch.equal(z, torch.zeros(3, dtype=torch.double)) and z.requires_grad
    (z * torch.tensor([1.0, 2.0, 3.0], dtype=torch.double)).sum().backward()
    assert torch.equal(x.grad, torch.zeros_like(x))


@pytest.mark.parametrize("mode,steps,every", [("gather", 7, 3), ("gather", 6, 3), ("reduce", 7, 3),
                                              ("reduce", 2, 64)])
def test_batch_exchange(tmp_path, mode, steps, every):
    """bench.py's K-batches-per-collective exchange (dkg_amd.dist.BatchExchange) over 2 gloo ranks:
    every step's values arrive, in order, in exactly ceil(steps / K) collectives, including a
    partially filled last buffer and double-buffer reuse across a warm-up and a timed pass."""
    out = str(tmp_path / f"xchg_{mode}_{steps}_{every}.pt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "exchange_worker.py"),
           mode, str(steps), str(every), out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=dict(os.environ, OMP_NUM_THREADS="1"))
    assert r.returncode == 0, r.stderr[-3000:]
    res = torch.load(out, weights_only=True)
    assert res["n"] == -(-steps // every)
    assert torch.equal(res["got"], res["exp"])
