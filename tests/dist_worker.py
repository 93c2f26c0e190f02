"""Rank body for tests/test_dist.py (launched by torch.distributed.run, gloo, CPU).

Each rank evaluates its shard with the oracle injected as the local forward and
rank 0 writes the combined result for the test process to compare.
"""

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "decoupled-kg_amd"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from dkg_amd.dist import ShardedDiscreteKG  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402
from helpers import to_oracle  # noqa: E402
from oracle.discretekg import discrete_kg_batched  # noqa: E402


def main():
    axis, B, S, target, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    target = None if target < 0 else target
    torch.set_default_dtype(torch.double)
    torch.set_num_threads(2)
    dist.init_process_group("gloo")
    model, D, X, W = make_problem(WORKLOADS["small"])
    X, W = X[:B], W[:S]
    om = to_oracle(model)
    calls = []

    def local(Xl, Wl):
        if not calls:  # the first call (the forward) is the one checked
            calls.append((Xl.shape[0], Wl.shape[0]))
        return discrete_kg_batched(om, Xl, D, Wl, target)[0]

    acq = ShardedDiscreteKG(model, D, W, target, axis=axis, local_forward=local)
    kg = acq(X.unsqueeze(-2))
    # the async exchange gives the same bits (two batches in flight before the first wait)
    p1, p2 = acq.forward_async(X.unsqueeze(-2)), acq.forward_async(X.flip(0).unsqueeze(-2))
    kg_async, kg_async_flip = p1.wait(), p2.wait()
    shapes = [None] * dist.get_world_size()
    dist.all_gather_object(shapes, calls)
    # gradient through the exchange: every rank gets the full dKG/dX
    Xr = X.clone().requires_grad_(True)
    wts = torch.arange(1.0, X.shape[0] + 1.0)
    (acq(Xr.unsqueeze(-2)) * wts).sum().backward()
    grads = [None] * dist.get_world_size()
    dist.all_gather_object(grads, Xr.grad)
    if dist.get_rank() == 0:
        torch.save({"kg": kg, "calls": shapes, "grads": grads, "kg_async": kg_async,
                    "kg_async_flip": kg_async_flip}, out)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
