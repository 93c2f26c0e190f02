"""Rank body for tests/test_gpu_dist.py and tests/test_gpu_rccl.py: the HIP forward sharded over ranks.

usage: dist_gpu_worker.py WORKLOAD OUT [BACKEND]
torch.distributed with gloo (test_gpu_dist: 2 ranks, both on cuda:0) or nccl = RCCL (test_gpu_rccl:
1 rank on cuda:0; RCCL needs one GPU per rank).  Rank r evaluates its shard through
DiscreteKnowledgeGradient (the C ABI); rank 0 also runs the unsharded forward and writes everything
for the test process.
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

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.dist import BatchExchange, ShardedDiscreteKG, shard_range  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402


def main():
    workload, out = sys.argv[1], sys.argv[2]
    backend = sys.argv[3] if len(sys.argv) > 3 else "gloo"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group(backend)
    rank, world = dist.get_rank(), dist.get_world_size()
    model, D, X, W = make_problem(WORKLOADS[workload])
    res = {}
    for target in (None, 1):
        for axis in ("scalarisations", "candidates"):
            acq = ShardedDiscreteKG(model, D, W, target, axis=axis, device=dev)
            kg = acq(X.unsqueeze(-2))
            Xr = X.clone().requires_grad_(True)
            wts = torch.linspace(0.5, 1.5, X.shape[0], dtype=torch.double)
            (acq(Xr.unsqueeze(-2)) * wts).sum().backward()
            res[(axis, target)] = (kg.cpu(), Xr.grad.clone())
            res[("async", axis, target)] = acq.forward_async(X.unsqueeze(-2)).wait().cpu()
    # bench.py's exchange: K forward batches per collective, both modes, HIP forwards into the rows
    B, S = X.shape[0], W.shape[0]
    for mode in ("reduce", "gather"):
        if mode == "reduce":
            lo, hi = shard_range(S, rank, world)
            acq = DiscreteKnowledgeGradient(model, D, W[lo:hi], device=dev)
            xs = [X] * 5
        else:
            acq = DiscreteKnowledgeGradient(model, D, W, device=dev)
            xs = [torch.roll(X, shifts=3 * k + 7 * rank, dims=0) for k in range(5)]
        plan = acq._plan_for(B)
        sink = []
        xchg = BatchExchange(B, 2, mode, S_local=(hi - lo) if mode == "reduce" else S, device=dev, sink=sink)
        for k, Xk in enumerate(xs):
            plan.forward_into(Xk.to(dev).contiguous(), xchg.row(k))
            torch.cuda.synchronize()
            xchg.done(k)
        xchg.flush(len(xs))
        res[("xchg", mode)] = [t.cpu() for t in sink]
        res[("xchg_x", mode)] = [x.clone() for x in xs]
    allres = [None] * world
    dist.all_gather_object(allres, res)
    if rank == 0:
        ref = {}
        for target in (None, 1):
            acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target, device=dev)
            Xr = X.clone().to(dev).requires_grad_(True)
            wts = torch.linspace(0.5, 1.5, X.shape[0], dtype=torch.double, device=dev)
            kg = acq(Xr.unsqueeze(-2))
            (kg * wts).sum().backward()
            ref[target] = (kg.detach().cpu(), Xr.grad.cpu())
        torch.save({"ranks": allres, "ref": ref}, out)
    res_backend = dist.get_backend()
    if rank == 0:
        with open(out + ".backend", "w") as f:
            f.write(f"{res_backend} world={world}")
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
