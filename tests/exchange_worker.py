"""torchrun worker (gloo, CPU) for tests/test_dist.py::test_batch_exchange: runs the bench's
BatchExchange over `steps` steps of K-batch exchanges and writes what every completed collective
delivered, plus the expected values, to <out>.  argv: mode steps every out"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(HERE), os.path.join(os.path.dirname(HERE), "decoupled-kg_amd")]

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from dkg_amd.dist import BatchExchange  # noqa: E402


def main():
    mode, steps, every, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    B, S_local = 5, 4
    sink = []
    x = BatchExchange(B, every, mode, S_local=S_local, sink=sink)

    def value(r, k):  # what rank r writes at step k
        return torch.arange(B, dtype=torch.double) + 100.0 * k + 10000.0 * r

    for warm in (True, False):  # a warm-up pass, then the "timed" pass, as bench.py does
        sink.clear()
        for k in range(steps):
            x.row(k).copy_(value(rank, k))
            x.done(k)
        x.flush(steps)
    got = torch.cat([t.reshape(-1) for t in sink]) if sink else torch.zeros(0, dtype=torch.double)
    exp = []
    for start in range(0, steps, every):
        ks = range(start, min(steps, start + every))
        if mode == "gather":
            exp.append(torch.stack([torch.stack([value(r, k) for k in ks]) for r in range(world)]).reshape(-1))
        else:
            exp.append(torch.stack([sum(value(r, k) * S_local for r in range(world)) for k in ks]).reshape(-1))
    if rank == 0:
        torch.save({"got": got, "exp": torch.cat(exp), "n": len(sink)}, out)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
