"""RCCL on the MI355X: the sharded HIP forward and the batch exchange through the `nccl` backend.

torch.distributed's "nccl" backend is RCCL on ROCm.  One rank on cuda:0 (world size 1: the box has one GPU, and
RCCL wants one GPU per rank), so every collective of dkg_amd.dist runs through an RCCL communicator over a single
rank: ShardedDiscreteKG's all-reduce (scalarisations) / all-gather (candidates) in the forward, the gradient
all-reduce in the backward, forward_async, and BatchExchange in both modes (SURVEY.md §8(e),
discretekg.py:200-235).  Results against the unsharded HIP forward of the same process: with one rank each
collective is an identity, so values and gradients are bit-identical up to the S-average's (x S_r) / S rescaling.
"""

import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def rank0(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    out = str(tmp_path_factory.mktemp("rccl") / "res.pt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "dist_gpu_worker.py"),
           "headline", out, "nccl"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, OMP_NUM_THREADS="2", HSA_ENABLE_IPC_MODE_LEGACY="0"))
    assert r.returncode == 0, r.stderr[-4000:]
    with open(out + ".backend") as f:
        backend = f.read()
    res = torch.load(out, weights_only=False)
    return res, backend


def test_backend_is_rccl(rank0):
    assert rank0[1] == "nccl world=1"


@pytest.mark.parametrize("target", [None, 1])
@pytest.mark.parametrize("axis", ["scalarisations", "candidates"])
def test_sharded_forward_and_gradient_over_rccl(rank0, axis, target):
    res, _ = rank0
    kg_ref, g_ref = res["ref"][target]
    (r,) = res["ranks"]
    kg, g = r[(axis, target)]
    if axis == "candidates":
        assert torch.equal(kg, kg_ref)
        assert torch.equal(g, g_ref)
    else:  # part = mean x S, all-reduced, / S
        torch.testing.assert_close(kg, kg_ref, rtol=1e-15, atol=1e-300)
        torch.testing.assert_close(g, g_ref, rtol=1e-14, atol=1e-12 * float(g_ref.abs().max()))
    if target is None:
        torch.testing.assert_close(r[("async", axis, target)], kg, rtol=0, atol=0)


def test_batch_exchange_over_rccl(rank0):
    res, _ = rank0
    kg_ref = res["ref"][None][0]
    (r,) = res["ranks"]
    S = 16
    rows = torch.cat(r[("xchg", "reduce")])
    assert rows.shape == (5, kg_ref.shape[0])
    for row in rows:
        torch.testing.assert_close(row / S, kg_ref, rtol=1e-15, atol=1e-300)
    allrows = torch.cat(r[("xchg", "gather")], dim=1)  # [1, 5, B]
    assert allrows.shape[:2] == (1, 5)
    for k in range(5):
        assert torch.equal(allrows[0, k], kg_ref[torch.roll(torch.arange(kg_ref.shape[0]), shifts=3 * k)])
