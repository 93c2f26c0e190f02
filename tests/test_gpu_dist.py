"""The HIP forward sharded over 2 processes on one MI355X (gloo, both ranks on cuda:0).

SURVEY.md §8(e): the (candidate x scalarisation) pairs split over ranks, combined by one
collective per forward (all-reduce over scalarisations, all-gather over candidates), and
bench.py's K-batches-per-collective exchange (dkg_amd.dist.BatchExchange).  Checked against
the unsharded HIP forward of the same process group:
  * candidates axis: bit-identical values (a candidate's KG does not depend on its batch);
  * scalarisations axis: the S-average of per-rank partial sums, within 1e-13 relative;
  * gradients (through the differentiable exchange): every rank holds the full dKG/dX.
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
def ranks(tmp_path_factory):
    if not torch.cuda.is_available():
        pytest.skip("no ROCm device")
    out = str(tmp_path_factory.mktemp("dist") / "res.pt")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(HERE, "dist_gpu_worker.py"),
           "headline", out]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240,
                       env=dict(os.environ, OMP_NUM_THREADS="2"))
    assert r.returncode == 0, r.stderr[-4000:]
    return torch.load(out, weights_only=False)


@pytest.mark.parametrize("target", [None, 1])
@pytest.mark.parametrize("axis", ["scalarisations", "candidates"])
def test_sharded_hip_forward_and_gradient(ranks, axis, target):
    kg_ref, g_ref = ranks["ref"][target]
    for r in ranks["ranks"]:
        kg, g = r[(axis, target)]
        if axis == "candidates":
            assert torch.equal(kg, kg_ref)
            assert torch.equal(g, g_ref)  # the other rank's rows arrive as exact zeros in the sum
        else:
            torch.testing.assert_close(kg, kg_ref, rtol=1e-13, atol=1e-300)
            # floor: 1e-9 of the largest component, as tests/test_gpu_grad.py
            torch.testing.assert_close(g, g_ref, rtol=1e-12, atol=1e-9 * float(g_ref.abs().max()))
    assert torch.equal(ranks["ranks"][0][(axis, target)][1], ranks["ranks"][1][(axis, target)][1])


def test_batch_exchange_with_hip_forwards(ranks):
    kg_ref = ranks["ref"][None][0]
    r0, r1 = ranks["ranks"]
    # reduce: every rank's rows are the all-reduced partial sums; / S gives the unsharded KG
    S = 16
    for r in (r0, r1):
        rows = torch.cat(r[("xchg", "reduce")])
        assert rows.shape == (5, kg_ref.shape[0])
        for row in rows:
            torch.testing.assert_close(row / S, kg_ref, rtol=1e-13, atol=1e-300)
    # gather: rank q's row k holds rank q's own batch k, bit-identical to the unsharded forward of it
    for r in (r0, r1):
        got = r[("xchg", "gather")]
        assert sum(t.shape[1] for t in got) == 5
        allrows = torch.cat(got, dim=1)  # [world, 5, B]
        for q, rq in enumerate((r0, r1)):
            for k, Xk in enumerate(rq[("xchg_x", "gather")]):
                perm_ref = kg_ref[torch.roll(torch.arange(kg_ref.shape[0]), shifts=3 * k + 7 * q)]
                assert torch.equal(allrows[q, k], perm_ref)
