"""The fp32 plan's slopes against the fp64 plan's, per candidate, at one workload (default stress32): a plan
for B candidates and one for 2B (the candidates twice).  Prints, per plan, the per-candidate relative slope
error max_k |b32 - b64| / max_k |b64| (scalarisation 0) and the candidates whose error stands out.

usage: python tools/f32_debug.py [workload]   (DKG_COV_BIG32 / DKG_CROSS_BIG select the kernels)
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]

import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402


def main():
    wname = sys.argv[1] if len(sys.argv) > 1 else "stress32"
    dev = torch.device("cuda", 0)
    w = WORKLOADS[wname]
    model, D, X, W = make_problem(w)
    acq = DiscreteKnowledgeGradient(model, D, W, device=dev)
    Xd = X.to(dev).contiguous()
    B = Xd.shape[0]
    _, b64 = acq._state.plan(acq._W, acq._target, B).lines(Xd)
    ref = b64[:, 0]
    den = ref.abs().amax(-1)
    del b64
    print(f"{wname} cov_big32={os.environ.get('DKG_COV_BIG32')} cross_big={os.environ.get('DKG_CROSS_BIG')}")
    for K in (1, 2):
        p = acq._state.plan(acq._W, acq._target, K * B, f32=True)
        _, b32 = p.lines(Xd.repeat(K, 1).contiguous())
        for j in range(K):
            e = ((b32[j * B:(j + 1) * B, 0] - ref).abs().amax(-1) / den).cpu()
            bad = torch.nonzero(e > 1e-2).flatten().tolist()
            print(f"  plan {K * B} batch {j}: rel slope error median {e.median():.3e} max {e.max():.3e}; "
                  f"> 1e-2 at {len(bad)} candidates {bad[:40]}")
        del b32, p
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
