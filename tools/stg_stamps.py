"""Wait vs compute of the staged streaming passes (library built with EXTRA=-DDKG_STG_STAMPS).

Run on the GPU box:  python tools/stg_stamps.py [workload]   (envelope workgroups: slot 3 = passes start,
4 = wave 0's cycles waiting at the chunk barriers, 5 = passes end, 6 = workgroup end)
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]
os.environ["DKG_DEBUG_STAMPS"] = "1"
import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient, _lib  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402

w = WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "stress"]
model, D, X, W = make_problem(w)
acq = DiscreteKnowledgeGradient(model, D, W)
plan = acq._plan_for(w.B)
Xd = X.cuda().contiguous()
kg = torch.empty(w.B, dtype=torch.double, device="cuda")
for _ in range(5):
    plan.forward_into(Xd, kg)
torch.cuda.synchronize()
n = 3 * 1024 * 8
buf = (ctypes.c_ulonglong * n)()
_lib.check(_lib.load().dkg_debug_read_kstamps(buf, n), "kstamps")
st = np.frombuffer(buf, dtype=np.uint64).reshape(3, 1024, 8).astype(np.int64)[2]
st = st[st[:, 0] > 0]
passes = st[:, 5] - st[:, 3]
wait = st[:, 4]
tail = st[:, 6] - st[:, 5]
q = lambda v: f"median {np.median(v):8.0f} p90 {np.percentile(v, 90):8.0f} max {v.max():8.0f}"
print(f"{len(st)} envelope WGs")
print("passes      ", q(passes))
print("  waiting   ", q(wait))
print("  computing ", q(passes - wait))
print("tail (refine/walk/sum)", q(tail))
if os.environ.get("DKG_STG_SAMPLE", "1") != "0":
    # sample-hull build: slot 4 = pass 0 (sample hull) done, slot 5 = the staged pass done; hull sizes hold
    # the list lengths
    p0 = st[:, 4] - st[:, 3]
    print("pass 0 (sample hull)", q(p0))
    print("staged pass         ", q(st[:, 5] - st[:, 4]))
    _, _, cnt = plan.forward_stats(Xd)
    c = cnt.flatten().cpu().numpy().astype(np.int64)
    print("list length          ", q(c), "over 512:", int((c > 512).sum()), "of", c.size)
