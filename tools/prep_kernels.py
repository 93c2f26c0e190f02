"""Device-state preparations for a kernel trace:  rocprofv3 --kernel-trace --stats -- python3 tools/prep_kernels.py"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]
import torch  # noqa: E402

from dkg_amd.gp_state import DeviceGPState  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402

w = WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "headline"]
model, D, X, W = make_problem(w)
for i in range(4):
    DeviceGPState(model, D)
torch.cuda.synchronize()
print("done")
