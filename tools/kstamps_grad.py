"""Per-workgroup phase stamps of the value+gradient kernels (DKG_DEBUG_STAMPS=1).

Run on the GPU box from the repo root:  python tools/kstamps_grad.py [workload] [B]
Prints, for the last of 20 back-to-back headline forwards: each kernel's
workgroup start/end window on the 100 MHz clock (relative to the first
cross_root start, so the gaps between kernels show), and the per-phase
s_memtime deltas (median / p90 / max over workgroups).
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

w = WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "headline"]
model, D, X, W = make_problem(w)
acq = DiscreteKnowledgeGradient(model, D, W)
B = int(sys.argv[2]) if len(sys.argv) > 2 else w.B
plan = acq._plan_for(B, grad=True)
Xd = X[:B].cuda().contiguous()
kg = torch.empty(w.B, dtype=torch.double, device="cuda")
for _ in range(20):
    plan.forward_grad(Xd)
torch.cuda.synchronize()
n = 3 * 1024 * 8
buf = (ctypes.c_ulonglong * n)()
_lib.check(_lib.load().dkg_debug_read_kstamps(buf, n), "kstamps")
st = np.frombuffer(buf, dtype=np.uint64).reshape(3, 1024, 8).astype(np.int64)
names = ["cross_root", "posterior_cov", "envelope"]
phases = {0: ["plan+prefetch", "stage X", "K fill", "MFMA", "reduce+store"],
          1: ["epi loads", "loads+MFMA", "LDS part", "reduce+store", "-"],
          2: ["pre+stage", "filter", "idx+hull", "flush", "tail(WG wait)"]}
t0 = None
for k in range(3):
    s = st[k]
    used = s[:, 0] > 0
    s = s[used]
    if not used.any():
        print(f"{names[k]}: no stamps")
        continue
    if t0 is None:
        t0 = s[:, 0].min()
    rt0, rt1 = (s[:, 0] - t0) / 100.0, (s[:, 7] - t0) / 100.0  # us
    print(f"{names[k]}: {used.sum()} WGs  start {rt0.min():.2f}..{rt0.max():.2f} us  end {rt1.min():.2f}..{rt1.max():.2f}"
          f" us  (span {rt1.max() - rt0.min():.2f} us)")
    cyc = s[:, 6] - s[:, 1]
    rate = np.median(cyc / np.maximum(1e-9, (s[:, 7] - s[:, 0]) / 100.0))
    print(f"   s_memtime rate ~{rate:.0f} cycles/us; WG lifetime median {np.median(cyc):.0f} max {cyc.max()} cycles")
    marks = [1, 2, 3, 4, 5, 6]
    for i in range(5):
        a, b = marks[i], marks[i + 1]
        valid = (s[:, a] > 0) & (s[:, b] > 0)
        if valid.sum() == 0:
            continue
        dd = (s[valid, b] - s[valid, a])
        print(f"   {phases[k][i]:>14}: median {np.median(dd):7.0f}  p90 {np.percentile(dd, 90):7.0f}  max {dd.max():7d}")
