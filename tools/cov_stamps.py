"""Per-workgroup phase stamps of the covariance (or, --env, the envelope) stage of one batched launch
(DKG_DEBUG_STAMPS=1).

usage: python tools/cov_stamps.py [G] [workload] [--env]      (DKG_COV_BIG=0/1 picks the block shape)
Runs dkg_plan_forward_batches over G headline batches a few times and prints, for the covariance kernel of
the last launch: workgroups, launch span, workgroup lifetime (median / p90 / max, cycles of the 100 MHz
s_memtime clock x 24 = 2.4 GHz cycles), the phases between the stamps, and the largest number of
workgroups resident at once (per CU: / 256).
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

ENV = "--env" in sys.argv
args = [a for a in sys.argv[1:] if a != "--env"]
G = int(args[0]) if args else 20
w = WORKLOADS[args[1] if len(args) > 1 else "headline"]
model, D, X, W = make_problem(w)
acq = DiscreteKnowledgeGradient(model, D, W)
plan = acq._state.plan(acq._W, acq._target, G * w.B)
Xd = X.cuda().repeat(G, 1).contiguous()
kg = torch.empty(G * w.B, dtype=torch.double, device="cuda")
for _ in range(5):
    plan.forward_batches_into(Xd, kg, w.B)
torch.cuda.synchronize()
n = 3 * 1024 * 8
buf = (ctypes.c_ulonglong * n)()
_lib.check(_lib.load().dkg_debug_read_kstamps(buf, n), "kstamps")
st = np.frombuffer(buf, dtype=np.uint64).reshape(3, 1024, 8).astype(np.int64)
s = st[2 if ENV else 1]
s = s[s[:, 0] > 0]
t0 = s[:, 0].min()
life = (s[:, 7] - s[:, 0]) * 24
print(f"{'envelope' if ENV else 'covariance'} G={G} cov_big={os.environ.get('DKG_COV_BIG')}: {len(s)} WGs (first 1024 stamped), span "
      f"{(s[:, 7].max() - t0) / 100:.2f} us, lifetime cycles median {np.median(life):.0f} p90 "
      f"{np.percentile(life, 90):.0f} max {life.max():.0f}")
# phases on the s_memtime clock (slots 1 .. 6), as fractions of the workgroup's own span
tot = (s[:, 6] - s[:, 1]).astype(np.float64)
phases = ((1, 2, "issue DMA"), (2, 3, "wait+sync"), (3, 4, "pairs"), (4, 5, "WG sum"), (5, 6, "combine")) if ENV else \
    ((1, 2, "stage"), (2, 3, "loop"), (3, 6, "epilogue"))
for a, b, nm in phases:
    ok = (s[:, a] > 0) & (s[:, b] > 0) & (tot > 0)
    if ok.any():
        f = (s[ok, b] - s[ok, a]) / tot[ok]
        print(f"  {nm:10s} fraction of lifetime median {np.median(f):.3f} p90 {np.percentile(f, 90):.3f}")
ev = sorted([(int(x), 1) for x in s[:, 0]] + [(int(x), -1) for x in s[:, 7]])
cur = peak = 0
for _, dlt in ev:
    cur += dlt
    peak = max(peak, cur)
span_ticks = s[:, 7].max() - s[:, 0].min()
print(f"  peak resident workgroups {peak} ({peak / 256:.2f} per CU), mean resident "
      f"{(s[:, 7] - s[:, 0]).sum() / span_ticks:.1f} ({(s[:, 7] - s[:, 0]).sum() / span_ticks / 256:.2f} per CU), "
      f"mean lifetime {life.mean():.0f} cycles")
