"""Per-pair phase stamps of the forward envelope (DKG_DEBUG_STAMPS=2).

Run on the GPU box from the repo root:  python tools/pair_stamps.py [workload]
For every (candidate, scalarisation) pair of the last of 10 forwards: s_memtime
cycles of the line build, the extremes, the margin chord compaction and the
list walk, the list length and the envelope size (whether the walk over all
lines was needed).
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd")]
os.environ["DKG_DEBUG_STAMPS"] = "2"
import torch  # noqa: E402

from dkg_amd import DiscreteKnowledgeGradient, _lib  # noqa: E402
from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402

w = WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "headline"]
target = int(sys.argv[2]) if len(sys.argv) > 2 else None
model, D, X, W = make_problem(w)
acq = DiscreteKnowledgeGradient(model, D, W, target_output_ix=target)
plan = acq._plan_for(w.B)
Xd = X.cuda().contiguous()
kg = torch.empty(w.B, dtype=torch.double, device="cuda")
n = 3 * 1024 * 8
lib = _lib.load()
for _ in range(10):
    plan.forward_into(Xd, kg)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * n)()
_lib.check(lib.dkg_debug_read_kstamps(buf, n), "kstamps")
st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 8).astype(np.int64)
P = min(w.B * w.S, st.shape[0])
st = st[:P]
ok = st[:, 3] > st[:, 0]
s = st[ok]
build = s[:, 1] - s[:, 0]
ext = s[:, 2] - s[:, 1]
comp = s[:, 3] - s[:, 2]
walked = (s[:, 4] > s[:, 3]) | (s[:, 5] > s[:, 3])
walk = np.where(s[:, 5] > s[:, 3], s[:, 5] - s[:, 3], np.where(walked, s[:, 4] - s[:, 3], 0))
full = (s[:, 7] >> 32) & 1
refilt = (s[:, 7] >> 33) & 1
flat = ((s[:, 7] >> 34) & 1).astype(bool)
hull = s[:, 7] & 0xffffffff
# pst[6]: the L-T-R list count (bits 0-15), after the chain refinement (16-31, 0: not refined), after the
# last re-filter of the walk loop (32-47, 0: none)
cnt0 = s[:, 6] & 0xffff
cnt1 = (s[:, 6] >> 16) & 0xffff
cnt2 = (s[:, 6] >> 32) & 0xffff
cnt = np.where(cnt2 > 0, cnt2, np.where(cnt1 > 0, cnt1, cnt0))


def q(v):
    v = np.asarray(v)
    if v.size == 0:
        return "-"
    return f"median {np.median(v):8.0f}  mean {v.mean():8.0f}  p90 {np.percentile(v, 90):8.0f}  max {v.max():8.0f}"


print(f"pairs {P}, with stamps {ok.sum()} (the rest short-circuited)")
print(f"flat (KG = 0 without a walk): {int(flat.sum())} pairs, compact/test {q(comp[flat])}")
build, ext, comp, walked, walk, full, refilt, hull, cnt, cnt0 = (
    v[~flat] for v in (build, ext, comp, walked, walk, full, refilt, hull, cnt, cnt0))
print("walked pairs:")
print("build   ", q(build))
print("extremes", q(ext))
print("compact ", q(comp))
print("walk    ", q(walk[walked]))
print("list cnt", q(cnt), " (L-T-R filter:", q(cnt0) + ")")
print("hull    ", q(hull), " full-walk pairs", int(full.sum()), " refiltered pairs", int(refilt.sum()))
print("list cnt hist", np.bincount(np.minimum(cnt, 130)).nonzero()[0][:40].tolist())
for lo, hi in [(0, 8), (8, 16), (16, 32), (32, 64), (64, 129), (129, 10**9)]:
    sel = (cnt >= lo) & (cnt < hi)
    if sel.any():
        print(f"  cnt [{lo},{hi}): {sel.sum():5d} pairs, walk {q(walk[sel & walked])}")

# the slowest pairs (they set the launch's tail): phase cycles, list length, envelope size
tot = np.where(s[:, 5] > s[:, 3], s[:, 5], np.where(s[:, 4] > s[:, 3], s[:, 4], s[:, 3])) - s[:, 0]
order = np.argsort(-tot)[:12]
print("slowest pairs: total / build / extremes / compact / walk cycles, list, hull, flags")
for r in order:
    w_ = (s[r, 5] - s[r, 3]) if s[r, 5] > s[r, 3] else (s[r, 4] - s[r, 3] if s[r, 4] > s[r, 3] else 0)
    print(f"  {tot[r]:6d} {s[r, 1] - s[r, 0]:6d} {s[r, 2] - s[r, 1]:6d} {s[r, 3] - s[r, 2]:6d} {w_:6d}"
          f"  cnt {s[r, 6] & 0xffff:4d}/{(s[r, 6] >> 16) & 0xffff:3d}/{(s[r, 6] >> 32) & 0xffff:3d} hull {s[r, 7] & 0xffffffff:3d} flags {s[r, 7] >> 32:#x}")
