"""Phase stamps of the envelope kernel (debug_flags & 4): per-wave s_memtime deltas."""
import ctypes, os, sys
import numpy as np
sys.path[:0] = ['.', 'decoupled-kg_amd']
os.environ['DKG_DEBUG_ENV_FLAGS'] = os.environ.get('DKG_DEBUG_ENV_FLAGS', '4')
import torch
from dkg_amd import DiscreteKnowledgeGradient, _lib
from dkg_amd.synthetic import WORKLOADS, make_problem
lib = _lib.load()
fn = lib.dkg_debug_read_stamps; fn.restype = ctypes.c_int; fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
model, D, X, W = make_problem(WORKLOADS['headline'])
acq = DiscreteKnowledgeGradient(model, D, W)
Xd = X.cuda().unsqueeze(-2)
for _ in range(5): acq(Xd)
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * (4096 * 8))()
_lib.check(fn(buf, 4096 * 8), 'stamps')
st = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.int64)[:2048]
t0 = st[:, 0].min()
names = ['start', 'staged', 'lines', 'hull', 'wgsum', 'end']
print('wave start spread (cycles):', np.percentile(st[:, 0] - t0, [0, 50, 100]))
for k in range(1, 6):
    d = st[:, k] - st[:, k - 1]
    print(f'{names[k-1]}->{names[k]}: median {np.median(d):.0f} p90 {np.percentile(d, 90):.0f} max {d.max()}')
print('end max - start min (cycles):', (st[:, 5] - t0).max())
