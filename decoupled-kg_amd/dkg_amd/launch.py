"""Side-by-side enqueue of captured forward graphs on several streams (C ABI ``dkg_launcher_*``).

Batches of forwards in flight on several HIP streams (one plan workspace each) are captured as one
single-stream graph per stream.  Enqueuing them from one host thread costs each stream the launches
of the streams before it (~1 us per kernel node plus ~9 us per ``hipGraphLaunch``); the native
launcher enqueues every stream's graphs from its own host thread, so all streams start together.
Host-side scheduling only: the graphs hold exactly the kernels the caller captured.
"""

from __future__ import annotations

import ctypes
from typing import Sequence

from . import _lib


class GraphLauncher:
    def __init__(self, threads: int):
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        _lib.check(self._lib.dkg_launcher_create(int(threads), ctypes.byref(h)), "dkg_launcher_create")
        self._h = h
        self.threads = int(threads)
        self._calls = {}

    def arm(self, seconds: float) -> None:
        """Workers spin (wake in ~1 us) for the next ``seconds``; afterwards they sleep again."""
        _lib.check(self._lib.dkg_launcher_arm(self._h, float(seconds)), "dkg_launcher_arm")

    def prepare(self, key, streams: Sequence[int], graphs: Sequence[Sequence[int]]) -> None:
        """Marshal one launch set once: stream i (raw hipStream_t) gets graphs[i] (raw hipGraphExec_t) in order."""
        n = len(streams)
        offs = [0]
        flat = []
        for g in graphs:
            flat.extend(int(x) for x in g)
            offs.append(len(flat))
        self._calls[key] = (n, (ctypes.c_void_p * max(1, n))(*[int(s) for s in streams]),
                            (ctypes.c_int * (n + 1))(*offs), (ctypes.c_void_p * max(1, len(flat)))(*flat))

    def launch(self, key) -> None:
        n, s, o, g = self._calls[key]
        st = self._lib.dkg_launcher_graphs(self._h, n, s, o, g)
        if st:
            _lib.check(st, "dkg_launcher_graphs")

    def close(self) -> None:
        if self._h is not None and self._h.value:
            self._lib.dkg_launcher_destroy(self._h)
        self._h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
