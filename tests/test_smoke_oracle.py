"""The SMOKE BO loop on the CPU oracle still reproduces its committed decisions (tests/golden/smoke_oracle.json,
tests/golden/make_smoke_oracle.py): guards the fixture the device run is compared with in
tests/test_gpu_bo_smoke.py against drift of the oracle or of the loop.  Candidates within the optimiser's
tolerance (1e-4, see test_gpu_bo_smoke.py): two runs on this CPU differ by ~1e-8 (BLAS thread splits)."""

import json
import os

import pytest

from helpers import load_golden
from smoke_oracle import run_oracle_smoke, trajectory

FIXTURE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "smoke_oracle.json")


def test_oracle_smoke_reproduces_fixture():
    want = json.load(open(FIXTURE))["seeds"]["0"]
    got = trajectory(run_oracle_smoke(load_golden("lengthscales0")[0], 0))
    for mode in ("separate", "full"):
        assert got[mode]["obj_index"] == want[mode]["obj_index"]
        for x, xr in zip(got[mode]["x"], want[mode]["x"]):
            assert x == pytest.approx(xr, abs=1e-4)
        assert got[mode]["acq"] == pytest.approx(want[mode]["acq"], rel=1e-6, abs=1e-8)
        assert all(a > 0 for a in got[mode]["acq"])  # a real optimisation: the KG is positive at every choice
