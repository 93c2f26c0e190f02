"""Generate tests/golden/smoke_oracle.json: the SMOKE BO loop's decisions on the CPU oracle.

``tests/smoke_oracle.run_oracle_smoke``: the product's SMOKE loop (dkg_amd.bo_smoke.run_mobo, reference
``pipeline/main.py:171-216`` -> ``bo_loop.py:353-421``, presets ``:122-131``) with the oracle's discrete KG
as the acquisition and the oracle GP's posterior mean as the objective, on the gp-sample problem
lengthscales/0 (the committed golden fixture ``lengthscales0.npz``, from the reference's own ``.pt``), seeds 0
and 1.  The GPU test (tests/test_gpu_bo_smoke.py) runs the same loop on the device and compares every step's
chosen objective, candidate and acquisition value with these.  Run from the repo root:
    python tests/golden/make_smoke_oracle.py
"""

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd"), os.path.dirname(HERE)]

from helpers import load_golden  # noqa: E402
from smoke_oracle import run_oracle_smoke, trajectory  # noqa: E402

SEEDS = (0, 1)


def main():
    state = load_golden("lengthscales0")[0]
    out = {"problem": "lengthscales0", "seeds": {str(s): trajectory(run_oracle_smoke(state, s)) for s in SEEDS}}
    with open(os.path.join(HERE, "smoke_oracle.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
