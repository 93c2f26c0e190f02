"""Worst parity ratios of the HIP forward against the oracle (GPU box, repo root).

usage: python tools/parity_report.py [out.json]   (default profiles/r04_parity.json)

For every workload and path, tests/helpers.parity_case on the same candidates the GPU parity
tests use: the device lines against oracle.lines_batched (relative gap), the envelope kernel on
identical lines against the reference walk + expectation (stated tolerance 1e-6 |KG| + 64 eps
max|a|), and KG end to end (stated tolerance + the measured line gap through KG's Lipschitz
bound).  A ratio <= 1 passes; the report records how far inside the tolerance each case is,
and the KG error against the stated tolerance alone.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "decoupled-kg_amd"), os.path.join(REPO, "tests")]

from dkg_amd.synthetic import WORKLOADS, make_problem  # noqa: E402
from helpers import LINE_RTOL, parity_case  # noqa: E402

CASES = [("small", 32), ("parity6d", 32), ("headline", 128), ("headline_nd", 128), ("stress", 64)]


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "profiles", "r04_parity.json")
    rep = {"line_rtol": LINE_RTOL, "cases": []}
    for wname, nX in CASES:
        model, D, X, W = make_problem(WORKLOADS[wname])
        for target in (None, 0, 1):
            res = parity_case(model, D, W, X[:nX], target)
            row = {"workload": wname, "target": target,
                   **{k: v for k, v in res.items() if not k.startswith("_")}}
            rep["cases"].append(row)
            print(json.dumps(row), flush=True)
    rep["worst"] = {k: max(c[k] for c in rep["cases"]) for k in
                    ("line_rel_a", "line_rel_b", "envelope_ratio", "kg_ratio", "kg_ratio_stated_only")}
    json.dump(rep, open(out, "w"), indent=1)
    print(json.dumps(rep["worst"]))


if __name__ == "__main__":
    main()
