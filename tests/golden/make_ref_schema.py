"""Generate tests/golden/ref_schema.json: the reference's checkpoint schema, as data.

Two things the SMOKE loop's checkpoints must match so the reference's ``build_model_from_checkpoint``
(``pipeline/nodes/bo_loop.py:663-667`` -> ``modules/model/factory.py:24-60``) can rebuild the surrogate:

* ``model_config``: the ``model`` section of ``config/experiment-lengthscales.yaml`` (YAML, read with
  ``yaml.safe_load``) -- the config of the SMOKE run's ``gp-sample:lengthscales`` problem;
* the ``ModelListGP`` state-dict keys and shapes of a reference-built model: those of the
  ``model_state_dict`` in ``data/shared/gp-problem/lengthscales/0.pt`` (``torch.load(weights_only=True)``),
  a ModelListGP of two SingleTaskGPs (``models.i.*`` plus the ``LikelihoodList`` copies
  ``likelihood.likelihoods.i.*``).

Run from the repo root where /root/reference exists:  python tests/golden/make_ref_schema.py
The JSON is data (a config section and a key list); the tests read it without /root/reference.
"""

import json
import os

import torch
import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def main():
    with open(os.path.join(REF, "config", "experiment-lengthscales.yaml")) as f:
        cfg = yaml.safe_load(f)
    blob = torch.load(os.path.join(REF, "data", "shared", "gp-problem", "lengthscales", "0.pt"), weights_only=True)
    keys = {k: list(v.shape) for k, v in blob["model_state_dict"].items()}
    out = {"source": {"model": "config/experiment-lengthscales.yaml: model",
                      "state_dict_keys": "data/shared/gp-problem/lengthscales/0.pt: model_state_dict"},
           "model": cfg["model"], "state_dict_keys": keys}
    with open(os.path.join(HERE, "ref_schema.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
