"""The SMOKE_TEST pipeline path on the device KG (dkg_amd.bo_smoke; reference pipeline/main.py:171-216,
bo_loop.py:48-59, 122-131, 380-450): the gp-sample problem lengthscales/0 (the committed golden
fixture, tests/golden/make_golden.py) with the reference's fixed hyperparameters (main.py:84-88)."""

import pytest
import torch

import json
import os

from dkg_amd.bo_smoke import GPProblem, run_smoke
from helpers import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
HYPER = dict(length_scales=[0.2, 1.8], output_scales=[1, 50], means=[0, 0])


def test_problem_objective_is_posterior_mean():
    """gp_testproblem.py:76-98: objective i = posterior mean of the problem GP's output i."""
    state, om, D, W, X, _ = load_golden("lengthscales0")
    problem = GPProblem(state, device=DEV)
    got = problem(X)
    ref = torch.stack([p[0] for p in om.posterior_list(X, observation_noise=False)], dim=-1)
    torch.testing.assert_close(got, ref, rtol=1e-9, atol=1e-9 * float(ref.abs().max()))


def test_smoke_pipeline_runs_both_modes():
    state, *_ = load_golden("lengthscales0")
    problem = GPProblem(state, device=DEV)
    res = run_smoke(problem, HYPER, seed=0)
    sep, full = res["separate"], res["full"]
    for h in (sep, full):
        assert len(h["x"]) == 2
        assert all(0.0 <= v <= 1.0 for x in h["x"] for v in x)
        assert all(a == a for a in h["acq"])  # finite acquisition values
    # decoupled: one objective per step, appended to that objective's data only (costs [1, 10])
    assert all(i in (0, 1) for i in sep["obj_index"])
    assert all(a > 0.0 for a in sep["acq"] + full["acq"])
    assert sum(sep["n_observations"]) == 2 * 6 + 2
    assert all(c == (1.0 if i == 0 else 10.0) for i, c in zip(sep["obj_index"], sep["cost"]))
    # full: every objective at every step
    assert full["n_observations"] == [8, 8]
    # deterministic under the seed
    again = run_smoke(GPProblem(state, device=DEV), HYPER, seed=0)
    assert again["full"]["x"] == full["x"] and again["separate"]["x"] == sep["x"]


def test_smoke_pipeline_writes_the_reference_catalog(tmp_path):
    """With a DataCatalog the loop writes the reference's files (data_catalog.py layout): the query history
    table in the reference's columns, one checkpoint per iteration (compressed at the end), and the
    checkpointed state dict rebuilds the surrogate the loop used (same KG on the device)."""
    from dkg_amd import DiscreteKnowledgeGradient
    from dkg_amd.bo_smoke import QUERY_COLUMNS, surrogate
    from dkg_amd.catalog import DataCatalog
    from dkg_amd.model import from_state_dict

    state, *_ = load_golden("lengthscales0")
    cat = DataCatalog("smoke", data_dir=str(tmp_path))
    res = run_smoke(GPProblem(state, device=DEV), HYPER, seed=0, catalog=cat)
    plain = run_smoke(GPProblem(state, device=DEV), HYPER, seed=0)
    assert res["full"]["x"] == plain["full"]["x"] and res["separate"]["x"] == plain["separate"]["x"]
    for key, mode in (("eval_separate", "separate"), ("eval_full", "full")):
        df = cat.load_bo_run(key)
        assert tuple(df.columns) == QUERY_COLUMNS
        n_new = 2 if mode == "separate" else 2 * 2
        assert len(df) == 2 * 6 + n_new and int(df["init"].sum()) == 12
        assert df["iteration"].max() == 2
        cat.uncompress_checkpoints(key)
        assert cat.num_checkpoints(key) == 3
        ck = cat.load_checkpoint(key, -1)
        assert ck["iteration"] == 2 and ck["model_config"]["fit_hyperparams"] == "never"
        assert [int(t.shape[0]) for t in ck["train_x"]] == res[mode]["n_observations"]
        rebuilt = from_state_dict(ck["model_state_dict"], ck["train_x"], ck["train_obj"], noise_constraint="raw")
        direct = surrogate(ck["train_x"], ck["train_obj"], HYPER)
        D = torch.rand(64, 2, dtype=torch.double, generator=torch.Generator().manual_seed(1))
        W = torch.tensor([[0.3, 0.7], [0.6, 0.4]], dtype=torch.double)
        Xc = torch.rand(8, 1, 2, dtype=torch.double, generator=torch.Generator().manual_seed(2))
        kg_a = DiscreteKnowledgeGradient(rebuilt, D, W)(Xc.to(DEV))
        kg_b = DiscreteKnowledgeGradient(direct, D, W)(Xc.to(DEV))
        torch.testing.assert_close(kg_a, kg_b, rtol=1e-9, atol=1e-15)


@pytest.mark.parametrize("seed", [0, 1])
def test_smoke_pipeline_matches_the_oracle_run(seed):
    """The device SMOKE loop against the same loop on the CPU oracle (tests/smoke_oracle.py; decisions
    committed in tests/golden/smoke_oracle.json by make_smoke_oracle.py): at every BO step of both runs the
    same objective is chosen (decoupled), the candidate agrees within the optimiser's tolerance (L-BFGS-B
    stops at a relative decrease of 2.2e-9: |dx| ~ sqrt(2 * 2.2e-9 / curvature) ~ 1e-4; two oracle runs
    on different BLAS thread splits already differ by 1e-8) and the acquisition value within 1e-6 relative
    plus the 1e-8 an x that far from the optimum can cost."""
    want = json.load(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                                       "smoke_oracle.json")))["seeds"][str(seed)]
    state, *_ = load_golden("lengthscales0")
    got = run_smoke(GPProblem(state, device=DEV), HYPER, seed=seed)
    for mode in ("separate", "full"):
        g, w = got[mode], want[mode]
        assert g["obj_index"] == w["obj_index"], mode
        for x, xr in zip(g["x"], w["x"]):
            assert x == pytest.approx(xr, abs=1e-4), (mode, x, xr)
        assert g["acq"] == pytest.approx(w["acq"], rel=1e-6, abs=1e-8), mode
        assert all(a > 0 for a in g["acq"])
