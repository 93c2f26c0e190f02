"""DataCatalog formats (dkg_amd.catalog, the reference's pipeline/data_catalog.py layout): CPU only."""

import os
import tarfile

import numpy as np
import pandas as pd
import pytest
import torch

from dkg_amd.catalog import DataCatalog
from dkg_amd.model import ModelListGPState, SingleTaskGPState, from_state_dict, to_state_dict

REF_DATA = "/root/reference/data"


def _model():
    g = torch.Generator().manual_seed(3)
    x = [torch.rand(7, 2, generator=g, dtype=torch.double), torch.rand(5, 2, generator=g, dtype=torch.double)]
    y = [torch.randn(7, generator=g, dtype=torch.double), torch.randn(5, generator=g, dtype=torch.double)]
    return ModelListGPState(
        SingleTaskGPState(x[0], y[0], torch.tensor([0.2, 0.7], dtype=torch.double), 1.5, 1e-8, 0.3),
        SingleTaskGPState(x[1], y[1], torch.tensor([1.8, 0.05], dtype=torch.double), 50.0, 1e-4, -0.1,
                          y_mean=2.0, y_std=3.0))


def test_state_dict_round_trip():
    m = _model()
    sd = to_state_dict(m)
    assert sd["models.0.covar_module.base_kernel.raw_lengthscale"].shape == (1, 2)
    assert "models.1.outcome_transform.means" in sd and "models.0.outcome_transform.means" not in sd
    y_problem = [st.train_y * st.y_std + st.y_mean for st in m.models]
    m2 = from_state_dict(sd, [st.train_x for st in m.models], y_problem, noise_constraint="raw")
    for a, b in zip(m.models, m2.models):
        assert torch.allclose(a.lengthscale, b.lengthscale, rtol=1e-15, atol=0)
        assert a.outputscale == pytest.approx(b.outputscale, rel=1e-15)
        assert (a.noise, a.mean_constant, a.y_mean, a.y_std) == (b.noise, b.mean_constant, b.y_mean, b.y_std)
        assert torch.allclose(a.train_y, b.train_y, rtol=0, atol=1e-15)


def test_namespace_rules(tmp_path):
    with pytest.raises(ValueError, match="reserved for shared data"):
        DataCatalog("shared/x", data_dir=str(tmp_path))
    assert DataCatalog(data_dir=str(tmp_path)).namespace  # timestamp namespace
    c = DataCatalog("ns", data_dir=str(tmp_path))
    assert c.get_new_log_file_path().endswith("run_00.log")
    open(c.get_new_log_file_path(), "w").close()
    assert c.get_new_log_file_path().endswith("run_01.log")


def test_files_round_trip(tmp_path):
    c = DataCatalog("exp/a", data_dir=str(tmp_path))
    c.save_config({"model": {"fit_hyperparams": "never"}, "seed": 3})
    assert c.load_config() == {"model": {"fit_hyperparams": "never"}, "seed": 3}
    c.save_commandline_args({"smoke_test": True})
    assert os.path.exists(c._get_path("commandline_args.json"))
    ps, pf = np.random.rand(4, 2), np.random.rand(4, 2)
    c.save_true_pareto(ps, pf)
    a, b = c.load_true_pareto()
    assert np.array_equal(a, ps) and np.array_equal(b, pf)
    c.save_problem_max_possible_expected_scalarisation(0.25)
    assert c.load_problem_max_possible_expected_scalarisation() == 0.25
    tx = [torch.rand(3, 2, dtype=torch.double)]
    c.save_initial_data(tx, [torch.rand(3)], [torch.rand(3)])
    assert torch.equal(c.load_initial_data()["train_x"][0], tx[0])
    sd = to_state_dict(_model())
    c.save_model_hyperparameters(sd)
    assert all(torch.equal(v, c.load_model_hyperparameters()[k]) for k, v in sd.items())
    c.delete_model_hyperparameters()
    assert not os.path.exists(c._get_path("hyperparameters.pt"))
    w = torch.rand(2, 4, 2, dtype=torch.double)
    c.save_scalarisations(w)
    assert torch.equal(c.load_scalarisations(), w)
    df = pd.DataFrame({"iteration": [0, 1], "x": [np.zeros(2), np.ones(2)], "obj_index": [0, 1],
                       "acq_per_cost": [float("nan"), 0.5], "scalarisation": [None, np.array([0.3, 0.7])]})
    c.save_bo_run("eval_full", df)
    back = c.load_bo_run("eval_full")
    assert list(back.columns) == list(df.columns) and np.array_equal(back["x"][1], np.ones(2))
    assert os.path.basename(c._get_path("bo_runs", "bo_run_eval_full.pqt")) in os.listdir(c._get_path("bo_runs"))
    c.save_metrics("eval_full", pd.DataFrame({"hv": [1.0]}))
    c.save_timings("eval_full", pd.DataFrame({"bo": [0.1]}))
    assert c.load_metrics("eval_full")["hv"][0] == 1.0 and c.load_timings("eval_full")["bo"][0] == 0.1
    for it in range(3):
        c.save_posterior_pareto("eval_full", it, ps + it, pf)
    assert c.num_posterior_pareto_iterations("eval_full") == 3
    assert np.array_equal(c.load_posterior_pareto("eval_full", -1)[0], ps + 2)
    c.delete_all_posterior_pareto()
    assert c.num_posterior_pareto_iterations("eval_full") == 0


def test_checkpoints(tmp_path):
    c = DataCatalog("ns", data_dir=str(tmp_path))
    with pytest.raises(RuntimeError, match="No checkpoints"):
        c.load_checkpoint("eval_separate", 0)
    m = _model()
    for it in range(3):
        c.save_checkpoint("eval_separate", it, to_state_dict(m), {"fit_hyperparams": "never"},
                          [st.train_x for st in m.models], [st.train_y for st in m.models],
                          [st.train_y for st in m.models], torch.tensor([[0.0, 0.0], [1.0, 1.0]]))
    assert c.num_checkpoints("eval_separate") == 3
    assert os.listdir(c._get_path("checkpoints", "eval_separate")).count("checkpoint_02.pt") == 1
    last = c.load_checkpoint("eval_separate", -1)
    assert last["iteration"] == 2 and last["run_key"] == "eval_separate"
    with pytest.raises(IndexError):
        c.load_checkpoint("eval_separate", -4)
    c.compress_checkpoints("eval_separate")
    assert c.num_checkpoints("eval_separate") == 0
    assert os.path.exists(c._get_path("checkpoints", "checkpoints-eval_separate.tgz"))
    c.uncompress_checkpoints("eval_separate")
    assert c.num_checkpoints("eval_separate") == 3
    with pytest.raises(FileExistsError):
        c.uncompress_checkpoints("eval_separate")
    # a stray file breaks the numbering check, as in the reference
    open(c._get_path("checkpoints", "eval_separate", "junk"), "w").close()
    with pytest.raises(ValueError, match="unexpected file names"):
        c.num_checkpoints("eval_separate")
    c.delete_all_checkpoints()
    assert c.num_checkpoints("eval_separate") == 0


def test_unsafe_archive_is_refused(tmp_path):
    c = DataCatalog("ns", data_dir=str(tmp_path))
    os.makedirs(c._get_path("checkpoints"))
    evil = tmp_path / "evil.txt"
    evil.write_text("x")
    with tarfile.open(c._get_path("checkpoints", "checkpoints-k.tgz"), "w:gz") as f:
        f.add(str(evil), arcname="../../evil.txt")
    with pytest.raises(ValueError, match="unsafe path"):
        c.uncompress_checkpoints("k")


@pytest.mark.skipif(not os.path.isdir(REF_DATA), reason="reference data not present")
def test_reads_the_reference_shared_gp_problem():
    """The reference's own shared GP problem file, read with weights_only=True (nothing executed)."""
    prob = DataCatalog.load_shared_gp_test_problem_data("lengthscales/0", data_dir=REF_DATA)
    assert {"bounds", "fixed_hyperparams", "model_state_dict", "train_x", "train_y"} <= set(prob)
    m = from_state_dict(prob["model_state_dict"], prob["train_x"], prob["train_y"], bounds=None)
    assert m.num_outputs == len(prob["bounds"]) or m.num_outputs >= 1


SCHEMA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ref_schema.json")


def test_checkpoint_model_config_is_the_reference_schema():
    """The SMOKE loop's checkpoint config is the reference's ``model`` section of
    config/experiment-lengthscales.yaml as cli.py:22-37 completes it for --fit-hyperparams never (the fixture
    tests/golden/ref_schema.json, made by make_ref_schema.py): what build_mll_and_model reads."""
    import copy
    import json

    from dkg_amd.bo_smoke import reference_model_config

    ref = copy.deepcopy(json.load(open(SCHEMA))["model"])
    ref["fit_hyperparams"] = "never"
    for o in ref["outputs"]:
        o["standardize_output"] = False
    assert reference_model_config(2, torch.tensor([[0.0, 0.0], [1.0, 1.0]])) == ref


def test_checkpoint_state_dict_has_the_reference_key_set():
    """Every key (and shape) of a reference-built ModelListGP state dict (the reference's own GP-problem
    fixture) is in the checkpointed state dict, with the never-path noise floor as the constraint's lower
    bound (factory.py:41-43, 95-104); the only extra keys are the config's Gamma priors' buffers."""
    import json

    from dkg_amd.bo_smoke import reference_model_config

    ref = json.load(open(SCHEMA))["state_dict_keys"]
    g = torch.Generator().manual_seed(4)
    m = ModelListGPState(*[SingleTaskGPState(torch.rand(6, 2, generator=g, dtype=torch.double),
                                             torch.randn(6, generator=g, dtype=torch.double),
                                             torch.tensor([0.2, 1.8], dtype=torch.double), 1.0, 1e-8, 0.0)
                           for _ in range(2)])
    sd = to_state_dict(m, reference_model_config(2, torch.tensor([[0.0, 0.0], [1.0, 1.0]])))
    for k, shape in ref.items():
        assert k in sd, k
        assert list(sd[k].shape) == shape, k
    assert all("_prior." in k for k in set(sd) - set(ref))
    assert float(sd["models.0.likelihood.noise_covar.raw_noise_constraint.lower_bound"]) == 1e-8
    assert float(sd["likelihood.likelihoods.1.noise_covar.raw_noise"]) == 1e-8
    assert float(sd["models.0.covar_module.base_kernel.lengthscale_prior.rate"]) == 10.0
    m2 = from_state_dict(sd, [st.train_x for st in m.models], [st.train_y for st in m.models],
                         noise_constraint="raw")
    assert [st.noise for st in m2.models] == [1e-8, 1e-8]
