"""The reference's on-disk result and checkpoint formats (``pipeline/data_catalog.py``), for the
SMOKE_TEST BO loop on the device KG (``dkg_amd.bo_smoke``).

Same directory layout, file names and payloads as ``DataCatalog``, so a run written here is read
by the reference's own loaders and post-processing, and a run the reference wrote is read here:

* ``<data_dir>/<namespace>/config.yaml`` / ``commandline_args.json``        (``:143-160``)
* ``true_pareto.npz``, ``max_possible_scalarisation_metric.npy``            (``:162-182``)
* ``initial_data.pt``, ``hyperparameters.pt``, ``scalarisations.pt``         (``:184-228``)
* ``bo_runs/bo_run_<run_key>.pqt``  (the query history, parquet)            (``:230-240``)
* ``posterior_pareto/<run_key>/posterior_pareto_NN.npz``                    (``:242-315``)
* ``checkpoints/<run_key>/checkpoint_NN.pt`` and ``checkpoints-<run_key>.tgz`` (``:317-420``)
* ``metrics/metrics_<run_key>.pqt``, ``timings/timings_<run_key>.pqt``      (``:422-445``)
* ``<data_dir>/shared/gp-problem/<name>.pt``  (the shared GP test problems)  (``:47-116``)

Differences, all on the reading side: every ``torch.load`` here is ``weights_only=True`` (tensors,
dicts, lists and plain values only; nothing in the file is executed), and the data root is an
argument (default ``$DKG_DATA_DIR`` or ``./data``) instead of the reference's checkout-relative
``DATA_DIR``.
"""

from __future__ import annotations

import json
import os
import re
import shutil
import tarfile
from datetime import datetime
from typing import Any, Dict, List, Optional, Tuple, Union

import numpy as np
import torch
import yaml
from torch import Tensor

SHARED_DNAME = "shared"
GP_PROBLEM_DNAME = "gp-problem"
GP_PROBLEM_FNAME_FMT = "{name}.pt"
LOGS_DNAME = "logs"
COMMANDLINE_ARGS_FNAME = "commandline_args.json"
CONFIG_FNAME = "config.yaml"
TRUE_PARETO_FNAME = "true_pareto.npz"
MAX_SCALARISED_PERFORMANCE_FNAME = "max_possible_scalarisation_metric.npy"
INITIAL_DATA_FNAME = "initial_data.pt"
HYPERPARAMETERS_FNAME = "hyperparameters.pt"
SCALARISATIONS_FNAME = "scalarisations.pt"
BO_RUN_DNAME = "bo_runs"
BO_RUN_FNAME_FMT = "bo_run_{run_key}.pqt"
POSTERIOR_PARETO_DNAME = "posterior_pareto"
POSTERIOR_PARETO_FNAME_FMT = "posterior_pareto_{:02d}.npz"
CHECKPOINTS_DNAME = "checkpoints"
CHECKPOINT_FNAME_FMT = "checkpoint_{:02d}.pt"
CHECKPOINTS_COMPRESSED_FNAME_FMT = "checkpoints-{run_key}.tgz"
METRICS_DNAME = "metrics"
METRICS_FNAME_FMT = "metrics_{run_key}.pqt"
TIMINGS_DNAME = "timings"
TIMINGS_FNAME_FMT = "timings_{run_key}.pqt"


def default_data_dir() -> str:
    return os.environ.get("DKG_DATA_DIR", os.path.join(os.getcwd(), "data"))


def _load(fpath: str, device=None):
    return torch.load(fpath, map_location=device, weights_only=True)


def _numbered(dpath: str, fmt: str, what: str) -> int:
    """How many files ``fmt.format(0..k-1)`` the directory holds; anything else in it is an error
    (the reference's ``num_checkpoints`` / ``num_posterior_pareto_iterations`` check)."""
    if not os.path.isdir(dpath):
        return 0
    fnames = os.listdir(dpath)
    if sorted(fnames) != sorted(fmt.format(i) for i in range(len(fnames))):
        raise ValueError(f"Found unexpected file names in {what}")
    return len(fnames)


class DataCatalog:
    """One run namespace under ``data_dir`` (``data_catalog.py:45``)."""

    def __init__(self, namespace: Optional[str] = None, data_dir: Optional[str] = None):
        if not namespace:
            namespace = datetime.now().strftime("%Y-%m-%dT%H-%M-%S")
        if namespace.split("/", maxsplit=1)[0] == SHARED_DNAME:
            raise ValueError(f"The namespace {SHARED_DNAME!r} is reserved for shared data.")
        self.namespace = namespace
        self.data_dir = os.path.normpath(data_dir or default_data_dir())

    # -- shared GP test problems (data_catalog.py:47-116)
    @classmethod
    def save_shared_gp_test_problem_data(cls, name: str, bounds, fixed_hyperparams: Dict[str, Any],
                                         model_state_dict: Dict[str, Any], train_x: Tensor, train_y: Tensor,
                                         ref_point, max_hv: float, negate: bool, data_dir: Optional[str] = None):
        fpath = os.path.join(data_dir or default_data_dir(), SHARED_DNAME, GP_PROBLEM_DNAME,
                             GP_PROBLEM_FNAME_FMT.format(name=name))
        os.makedirs(os.path.dirname(fpath), exist_ok=True)  # names may hold '/' (repeated instances)
        torch.save({"bounds": bounds, "fixed_hyperparams": fixed_hyperparams, "model_state_dict": model_state_dict,
                    "train_x": train_x, "train_y": train_y, "ref_point": ref_point, "max_hv": max_hv,
                    "negate": negate}, fpath)

    @staticmethod
    def load_shared_gp_test_problem_data(name: str, device=None, data_dir: Optional[str] = None) -> Dict[str, Any]:
        return _load(os.path.join(data_dir or default_data_dir(), SHARED_DNAME, GP_PROBLEM_DNAME,
                                  GP_PROBLEM_FNAME_FMT.format(name=name)), device)

    # -- paths
    def _get_path(self, *parts: str) -> str:
        return os.path.join(self.data_dir, self.namespace, *parts)

    def _dir(self, *parts: str) -> str:
        p = self._get_path(*parts)
        os.makedirs(p, exist_ok=True)
        return p

    def get_new_log_file_path(self) -> str:
        dpath = self._dir(LOGS_DNAME)
        idx = [int(m.group(1)) for m in (re.match(r"^run_(\d+).log$", f) for f in os.listdir(dpath)) if m]
        return os.path.join(dpath, f"run_{max(idx, default=-1) + 1:02}.log")

    # -- run configuration (data_catalog.py:143-160)
    def save_config(self, config: Dict[str, Any]) -> None:
        with open(os.path.join(self._dir(), CONFIG_FNAME), "w") as f:
            yaml.dump(config, f, indent=2, default_flow_style=None)

    def load_config(self) -> Dict[str, Any]:
        with open(self._get_path(CONFIG_FNAME)) as f:
            return yaml.safe_load(f)

    def save_commandline_args(self, commandline_args) -> None:
        args = commandline_args if isinstance(commandline_args, dict) else vars(commandline_args)
        with open(os.path.join(self._dir(), COMMANDLINE_ARGS_FNAME), "w") as f:
            json.dump(args, f, indent=2)

    # -- problem-level results (data_catalog.py:162-182)
    def save_true_pareto(self, pareto_set, pareto_front) -> None:
        np.savez(os.path.join(self._dir(), TRUE_PARETO_FNAME), pareto_set=pareto_set, pareto_front=pareto_front)

    def load_true_pareto(self) -> Tuple[np.ndarray, np.ndarray]:
        with np.load(self._get_path(TRUE_PARETO_FNAME)) as z:
            return z["pareto_set"], z["pareto_front"]

    def save_problem_max_possible_expected_scalarisation(self, expected_best: float) -> None:
        np.save(os.path.join(self._dir(), MAX_SCALARISED_PERFORMANCE_FNAME), expected_best)

    def load_problem_max_possible_expected_scalarisation(self) -> float:
        return np.load(self._get_path(MAX_SCALARISED_PERFORMANCE_FNAME)).item()

    # -- shared inputs of the BO runs (data_catalog.py:184-228)
    def save_initial_data(self, train_x, train_obj, train_obj_true) -> None:
        torch.save({"train_x": train_x, "train_obj": train_obj, "train_obj_true": train_obj_true},
                   os.path.join(self._dir(), INITIAL_DATA_FNAME))

    def load_initial_data(self, device=None) -> Dict[str, Any]:
        return _load(self._get_path(INITIAL_DATA_FNAME), device)

    def save_model_hyperparameters(self, model_state_dict: Dict[str, Any]) -> None:
        torch.save(model_state_dict, os.path.join(self._dir(), HYPERPARAMETERS_FNAME))

    def load_model_hyperparameters(self, device=None) -> Dict[str, Any]:
        return _load(self._get_path(HYPERPARAMETERS_FNAME), device)

    def delete_model_hyperparameters(self) -> None:
        fpath = self._get_path(HYPERPARAMETERS_FNAME)
        if os.path.exists(fpath):
            os.remove(fpath)

    def save_scalarisations(self, weights: Tensor) -> None:
        torch.save(weights, os.path.join(self._dir(), SCALARISATIONS_FNAME))

    def load_scalarisations(self, device=None) -> Tensor:
        return _load(self._get_path(SCALARISATIONS_FNAME), device)

    # -- per-run tables (data_catalog.py:230-240, 422-445)
    def _save_table(self, dname: str, fmt: str, run_key: str, df) -> None:
        df.to_parquet(os.path.join(self._dir(dname), fmt.format(run_key=run_key)))

    def _load_table(self, dname: str, fmt: str, run_key: str):
        import pandas as pd

        return pd.read_parquet(self._get_path(dname, fmt.format(run_key=run_key)))

    def save_bo_run(self, run_key: str, query_history_df) -> None:
        self._save_table(BO_RUN_DNAME, BO_RUN_FNAME_FMT, run_key, query_history_df)

    def load_bo_run(self, run_key: str):
        return self._load_table(BO_RUN_DNAME, BO_RUN_FNAME_FMT, run_key)

    def save_metrics(self, run_key: str, metrics_df) -> None:
        self._save_table(METRICS_DNAME, METRICS_FNAME_FMT, run_key, metrics_df)

    def load_metrics(self, run_key: str):
        return self._load_table(METRICS_DNAME, METRICS_FNAME_FMT, run_key)

    def save_timings(self, run_key: str, timings_history_df) -> None:
        self._save_table(TIMINGS_DNAME, TIMINGS_FNAME_FMT, run_key, timings_history_df)

    def load_timings(self, run_key: str):
        return self._load_table(TIMINGS_DNAME, TIMINGS_FNAME_FMT, run_key)

    # -- posterior Pareto fronts per iteration (data_catalog.py:242-315)
    def save_posterior_pareto(self, run_key: str, iteration: int, pareto_set: np.ndarray,
                              pareto_front: np.ndarray) -> None:
        np.savez(os.path.join(self._dir(POSTERIOR_PARETO_DNAME, run_key), POSTERIOR_PARETO_FNAME_FMT.format(iteration)),
                 pareto_set=pareto_set, pareto_front=pareto_front)

    def num_posterior_pareto_iterations(self, run_key: str) -> int:
        return _numbered(self._get_path(POSTERIOR_PARETO_DNAME, run_key), POSTERIOR_PARETO_FNAME_FMT,
                         f"{POSTERIOR_PARETO_DNAME!r} directory")

    def load_posterior_pareto(self, run_key: str, iteration: int) -> Tuple[np.ndarray, np.ndarray]:
        if iteration < 0:  # -1 is the last iteration
            iteration += self.num_posterior_pareto_iterations(run_key)
        with np.load(self._get_path(POSTERIOR_PARETO_DNAME, run_key,
                                    POSTERIOR_PARETO_FNAME_FMT.format(iteration))) as z:
            return z["pareto_set"], z["pareto_front"]

    def delete_all_posterior_pareto(self) -> None:
        dpath = self._get_path(POSTERIOR_PARETO_DNAME)
        if os.path.isdir(dpath):
            shutil.rmtree(dpath)

    # -- checkpoints (data_catalog.py:317-420)
    def save_checkpoint(self, run_key: str, iteration: int, model_state_dict: Dict[str, Any],
                        model_config: Dict[str, Any], train_x: List[Union[Tensor, np.ndarray]],
                        train_obj: List[Union[Tensor, np.ndarray]], train_obj_true: List[Union[Tensor, np.ndarray]],
                        problem_bounds: Tensor) -> None:
        """Enough to resume the run: the surrogate's hyperparameters and every observation so far."""
        torch.save({"run_key": run_key, "iteration": iteration, "model_state_dict": model_state_dict,
                    "model_config": model_config, "train_x": train_x, "train_obj": train_obj,
                    "train_obj_true": train_obj_true, "problem_bounds": problem_bounds},
                   os.path.join(self._dir(CHECKPOINTS_DNAME, run_key), CHECKPOINT_FNAME_FMT.format(iteration)))

    def num_checkpoints(self, run_key: str) -> int:
        return _numbered(self._get_path(CHECKPOINTS_DNAME, run_key), CHECKPOINT_FNAME_FMT, "checkpoints directory")

    def load_checkpoint(self, run_key: str, iteration: int, device=None) -> Dict[str, Any]:
        n = self.num_checkpoints(run_key)
        if n == 0:
            raise RuntimeError("No checkpoints! Did you forget to uncompress them?")
        if iteration < 0:  # -1 is the last checkpoint
            iteration += n
        if iteration < 0:
            raise IndexError("checkpoint index out of range")
        return _load(self._get_path(CHECKPOINTS_DNAME, run_key, CHECKPOINT_FNAME_FMT.format(iteration)), device)

    def compress_checkpoints(self, run_key: str) -> None:
        src = self._get_path(CHECKPOINTS_DNAME, run_key)
        dst = self._get_path(CHECKPOINTS_DNAME, CHECKPOINTS_COMPRESSED_FNAME_FMT.format(run_key=run_key))
        with tarfile.open(dst, "w:gz") as f:
            f.add(src, arcname="")
        shutil.rmtree(src)

    def uncompress_checkpoints(self, run_key: str) -> None:
        dst = self._get_path(CHECKPOINTS_DNAME, run_key)
        src = self._get_path(CHECKPOINTS_DNAME, CHECKPOINTS_COMPRESSED_FNAME_FMT.format(run_key=run_key))
        if os.path.exists(dst):
            raise FileExistsError(dst)
        with tarfile.open(src, "r:gz") as f:
            members = [m for m in f.getmembers() if m.isfile() or m.isdir()]
            for m in members:  # only plain files and directories, none outside the target
                if os.path.isabs(m.name) or ".." in m.name.split("/"):
                    raise ValueError(f"unsafe path in checkpoint archive: {m.name!r}")
            f.extractall(dst, members=members)
        os.remove(src)

    def delete_all_checkpoints(self) -> None:
        dpath = self._get_path(CHECKPOINTS_DNAME)
        if os.path.isdir(dpath):
            shutil.rmtree(dpath)
