"""bench.py's algorithmic cost models against the figures SURVEY.md §8(d) / BASELINE.md state for them
(CPU only: the models are arithmetic)."""

import importlib.util
import os

HERE = os.path.dirname(os.path.abspath(__file__))


def _bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(os.path.dirname(HERE), "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_survey_model_matches_survey_figures():
    b = _bench()
    # headline: m=2, n=256, N=1024, S=16, B=128, d=2 -> 1.53 MFLOP per KG-eval, 5.29 MB per batch
    f, by = b.survey_model(2, [256, 256], 1024, 16, 128, 2)
    assert abs(f / 128 - 1.527e6) / 1.527e6 < 1e-3
    assert abs(by - 5.287e6) / 5.287e6 < 1e-3
    # small: 0.11 MFLOP per eval; stress: 33.8 MFLOP per eval
    f_small, _ = b.survey_model(2, [64, 64], 256, 8, 32, 2)
    assert abs(f_small / 32 - 0.11e6) / 0.11e6 < 0.05
    f_stress, _ = b.survey_model(3, [1024] * 3, 4096, 32, 256, 2)
    assert abs(f_stress / 256 - 33.8e6) / 33.8e6 < 0.01
    # the headline forward's fp64 floor: max(F/78.6 TF, bytes/8 TB/s) ~ 2.49 us
    t_min = max(f / 78.6e12, by / 8e12)
    assert 2.4e-6 < t_min < 2.6e-6


def test_stage_model_matches_design_table():
    """DESIGN.md §4's per-launch table: 17.9 / 137.9 / 21.0 MFLOP at the headline."""
    b = _bench()

    class W:
        m, S, d = 2, 16, 2

    st = b.stage_model(W, 2, [256, 256], 1024, 128, 16, 2)
    assert abs(st["cross_root_kernel"][0] / 1e6 - 17.9) < 0.1
    assert abs(st["posterior_cov_kernel"][0] / 1e6 - 137.9) < 0.1
    assert abs(st["envelope_kernel"][0] / 1e6 - 21.0) < 0.1


def test_default_run_is_whole_graph_periods(monkeypatch):
    """The default bench line: four launch streams, one single-stream graph per stream replayed (graph
    mode 2), a step count that is a whole number of exchange periods (no timed step falls back to eager
    launches), and batches per launch that divide the period."""
    b = _bench()
    monkeypatch.setattr("sys.argv", ["bench.py"])
    a = b.parse()
    assert a.gpus == 1 and a.streams == 4 and a.graph == 2
    assert a.steps % a.exchange_every == 0
    assert b.batches_per_launch(a.exchange_every, a) == 32


def test_batches_per_launch_divides_the_period(monkeypatch):
    """Auto batches per launch: the largest divisor of the exchange period E that gives every stream a
    launch of its own, at most 32 (the driver's --steps 20: E = 20, four streams of 5 batches each)."""
    b = _bench()
    for argv, E, want in ((["bench.py", "--steps", "20"], 20, 5), (["bench.py", "--streams", "2"], 20, 10),
                          (["bench.py", "--streams", "4"], 256, 32),
                          (["bench.py", "--streams", "3"], 20, 5), (["bench.py", "--streams", "1"], 7, 7),
                          (["bench.py", "--batches-per-launch", "4"], 20, 4),
                          # an explicit G under a leg whose period it does not divide (headline_nd's E = 256 under
                          # the driver-shaped --steps 20 --batches-per-launch 5): that leg's largest divisor below it
                          (["bench.py", "--steps", "20", "--batches-per-launch", "5"], 256, 4),
                          (["bench.py", "--steps", "20", "--batches-per-launch", "5"], 20, 5),
                          (["bench.py", "--batches-per-launch", "64"], 16, 16)):
        monkeypatch.setattr("sys.argv", argv)
        a = b.parse()
        g = b.batches_per_launch(E, a)
        assert g == want and E % g == 0
