"""ICLR-2018 PATE analysis driver (smooth_sensitivity_table.py semantics)."""
import numpy as np

from mifx.privacy.pate import iclr2018 as m


def test_synthetic_votes_shape_and_totals():
    v = m.synthetic_votes(50, 250, 10, 0.9, seed=1)
    assert v.shape == (50, 10) and m.count_teachers(v) == 250


def test_data_dependent_beats_data_independent_and_ss_costs_extra(tmp_path):
    v = m.synthetic_votes(120, 250, 10, 0.95, seed=0)
    dd = m.analyze(v, None, 200.0, 150.0, 40.0, 1e-5, log=None)
    di = m.analyze(v, None, 200.0, 150.0, 40.0, 1e-5, data_independent=True, log=None)
    assert di["data_independent"] and not dd["data_independent"]
    assert dd["eps"] < di["eps"]
    assert 0 < dd["answered"] < 120
    ss = dd["smooth_sensitivity"]
    assert dd["conditions_hold"] and ss["eps_with_ss"] > ss["eps_before_ss"] > 0
    # counts-file CLI path (np.load without pickle)
    np.save(tmp_path / "votes.npy", v)
    r = m.main(["--counts_file", str(tmp_path / "votes.npy"), "--threshold", "200", "--sigma1", "150",
                "--sigma2", "40", "--queries", "60", "--delta", "1e-5"])
    assert r["rows"][-1]["queries"] == 60


def test_plain_gnmax_has_no_threshold_step():
    v = m.synthetic_votes(40, 100, 10, 0.97, seed=3)
    r = m.analyze(v, None, None, None, 20.0, 1e-5, check_conditions=False, log=None)
    assert abs(r["answered"] - 40) < 1e-9
