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


def test_iclr2018_figure_analyses_on_synthetic_votes(tmp_path):
    """rdp_cumulative / rdp_bucketized / plot_ls_q / utility_queries_answered equivalents (synthetic votes: no
    network for the paper's vote files). The vectorised cumulative eps must equal eps computed prefix by prefix
    with compute_eps_from_delta."""
    import numpy as np

    from mifx.privacy.pate import iclr2018_figures as F
    from mifx.privacy.pate import rdp2018 as core
    from mifx.privacy.pate.iclr2018 import synthetic_votes

    votes = synthetic_votes(60, 250, 10, seed=3)
    for mech, kw in (("lnmax", {}), ("gnmax", {}), ("gnmax_conf", {"threshold": 200.0, "sigma1": 150.0})):
        res = F.cumulative_privacy(votes, mech, 50.0 if mech == "lnmax" else 40.0, **kw)
        q = F.per_query_rdp(votes, mech, 50.0 if mech == "lnmax" else 40.0, kw.get("threshold"), kw.get("sigma1"))
        for i in (0, 17, 59):
            eps, order = core.compute_eps_from_delta(F.ORDERS, q["rdp"][: i + 1].sum(0), 1e-8)
            assert abs(res["eps"][i] - eps) < 1e-9 * max(1.0, eps) and res["order_opt"][i] == order
        assert np.all(np.diff(res["eps"]) >= -1e-12)  # costs only accumulate
        np.testing.assert_allclose(res["partition"].sum(1), 1.0, rtol=1e-9)
        if mech != "gnmax_conf":
            assert res["answered"][-1] == 60
        else:
            assert 0 < res["answered"][-1] < 60
    b = F.bucketized(votes, 5, 200.0, 150.0, 40.0, 50.0)
    assert b["counts"].sum() == 60 and np.all(b["expected_answered"] <= b["counts"] + 1e-9)
    ls = F.ls_of_q(num=50)
    assert 0 < ls["q1"] <= ls["q0"] < 1 and np.all(ls["ls"] >= 0)
    u = F.UTILITY_QUERIES_ANSWERED
    assert all(len(v["answered"]) == len(v["accuracy"]) for v in u.values())
    assert u["gnmax_conf"]["answered"][-1] == 10842 and u["gnmax_conf"]["accuracy"][-1] == 75.4
    assert F.main(["--queries", "40", "--figures-dir", str(tmp_path)]) == 0
    assert (tmp_path / "iclr2018_figures.json").exists()
