"""Seldon-style inference graphs: A/B split, epsilon-greedy bandit learning from feedback,
Mahalanobis outlier transformer, REST protocol."""
import numpy as np
from fastapi.testclient import TestClient

from mifx.serving.graph import GraphServer, build_graph, create_app, predictor_graph

A = lambda x: np.tile([1.0, 0.0], (len(x), 1))  # noqa: E731
B = lambda x: np.tile([0.0, 1.0], (len(x), 1))  # noqa: E731


def _ab_deployment(ratio):
    return {"spec": {"predictors": [{"graph": {
        "name": "random-ab-test", "endpoint": {}, "implementation": "RANDOM_ABTEST",
        "parameters": [{"name": "ratioA", "value": str(ratio), "type": "FLOAT"}],
        "children": [{"name": "classifier-1", "type": "MODEL", "endpoint": {"type": "REST"}},
                     {"name": "classifier-2", "type": "MODEL", "endpoint": {"type": "REST"}}]}}]}}


def test_random_abtest_split_ratio_and_routing_meta():
    root = build_graph(predictor_graph(_ab_deployment(0.25)), {"classifier-1": A, "classifier-2": B}, seed=0)
    srv = GraphServer(root)
    hits = [srv.predict({"data": {"ndarray": [[0.0, 1.0]]}})["meta"]["routing"]["random-ab-test"]
            for _ in range(2000)]
    assert abs(hits.count(0) / 2000 - 0.25) < 0.04


def test_epsilon_greedy_converges_to_rewarded_branch():
    g = {"name": "eg-router", "type": "ROUTER",
         "parameters": [{"name": "n_branches", "value": "2", "type": "INT"},
                        {"name": "epsilon", "value": "0.2", "type": "FLOAT"},
                        {"name": "verbose", "value": "false", "type": "BOOL"}],
         "children": [{"name": "classifier-1", "type": "MODEL"}, {"name": "classifier-2", "type": "MODEL"}]}
    srv = GraphServer(build_graph(g, {"classifier-1": A, "classifier-2": B}, seed=1))
    picks = []
    for _ in range(600):
        resp = srv.predict({"data": {"ndarray": [[1.0]]}})
        b = resp["meta"]["routing"]["eg-router"]
        picks.append(b)
        srv.feedback({"request": {}, "response": resp, "reward": 1.0 if b == 1 else 0.0})
    assert np.mean(np.array(picks[-300:]) == 1) > 0.8  # 1 - eps/2 expected


def test_outlier_detector_flags_far_points_and_forwards():
    g = {"name": "outlier-detector", "type": "TRANSFORMER",
         "parameters": [{"name": "threshold", "value": "30", "type": "FLOAT"},
                        {"name": "start_clip", "value": "20", "type": "INT"}],
         "children": [{"name": "clf", "type": "MODEL"}]}
    srv = GraphServer(build_graph(g, {"clf": A}), names=["a", "b"])
    rng = np.random.default_rng(0)
    for _ in range(10):
        srv.predict({"data": {"ndarray": rng.normal(size=(16, 3)).tolist()}})
    r = srv.predict({"data": {"ndarray": [[0.1, -0.2, 0.0], [12.0, -9.0, 15.0]]}})
    assert r["meta"]["tags"]["is-outlier"] == [False, True]
    assert r["data"]["names"] == ["a", "b"] and r["data"]["ndarray"][0] == [1.0, 0.0]


def test_rest_protocol():
    root = build_graph(predictor_graph(_ab_deployment(1.0)), {"classifier-1": A, "classifier-2": B}, seed=0)
    c = TestClient(create_app(GraphServer(root)))
    r = c.post("/api/v0.1/predictions", json={"data": {"tensor": {"shape": [2, 2], "values": [1, 2, 3, 4]}}})
    assert r.status_code == 200 and r.json()["data"]["ndarray"] == [[1.0, 0.0], [1.0, 0.0]]
    fb = c.post("/api/v0.1/feedback", json={"response": r.json(), "reward": 1})
    assert fb.status_code == 200 and fb.json()["meta"]["routing"] == {"random-ab-test": 0}
    assert c.post("/api/v0.1/predictions", json={"data": {}}).status_code == 400
