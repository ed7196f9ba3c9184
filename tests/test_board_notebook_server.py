"""The TensorBoard-role scalar dashboard (mifx.board) and the Jupyter-role notebook server (mifx.notebook_server):
HTTP contracts through FastAPI's test client, on event files written by mifx.utils.summary and on a temporary
notebook directory."""
import os

import pytest

pytest.importorskip("fastapi")
from fastapi.testclient import TestClient  # noqa: E402

from mifx.utils.summary import SummaryWriter  # noqa: E402


def test_board_serves_tensorboard_scalar_routes(tmp_path):
    from mifx.board.server import create_app

    for run, scale in (("train", 1.0), ("eval/chicago-taxi", 2.0)):
        with SummaryWriter(str(tmp_path / run)) as w:
            for s in range(5):
                w.add_scalar("loss", scale / (s + 1), s)
                w.add_scalar("accuracy", 0.5 + 0.1 * s, s)
    c = TestClient(create_app(str(tmp_path)))
    assert c.get("/healthz").json() == {"status": "ok"}
    assert c.get("/data/runs").json() == ["eval/chicago-taxi", "train"]
    tags = c.get("/data/plugin/scalars/tags").json()
    assert set(tags["train"]) == {"loss", "accuracy"}
    rows = c.get("/data/plugin/scalars/scalars", params={"run": "eval/chicago-taxi", "tag": "loss"}).json()
    assert [r[1] for r in rows] == [0, 1, 2, 3, 4]
    assert rows[1][2] == pytest.approx(1.0) and rows[0][0] > 1e9  # [wall_time, step, value]
    assert c.get("/data/plugin/scalars/scalars", params={"run": "nope", "tag": "loss"}).status_code == 404
    page = c.get("/").text
    assert "<svg" in page and "accuracy" in page and "eval/chicago-taxi" in page


def test_notebook_server_lists_shows_and_runs(tmp_path):
    from mifx.notebook_server.server import create_app

    (tmp_path / "n01_hello.py").write_text('"""Hello notebook: prints a sum."""\nprint("sum", 2 + 3)\n')
    (tmp_path / "n02_fail.py").write_text('"""Failing notebook."""\nraise SystemExit(3)\n')
    app = create_app(str(tmp_path), timeout_s=60)
    c = TestClient(app)
    nbs = c.get("/api/notebooks").json()
    assert nbs == [{"name": "n01_hello", "title": "Hello notebook: prints a sum."},
                   {"name": "n02_fail", "title": "Failing notebook."}]
    assert "print(" in c.get("/api/notebooks/n01_hello").json()["source"]
    rid = c.post("/api/notebooks/n01_hello/run").json()["run_id"]
    r = app.state.runner.wait(rid, 60)
    assert r["status"] == "succeeded" and r["returncode"] == 0 and "sum 5" in r["output"]
    rid2 = c.post("/api/notebooks/n02_fail/run").json()["run_id"]
    assert app.state.runner.wait(rid2, 60)["status"] == "failed"
    assert c.get(f"/api/runs/{rid}").json()["status"] == "succeeded"
    assert c.post("/api/notebooks/missing/run").status_code == 404
    # only listed notebooks: a name is never turned into a path from the request
    assert c.post("/api/notebooks/..%2F..%2Fetc%2Fpasswd/run").status_code == 404
    assert c.get("/api/notebooks/_private").status_code == 404
    assert "n01_hello" in c.get("/").text


def test_notebook_server_lists_the_workshop_notebooks():
    from mifx.notebook_server.server import list_notebooks

    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples", "notebooks")
    names = [n["name"] for n in list_notebooks(root)]
    assert len(names) >= 15 and "n16_eager_execution" in names
