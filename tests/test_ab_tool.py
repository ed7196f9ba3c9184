"""tools/ab.sh (the same-box A/B runner): variants alternate, env / relative-path / DIR handling, JSONL record,
and a failing run stops the comparison. CPU only (the command under test is a tiny Python one-liner)."""
import json
import os
import subprocess
import sys

import pytest

AB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools", "ab.sh")
EMIT = ("import os, json; print('noise'); print(json.dumps({'ms_per_step': 1.5, 'loss': os.environ.get('FOO'), "
        "'lib': os.environ.get('MIFX_LIB_X'), 'cwd': os.getcwd()}))")


def _run(cwd, *args):
    return subprocess.run(["bash", AB, *args], cwd=cwd, capture_output=True, text=True, timeout=60)


def test_ab_alternates_variants_and_records_jsonl(tmp_path):
    (tmp_path / "lib.so").write_text("")
    other = tmp_path / "other"
    other.mkdir()
    r = _run(tmp_path, "-n", "2", "-o", "t", "a", "b=FOO=1,MIFX_LIB_X=lib.so", f"c=DIR={other}",
             "--", sys.executable, "-c", EMIT)
    assert r.returncode == 0, r.stderr
    recs = [json.loads(l) for l in (tmp_path / "gpurun_out" / "ab_t.jsonl").read_text().splitlines()]
    assert [(x["variant"], x["run"]) for x in recs] == [("a", 1), ("b", 1), ("c", 1), ("a", 2), ("b", 2), ("c", 2)]
    a, b, c = recs[:3]
    assert a["result"]["loss"] is None and b["result"]["loss"] == "1"
    assert b["result"]["lib"] == str(tmp_path / "lib.so")          # relative path made absolute
    assert c["result"]["cwd"] == str(other) and c["result"]["loss"] is None
    assert "a 1 ms/step=1.5" in r.stdout
    assert (tmp_path / "gpurun_out" / "ab_t_b2.log").exists()


@pytest.mark.parametrize("cmd", [["false"], [sys.executable, "-c", "print('no json')"]])
def test_ab_stops_on_failure(tmp_path, cmd):
    r = _run(tmp_path, "-n", "3", "x", "y=FOO=2", "--", *cmd)
    assert r.returncode != 0
    assert "y run 1" not in r.stdout


def test_ab_usage_errors(tmp_path):
    assert _run(tmp_path, "--", "true").returncode == 2
    assert _run(tmp_path, "a").returncode == 2
