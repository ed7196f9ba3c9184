"""Model server (TF-Serving REST semantics), dynamic batching, version policy, tensor store."""
import os
import threading

import numpy as np
import pytest
import torch
from fastapi.testclient import TestClient

from mifx.models.cnn import FashionCNN
from mifx.models.resnet import PREPROCESS_SCRIPT, resnet50_v2
from mifx.serving.saved_model import save_module
from mifx.serving.server import DynamicBatcher, ModelManager, create_app
from mifx.serving.tensorstore import TensorStore


def _export(base, version, seed):
    torch.manual_seed(seed)
    m = FashionCNN()
    save_module(os.path.join(base, str(version)), m, "mifx.models.cnn:FashionCNN", {}, [28, 28],
                class_names=[str(i) for i in range(10)])
    return m


def test_rest_predict_versions_status_metadata(tmp_path):
    base = str(tmp_path / "fashion")
    m1 = _export(base, 1, 1)
    mgr = ModelManager("fashion", base, policy="all", device="cpu", poll_s=0)
    client = TestClient(create_app({"fashion": mgr}))
    x = np.random.default_rng(0).random((3, 28, 28)).astype(np.float32)
    r = client.post("/v1/models/fashion:predict", json={"instances": x.tolist()})
    assert r.status_code == 200
    with torch.no_grad():
        ref = m1(torch.from_numpy(x)).numpy()
    np.testing.assert_allclose(np.array(r.json()["predictions"]), ref, rtol=1e-5, atol=1e-5)
    m2 = _export(base, 2, 2)
    mgr.refresh()
    st = client.get("/v1/models/fashion").json()
    assert [s["version"] for s in st["model_version_status"]] == ["2", "1"]
    r2 = client.post("/v1/models/fashion:predict", json={"instances": x.tolist()}).json()["predictions"]
    with torch.no_grad():
        np.testing.assert_allclose(np.array(r2), m2(torch.from_numpy(x)).numpy(), rtol=1e-5, atol=1e-5)
    r1 = client.post("/v1/models/fashion/versions/1:predict", json={"inputs": x.tolist()}).json()["outputs"]
    np.testing.assert_allclose(np.array(r1), ref, rtol=1e-5, atol=1e-5)
    md = client.get("/v1/models/fashion/metadata").json()
    assert md["model_spec"]["version"] == "2" and "serving_default" in md["metadata"]["signature_def"]
    assert client.post("/v1/models/fashion/versions/7:predict", json={"instances": []}).status_code == 404
    assert client.post("/v1/models/nope:predict", json={"instances": []}).status_code == 404
    cls = client.post("/v1/models/fashion:classify", json={"examples": x.tolist()}).json()["results"]
    assert len(cls) == 3 and len(cls[0]) == 10
    metrics = client.get("/monitoring/prometheus/metrics").text
    assert 'mifx_serving_requests_total{method="predict",model="fashion",status="ok"}' in metrics
    mgr.close()


def test_latest_policy_unloads_old_versions(tmp_path):
    base = str(tmp_path / "m")
    _export(base, 1, 1)
    mgr = ModelManager("m", base, policy="latest", device="cpu", poll_s=0)
    assert list(mgr.servables) == [1]
    _export(base, 5, 5)
    mgr.refresh()
    assert list(mgr.servables) == [5]
    with pytest.raises(KeyError):
        mgr.get(1)
    mgr.close()


def test_dynamic_batcher_merges_concurrent_requests():
    calls = []

    def run(items):
        calls.append(len(items))
        a = np.asarray(items, dtype=np.float32)
        return {"y": a * 2}

    b = DynamicBatcher(run, max_batch_size=64, batch_timeout_s=0.05)
    results = {}

    def worker(i):
        results[i] = b.submit([[float(i)], [float(i) + 0.5]]).result()

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    b.close()
    for i in range(8):
        np.testing.assert_allclose(results[i]["y"], [[2.0 * i], [2.0 * i + 1.0]])
    assert sum(calls) == 16 and len(calls) < 8  # merged into fewer device launches


def test_tensorstore_resnet_dag():
    ts = TensorStore()
    torch.manual_seed(0)
    m = resnet50_v2()
    ts.modelset("r50", "TORCH", "CPU", model=m)
    ts.scriptset("pp", "CPU", PREPROCESS_SCRIPT)
    img = np.random.default_rng(0).integers(0, 255, (64, 64, 3))
    ts.tensorset("img", "UINT8", [64, 64, 3], values=img)
    ts.dagrun([("SCRIPTRUN", "pp", "pre_process", ["img"], ["x"]), ("MODELRUN", "r50", ["x"], ["y"]),
               ("SCRIPTRUN", "pp", "post_process", ["y"], ["label"])])
    with torch.no_grad():
        ref = m.eval()(torch.from_numpy(img).float().div(255).permute(2, 0, 1)[None]).argmax(1) - 1
    assert ts.tensorget("label")["values"] == ref.tolist()
    assert ts.tensorget("y", "META") == {"dtype": "FLOAT", "shape": [1, 1001]}
    blob = ts.tensorget("img", "BLOB")
    ts.tensorset("img2", "UINT8", [64, 64, 3], blob=blob)
    assert ts.tensorget("img2")["values"][:5] == img.reshape(-1)[:5].tolist()


# ---------------------------------------------------------------- gRPC PredictionService (TF-Serving --port API)
def test_grpc_predict_metadata_status_over_localhost(tmp_path):
    """A client drives the gRPC API over a localhost socket: Predict (latest / pinned version / output_filter),
    GetModelMetadata (SignatureDefMap in an Any), GetModelStatus, NOT_FOUND / INVALID_ARGUMENT errors; the REST and
    gRPC APIs share one ModelManager."""
    import grpc

    from mifx.serving import grpc_service as gs

    base = str(tmp_path / "fashion")
    m1 = _export(base, 1, 1)
    m2 = _export(base, 2, 2)
    mgr = ModelManager("fashion", base, policy="all", device="cpu", poll_s=0)
    server, port = gs.serve({"fashion": mgr}, port=0, host="127.0.0.1")
    cli = gs.PredictionClient(f"127.0.0.1:{port}")
    try:
        x = np.random.default_rng(0).random((3, 28, 28)).astype(np.float32)
        out = cli.predict("fashion", {"input": x})
        with torch.no_grad():
            np.testing.assert_allclose(out["scores"], m2(torch.from_numpy(x)).numpy(), rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(cli.predict("fashion", {"input": x}, version=1)["scores"],
                                       m1(torch.from_numpy(x)).numpy(), rtol=1e-5, atol=1e-5)
        assert out["scores"].dtype == np.float32 and out["scores"].shape == (3, 10)
        assert list(cli.predict("fashion", {"input": x}, output_filter=["scores"])) == ["scores"]
        v, sm = cli.metadata("fashion")
        assert v == 2 and "serving_default" in sm.signature_def
        assert [d.size for d in sm.signature_def["serving_default"].inputs["input"].tensor_shape.dim] == [-1, 28, 28]
        assert cli.status("fashion") == [(2, "AVAILABLE"), (1, "AVAILABLE")]
        with pytest.raises(grpc.RpcError) as e:
            cli.predict("nope", {"input": x})
        assert e.value.code() == grpc.StatusCode.NOT_FOUND
        with pytest.raises(grpc.RpcError) as e:
            cli.predict("fashion", {"input": x}, version=7)
        assert e.value.code() == grpc.StatusCode.NOT_FOUND
        with pytest.raises(grpc.RpcError) as e:
            cli.predict("fashion", {"input": x}, output_filter=["bogus"])
        assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    finally:
        cli.close()
        server.stop(grace=None)
        mgr.close()


def test_tensor_proto_round_trip_and_wire_format():
    """TensorProto <-> numpy for every supported dtype; the typed *_val fields and a broadcast single value decode as
    TensorFlow does; the serialized PredictRequest carries TF-Serving's field numbers."""
    from mifx.serving import grpc_service as gs

    m = gs.messages()
    for dt in (np.float32, np.float64, np.int32, np.int64, np.uint8, np.int8, np.int16, np.bool_, np.float16):
        a = (np.arange(12).reshape(3, 4) % 3).astype(dt)
        back = gs.make_ndarray(m["TensorProto"].FromString(gs.make_tensor_proto(a).SerializeToString()))
        assert back.dtype == a.dtype and np.array_equal(back, a)
    s = np.array([["a", "bc"], ["d", ""]])
    assert gs.make_ndarray(gs.make_tensor_proto(s)).tolist() == s.tolist()
    t = m["TensorProto"](dtype=gs.DT["float32"])
    for d in (2, 3):
        t.tensor_shape.dim.add(size=d)
    t.float_val.append(1.5)  # a single value fills the shape
    assert np.array_equal(gs.make_ndarray(t), np.full((2, 3), 1.5, np.float32))
    req = m["PredictRequest"]()
    req.model_spec.name = "m"
    req.model_spec.version.value = 5
    raw = req.SerializeToString()
    # field 1 (model_spec, length-delimited) = {field 1 "m", field 2 {field 1 varint 5}}
    assert raw == bytes([0x0A, 0x07, 0x0A, 0x01, ord("m"), 0x12, 0x02, 0x08, 0x05])


# ---------------------------------------------------------------- RESP server (RedisAI client <-> server flow)
def test_resp_server_notebook18_flow_over_localhost(tmp_path):
    """The RedisAI notebook's flow over a real socket: TENSORSET by VALUES and BLOB, TENSORGET META / VALUES / BLOB,
    MODELSET from a saved-model blob, SCRIPTSET, SCRIPTRUN -> MODELRUN -> SCRIPTRUN, errors as -ERR replies."""
    from mifx.serving.resp_server import RespClient, RespError, RespServer, saved_model_blob

    srv = RespServer(port=0)
    port = srv.start()
    c = RespClient("127.0.0.1", port)
    try:
        assert c.ping()
        assert c.execute_command("AI.TENSORSET", "v", "DOUBLE", 3, "VALUES", 1.0, 2.0, 3.0) == "OK"
        r = c.execute_command("AI.TENSORGET", "v", "VALUES")
        assert r[:4] == [b"dtype", b"DOUBLE", b"shape", [3]] and [float(x) for x in r[5]] == [1.0, 2.0, 3.0]
        blob = np.array([1.5, -2.0], np.float32).tobytes()
        c.execute_command("AI.TENSORSET", "b", "FLOAT", 2, "BLOB", blob)
        assert c.execute_command("AI.TENSORGET", "b", "BLOB")[5] == blob
        assert c.execute_command("AI.TENSORGET", "b", "META") == [b"dtype", b"FLOAT", b"shape", [2]]
        # model from a saved-model export sent as a blob; TorchScript pre/post-processing
        m = _export(str(tmp_path / "f"), 1, 3)
        assert c.execute_command("AI.MODELSET", "fash", "MIFX", "CPU", "INPUTS", "x", "OUTPUTS", "y", "BLOB",
                                 saved_model_blob(str(tmp_path / "f" / "1"))) == "OK"
        c.execute_command("AI.SCRIPTSET", "pp", "CPU", "SOURCE",
                          "def pre(img):\n    return img.float().div(255).unsqueeze(0)\n"
                          "def post(out):\n    return out.max(1)[1]\n")
        img = np.random.default_rng(1).integers(0, 256, (28, 28), dtype=np.uint8)
        c.execute_command("AI.TENSORSET", "img", "UINT8", 28, 28, "BLOB", img.tobytes())
        c.execute_command("AI.SCRIPTRUN", "pp", "pre", "INPUTS", "img", "OUTPUTS", "x")
        c.execute_command("AI.MODELRUN", "fash", "INPUTS", "x", "OUTPUTS", "y")
        c.execute_command("AI.SCRIPTRUN", "pp", "post", "INPUTS", "y", "OUTPUTS", "label")
        got = c.execute_command("AI.TENSORGET", "label", "VALUES")[5]
        with torch.no_grad():
            ref = m.eval()(torch.from_numpy(img).float().div(255)[None]).argmax(1)
        assert [int(x) for x in got] == ref.tolist()
        assert sorted(c.execute_command("KEYS", "*")) == [b"b", b"fash", b"img", b"label", b"pp", b"v", b"x", b"y"]
        assert c.execute_command("DEL", "v", "nope") == 1
        with pytest.raises(RespError):
            c.execute_command("AI.TENSORGET", "v")
        with pytest.raises(RespError):
            c.execute_command("AI.BOGUS")
        assert c.ping()  # the connection survives error replies
        # a second client sees the same store (tensors live in the server)
        c2 = RespClient("127.0.0.1", port)
        assert c2.execute_command("EXISTS", "label", "b") == 2
        c2.close()
    finally:
        c.close()
        srv.stop()


def test_resp_server_refuses_code_loading_and_unauthenticated_clients(tmp_path):
    """An export naming a callable off the allow-list (here the rank launcher, which would start `python -c`), a
    PATH outside the model roots, a compressed blob, deep nesting, and commands before AUTH are all refused."""
    import io
    import json as _json
    import socket as _socket
    import tarfile

    from mifx.serving import saved_model as sm
    from mifx.serving.resp_server import RespClient, RespError, RespServer, _Reader, encode, saved_model_blob

    with pytest.raises(ValueError):
        RespServer(host="0.0.0.0", port=0)  # no password on a non-loopback address
    _export(str(tmp_path / "f"), 1, 3)
    evil = tmp_path / "evil"
    (evil / "variables").mkdir(parents=True)
    from safetensors.torch import save_file

    save_file({}, str(evil / "variables" / "variables.safetensors"))
    (evil / "saved_model.json").write_text(_json.dumps({
        "format": sm.FORMAT, "family": "module", "model_class": "mifx.trainer.distributed:run_ranks",
        "model_config": {"args": ["-c", "open('/tmp/pwned','w')"], "num_procs": 1}, "signatures": {}}))
    with pytest.raises(PermissionError):
        sm.LoadedModel(str(evil), "cpu")  # the loader itself enforces the allow-list
    srv = RespServer(port=0, requirepass="s3cret", model_roots=[str(tmp_path / "f")])
    port = srv.start()
    try:
        c = RespClient("127.0.0.1", port)
        with pytest.raises(RespError, match="NOAUTH"):
            c.execute_command("KEYS", "*")
        with pytest.raises(RespError, match="WRONGPASS"):
            c.execute_command("AUTH", "nope")
        assert c.execute_command("AUTH", "s3cret") == "OK"
        with pytest.raises(RespError, match="allow-list"):
            c.execute_command("AI.MODELSET", "m", "MIFX", "CPU", "BLOB", saved_model_blob(str(evil)))
        with pytest.raises(RespError, match="model roots"):
            c.execute_command("AI.MODELSET", "m", "MIFX", "CPU", "PATH", str(evil))
        assert c.execute_command("AI.MODELSET", "m", "MIFX", "CPU", "PATH", str(tmp_path / "f" / "1")) == "OK"
        gz = io.BytesIO()
        with tarfile.open(fileobj=gz, mode="w:gz") as tf:
            tf.add(str(tmp_path / "f" / "1"), arcname=".")
        with pytest.raises(RespError, match="uncompressed"):
            c.execute_command("AI.MODELSET", "m2", "MIFX", "CPU", "BLOB", gz.getvalue())
        c.close()
        c2 = RespClient("127.0.0.1", port, password="s3cret")
        assert c2.ping()
        c2.close()
    finally:
        srv.stop()
    a, b = _socket.socketpair()
    a.sendall(b"*1\r\n" * 64 + b":1\r\n")
    with pytest.raises(ValueError, match="nested"):
        _Reader(b).value()
    a.sendall(encode([1]).replace(b"*1", b"*99999999"))
    with pytest.raises(ValueError, match="too long"):
        _Reader(b).value()
    a.close()
    b.close()


def test_resp_codec_round_trip():
    import socket as _socket

    from mifx.serving.resp_server import RespError, _Reader, encode

    a, b = _socket.socketpair()
    vals = ["OK", 42, b"bin\r\n\x00ary", None, [1, [b"x", "PONG"], b""], RespError("ERR boom")]
    for v in vals:
        a.sendall(encode(v))
    rd = _Reader(b)
    got = [rd.value() for _ in vals]
    assert got[:3] == ["OK", 42, b"bin\r\n\x00ary"] and got[3] is None
    assert got[4] == [1, [b"x", "PONG"], b""] and isinstance(got[5], RespError) and str(got[5]) == "ERR boom"
    a.close()
    b.close()
