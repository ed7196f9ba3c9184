"""TF-Serving gRPC API (`tensorflow.serving.PredictionService` / `ModelService`) for the model server.

Reference: the TF-Serving deployment runs `tensorflow_model_server --port=9000 --rest_api_port=8500` with a TCP
liveness probe on 9000 (`install-kubeflow/ks_app/vendor/kubeflow/tf-serving/tf-serving-template.libsonnet:33-34,72`);
clients call `PredictionService.Predict` with `TensorProto` inputs. This module serves the same RPCs over grpcio:

  /tensorflow.serving.PredictionService/Predict           PredictRequest -> PredictResponse
  /tensorflow.serving.PredictionService/GetModelMetadata  GetModelMetadataRequest -> GetModelMetadataResponse
                                                           (metadata["signature_def"] = Any(SignatureDefMap))
  /tensorflow.serving.ModelService/GetModelStatus         GetModelStatusRequest -> GetModelStatusResponse

The messages are declared here field-for-field with the TF-Serving / TensorFlow protos (same field numbers and wire
types: `tensorflow/core/framework/tensor.proto`, `tensor_shape.proto`, `meta_graph.proto` TensorInfo / SignatureDef,
`tensorflow_serving/apis/{model,predict,get_model_metadata,get_model_status}.proto`), built from descriptors in a
private descriptor pool (no protoc / generated stubs needed, no clash with a real tensorflow install), so a stock
TF-Serving client interoperates byte for byte. Enums are carried as their integer values (same varint encoding).
`PredictionClient` is the matching Python client."""
from __future__ import annotations

import concurrent.futures as cf
import functools

import numpy as np
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

# tensorflow.DataType values used here
DT = {"float32": 1, "float64": 2, "int32": 3, "uint8": 4, "int16": 5, "int8": 6, "string": 7, "int64": 9,
      "bool": 10, "uint16": 17, "float16": 19, "uint32": 22, "uint64": 23}
_NP_OF = {v: np.dtype(k) for k, v in DT.items() if k != "string"}
# ModelVersionStatus.State
_STATE = {"UNKNOWN": 0, "START": 10, "LOADING": 20, "AVAILABLE": 30, "UNLOADING": 40, "END": 50}

_T = descriptor_pb2.FieldDescriptorProto
_SCALAR = {"int32": _T.TYPE_INT32, "int64": _T.TYPE_INT64, "string": _T.TYPE_STRING, "bytes": _T.TYPE_BYTES,
           "float": _T.TYPE_FLOAT, "double": _T.TYPE_DOUBLE, "bool": _T.TYPE_BOOL}


def _msg(fdp, name, fields):
    """Add message `name` with (field name, number, scalar type name or '.full.MessageName', repeated) fields."""
    m = fdp.message_type.add()
    m.name = name
    for fname, num, typ, rep in fields:
        f = m.field.add()
        f.name, f.number = fname, num
        f.label = _T.LABEL_REPEATED if rep else _T.LABEL_OPTIONAL
        if typ in _SCALAR:
            f.type = _SCALAR[typ]
        else:
            f.type, f.type_name = _T.TYPE_MESSAGE, typ
    return m


def _with_map(m, full_name, fname, num, value_type):
    """map<string, value_type> fname = num on message m (= `full_name`): a repeated nested *Entry message with
    map_entry set, as protoc emits it."""
    e = m.nested_type.add()
    e.name = "".join(p.capitalize() for p in fname.split("_")) + "Entry"
    e.options.map_entry = True
    k = e.field.add()
    k.name, k.number, k.label, k.type = "key", 1, _T.LABEL_OPTIONAL, _T.TYPE_STRING
    v = e.field.add()
    v.name, v.number, v.label = "value", 2, _T.LABEL_OPTIONAL
    v.type, v.type_name = _T.TYPE_MESSAGE, value_type
    f = m.field.add()
    f.name, f.number, f.label, f.type = fname, num, _T.LABEL_REPEATED, _T.TYPE_MESSAGE
    f.type_name = f"{full_name}.{e.name}"


@functools.lru_cache(maxsize=None)
def messages() -> dict:
    """name -> message class, from a private descriptor pool."""
    pool = descriptor_pool.DescriptorPool()

    tf = descriptor_pb2.FileDescriptorProto(name="mifx_tf_framework.proto", package="tensorflow", syntax="proto3")
    shape = _msg(tf, "TensorShapeProto", [("unknown_rank", 3, "bool", False)])
    dim = shape.nested_type.add()
    dim.name = "Dim"
    for fname, num, typ in (("size", 1, _T.TYPE_INT64), ("name", 2, _T.TYPE_STRING)):
        f = dim.field.add()
        f.name, f.number, f.label, f.type = fname, num, _T.LABEL_OPTIONAL, typ
    f = shape.field.add()
    f.name, f.number, f.label = "dim", 2, _T.LABEL_REPEATED
    f.type, f.type_name = _T.TYPE_MESSAGE, ".tensorflow.TensorShapeProto.Dim"
    _msg(tf, "TensorProto", [("dtype", 1, "int32", False), ("tensor_shape", 2, ".tensorflow.TensorShapeProto", False),
                             ("version_number", 3, "int32", False), ("tensor_content", 4, "bytes", False),
                             ("float_val", 5, "float", True), ("double_val", 6, "double", True),
                             ("int_val", 7, "int32", True), ("string_val", 8, "bytes", True),
                             ("int64_val", 10, "int64", True), ("bool_val", 11, "bool", True),
                             ("half_val", 13, "int32", True)])
    _msg(tf, "TensorInfo", [("name", 1, "string", False), ("dtype", 2, "int32", False),
                            ("tensor_shape", 3, ".tensorflow.TensorShapeProto", False)])
    sig = _msg(tf, "SignatureDef", [("method_name", 3, "string", False)])
    _with_map(sig, ".tensorflow.SignatureDef", "inputs", 1, ".tensorflow.TensorInfo")
    _with_map(sig, ".tensorflow.SignatureDef", "outputs", 2, ".tensorflow.TensorInfo")
    pool.Add(tf)

    gp = descriptor_pb2.FileDescriptorProto(name="mifx_pb_wrappers.proto", package="google.protobuf", syntax="proto3")
    _msg(gp, "Int64Value", [("value", 1, "int64", False)])
    _msg(gp, "Any", [("type_url", 1, "string", False), ("value", 2, "bytes", False)])
    pool.Add(gp)

    sv = descriptor_pb2.FileDescriptorProto(name="mifx_tf_serving_apis.proto", package="tensorflow.serving",
                                            syntax="proto3", dependency=["mifx_tf_framework.proto",
                                                                         "mifx_pb_wrappers.proto"])
    _msg(sv, "ModelSpec", [("name", 1, "string", False), ("version", 2, ".google.protobuf.Int64Value", False),
                           ("signature_name", 3, "string", False), ("version_label", 4, "string", False)])
    req = _msg(sv, "PredictRequest", [("model_spec", 1, ".tensorflow.serving.ModelSpec", False),
                                      ("output_filter", 3, "string", True)])
    _with_map(req, ".tensorflow.serving.PredictRequest", "inputs", 2, ".tensorflow.TensorProto")
    resp = _msg(sv, "PredictResponse", [("model_spec", 2, ".tensorflow.serving.ModelSpec", False)])
    _with_map(resp, ".tensorflow.serving.PredictResponse", "outputs", 1, ".tensorflow.TensorProto")
    _msg(sv, "GetModelMetadataRequest", [("model_spec", 1, ".tensorflow.serving.ModelSpec", False),
                                         ("metadata_field", 2, "string", True)])
    mdr = _msg(sv, "GetModelMetadataResponse", [("model_spec", 1, ".tensorflow.serving.ModelSpec", False)])
    _with_map(mdr, ".tensorflow.serving.GetModelMetadataResponse", "metadata", 2, ".google.protobuf.Any")
    sdm = _msg(sv, "SignatureDefMap", [])
    _with_map(sdm, ".tensorflow.serving.SignatureDefMap", "signature_def", 1, ".tensorflow.SignatureDef")
    _msg(sv, "StatusProto", [("error_code", 1, "int32", False), ("error_message", 2, "string", False)])
    _msg(sv, "ModelVersionStatus", [("version", 1, "int64", False), ("state", 2, "int32", False),
                                    ("status", 3, ".tensorflow.serving.StatusProto", False)])
    _msg(sv, "GetModelStatusRequest", [("model_spec", 1, ".tensorflow.serving.ModelSpec", False)])
    _msg(sv, "GetModelStatusResponse", [("model_version_status", 1, ".tensorflow.serving.ModelVersionStatus", True)])
    pool.Add(sv)

    out = {}
    for full in ("tensorflow.TensorShapeProto", "tensorflow.TensorProto", "tensorflow.TensorInfo",
                 "tensorflow.SignatureDef", "google.protobuf.Int64Value", "google.protobuf.Any",
                 "tensorflow.serving.ModelSpec", "tensorflow.serving.PredictRequest",
                 "tensorflow.serving.PredictResponse", "tensorflow.serving.GetModelMetadataRequest",
                 "tensorflow.serving.GetModelMetadataResponse", "tensorflow.serving.SignatureDefMap",
                 "tensorflow.serving.ModelVersionStatus", "tensorflow.serving.GetModelStatusRequest",
                 "tensorflow.serving.GetModelStatusResponse"):
        out[full.rsplit(".", 1)[1]] = message_factory.GetMessageClass(pool.FindMessageTypeByName(full))
    return out


# ---------------------------------------------------------------- TensorProto <-> numpy
def make_tensor_proto(a) -> object:
    """numpy array (or nested list / scalar) -> tensorflow.TensorProto (numeric: tensor_content, little-endian;
    strings: string_val)."""
    TP = messages()["TensorProto"]
    arr = np.asarray(a)
    t = TP()
    for d in arr.shape:
        t.tensor_shape.dim.add(size=int(d))
    if arr.dtype.kind in "USO":
        t.dtype = DT["string"]
        t.string_val.extend(x.encode() if isinstance(x, str) else bytes(x) for x in arr.reshape(-1).tolist())
        return t
    if arr.dtype == np.float16:
        name = "float16"
    else:
        name = arr.dtype.name
    if name not in DT:
        raise ValueError(f"unsupported dtype {arr.dtype}")
    t.dtype = DT[name]
    t.tensor_content = np.ascontiguousarray(arr, dtype=arr.dtype.newbyteorder("<")).tobytes()
    return t


def make_ndarray(t) -> np.ndarray:
    """tensorflow.TensorProto -> numpy array (tensor_content, or the typed *_val field; a single value fills the
    shape, as in TensorFlow)."""
    shape = tuple(int(d.size) for d in t.tensor_shape.dim)
    n = int(np.prod(shape)) if shape else 1
    if t.dtype == DT["string"]:
        vals = np.array([v.decode(errors="replace") for v in t.string_val], dtype=object)
        return (np.repeat(vals, n) if len(vals) == 1 and n > 1 else vals).reshape(shape)
    if t.dtype not in _NP_OF:
        raise ValueError(f"unsupported TensorProto dtype {t.dtype}")
    dt = _NP_OF[t.dtype]
    if t.tensor_content:
        return np.frombuffer(t.tensor_content, dtype=dt.newbyteorder("<")).astype(dt).reshape(shape)
    field = {1: "float_val", 2: "double_val", 3: "int_val", 4: "int_val", 5: "int_val", 6: "int_val",
             9: "int64_val", 10: "bool_val", 19: "half_val", 17: "int_val", 22: "int64_val", 23: "int64_val"}[t.dtype]
    vals = list(getattr(t, field))
    if t.dtype == DT["float16"]:
        arr = np.array(vals, dtype=np.uint16).view(np.float16)
    else:
        arr = np.array(vals, dtype=dt)
    if arr.size == 1 and n > 1:
        arr = np.repeat(arr, n)
    return arr.reshape(shape)


# ---------------------------------------------------------------- server
def _tensor_info(spec) -> object:
    """A saved_model.json signature entry (shape list, or feature spec) -> TensorInfo."""
    TI = messages()["TensorInfo"]
    ti = TI(dtype=DT["float32"])
    if isinstance(spec, (list, tuple)):
        ti.tensor_shape.dim.add(size=-1)
        for d in spec:
            ti.tensor_shape.dim.add(size=int(d))
    elif isinstance(spec, dict) and spec.get("dtype") in ("string", "str"):
        ti.dtype = DT["string"]
    return ti


def _signature_map(sigs: dict) -> object:
    m = messages()
    out = m["SignatureDefMap"]()
    for name, s in sigs.items():
        sd = out.signature_def[name]
        sd.method_name = f"tensorflow/serving/{s.get('method', 'predict')}"
        for k, v in (s.get("inputs") or {}).items():
            sd.inputs[k].CopyFrom(_tensor_info(v))
        for k in s.get("outputs") or ["scores"]:
            sd.outputs[k].CopyFrom(messages()["TensorInfo"](name=k, dtype=DT["float32"]))
    return out


class PredictionServicer:
    """The RPC handlers over a dict of ModelManagers (shared with the REST app)."""

    def __init__(self, models: dict):
        self.models = models

    def _servable(self, spec, context):
        import grpc

        mgr = self.models.get(spec.name)
        if mgr is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"Servable not found for request: Latest({spec.name})")
        version = spec.version.value if spec.HasField("version") else None
        try:
            return mgr.get(version)
        except KeyError as e:
            context.abort(grpc.StatusCode.NOT_FOUND, str(e))

    def Predict(self, request, context):
        import grpc

        m = messages()
        s = self._servable(request.model_spec, context)
        inputs = {k: make_ndarray(v) for k, v in request.inputs.items()}
        try:
            if s.model.family == "wide_deep":
                out = s.predict({k: v.reshape(-1) for k, v in inputs.items()})  # columns
            else:
                if len(inputs) != 1:
                    raise ValueError(f"this signature takes one input tensor, got {sorted(inputs)}")
                out = s.predict(next(iter(inputs.values())))
        except Exception as e:  # noqa: BLE001 - TF-Serving maps model errors to INVALID_ARGUMENT
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, str(e))
        keys = list(request.output_filter) or list(out)
        resp = m["PredictResponse"]()
        resp.model_spec.name = request.model_spec.name
        resp.model_spec.version.value = s.version
        resp.model_spec.signature_name = request.model_spec.signature_name or "serving_default"
        for k in keys:
            if k not in out:
                context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"output_filter: unknown output '{k}'")
            resp.outputs[k].CopyFrom(make_tensor_proto(np.asarray(out[k])))
        return resp

    def GetModelMetadata(self, request, context):
        import grpc

        m = messages()
        fields = list(request.metadata_field) or ["signature_def"]
        if fields != ["signature_def"]:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, "metadata_field must be 'signature_def'")
        s = self._servable(request.model_spec, context)
        resp = m["GetModelMetadataResponse"]()
        resp.model_spec.name = request.model_spec.name
        resp.model_spec.version.value = s.version
        sm = _signature_map(s.model.signatures)
        resp.metadata["signature_def"].type_url = "type.googleapis.com/tensorflow.serving.SignatureDefMap"
        resp.metadata["signature_def"].value = sm.SerializeToString()
        return resp

    def GetModelStatus(self, request, context):
        import grpc

        m = messages()
        mgr = self.models.get(request.model_spec.name)
        if mgr is None:
            context.abort(grpc.StatusCode.NOT_FOUND, f"Could not find any versions of model {request.model_spec.name}")
        version = request.model_spec.version.value if request.model_spec.HasField("version") else None
        st = mgr.status(version)
        resp = m["GetModelStatusResponse"]()
        for v in st["model_version_status"]:
            e = resp.model_version_status.add(version=int(v["version"]), state=_STATE.get(v["state"], 0))
            e.status.error_code = 0 if v["state"] != "UNKNOWN" else 5
        return resp


def _handlers(servicer: PredictionServicer):
    import grpc

    m = messages()
    ser = lambda msg: msg.SerializeToString()  # noqa: E731
    pred = grpc.method_handlers_generic_handler("tensorflow.serving.PredictionService", {
        "Predict": grpc.unary_unary_rpc_method_handler(servicer.Predict, m["PredictRequest"].FromString, ser),
        "GetModelMetadata": grpc.unary_unary_rpc_method_handler(servicer.GetModelMetadata,
                                                                m["GetModelMetadataRequest"].FromString, ser)})
    model = grpc.method_handlers_generic_handler("tensorflow.serving.ModelService", {
        "GetModelStatus": grpc.unary_unary_rpc_method_handler(servicer.GetModelStatus,
                                                              m["GetModelStatusRequest"].FromString, ser)})
    return [pred, model]


def serve(models: dict, port: int = 9000, host: str = "0.0.0.0", workers: int = 16,
          max_message_mb: int = 256):
    """Start the gRPC server (non-blocking) on host:port; returns (server, bound port). port 0 picks a free port."""
    import grpc

    opts = [("grpc.max_receive_message_length", max_message_mb << 20),
            ("grpc.max_send_message_length", max_message_mb << 20)]
    server = grpc.server(cf.ThreadPoolExecutor(max_workers=workers), options=opts)
    server.add_generic_rpc_handlers(_handlers(PredictionServicer(models)))
    bound = server.add_insecure_port(f"{host}:{port}")
    if bound == 0:
        raise OSError(f"gRPC: could not bind {host}:{port}")
    server.start()
    return server, bound


# ---------------------------------------------------------------- client
class PredictionClient:
    """Client of the PredictionService / ModelService RPCs (what a TF-Serving client's stubs send)."""

    def __init__(self, target: str, timeout: float = 30.0, max_message_mb: int = 256):
        import grpc

        self.channel = grpc.insecure_channel(target, options=[("grpc.max_receive_message_length", max_message_mb << 20),
                                                               ("grpc.max_send_message_length", max_message_mb << 20)])
        self.timeout = timeout
        m = messages()
        ser = lambda msg: msg.SerializeToString()  # noqa: E731
        self._predict = self.channel.unary_unary("/tensorflow.serving.PredictionService/Predict", ser,
                                                 m["PredictResponse"].FromString)
        self._meta = self.channel.unary_unary("/tensorflow.serving.PredictionService/GetModelMetadata", ser,
                                              m["GetModelMetadataResponse"].FromString)
        self._status = self.channel.unary_unary("/tensorflow.serving.ModelService/GetModelStatus", ser,
                                                m["GetModelStatusResponse"].FromString)

    def _spec(self, msg, name, version, signature=None):
        msg.model_spec.name = name
        if version is not None:
            msg.model_spec.version.value = int(version)
        if signature:
            msg.model_spec.signature_name = signature

    def predict(self, name: str, inputs: dict, version: int | None = None, output_filter=(),
                signature: str | None = None) -> dict:
        req = messages()["PredictRequest"]()
        self._spec(req, name, version, signature)
        for k, v in inputs.items():
            req.inputs[k].CopyFrom(make_tensor_proto(v))
        req.output_filter.extend(output_filter)
        resp = self._predict(req, timeout=self.timeout)
        return {k: make_ndarray(v) for k, v in resp.outputs.items()}

    def metadata(self, name: str, version: int | None = None):
        m = messages()
        req = m["GetModelMetadataRequest"]()
        self._spec(req, name, version)
        req.metadata_field.append("signature_def")
        resp = self._meta(req, timeout=self.timeout)
        sm = m["SignatureDefMap"].FromString(resp.metadata["signature_def"].value)
        return resp.model_spec.version.value, sm

    def status(self, name: str, version: int | None = None) -> list:
        req = messages()["GetModelStatusRequest"]()
        self._spec(req, name, version)
        resp = self._status(req, timeout=self.timeout)
        inv = {v: k for k, v in _STATE.items()}
        return [(e.version, inv.get(e.state, str(e.state))) for e in resp.model_version_status]

    def close(self):
        self.channel.close()
