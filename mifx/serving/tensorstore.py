"""In-memory tensor / model / script store with RedisAI-style commands (in-database inference).

Reference: the RedisAI notebook (`notebooks/redis/RedisAI_TensorFlow.ipynb`):
`AI.TENSORSET/TENSORGET`, `AI.MODELSET <key> TF CPU` (frozen ResNet-50), `AI.SCRIPTSET` (TorchScript
pre/post-processing), `AI.SCRIPTRUN -> AI.MODELRUN -> AI.SCRIPTRUN`. Here tensors stay resident on
the chosen device (HBM on MI355X) between commands, so a pre -> model -> post chain never
round-trips through the host; scripts are TorchScript source compiled with
`torch.jit.CompilationUnit` (no arbitrary Python is executed)."""
from __future__ import annotations

import threading

import numpy as np
import torch

_DT = {"FLOAT": torch.float32, "DOUBLE": torch.float64, "INT8": torch.int8, "INT16": torch.int16,
       "INT32": torch.int32, "INT64": torch.int64, "UINT8": torch.uint8, "HALF": torch.float16,
       "BFLOAT16": torch.bfloat16, "BOOL": torch.bool}
_DT_NAME = {v: k for k, v in _DT.items()}


def _dev(device: str) -> torch.device:
    d = device.upper()
    if d == "CPU":
        return torch.device("cpu")
    if d.startswith("GPU"):
        idx = int(d[4:]) if ":" in d else 0
        return torch.device("cuda", idx)
    return torch.device(device)


class TensorStore:
    def __init__(self):
        self._t: dict[str, torch.Tensor] = {}
        self._models: dict[str, tuple] = {}
        self._scripts: dict[str, tuple] = {}
        self._lock = threading.RLock()

    # ---- tensors --------------------------------------------------------------------------
    def tensorset(self, key: str, dtype: str, shape, values=None, blob: bytes | None = None, device: str = "CPU"):
        dt = _DT[dtype.upper()]
        if blob is not None:
            t = torch.frombuffer(bytearray(blob), dtype=dt).reshape(shape)
        elif values is not None:
            t = torch.as_tensor(np.asarray(values), dtype=dt).reshape(shape)
        else:
            t = torch.zeros(shape, dtype=dt)
        with self._lock:
            self._t[key] = t.to(_dev(device))
        return "OK"

    def put(self, key: str, t: torch.Tensor):
        with self._lock:
            self._t[key] = t
        return "OK"

    def tensorget(self, key: str, fmt: str = "VALUES"):
        with self._lock:
            if key not in self._t:
                raise KeyError(f"tensor key {key} is empty")
            t = self._t[key]
        fmt = fmt.upper()
        if fmt == "META":
            return {"dtype": _DT_NAME[t.dtype], "shape": list(t.shape)}
        if fmt == "BLOB":
            return t.detach().cpu().contiguous().numpy().tobytes()
        if fmt == "TENSOR":
            return t
        return {"dtype": _DT_NAME[t.dtype], "shape": list(t.shape), "values": t.detach().cpu().reshape(-1).tolist()}

    def exists(self, key: str) -> bool:
        with self._lock:
            return key in self._t or key in self._models or key in self._scripts

    def keys(self) -> list:
        with self._lock:
            return sorted(set(self._t) | set(self._models) | set(self._scripts))

    def delete(self, key: str):
        with self._lock:
            for d in (self._t, self._models, self._scripts):
                d.pop(key, None)
        return "OK"

    # ---- models -----------------------------------------------------------------------------
    def modelset(self, key: str, backend: str, device: str, model=None, path: str | None = None):
        """backend 'TORCH' with an nn.Module, or 'MIFX' with a saved-model directory."""
        dev = _dev(device)
        if backend.upper() == "MIFX":
            from .saved_model import LoadedModel

            lm = LoadedModel(path, str(dev))
            model = lm.model
        if not isinstance(model, torch.nn.Module):
            raise TypeError("model must be a torch.nn.Module (or backend MIFX with a path)")
        model = model.to(dev).eval()
        with self._lock:
            self._models[key] = (model, dev)
        return "OK"

    def modelrun(self, key: str, inputs: list, outputs: list):
        with self._lock:
            model, dev = self._models[key]
            xs = [self._t[k].to(dev) for k in inputs]
        with torch.no_grad():
            ys = model(*xs)
        ys = ys if isinstance(ys, (tuple, list)) else (ys,)
        if len(ys) != len(outputs):
            raise ValueError(f"model produced {len(ys)} outputs, {len(outputs)} keys given")
        with self._lock:
            for k, y in zip(outputs, ys):
                self._t[k] = y
        return "OK"

    # ---- scripts ----------------------------------------------------------------------------
    def scriptset(self, key: str, device: str, source: str):
        cu = torch.jit.CompilationUnit(source)
        with self._lock:
            self._scripts[key] = (cu, _dev(device))
        return "OK"

    def scriptrun(self, key: str, fn: str, inputs: list, outputs: list):
        with self._lock:
            cu, dev = self._scripts[key]
            xs = [self._t[k].to(dev) for k in inputs]
        ys = getattr(cu, fn)(*xs)
        ys = ys if isinstance(ys, (tuple, list)) else (ys,)
        with self._lock:
            for k, y in zip(outputs, ys):
                self._t[k] = y
        return "OK"

    def dagrun(self, commands: list):
        """Run a list of ('SCRIPTRUN'|'MODELRUN', args...) in order (AI.DAGRUN)."""
        for c in commands:
            op, *args = c
            getattr(self, op.lower())(*args)
        return "OK"

    # ---- command interface (`rai.execute_command('AI.TENSORSET', ...)` in the notebook) ----------
    def execute_command(self, cmd: str, *args):
        """RedisAI command syntax: AI.TENSORSET key TYPE d1..dn [BLOB b | VALUES v..]; AI.TENSORGET key
        [VALUES|BLOB|META]; AI.MODELSET key BACKEND DEVICE [INPUTS ..] [OUTPUTS ..] <model>;
        AI.SCRIPTSET key DEVICE <source>; AI.SCRIPTRUN key fn INPUTS .. OUTPUTS ..;
        AI.MODELRUN key INPUTS .. OUTPUTS ..; AI.TENSORDEL / AI.DAGRUN-free subset."""
        c = cmd.upper()
        a = [x.decode() if isinstance(x, bytes) and i < 1 else x for i, x in enumerate(args)]
        if c == "AI.TENSORSET":
            key, dtype, rest = a[0], str(a[1]), list(a[2:])
            shape = []
            while rest and not (isinstance(rest[0], str) and rest[0].upper() in ("BLOB", "VALUES")):
                shape.append(int(rest.pop(0)))
            if rest and rest[0].upper() == "BLOB":
                return self.tensorset(key, dtype, shape, blob=rest[1])
            if rest and rest[0].upper() == "VALUES":
                return self.tensorset(key, dtype, shape, values=[float(v) for v in rest[1:]])
            return self.tensorset(key, dtype, shape)
        if c == "AI.TENSORGET":
            return self.tensorget(a[0], str(a[1]) if len(a) > 1 else "VALUES")
        if c == "AI.TENSORDEL":
            return self.delete(a[0])
        if c == "AI.MODELSET":
            key, backend, device = a[0], str(a[1]), str(a[2])
            model = a[-1]
            if isinstance(model, str):
                return self.modelset(key, backend, device, path=model)
            return self.modelset(key, "TORCH", device, model=model)
        if c == "AI.SCRIPTSET":
            src = a[2].decode() if isinstance(a[2], bytes) else a[2]
            return self.scriptset(a[0], str(a[1]), src)
        if c in ("AI.SCRIPTRUN", "AI.MODELRUN"):
            key = a[0]
            rest = list(a[1:])
            fn = rest.pop(0) if c == "AI.SCRIPTRUN" else None
            i_in, i_out = rest.index("INPUTS"), rest.index("OUTPUTS")
            ins, outs = rest[i_in + 1:i_out], rest[i_out + 1:]
            return self.scriptrun(key, fn, ins, outs) if fn else self.modelrun(key, ins, outs)
        raise ValueError(f"unsupported command {cmd}")
