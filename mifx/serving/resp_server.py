"""RESP (Redis protocol) network front-end for the RedisAI-style TensorStore: client <-> server in-database inference.

Reference: the RedisAI notebook connects to a server (`Client(host="redis-master", port=6379)`,
`notebooks/redis/RedisAI_TensorFlow.ipynb:63`) and drives it with `AI.TENSORSET / AI.MODELSET / AI.SCRIPTSET /
AI.SCRIPTRUN / AI.MODELRUN / AI.TENSORGET` over the wire (`:176`), the tensors living in the server between commands.
`RespServer` speaks RESP2 on a TCP port (one thread per connection, like redis-server's clients), executing every
command on one `TensorStore` whose tensors stay resident in the server's device memory (HBM on MI355X), so the
SCRIPTRUN -> MODELRUN -> SCRIPTRUN chain of a request never leaves the GPU; only TENSORSET / TENSORGET payloads cross
the socket. `RespClient` is a minimal redis-py-compatible client (`execute_command`).

Commands: PING, ECHO, DEL, EXISTS, KEYS, FLUSHALL, QUIT, AI.TENSORSET key TYPE d1..dn [BLOB b | VALUES v..],
AI.TENSORGET key [META | VALUES | BLOB] (RedisAI 1.x reply: [dtype, TYPE, shape, [dims]] + [values, [...]] /
[blob, bytes]), AI.TENSORDEL, AI.MODELSET key MIFX device [INPUTS ..] [OUTPUTS ..] BLOB <tar of a saved-model
export> | PATH <server-side export dir> (a model whose class is inside the `mifx` package: a blob never names code
to import from elsewhere, and the weights are safetensors), AI.MODELRUN key INPUTS .. OUTPUTS .., AI.SCRIPTSET key
device [SOURCE] <TorchScript source> (compiled by torch.jit, no Python executed), AI.SCRIPTRUN key fn INPUTS ..
OUTPUTS .., AI.DAGRUN-free subset as in TensorStore. Errors reply `-ERR <message>` and leave the connection open."""
from __future__ import annotations

import io
import json
import os
import socket
import socketserver
import tarfile
import tempfile
import threading

from .tensorstore import TensorStore

# ---------------------------------------------------------------- RESP2 codec


class RespError(Exception):
    """An error reply (-ERR ...) from the server."""


def encode(value) -> bytes:
    """Python value -> RESP2 reply."""
    if value is None:
        return b"$-1\r\n"
    if isinstance(value, RespError):
        return b"-" + str(value).replace("\r", " ").replace("\n", " ").encode() + b"\r\n"
    if isinstance(value, bool):
        return b":%d\r\n" % int(value)
    if isinstance(value, int):
        return b":%d\r\n" % value
    if isinstance(value, str):
        if value == "OK" or value == "PONG":
            return b"+" + value.encode() + b"\r\n"
        value = value.encode()
    if isinstance(value, (bytes, bytearray, memoryview)):
        b = bytes(value)
        return b"$%d\r\n%s\r\n" % (len(b), b)
    if isinstance(value, float):
        return encode(repr(value))
    if isinstance(value, (list, tuple)):
        return b"*%d\r\n" % len(value) + b"".join(encode(v) for v in value)
    raise TypeError(f"cannot encode {type(value)}")


def encode_command(*args) -> bytes:
    """A client command as a RESP array of bulk strings."""
    parts = []
    for a in args:
        if isinstance(a, (bytes, bytearray, memoryview)):
            b = bytes(a)
        elif isinstance(a, float):
            b = repr(a).encode()
        else:
            b = str(a).encode()
        parts.append(b"$%d\r\n%s\r\n" % (len(b), b))
    return b"*%d\r\n" % len(parts) + b"".join(parts)


class _Reader:
    def __init__(self, sock: socket.socket):
        self.f = sock.makefile("rb", buffering=1 << 16)

    def line(self) -> bytes:
        ln = self.f.readline()
        if not ln:
            raise ConnectionError("connection closed")
        if not ln.endswith(b"\r\n"):
            raise ValueError("protocol error: line not terminated by CRLF")
        return ln[:-2]

    def exact(self, n: int) -> bytes:
        b = self.f.read(n + 2)
        if len(b) != n + 2 or b[-2:] != b"\r\n":
            raise ConnectionError("connection closed inside a bulk string")
        return b[:-2]

    MAX_DEPTH = 8            # nested arrays (a command is depth 1; replies here nest at most 3 deep)
    MAX_ARRAY = 1 << 22      # elements per array (AI.TENSORSET ... VALUES v1 .. vn)

    def value(self, max_bulk: int = 1 << 31, depth: int = 0):
        ln = self.line()
        t, rest = ln[:1], ln[1:]
        if t == b"+":
            return rest.decode()
        if t == b"-":
            return RespError(rest.decode())
        if t == b":":
            return int(rest)
        if t == b"$":
            n = int(rest)
            if n < 0:
                return None
            if n > max_bulk:
                raise ValueError("protocol error: bulk string too large")
            return self.exact(n)
        if t == b"*":
            n = int(rest)
            if n > self.MAX_ARRAY:
                raise ValueError("protocol error: array too long")
            if depth >= self.MAX_DEPTH:
                raise ValueError("protocol error: arrays nested too deep")
            return None if n < 0 else [self.value(max_bulk, depth + 1) for _ in range(n)]
        # inline command (telnet style): space-separated words
        return ln.split()


# ---------------------------------------------------------------- server


def _s(x) -> str:
    return x.decode() if isinstance(x, (bytes, bytearray)) else str(x)


def _loopback(host: str) -> bool:
    return host in ("127.0.0.1", "::1", "localhost") or host.startswith("127.")


class RespServer:
    """Serve a TensorStore over RESP on host:port (port 0 picks a free one). start() returns the bound port.

    Security model (a model server executes what it loads, so who may load matters):
      * `requirepass`: like redis-server's, every command but AUTH / QUIT answers NOAUTH until the connection has
        sent `AUTH <password>`. Binding a non-loopback address without a password is refused.
      * AI.MODELSET BLOB payloads are plain (uncompressed) tars of saved-model exports; the class an export names must
        be on the serving allow-list (`mifx.serving.saved_model.servable_classes`), enforced by LoadedModel itself.
      * AI.MODELSET PATH reads server-side directories only under `model_roots` (none by default: PATH is off)."""

    def __init__(self, store: TensorStore | None = None, host: str = "127.0.0.1", port: int = 6379,
                 max_bulk_mb: int = 512, requirepass: str | None = None, model_roots: list[str] | None = None):
        if not _loopback(host) and not requirepass:
            raise ValueError(f"refusing to serve on {host} without a password (requirepass)")
        self.store = store or TensorStore()
        self.host, self.port = host, port
        self.max_bulk = max_bulk_mb << 20
        self.requirepass = requirepass
        self.model_roots = [os.path.realpath(r) for r in (model_roots or [])]
        self._srv = None
        self._thread = None
        self._tmp = tempfile.TemporaryDirectory(prefix="mifx_resp_models_")

    # -- commands
    def _tensorget(self, key, fmt):
        fmt = fmt.upper()
        meta = self.store.tensorget(key, "META")
        head = ["dtype", meta["dtype"], "shape", list(meta["shape"])]
        if fmt == "META":
            return head
        if fmt == "BLOB":
            return head + ["blob", self.store.tensorget(key, "BLOB")]
        vals = self.store.tensorget(key, "VALUES")["values"]
        return head + ["values", [repr(float(v)) if isinstance(v, float) else int(v) for v in vals]]

    def _modelset(self, key, backend, device, rest):
        backend = backend.upper()
        if backend not in ("MIFX", "TORCH"):
            raise RespError(f"ERR unsupported backend {backend} (this server runs MIFX saved-model exports)")
        kw = [_s(x).upper() if isinstance(x, (bytes, str)) and len(x) < 16 else None for x in rest]
        if "BLOB" in kw:
            blob = bytes(rest[kw.index("BLOB") + 1])
            d = os.path.join(self._tmp.name, f"m{len(os.listdir(self._tmp.name))}")
            os.makedirs(d)
            try:  # "r:" = no decompression: the extracted size is bounded by the blob's own (max_bulk)
                tf = tarfile.open(fileobj=io.BytesIO(blob), mode="r:")
            except tarfile.TarError as e:
                raise RespError(f"ERR model blob: not an uncompressed tar ({e})") from None
            with tf:
                total = 0
                for m in tf.getmembers():  # regular files and directories only, inside the target
                    if not (m.isfile() or m.isdir()) or m.name.startswith(("/", "..")) or ".." in m.name.split("/"):
                        raise RespError("ERR model blob: unsafe tar member")
                    total += m.size
                if total > len(blob):
                    raise RespError("ERR model blob: members larger than the blob")
                tf.extractall(d)
            path = d
        elif "PATH" in kw:
            path = os.path.realpath(_s(rest[kw.index("PATH") + 1]))
            if not any(path == r or path.startswith(r + os.sep) for r in self.model_roots):
                raise RespError("ERR AI.MODELSET PATH is outside the server's model roots")
        else:
            raise RespError("ERR AI.MODELSET needs BLOB <saved-model tar> or PATH <dir>")
        with open(os.path.join(path, "saved_model.json")) as f:
            meta = json.load(f)
        from .saved_model import servable_classes

        cls = meta.get("model_class", "")
        if meta.get("family") != "wide_deep" and cls not in servable_classes():
            raise RespError(f"ERR model class {cls!r} is not on the serving allow-list")
        return self.store.modelset(key, "MIFX", device, path=path)

    def execute(self, args: list):
        if not args:
            raise RespError("ERR empty command")
        cmd = _s(args[0]).upper()
        a = args[1:]
        st = self.store
        if cmd == "PING":
            return "PONG" if not a else a[0]
        if cmd == "ECHO":
            return a[0]
        if cmd in ("DEL", "AI.TENSORDEL"):
            n = 0
            for k in a:
                k = _s(k)
                if st.exists(k):
                    n += 1
                st.delete(k)
            return n if cmd == "DEL" else "OK"
        if cmd == "EXISTS":
            return sum(1 for k in a if st.exists(_s(k)))
        if cmd == "KEYS":
            import fnmatch

            pat = _s(a[0]) if a else "*"
            return [k for k in st.keys() if fnmatch.fnmatchcase(k, pat)]
        if cmd == "FLUSHALL":
            for k in list(st.keys()):
                st.delete(k)
            return "OK"
        if cmd == "AI.TENSORSET":
            key, dtype, rest = _s(a[0]), _s(a[1]), list(a[2:])
            shape = []
            while rest and _s(rest[0]).upper() not in ("BLOB", "VALUES"):
                shape.append(int(rest.pop(0)))
            if rest and _s(rest[0]).upper() == "BLOB":
                return st.tensorset(key, dtype, shape, blob=bytes(rest[1]))
            if rest and _s(rest[0]).upper() == "VALUES":
                return st.tensorset(key, dtype, shape, values=[float(_s(v)) for v in rest[1:]])
            return st.tensorset(key, dtype, shape)
        if cmd == "AI.TENSORGET":
            return self._tensorget(_s(a[0]), _s(a[1]) if len(a) > 1 else "VALUES")
        if cmd == "AI.MODELSET":
            return self._modelset(_s(a[0]), _s(a[1]), _s(a[2]), list(a[3:]))
        if cmd == "AI.SCRIPTSET":
            rest = list(a[2:])
            if rest and isinstance(rest[0], (bytes, str)) and _s(rest[0]).upper() == "SOURCE":
                rest = rest[1:]
            return st.scriptset(_s(a[0]), _s(a[1]), _s(rest[0]))
        if cmd in ("AI.SCRIPTRUN", "AI.MODELRUN"):
            return st.execute_command(cmd, *[_s(x) for x in a])
        raise RespError(f"ERR unknown command '{cmd}'")

    # -- connection loop
    def _handle(self, sock: socket.socket):
        import hmac

        rd = _Reader(sock)
        authed = self.requirepass is None
        while True:
            try:
                req = rd.value(self.max_bulk)
            except (ConnectionError, OSError):
                return
            except (ValueError, RecursionError) as e:
                sock.sendall(encode(RespError(f"ERR {e}")))
                return
            if not isinstance(req, list) or not all(isinstance(x, (bytes, str)) for x in req):
                sock.sendall(encode(RespError("ERR protocol error: expected an array of bulk strings")))
                continue
            cmd = _s(req[0]).upper() if req else ""
            if cmd == "QUIT":
                sock.sendall(encode("OK"))
                return
            if cmd == "AUTH":
                ok = self.requirepass is not None and len(req) == 2 and hmac.compare_digest(
                    _s(req[1]).encode(), self.requirepass.encode())
                authed = authed or ok
                sock.sendall(encode("OK" if ok else RespError("WRONGPASS invalid password")))
                continue
            if not authed:
                sock.sendall(encode(RespError("NOAUTH Authentication required.")))
                continue
            try:
                out = self.execute(req)
            except RespError as e:
                out = e
            except Exception as e:  # noqa: BLE001 -- every command error is a reply, never a dropped connection
                out = RespError(f"ERR {type(e).__name__}: {e}")
            sock.sendall(encode(out))

    def start(self) -> int:
        outer = self

        class _H(socketserver.BaseRequestHandler):
            def handle(self):
                outer._handle(self.request)

        class _S(socketserver.ThreadingTCPServer):
            daemon_threads = True
            allow_reuse_address = True

        self._srv = _S((self.host, self.port), _H)
        self.port = self._srv.server_address[1]
        self._thread = threading.Thread(target=self._srv.serve_forever, daemon=True)
        self._thread.start()
        return self.port

    def stop(self):
        if self._srv is not None:
            self._srv.shutdown()
            self._srv.server_close()
            self._srv = None
        self._tmp.cleanup()


# ---------------------------------------------------------------- client


class RespClient:
    """Minimal redis-py-style client: `execute_command(*args)` sends one RESP command and returns the decoded reply
    (bulk strings as bytes, arrays as lists); an error reply raises RespError."""

    def __init__(self, host: str = "127.0.0.1", port: int = 6379, timeout: float | None = 60.0,
                 password: str | None = None):
        self.sock = socket.create_connection((host, port), timeout=timeout)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.rd = _Reader(self.sock)
        if password is not None:
            self.execute_command("AUTH", password)

    def execute_command(self, *args):
        self.sock.sendall(encode_command(*args))
        r = self.rd.value()
        if isinstance(r, RespError):
            raise r
        return r

    def ping(self) -> bool:
        return self.execute_command("PING") == "PONG"

    def close(self):
        try:
            self.sock.sendall(encode_command("QUIT"))
            self.rd.value()
        except OSError:
            pass
        self.sock.close()


def saved_model_blob(path: str) -> bytes:
    """tar (in memory) of a saved-model export directory: the AI.MODELSET ... BLOB payload."""
    buf = io.BytesIO()
    with tarfile.open(fileobj=buf, mode="w") as tf:
        for name in sorted(os.listdir(path)):
            tf.add(os.path.join(path, name), arcname=name)
    return buf.getvalue()


def main(argv=None):
    import argparse

    ap = argparse.ArgumentParser(prog="python -m mifx.serving.resp_server", description=__doc__.split("\n")[0])
    ap.add_argument("--host", default="127.0.0.1",
                    help="bind address; a non-loopback address needs --requirepass (or MIFX_RESP_PASSWORD)")
    ap.add_argument("--port", type=int, default=6379)
    ap.add_argument("--requirepass", default=os.environ.get("MIFX_RESP_PASSWORD"))
    ap.add_argument("--model-root", action="append", default=[],
                    help="server-side directory AI.MODELSET PATH may load from (repeatable; default: PATH disabled)")
    a = ap.parse_args(argv)
    srv = RespServer(host=a.host, port=a.port, requirepass=a.requirepass, model_roots=a.model_root)
    port = srv.start()
    print(f"mifx RESP tensor store listening on {a.host}:{port}", flush=True)
    try:
        threading.Event().wait()
    except KeyboardInterrupt:
        srv.stop()


if __name__ == "__main__":
    main()
