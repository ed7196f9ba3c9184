"""String-vocabulary kernels (csrc/vocab.hip): FNV-1a string hashing, GPU hash-table counting and
vocabulary lookup for tft.compute_and_apply_vocabulary / string_to_int / hash_strings (SURVEY KN7,
reference call sites `airflow-dags/taxi_utils.py:121-126`, `kubeflow-pipelines/taxi/preprocessing.py:77-85`).

Host side packs a string column into one byte buffer + int64 offsets. Counting runs on the device;
the handful of unique (count, token) pairs come back to the host for the tft ordering (frequency
descending, ties by token descending) and the top_k / frequency_threshold cut. Any genuine 64-bit
hash collision between distinct strings is detected on the device (byte comparison) and the column
is then processed by the exact CPU path, so results are always identical to :mod:`mifx.transform.api`.
On a CUDA/HIP device the native library is REQUIRED; on CPU the numpy/Python path runs."""
from __future__ import annotations

import functools

import numpy as np
import torch

from . import _lib
from ._lib import I32, I64, VP, check, ptr, sig, stream_handle

_INT_MAX = 2**31 - 1


@functools.lru_cache(maxsize=None)
def _fns():
    lib = _lib.load("vocab")
    return {
        "hash": sig(lib, "mifx_vocab_hash", [VP, VP, I64, VP, VP]),
        "count": sig(lib, "mifx_vocab_count", [VP, VP, I64, VP, VP, VP, VP, I64, VP, VP]),
        "build": sig(lib, "mifx_vocab_build", [VP, VP, I32, VP, VP, I64, VP, VP]),
        "lookup": sig(lib, "mifx_vocab_lookup", [VP, VP, I64, VP, VP, I64, VP, VP, I32, I32, I64, VP, VP]),
    }


def _is_gpu(device) -> bool:
    return device is not None and torch.device(device).type == "cuda"


def _as_str(v) -> str:
    if v is None:
        return ""
    return v.decode() if isinstance(v, bytes) else str(v)


def _is_arrow(values) -> bool:
    return type(values).__module__.startswith("pyarrow")


def _pack_arrow(values):
    """Arrow string/binary column -> its own (data, int64 offsets) buffers: no per-row Python work
    (nulls read as "")."""
    import pyarrow as pa
    import pyarrow.compute as pc

    a = values.combine_chunks() if isinstance(values, pa.ChunkedArray) else values
    if a.null_count:
        a = pc.fill_null(a, "")
    a = a.cast(pa.large_binary())  # int64 offsets
    _, ob, db = a.buffers()
    offs = np.frombuffer(ob, dtype=np.int64)[a.offset:a.offset + len(a) + 1]
    buf = np.frombuffer(db, dtype=np.uint8) if db is not None and db.size else np.zeros(1, dtype=np.uint8)
    return buf, offs, lambda i: a[i].as_py().decode()


def pack_strings(values) -> tuple[np.ndarray, np.ndarray, "callable"]:
    """-> (uint8 byte buffer, int64 offsets [n+1], row -> str) for a column of str/bytes/None, or an
    Arrow string/binary column (zero-copy)."""
    if _is_arrow(values):
        return _pack_arrow(values)
    enc = [v if isinstance(v, bytes) else _as_str(v).encode() for v in values]
    lens = np.fromiter((len(b) for b in enc), dtype=np.int64, count=len(enc))
    offs = np.zeros(len(enc) + 1, dtype=np.int64)
    np.cumsum(lens, out=offs[1:])
    buf = np.frombuffer(b"".join(enc), dtype=np.uint8) if offs[-1] else np.zeros(1, dtype=np.uint8)
    return buf, offs, lambda i: enc[i].decode()


def _to_dev(buf: np.ndarray, offs: np.ndarray, dev):
    # host buffers may be read-only views (bytes / Arrow): torch copies them to the device anyway
    return (torch.from_numpy(np.require(buf, requirements=["C", "W"])).to(dev),
            torch.from_numpy(np.require(offs, requirements=["C", "W"])).to(dev))


def _host_strs(values) -> list[str]:
    if _is_arrow(values):
        return ["" if v is None else (v.decode() if isinstance(v, bytes) else v) for v in values.to_pylist()]
    return [_as_str(v) for v in values]


def _capacity(n: int) -> int:
    """power-of-two table size >= 2n (>= 1024)."""
    return 1 << max(10, int(2 * max(n, 1) - 1).bit_length())


_FNV_OFF, _FNV_PRIME, _M64 = 0xCBF29CE484222325, 0x100000001B3, 0xFFFFFFFFFFFFFFFF


def fnv1a64(b: bytes) -> int:
    h = _FNV_OFF
    for c in b:
        h = ((h ^ c) * _FNV_PRIME) & _M64
    return h


def hash_strings(values, device=None) -> np.ndarray:
    """uint64 FNV-1a fingerprints of a string column (== mifx.transform.api.fingerprint64)."""
    if not _is_gpu(device):
        return np.array([fnv1a64(v.encode()) for v in _host_strs(values)], dtype=np.uint64)
    dev = torch.device(device)
    buf, offs, _ = pack_strings(values)
    n = len(offs) - 1
    tb, to = _to_dev(buf, offs, dev)
    out = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    check(_fns()["hash"](ptr(tb), ptr(to), n, ptr(out), stream_handle(dev)), "mifx_vocab_hash")
    return out[:n].cpu().numpy().view(np.uint64)


def count_unique(values, device=None) -> tuple[list[str], list[int]] | None:
    """Unique tokens and their counts. GPU: hash-table count; returns None on a detected hash
    collision / table overflow (the caller then uses the exact CPU path)."""
    if not _is_gpu(device):
        vals, counts = np.unique(np.array(_host_strs(values), dtype=object), return_counts=True)
        return [str(v) for v in vals.tolist()], [int(c) for c in counts.tolist()]
    dev = torch.device(device)
    buf, offs, get = pack_strings(values)
    n = len(offs) - 1
    if n == 0:
        return [], []
    cap = _capacity(n)
    tb, to = _to_dev(buf, offs, dev)
    hsh = torch.empty(n, dtype=torch.int64, device=dev)
    keys = torch.zeros(cap, dtype=torch.int64, device=dev)
    counts = torch.zeros(cap, dtype=torch.int32, device=dev)
    rep = torch.full((cap,), _INT_MAX, dtype=torch.int32, device=dev)
    flags = torch.zeros(2, dtype=torch.int32, device=dev)
    check(_fns()["count"](ptr(tb), ptr(to), n, ptr(hsh), ptr(keys), ptr(counts), ptr(rep), cap, ptr(flags),
                          stream_handle(dev)), "mifx_vocab_count")
    if int(flags.abs().sum().item()) != 0:
        return None
    used = counts > 0
    c = counts[used].cpu().tolist()
    r = rep[used].cpu().tolist()
    return [get(i) for i in r], c


def order_vocabulary(tokens: list[str], counts: list[int], top_k: int | None = None,
                     frequency_threshold: int | None = None) -> list[str]:
    """tft ordering: frequency descending, ties broken by token descending; then threshold / top_k."""
    order = sorted(zip(counts, tokens), reverse=True)
    if frequency_threshold is not None:
        order = [(c, v) for c, v in order if c >= frequency_threshold]
    if top_k is not None:
        order = order[:top_k]
    return [v for _, v in order]


def vocabulary(values, top_k: int | None = None, frequency_threshold: int | None = None, device=None) -> list[str]:
    got = count_unique(values, device=device)
    if got is None:  # collision detected on the device: exact host path
        got = count_unique(values, device=None)
    return order_vocabulary(got[0], got[1], top_k, frequency_threshold)


def _lookup_host(values, vocab: list[str], default_value: int, num_oov_buckets: int) -> np.ndarray:
    index = {v: i for i, v in enumerate(vocab)}
    n = len(vocab)
    out = np.empty(len(values), dtype=np.int64)
    for i, s in enumerate(_host_strs(values)):
        j = index.get(s)
        if j is not None:
            out[i] = j
        elif num_oov_buckets > 0:
            out[i] = n + fnv1a64(s.encode()) % num_oov_buckets
        else:
            out[i] = default_value
    return out


class DeviceVocabulary:
    """A vocabulary resident on the device (hash table + packed bytes) for repeated apply calls."""

    def __init__(self, vocab: list[str], device):
        self.vocab = list(vocab)
        self.device = torch.device(device)
        vbuf, voffs, _ = pack_strings(self.vocab)
        self.cap = _capacity(len(self.vocab))
        self.vbuf, self.voffs = _to_dev(vbuf, voffs, self.device)
        self.keys = torch.zeros(self.cap, dtype=torch.int64, device=self.device)
        self.vals = torch.zeros(self.cap, dtype=torch.int32, device=self.device)
        flag = torch.zeros(1, dtype=torch.int32, device=self.device)
        check(_fns()["build"](ptr(self.vbuf), ptr(self.voffs), len(self.vocab), ptr(self.keys), ptr(self.vals),
                              self.cap, ptr(flag), stream_handle(self.device)), "mifx_vocab_build")
        # two vocab entries with one hash (or a repeated entry): the device table is unusable
        self.ok = int(flag.item()) == 0 and len(set(self.vocab)) == len(self.vocab)

    def lookup(self, values, default_value: int = -1, num_oov_buckets: int = 0) -> np.ndarray:
        if not self.ok:
            return _lookup_host(values, self.vocab, default_value, num_oov_buckets)
        buf, offs, _ = pack_strings(values)
        n = len(offs) - 1
        if n == 0:
            return np.zeros(0, dtype=np.int64)
        tb, to = _to_dev(buf, offs, self.device)
        out = torch.empty(n, dtype=torch.int64, device=self.device)
        check(_fns()["lookup"](ptr(tb), ptr(to), n, ptr(self.keys), ptr(self.vals), self.cap, ptr(self.vbuf),
                               ptr(self.voffs), len(self.vocab), int(num_oov_buckets), int(default_value), ptr(out),
                               stream_handle(self.device)), "mifx_vocab_lookup")
        return out.cpu().numpy()


def apply_vocabulary(values, vocab: list[str], default_value: int = -1, num_oov_buckets: int = 0,
                     device=None) -> np.ndarray:
    if not _is_gpu(device):
        return _lookup_host(values, vocab, default_value, num_oov_buckets)
    return DeviceVocabulary(vocab, device).lookup(values, default_value, num_oov_buckets)
