"""TFRecord container (+gzip) and `tf.train.Example` wire-format codec, dependency-free.

Reference: TFX ExampleGen writes gzip TFRecords of tf.Example that Transform/Trainer read back
(`airflow-dags/taxi_utils.py:79-83,260-281` — `_gzip_reader_fn`, `read_batch_features`).
Record framing: u64 length, masked CRC32C(length), payload, masked CRC32C(payload). CRC32C is
computed by the native host library (csrc/io_native.cpp) when built, else a table fallback.
"""
from __future__ import annotations

import ctypes
import gzip
import struct
from typing import Iterable, Iterator

import numpy as np

# ---------------------------------------------------------------------------------- CRC32C
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)

_native = None


def _native_lib():
    global _native
    if _native is None:
        try:
            from ..ops import _lib

            lib = _lib.load("io_native")
            lib.mifx_crc32c.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_uint32]
            lib.mifx_crc32c.restype = ctypes.c_uint32
            _native = lib
        except Exception:  # host library not built: pure-Python fallback
            _native = False
    return _native


def crc32c(data: bytes, crc: int = 0) -> int:
    lib = _native_lib()
    if lib:
        return lib.mifx_crc32c(data, len(data), crc)
    crc ^= 0xFFFFFFFF
    t = _TABLE
    for b in data:
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _open(path: str, mode: str, compression: str | None):
    if compression is None:
        compression = "GZIP" if path.endswith(".gz") else ""
    if compression.upper() == "GZIP":
        return gzip.open(path, mode)
    return open(path, mode)


def write_tfrecords(path: str, records: Iterable[bytes], compression: str | None = None) -> int:
    n = 0
    with _open(path, "wb", compression) as f:
        for r in records:
            hdr = struct.pack("<Q", len(r))
            f.write(hdr)
            f.write(struct.pack("<I", masked_crc32c(hdr)))
            f.write(r)
            f.write(struct.pack("<I", masked_crc32c(r)))
            n += 1
    return n


def read_tfrecords(path: str, compression: str | None = None, verify: bool = True) -> Iterator[bytes]:
    with _open(path, "rb", compression) as f:
        while True:
            hdr = f.read(8)
            if not hdr:
                return
            if len(hdr) < 8:
                raise IOError(f"{path}: truncated record header")
            (n,) = struct.unpack("<Q", hdr)
            (hc,) = struct.unpack("<I", f.read(4))
            if verify and hc != masked_crc32c(hdr):
                raise IOError(f"{path}: corrupt record length crc")
            data = f.read(n)
            (dc,) = struct.unpack("<I", f.read(4))
            if verify and dc != masked_crc32c(data):
                raise IOError(f"{path}: corrupt record data crc")
            yield data


# ------------------------------------------------------------------------- protobuf codec
def _varint(v: int) -> bytes:
    v &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _ld(field: int, payload: bytes) -> bytes:
    return _varint((field << 3) | 2) + _varint(len(payload)) + payload


def _read_varint(buf: bytes, i: int) -> tuple[int, int]:
    shift = v = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, i
        shift += 7


def _fields(buf: bytes):
    i, n = 0, len(buf)
    while i < n:
        key, i = _read_varint(buf, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
            yield f, wt, v
        elif wt == 2:
            ln, i = _read_varint(buf, i)
            yield f, wt, buf[i:i + ln]
            i += ln
        elif wt == 5:
            yield f, wt, buf[i:i + 4]
            i += 4
        elif wt == 1:
            yield f, wt, buf[i:i + 8]
            i += 8
        else:
            raise ValueError(f"unsupported wire type {wt}")


def _feature_bytes(values) -> bytes:
    """Encode one Feature from a python list / numpy array / scalar."""
    if isinstance(values, (bytes, str)) or np.isscalar(values):
        values = [values]
    values = list(values)
    if not values:
        return _ld(3, b"")  # empty int64 list
    v0 = values[0]
    if isinstance(v0, (bytes, str)):
        body = b"".join(_ld(1, v.encode() if isinstance(v, str) else v) for v in values)
        return _ld(1, body)
    if isinstance(v0, (float, np.floating)):
        packed = np.asarray(values, "<f4").tobytes()
        return _ld(2, _ld(1, packed))
    packed = b"".join(_varint(int(v)) for v in values)
    return _ld(3, _ld(1, packed))


def encode_example(features: dict) -> bytes:
    entries = b"".join(_ld(1, _ld(1, k.encode()) + _ld(2, _feature_bytes(v))) for k, v in sorted(features.items()))
    return _ld(1, entries)


def _decode_feature(buf: bytes):
    for f, _, payload in _fields(buf):
        if f == 1:
            return [bytes(p) for ff, _, p in _fields(payload) if ff == 1]
        if f == 2:
            out = []
            for ff, wt, p in _fields(payload):
                if ff == 1:
                    out.extend(np.frombuffer(p, "<f4").tolist() if wt == 2 else [struct.unpack("<f", p)[0]])
            return out
        if f == 3:
            out = []
            for ff, wt, p in _fields(payload):
                if ff != 1:
                    continue
                if wt == 2:
                    j = 0
                    while j < len(p):
                        v, j = _read_varint(p, j)
                        out.append(v - (1 << 64) if v >= 1 << 63 else v)
                else:
                    out.append(p - (1 << 64) if p >= 1 << 63 else p)
            return out
    return []


def decode_example(buf: bytes) -> dict:
    out = {}
    for f, _, feats in _fields(buf):
        if f != 1:
            continue
        for ff, _, entry in _fields(feats):
            if ff != 1:
                continue
            key, val = None, b""
            for ef, _, p in _fields(entry):
                if ef == 1:
                    key = bytes(p).decode()
                elif ef == 2:
                    val = p
            out[key] = _decode_feature(val)
    return out
