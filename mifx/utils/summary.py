"""TensorBoard-compatible scalar summaries without TensorFlow/TensorBoard installed.

Writes `events.out.tfevents.<time>.<host>` files: TFRecord framing (masked CRC32C, native
mifx.io.tfrecord) around hand-encoded `tensorflow.Event` protos — `file_version` first, then
`Event{wall_time, step, summary{value{tag, simple_value}}}` per scalar. TensorBoard reads them as the
`tf.summary.scalar` + `FileWriter` output of the reference (`fairing_tf.py:54-74`,
`deep_cnn.py:402,415-417`). `read_scalars` parses the files back (used by tests and dashboards)."""
from __future__ import annotations

import os
import socket
import struct
import time

from ..io.tfrecord import _ld, _varint, masked_crc32c, read_tfrecords


def _double(field: int, v: float) -> bytes:
    return _varint((field << 3) | 1) + struct.pack("<d", v)


def _float(field: int, v: float) -> bytes:
    return _varint((field << 3) | 5) + struct.pack("<f", v)


def _int(field: int, v: int) -> bytes:
    return _varint(field << 3) + _varint(v)


def encode_scalar_event(tag: str, value: float, step: int, wall_time: float | None = None) -> bytes:
    val = _ld(1, tag.encode()) + _float(2, float(value))
    summary = _ld(1, val)
    return _double(1, time.time() if wall_time is None else wall_time) + _int(2, int(step)) + _ld(5, summary)


class SummaryWriter:
    def __init__(self, logdir: str, filename_suffix: str = ""):
        os.makedirs(logdir, exist_ok=True)
        self.path = os.path.join(logdir, f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}"
                                         f"{filename_suffix}")
        self._f = open(self.path, "wb")
        self._write(_double(1, time.time()) + _ld(3, b"brain.Event:2"))

    def _write(self, rec: bytes) -> None:
        hdr = struct.pack("<Q", len(rec))
        self._f.write(hdr + struct.pack("<I", masked_crc32c(hdr)) + rec + struct.pack("<I", masked_crc32c(rec)))

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        self._write(encode_scalar_event(tag, value, step))

    def flush(self) -> None:
        self._f.flush()

    def close(self) -> None:
        if not self._f.closed:
            self._f.close()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def _fields(buf: bytes):
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        f, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 1:
            v = struct.unpack_from("<d", buf, i)[0]
            i += 8
        elif wt == 5:
            v = struct.unpack_from("<f", buf, i)[0]
            i += 4
        elif wt == 2:
            n, i = _read_varint(buf, i)
            v = buf[i:i + n]
            i += n
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield f, v


def _read_varint(buf: bytes, i: int):
    shift = v = 0
    while True:
        b = buf[i]
        i += 1
        v |= (b & 0x7F) << shift
        if not b & 0x80:
            return v, i
        shift += 7


def read_scalars(path_or_dir: str, with_wall_time: bool = False) -> dict[str, list[tuple]]:
    """{tag: [(step, value), ...]} from one events file or every events file in a directory
    ([(wall_time, step, value), ...] with with_wall_time)."""
    files = [path_or_dir] if os.path.isfile(path_or_dir) else sorted(
        os.path.join(path_or_dir, f) for f in os.listdir(path_or_dir) if f.startswith("events.out.tfevents"))
    out: dict[str, list] = {}
    for p in files:
        for rec in read_tfrecords(p, compression=""):
            ev = dict(_fields(rec))
            if 5 not in ev:
                continue
            for f, val in _fields(ev[5]):
                if f != 1:
                    continue
                d = dict(_fields(val))
                row = (int(ev.get(2, 0)), float(d.get(2, 0.0)))
                out.setdefault(d[1].decode(), []).append((float(ev.get(1, 0.0)),) + row if with_wall_time else row)
    return out
