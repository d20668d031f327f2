"""Minimal TensorBoard event-file writer (tensorboard is not a dependency).

Writes the TFRecord framing (``uint64 length, masked crc32c(length), data,
masked crc32c(data)``) of ``tensorflow.Event`` protos holding scalar
summaries, hand-encoded in protobuf wire format:
``Event{wall_time=1:double, step=2:int64, file_version=3:string,
summary=5:Summary{value=1:Value{tag=1:string, simple_value=2:float}}}``.
The reference logs to TensorBoard through Lightning
(``distribute_train.py:225-228``); scalars written here open in TensorBoard.
"""
from __future__ import annotations

import os
import socket
import struct
import time


def _make_crc_table():
    poly = 0x82F63B78
    table = []
    for i in range(256):
        c = i
        for _ in range(8):
            c = (c >> 1) ^ poly if c & 1 else c >> 1
        table.append(c)
    return table


_TABLE = _make_crc_table()


def crc32c(data: bytes) -> int:
    c = 0xFFFFFFFF
    for b in data:
        c = _TABLE[(c ^ b) & 0xFF] ^ (c >> 8)
    return c ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _field_bytes(num: int, payload: bytes) -> bytes:
    return _varint((num << 3) | 2) + _varint(len(payload)) + payload


def encode_event(step: int, wall_time: float, tag: str = None, value: float = None, file_version: str = None) -> bytes:
    msg = _varint((1 << 3) | 1) + struct.pack("<d", wall_time)
    msg += _varint((2 << 3) | 0) + _varint(int(step))
    if file_version is not None:
        msg += _field_bytes(3, file_version.encode())
    if tag is not None:
        val = _field_bytes(1, tag.encode()) + _varint((2 << 3) | 5) + struct.pack("<f", float(value))
        msg += _field_bytes(5, _field_bytes(1, val))
    return msg


class EventWriter:
    def __init__(self, logdir: str):
        os.makedirs(logdir, exist_ok=True)
        name = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}.0"
        self.path = os.path.join(logdir, name)
        self._f = open(self.path, "ab")
        self._write(encode_event(0, time.time(), file_version="brain.Event:2"))

    def _write(self, data: bytes):
        header = struct.pack("<Q", len(data))
        self._f.write(header + struct.pack("<I", masked_crc(header)) + data + struct.pack("<I", masked_crc(data)))

    def add_scalar(self, tag: str, value: float, step: int):
        self._write(encode_event(step, time.time(), tag, value))

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


def read_scalars(path: str):
    """Parse an event file written by ``EventWriter`` -> list of (step, tag, value)."""
    out = []
    with open(path, "rb") as f:
        data = f.read()
    i = 0
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        i += 12
        rec = data[i:i + n]
        i += n + 4
        step, tag, val = _parse_event(rec)
        if tag is not None:
            out.append((step, tag, val))
    return out


def _read_varint(b, i):
    shift = res = 0
    while True:
        c = b[i]
        i += 1
        res |= (c & 0x7F) << shift
        if not c & 0x80:
            return res, i
        shift += 7


def _parse_fields(b):
    i, out = 0, []
    while i < len(b):
        key, i = _read_varint(b, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(b, i)
        elif wt == 1:
            v = b[i:i + 8]
            i += 8
        elif wt == 5:
            v = b[i:i + 4]
            i += 4
        else:
            n, i = _read_varint(b, i)
            v = b[i:i + n]
            i += n
        out.append((num, v))
    return out


def _parse_event(rec):
    step, tag, val = 0, None, None
    for num, v in _parse_fields(rec):
        if num == 2:
            step = v
        elif num == 5:
            for _, value in _parse_fields(v):
                for n2, v2 in _parse_fields(value):
                    if n2 == 1:
                        tag = v2.decode()
                    elif n2 == 2:
                        val = struct.unpack("<f", v2)[0]
    return step, tag, val
