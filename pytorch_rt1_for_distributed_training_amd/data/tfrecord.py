"""TensorFlow-free TFRecord + ``tf.train.Example`` codec, and an RLDS episode reader on top of it.

The reference reads Language-Table's RLDS release through ``tensorflow_datasets``
(``/root/reference/rlds_np_convert.py:1-40``, ``language_table/train/input_pipeline_rlds.py``).  TensorFlow is not
part of this stack, but the on-disk format is simple and fixed, so it is decoded here directly:

* TFRecord framing: ``uint64 length | uint32 masked_crc32c(length) | data | uint32 masked_crc32c(data)``;
* ``tf.train.Example`` protobuf wire format: ``Example{features=1}``, ``Features{map<string, Feature> feature=1}``,
  ``Feature{oneof bytes_list=1 | float_list=2 | int64_list=3}``, each list a repeated field 1 (packed or not);
* tfds stores one RLDS episode per Example, its ``steps`` sequence flattened into ``steps/<key>[/<subkey>]``
  features of ``n_steps`` entries each (images as one encoded PNG / JPEG per step, int32 as int64).

    for ep in read_rlds_episodes(builder_dir):            # dicts of per-step numpy arrays, "steps" as in tfds
        ep["steps"]["observation"]["rgb"].shape           # (T, H, W, 3) uint8
"""
from __future__ import annotations

import glob
import io
import json
import os
import struct
from typing import Dict, Iterable, Iterator, List, Optional, Sequence, Union

import numpy as np

# ---------------------------------------------------------------- CRC-32C (Castagnoli), TFRecord's masked form
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)
del _i, _c


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    t = _TABLE
    for b in data:
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------- TFRecord framing
def read_records(path: str, verify_data: bool = False) -> Iterator[bytes]:
    """Yield the records of one TFRecord file.  The length CRC is always checked; the data CRC (pure Python,
    ~5 MB/s) only with ``verify_data``."""
    with open(path, "rb") as fh:
        while True:
            head = fh.read(12)
            if not head:
                return
            if len(head) < 12:
                raise ValueError(f"{path}: truncated record header")
            length, lcrc = struct.unpack("<QI", head)
            if masked_crc(head[:8]) != lcrc:
                raise ValueError(f"{path}: corrupt record length")
            data = fh.read(length)
            tail = fh.read(4)
            if len(data) < length or len(tail) < 4:
                raise ValueError(f"{path}: truncated record")
            if verify_data and masked_crc(data) != struct.unpack("<I", tail)[0]:
                raise ValueError(f"{path}: corrupt record data")
            yield data


def write_records(path: str, records: Iterable[bytes]) -> None:
    with open(path, "wb") as fh:
        for r in records:
            n = struct.pack("<Q", len(r))
            fh.write(n + struct.pack("<I", masked_crc(n)) + r + struct.pack("<I", masked_crc(r)))


# ---------------------------------------------------------------- protobuf wire format
def _varint(buf: memoryview, i: int):
    shift = result = 0
    while True:
        b = buf[i]
        i += 1
        result |= (b & 0x7F) << shift
        if not b & 0x80:
            return result, i
        shift += 7


def _fields(buf: memoryview):
    """(field number, wire type, value) over one message; LEN values are memoryviews."""
    i, n = 0, len(buf)
    while i < n:
        key, i = _varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _varint(buf, i)
        elif wt == 1:
            v, i = buf[i:i + 8], i + 8
        elif wt == 2:
            ln, i = _varint(buf, i)
            v, i = buf[i:i + ln], i + ln
        elif wt == 5:
            v, i = buf[i:i + 4], i + 4
        else:
            raise ValueError(f"unsupported protobuf wire type {wt}")
        yield num, wt, v


def _feature(buf: memoryview) -> Union[List[bytes], np.ndarray]:
    for num, _, body in _fields(buf):
        if num == 1:                                                      # BytesList
            return [bytes(v) for f, _, v in _fields(body) if f == 1]
        if num == 2:                                                      # FloatList
            parts = [np.frombuffer(v, "<f4") for f, _, v in _fields(body) if f == 1]
            return np.concatenate(parts).astype(np.float32) if parts else np.zeros(0, np.float32)
        if num == 3:                                                      # Int64List
            vals: List[int] = []
            for f, wt, v in _fields(body):
                if f != 1:
                    continue
                if wt == 2:
                    j = 0
                    while j < len(v):
                        x, j = _varint(v, j)
                        vals.append(x)
                else:
                    vals.append(v)
            return (np.array(vals, np.uint64).view(np.int64) if vals else np.zeros(0, np.int64))
    return []


def parse_example(data: bytes) -> Dict[str, Union[List[bytes], np.ndarray]]:
    """``tf.train.Example`` bytes -> {feature name: list of bytes | float32 array | int64 array}."""
    out: Dict[str, Union[List[bytes], np.ndarray]] = {}
    for num, _, feats in _fields(memoryview(data)):
        if num != 1:
            continue
        for fnum, _, entry in _fields(feats):
            if fnum != 1:
                continue
            key, val = None, memoryview(b"")
            for enum, _, v in _fields(entry):
                if enum == 1:
                    key = bytes(v).decode("utf-8")
                elif enum == 2:
                    val = v
            out[key] = _feature(val)
    return out


def _enc_varint(x: int) -> bytes:
    x &= (1 << 64) - 1
    out = bytearray()
    while True:
        b = x & 0x7F
        x >>= 7
        if x:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _len_field(num: int, body: bytes) -> bytes:
    return _enc_varint(num << 3 | 2) + _enc_varint(len(body)) + body


def encode_example(features: Dict[str, Union[Sequence[bytes], np.ndarray]]) -> bytes:
    """Inverse of :func:`parse_example`: bytes lists, float arrays (FloatList) and integer arrays (Int64List)."""
    entries = b""
    for key, val in features.items():
        if isinstance(val, (list, tuple)) and (not val or isinstance(val[0], (bytes, bytearray))):
            feat = _len_field(1, b"".join(_len_field(1, bytes(v)) for v in val))
        else:
            a = np.asarray(val).reshape(-1)
            if a.dtype.kind == "f":
                feat = _len_field(2, _len_field(1, a.astype("<f4").tobytes()))
            else:
                feat = _len_field(3, _len_field(1, b"".join(_enc_varint(int(x)) for x in a)))
        entries += _len_field(1, _len_field(1, key.encode("utf-8")) + _len_field(2, feat))
    return _len_field(1, entries)


# ---------------------------------------------------------------- RLDS episodes
def _unflatten(flat: Dict[str, object]) -> Dict:
    root: Dict = {}
    for key, v in flat.items():
        node = root
        parts = key.split("/")
        for p in parts[:-1]:
            node = node.setdefault(p, {})
        node[parts[-1]] = v
    return root


def _is_image(b: bytes) -> bool:
    return b.startswith(b"\x89PNG\r\n\x1a\n") or b.startswith(b"\xff\xd8\xff")            # PNG / JPEG


def _decode_image(b: bytes) -> np.ndarray:
    from PIL import Image
    return np.asarray(Image.open(io.BytesIO(b)).convert("RGB"))


def _feature_shapes(builder_dir: str) -> Dict[str, List[int]]:
    """Per-step shapes of the ``steps`` tensors from tfds' ``features.json`` when present ({} otherwise)."""
    path = os.path.join(builder_dir, "features.json")
    if not os.path.exists(path):
        return {}
    shapes: Dict[str, List[int]] = {}

    def walk(node, prefix):
        if isinstance(node, dict):
            if "shape" in node and isinstance(node["shape"], dict) and "dimensions" in node["shape"]:
                shapes[prefix] = [int(d) for d in node["shape"]["dimensions"]]
            for k, v in node.items():
                if k == "features" and isinstance(v, dict):
                    for name, sub in v.items():
                        walk(sub, f"{prefix}/{name}" if prefix else name)
                elif isinstance(v, dict):
                    walk(v, prefix)
    with open(path) as fh:
        walk(json.load(fh), "")
    return shapes


def episode_from_example(ex: Dict[str, object], shapes: Optional[Dict[str, List[int]]] = None) -> Dict:
    """One tfds RLDS Example -> nested dict; ``steps/*`` become per-step arrays [T, ...] (images decoded)."""
    shapes = shapes or {}
    n = None
    for key in ("steps/is_first", "steps/is_last", "steps/is_terminal", "steps/reward"):
        if key in ex:
            n = len(ex[key])
            break
    flat: Dict[str, object] = {}
    for key, v in ex.items():
        if key.startswith("steps/") and n:
            if isinstance(v, list):                                       # encoded images / strings, one per step
                flat[key] = np.stack([_decode_image(b) for b in v]) if v and _is_image(v[0]) else v
                continue
            arr = np.asarray(v)
            shape = [d for d in shapes.get(key, []) if d != -1]
            arr = arr.reshape([n] + shape) if shape and int(np.prod(shape)) * n == arr.size else arr.reshape(n, -1)
            if key.rsplit("/", 1)[-1].startswith("is_"):
                arr = arr.reshape(n).astype(bool)
            flat[key] = arr
        else:
            flat[key] = v
    return _unflatten(flat)


def rlds_shards(builder_dir: str, split: str = "train") -> List[str]:
    files = sorted(glob.glob(os.path.join(builder_dir, f"*-{split}.tfrecord*")))
    if not files:
        raise FileNotFoundError(f"no '{split}' TFRecord shards under {builder_dir}")
    return files


def read_rlds_episodes(builder_dir: str, split: str = "train", verify_data: bool = False,
                       select=None, limit: int = 0) -> Iterator[Dict]:
    """Episodes of a tfds RLDS builder directory, in shard order, without TensorFlow.

    ``select(i) -> bool`` picks records by their global index BEFORE they are parsed: a rank's skipped records cost a
    framing read only, never an Example parse or an image decode.  ``limit`` stops after that many records."""
    shapes = _feature_shapes(builder_dir)
    i = 0
    for path in rlds_shards(builder_dir, split):
        for rec in read_records(path, verify_data):
            if limit and i >= limit:
                return
            take = select is None or select(i)
            i += 1
            if take:
                yield episode_from_example(parse_example(rec), shapes)
