"""Save / restore of a Language-Table board to a gzip-JSON file.

Behavioural spec: ``language_table/environments/utils/utils_pybullet.py:376-445`` -- the reference turns the
pybullet state (per-object ``ObjState`` / ``XarmState`` records) into plain JSON types, tags every typed record
with its class name, and writes ``{state, state_version, ts_ms, user, task, actions}`` through gzip;
``read_*`` checks the version and rebuilds the typed records.  Here the state is the planar simulator's
(``LanguageTable.get_state``: block poses, effector, arm joints, the task record) and the same file layout is
used, so a recorded board plus its action list replays on any host:

    write_state("ep.json.gz", env.get_state(), task=env.instruction_str, actions=acts)
    data = read_state("ep.json.gz"); env.set_state(data["state"])

numpy arrays and task records are tagged (``_serialized_obj_name``), as the reference tags its records.
"""
from __future__ import annotations

import dataclasses
import datetime
import getpass
import gzip
import json
import time
from typing import Any, Dict, List, Optional, Sequence

import numpy as np

from . import tasks

STATE_VERSION = 1
_TAG, _DATA = "_serialized_obj_name", "_serialized_data"
_TASK_TYPES = {c.__name__: c for c in (tasks.Block2BlockTaskInfo, tasks.Block2LocationTaskInfo,
                                       tasks.Block2RelativeLocationTaskInfo,
                                       tasks.Block2BlockRelativeLocationTaskInfo, tasks.SeparateBlocksTaskInfo,
                                       tasks.Point2BlockTaskInfo)}


def serialize(obj: Any) -> Any:
    """State -> JSON types.  Arrays keep dtype and shape; task records keep their class."""
    if isinstance(obj, dict):
        if _TAG in obj:
            raise ValueError(f"reserved key {_TAG!r} in a state dict")
        return {str(k): serialize(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return [serialize(v) for v in obj]
    if isinstance(obj, np.ndarray):
        return {_TAG: "ndarray", _DATA: {"dtype": obj.dtype.str, "shape": list(obj.shape),
                                         "values": obj.ravel().tolist()}}
    if type(obj).__name__ in _TASK_TYPES and dataclasses.is_dataclass(obj):
        return {_TAG: type(obj).__name__,
                _DATA: {f.name: serialize(getattr(obj, f.name)) for f in dataclasses.fields(obj)}}
    if isinstance(obj, (np.integer, np.floating, np.bool_)):
        return obj.item()
    if obj is None or isinstance(obj, (bool, int, float, str)):
        return obj
    raise ValueError(f"unhandled type {type(obj).__name__} for {obj!r}")


def deserialize(obj: Any) -> Any:
    """Inverse of :func:`serialize` (lists stay lists)."""
    if isinstance(obj, list):
        return [deserialize(v) for v in obj]
    if isinstance(obj, dict):
        if _TAG not in obj:
            return {k: deserialize(v) for k, v in obj.items()}
        name, data = obj[_TAG], obj[_DATA]
        if name == "ndarray":
            return np.asarray(data["values"], dtype=np.dtype(data["dtype"])).reshape(data["shape"])
        if name in _TASK_TYPES:
            return _TASK_TYPES[name](**{k: deserialize(v) for k, v in data.items()})
        raise ValueError(f"unsupported record {name!r}")
    return obj


def write_state(filename: str, state: Dict, task: Optional[str] = None,
                actions: Optional[Sequence] = None) -> None:
    data = {"state": serialize(state), "state_version": STATE_VERSION,
            "ts_ms": int(time.mktime(datetime.datetime.now().timetuple())) * 1000,
            "user": _user(), "task": task,
            "actions": [np.asarray(a, np.float64).tolist() for a in actions] if actions is not None else []}
    with gzip.open(filename, "wb") as fh:
        fh.write(json.dumps(data).encode("utf-8"))


def read_state(filename: str) -> Dict:
    with gzip.open(filename, "rb") as fh:
        data = json.loads(fh.read().decode("utf-8"))
    if not isinstance(data, dict):
        raise ValueError(f"{filename}: not a state record")
    if data.get("state_version") != STATE_VERSION:
        raise ValueError(f"incompatible state data (version {data.get('state_version')}, expected {STATE_VERSION})")
    data["state"] = _restore_tuples(deserialize(data["state"]))
    return data


def _restore_tuples(state: Dict) -> Dict:
    # set_state takes blocks_on_table as any sequence; keep the env's own tuple type after a round trip
    if isinstance(state, dict) and isinstance(state.get("blocks_on_table"), list):
        state["blocks_on_table"] = tuple(state["blocks_on_table"])
    return state


def _user() -> str:
    try:
        return getpass.getuser()
    except Exception:  # no passwd entry (containers)
        return "unknown"


def replay(env, data: Dict) -> List[Dict]:
    """Restore ``data["state"]`` into ``env`` and step its recorded actions; returns the observations."""
    env.set_state(data["state"])
    return [env.step(np.asarray(a))[0] for a in data["actions"]]
