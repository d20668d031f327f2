"""Local multi-process launcher: one child process per rank, started BEFORE the parent touches the GPU.

The reference gets its ranks from Lightning's DDP launcher, which re-executes the script once per visible GPU
(``/root/reference/distribute_train.py:231-238``).  Here ``bench.py --gpus N`` and ``distribute_train.py --gpus
0,1,..`` call :func:`spawn_local` when no launcher environment (``RANK``) is present: the parent only parses
arguments, picks a free rendezvous port on 127.0.0.1, starts N fresh ``python`` children with
``RANK/LOCAL_RANK/WORLD_SIZE/MASTER_ADDR/MASTER_PORT`` set, and waits.  It never initialises HIP itself (no
``torch.cuda`` call), so nothing is ever exec'ed from a GPU-initialised process.  If one rank fails, the others
are terminated (they would otherwise block forever in a collective) and the first failing exit code is returned.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time
from typing import Dict, List, Optional, Sequence


def free_port(host: str = "127.0.0.1") -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind((host, 0))
        return s.getsockname()[1]


def launcher_env_present() -> bool:
    return "RANK" in os.environ and "WORLD_SIZE" in os.environ


def spawn_local(nproc: int, argv: Sequence[str], extra_env: Optional[Dict[str, str]] = None,
                poll_s: float = 0.2, grace_s: float = 10.0) -> int:
    """Run ``python argv...`` as ``nproc`` ranks on this node; return 0 or the first non-zero exit code."""
    if nproc < 1:
        raise ValueError("nproc must be >= 1")
    base = dict(os.environ)
    base.update(extra_env or {})
    base["WORLD_SIZE"] = str(nproc)
    base["LOCAL_WORLD_SIZE"] = str(nproc)
    base["MASTER_ADDR"] = "127.0.0.1"
    base.setdefault("MASTER_PORT", str(free_port()))
    base["RT1_SPAWNED"] = "1"
    # N ranks x all-cores intra-op pools oversubscribe the CPU (gloo rehearsals); split the cores unless set
    base.setdefault("OMP_NUM_THREADS", str(max(1, (os.cpu_count() or 1) // nproc)))
    procs: List[subprocess.Popen] = []

    class _Signalled(Exception):
        def __init__(self, signum):
            self.signum = signum

    def _on_signal(signum, _frame):
        raise _Signalled(signum)

    # a scheduler / plain kill that signals only the parent must not orphan the ranks (they would sit in a
    # collective holding their GPUs): SIGTERM / SIGHUP tear the ranks down and return 128 + signum
    previous = {}
    for sig in (signal.SIGTERM, signal.SIGHUP):
        try:
            previous[sig] = signal.signal(sig, _on_signal)
        except (ValueError, OSError):      # not the main thread: leave the handlers alone
            pass
    rc = 0
    try:
        # spawning inside the try: a signal that lands while ranks are still being started tears down the ones
        # already running instead of orphaning them
        for r in range(nproc):
            env = dict(base, RANK=str(r), LOCAL_RANK=str(r))
            procs.append(subprocess.Popen([sys.executable] + list(argv), env=env))
        alive = set(range(nproc))
        while alive:
            for r in sorted(alive):
                code = procs[r].poll()
                if code is None:
                    continue
                alive.discard(r)
                if code != 0 and rc == 0:
                    rc = code
                    print(f"[launch] rank {r} exited with {code}; stopping the other ranks", file=sys.stderr,
                          flush=True)
                    _terminate([procs[i] for i in alive], grace_s)
                    alive.clear()
                    break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        _ignore_signals(previous)
        _terminate(procs, grace_s)
        rc = rc or 130
    except _Signalled as e:
        # a second SIGTERM / SIGHUP must not interrupt the teardown halfway
        _ignore_signals(previous)
        print(f"[launch] received signal {e.signum}; stopping the ranks", file=sys.stderr, flush=True)
        _terminate(procs, grace_s)
        rc = 128 + e.signum
    finally:
        for sig, h in previous.items():
            signal.signal(sig, h)
    return rc


def _ignore_signals(handlers: Dict):
    for sig in handlers:
        try:
            signal.signal(sig, signal.SIG_IGN)
        except (ValueError, OSError):
            pass


def _terminate(procs: Sequence[subprocess.Popen], grace_s: float):
    for p in procs:
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    deadline = time.time() + grace_s
    for p in procs:
        try:
            p.wait(timeout=max(0.1, deadline - time.time()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
