"""One process per GPU: start N ranks of a script from a parent that never touches the GPU.

`python bench.py --gpus N` (no torch.distributed.run around it) comes here: the parent
starts N children of the same script with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR /
MASTER_PORT set (the torch.distributed.run environment), waits for them, and exits with the
worst exit code.  Children are started as new processes (never by exec from a process that
initialised the GPU), and if one rank fails the others are stopped so no rank hangs in a
collective.  This module imports neither torch nor HIP.
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time


def rank_env():
    """(world, rank, local_rank) of this process (1, 0, 0 outside a launcher)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return world, rank, local


def dist_backend() -> str:
    """The process group's backend: RCCL ("nccl") between GPUs.  BITAR_DIST_BACKEND=gloo is
    the one-GPU rehearsal of the N-rank path: the collectives run over gloo on host copies
    and the ranks share the visible GPUs (rank_device)."""
    return os.environ.get("BITAR_DIST_BACKEND", "nccl")


def rank_device(local: int, ndev: int) -> int:
    """The GPU of local rank `local`: one GPU per rank (RCCL refuses two ranks on one
    device); under the gloo rehearsal, ranks beyond the visible GPUs share them."""
    if dist_backend() == "gloo" and ndev > 0:
        return local % ndev
    return local


def is_rank_process() -> bool:
    return "WORLD_SIZE" in os.environ and "RANK" in os.environ


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn(nprocs: int, script: str, argv, extra_env=None, timeout=None) -> int:
    """Run `python script *argv` as ranks 0..nprocs-1 on 127.0.0.1; returns the worst exit
    code (0 if every rank succeeded).  stdout / stderr are inherited."""
    if nprocs < 1:
        raise ValueError("nprocs must be >= 1")
    port = free_port()
    procs = []
    for r in range(nprocs):
        env = dict(os.environ)
        env.update(extra_env or {})
        env.update({"WORLD_SIZE": str(nprocs), "RANK": str(r), "LOCAL_RANK": str(r),
                    "LOCAL_WORLD_SIZE": str(nprocs), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port)})
        procs.append(subprocess.Popen([sys.executable, script, *argv], env=env))
    deadline = None if timeout is None else time.monotonic() + timeout
    worst = 0
    live = set(range(nprocs))
    while live:
        for r in sorted(live):
            rc = procs[r].poll()
            if rc is None:
                continue
            live.discard(r)
            if rc != 0:
                worst = rc if worst == 0 else worst
                _stop(procs, live)
        if deadline is not None and time.monotonic() > deadline and live:
            _stop(procs, live)
            worst = worst or 124
        time.sleep(0.05)
    return worst


def _stop(procs, live):
    for r in list(live):
        p = procs[r]
        if p.poll() is None:
            p.send_signal(signal.SIGTERM)
    t0 = time.monotonic()
    for r in list(live):
        p = procs[r]
        try:
            p.wait(timeout=max(0.1, 20 - (time.monotonic() - t0)))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
