"""One process per GPU: start the ranks of a job from a launcher process, or join them.

The reference starts its own DDP ranks with `mp.spawn(train, nprocs=world_size)`
(ddp.py:179-181).  Here a launcher process that has NOT touched the GPU starts N children
(fresh interpreters running the same command, never an exec of a GPU-initialised process)
with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set exactly as torchrun sets
them, so the rank code is identical under torchrun and under self-launch.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def under_launcher() -> bool:
    """True inside a rank (torchrun or launch_ranks set WORLD_SIZE)."""
    return "WORLD_SIZE" in os.environ


def launch_ranks(n: int, argv, tag: str = "self-spawn") -> int:
    """Run `python argv...` as n ranks and wait; returns 0 or the first non-zero exit code."""
    if n < 1:
        raise ValueError("need at least one rank")
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(n),
                    "LOCAL_WORLD_SIZE": str(n), "MASTER_ADDR": "127.0.0.1",
                    "MASTER_PORT": str(port), "DD_LAUNCHER": tag})
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this driver
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=env))
    rcs = [p.wait() for p in procs]
    bad = [rc for rc in rcs if rc != 0]
    return bad[0] if bad else 0


def rank_env():
    """(world, rank, local_rank) from the environment (1, 0, 0 outside a launcher)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def launcher_name(world: int) -> str:
    if "DD_LAUNCHER" in os.environ:
        return os.environ["DD_LAUNCHER"]
    if "TORCHELASTIC_RUN_ID" in os.environ:
        return "torchrun"
    return "single process" if world == 1 else "external"
