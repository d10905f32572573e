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
import time


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def under_launcher() -> bool:
    """True inside a rank (torchrun or launch_ranks set WORLD_SIZE)."""
    return "WORLD_SIZE" in os.environ


def launch_ranks(n: int, argv, tag: str = "self-spawn", poll_s: float = 0.2,
                 grace_s: float = 10.0) -> int:
    """Run `python argv...` as n ranks and wait; returns 0 or the first non-zero exit code.

    Fail-fast like torchrun: the children are polled, and the first one to exit non-zero
    gets its siblings terminated (SIGTERM, then SIGKILL after `grace_s`), so a rank that dies
    before or inside a collective does not leave the others blocked until the process-group
    timeout."""
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
    first_bad = 0
    try:
        while True:
            live = [p for p in procs if p.poll() is None]
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                first_bad = bad[0]
                break
            if not live:
                return 0
            time.sleep(poll_s)
    except BaseException:  # KeyboardInterrupt: take the ranks down with the launcher
        first_bad = first_bad or 1
        _stop(procs, grace_s)
        raise
    _stop(procs, grace_s)
    return first_bad


def _stop(procs, grace_s: float):
    for p in procs:
        if p.poll() is None:
            p.terminate()
    deadline = time.monotonic() + grace_s
    for p in procs:
        try:
            p.wait(timeout=max(0.0, deadline - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def init_process_group(backend: str, rank: int, world: int, device=None,
                       timeout_s: float = None):
    """torch.distributed.init_process_group with a bounded timeout (default
    $DD_PG_TIMEOUT_S or 300 s, instead of torch's 10 min for RCCL), so a lost peer ends the
    job instead of stalling it.  `device` binds the RCCL communicator to this rank's GPU."""
    import datetime

    import torch.distributed as dist
    if timeout_s is None:
        timeout_s = float(os.environ.get("DD_PG_TIMEOUT_S", "300"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    kw = {"device_id": device} if device is not None and backend == "nccl" else {}
    dist.init_process_group(backend, rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=timeout_s), **kw)


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
