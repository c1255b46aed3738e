"""One process per GPU, started by bench.py itself.

``python bench.py --gpus N`` without a launcher around it: the parent process
starts N fresh children, one per GPU, each with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT set as ``torch.distributed.run`` would set them, waits
for all of them and exits non-zero if any fails (the others are then stopped).
The parent never touches the GPU: it only counts devices (which initialises no
HIP context on this image) before any child starts.  Under an external launcher
(WORLD_SIZE already set) nothing is spawned and WORLD_SIZE must equal --gpus.
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
import time

MASTER_ADDR = "127.0.0.1"


class LaunchError(RuntimeError):
    pass


def free_port(addr: str = MASTER_ADDR) -> int:
    s = socket.socket()
    try:
        s.bind((addr, 0))
        return int(s.getsockname()[1])
    finally:
        s.close()


def child_envs(n: int, base: dict, port: int, addr: str = MASTER_ADDR):
    """The environments of the N rank processes (torch.distributed.run's variables)."""
    if n < 1:
        raise LaunchError(f"--gpus {n}: need at least one rank")
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR=addr, MASTER_PORT=str(port))
        # dmabuf IPC is the only one the host driver supports (RCCL between processes)
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        envs.append(e)
    return envs


def resolve_world(gpus, env=None):
    """(world size, spawn?) for ``--gpus`` (None = not given) under ``env``.

    WORLD_SIZE set: an external launcher started this rank; --gpus, if given, must
    match.  WORLD_SIZE unset: spawn when --gpus > 1."""
    env = os.environ if env is None else env
    ws = env.get("WORLD_SIZE")
    if ws is not None:
        w = int(ws)
        if gpus is not None and gpus != w:
            raise LaunchError(f"--gpus {gpus} but WORLD_SIZE={w} (the launcher started {w} ranks)")
        return w, False
    n = 1 if gpus is None else int(gpus)
    if n < 1:
        raise LaunchError(f"--gpus {n}: need at least one rank")
    return n, n > 1


def check_devices(n: int, backend: str, count=None):
    """Under RCCL every rank needs a GPU of its own; gloo rehearsals may share."""
    if backend != "nccl":
        return
    if count is None:
        import torch
        count = torch.cuda.device_count()
    if n > count:
        raise LaunchError(f"--gpus {n} but {count} GPU(s) visible (backend nccl needs one per rank; "
                          "MPCQ_DIST_BACKEND=gloo rehearses more ranks than GPUs)")


def run_ranks(cmd, n: int, env=None, poll_s: float = 0.2, timeout_s: float | None = None) -> int:
    """Start ``cmd`` once per rank and wait.  Returns 0 when every rank exits 0;
    otherwise stops the ranks still running and returns the first failure's code
    (or 1 for a rank killed by a signal / the timeout)."""
    base = dict(os.environ if env is None else env)
    port = free_port()
    procs = [subprocess.Popen(cmd, env=e) for e in child_envs(n, base, port)]
    t0 = time.monotonic()
    rc = 0
    try:
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c not in (None, 0)]
            if bad:
                rc = bad[0] if bad[0] > 0 else 1
                print(f"[launch] a rank exited with {bad[0]}; stopping the others", file=sys.stderr, flush=True)
                break
            if all(c == 0 for c in codes):
                return 0
            if timeout_s is not None and time.monotonic() - t0 > timeout_s:
                rc = 1
                print(f"[launch] ranks still running after {timeout_s} s; stopping them", file=sys.stderr,
                      flush=True)
                break
            time.sleep(poll_s)
    except KeyboardInterrupt:
        rc = 130
    for p in procs:
        if p.poll() is None:
            p.terminate()
    for p in procs:
        try:
            p.wait(timeout=20)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
    return rc
