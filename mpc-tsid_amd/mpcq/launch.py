"""One process per GPU, started by bench.py itself.

``python bench.py --gpus N`` without a launcher around it: the parent process
starts N fresh children, one per GPU, each with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR / MASTER_PORT set as ``torch.distributed.run`` would set them, waits
for all of them and exits non-zero if any fails (the others are then stopped, and
so are they when the parent is signalled or dies).  Under an external launcher
(WORLD_SIZE already set) nothing is spawned and WORLD_SIZE must equal --gpus.

The parent never touches the GPU, not even to count devices: ``count_gpus`` reads
the KFD topology in sysfs (a GPU node has ``simd_count > 0``) and applies the
visible-devices variables, so no HIP runtime is loaded or initialised before the
children start (torch's ``device_count`` may fall back to ``hipGetDeviceCount``,
and a process that has initialised HIP must not fork-and-exec ranks).
"""
from __future__ import annotations

import os
import signal
import socket
import subprocess
import sys
import time

MASTER_ADDR = "127.0.0.1"
KFD_TOPOLOGY = "/sys/class/kfd/kfd/topology/nodes"


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


def _visible_list(v: str):
    """Entries of a *_VISIBLE_DEVICES value (ROCm stops at the first invalid index)."""
    out = []
    for tok in v.split(","):
        tok = tok.strip()
        if not tok:
            break
        if tok.startswith("GPU-"):  # ROCR_VISIBLE_DEVICES accepts UUIDs
            out.append(tok)
            continue
        try:
            if int(tok) < 0:
                break
        except ValueError:
            break
        out.append(tok)
    return out


def count_gpus(env=None, topology: str | None = None) -> int:
    """GPUs this process would see, without loading the HIP runtime: the KFD topology's
    GPU nodes (simd_count > 0; CPU nodes have none), narrowed by ROCR_VISIBLE_DEVICES
    and then HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (empty = unset, as HIP reads
    them).  No topology (no amdgpu
    driver) counts 0.  ``topology`` (or MPCQ_KFD_TOPOLOGY) points elsewhere: tests."""
    env = os.environ if env is None else env
    root = topology or env.get("MPCQ_KFD_TOPOLOGY") or KFD_TOPOLOGY
    n = 0
    try:
        nodes = sorted(os.listdir(root))
    except OSError:
        nodes = []
    for node in nodes:
        try:
            with open(os.path.join(root, node, "properties")) as f:
                props = dict(ln.split(None, 1) for ln in f.read().splitlines() if len(ln.split(None, 1)) == 2)
        except OSError:
            continue
        try:
            if int(props.get("simd_count", "0")) > 0:
                n += 1
        except ValueError:
            continue
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        if env.get(var, "").strip():  # HIP reads an empty value as unset (every device visible)
            n = min(n, len(_visible_list(env[var])))
    return n


def local_world(world: int, env=None) -> int:
    """Ranks on this node: LOCAL_WORLD_SIZE under a launcher (a multi-node job's
    WORLD_SIZE counts every node's ranks), else the world."""
    env = os.environ if env is None else env
    lw = env.get("LOCAL_WORLD_SIZE")
    return int(lw) if lw else world


def check_devices(n: int, backend: str, count=None, env=None):
    """Under RCCL every rank on this node needs a GPU of its own; gloo rehearsals may
    share.  ``n`` = the world size; the node's share is local_world(n)."""
    if backend != "nccl":
        return
    local = local_world(n, env)
    if count is None:
        count = count_gpus(env)
    if local > count:
        raise LaunchError(f"--gpus {n}: {local} rank(s) on this node but {count} GPU(s) visible (backend nccl needs "
                          "one per rank; MPCQ_DIST_BACKEND=gloo rehearses more ranks than GPUs)")


def _child_preexec():
    """In each rank, before exec: die with the launcher (PR_SET_PDEATHSIG = SIGTERM), so a
    launcher killed by SIGKILL leaves no rank holding a GPU or the rendezvous port."""
    try:
        import ctypes
        libc = ctypes.CDLL(None, use_errno=True)
        libc.prctl(1, int(signal.SIGTERM), 0, 0, 0)  # PR_SET_PDEATHSIG
    except Exception:  # noqa: BLE001 -- best effort; the signal handlers below still stop the ranks
        pass


class _Stop(Exception):
    def __init__(self, signum):
        super().__init__(signum)
        self.signum = signum


def run_ranks(cmd, n: int, env=None, poll_s: float = 0.2, timeout_s: float | None = None) -> int:
    """Start ``cmd`` once per rank and wait.  Returns 0 when every rank exits 0;
    otherwise stops the ranks still running and returns the first failure's code
    (or 1 for a rank killed by a signal / the timeout, 128 + s when the launcher
    itself gets SIGTERM / SIGHUP / SIGINT)."""
    base = dict(os.environ if env is None else env)
    port = free_port()

    def on_signal(signum, _frame):
        raise _Stop(signum)

    old = {}
    for s in (signal.SIGTERM, signal.SIGHUP):
        try:
            old[s] = signal.signal(s, on_signal)
        except ValueError:  # not the main thread: the pdeath signal still covers the ranks
            pass
    procs = []
    rc = 0
    try:
        for e in child_envs(n, base, port):
            procs.append(subprocess.Popen(cmd, env=e, preexec_fn=_child_preexec))
        t0 = time.monotonic()
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
    except _Stop as e:
        rc = 128 + int(e.signum)
        print(f"[launch] got signal {int(e.signum)}; stopping the ranks", file=sys.stderr, flush=True)
    finally:
        for s, h in old.items():
            signal.signal(s, h)
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
