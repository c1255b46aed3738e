"""CPU: bench.py's stdout carries only its JSON line -- the process-group initialisation
(RCCL prints a banner on fd 1) runs with fd 1 pointed at stderr (bench.init_group_quiet).
A stand-in process group writes to fd 1 from C-level I/O (os.write) and Python's print,
as RCCL's banner would, in a child process whose stdout is captured."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys
sys.path.insert(0, %r)
import bench

class FakeDist:
    calls = []
    def init_process_group(self, backend, init_method=None, rank=0, world_size=1):
        os.write(1, b"RCCL version 2.99.0+hip banner on fd 1\n")
        print("a python print during init")
        self.calls.append(("init", backend, rank, world_size))
    def barrier(self):
        os.write(1, b"barrier noise on fd 1\n")
        self.calls.append(("barrier",))

d = FakeDist()
bench.init_group_quiet(d, sys.argv[1], 0, 1)
print(json.dumps({"metric": "m", "value": 1.0, "calls": d.calls}), flush=True)
"""


def run(backend):
    r = subprocess.run([sys.executable, "-c", CHILD % REPO, backend], capture_output=True, text=True,
                       timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr
    return r


def test_rccl_banner_stays_off_stdout():
    r = run("nccl")
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    rec = json.loads(lines[0])
    assert rec["calls"] == [["init", "nccl", 0, 1], ["barrier"]]  # the eager barrier ran under the redirect
    assert "RCCL version" in r.stderr and "barrier noise" in r.stderr and "python print" in r.stderr


def test_gloo_init_is_quiet_too_without_the_barrier():
    r = run("gloo")
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and json.loads(lines[0])["calls"] == [["init", "gloo", 0, 1]]
