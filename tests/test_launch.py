"""CPU: bench.py's own rank launcher (mpcq/launch.py) -- `python bench.py --gpus N`
starts N rank processes with torch.distributed.run's environment, checks an
external launcher's WORLD_SIZE against --gpus, and fails loudly on a mismatch,
on too few GPUs under RCCL, and when a rank fails."""
import os
import subprocess
import sys
import textwrap

import pytest

from mpcq import launch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_child_envs():
    envs = launch.child_envs(3, {"FOO": "1", "HSA_ENABLE_IPC_MODE_LEGACY": "0"}, 29555)
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    for e in envs:
        assert e["WORLD_SIZE"] == "3" and e["LOCAL_WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
        assert e["FOO"] == "1" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    with pytest.raises(launch.LaunchError):
        launch.child_envs(0, {}, 1)


def test_resolve_world():
    assert launch.resolve_world(None, {}) == (1, False)
    assert launch.resolve_world(1, {}) == (1, False)
    assert launch.resolve_world(8, {}) == (8, True)
    assert launch.resolve_world(None, {"WORLD_SIZE": "4"}) == (4, False)
    assert launch.resolve_world(4, {"WORLD_SIZE": "4"}) == (4, False)
    with pytest.raises(launch.LaunchError, match="WORLD_SIZE"):
        launch.resolve_world(8, {"WORLD_SIZE": "2"})
    with pytest.raises(launch.LaunchError):
        launch.resolve_world(0, {})


def test_check_devices():
    launch.check_devices(8, "nccl", count=8, env={})
    launch.check_devices(8, "gloo", count=1, env={})      # rehearsal: ranks share the card
    with pytest.raises(launch.LaunchError, match="visible"):
        launch.check_devices(8, "nccl", count=1, env={})
    # an external multi-node launcher: WORLD_SIZE counts every node, LOCAL_WORLD_SIZE this one
    launch.check_devices(16, "nccl", count=8, env={"WORLD_SIZE": "16", "LOCAL_WORLD_SIZE": "8"})
    with pytest.raises(launch.LaunchError, match="visible"):
        launch.check_devices(16, "nccl", count=4, env={"WORLD_SIZE": "16", "LOCAL_WORLD_SIZE": "8"})


def fake_topology(root, gpus, cpus=1):
    """A /sys/class/kfd/kfd/topology/nodes look-alike: CPU nodes (simd_count 0) first."""
    for i in range(cpus + gpus):
        d = root / str(i)
        d.mkdir(parents=True)
        simd = 0 if i < cpus else 1024
        (d / "properties").write_text(f"cpu_cores_count {64 if i < cpus else 0}\nsimd_count {simd}\n"
                                      f"gfx_target_version {0 if i < cpus else 90500}\n")
    return str(root)


def test_count_gpus_from_sysfs(tmp_path):
    topo = fake_topology(tmp_path / "nodes", gpus=8, cpus=2)
    assert launch.count_gpus({}, topo) == 8
    assert launch.count_gpus({"HIP_VISIBLE_DEVICES": "0,1,2"}, topo) == 3
    assert launch.count_gpus({"ROCR_VISIBLE_DEVICES": "4,5", "HIP_VISIBLE_DEVICES": "0,1,2"}, topo) == 2
    assert launch.count_gpus({"HIP_VISIBLE_DEVICES": ""}, topo) == 8          # empty = unset, as HIP reads it
    assert launch.count_gpus({"HIP_VISIBLE_DEVICES": "0,-1,2"}, topo) == 1   # stops at the first invalid index
    assert launch.count_gpus({"ROCR_VISIBLE_DEVICES": "GPU-abc,GPU-def"}, topo) == 2
    assert launch.count_gpus({}, str(tmp_path / "absent")) == 0              # no amdgpu driver: no GPU
    assert launch.count_gpus({"MPCQ_KFD_TOPOLOGY": topo}) == 8


def _env(**kw):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(kw)
    return e


def test_bench_world_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "4"], env=_env(WORLD_SIZE="2"),
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r
    assert "WORLD_SIZE=2" in r.stderr and r.stdout == ""


def test_bench_too_many_gpus_exits_nonzero():
    # no GPU in this container: 2 ranks under RCCL cannot get a device each
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"],
                       env=_env(MPCQ_DIST_BACKEND="nccl"), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2, r
    assert "visible" in r.stderr and r.stdout == ""


RANK_SCRIPT = textwrap.dedent("""
    import os, sys, torch, torch.distributed as dist
    dist.init_process_group("gloo", init_method="env://")
    r, w = dist.get_rank(), dist.get_world_size()
    assert r == int(os.environ["RANK"]) == int(os.environ["LOCAL_RANK"]) and w == int(os.environ["WORLD_SIZE"])
    t = torch.tensor([float(r + 1)])
    dist.all_reduce(t)
    if r == 0:
        print("SUM", int(t.item()), "WORLD", w, flush=True)
    dist.destroy_process_group()
""")


def test_run_ranks_rendezvous(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    out = tmp_path / "out.txt"
    with open(out, "w") as f:
        # children inherit stdout: route it to the file through a wrapper process
        code = ("import sys; sys.path.insert(0, %r); from mpcq import launch; "
                "sys.exit(launch.run_ranks([sys.executable, %r], 3, timeout_s=120))"
                % (os.path.join(REPO, "mpc-tsid_amd"), str(script)))
        rc = subprocess.run([sys.executable, "-c", code], stdout=f, env=_env(), timeout=180).returncode
    assert rc == 0
    lines = [ln.split() for ln in out.read_text().splitlines() if ln.startswith("SUM")]
    assert lines == [["SUM", "6", "WORLD", "3"]]  # rank 0 alone prints


def test_run_ranks_failure_stops_the_others(tmp_path):
    script = tmp_path / "rank.py"
    script.write_text("import os, sys, time\n"
                      "if os.environ['RANK'] == '1':\n    sys.exit(3)\n"
                      "time.sleep(600)\n")
    import time
    t = time.monotonic()
    rc = launch.run_ranks([sys.executable, str(script)], 3, env=_env())
    assert rc == 3
    assert time.monotonic() - t < 60  # the sleeping ranks were stopped, not waited for


PARENT_PROBE = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, {repo!r})
    sys.argv = ["bench.py", "--gpus", "2"]
    import bench
    from mpcq import launch

    def probe(cmd, n, **kw):
        # what bench.py's parent has mapped at the moment it would start the ranks
        maps = open("/proc/self/maps").read()
        print("RANKS", n, "HIP_MAPPED", int("libamdhip64" in maps), "TORCH", int("torch" in sys.modules), flush=True)
        return 0

    launch.run_ranks = probe
    bench.launch_or_check(bench.parse())
""")


def test_bench_parent_never_loads_hip_under_nccl(tmp_path):
    """--gpus 2 under RCCL on a (faked) two-GPU node: the parent counts the GPUs from
    sysfs and reaches the rank spawn without the HIP runtime mapped or torch imported."""
    topo = fake_topology(tmp_path / "nodes", gpus=2)
    script = tmp_path / "probe.py"
    script.write_text(PARENT_PROBE.format(repo=REPO))
    r = subprocess.run([sys.executable, str(script)], env=_env(MPCQ_DIST_BACKEND="nccl", MPCQ_KFD_TOPOLOGY=topo),
                       capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode == 0, r
    assert "RANKS 2 HIP_MAPPED 0 TORCH 0" in r.stdout, r


def test_launcher_sigterm_stops_the_ranks(tmp_path):
    """SIGTERM to the launcher (from outside its process group) stops the sleeping ranks."""
    import signal
    import time
    pidfile = tmp_path / "pids"
    script = tmp_path / "rank.py"
    script.write_text("import os, time\n"
                      f"open({str(pidfile)!r}, 'a').write(str(os.getpid()) + '\\n')\n"
                      "time.sleep(600)\n")
    code = ("import sys; sys.path.insert(0, %r); from mpcq import launch; "
            "sys.exit(launch.run_ranks([sys.executable, %r], 3))" % (os.path.join(REPO, "mpc-tsid_amd"), str(script)))
    p = subprocess.Popen([sys.executable, "-c", code], env=_env(), start_new_session=True)
    t = time.monotonic()
    while time.monotonic() - t < 60:
        if pidfile.exists() and len(pidfile.read_text().split()) == 3:
            break
        time.sleep(0.1)
    pids = [int(x) for x in pidfile.read_text().split()]
    assert len(pids) == 3
    p.send_signal(signal.SIGTERM)
    assert p.wait(timeout=60) == 128 + signal.SIGTERM
    for pid in pids:
        gone = False
        for _ in range(100):
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                gone = True
                break
            time.sleep(0.1)
        assert gone, pid


def test_launcher_sigkill_takes_the_ranks_down(tmp_path):
    """A launcher killed outright (no handler runs): the ranks' parent-death signal stops them."""
    import signal
    import time
    pidfile = tmp_path / "pids"
    script = tmp_path / "rank.py"
    script.write_text("import os, time\n"
                      f"open({str(pidfile)!r}, 'a').write(str(os.getpid()) + '\\n')\n"
                      "time.sleep(600)\n")
    code = ("import sys; sys.path.insert(0, %r); from mpcq import launch; "
            "sys.exit(launch.run_ranks([sys.executable, %r], 2))" % (os.path.join(REPO, "mpc-tsid_amd"), str(script)))
    p = subprocess.Popen([sys.executable, "-c", code], env=_env(), start_new_session=True)
    t = time.monotonic()
    while time.monotonic() - t < 60:
        if pidfile.exists() and len(pidfile.read_text().split()) == 2:
            break
        time.sleep(0.1)
    pids = [int(x) for x in pidfile.read_text().split()]
    p.send_signal(signal.SIGKILL)
    p.wait(timeout=30)
    for pid in pids:
        gone = False
        for _ in range(100):
            try:
                os.kill(pid, 0)
            except ProcessLookupError:
                gone = True
                break
            time.sleep(0.1)
        assert gone, pid
