#!/usr/bin/env python3
"""Benchmark of the MI355X batched MPC-QP hot path (MPC.py formulation + OSQP solve).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
           --master-port P bench.py --gpus N --steps K --warmup W

Without an external launcher, --gpus N > 1 starts the N rank processes itself
(mpcq/launch.py: fresh interpreters with RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / MASTER_PORT set, before this process touches the GPU; a
failing rank stops the others and the exit status is non-zero).  Under a launcher
WORLD_SIZE must equal --gpus.  RCCL ("nccl") needs a GPU per rank;
MPCQ_DIST_BACKEND=gloo rehearses more ranks than GPUs.

One step = one launch of the fused engine kernel (formulation + Ruiz scaling +
KKT factorisation + OSQP ADMM to eps 1e-7) over this rank's batch of
synthetic (xref, fsteps) instances, inputs resident in HBM.  Ranks shard the
instances (no data-path collective): value = instances solved by all ranks /
max-over-ranks wall time of the K timed steps.

The headline runs OSQP as MPC.py configures it (--headline reference, the
default: polish off, MPC.py:414-416), so "f_osqp" of the metric is that
solver's output; on one GPU the line also carries a "companion" object with
the engine's accuracy extension (polish=2: forces on the certified optimum x*)
timed the same way, and "parity" reports each mode against both readings of
f_osqp (the restated OSQP with MPC.py's settings, and x*) with which of them
meets 1e-4.

Workloads (BASELINE.json configs):
  c1            1 instance per GPU, N=16, static trot    -> latency of one tick
  c2 (default)  1024 instances per GPU, N=16, trot      -> weak scaling
  c3            1024 instances per GPU, N=32, trot      -> weak scaling
  c4            65536 instances in total, N=16, trot    -> strong scaling
  c5            32768 instances in total, N=16, trot/bound/pace interleaved -> strong scaling
Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))
sys.path.insert(0, REPO)

METRIC = "QP instances/s (12-state, N=16) at 1/2/4/8 MI355X; max |f - f_osqp|"
PEAK_HBM_GBS = 8000.0     # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
PEAK_FP64_TFLOPS = 78.6   # MI355X FP64 (vector and matrix peaks coincide on gfx950)

CONFIGS = {
    "c1": dict(total=None, per_gpu=1, N=16, gaits=("trot",), static=True,
               desc="C1: a single QP, N=16, trot, static xref (latency of one tick)"),
    "c2": dict(total=None, per_gpu=1024, N=16, gaits=("trot",), desc="C2: batch 1024 synthetic instances per GPU, N=16, trot"),
    "c3": dict(total=None, per_gpu=1024, N=32, gaits=("trot",), desc="C3: batch 1024 synthetic instances per GPU, N=32, trot"),
    "c4": dict(total=65536, per_gpu=None, N=16, gaits=("trot",), desc="C4: 65536 synthetic instances sharded over the GPUs, N=16, trot"),
    "c5": dict(total=32768, per_gpu=None, N=16, gaits=("trot", "bound", "pace"),
               desc="C5: 32768 mixed-gait instances (trot/bound/pace interleaved) sharded over the GPUs, N=16"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE, else 1); without an external launcher "
                         "bench.py starts the N rank processes itself (mpcq/launch.py)")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="override instances per GPU")
    ap.add_argument("--headline", default="reference", choices=("reference", "accuracy"),
                    help="reference (default): OSQP as MPC.py configures it (eps 1e-7, every other setting at "
                         "the OSQP 0.6 default, polish off: MPC.py:414-416); accuracy: the engine extension "
                         "polish=2 (OSQP's polish after the ADMM, also after MAX_ITER / SOLVED_INACCURATE exits, "
                         "up to 8 active-set rounds, 10 refinements): forces on the QP's certified optimum")
    ap.add_argument("--polish", dest="headline", action="store_const", const="accuracy",
                    help="= --headline accuracy")
    ap.add_argument("--no-polish", dest="headline", action="store_const", const="reference",
                    help="= --headline reference")
    ap.add_argument("--companion", type=int, default=1,
                    help="1 (default, one GPU): after the headline, time the other mode on the same batch and "
                         "report it in the line's 'companion' object; 0 = skip")
    ap.add_argument("--reference25", type=int, default=1,
                    help="1 (default, one GPU, reference headline): also time OSQP at MPC.py's settings with "
                         "adaptive_rho_interval 25 (the timing-derived interval of a PROFILING osqp build on a fast "
                         "host) on the same batch, with its own parity against the restatement at 25; 0 = skip")
    ap.add_argument("--order-by-class", type=int, default=1,
                    help="1 (default): MPCQ_FLAG_ORDER_BY_CLASS -- each launch dispatches the instances by the "
                         "mean iteration count their gait class showed in the engine's earlier launches (the "
                         "warm-up ones first), the most expensive first; a one-gait batch keeps index order. "
                         "Scheduling only (results bit-identical); 0 = index order")
    ap.add_argument("--slice", type=int, default=-1,
                    help="> 0: sliced solves (mpcq_set_slice, beyond 16 stages): each step's first launch "
                         "suspends the instances still iterating after SLICE ADMM iterations, a second launch "
                         "resumes them, the farthest from convergence first, to their end (results bit-identical; "
                         "the step's time spans both launches); 0 = one launch; "
                         f"-1 (default) = {AUTO_SLICE} beyond 16 stages (C3's best measured, "
                         "profiles/r06*_bench_c3_*s*.json), 0 up to 16")
    ap.add_argument("--rho-interval", type=int, default=0,
                    help="override adaptive_rho_interval (0 = the library default)")
    ap.add_argument("--cpu-sample", type=float, default=1.5,
                    help="seconds of CPU work per CPU-baseline run (3 warm-up + 10 timed runs, each over "
                         "instances cycling through the rank-0 batch; 0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every CPU this process may use")
    ap.add_argument("--certify", type=int, default=1024,
                    help="instances (the first ones of rank 0) whose forces are checked against the "
                         "KKT-certified optimum (-1 = all, 0 = skip)")
    ap.add_argument("--restatement", type=int, default=1024,
                    help="instances (the first ones of rank 0) solved again by the oracle's restatement of "
                         "each mode, and at adaptive_rho_interval 25 and 100 for the OSQP band (0 = skip)")
    ap.add_argument("--gather", action="store_true", help="include an RCCL all-gather of f0 in the timed region")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--mode", default="qp", choices=("qp", "plan", "tick"),
                    help="qp: the headline (fused formulation + OSQP per instance); plan: the batched "
                         "FootstepPlanner kernel alone; tick: closed-loop sessions (planner + warm-started "
                         "solve + retrieve per robot and tick, virtual robot)")
    return ap.parse_args()


AUTO_SLICE = 1000  # bench.py --slice -1 beyond 16 stages (C3: r06y / r06z)


def load_pmc(tag: str, src_sha: str | None = None, path: str | None = None) -> dict:
    """Per-launch PMC figures (HBM bytes, issued FP64 flops, that run's kernel ms) from the
    committed rocprofv3 summary profiles/pmc_traffic.json, if any -- only when the entry
    was profiled on the build that is running: its "engine_src_sha" (the stamp of the
    profiled libmpcq.so, tools/prof_summary.py) must equal ``src_sha`` (the running
    library's mpcq_build_info).  Otherwise {"stale": reason} and no figures."""
    path = path or os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}
    e = dict(d.get(tag) or {})
    if not e:
        return {}
    have = e.get("engine_src_sha")
    if src_sha is None or have != src_sha:
        return {"stale": f"profiles/pmc_traffic.json[{tag!r}] (tag {e.get('tag')}) was profiled on build "
                         f"{have or 'unstamped'}, this library is {src_sha or 'unknown'}: figures dropped"}
    return e


def lib_sha():
    """The running libmpcq.so's source stamp (mpcq_build_info), or None."""
    try:
        import mpcq
        return mpcq.build_info().get("src_sha256")
    except Exception:  # noqa: BLE001 -- no library: no stamp, so no PMC figure is trusted
        return None


def load_traffic(tag: str, src_sha: str | None = None):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any (same build only)."""
    v = load_pmc(tag, src_sha).get("bytes_per_launch")
    return float(v) if v is not None else None


def dist_fields(world: int, backend: str, distributed: bool, torch) -> dict:
    """How the ranks were spread: the backend, the distinct devices they used (gloo
    rehearsals share one card round-robin) and whether the line is a rehearsal (ranks
    sharing devices: not an N-GPU measurement)."""
    ndev = torch.cuda.device_count()
    distinct = min(world, ndev) if backend == "gloo" else world
    return {"backend": backend if distributed else None, "distinct_devices": distinct,
            "rehearsal": bool(distinct < world)}


def workload_label(name, cfg, batch, world):
    """config.workload: the BASELINE config's description, or -- when --batch overrides the
    instances per GPU of a fixed-total config (C4 / C5) -- what the line really measures: one
    rank's shard of that total (e.g. C4 at 8 GPUs: 8192 of 65536 per GPU)."""
    if batch > 0 and cfg.get("total"):
        split = cfg["total"] // batch if batch and cfg["total"] % batch == 0 else None
        return (f"{name.upper()} rank shard: {batch} of {cfg['total']} instances per GPU"
                + (f" (the per-GPU share at {split} GPUs)" if split else "")
                + f", {world} GPU(s) here, N={cfg['N']}, gaits {'/'.join(cfg['gaits'])}")
    if batch > 0:
        return f"{cfg['desc']} -- batch overridden: {batch} instances per GPU"
    return cfg["desc"]


def init_group_quiet(dist, backend, rank, world):
    """init_process_group (+ the first barrier under RCCL, which creates the communicator
    lazily) with file descriptor 1 pointed at stderr: RCCL prints its version banner on
    stdout at initialisation, and stdout carries only the one JSON line
    (tests/test_bench_stdout.py runs this with a stand-in that writes to fd 1)."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        dist.init_process_group(backend, init_method="env://", rank=rank, world_size=world)
        if backend == "nccl":  # the communicator is created lazily: make it now, under the redirect
            dist.barrier()
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)


def _dist_setup():
    """One process per GPU (RANK / LOCAL_RANK / WORLD_SIZE from torch.distributed.run),
    RCCL ("nccl") between them.  MPCQ_DIST_BACKEND=gloo is the rehearsal mode of the
    N > 1 path on a box with fewer GPUs than ranks: ranks share devices round-robin
    and the collectives (barriers, max-over-ranks, stats) run over gloo on the host.
    MPCQ_FORCE_DIST=1 initialises the process group (and so runs every collective of
    the N > 1 path) at world size 1 too: on a one-GPU box it exercises RCCL itself."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("MPCQ_DIST_BACKEND", "nccl")
    if backend not in ("nccl", "gloo"):
        raise ValueError(f"MPCQ_DIST_BACKEND={backend!r}: 'nccl' (RCCL) or 'gloo'")
    if backend == "gloo":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1 or os.environ.get("MPCQ_FORCE_DIST") == "1":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            from mpcq import launch
            os.environ["MASTER_PORT"] = str(launch.free_port())
        torch.cuda.set_device(local)
        init_group_quiet(dist, backend, rank, world)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    coll = dev if backend == "nccl" else torch.device("cpu")  # where collective tensors live
    return torch, dist, world, rank, local, dev, coll


def _distributed(dist) -> bool:
    return dist.is_available() and dist.is_initialized()


def _timed(torch, dist, dev, coll, world, stream, step, steps, warmup):
    """W untimed steps, then K steps between barriers + synchronisations; returns
    (max-over-ranks wall seconds, HIP-event ms per step on the launch stream)."""
    from mpcq import shard
    torch.cuda.set_stream(stream)
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize(dev)
    if _distributed(dist):
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(steps):
        step(warmup + i)
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if _distributed(dist):
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    return shard.max_over_ranks(dist, wall, coll, world), ev0.elapsed_time(ev1) / max(steps, 1)


def main_plan(args):
    """Batched FootstepPlanner (mpcq_plan_batch, MPCQ_PLAN_TICK) on device-resident
    robots: one step = one planner launch over this rank's robots."""
    torch, dist, world, rank, local, dev, coll = _dist_setup()
    import mpcq
    from mpcq import model, synth
    N = CONFIGS[args.config]["N"]
    per = args.batch or 65536
    rng = np.random.default_rng(args.seed + rank)
    gaits = np.stack([synth.gait_table(("trot", "bound", "pace")[b % 3], N) for b in range(per)])
    state = np.concatenate([np.zeros((per, 2)), 0.2 + rng.uniform(-.01, .01, (per, 1)), rng.normal(0, .02, (per, 2)),
                            np.zeros((per, 1)), rng.normal(0, .2, (per, 6))], axis=1)
    sh = np.array([[0.19, 0.19, -0.19, -0.19], [0.15005, -0.15005, 0.15005, -0.15005]])
    l_feet = np.concatenate([sh + rng.uniform(-.03, .03, (per, 2, 4)), np.zeros((per, 1, 4))], axis=1)
    v_ref = np.stack([rng.uniform(-.5, 1, per), rng.uniform(-.3, .3, per), np.zeros(per), rng.normal(0, .1, per),
                      rng.normal(0, .1, per), rng.uniform(-.5, .5, per)], axis=1)
    T = lambda a, dt=torch.float64: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    d = dict(state=T(state), l_feet=T(l_feet), v_ref=T(v_ref), gait=T(gaits), xref=T(np.zeros((per, 12, N + 1))),
             fsteps=T(np.zeros((per, 20, 13))), rot=T(np.zeros(per), torch.int32), h_rot=T(np.full(per, 0.2)),
             status=T(np.zeros(per), torch.int32), red=T(np.zeros(per), torch.int32))
    eng = mpcq.Engine(N, device=local)
    stream = torch.cuda.Stream(dev)
    eng.set_stream(stream.cuda_stream)

    def step(i):
        eng.plan_device(per, mpcq.PLAN_TICK, i, d["state"].data_ptr(), d["l_feet"].data_ptr(), d["v_ref"].data_ptr(),
                        d["gait"].data_ptr(), d["rot"].data_ptr(), d["h_rot"].data_ptr(), d["xref"].data_ptr(),
                        d["fsteps"].data_ptr(), status_ptr=d["status"].data_ptr(), reduced_ptr=d["red"].data_ptr(),
                        asynchronous=True)

    wall, ms = _timed(torch, dist, dev, coll, world, stream, step, args.steps, args.warmup)
    ok = int((d["status"] == 0).sum().item())
    if rank == 0:
        by = model.planner_bytes_per_instance(N) * per
        ach = by / (ms * 1e-3) / 1e9
        out = {"metric": "FootstepPlanner instances/s (update_fsteps + getRefStates per robot)", "value":
               per * world * args.steps / wall, "unit": "planner instances/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic robots (trot/bound/pace)",
               "config": {"workload": f"planner tick, {per} robots per GPU, N={N}", "horizon": N,
                          "parallelism": f"shard{world}"},
               "roofline": {"bound": "hbm", "achieved": ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": ach / PEAK_HBM_GBS, "traffic": load_traffic(f"plan_N{N}_B{per}", lib_sha()),
                            "note": f"algorithmic {model.planner_bytes_per_instance(N)} B/robot x {per} robots "
                                    "per launch / HIP-event launch time"},
               "kernel_ms_per_launch": ms, "ok_fraction": ok / per,
               "dist": dist_fields(world, os.environ.get("MPCQ_DIST_BACKEND", "nccl"), _distributed(dist), torch)}
        if world == 1 and args.cpu_sample > 0:
            from oracle import oracle as O
            O.build()
            ns = min(4096, per)
            pls = [O.Planner(N, gaits[b]) for b in range(ns)]
            t = time.perf_counter()
            reps = 0
            while time.perf_counter() - t < 10.0:
                for b in range(ns):
                    pls[b].plan(O.PLAN_TICK, reps + 1, state[b], l_feet[b], v_ref[b])
                reps += 1
            tc = time.perf_counter() - t
            out["cpu_baseline"] = {"value": ns * reps / tc, "unit": "planner instances/s", "cores": 1, "kind": "port",
                                   "sample": f"{ns} robots x {reps} ticks, oracle/planner_oracle.c through ctypes, "
                                             f"1 thread, {tc:.1f} s"}
        print(json.dumps(out), flush=True)
    eng.close()
    if _distributed(dist):
        dist.destroy_process_group()


def main_tick(args):
    """Closed-loop sessions: one step = one tick of every robot on this rank
    (planner + warm-started fused solve + retrieve), virtual robot."""
    torch, dist, world, rank, local, dev, coll = _dist_setup()
    import mpcq
    from mpcq import model, synth
    cfg = CONFIGS[args.config]
    N = cfg["N"]
    per = args.batch or (cfg["per_gpu"] or -(-cfg["total"] // world))
    rng = np.random.default_rng(args.seed + rank)
    gaits = np.stack([synth.gait_table(cfg["gaits"][b % len(cfg["gaits"])], N) for b in range(per)])
    v_ref = np.stack([rng.uniform(-.5, 1, per), rng.uniform(-.3, .3, per), np.zeros(per), np.zeros(per),
                      np.zeros(per), rng.uniform(-.5, .5, per)], axis=1)
    vr = torch.from_numpy(v_ref).to(dev)
    eng = mpcq.Engine(N, device=local)
    stream = torch.cuda.Stream(dev)
    eng.set_stream(stream.cuda_stream)
    sess = mpcq.Session(eng, per, gait0=gaits)
    warm = max(args.warmup, 1)  # tick 0 (setup, cold) is always a warm-up tick

    def step(i):
        sess.tick_device(vr.data_ptr(), k=i, asynchronous=True)

    wall, ms = _timed(torch, dist, dev, coll, world, stream, step, args.steps, warm)
    plan_ms, solve_ms = eng.last_kernel_ms()
    st = sess.read(mpcq.SV_STATUS)
    it = sess.read(mpcq.SV_ITERS)
    if rank == 0:
        fl = model.flops(N, it, np.zeros_like(it)).sum()
        ach = fl / (solve_ms * 1e-3) / 1e12
        out = {"metric": "closed-loop robot ticks/s (planner + warm-started OSQP solve + retrieve per robot)",
               "value": per * world * args.steps / wall, "unit": "robot ticks/s", "n_gpus": world,
               "steps": args.steps, "warmup": warm, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
               "scaling": "weak", "vs_baseline": None, "dtype": "f64",
               "data": "synthetic robots, virtual robot closed loop (state from the previous prediction)",
               "config": {"workload": f"session tick, {per} robots per GPU, N={N}, gaits {list(cfg['gaits'])}",
                          "horizon": N, "parallelism": f"shard{world}"},
               "roofline": {"bound": "valu_fp64", "achieved": ach, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                            "frac": ach / PEAK_FP64_TFLOPS, "traffic": None,
                            "note": "engine kernel of the last tick: model.flops(measured iterations, rho updates "
                                    "taken as 0 -- a lower bound) / its HIP-event time"},
               "kernel_ms": {"step": ms, "planner_last_tick": plan_ms, "solve_last_tick": solve_ms},
               "solved_fraction": float(np.isin(st, (1, 2)).mean()),
               "dist": dist_fields(world, os.environ.get("MPCQ_DIST_BACKEND", "nccl"), _distributed(dist), torch),
               "iters_warm": {"median": float(np.median(it)), "p90": float(np.percentile(it, 90)),
                              "max": int(it.max())}}
        if world == 1 and args.cpu_sample > 0:
            from oracle import oracle as O
            O.build()
            ns = min(16, per)
            ors = [O.Session(N, gaits[b]) for b in range(ns)]
            t = time.perf_counter()
            ticks = 0
            while time.perf_counter() - t < 10.0 and ticks < 200:
                for b in range(ns):
                    ors[b].tick(ticks, v_ref[b])
                ticks += 1
            tc = time.perf_counter() - t
            out["cpu_baseline"] = {"value": ns * ticks / tc, "unit": "robot ticks/s", "cores": 1, "kind": "port",
                                   "sample": f"{ns} robots x {ticks} ticks of oracle.Session (C restatements via "
                                             f"ctypes), 1 thread, {tc:.1f} s"}
        print(json.dumps(out), flush=True)
    sess.close()
    eng.close()
    if _distributed(dist):
        dist.destroy_process_group()


def host_cpus():
    """CPUs this process may use on this host: affinity mask, capped by a cgroup CPU quota."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    return dict(nproc=os.cpu_count(), affinity=aff, cgroup_quota=quota, usable=usable, model=model)


def cpu_baseline(O, syn, per, params, threads, seconds):
    """The oracle's native build (-O3 -march=native, OpenMP over `threads`) on
    instances cycling through this rank's batch: 3 warm-up runs, then the median
    of 10 timed runs, each sized to about `seconds` of work."""
    def run(ns):
        sel = np.arange(ns) % per
        xr, fs = syn["xref"][sel], syn["fsteps"][sel]
        t = time.perf_counter()
        O.solve_batch(xr, fs, 0, params=params, nthreads=threads, native=True)
        return time.perf_counter() - t

    O.native_lib()
    ns = 2 * threads
    t = run(ns)                                  # warm-up 1 (also sizes the runs)
    ns = max(threads, int(ns * seconds / max(t, 1e-3)))
    run(ns)                                      # warm-ups 2 and 3
    run(ns)
    times = [run(ns) for _ in range(10)]
    med = float(np.median(times))
    return ns / med, ns, times


MODES = {
    # OSQP as MPC.py configures it: eps_abs = eps_rel = 1e-7, everything else at the OSQP 0.6
    # default (polish off, MPC.py:414-416)
    "reference": {},
    # the engine extension: polish after the ADMM, also after a MAX_ITER / SOLVED_INACCURATE exit
    # (status upgraded to SOLVED when the polished point meets eps), up to 8 active-set rounds
    "accuracy": dict(polish=2, polish_rounds=8, polish_refine_iter=10),
    # the second reading of f_osqp: OSQP at MPC.py's settings with the adaptive-rho interval that
    # osqp 0.6 built with PROFILING derives from its own timing on a fast host (25)
    "reference25": dict(adaptive_rho_interval=25),
}
MODE_DESC = {
    "reference": "OSQP-0.6 ADMM restated with MPC.py's settings (eps 1e-7; rho 0.1, sigma 1e-6, alpha 1.6, "
                 "Ruiz 10, adaptive rho every {ival}, polish off: MPC.py:414-416)",
    "reference25": "OSQP-0.6 ADMM restated with MPC.py's settings and osqp's timing-derived adaptive-rho "
                   "interval as a fast host picks it ({ival}; the headline uses 100, OSQP's rule without PROFILING)",
    "accuracy": "engine extension beyond OSQP 0.6: the same ADMM, then polish=2 (OSQP's active-set polish, also "
                "after MAX_ITER / SOLVED_INACCURATE exits, status upgraded to SOLVED when the polished point "
                "meets eps; up to 8 active-set rounds, 10 refinements; adaptive rho every {ival})",
}
TOL_F = 1e-4  # north_star: forces within 1e-4 of OSQP


def launch_or_check(args):
    """--gpus N: under an external launcher (WORLD_SIZE set) check it started N ranks;
    otherwise, for N > 1, start the N rank processes here (one per GPU, fresh
    interpreters, before this process touches the GPU) and exit with their status."""
    from mpcq import launch
    backend = os.environ.get("MPCQ_DIST_BACKEND", "nccl")
    try:
        world, spawn = launch.resolve_world(args.gpus)
        if world > 1:
            launch.check_devices(world, backend)
    except launch.LaunchError as e:
        print(f"bench.py: {e}", file=sys.stderr, flush=True)
        sys.exit(2)
    if spawn:
        sys.exit(launch.run_ranks([sys.executable, "-u", os.path.abspath(__file__)] + sys.argv[1:], world))


def main():
    args = parse()
    launch_or_check(args)
    if args.mode == "plan":
        return main_plan(args)
    if args.mode == "tick":
        return main_tick(args)
    torch, dist, world, rank, local, dev, coll = _dist_setup()

    import mpcq
    from mpcq import model, shard

    cfg = CONFIGS[args.config]
    N = cfg["N"]
    if args.slice < 0:  # (auto) sliced beyond 16 stages: one instance per CU there
        args.slice = AUTO_SLICE if N > 16 else 0
    if args.batch > 0:
        total = args.batch * world
    elif cfg["per_gpu"]:
        total = cfg["per_gpu"] * world
    else:
        total = cfg["total"]
    scaling = "weak" if (cfg["per_gpu"] or args.batch > 0) else "strong"

    # this rank's contiguous shard of the seeded global synthetic batch (mpcq/shard.py)
    if cfg.get("static"):
        from mpcq import synth
        syn = synth.make_batch(total // world, N, gaits=cfg["gaits"], seed=args.seed, static=True)
    else:
        syn = shard.shard_batch(total, world, rank, N, cfg["gaits"], seed=args.seed)
    per = int(syn["xref"].shape[0])
    xref_d = torch.from_numpy(np.ascontiguousarray(syn["xref"])).to(dev)
    fs_d = torch.from_numpy(np.ascontiguousarray(syn["fsteps"])).to(dev)
    # a dedicated (non-default) HIP stream: the engine launches on it and the
    # HIP events that time the kernel are recorded on the same stream
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)

    def run_mode(mode, timed_steps, warmup, gather):
        """W untimed + K timed launches of one mode (barrier + synchronisation on both sides
        of the timed region), then one more launch that also returns x and y."""
        over = dict(MODES[mode])
        if args.rho_interval > 0:
            over["adaptive_rho_interval"] = args.rho_interval
        eng = mpcq.Engine(N, device=local, **over)
        eng.set_stream(stream.cuda_stream)
        if args.slice > 0:
            eng.set_slice(args.slice)
        f0_d = torch.empty((per, 12), dtype=torch.float64, device=dev)
        st_d = torch.empty(per, dtype=torch.int32, device=dev)
        it_d = torch.empty(per, dtype=torch.int32, device=dev)
        info_d = torch.empty((per, 4), dtype=torch.int32, device=dev)

        def launch(x_ptr=0, y_ptr=0):
            eng.solve_device(per, xref_d.data_ptr(), fs_d.data_ptr(), f0_d.data_ptr(), st_d.data_ptr(),
                             it_d.data_ptr(), x_ptr=x_ptr, y_ptr=y_ptr, info_ptr=info_d.data_ptr(), asynchronous=True,
                             order_by_class=bool(args.order_by_class))

        def step():
            launch()
            if gather and _distributed(dist):
                shard.gather_rows(dist, f0_d if coll.type == "cuda" else f0_d.cpu(), total, world, rank)

        for _ in range(warmup):
            step()
        torch.cuda.synchronize(dev)
        if _distributed(dist):
            dist.barrier()
        torch.cuda.synchronize(dev)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(timed_steps + 1)]
        t0 = time.perf_counter()
        evs[0].record(stream)
        for i in range(timed_steps):
            step()
            evs[i + 1].record(stream)
        torch.cuda.synchronize(dev)
        if _distributed(dist):
            dist.barrier()
        torch.cuda.synchronize(dev)
        wall = time.perf_counter() - t0
        launch_ms = (np.array([evs[i].elapsed_time(evs[i + 1]) for i in range(timed_steps)]) if timed_steps
                     else np.zeros(1))
        r = dict(mode=mode, over=over, params=eng.params, wall=wall, launch_ms=launch_ms,
                 kern_ms=float(launch_ms.mean()), status=st_d.cpu().numpy(), iters=it_d.cpu().numpy(),
                 info=info_d.cpu().numpy(), f0=f0_d.cpu().numpy())
        # after the timed region: one more launch that also returns x and y (the certificate's
        # active-set seed), and the host-buffer end-to-end path
        x_d = torch.empty((per, 24 * N), dtype=torch.float64, device=dev)
        y_d = torch.empty((per, 44 * N), dtype=torch.float64, device=dev)
        launch(x_d.data_ptr(), y_d.data_ptr())
        torch.cuda.synchronize(dev)
        r["same"] = bool(np.array_equal(f0_d.cpu().numpy(), r["f0"], equal_nan=True))
        r["x"], r["y"] = x_d.cpu().numpy(), y_d.cpu().numpy()
        e2e = []
        for _ in range(3):
            t_ = time.perf_counter()
            eng.solve(syn["xref"], syn["fsteps"], mpcq.MODE_UPDATE, want_x=False,
                      order_by_class=bool(args.order_by_class))
            e2e.append(time.perf_counter() - t_)
        r["e2e_ms"] = float(np.median(e2e)) * 1e3
        eng.close()
        del x_d, y_d
        return r

    head = run_mode(args.headline, args.steps, args.warmup, args.gather)
    wall_max = shard.max_over_ranks(dist, head["wall"], coll, world)
    kern_ms = head["kern_ms"]
    status, iters, info, f0 = head["status"], head["iters"], head["info"], head["f0"]
    solved = int(np.isin(status, (1, 2)).sum())
    p = head["params"]
    pol = args.headline == "accuracy"

    def work(r, structured=True):
        pp = r["params"]
        return model.flops(N, r["iters"], r["info"][:, 0], pp.check_termination,
                           pp.adaptive_rho_interval if pp.adaptive_rho else 0, pp.scaling,
                           polish_rounds=r["info"][:, 2] if pp.polish else None,
                           polish_solves=1 + max(pp.polish_refine_iter, model.polish_min_refinements(N)),
                           structured=structured).sum()

    fl, fl_dense = work(head), work(head, structured=False)
    by = model.bytes_per_instance(N) * per
    stats = torch.tensor([solved, per, fl, by, kern_ms], dtype=torch.float64, device=coll)
    if _distributed(dist):
        allst = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allst, stats)
        allst = torch.stack(allst).cpu().numpy()
    else:
        allst = stats.cpu().numpy()[None]
    other = "accuracy" if args.headline == "reference" else "reference"
    comp = run_mode(other, args.steps, min(args.warmup, 1), False) if (args.companion and world == 1) else None
    r25 = (run_mode("reference25", args.steps, min(args.warmup, 1), False)
           if (args.reference25 and world == 1 and args.headline == "reference" and args.rho_interval == 0)
           else None)

    def hist_of(r):
        sts, cnt = np.unique(r["status"], return_counts=True)
        return {int(a): int(b) for a, b in zip(sts, cnt)}

    def upgraded(r):  # polish = 2 turned a MAX_ITER / SOLVED_INACCURATE exit into SOLVED
        return int(((r["info"][:, 3] != 1) & (r["status"] == 1)).sum())

    if rank == 0:
        # QP instances solved (status 1 solved / 2 solved inaccurate) by all ranks per second
        value = float(allst[:, 0].sum()) * args.steps / wall_max
        fl0, by0 = float(allst[0, 2]), float(allst[0, 3])
        tag = (f"{args.config}_N{N}_B{per}" + ("_polish" if pol else "")
               + (f"_s{args.slice}" if args.slice > 0 and N > 16 else ""))
        src_sha = lib_sha()
        pmc = load_pmc(tag, src_sha)
        roof = {"bound": "valu_fp64", "achieved": fl0 / (kern_ms * 1e-3) / 1e12, "peak": PEAK_FP64_TFLOPS,
                "unit": "TFLOP/s", "frac": None, "traffic": pmc.get("bytes_per_launch"),
                "achieved_dense_model": fl_dense / (kern_ms * 1e-3) / 1e12,
                "achieved_counters": (pmc["fp64_flops_per_launch"] / (pmc["kernel_ms"] * 1e-3) / 1e12
                                      if pmc.get("fp64_flops_per_launch") and pmc.get("kernel_ms") else None),
                "note": "FP64 on VALU FMA (no MFMA: the stage blocks are 12x12 with sequential recurrences; gfx950's "
                        "FP64 vector and matrix peaks coincide, 78.6 TF). achieved = mpcq/model.py algorithmic flops "
                        "(measured iterations, rho updates, polish rounds; structural zeros excluded) per launch / mean "
                        "HIP-event launch time; achieved_dense_model counts the dense 24x24 stage blocks (round-1 model); "
                        "achieved_counters = issued FP64 lane-ops from the committed rocprofv3 PMC pass "
                        "(2 SQ_INSTS_VALU_FMA_F64 + MUL_F64 + ADD_F64) x 64 / that run's kernel time; traffic = HBM "
                        "bytes per launch from the PMC FETCH_SIZE / WRITE_SIZE passes (profiles/pmc_traffic.json)"}
        roof["frac"] = roof["achieved"] / roof["peak"]
        hbm_ach = by0 / (kern_ms * 1e-3) / 1e9
        roof_hbm = {"bound": "hbm", "achieved": hbm_ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": hbm_ach / PEAK_HBM_GBS, "traffic": pmc.get("bytes_per_launch"),
                    "note": f"algorithmic bytes {model.bytes_per_instance(N)} B/instance x {per} instances per launch"}
        edges = np.arange(0, p.max_iter + 251, 250)
        hist, _ = np.histogram(iters, bins=edges)
        launch_ms = head["launch_ms"]
        ival = p.adaptive_rho_interval
        out = {
            "metric": METRIC,
            "value": value,
            "unit": "QP instances/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": wall_max / max(args.steps, 1) * 1e3,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (seeded FootstepPlanner-shaped xref/fsteps, mpcq.synth)",
            "config": {"workload": workload_label(args.config, cfg, args.batch, world), "instances_per_gpu": per,
                       "instances_total": total,
                       "horizon": N, "gaits": list(cfg["gaits"]), "headline_mode": args.headline,
                       "solver": MODE_DESC[args.headline].format(ival=ival),
                       "parallelism": f"shard{world}" + ("+gather" if args.gather else ""),
                       "dispatch": ("by gait class: the mean iteration count of each instance's class over the "
                                    "engine's earlier launches, most expensive first (MPCQ_FLAG_ORDER_BY_CLASS, in "
                                    "the timed region)" if args.order_by_class else "index order")
                                   + (f"; sliced: the instances still iterating after {args.slice} ADMM iterations "
                                      "suspended and resumed in a second launch, the farthest from convergence first "
                                      "(mpcq_set_slice; both launches in the timed region)"
                                      if args.slice > 0 and N > 16 else "")},
            "roofline": roof,
            "roofline_hbm": roof_hbm,
            "build": {"engine_src_sha": src_sha, "pmc_tag": pmc.get("tag"), "pmc_stale": pmc.get("stale")},
            "dist": dist_fields(world, os.environ.get("MPCQ_DIST_BACKEND", "nccl"), _distributed(dist), torch),
            "kernel_ms_per_launch": kern_ms,
            "kernel_ms_launches": {"median": float(np.median(launch_ms)), "min": float(launch_ms.min()),
                                   "max": float(launch_ms.max())},
            "end_to_end_host_ms": head["e2e_ms"],
            "end_to_end_host_value": per / (head["e2e_ms"] * 1e-3),
            "solved_fraction": float(allst[:, 0].sum() / allst[:, 1].sum()),
            "status_hist": hist_of(head),
            "iters": {"median": float(np.median(iters)), "p90": float(np.percentile(iters, 90)),
                      "max": int(iters.max()), "rho_updates_mean": float(info[:, 0].mean()),
                      "hist_edges_step": 250, "hist": hist.tolist()},
        }
        if pol:
            out["polish"] = {"accepted_fraction": float((info[:, 1] == 1).mean()),
                             "rounds_mean": float(info[:, 2].mean()), "rounds_max": int(info[:, 2].max()),
                             "polish_upgraded": upgraded(head),
                             "admm_status_hist": {int(a): int(b) for a, b in
                                                  zip(*np.unique(info[:, 3], return_counts=True))}}
        if comp is not None:
            c_solved = int(np.isin(comp["status"], (1, 2)).sum())
            cd = {"mode": other, "solver": MODE_DESC[other].format(ival=comp["params"].adaptive_rho_interval),
                  "value": c_solved * args.steps / comp["wall"], "unit": "QP instances/s",
                  "ms_per_step": comp["wall"] / max(args.steps, 1) * 1e3, "kernel_ms_per_launch": comp["kern_ms"],
                  "roofline_frac": work(comp) / (comp["kern_ms"] * 1e-3) / 1e12 / PEAK_FP64_TFLOPS,
                  "status_hist": hist_of(comp),
                  "iters": {"median": float(np.median(comp["iters"])), "max": int(comp["iters"].max())},
                  "note": "timed after the headline on the same batch and box, same protocol (not the headline)"}
            if comp["params"].polish:
                cd["polish"] = {"accepted_fraction": float((comp["info"][:, 1] == 1).mean()),
                                "polish_upgraded": upgraded(comp),
                                "admm_status_hist": {int(a): int(b) for a, b in
                                                     zip(*np.unique(comp["info"][:, 3], return_counts=True))}}
            out["companion"] = cd
        if r25 is not None:
            r25_solved = int(np.isin(r25["status"], (1, 2)).sum())
            out["reference25"] = {
                "solver": MODE_DESC["reference25"].format(ival=r25["params"].adaptive_rho_interval),
                "value": r25_solved * args.steps / r25["wall"], "unit": "QP instances/s",
                "ms_per_step": r25["wall"] / max(args.steps, 1) * 1e3, "kernel_ms_per_launch": r25["kern_ms"],
                "roofline_frac": work(r25) / (r25["kern_ms"] * 1e-3) / 1e12 / PEAK_FP64_TFLOPS,
                "status_hist": hist_of(r25),
                "iters": {"median": float(np.median(r25["iters"])), "max": int(r25["iters"].max())},
                "note": "the second plausible f_osqp (osqp built with PROFILING picks the adaptive-rho interval from "
                        "its own timing; a fast host lands on 25): timed after the headline on the same batch and "
                        "box, same protocol; parity against the oracle's restatement at interval 25 under 'parity'"}
        if world == 1 and (args.cpu_sample > 0 or args.certify != 0 or args.restatement > 0):
            from oracle import oracle as O
            O.build()
        par = {"repeat_launch_bitwise_equal": head["same"] and (comp is None or comp["same"])}
        runs = {args.headline: head}
        if comp is not None:
            runs[other] = comp
        if world == 1 and args.certify != 0:
            from oracle import certify
            nc = per if args.certify < 0 else min(args.certify, per)
            t = time.perf_counter()
            ix = np.arange(nc)
            seed = runs.get("accuracy", head)  # the polished (x, y) is the closer active-set seed
            fstar, kkt, okc = certify.certified_forces(syn["xref"][ix], syn["fsteps"][ix], seed["x"][ix],
                                                       seed["y"][ix])
            par.update({"optimum_certified_fraction": float(okc.mean()), "optimum_kkt_max": float(kkt.max()),
                        "optimum_instances": int(nc), "optimum_seconds": time.perf_counter() - t,
                        "optimum": "x* of each instance's QP (oracle formulation, pinned to the reference's A/l/u): "
                                   "active-set solve of the unscaled KKT seeded by the GPU's (x, y), certified by "
                                   "KKT residuals < 1e-9 (oracle/certify.py)"})
            for name, r in runs.items():
                dfo = np.abs(r["f0"][:nc] - fstar).max(axis=1)
                par[f"{name}_max_abs_df0_vs_optimum"] = float(dfo.max())
                par[f"{name}_median_abs_df0_vs_optimum"] = float(np.median(dfo))
            par["max_abs_df0_vs_optimum"] = par[f"{args.headline}_max_abs_df0_vs_optimum"]
        hc = host_cpus()
        thr = args.cpu_threads or hc["usable"]
        if world == 1 and args.cpu_sample > 0:
            rate, ns, times = cpu_baseline(O, syn, per, O.default_params(**head["over"]), thr, args.cpu_sample)
            out["cpu_baseline"] = {"value": rate, "unit": "QP instances/s", "cores": thr, "kind": "port",
                                   "host": hc,
                                   "sample": f"{ns} instances per run cycling over the rank-0 batch of {per}; "
                                             "oracle/mpcq_oracle.c (C restatement of MPC.py + OSQP 0.6 ADMM"
                                             + (" + polish=2" if pol else ", polish off") + ") built -O3 "
                                             f"-march=native on this host, OpenMP over {thr} threads; 3 warm-up "
                                             f"runs, median of 10 ({min(times):.2f}-{max(times):.2f} s per run)"}
        if world == 1 and args.restatement > 0:
            # the checker build (the rounding the tests pin) against the GPU: OSQP as MPC.py configures
            # it (f_osqp of the metric), and the polish=2 restatement, each on the same instances
            nck = min(per, args.restatement)
            ref_o = {}
            for name in runs:
                ref_o[name] = O.solve_batch(syn["xref"][:nck], syn["fsteps"][:nck], 0,
                                            params=O.default_params(**runs[name]["over"]), nthreads=thr)
            par["restatement_instances"] = nck
            for name, r in runs.items():
                ro = ref_o[name]
                df = np.abs(ro["f0"] - r["f0"][:nck]).max(axis=1)
                par[f"{name}_max_abs_df0_vs_same_mode_restatement"] = float(df.max())
                par[f"{name}_status_agree"] = float((ro["status"] == r["status"][:nck]).mean())
                par[f"{name}_iters_agree"] = float((ro["iters"] == r["iters"][:nck]).mean())
                if "reference" in ref_o:
                    dm = np.abs(ref_o["reference"]["f0"] - r["f0"][:nck]).max(axis=1)
                    par[f"{name}_max_abs_df0_vs_osqp_mpcpy_settings"] = float(dm.max())
                    par[f"{name}_median_abs_df0_vs_osqp_mpcpy_settings"] = float(np.median(dm))
            if f"{args.headline}_max_abs_df0_vs_osqp_mpcpy_settings" in par:
                par["max_abs_df0_vs_osqp_mpcpy_settings"] = par[f"{args.headline}_max_abs_df0_vs_osqp_mpcpy_settings"]
            # how far OSQP's own machine-dependent choice moves f_osqp: osqp 0.6 built with PROFILING
            # picks adaptive_rho_interval from measured setup/iteration time (25 is what a fast host
            # lands on, 100 the rule without timing), so f_osqp itself is known only to this band
            band = {}
            for iv in (25, 100):
                if "reference" in ref_o and head["params"].adaptive_rho_interval == iv and args.headline == \
                        "reference":
                    band[iv] = ref_o["reference"]
                else:
                    band[iv] = O.solve_batch(syn["xref"][:nck], syn["fsteps"][:nck], 0,
                                             params=O.default_params(adaptive_rho_interval=iv), nthreads=thr)
            if r25 is not None:  # the GPU at interval 25 against the restatement at 25
                d25 = np.abs(band[25]["f0"] - r25["f0"][:nck]).max(axis=1)
                par["reference25_max_abs_df0_vs_same_mode_restatement"] = float(d25.max())
                par["reference25_status_agree"] = float((band[25]["status"] == r25["status"][:nck]).mean())
                par["reference25_iters_agree"] = float((band[25]["iters"] == r25["iters"][:nck]).mean())
                out["reference25"]["parity"] = {k[len("reference25_"):]: par[k] for k in
                                                ("reference25_max_abs_df0_vs_same_mode_restatement",
                                                 "reference25_status_agree", "reference25_iters_agree")}
            db = np.abs(band[25]["f0"] - band[100]["f0"]).max(axis=1)
            par["osqp_interval_band"] = float(db.max())
            par["osqp_interval_band_median"] = float(np.median(db))
            par["osqp_interval_band_note"] = (
                "max / median over the restatement instances of |f0(adaptive_rho_interval 25) - f0(100)|, "
                "OSQP at MPC.py's settings (oracle): the spread of f_osqp over OSQP's own timing-dependent "
                "choice of interval (MPC.py:414-416 sets only eps); a difference from f_osqp below it is not "
                "resolvable against the real library")
        # which reading of "max |f - f_osqp| <= 1e-4" each mode meets (from whichever comparisons ran)
        meets = {}
        for name in runs:
            mm = {}
            for key, lab in (("max_abs_df0_vs_osqp_mpcpy_settings", "f_osqp = OSQP restated with MPC.py's "
                              "settings (polish off)"), ("max_abs_df0_vs_optimum", "f_osqp = the QP's certified "
                                                         "optimum x*")):
                v = par.get(f"{name}_{key}")
                if v is not None:
                    mm[lab] = bool(v <= TOL_F)
            meets[name] = mm
        if any(meets.values()):
            par["meets_1e-4"] = meets
        out["parity"] = par
        print(json.dumps(out), flush=True)

    if _distributed(dist):
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
