#!/usr/bin/env python3
"""Benchmark of the MI355X batched MPC-QP hot path (MPC.py formulation + OSQP solve).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
           --master-port P bench.py --gpus N --steps K --warmup W

One step = one launch of the fused engine kernel (formulation + Ruiz scaling +
KKT factorisation + OSQP ADMM to eps 1e-7) over this rank's batch of
synthetic (xref, fsteps) instances, inputs resident in HBM.  Ranks shard the
instances (no data-path collective): value = instances solved by all ranks /
max-over-ranks wall time of the K timed steps.

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
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c2", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=0, help="override instances per GPU")
    ap.add_argument("--polish", action="store_true", help="accurate mode: polish=2, 8 rounds, 10 refinements")
    ap.add_argument("--cpu-sample", type=int, default=12288,
                    help="instances in the CPU-baseline sample, cycling over the rank-0 batch (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--gather", action="store_true", help="include an RCCL all-gather of f0 in the timed region")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--mode", default="qp", choices=("qp", "plan", "tick"),
                    help="qp: the headline (fused formulation + OSQP per instance); plan: the batched "
                         "FootstepPlanner kernel alone; tick: closed-loop sessions (planner + warm-started "
                         "solve + retrieve per robot and tick, virtual robot)")
    return ap.parse_args()


def load_traffic(tag: str):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if any."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(tag)
        return float(e["bytes_per_launch"]) if e else None
    except (OSError, ValueError):
        return None


def _dist_setup():
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    return torch, dist, world, rank, local, dev


def _timed(torch, dist, dev, world, stream, step, steps, warmup):
    """W untimed steps, then K steps between barriers + synchronisations; returns
    (max-over-ranks wall seconds, HIP-event ms per step on the launch stream)."""
    from mpcq import shard
    torch.cuda.set_stream(stream)
    for i in range(warmup):
        step(i)
    torch.cuda.synchronize(dev)
    if world > 1:
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
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    return shard.max_over_ranks(dist, wall, dev, world), ev0.elapsed_time(ev1) / max(steps, 1)


def main_plan(args):
    """Batched FootstepPlanner (mpcq_plan_batch, MPCQ_PLAN_TICK) on device-resident
    robots: one step = one planner launch over this rank's robots."""
    torch, dist, world, rank, local, dev = _dist_setup()
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

    wall, ms = _timed(torch, dist, dev, world, stream, step, args.steps, args.warmup)
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
                            "frac": ach / PEAK_HBM_GBS, "traffic": load_traffic(f"plan_N{N}_B{per}"),
                            "note": f"algorithmic {model.planner_bytes_per_instance(N)} B/robot x {per} robots "
                                    "per launch / HIP-event launch time"},
               "kernel_ms_per_launch": ms, "ok_fraction": ok / per}
        if world == 1 and args.cpu_sample > 0:
            from oracle import oracle as O
            O.build()
            ns = min(args.cpu_sample, per)
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
    if world > 1:
        dist.destroy_process_group()


def main_tick(args):
    """Closed-loop sessions: one step = one tick of every robot on this rank
    (planner + warm-started fused solve + retrieve), virtual robot."""
    torch, dist, world, rank, local, dev = _dist_setup()
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

    wall, ms = _timed(torch, dist, dev, world, stream, step, args.steps, warm)
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
               "roofline": {"bound": "mfma", "achieved": ach, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                            "frac": ach / PEAK_FP64_TFLOPS, "traffic": None,
                            "note": "engine kernel of the last tick: model.flops(measured iterations, rho updates "
                                    "taken as 0 -- a lower bound) / its HIP-event time"},
               "kernel_ms": {"step": ms, "planner_last_tick": plan_ms, "solve_last_tick": solve_ms},
               "solved_fraction": float(np.isin(st, (1, 2)).mean()),
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
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.mode == "plan":
        return main_plan(args)
    if args.mode == "tick":
        return main_tick(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", init_method="env://")
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    import mpcq
    from mpcq import model, shard

    cfg = CONFIGS[args.config]
    N = cfg["N"]
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
    f0_d = torch.empty((per, 12), dtype=torch.float64, device=dev)
    st_d = torch.empty(per, dtype=torch.int32, device=dev)
    it_d = torch.empty(per, dtype=torch.int32, device=dev)
    info_d = torch.empty((per, 4), dtype=torch.int32, device=dev)

    over = dict(polish=2, polish_rounds=8, polish_refine_iter=10) if args.polish else {}
    eng = mpcq.Engine(N, device=local, **over)
    # a dedicated (non-default) HIP stream: the engine launches on it and the
    # HIP events that time the kernel are recorded on the same stream
    stream = torch.cuda.Stream(dev)
    eng.set_stream(stream.cuda_stream)

    def step():
        eng.solve_device(per, xref_d.data_ptr(), fs_d.data_ptr(), f0_d.data_ptr(), st_d.data_ptr(),
                         it_d.data_ptr(), info_ptr=info_d.data_ptr(), asynchronous=True)
        if args.gather and world > 1:
            shard.gather_rows(dist, f0_d, total, world, rank)  # forces of every instance on every rank

    torch.cuda.set_stream(stream)
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(args.steps):
        step()
    ev1.record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / max(args.steps, 1)

    wall_max = shard.max_over_ranks(dist, wall, dev, world)

    # end to end through host buffers (H2D + kernel + D2H, the façade's path):
    # measured after the timed region, reported beside it, never as `value`
    e2e = []
    for _ in range(3):
        t_ = time.perf_counter()
        eng.solve(syn["xref"], syn["fsteps"], mpcq.MODE_UPDATE, want_x=False)
        e2e.append(time.perf_counter() - t_)
    e2e_ms = float(np.median(e2e)) * 1e3

    status = st_d.cpu().numpy()
    iters = it_d.cpu().numpy()
    info = info_d.cpu().numpy()
    f0 = f0_d.cpu().numpy()
    solved = int(np.isin(status, (1, 2)).sum())
    # per-launch algorithmic work of this rank
    p = eng.params
    fl = model.flops(N, iters, info[:, 0], p.check_termination,
                     p.adaptive_rho_interval if p.adaptive_rho else 0, p.scaling).sum()
    by = model.bytes_per_instance(N) * per

    stats = torch.tensor([solved, per, fl, by, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        allst = [torch.zeros_like(stats) for _ in range(world)]
        dist.all_gather(allst, stats)
        allst = torch.stack(allst).cpu().numpy()
    else:
        allst = stats.cpu().numpy()[None]

    if rank == 0:
        value = float(allst[:, 1].sum()) * args.steps / wall_max
        avg_ms = float(kern_ms)
        fl0, by0 = float(allst[0, 2]), float(allst[0, 3])
        tr = load_traffic(f"{args.config}_N{N}_B{per}")
        roof = {"bound": "mfma", "achieved": fl0 / (avg_ms * 1e-3) / 1e12, "peak": PEAK_FP64_TFLOPS,
                "unit": "TFLOP/s", "frac": None, "traffic": tr,
                "note": "fp64: the kernel runs on VALU FMA; gfx950's FP64 MFMA and vector peaks coincide (78.6 TF). "
                        "achieved = model.flops(measured iterations, rho updates) per launch / mean launch time; "
                        "traffic = HBM bytes per launch from the committed rocprofv3 PMC passes (profiles/pmc_traffic.json)"}
        roof["frac"] = roof["achieved"] / roof["peak"]
        hbm_ach = by0 / (avg_ms * 1e-3) / 1e9
        roof_hbm = {"bound": "hbm", "achieved": hbm_ach, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                    "frac": hbm_ach / PEAK_HBM_GBS, "traffic": tr,
                    "note": f"algorithmic bytes {model.bytes_per_instance(N)} B/instance x {per} instances per launch"}
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
            "config": {"workload": cfg["desc"], "instances_per_gpu": per, "instances_total": total,
                       "horizon": N, "gaits": list(cfg["gaits"]),
                       "solver": "OSQP-0.6 ADMM restated (eps 1e-7, rho 0.1, sigma 1e-6, alpha 1.6, Ruiz 10, adaptive rho/100)"
                       + (" + active-set polish" if args.polish else ""),
                       "parallelism": f"shard{world}" + ("+gather" if args.gather else "")},
            "roofline": roof,
            "roofline_hbm": roof_hbm,
            "kernel_ms_per_launch": avg_ms,
            "end_to_end_host_ms": e2e_ms,
            "end_to_end_host_value": per / (e2e_ms * 1e-3),
            "solved_fraction": float(allst[:, 0].sum() / allst[:, 1].sum()),
            "iters": {"median": float(np.median(iters)), "p90": float(np.percentile(iters, 90)),
                      "max": int(iters.max()), "rho_updates_mean": float(info[:, 0].mean())},
        }
        if world == 1 and args.cpu_sample > 0:
            from oracle import oracle as O
            O.build()
            ns = args.cpu_sample
            sel = np.arange(ns) % per  # cycle over the GPU batch: same instance mix
            thr = args.cpu_threads or int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
            op = O.default_params(**over)
            t = time.perf_counter()
            ro = O.solve_batch(syn["xref"][sel], syn["fsteps"][sel], 0, params=op, nthreads=thr)
            tc = time.perf_counter() - t
            nc = min(ns, per)
            df = np.abs(ro["f0"][:nc] - f0[:nc]).max(axis=1)
            out["cpu_baseline"] = {"value": ns / tc, "unit": "QP instances/s", "cores": thr, "kind": "port",
                                   "sample": f"{ns} instances cycling over the rank-0 batch of {per}, oracle/mpcq_oracle.c "
                                             f"(C restatement of MPC.py + OSQP 0.6 ADMM), OpenMP over {thr} threads, {tc:.1f} s"}
            out["parity"] = {"max_abs_df0_vs_osqp_restatement": float(df.max()),
                             "median_abs_df0_vs_osqp_restatement": float(np.median(df)),
                             "status_agree": float((ro["status"][:nc] == status[:nc]).mean()),
                             "iters_agree": float((ro["iters"][:nc] == iters[:nc]).mean())}
        print(json.dumps(out), flush=True)

    eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
