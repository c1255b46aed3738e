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


def main():
    args = parse()
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
