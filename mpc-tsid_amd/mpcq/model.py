"""Algorithmic cost model of the engine (used by bench.py and DESIGN.md).

Bytes: the compulsory HBM traffic of the fused path per instance -- inputs
xref (12(N+1) doubles) and fsteps (20x13 doubles), outputs f0 (12 doubles),
status, iterations and the 4-int info record.

Flops (float64, a multiply and an add count as two): what the algorithm
needs per instance, counted on the structured operators the kernel applies
(zeros of the dense 24x24 stage blocks are counted; idle lanes are not):
  F = F_form + F_scale + (1 + R) F_fact + K F_iter + C F_check
with K ADMM iterations, R rho updates (refactorisations) and C residual
evaluations (every check_termination / adaptive-rho iteration), all three
measured per instance by the kernel.
"""
from __future__ import annotations

import numpy as np


def bytes_per_instance(N: int, with_x: bool = False, with_y: bool = False) -> int:
    b_in = 8 * (12 * (N + 1) + 20 * 13)
    b_out = 8 * 12 + 4 + 4 + 16
    if with_x:
        b_out += 8 * 24 * N
    if with_y:
        b_out += 8 * 44 * N
    return b_in + b_out


def flops_components(N: int, scaling_iters: int = 10) -> dict:
    n, m, nnz = 24 * N, 44 * N, 126 * N - 18
    form = 375 * N                                      # B blocks + bounds
    scale = scaling_iters * (4 * nnz + 2 * (n + m) + 4 * n) + 2 * m
    # per stage: K_k from the 56 rows touching it (~2.1k), C_k (~0.2k),
    # C Y (24x12x12), Schur update (24x24x12), Gauss-Jordan inverse (2*24^3),
    # Gamma = S^-1_{X,:} C (12x12x24)
    fact = N * (2100 + 200 + 2 * 24 * 12 * 12 + 2 * 24 * 24 * 12 + 2 * 24 ** 3 + 2 * 12 * 12 * 24)
    # per stage: alpha (12x24), forward step (12x12), C s, bhat, S^-1 bhat (24x24),
    # C' t, backward step, S^-1_{:,X} v (24x12); then A'w, A x, vector updates
    it = N * (576 + 288 + 180 + 24 + 1152 + 180 + 288 + 600) + 4 * nnz + 10 * m + 5 * n
    check = 4 * nnz + n + 6 * (n + m)
    return dict(form=form, scale=scale, fact=fact, iter=it, check=check)


def flops(N: int, iters, rho_updates, check_every: int = 25, adapt_every: int = 100,
          scaling_iters: int = 10) -> np.ndarray:
    """Per-instance algorithmic flops for measured iteration / rho-update counts."""
    c = flops_components(N, scaling_iters)
    K = np.asarray(iters, dtype=np.float64)
    R = np.asarray(rho_updates, dtype=np.float64)
    n_checks = np.floor(K / check_every)
    if adapt_every:
        n_checks += np.floor(K / adapt_every) - np.floor(K / np.lcm(check_every, adapt_every))
    n_checks += 1  # final evaluation when the loop exits on max_iter without a check
    return c["form"] + c["scale"] + (1 + R) * c["fact"] + K * c["iter"] + n_checks * c["check"]


def planner_bytes_per_instance(N: int, with_reduced: bool = True) -> int:
    """Compulsory HBM bytes of one MPCQ_PLAN_TICK planner instance: reads gait,
    state, l_feet, v_ref, (reduced), rotation flag / height and xref (in/out);
    writes gait, xref, fsteps, rotation flag / height and status."""
    nx = 8 * 12 * (N + 1)
    rd = 800 + 96 + 96 + 48 + (4 if with_reduced else 0) + 4 + 8 + nx
    wr = 800 + nx + 8 * 260 + 4 + 8 + 4
    return rd + wr


def retrieve_bytes_per_instance(N: int) -> int:
    """Compulsory HBM bytes of the session epilogue: reads x, xref, status, plan
    status, fsteps rows 0-1, gait row 0, q_w; writes x_robot, warm_x, cost, q_w,
    next state and feet."""
    rd = 8 * 24 * N + 8 * 12 * (N + 1) + 4 + 4 + 8 * 26 + 8 + 48
    wr = 8 * 12 * N + 8 * 24 * N + 8 * 13 + 48 + 96 + 96
    return rd + wr
