"""Algorithmic cost model of the engine (used by bench.py and DESIGN.md).

Bytes: the compulsory HBM traffic of the fused path per instance -- inputs
xref (12(N+1) doubles) and fsteps (20x13 doubles), outputs f0 (12 doubles),
status, iterations and the 4-int info record.

Flops (float64, a multiply and an add count as two): what the algorithm
needs per instance, counted on the structured operators the kernel applies
(structural zeros excluded; see flops_components):
  F = F_form + F_scale + (1 + R) F_fact + K F_iter + C F_check (+ polish)
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


def flops_components(N: int, scaling_iters: int = 10, structured: bool = True) -> dict:
    """Flops per instance of each phase.

    structured=True (the default, what bench.py reports): the useful
    operations of the engine's algorithm, structural zeros excluded -- the
    forces eliminated per stage through the 12x12 block K_ff^-1 (Gauss-Jordan,
    12 x 12 x 11 FMAs), F W and Q = W' F W on the six rows B touches (B's
    position rows are dt/m on one force column each), the 12x12 state system
    solved two-ended with 12x12 Schur couplings that are seven columns wide,
    and per iteration the 12x12 sweep products, the force recovery and the
    row updates.  Shadow lanes and masked terms the kernel issues are not
    counted (the PMC pass's issued FP64 lane-ops count them).

    structured=False: the round-1 model, dense 24x24 stage blocks with their
    zeros counted (an upper bound, kept for comparison)."""
    n, m, nnz = 24 * N, 44 * N, 126 * N - 18
    form = 375 * N                                      # B blocks + bounds
    scale = scaling_iters * (4 * nnz + 2 * (n + m) + 4 * n) + 2 * m
    check = 4 * nnz + n + 6 * (n + m)
    if not structured:
        fact = N * (2100 + 200 + 2 * 24 * 12 * 12 + 2 * 24 * 24 * 12 + 2 * 24 ** 3 + 2 * 12 * 12 * 24)
        it = N * (576 + 288 + 180 + 24 + 1152 + 180 + 288 + 600) + 4 * nnz + 10 * m + 5 * n
        return dict(form=form, scale=scale, fact=fact, iter=it, check=check, solve=it)
    fma = 2
    gj = 12 * 12 * 11 * fma + 12 * 4                     # 12x12 Gauss-Jordan (+ Newton reciprocal)
    fact = N * (144 * 5 * fma                           # K_ff: B' R B on rows 6..11 + swing + friction
                + gj                                    # F = K_ff^-1
                + (3 * 4 + 3 * 12) * 12 * fma           # F W (rows 6..8 touch one force per foot)
                + 36 * 12 * fma                         # Q = W' F W
                + 12 * 30 * fma                         # D / L rows of the state block
                + 2 * 12 * 12 * 7 * fma                 # coupling C S^-1 (seven-wide C) and its Schur update
                + gj)                                   # S^-1 (or U^-1, M^-1)
    # per stage: A_f' w (10 terms per force column), u = F b_f (12x12), beta = (F W)' b_f (6x12),
    # the three sweep products (G y, S^-1 y, G' x: 12x12 each), the force recovery (F W) g (12x6),
    # (R^-1 Q) g (6x6), A x~ on the 44 rows, the z / y / x updates
    solve = N * ((12 * 10 + 144 + 72 + 3 * 144 + 72 + 36) * fma + 44 * 4)
    it = solve + N * (44 * 8 + 24 * 3)
    return dict(form=form, scale=scale, fact=fact, iter=it, check=check, solve=solve)


def flops(N: int, iters, rho_updates, check_every: int = 25, adapt_every: int = 100,
          scaling_iters: int = 10, polish_rounds=None, polish_solves: int = 11,
          structured: bool = True) -> np.ndarray:
    """Per-instance algorithmic flops for measured iteration / rho-update counts
    (and, with polish, measured polish rounds: each one factorisation, 1 +
    refinement KKT solves and a residual evaluation)."""
    c = flops_components(N, scaling_iters, structured)
    K = np.asarray(iters, dtype=np.float64)
    R = np.asarray(rho_updates, dtype=np.float64)
    n_checks = np.floor(K / check_every)
    if adapt_every:
        n_checks += np.floor(K / adapt_every) - np.floor(K / np.lcm(check_every, adapt_every))
    n_checks += 1  # final evaluation when the loop exits on max_iter without a check
    f = c["form"] + c["scale"] + (1 + R) * c["fact"] + K * c["iter"] + n_checks * c["check"]
    if polish_rounds is not None:
        P = np.asarray(polish_rounds, dtype=np.float64)
        f = f + P * (c["fact"] + polish_solves * c["solve"] + c["check"])
    return f


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


def polish_min_refinements(N: int) -> int:
    """The engine's floor on polish refinement steps (mpcq_engine.hip kPolishMinIter)."""
    return 30 if N > 48 else (20 if N > 32 else 10)
