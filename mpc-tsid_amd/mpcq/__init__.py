"""mpcq — MI355X-native batched convex-MPC QP engine (the MPC.py hot path of
thomascbrs/mpc-tsid).  See DESIGN.md.

Public surface:
  Engine            batched formulate / qp_solve / solve over libmpcq.so
  default_params    reference constants + OSQP 0.6 settings (MPC.py:25-39, 414-416)
  pattern, dims     CSC pattern / sizes of MPC.create_ML
  Engine.plan       batched FootstepPlanner (roll / compute_footsteps / getRefStates)
  Session           B robots in closed loop, all per-tick state resident in HBM
  synth             seeded synthetic inputs shaped like FootstepPlanner's
"""
from . import synth  # noqa: F401
from ._lib import (FLAG_ASYNC, FLAG_DEVICE_PTRS, FLAG_ORDER_BY_CLASS, MODE_SETUP, MODE_UPDATE,  # noqa: F401
                   PLAN_FOOTSTEPS, PLAN_REFSTATES, PLAN_ROLL, PLAN_TICK, PlannerParams,
                   default_planner_params, STATUS_BAD_GAIT, SV_COST, SV_F0, SV_FSTEPS, SV_GAIT,
                   SV_H_ROT, SV_ITERS, SV_ORDER, SV_L_FEET, SV_Q_W, SV_RHO, SV_ROT_FLAG, SV_STATE, SV_STATUS, SV_X,
                   SV_X_ROBOT, SV_XREF, SV_Y, STATUS_FACTOR_FAILED, STATUS_MAX_ITER_REACHED,
                   STATUS_NONFINITE, STATUS_SOLVED, STATUS_SOLVED_INACCURATE, STATUS_PRIMAL_INFEASIBLE,
                   STATUS_DUAL_INFEASIBLE, STATUS_PRIMAL_INFEASIBLE_INACCURATE,
                   STATUS_DUAL_INFEASIBLE_INACCURATE, STATUS_BAD_BOUNDS, MpcqError,
                   Params, build, build_info, default_params, lib, source_sha, supported_horizons)
from .engine import Engine, dims, pattern  # noqa: F401
from .session import Session  # noqa: F401

__version__ = "0.1.0"
