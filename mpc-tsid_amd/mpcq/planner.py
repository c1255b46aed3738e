"""Drop-in FootstepPlanner over the HIP planner kernel (mpcq_plan_batch).

Mirrors the reference class FootstepPlanner (FootstepPlanner.py:7-459) name for
name: the constructor ``FootstepPlanner(dt, n_periods)``, the attributes the
control loop and MPC_Wrapper read (``xref``, ``fsteps``, ``gait``, ``x0``,
``n_steps``, ``T_gait``, ``shoulders``, ``flag_rotation_command``,
``h_rotation_command``, ...) and the methods ``getRefStates``,
``compute_footsteps``, ``roll``, ``update_fsteps`` and the gait creators.
Every method runs on the device (one robot = a batch of one); there is no CPU
fallback.

Errors as in the reference: ``roll`` on a table without a zero-duration row
raises TypeError (FootstepPlanner.py:405 ``next(...)[0]`` on the 0.0 default),
``compute_footsteps`` walking past row 19 raises IndexError; the planner state
is then left unchanged.

Deliberate differences: ``create_bounding`` / ``create_side_walking`` /
``create_static`` fill the 20-row table the rest of the class uses (the
reference writes a 6-row one, which its own compute_footsteps cannot broadcast
into fsteps, FootstepPlanner.py:295); ``update_viewer`` and the ``oMl`` /
``ftps_Ids`` visualisation arguments are accepted and ignored; compute_next_footstep
is evaluated inside the kernel only (its result is not exposed).
"""
from __future__ import annotations

import numpy as np

from . import _lib as L
from .engine import Engine

_MASKS = {
    "trot": ((1, 1, 1, 1), (1, 0, 0, 1), (1, 1, 1, 1), (0, 1, 1, 0)),    # FootstepPlanner.py:226-229
    "bound": ((1, 1, 1, 1), (1, 1, 0, 0), (1, 1, 1, 1), (0, 0, 1, 1)),   # :251-254
    "side": ((1, 1, 1, 1), (1, 0, 1, 0), (1, 1, 1, 1), (0, 1, 0, 1)),    # :276-279
}


class FootstepPlanner:
    def __init__(self, dt, n_periods, device: int = 0, engine: Engine | None = None):
        self.k_feedback = 0.03
        self.shoulders = np.array([[0.19, 0.19, -0.19, -0.19], [0.15005, -0.15005, 0.15005, -0.15005]])
        self.dt = float(dt)
        self.g = 9.81
        self.L = 0.12
        self.footsteps = self.shoulders.copy()
        self.footsteps_world = self.footsteps.copy()
        self.n_periods = int(n_periods)
        self.T_gait = 0.32
        self.n_steps = int(self.n_periods * self.T_gait / self.dt)
        self.engine = engine if engine is not None else Engine(self.n_steps, device=device, dt=self.dt)
        if self.engine.n_steps != self.n_steps:
            raise ValueError(f"engine horizon {self.engine.n_steps} != planner horizon {self.n_steps}")
        self.xref = np.zeros((12, 1 + self.n_steps))
        self.gait = np.zeros((20, 5))
        self.fsteps = np.full((20, 13), np.nan)
        self._flag = np.zeros(1, np.int32)
        self._h_rot = np.array([0.20])
        self.x0 = self.xref[:, 0:1]
        self.create_walking_trot()

    # the rotation-command state machine (FootstepPlanner.py:67-68)
    @property
    def flag_rotation_command(self):
        return int(self._flag[0])

    @flag_rotation_command.setter
    def flag_rotation_command(self, v):
        self._flag[0] = int(v)

    @property
    def h_rotation_command(self):
        return float(self._h_rot[0])

    @h_rotation_command.setter
    def h_rotation_command(self, v):
        self._h_rot[0] = float(v)

    def _params(self, T_gait=None, h_ref=None):
        p = L.default_planner_params(dt=self.dt, k_feedback=self.k_feedback, L=self.L, g=self.g)
        if T_gait is not None:
            p.T_gait = float(T_gait)
        if h_ref is not None:
            p.h_ref = float(h_ref)
        for i, v in enumerate(self.shoulders.ravel()):
            p.shoulders[i] = float(v)
        return p

    def _run(self, ops, k, state, l_feet=None, v_ref=None, v_cur=None, h=None, reduced=False, params=None):
        self.gait = np.ascontiguousarray(self.gait, np.float64)
        self.xref = np.ascontiguousarray(self.xref, np.float64)
        self.fsteps = np.ascontiguousarray(self.fsteps, np.float64)
        if self.gait.shape != (20, 5):
            raise ValueError(f"gait must be (20, 5), got {self.gait.shape}")
        st = self.engine.plan(
            ops, int(k), np.asarray(state, np.float64).reshape(1, 12),
            None if l_feet is None else np.asarray(l_feet, np.float64).reshape(1, 3, 4),
            np.asarray(v_ref, np.float64).reshape(1, 6), self.gait.reshape(1, 20, 5), self._flag, self._h_rot,
            self.xref.reshape(1, 12, self.n_steps + 1), self.fsteps.reshape(1, 20, 13),
            reduced=np.array([int(bool(reduced))], np.int32),
            v_cur=None if v_cur is None else np.asarray(v_cur, np.float64).reshape(1, 6),
            h=None if h is None else np.array([float(h)]), params=params or self._params())
        return int(st[0])

    # ------------------------------------------------------------------ reference methods
    def getRefStates(self, k, T_gait, lC, abg, lV, lW, v_ref, h_ref=0.2027682):
        """FootstepPlanner.py:76-159 (k == 0 sets the reference height)."""
        state = np.concatenate([np.ravel(lC), np.ravel(abg), np.ravel(lV), np.ravel(lW)])
        self._run(L.PLAN_REFSTATES, 0 if k == 0 else 1, state, v_ref=v_ref,
                  params=self._params(T_gait=T_gait, h_ref=h_ref))
        self.x0 = self.xref[:, 0:1]
        return 0

    def compute_footsteps(self, l_feet, v_cur, v_ref, h, reduced):
        """FootstepPlanner.py:284-361."""
        state = np.zeros(12)
        if self._run(L.PLAN_FOOTSTEPS, 1, state, l_feet=l_feet, v_ref=v_ref, v_cur=v_cur, h=h, reduced=reduced):
            raise IndexError("index 20 is out of bounds for axis 0 with size 20")
        return 0

    def roll(self):
        """FootstepPlanner.py:401-425."""
        if self._run(L.PLAN_ROLL, 1, np.zeros(12), v_ref=np.zeros(6)):
            raise TypeError("'float' object is not subscriptable")
        return 0

    def update_fsteps(self, k, l_feet, v_cur, v_ref, h, oMl=None, ftps_Ids=None, reduced=False):
        """FootstepPlanner.py:427-459 (visualisation arguments ignored)."""
        if k > 0:
            self.roll()
        self.compute_footsteps(l_feet, v_cur, v_ref, h, reduced)
        return 0

    def update_viewer(self, viewer, initialisation):
        return 0

    # ------------------------------------------------------------------ gaits (FootstepPlanner.py:179-282)
    def _periodic(self, masks):
        half = int(0.5 * self.T_gait / self.dt)
        self.gait = np.zeros((20, 5))
        for i in range(self.n_periods):
            self.gait[4 * i:4 * i + 4, 0] = (1, half - 1, 1, half - 1)
            self.gait[4 * i:4 * i + 4, 1:] = masks
            self.fsteps[4 * i:4 * i + 4, 0] = self.gait[4 * i:4 * i + 4, 0]
        return 0

    def create_walking_trot(self):
        return self._periodic(_MASKS["trot"])

    def create_bounding(self):
        return self._periodic(_MASKS["bound"])

    def create_side_walking(self):
        return self._periodic(_MASKS["side"])

    def create_static(self):
        self.gait = np.zeros((20, 5))
        self.gait[0, 0] = self.n_steps
        self.gait[0, 1:] = 1.0
        self.fsteps[0, 0] = self.gait[0, 0]
        return 0
