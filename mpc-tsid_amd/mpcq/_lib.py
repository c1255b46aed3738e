"""ctypes binding of libmpcq.so (the C ABI in include/mpcq.h).

The shared library is built in-tree (mpc-tsid_amd/csrc/Makefile ->
mpc-tsid_amd/mpcq/libmpcq.so) and loaded from here.  There is no fallback:
if the library or a HIP device is missing, the calls raise.

torch bundles its own HIP runtime (torch/lib/libamdhip64.so, soname
libamdhip64.so.7, the same as /opt/rocm's).  If libmpcq.so were loaded first
it would bind /opt/rocm's copy, torch would load its own next to it, and two
runtimes in one process leave torch without a device (tools/diag_runtime.py).
So before loading libmpcq.so this module loads the HIP runtime torch will use
(torch's own copy, found without importing torch) with RTLD_GLOBAL: libmpcq.so
binds to it whatever the import order, and there is one runtime per process.
Without torch installed, /opt/rocm's runtime is used.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
# MPCQ_LIB_VARIANT=stamps loads the diagnostic build of the same Makefile
# (per-phase cycle stamps, tools/stamps.py); MPCQ_LIB_VARIANT=exp:<name> loads an
# experiment build from csrc/build/variants (tools/build_variant.sh, timing tools
# only -- outside the package, never shipped)
_VARIANT = os.environ.get("MPCQ_LIB_VARIANT") or ""
if _VARIANT == "stamps":
    LIB_PATH = os.path.join(HERE, "libmpcq_stamps.so")
elif _VARIANT.startswith("exp:"):
    LIB_PATH = os.path.join(CSRC, "build", "variants", f"libmpcq_{_VARIANT[4:]}.so")
elif _VARIANT:
    raise ImportError(f"MPCQ_LIB_VARIANT={_VARIANT!r}: 'stamps' or 'exp:<name>'")
else:
    LIB_PATH = os.path.join(HERE, "libmpcq.so")

# return codes / status / flags / modes (include/mpcq.h)
OK = 0
E_INVALID, E_DEVICE, E_NOMEM, E_UNSUPPORTED = -1, -2, -3, -4
STATUS_SOLVED = 1
STATUS_SOLVED_INACCURATE = 2
STATUS_MAX_ITER_REACHED = -2
STATUS_PRIMAL_INFEASIBLE = -3
STATUS_DUAL_INFEASIBLE = -4
STATUS_PRIMAL_INFEASIBLE_INACCURATE = 3
STATUS_DUAL_INFEASIBLE_INACCURATE = 4
STATUS_NONFINITE = -10
STATUS_BAD_GAIT = -11
STATUS_FACTOR_FAILED = -12
STATUS_BAD_BOUNDS = -13
FLAG_DEVICE_PTRS = 1
FLAG_ASYNC = 2
FLAG_ORDER_BY_CLASS = 4  # mpcq_solve_batch: dispatch by the learned cost of each gait class
MODE_UPDATE = 0
MODE_SETUP = 1
PLAN_ROLL, PLAN_FOOTSTEPS, PLAN_REFSTATES = 1, 2, 4
PLAN_TICK = PLAN_ROLL | PLAN_FOOTSTEPS | PLAN_REFSTATES
# closed-loop session arrays (MPCQ_SV_*)
SV_F0, SV_X, SV_X_ROBOT, SV_Q_W, SV_COST, SV_XREF, SV_FSTEPS, SV_GAIT = range(8)
SV_STATUS, SV_ITERS, SV_RHO, SV_Y, SV_STATE, SV_L_FEET, SV_ROT_FLAG, SV_H_ROT = range(8, 16)
SV_ORDER = 16  # read-only: the next tick's dispatch order

EXPORTS = ("mpcq_abi_version", "mpcq_default_params", "mpcq_dims", "mpcq_pattern",
           "mpcq_supported_horizons", "mpcq_last_error", "mpcq_create", "mpcq_destroy",
           "mpcq_set_stream", "mpcq_set_slice", "mpcq_last_kernel_ms", "mpcq_formulate_batch",
           "mpcq_qp_solve_batch", "mpcq_solve_batch", "mpcq_default_planner_params",
           "mpcq_plan_batch", "mpcq_session_create", "mpcq_session_destroy", "mpcq_session_tick",
           "mpcq_session_read", "mpcq_session_write", "mpcq_session_device_ptr", "mpcq_debug_set_stamps",
           "mpcq_build_info")


class MpcqError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"mpcq error {code}: {msg}")
        self.code = code


class Params(C.Structure):
    """struct mpcq_params (include/mpcq.h)."""

    _fields_ = [
        ("dt", C.c_double),
        ("mass", C.c_double),
        ("gI", C.c_double * 9),
        ("mu", C.c_double),
        ("fz_max", C.c_double),
        ("gravity", C.c_double),
        ("state_weights", C.c_double * 12),
        ("force_weight", C.c_double),
        ("footholds", C.c_double * 12),
        ("rho", C.c_double),
        ("sigma", C.c_double),
        ("alpha", C.c_double),
        ("eps_abs", C.c_double),
        ("eps_rel", C.c_double),
        ("adaptive_rho_tolerance", C.c_double),
        ("delta", C.c_double),
        ("eps_prim_inf", C.c_double),
        ("eps_dual_inf", C.c_double),
        ("max_iter", C.c_int32),
        ("check_termination", C.c_int32),
        ("adaptive_rho", C.c_int32),
        ("adaptive_rho_interval", C.c_int32),
        ("scaling", C.c_int32),
        ("polish", C.c_int32),
        ("polish_refine_iter", C.c_int32),
        ("polish_rounds", C.c_int32),
        ("dual_warm", C.c_int32),
        ("reserved", C.c_int32 * 7),
    ]

    def as_dict(self):
        out = {}
        for name, _ in self._fields_:
            v = getattr(self, name)
            out[name] = list(v) if hasattr(v, "__len__") else v
        return out


class PlannerParams(C.Structure):
    """struct mpcq_planner_params (include/mpcq.h)."""

    _fields_ = [
        ("dt", C.c_double),
        ("T_gait", C.c_double),
        ("h_ref", C.c_double),
        ("k_feedback", C.c_double),
        ("L", C.c_double),
        ("g", C.c_double),
        ("t_stance", C.c_double),
        ("cmd_threshold", C.c_double),
        ("shoulders", C.c_double * 8),
        ("reduced_offset", C.c_double * 8),
        ("reserved", C.c_int32 * 8),
    ]


def build(force: bool = False) -> str:
    """Compile libmpcq.so for gfx950 with hipcc (csrc/Makefile)."""
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-j8", "-C", CSRC], check=True)
    return LIB_PATH


ABI_VERSION = 3  # include/mpcq.h MPCQ_ABI_VERSION these bindings follow
_lib = None
_hip_runtime = None


def hip_runtime_path():
    """The libamdhip64 this process uses: torch's bundled copy when torch is
    installed (whether or not it is imported yet), else the system one."""
    import importlib.util
    import sys
    t = sys.modules.get("torch")
    base = os.path.dirname(t.__file__) if t is not None and getattr(t, "__file__", None) else None
    if base is None:
        spec = importlib.util.find_spec("torch")
        base = os.path.dirname(spec.origin) if spec is not None and spec.origin else None
    if base is not None:
        cand = os.path.join(base, "lib", "libamdhip64.so")
        if os.path.exists(cand):
            return cand
    return None


def _preload_hip_runtime():
    global _hip_runtime
    if _hip_runtime is None:
        path = hip_runtime_path()
        _hip_runtime = C.CDLL(path, mode=C.RTLD_GLOBAL) if path else False
    return _hip_runtime


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise MpcqError(E_DEVICE, f"{LIB_PATH} is missing: run `make -C {CSRC}` (or __graft_entry__.build())")
    _preload_hip_runtime()
    L = C.CDLL(LIB_PATH)
    dp, ip, vp = C.POINTER(C.c_double), C.POINTER(C.c_int32), C.c_void_p
    PP = C.POINTER(Params)
    L.mpcq_abi_version.restype = C.c_int
    L.mpcq_default_params.argtypes = [PP]
    L.mpcq_default_params.restype = None
    L.mpcq_dims.argtypes = [C.c_int, ip, ip, ip]
    L.mpcq_pattern.argtypes = [C.c_int, ip, ip]
    L.mpcq_supported_horizons.argtypes = [ip, C.c_int]
    L.mpcq_last_error.restype = C.c_char_p
    L.mpcq_build_info.restype = C.c_char_p
    L.mpcq_create.argtypes = [C.c_int, C.c_int, PP, C.POINTER(vp)]
    L.mpcq_destroy.argtypes = [vp]
    L.mpcq_set_stream.argtypes = [vp, vp]
    L.mpcq_set_slice.argtypes = [vp, C.c_int32]
    L.mpcq_last_kernel_ms.argtypes = [vp, dp, dp]
    L.mpcq_formulate_batch.argtypes = [vp, C.c_int64, vp, vp, C.c_int, vp, vp, vp, vp, C.c_uint32]
    L.mpcq_qp_solve_batch.argtypes = [vp, C.c_int64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                      vp, C.c_uint32]
    L.mpcq_solve_batch.argtypes = [vp, C.c_int64, vp, vp, C.c_int, vp, vp, vp, vp, vp, vp, vp, vp, vp,
                                   vp, C.c_uint32]
    L.mpcq_debug_set_stamps.argtypes = [vp, vp]
    L.mpcq_default_planner_params.argtypes = [C.POINTER(PlannerParams)]
    L.mpcq_default_planner_params.restype = None
    L.mpcq_session_create.argtypes = [vp, C.c_int64, C.POINTER(PlannerParams), vp, C.POINTER(vp)]
    L.mpcq_session_destroy.argtypes = [vp]
    L.mpcq_session_tick.argtypes = [vp, C.c_int, vp, vp, vp, vp, C.c_uint32]
    L.mpcq_session_read.argtypes = [vp, C.c_int, vp, C.c_uint32]
    L.mpcq_session_write.argtypes = [vp, C.c_int, vp, C.c_uint32]
    L.mpcq_session_device_ptr.argtypes = [vp, C.c_int, C.POINTER(vp)]
    L.mpcq_plan_batch.argtypes = [vp, C.POINTER(PlannerParams), C.c_int64, C.c_uint32, C.c_int] + [vp] * 12 + [C.c_uint32]
    for name in ("mpcq_dims", "mpcq_pattern", "mpcq_supported_horizons", "mpcq_create",
                 "mpcq_destroy", "mpcq_set_stream", "mpcq_set_slice", "mpcq_last_kernel_ms", "mpcq_formulate_batch",
                 "mpcq_qp_solve_batch", "mpcq_solve_batch", "mpcq_default_planner_params",
           "mpcq_plan_batch", "mpcq_session_create", "mpcq_session_destroy", "mpcq_session_tick",
           "mpcq_session_read", "mpcq_session_write", "mpcq_session_device_ptr", "mpcq_debug_set_stamps"):
        getattr(L, name).restype = C.c_int
    if L.mpcq_abi_version() != ABI_VERSION:
        raise MpcqError(E_UNSUPPORTED, f"{LIB_PATH} has ABI {L.mpcq_abi_version()}, these bindings ABI {ABI_VERSION}: "
                        f"rebuild it (`make -C {CSRC}`)")
    _lib = L
    return L


def check(rc: int):
    if rc != OK:
        msg = lib().mpcq_last_error()
        raise MpcqError(rc, msg.decode() if msg else "")
    return rc


def default_params(**overrides) -> Params:
    p = Params()
    lib().mpcq_default_params(C.byref(p))
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise AttributeError(f"unknown parameter {k}")
        setattr(p, k, v)
    return p


def default_planner_params(**overrides) -> PlannerParams:
    p = PlannerParams()
    lib().mpcq_default_planner_params(C.byref(p))
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise AttributeError(f"unknown planner parameter {k}")
        setattr(p, k, v)
    return p


def build_info() -> dict:
    """The loaded library's build stamp (mpcq_build_info): {"src_sha256": ..., "arch": ...}."""
    raw = lib().mpcq_build_info().decode()
    return dict(kv.split("=", 1) for kv in raw.split() if "=" in kv)


def source_sha(csrc: str = CSRC) -> str:
    """The stamp a default `make` gives the sources in ``csrc`` (csrc/stamp.py: sha256 over
    the HIP sources, the assembly pass, the Makefile, the headers, the C++ units and the
    Makefile's default flags; first 16 hex digits)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("mpcq_stamp", os.path.join(csrc, "stamp.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod.stamp(csrc)


def supported_horizons():
    buf = (C.c_int32 * 64)()
    n = lib().mpcq_supported_horizons(buf, 64)
    return [buf[i] for i in range(min(n, 64))]
