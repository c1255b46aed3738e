"""Drop-in module name of the reference's `FootstepPlanner.py`: re-exports the
HIP-planner façade (mpcq/planner.py).  Put this directory on sys.path and
`import FootstepPlanner`."""
import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))
if _here not in _sys.path:
    _sys.path.insert(0, _here)

from mpcq.planner import FootstepPlanner  # noqa: E402,F401
