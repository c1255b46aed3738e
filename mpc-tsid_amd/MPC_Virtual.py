"""Drop-in module name of the reference's `MPC_Virtual.py`: re-exports the HIP-engine
façade (mpcq/wrapper.py).  Put this directory on sys.path and `import MPC_Virtual`."""
import os as _os
import sys as _sys

_here = _os.path.dirname(_os.path.abspath(__file__))
if _here not in _sys.path:
    _sys.path.insert(0, _here)

from mpcq.wrapper import MPC_Virtual  # noqa: E402,F401
import MPC_Wrapper  # noqa: E402,F401  (the reference module imports it by this name)
