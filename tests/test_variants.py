"""CPU: the engine's opt-in compile switches still build (mpc-tsid_amd/csrc/Makefile
`variants`: MPCQ_FR_HELD / ZC_HELD / SPLIT_OUT / NO_LDS_ZERO / FACTIME / STAMPS /
DEBUG_* at horizons where each changes the code).  Compile only, nothing runs: the
objects are rebuilt when the engine source is newer than them (a few minutes after an
engine edit, seconds otherwise)."""
import os
import subprocess

from conftest import REPO

CSRC = os.path.join(REPO, "mpc-tsid_amd", "csrc")


def test_engine_variants_compile():
    if subprocess.run(["make", "-q", "-C", CSRC, "variants"], capture_output=True).returncode == 0:
        return  # every variant object is newer than the engine source
    r = subprocess.run(["make", "-s", "-j8", "-C", CSRC, "variants"], capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, r.stderr[-4000:]
