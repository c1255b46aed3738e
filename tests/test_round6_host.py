"""CPU: round-6 host logic -- the bench line's workload label for shard runs, the reference25
reading's mode, the class-order flag's value in the header and the bindings, and the
nested-dissection horizons' workspace size (mpcq_internal.h) as the engine's static layout
states it."""
import os
import re
import sys

from conftest import REPO

sys.path.insert(0, REPO)


def test_shard_lines_name_the_shard():
    import bench
    lab = bench.workload_label("c4", bench.CONFIGS["c4"], 8192, 1)
    assert lab.startswith("C4 rank shard: 8192 of 65536") and "8 GPUs" in lab
    lab = bench.workload_label("c5", bench.CONFIGS["c5"], 4096, 1)
    assert lab.startswith("C5 rank shard: 4096 of 32768") and "trot/bound/pace" in lab
    assert bench.workload_label("c2", bench.CONFIGS["c2"], 0, 1) == bench.CONFIGS["c2"]["desc"]
    assert "batch overridden: 512" in bench.workload_label("c3", bench.CONFIGS["c3"], 512, 1)


def test_reference25_is_osqp_at_the_timed_interval():
    import bench
    assert bench.MODES["reference25"] == {"adaptive_rho_interval": 25}
    assert bench.MODES["reference"] == {}
    assert "25" in bench.MODE_DESC["reference25"].format(ival=25)


def test_class_order_flag_matches_the_header():
    hdr = open(os.path.join(REPO, "include", "mpcq.h")).read()
    m = re.search(r"#define MPCQ_FLAG_ORDER_BY_CLASS (\d+)u", hdr)
    assert m
    sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))
    from mpcq import _lib
    assert _lib.FLAG_ORDER_BY_CLASS == int(m.group(1))
    assert _lib.FLAG_ORDER_BY_CLASS & (_lib.FLAG_DEVICE_PTRS | _lib.FLAG_ASYNC) == 0


def test_nd_workspace_size_formula():
    """work_doubles(N) at the nested-dissection horizons: a 72-double zero block and the
    scaled constraint values (126 N - 18, rounded up to even) -- mirrored from
    mpcq_internal.h (the engine static_asserts Work<N>::SIZE against it)."""
    src = open(os.path.join(REPO, "mpc-tsid_amd", "csrc", "mpcq_internal.h")).read()
    m = re.search(r"#elif defined\(MPCQ_ND\)\nconstexpr bool nd_layout\(int N\) \{ return N == (\d+); \}", src)
    assert m and int(m.group(1)) == 32
    assert "#else\nconstexpr bool nd_layout(int) { return false; }" in src  # the production build
    assert "if (nd_layout(N)) return 72 + ((126 * (int64_t)N - 18 + 1) & ~1);" in src
