"""CPU: provenance of the committed profiles and the bench line's distribution fields.

bench.py quotes HBM traffic and issued FP64 flops from profiles/pmc_traffic.json only
when the entry was profiled on the library that is running (its engine_src_sha stamp,
written by tools/prof_summary.py from the profiled process's own bench line)."""
import json
import os
import sys

import pytest

from conftest import REPO

sys.path.insert(0, REPO)


@pytest.fixture(scope="module")
def bench():
    import bench as b
    return b


def test_load_pmc_drops_other_builds(bench, tmp_path):
    path = tmp_path / "pmc.json"
    path.write_text(json.dumps({
        "c2_N16_B1024": {"bytes_per_launch": 1.0e8, "tag": "r05x", "engine_src_sha": "aaaaaaaaaaaaaaaa"},
        "c3_N32_B1024": {"bytes_per_launch": 6.1e8, "tag": "r04uc3"},  # unstamped (a pre-stamp entry)
    }))
    ok = bench.load_pmc("c2_N16_B1024", "aaaaaaaaaaaaaaaa", str(path))
    assert ok["bytes_per_launch"] == 1.0e8 and "stale" not in ok
    other = bench.load_pmc("c2_N16_B1024", "bbbbbbbbbbbbbbbb", str(path))
    assert "bytes_per_launch" not in other and "aaaaaaaaaaaaaaaa" in other["stale"]
    unst = bench.load_pmc("c3_N32_B1024", "aaaaaaaaaaaaaaaa", str(path))
    assert "bytes_per_launch" not in unst and "unstamped" in unst["stale"]
    assert bench.load_pmc("c2_N16_B1024", None, str(path)).get("bytes_per_launch") is None
    assert bench.load_pmc("c5_N16_B32768", "aaaaaaaaaaaaaaaa", str(path)) == {}


def test_committed_entries_are_stamped():
    """Every entry bench.py may quote carries the stamp of the build it profiled."""
    d = json.load(open(os.path.join(REPO, "profiles", "pmc_traffic.json")))
    for key, e in d.items():
        assert e.get("engine_src_sha") and len(e["engine_src_sha"]) == 16, key


@pytest.fixture(scope="module")
def mpcq_built():
    import mpcq
    mpcq.build()
    return mpcq


def test_library_stamp_is_its_source(mpcq_built):
    """The library's mpcq_build_info is the sha of the .hip sources in the tree (the
    Makefile's rule and mpcq.source_sha agree), so a stale build shows up as a mismatch."""
    import mpcq
    info = mpcq.build_info()
    assert info["arch"] == "gfx950"
    assert info["src_sha256"] == mpcq.source_sha()


def test_prof_summary_reads_the_profiled_stamp(tmp_path):
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import prof_summary
    log = tmp_path / "trace.log"
    log.write_text("rocprofv3 noise\n" + json.dumps({"metric": "m", "build": {"engine_src_sha": "0123456789abcdef"}})
                   + "\nprofile rc=0\n")
    assert prof_summary.bench_stamp(str(log)) == "0123456789abcdef"
    assert prof_summary.bench_stamp(str(tmp_path / "absent.log")) is None


class _FakeCuda:
    def __init__(self, n):
        self.n = n

    def device_count(self):
        return self.n


class _FakeTorch:
    def __init__(self, n):
        self.cuda = _FakeCuda(n)


def test_dist_fields_mark_rehearsals(bench):
    assert bench.dist_fields(4, "gloo", True, _FakeTorch(1)) == {"backend": "gloo", "distinct_devices": 1,
                                                                 "rehearsal": True}
    assert bench.dist_fields(8, "nccl", True, _FakeTorch(8)) == {"backend": "nccl", "distinct_devices": 8,
                                                                 "rehearsal": False}
    assert bench.dist_fields(1, "nccl", False, _FakeTorch(1))["backend"] is None


def test_variant_and_stamps_builds_carry_their_own_stamp():
    """an experiment variant (tools/build_variant.sh) and the stamps library link
    their own mpcq_build.o, so their mpcq_build_info differs from the production build's and
    bench.py's provenance gate drops production PMC figures for them."""
    import subprocess
    sys.path.insert(0, os.path.join(REPO, "mpc-tsid_amd"))
    import mpcq
    prod = mpcq.source_sha()
    src = os.path.join(REPO, "mpc-tsid_amd", "csrc", "mpcq_engine.hip")

    def vstamp(*flags):
        r = subprocess.run(["bash", os.path.join(REPO, "tools", "build_variant.sh"), "--stamp-only", "ilp32", src,
                            *flags], capture_output=True, text=True, timeout=60, check=True)
        return r.stdout.strip()
    a, b = vstamp(), vstamp("-DMPCQ_FR_HELD")
    assert a.startswith(prod + "+exp:ilp32:") and b.startswith(prod + "+exp:ilp32:") and a != b
    import bench
    sys.path.insert(0, REPO)
    entry = {"c3_N32_B1024": {"bytes_per_launch": 1.0, "tag": "rX", "engine_src_sha": prod}}
    import json as _json
    import tempfile
    with tempfile.NamedTemporaryFile("w", suffix=".json", delete=False) as f:
        _json.dump(entry, f)
    try:
        assert bench.load_pmc("c3_N32_B1024", prod, f.name)["bytes_per_launch"] == 1.0
        assert "stale" in bench.load_pmc("c3_N32_B1024", a, f.name)
    finally:
        os.unlink(f.name)
    # the stamps library links mpcq_build_stamps.o (stamp + "+stamps"), not the production object
    r = subprocess.run(["make", "-s", "-n", "-B", "-C", os.path.join(REPO, "mpc-tsid_amd", "csrc"), "../mpcq/libmpcq_stamps.so"],
                       capture_output=True, text=True, timeout=120)
    link = [ln for ln in r.stdout.splitlines() if "-shared" in ln and "libmpcq_stamps.so" in ln]
    assert link and "mpcq_build_stamps.o" in link[-1] and "build/mpcq_build.o" not in link[-1]
    assert any("+stamps" in ln for ln in r.stdout.splitlines()) or os.path.exists(
        os.path.join(REPO, "mpc-tsid_amd", "csrc", "build", "mpcq_build_stamps.o"))
