"""tools/prof_summary.py on a synthetic profile.sh output (CPU): per-solve figures for sliced
solves (two engine launches per solve) and per-launch figures otherwise, the stamp copied into
pmc_traffic.json, the gfx950 x2 read correction."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
K = "void mpcq::(anonymous namespace)::engine_kernel<32, true, true, false>(mpcq_params, mpcq::LaunchArgs)"


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def _fake(root, grids, durations_ns, fetch_kib, write_kib, sha="0123456789abcdef", compactions=0):
    tr = [[K, g, 512, 159232, 224, 128, 0, 112] for g in grids]
    _write(os.path.join(root, "trace", "run_kernel_trace.csv"),
           ["Kernel_Name", "Grid_Size_X", "Workgroup_Size_X", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
            "Accum_VGPR_Count", "SGPR_Count"], tr)
    tot = sum(durations_ns)
    rows = [[K, len(durations_ns), tot / len(durations_ns), min(durations_ns), max(durations_ns), 99.0]]
    if compactions:
        rows.append(["mpcq::(anonymous namespace)::suspended_kernel(int const*, long, int const*, double const*)",
                     compactions, 10e3, 9e3, 11e3, 0.04])
    _write(os.path.join(root, "trace", "run_kernel_stats.csv"),
           ["Name", "Calls", "AverageNs", "MinNs", "MaxNs", "Percentage"], rows)
    for p, name, vals in (("fetch", "FETCH_SIZE", fetch_kib), ("write", "WRITE_SIZE", write_kib)):
        _write(os.path.join(root, p, "run_counter_collection.csv"), ["Kernel_Name", "Counter_Name", "Counter_Value"],
               [[K, name, v] for v in vals])
    line = json.dumps({"metric": "m", "build": {"engine_src_sha": sha}})
    for p in ("trace", "fetch", "write"):
        open(os.path.join(root, f"{p}.log"), "w").write("banner\n" + line + "\n")


def _run(tmp_path, key, **kw):
    src, out = tmp_path / "prof", tmp_path / "out"
    _fake(str(src), **kw)
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "prof_summary.py"), "tX", "--key", key,
                        "--instances", "1024", "--src-dir", str(src), "--out-dir", str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return json.load(open(out / "pmc_traffic.json"))[key], (out / "tX_summary.md").read_text()


def test_sliced_solves_are_summed_per_solve(tmp_path):
    # two solves, each a first launch and a resumed one (both sized for the batch) around a compaction
    e, md = _run(tmp_path, "c3_N32_B1024_s1200", grids=[524288] * 4, compactions=2,
                 durations_ns=[12e6, 11e6, 12.5e6, 10.5e6], fetch_kib=[100.0, 60.0, 100.0, 60.0],
                 write_kib=[50.0, 30.0, 50.0, 30.0])
    assert e["launches_per_solve"] == 2.0
    assert abs(e["kernel_ms"] - 23.0) < 1e-9
    assert abs(e["bytes_per_launch"] - (2 * 160.0 + 80.0) * 1024) < 1e-6  # per solve
    assert e["engine_src_sha"] == "0123456789abcdef"
    assert "sliced solves: 4 engine launches for 2 solves" in md and "HBM counters (per solve)" in md


def test_unsliced_launches_are_averaged(tmp_path):
    e, md = _run(tmp_path, "c2_N16_B1024", grids=[262144] * 3, durations_ns=[7.6e6, 7.7e6, 7.5e6],
                 fetch_kib=[14000.0, 14200.0, 14100.0], write_kib=[46000.0, 46100.0, 46200.0])
    assert e["launches_per_solve"] == 1.0
    assert abs(e["kernel_ms"] - 7.6) < 1e-9
    assert abs(e["bytes_per_launch"] - (2 * 14100.0 + 46100.0) * 1024) < 1e-6
    assert "sliced" not in md
